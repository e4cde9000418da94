"""Sensitivity ensembles of the CARLA compute_cem_mmd oracle (test
infrastructure for tests/test_gpu_carla.py::test_carla_mmd_free_run).

A free-running GPU solve and the oracle part once their fp32 MMD values
(~1e-7 relative apart) move the CEM weights by an ulp: from that iteration on
the two populations differ and the 19 remaining CEM iterations may amplify the
difference (the projection order of feasible candidates is rounding noise,
SURVEY Q6).  What a correct GPU solve must satisfy after such a parting is
measured on the oracle itself: each ensemble member resumes the oracle from its
carry at the parting iteration and shifts that iteration's risks (obstacle,
lane, desired lane) by 1-2 ulp per candidate with its own seed -- the size of
the GPU-vs-oracle difference -- then runs unperturbed to the end.  The spread
of the members' returned tuples is the oracle's own sensitivity to an ulp at
that point.

Members run in child processes (spawn: a fresh interpreter that imports only
NumPy and oracle/, never HIP), eight at a time (the GPU box gives a job 16
CPUs).
"""
import concurrent.futures as cf
import multiprocessing as mp

import numpy as np

MEAN = np.array([10.0] * 4 + [0.0] * 4, np.float32)   # main_carla.py:306-318 (v_des = 10, y = 0)
COV = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
KEYS = ("cx", "cy", "v_best", "steering", "mean_param")


def ulp_shift(a, rng):
    """Every finite nonzero entry moved by +-1 or +-2 ulp (fp32)."""
    a = np.array(a, np.float32, copy=True)
    m = np.isfinite(a) & (a != 0)
    k = rng.choice(np.array([-2, -1, 1, 2], np.int32), size=a.shape)
    bits = a.view(np.int32)
    bits[m] = bits[m] + k[m]
    return a


def _member(args):
    (n, B, H, O, T, level, town, idx, draw_seed, init, xo, yo, path, tp, snap, k) = args
    from oracle import carla as K
    ora = K.CarlaCEM(n, 1, O, level, H, "gaussian", town, 0.0, 0.0, num_batch=B, maxiter_cem=T)
    draws = K.CarlaDraws.random(ora.prob, np.random.default_rng(draw_seed), idx_mpc=idx, with_beta_cem=True)
    rng = np.random.default_rng(1000 + k)

    def perturb(t, obs, lane, des):
        if t != tp:
            return obs, lane, des
        return ulp_shift(obs, rng), ulp_shift(lane, rng), ulp_shift(des, rng)

    cx, cy, v, steer, mean, _ = ora.solve_carla("mmd_opt", idx, init, MEAN, COV, xo, yo, 10.0, path, draws,
                                                start=(tp, snap), perturb=perturb)
    cost = K.plan_cost(ora.prob, "mmd_opt", cx, cy, steer, xo, yo, path, 10.0)
    return dict(cx=cx, cy=cy, v_best=v, steering=steer, mean_param=mean, cost=cost)


_ONE_THREAD = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")


def run(shape, inputs, tp, snap, members=16, workers=8):
    """shape = (n, B, H, O, T, level, town, idx, draw_seed); inputs = (init,
    xo, yo, path).  Returns the members' result dicts.  The children's BLAS
    runs single-threaded (each member already spreads its beta-CEMs over a
    4-thread pool; a BLAS pool per child sized to the machine oversubscribes
    the CPUs several times over)."""
    import os
    jobs = [tuple(shape) + tuple(inputs) + (tp, snap, k) for k in range(members)]
    saved = {k: os.environ.get(k) for k in _ONE_THREAD}
    os.environ.update({k: "1" for k in _ONE_THREAD})
    try:
        with cf.ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
            futs = [ex.submit(_member, j) for j in jobs]   # the children start here, with the env above
            return [f.result() for f in futs]
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def spread_check(got, ref, members, margin=1.25, atol=1e-4):
    """The GPU tuple against the ensemble's spread.  Per returned quantity,
    D(a, b) = max |a - b| over its elements; the GPU's distance from the
    unperturbed oracle must not exceed `margin` times the ensemble's diameter
    (the largest D between any two of members + oracle) plus atol.  The GPU
    solve is, for the oracle, one more ulp-perturbed run: a bound by the
    ensemble's extreme (its per-element range, or its worst cost) would
    reject such a run with probability ~1/(members + 2) by construction, so
    the bound is the diameter, widened by the margin.  Returns {key: (GPU
    distance, diameter)}."""
    pts = list(members) + [ref]
    rep = {}
    for k in KEYS:
        a = [np.asarray(m[k], np.float64) for m in pts]
        diam = max(float(np.max(np.abs(a[i] - a[j]))) for i in range(len(a)) for j in range(i))
        rep[k] = (float(np.max(np.abs(np.asarray(got[k], np.float64) - np.asarray(ref[k], np.float64)))), diam)
    return rep


def cost_bound(costs, margin=0.5):
    """The worst plan cost a correct solve may reach: the members' (and the
    oracle's) worst, widened by `margin` times their range (same reason as
    spread_check)."""
    lo, hi = min(costs), max(costs)
    return hi + margin * (hi - lo) + 1e-4 * abs(hi)
