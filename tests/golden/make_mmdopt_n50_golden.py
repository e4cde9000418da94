"""Generate tests/golden/mmdopt_n50_ref.npz: the ORACLE's (oracle/, the NumPy
restatement of the reference) solve of BASELINE configs[0] -- the drop-in
``CEM(50, 4, 0.1, 20, "gaussian", 0, 0)`` (num_batch 100, M = 2500 mother
rollouts) on configuration k = 0 of S/main_mpc.py:10-21 -- for two outer
iterations, from injected draws ``Draws.random(prob,
np.random.default_rng(SEED))`` that the GPU test regenerates.

The oracle's beta-CEM at M = 2500 takes ~10 s per candidate and outer
iteration (a 2501-dim Cholesky per beta-iteration), too slow for a GPU
test, so its result is precomputed here (8 processes, a few minutes).
Stored: the result tuple, per iteration the elite index sets and every
candidate's costs / beta-CEM outputs, and per (iteration, candidate,
beta-iteration) the relative gaps of the sorted QP costs at the argmin
(0/1) and at the elite boundary (10/11), so the GPU test can tell a
near-tie from a real difference without re-running the oracle.

    python tests/golden/make_mmdopt_n50_golden.py     (no reference access needed)
"""
import multiprocessing as mp
import os
import sys

for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[k] = "1"

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from oracle import beta_cem as bc  # noqa: E402
from oracle import costs as C  # noqa: E402
from oracle import helper as Hh  # noqa: E402

N, O, LEVEL, H, B, T, SEED = 50, 4, 0.1, 20, 100, 2, 5
_G = {}


def _init(prob, z0, z):
    _G.update(prob=prob, z0=z0, z=z)


def _one(args):
    cxm, cym = args
    tr = []
    beta, res, sigma, sel = bc.compute_cem(_G["prob"], cxm, cym, _G["z0"], _G["z"], tr)
    gaps = np.zeros((20, 2))
    for t, d in enumerate(tr):
        c = np.sort(np.asarray(d["cost"], np.float64))
        for j, i in enumerate((0, 10)):
            gaps[t, j] = abs(c[i + 1] - c[i]) / max(abs(c[i]), 1e-6)
    return beta, res, sigma, sel, gaps


class ParallelCEM(oracle.CEM):
    """oracle.CEM with the per-candidate beta-CEM loop of candidate_costs
    spread over processes (same arithmetic, same order of results)."""

    def __init__(self, *a, pool=None, **k):
        super().__init__(*a, **k)
        self.pool = pool
        self.gaps = []

    def candidate_costs(self, cost, st, acc, steer, x_obs, y_obs, draws, t):
        p = self.prob
        n, Hp = p.num_reduced, p.num_prime
        xo, yo = x_obs[:, :Hp], y_obs[:, :Hp]
        acc_n, steer_n = Hh.noisy_controls(p, acc[:, :Hp], steer[:, :Hp], draws, t, n)
        acc_m, steer_m = Hh.mother_controls(acc_n, steer_n)
        xm, ym = Hh.rollout(p, acc_m, steer_m, st["st0"])
        cxm, cym = Hh.compute_coeff(p, xm, ym)
        out = self.pool.map(_one, [(cxm[b], cym[b]) for b in range(acc.shape[0])])
        beta = np.stack([o[0] for o in out]).astype(np.float32)
        res_beta = np.stack([o[1] for o in out]).astype(np.float32)
        sigma = np.array([o[2] for o in out], np.float32)
        sel = np.stack([o[3] for o in out]).astype(np.int64)
        self.gaps.append(np.stack([o[4] for o in out]))
        xr = np.take_along_axis(xm, sel[:, :, None], axis=1)
        yr = np.take_along_axis(ym, sel[:, :, None], axis=1)
        cb = C.compute_f_bar_max(p, xr, yr, xo, yo)
        obs = C.mmd(p, beta, cb, sigma)
        lane = C.mmd_lane(p, beta, sigma, yr)
        return obs, lane, dict(beta=beta, sigma=sigma, res_beta=res_beta, sel=sel)


def main():
    from optimizer.sweep import static_obstacles
    probe = oracle.CEM(N, O, LEVEL, H, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=T)
    draws = oracle.Draws.random(probe.prob, np.random.default_rng(SEED), idx_mpc=0, with_beta_cem=True)
    ob = static_obstacles(0, O)
    xo, yo, _ = Hh.compute_obs_trajectories(probe.prob, ob["x"], ob["y"], ob["vx"], ob["vy"], ob["psi"])
    init = np.array([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
    mean = np.array([15] * 4 + [0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    draws.idx_mpc = ob["idx_mpc"]
    with mp.get_context("fork").Pool(8, initializer=_init, initargs=(probe.prob, draws.beta_z0, draws.beta_z)) as pool:
        ora = ParallelCEM(N, O, LEVEL, H, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=T, pool=pool)
        trace = []
        ref = ora.solve("mmd_opt", ob["idx_mpc"], init, mean, cov, xo, yo, 15.0, draws=draws, trace=trace)
    out = dict(seed=SEED, idx_mpc=ob["idx_mpc"], x_obs=xo, y_obs=yo, init=init, mean=mean, cov=cov,
               cx=ref[0], cy=ref[1], cost_lane=ref[2], cost_obs=ref[3], beta=ref[4], sigma=ref[5], res_beta=ref[6],
               gaps=np.stack(ora.gaps))
    for t, d in enumerate(trace):
        for key in ("perm", "elite_obs", "elite_cem", "obs", "lane", "res_beta", "sigma", "beta", "res_norm", "cost20"):
            out[f"t{t}_{key}"] = np.asarray(d[key])
    dst = os.path.join(HERE, "mmdopt_n50_ref.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, "cost_obs", ref[3], "sigma", ref[5])


if __name__ == "__main__":
    main()
