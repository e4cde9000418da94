"""Shared helpers for GPU-vs-oracle parity tests.

Tolerance contract (Numerics): costs and trajectories within
1e-4 relative (with an absolute floor for values near 0); elite index sets
bit-exact unless the compared keys are a near-tie (within tolerance), in
which case the difference is reported, not hidden.
"""
from __future__ import annotations

import numpy as np

import oracle
from oracle.helper import compute_obs_trajectories

RTOL = 1e-4


def close(name, got, ref, rtol=RTOL, atol=1e-5, frac_ok=0.0):
    """Assert |got - ref| <= atol + rtol |ref| elementwise (NaN == NaN).
    ``frac_ok``: tolerated fraction of mismatching elements (rejection-
    sampled Beta draws, documented)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, f"{name}: shape {got.shape} vs {ref.shape}"
    both_nan = np.isnan(got) & np.isnan(ref)
    err = np.abs(got - ref)
    bad = ~both_nan & ~(err <= atol + rtol * np.abs(ref))
    if bad.mean() > frac_ok:
        i = np.argwhere(bad)[:5]
        detail = [(tuple(j), got[tuple(j)], ref[tuple(j)]) for j in i]
        raise AssertionError(f"{name}: {bad.sum()}/{bad.size} outside tol; worst {np.nanmax(err):.3g}; {detail}")
    return float(np.nanmax(np.where(both_nan, 0, err))) if err.size else 0.0


def elite_equal(name, got, ref, keys, tol=RTOL):
    """Index sets must agree; where they differ, every differing candidate's
    key must be within ``tol`` (relative) of the boundary key."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    if np.array_equal(got, ref):
        return True
    keys = np.asarray(keys, np.float64)
    bound = keys[ref[-1]]
    diff = np.setxor1d(got, ref)
    scale = max(abs(bound), 1e-6)
    near = np.all(np.abs(keys[diff] - bound) <= tol * scale + 1e-6)
    if np.array_equal(np.sort(got), np.sort(ref)):
        # same set, different order: order ties must be near-ties too
        pos = np.nonzero(got != ref)[0]
        near = np.all(np.abs(keys[got[pos]] - keys[ref[pos]]) <= tol * np.maximum(np.abs(keys[ref[pos]]), 1e-6) + 1e-6)
    assert near, f"{name}: index sets differ beyond a near-tie: got {got} ref {ref}"
    return False


def scenario(num_obs, seed=0):
    """Static-obstacle scenario like S/main_mpc.py:10-21 on an extended x grid
    (the reference's 9-slot grid cannot place > 9 obstacles)."""
    rng = np.random.RandomState(seed)
    xs = np.arange(35, 35 + 5 * max(9, num_obs), 5, dtype=np.float64)
    x = rng.choice(xs, num_obs, replace=False)
    y = rng.choice(np.array([-1.75, 1.75]), num_obs)
    z = np.zeros(num_obs)
    return x, y, z, z, z


DEFAULT_INIT = np.array([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], np.float32)   # S/main_mpc.py:46-54
DEFAULT_MEAN = np.array([15] * 4 + [0] * 4, np.float32)                 # S/main_mpc.py:58-71
DEFAULT_COV = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)      # S/main_mpc.py:69-74


def make_pair(native, cost, noise="gaussian", n=16, O=3, H=10, B=32, T=3, level=None, variant="static",
              acc_c=0.0, steer_c=0.0, seed=0):
    level = (0.1 if noise == "gaussian" else 0.3) if level is None else level
    ora = oracle.CEM(n, O, level, H, noise, acc_c, steer_c, num_batch=B, variant=variant, maxiter_cem=T)
    cfg = native.make_config(n, O, level, H, noise, acc_c, steer_c, num_batch=B, variant=variant,
                             maxiter_cem=T, device=0, seed=seed)
    nat = native.Handle(cfg)
    x, y, vx, vy, psi = scenario(O, seed)
    xo, yo, _ = compute_obs_trajectories(ora.prob, x, y, vx, vy, psi)
    return ora, nat, xo, yo


def beta_cem_trace(ora, st, acc, steer, draws, t):
    """The oracle's beta-CEM of ONE candidate (controls acc, steer [100]) at
    outer iteration t, with its per-iteration trace (costs, elites)."""
    from oracle import beta_cem as bc
    from oracle import helper as Hh
    p = ora.prob
    H = p.num_prime
    acc_n, steer_n = Hh.noisy_controls(p, acc[None, :H], steer[None, :H], draws, t, p.num_reduced)
    acc_m, steer_m = Hh.mother_controls(acc_n, steer_n)
    xm, ym = Hh.rollout(p, acc_m, steer_m, st["st0"])
    cxm, cym = Hh.compute_coeff(p, xm, ym)
    trace = []
    beta, res, sigma, sel = bc.compute_cem(p, cxm[0], cym[0], draws.beta_z0, draws.beta_z, trace)
    return dict(beta=beta, res=res, sigma=sigma, sel=sel, trace=trace)


# Explaining a divergence of one candidate's beta-CEM (compute_beta.py:93-157)
# between the GPU and the oracle.  The two runs see the same samples until an
# elite set differs; a flip of the 11th / 12th smallest QP cost at
# beta-iteration t changes the samples of t + 1 -- every later cost -- while
# an argmin flip at t changes only that iteration's outputs (beta_best,
# sigma_best are taken from the LAST iteration, Q4).  The GPU writes, per
# beta-iteration, the minimum cost (res_beta) and the sum of the 11 elite
# costs (btrace); the first iteration t0 where either differs from the
# oracle's is where the runs parted, and only a near-tie at the elite boundary
# of t0 - 1 can explain it.  When both traces agree through iteration 19 but
# the outputs differ, only a near-tie of the last iteration can.
#
# TIE_REL: GPU and oracle QP costs of identical samples agree to ~1e-7
# relative (v_exp_f32 kernels, fp32 inputs; measured in the lockstep test,
# test_gpu_parity_mmdopt.py), so a gap below TIE_REL may order differently on
# the two sides and a larger one may not.
TIE_REL = 2e-6
AGREE_REL = 1e-6   # trace entries "equal" (GPU vs oracle, same samples)


def beta_trace(tr):
    """Per beta-iteration arrays of an oracle trace (beta_cem.compute_cem's
    ``trace`` list): res [20], elite-cost sum [20], relative gaps [20, 2] of
    the sorted costs at the argmin (0 / 1) and at the elite boundary (10 / 11)."""
    T = len(tr)
    res = np.zeros(T)
    esum = np.zeros(T)
    gaps = np.zeros((T, 2))
    for t, d in enumerate(tr):
        c = np.asarray(d["cost"], np.float32)
        order = oracle.helper.argsort_stable(c)
        cs = c[order].astype(np.float64)
        res[t] = cs[0]
        esum[t] = np.float32(cs[:11].sum())
        for j, i in enumerate((0, 10)):
            gaps[t, j] = abs(cs[i + 1] - cs[i]) / max(abs(cs[i]), 1e-6)
    return res, esum, gaps


def _differ(a, b, rel=AGREE_REL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return ~(np.abs(a - b) <= rel * np.maximum(np.abs(a), 1e-3))


def beta_divergence(res, esum, gaps, res_gpu, esum_gpu, tie=TIE_REL):
    """(t0, explained, detail) for one candidate whose beta-CEM outputs
    differ between GPU and oracle (see the comment above)."""
    d = _differ(res, res_gpu) | _differ(esum, esum_gpu)
    if d.any():
        t0 = int(np.argmax(d))
        if t0 == 0:
            return 0, False, "traces differ at beta-iteration 0 (same samples: no tie can explain it)"
        g = float(gaps[t0 - 1, 1])
        return t0, g < tie, f"traces part at beta-iteration {t0}; elite-boundary gap at {t0 - 1}: {g:.3g}"
    g = float(min(gaps[-1, 0], gaps[-1, 1]))
    return len(res) - 1, g < tie, f"traces agree; last-iteration argmin / boundary gap {g:.3g}"


def beta_near_tie(tr, res_gpu, esum_gpu, tie=TIE_REL):
    """beta_divergence from a live oracle trace (beta_cem_trace)."""
    res, esum, gaps = beta_trace(tr["trace"])
    return beta_divergence(res, esum, gaps, res_gpu, esum_gpu, tie)
