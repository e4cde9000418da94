"""Generate tests/golden/mmdopt_n50_ref.npz: the ORACLE's (oracle/, the NumPy
restatement of the reference) solve of BASELINE configs[0]'s shape -- the
drop-in ``CEM(50, 4, 0.1, 20, "gaussian", 0, 0)`` (num_batch 100, M = 2500
mother rollouts) -- for two outer iterations, from injected draws
``Draws.random(prob, np.random.default_rng(SEED))`` that the GPU test
regenerates.  The four obstacles sit INSIDE the H = 20 (3 s) rollout horizon
(BLOCK_X / BLOCK_Y: one grazing the ego lane, one on it, two on the other
lane), so a share of the noisy rollouts collides and the MMD obstacle costs
separate the candidates (configuration k = 0 of S/main_mpc.py:10-21 places
every obstacle at x >= 35 m, beyond the horizon: every cost is the MMD floor).

The oracle's beta-CEM at M = 2500 takes ~10 s per candidate and outer
iteration (a 2501-dim Cholesky per beta-iteration), too slow for a GPU
test, so its result is precomputed here (8 processes, a few minutes).
Stored: the result tuple, per iteration the elite index sets and every
candidate's costs / beta-CEM outputs, and per (iteration, candidate,
beta-iteration) the minimum QP cost, the sum of the 11 elite costs (the
trace the GPU records in ``btrace``) and the relative gaps of the sorted QP
costs at the argmin (0/1) and at the elite boundary (10/11), so the GPU test
can tell a near-tie from a real difference without re-running the oracle
(tests/parity.py: beta_divergence).

    python tests/golden/make_mmdopt_n50_golden.py     (no reference access needed)
"""
import multiprocessing as mp
import os
import sys

for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[k] = "1"

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from oracle import beta_cem as bc  # noqa: E402
from oracle import costs as C  # noqa: E402
from oracle import helper as Hh  # noqa: E402

N, O, LEVEL, H, B, T, SEED = 50, 4, 0.1, 20, 100, 2, 5
BLOCK_X = [13.0, 24.0, 18.0, 30.0]
BLOCK_Y = [4.4, 1.75, -1.75, -1.75]
IDX_MPC = 4242
_G = {}


def _init(prob, z0, z):
    _G.update(prob=prob, z0=z0, z=z)


def _one(args):
    from parity import beta_trace
    cxm, cym = args
    tr = []
    beta, res, sigma, sel = bc.compute_cem(_G["prob"], cxm, cym, _G["z0"], _G["z"], tr)
    _, esum, gaps = beta_trace(tr)
    return beta, res, sigma, sel, gaps, esum


class ParallelCEM(oracle.CEM):
    """oracle.CEM with the per-candidate beta-CEM loop of candidate_costs
    spread over processes (same arithmetic, same order of results)."""

    def __init__(self, *a, pool=None, **k):
        super().__init__(*a, **k)
        self.pool = pool
        self.gaps = []
        self.esum = []

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
        self.esum.append(np.stack([o[5] for o in out]))
        xr = np.take_along_axis(xm, sel[:, :, None], axis=1)
        yr = np.take_along_axis(ym, sel[:, :, None], axis=1)
        cb = C.compute_f_bar_max(p, xr, yr, xo, yo)
        obs = C.mmd(p, beta, cb, sigma)
        lane = C.mmd_lane(p, beta, sigma, yr)
        return obs, lane, dict(beta=beta, sigma=sigma, res_beta=res_beta, sel=sel)


def main():
    probe = oracle.CEM(N, O, LEVEL, H, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=T)
    draws = oracle.Draws.random(probe.prob, np.random.default_rng(SEED), idx_mpc=0, with_beta_cem=True)
    z = np.zeros(O)
    ob = dict(idx_mpc=IDX_MPC)
    xo, yo, _ = Hh.compute_obs_trajectories(probe.prob, BLOCK_X, BLOCK_Y, z, z, z)
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
               gaps=np.stack(ora.gaps), esum=np.stack(ora.esum))
    for t, d in enumerate(trace):
        for key in ("perm", "elite_obs", "elite_cem", "obs", "lane", "res_beta", "sigma", "beta", "res_norm", "cost20"):
            out[f"t{t}_{key}"] = np.asarray(d[key])
    dst = os.path.join(HERE, "mmdopt_n50_ref.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, "cost_obs", ref[3], "sigma", ref[5])
    for t in range(T):
        o = out[f"t{t}_obs"]
        print(f"iteration {t}: obs min {o.min():.4f} max {o.max():.4f}, {(o > o.min() + 1e-2).sum()} candidates above the floor")


if __name__ == "__main__":
    main()
