"""BASELINE configs[0] on the GPU: the drop-in
``CEM(50, 4, 0.1, 20, "gaussian", 0, 0).compute_cem_mmd_opt(...)``
(num_reduced 50 -> M = 2500 mother rollouts, the reference's num_batch 100),
two outer iterations on a scenario whose four obstacles lie inside the 3 s
horizon (collisions separate the candidates), against the oracle's solve of
the same call from the same injected draws (tests/golden/mmdopt_n50_ref.npz,
made by make_mmdopt_n50_golden.py: the oracle needs ~10 s per candidate and
iteration at M = 2500).

Per outer iteration every candidate's obs / lane costs (1e-4 relative), its
beta-CEM trace (per beta-iteration minimum and elite-cost sum), res_beta and
sigma must agree.  A candidate may differ only where its beta-CEM parted at a
near-tie the fixture records at the ONE iteration that can explain the
parting (tests/parity.py: beta_divergence -- the elite boundary just before
the first differing beta-iteration, or the last iteration's argmin /
boundary).  The elite index sets must then be identical, the run must reach
the last iteration in lockstep, and the result tuple (cx, cy, lane, obs,
beta, sigma, res_beta) must agree within 1e-4 -- its beta-CEM outputs
whenever the result candidate's trace is tie-free."""
import os

import numpy as np
import pytest

import oracle
from parity import _differ, beta_divergence, close, elite_equal

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mmdopt_n50_ref.npz")
N, O, LEVEL, H, B, T = 50, 4, 0.1, 20, 100, 2


def test_configs0_dropin_mmdopt_n50():
    from optimizer.cem import CEM
    gold = np.load(GOLD)
    prob = CEM(N, O, LEVEL, H, "gaussian", 0.0, 0.0, maxiter_cem=T)
    assert prob.num_batch == B and prob.num_mother == 2500
    ora = oracle.CEM(N, O, LEVEL, H, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=T)
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(int(gold["seed"])), idx_mpc=0, with_beta_cem=True)
    args = (int(gold["idx_mpc"]), gold["init"], gold["mean"], gold["cov"], gold["x_obs"], gold["y_obs"], 15.0)
    # the scenario separates the candidates (not every cost at the MMD floor)
    assert (gold["t0_obs"] > gold["t0_obs"].min() + 1e-2).sum() >= 10
    # the drop-in call itself (cem.py:201-204 signature, draws injected)
    got = prob.compute_cem_mmd_opt(*args, draws=draws, trace=True)
    elites = prob.last_trace
    # the same solve again, one iteration at a time, for the per-candidate checks
    h = prob.handle
    h.begin("mmd_opt", *args, draws=draws)
    parted = {}
    for t in range(T):
        h.iterate(t, 1)
        h.sync()
        obs_g, lane_g = h.read("obs_cost")[:B], h.read("lane_cost")[:B]
        res_g = h.read("res_beta").reshape(B, 20)
        esum_g = h.read("btrace").reshape(B, 20)
        sig_g = h.read("sigma")[:B]
        obs_r, lane_r = gold[f"t{t}_obs"], gold[f"t{t}_lane"]
        ok = np.abs(obs_g - obs_r) <= 1e-2 + 1e-4 * np.abs(obs_r)
        ok &= np.abs(lane_g - lane_r) <= 1e-2 + 1e-4 * np.abs(lane_r)
        ok &= np.abs(sig_g - gold[f"t{t}_sigma"]) <= 1e-6 * np.abs(gold[f"t{t}_sigma"])
        ok &= np.all(np.abs(res_g - gold[f"t{t}_res_beta"]) <= 1e-4 * np.abs(gold[f"t{t}_res_beta"]) + 1e-6, axis=1)
        ok &= ~np.any(_differ(esum_g, gold["esum"][t]), axis=1)
        beta_g = h.read("beta").reshape(B, N)
        ok &= np.all(np.abs(beta_g - gold[f"t{t}_beta"]) <= 1e-3 * np.abs(gold[f"t{t}_beta"]) + 1e-4, axis=1)
        for b in np.nonzero(~ok)[0]:
            t0, tie, detail = beta_divergence(gold[f"t{t}_res_beta"][b], gold["esum"][t, b], gold["gaps"][t, b],
                                              res_g[b], esum_g[b])
            print(f"iteration {t} candidate {b}: GPU obs {obs_g[b]} oracle {obs_r[b]}; {detail}")
            assert tie, f"iteration {t} candidate {b} differs without a qualifying near-tie ({detail})"
            parted[(t, int(b))] = detail
        # the elite sets decide the next population: they must be identical
        # (or differ only by a near-tie of their keys, which elite_equal reports)
        same = (elite_equal(f"elite_proj[{t}]", elites["elite_proj"][t], gold[f"t{t}_perm"], gold[f"t{t}_res_norm"],
                            tol=1e-3)
                and elite_equal(f"elite_obs[{t}]", elites["elite_obs"][t], gold[f"t{t}_elite_obs"], obs_r)
                and elite_equal(f"elite_cem[{t}]", elites["elite_cem"][t], gold[f"t{t}_elite_cem"],
                                gold[f"t{t}_cost20"]))
        assert same, f"iteration {t}: the elite sets differ (near-tie), the runs part before the last iteration"
    h.close()
    print(f"explained beta-CEM partings: {len(parted)} of {B * T} (candidate, iteration) pairs: {parted}")
    cx, cy, lane, obs, beta, sigma, res_beta = got
    close("cx", cx, gold["cx"], rtol=1e-4, atol=1e-4)
    close("cy", cy, gold["cy"], rtol=1e-4, atol=1e-4)
    e0 = int(elites["elite_obs"][T - 1][0])
    if (T - 1, e0) not in parted:   # the result candidate's own costs and beta-CEM outputs
        close("cost_obs", obs, gold["cost_obs"], rtol=1e-4, atol=1e-2)
        close("cost_lane", lane, gold["cost_lane"], rtol=1e-4, atol=1e-2)
        close("beta", beta[:N], gold["beta"], rtol=1e-3, atol=1e-4)
        close("sigma", sigma, gold["sigma"], rtol=1e-6, atol=0)
        close("res_beta", res_beta, gold["res_beta"], rtol=1e-4, atol=1e-6)
