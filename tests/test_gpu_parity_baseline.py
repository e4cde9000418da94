"""GPU parity of the cvar / saa / mmd_random paths against the oracle.

Stage-level lockstep: before every stage the oracle is given the GPU's
current state, so each kernel is checked in isolation on identical inputs
(front: guess + projection + controls; risk: rollouts + collision residual +
reducer; select: argsorts, cost, elites, CEM update).
"""
import numpy as np
import pytest

import oracle
from parity import DEFAULT_COV, DEFAULT_INIT, DEFAULT_MEAN, close, elite_equal, make_pair

pytestmark = pytest.mark.gpu

B, N_S, O, H, T = 32, 24, 3, 12, 3


def _sync_state(nat, st, B):
    st["pop"] = nat.read("pop")[: B * 8].reshape(B, 8).copy()
    st["mean"] = nat.read("mean")[:8].copy()
    st["cov"] = nat.read("cov")[:64].reshape(8, 8).copy()
    st["lam_x"] = nat.read("lam_x").reshape(B, 11).copy()
    st["lam_y"] = nat.read("lam_y").reshape(B, 11).copy()
    st["s_lane"] = nat.read("s_lane").reshape(B, 198).copy()


@pytest.mark.parametrize("cost,noise", [("cvar", "gaussian"), ("saa", "gaussian"), ("mmd_random", "gaussian"),
                                        ("cvar", "beta")])
def test_stage_lockstep(native, cost, noise):
    ora, nat, xo, yo = make_pair(native, cost, noise, n=N_S, O=O, H=H, B=B, T=T, acc_c=0.05, steer_c=0.01)
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(3), idx_mpc=123, seed=0, with_beta_cem=False)
    nat.begin(cost, 123, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
    st = ora.init_state(DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, draws)
    pop_gpu = nat.read("pop")[: B * 8].reshape(B, 8)
    close("pop0", pop_gpu, st["pop"], rtol=1e-6, atol=1e-6)
    for t in range(T):
        _sync_state(nat, st, B)
        if t > 0:  # population lives in the other buffer half
            st["pop"] = nat.read("pop")[(t & 1) * B * 8:(t & 1) * B * 8 + B * 8].reshape(B, 8).copy()
        nat.run_stage(1, t)
        pr, acc, steer = ora.front(st)
        close("cx", nat.read("cx").reshape(B, 11), pr["c_x"], atol=1e-4)
        close("cy", nat.read("cy").reshape(B, 11), pr["c_y"], atol=1e-4)
        traj = nat.read("traj").reshape(6, B, 100)
        for k, nm in enumerate(["x", "y", "xd", "yd", "xdd", "ydd"]):
            close(nm, traj[k], pr[nm], atol=1e-4)
        close("res_norm", nat.read("res_norm")[:B], pr["res_norm"], atol=1e-5)
        close("lam_x", nat.read("lam_x").reshape(B, 11), st["lam_x"], atol=1e-3)
        close("lam_y", nat.read("lam_y").reshape(B, 11), st["lam_y"], atol=1e-3)
        close("s_lane", nat.read("s_lane").reshape(B, 198), st["s_lane"], atol=1e-5)
        acc_g = nat.read("acc").reshape(B, 100)
        steer_g = nat.read("steer").reshape(B, 100)
        close("acc", acc_g, acc[:, :100], atol=1e-3)
        close("steer", steer_g, steer, atol=1e-5)
        # risk on the GPU's controls
        nat.run_stage(2, t)
        obs, lane, _ = ora.candidate_costs(cost, st, acc_g, steer_g, xo, yo, draws, t)
        close("obs_cost", nat.read("obs_cost")[:B], obs, atol=1e-4,
              frac_ok=0.05 if noise == "beta" else 0.0)
        close("lane_cost", nat.read("lane_cost")[:B], lane, atol=1e-4,
              frac_ok=0.05 if noise == "beta" else 0.0)
        # select on the GPU's front/risk outputs
        pr_g = dict(res_norm=nat.read("res_norm")[:B], c_x=nat.read("cx").reshape(B, 11),
                    c_y=nat.read("cy").reshape(B, 11))
        for k, nm in enumerate(["x", "y", "xd", "yd", "xdd", "ydd"]):
            pr_g[nm] = traj[k]
        obs_g = nat.read("obs_cost")[:B]
        lane_g = nat.read("lane_cost")[:B]
        nat.run_stage(3, t)
        out, info = ora.select(cost, st, t, pr_g, steer_g, obs_g, lane_g, np.float32(15.0), draws)
        tp = nat.read("tr_proj", np.int32).reshape(T, B)[t]
        to = nat.read("tr_obs", np.int32).reshape(T, 20)[t]
        tc = nat.read("tr_cem", np.int32).reshape(T, 5)[t]
        assert np.array_equal(tp, info["perm"]), "argsort(res_norm) differs on identical input"
        assert np.array_equal(to, info["elite_obs"]), "obstacle elites differ on identical input"
        assert np.array_equal(tc, info["elite_cem"]), "cost elites differ"
        nxt = ((t + 1) & 1) * B * 8
        close("pop_next", nat.read("pop")[nxt:nxt + B * 8].reshape(B, 8), st["pop"], rtol=1e-5, atol=1e-5)
        close("mean", nat.read("mean")[:8], st["mean"], rtol=1e-5, atol=1e-6)
        close("cov", nat.read("cov")[:64].reshape(8, 8), st["cov"], rtol=1e-5, atol=1e-6)
        res = nat.read("results").reshape(T, -1)[t]
        close("result_cx", res[:11], out["cx"], atol=1e-5)
        close("result_obs", res[23], out["obs"], atol=1e-5)


# Beta draws (k_beta_planes / k_beta_fix): the gamma accept / reject decisions
# are fp64 and exact, the Beta combine is fp32 on the GPU (csrc/rng.hpp:
# beta_combine) vs fp64 in the oracle -- a few ulp where the draw is not
# saturated at 0 or 1
BETA_RTOL, BETA_ATOL = 1e-5, 3e-7


@pytest.mark.parametrize("fused", ["1", "0"])
def test_beta_planes(native, monkeypatch, fused):
    """The Beta draws of the baseline rollouts against the oracle's: the
    fused rollouts (candidate lanes, draws inside the rollout; stored as
    planes only under MPCMMD_BETA_DUMP for this test) and the row-lane plane
    kernel (MPCMMD_RISK_FUSED=0)."""
    from oracle.rng import (STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B,
                            beta_draws, iteration_key)
    monkeypatch.setenv("MPCMMD_BETA_DUMP", "1")   # read when the handle is created
    monkeypatch.setenv("MPCMMD_RISK_FUSED", fused)
    ora, nat, xo, yo = make_pair(native, "cvar", "beta", n=N_S, O=O, H=H, B=B, T=T, acc_c=0.05, steer_c=0.01)
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(3), idx_mpc=123, seed=0, with_beta_cem=False)
    nat.begin("cvar", 123, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
    p = ora.prob
    worst = 0.0
    for t in range(2):
        nat.run_stage(1, t)
        nat.run_stage(2, t)
        acc = nat.read("acc").reshape(B, 100)[:, :H]
        steer = nat.read("steer").reshape(B, 100)[:, :H]
        planes = nat.read("bplane", np.float32, (B, 2, H, N_S))
        key = iteration_key(123, t, draws.seed)
        elem = np.arange(N_S, dtype=np.uint64)[:, None] * np.uint64(H) + np.arange(H, dtype=np.uint64)[None, :]
        elem = np.broadcast_to(elem, (B, N_S, H))
        for k, (ctl, sa, sb) in enumerate([(acc, STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B),
                                           (steer, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B)]):
            c = np.broadcast_to(np.abs(ctl)[:, None, :], (B, N_S, H))
            ref = beta_draws((np.float32(p.beta_a) * c).astype(np.float64),
                             (np.float32(p.beta_b) * c).astype(np.float64), key, sa, sb, elem)
            got = planes[:, k].transpose(0, 2, 1)
            err = np.abs(got.astype(np.float64) - ref)
            lim = BETA_ATOL + BETA_RTOL * np.abs(ref)
            assert np.all(err <= lim), f"beta plane {k} t={t}: {int((err > lim).sum())} outside, worst {err.max():.3g}"
            worst = max(worst, float((err / np.maximum(np.abs(ref), 1e-30)).max()))
        nat.run_stage(3, t)
    print(f"Beta draws: worst relative difference {worst:.3g}")


def run_iteration_lockstep(native, cost, noise, Tf=20, n=N_S, B=B, H=H, O=O, seed=7, idx=5):
    """20 full GPU iterations (noise, front, risk, select).  Before each, the
    oracle is synchronised to the GPU's carry and runs the same iteration on
    its own; outputs must agree within tolerance, and every elite index set
    exactly unless the differing entries are a near-tie of the sort keys
    (feasible candidates' res_norm is fp32 rounding noise of
    x - d cos(atan2), projection.py:249-265, so their order is noise)."""
    ora, nat, xo, yo = make_pair(native, cost, noise, n=n, O=O, H=H, B=B, T=Tf)
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(seed), idx_mpc=idx,
                                with_beta_cem=(cost == "mmd_opt"))
    nat.begin(cost, idx, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
    st = ora.init_state(DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, draws)
    exact = 0
    for t in range(Tf):
        _sync_state(nat, st, B)
        st["pop"] = nat.read("pop")[(t & 1) * B * 8:(t & 1) * B * 8 + B * 8].reshape(B, 8).copy()
        out = ora.iteration(cost, st, t, xo, yo, np.float32(15.0), draws, trace := [])
        tr = trace[0]
        nat.iterate(t, 1)
        nat.sync()
        frac = 0.05 if noise == "beta" else 0.0
        close(f"obs[{t}]", nat.read("obs_cost")[:B], tr["obs"], atol=1e-4, frac_ok=frac)
        close(f"lane[{t}]", nat.read("lane_cost")[:B], tr["lane"], atol=1e-4, frac_ok=frac)
        close(f"res_norm[{t}]", nat.read("res_norm")[:B], tr["res_norm"], atol=1e-5)
        tp = nat.read("tr_proj", np.int32).reshape(Tf, B)[t]
        to = nat.read("tr_obs", np.int32).reshape(Tf, 20)[t]
        tc = nat.read("tr_cem", np.int32).reshape(Tf, 5)[t]
        if not elite_equal(f"elite_proj[{t}]", tp, tr["perm"], tr["res_norm"], tol=1e-3):
            continue
        if not elite_equal(f"elite_obs[{t}]", to, tr["elite_obs"], tr["obs"]):
            continue
        if not elite_equal(f"elite_cem[{t}]", tc, tr["elite_cem"], tr["cost20"]):
            continue
        exact += 1
        nxt = ((t + 1) & 1) * B * 8
        close(f"pop[{t}]", nat.read("pop")[nxt:nxt + B * 8].reshape(B, 8), st["pop"], rtol=1e-4, atol=1e-4)
        close(f"mean[{t}]", nat.read("mean")[:8], st["mean"], rtol=1e-4, atol=1e-5)
        res = nat.read("results").reshape(Tf, -1)[t]
        close(f"result_cx[{t}]", res[:11], out["cx"], atol=1e-3)
        close(f"result_cy[{t}]", res[11:22], out["cy"], atol=1e-3)
        close(f"result_obs[{t}]", res[23], out["obs"], atol=1e-4)
    return exact


@pytest.mark.parametrize("cost,noise", [("cvar", "gaussian"), ("saa", "gaussian"), ("mmd_random", "gaussian"),
                                        ("cvar", "beta"), ("saa", "beta")])
def test_iteration_lockstep(native, cost, noise):
    exact = run_iteration_lockstep(native, cost, noise)
    # most iterations must agree exactly (near-ties are rare and reported)
    assert exact >= 15, f"only {exact}/20 iterations had identical elite sets"


def test_free_run_solve(native):
    """Unsynchronised 20-iteration solves (GPU vs oracle) on a collision-free
    scenario: both must find cost_obs == 0 and the same boundary-fixed
    coefficients (cx[0..2], cy[0..2])."""
    ora, nat, xo, yo = make_pair(native, "cvar", "gaussian", n=N_S, O=O, H=H, B=B, T=20)
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(9), idx_mpc=2, with_beta_cem=False)
    ref = ora.solve("cvar", 2, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws=draws)
    got = nat.solve("cvar", 2, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws=draws)
    assert float(ref[3]) == 0.0 and float(got["cost_obs"]) == 0.0
    close("cx[:3]", got["cx"][:3], ref[0][:3], atol=1e-4)
    close("cy[:3]", got["cy"][:3], ref[1][:3], atol=1e-4)


@pytest.mark.parametrize("cost,noise", [("cvar", "beta"), ("saa", "gaussian")])
def test_iteration_lockstep_fused_risk(native, monkeypatch, cost, noise):
    """The opt-in fused risk path (MPCMMD_RISK_FUSED=1: Beta draws inside the
    candidate-lane rollouts, k_risk_reduce) against the oracle, iteration by
    iteration, like the default row-lane path."""
    monkeypatch.setenv("MPCMMD_RISK_FUSED", "1")  # read when the handle is created
    exact = run_iteration_lockstep(native, cost, noise)
    assert exact >= 15, f"only {exact}/20 iterations had identical elite sets"
