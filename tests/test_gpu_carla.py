"""The CARLA optimizer (BASELINE configs[4]; carla/optimizer/cem.py:217-629 of
the reference) on the GPU against its restatement (oracle/carla.py): one
simulator tick of compute_cem_mmd and compute_cem_cvar at H = 60 on inputs
built from a synthetic replay tick (mpc-mmd_amd/carla/replay.py) through the
library's own path helpers, with injected draws.

Every outer iteration is checked in lockstep: per-candidate obstacle / lane /
desired-lane risks, steering and curvature of the projection, and the three
elite index sets (projection order, obstacle elites, cost elites) exact; the
returned (cx, cy, v_best, steering_best, mean_param) within 1e-4.  As for the
static mmd_opt free run (tests/test_gpu_free_run.py), a candidate whose
beta-CEM parted from the oracle's is accepted only at the near-tie that
explains it (tests/parity.py: beta_divergence), and must not move an elite set.
"""
import importlib
import importlib.util
import os
import sys

import numpy as np
import pytest

from oracle import beta_cem as bc
from oracle import carla as K
from oracle import helper as Hh
from parity import beta_near_tie, close

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CARLA = os.path.join(ROOT, "mpc-mmd_amd", "carla")


def _replay():
    spec = importlib.util.spec_from_file_location("mpcmmd_carla_replay", os.path.join(CARLA, "replay.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def carla_package():
    """The CARLA drop-in package (mpc-mmd_amd/carla/optimizer).  It is named
    ``optimizer`` like the static one (the reference has two packages of that
    name), so the tests, which already import the static package, load it
    under an alias."""
    name = "mpcmmd_carla_optimizer"
    if name not in sys.modules:
        d = os.path.join(CARLA, "optimizer")
        spec = importlib.util.spec_from_file_location(name, os.path.join(d, "__init__.py"),
                                                      submodule_search_locations=[d])
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
    return name


def _tick(k, num_obs=3, H=60):
    R = _replay()
    Helper = importlib.import_module(carla_package() + ".cem_helper").Helper
    rec = R.record_synthetic(ticks=k + 1)
    return R.tick_inputs(rec, k, Helper(num_prime=H), num_obs)


MEAN = np.array([10.0] * 4 + [0.0] * 4, np.float32)               # main_carla.py:306-318 (v_des = 10, y = 0)
COV = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)


def _beta_trace_carla(ora, st, acc, steer, draws, t):
    """The oracle's beta-CEM of one candidate at outer iteration t (CARLA
    mother rollouts from the noisy initial rows)."""
    p = ora.prob
    H = p.num_prime
    acc_n, steer_n = Hh.noisy_controls(p, acc[None, :H], steer[None, :H], draws, t, p.num_reduced)
    acc_m, steer_m = Hh.mother_controls(acc_n, steer_n)
    xm, ym = K.rollout_cr(p, acc_m, steer_m, st["rows0"][None, :, :])
    cxm, cym = Hh.compute_coeff(p, xm, ym)
    trace = []
    beta, res, sigma, sel = bc.compute_cem(p, cxm[0], cym[0], draws.beta_z0, draws.beta_z, trace)
    return dict(beta=beta, res=res, sigma=sigma, sel=sel, trace=trace)


def _sync_carry(nat, st, t, B):
    """The oracle continues from the GPU's carry (population of iteration t,
    CEM mean / covariance, ADMM multipliers and lane slacks)."""
    st["pop"] = nat.read("pop")[(t & 1) * B * 8:(t & 1) * B * 8 + B * 8].reshape(B, 8).copy()
    st["mean"] = nat.read("mean")[:8].copy()
    st["cov"] = nat.read("cov")[:64].reshape(8, 8).copy()
    st["lam_x"] = nat.read("lam_x").reshape(-1, 11)[:B].copy()
    st["lam_y"] = nat.read("lam_y").reshape(-1, 11)[:B].copy()
    st["s_lane"] = nat.read("s_lane").reshape(-1, 198)[:B].copy()


@pytest.mark.parametrize("n,B,noise,const", [(4, 24, "gaussian", (0.0, 0.0)), (10, 100, "gaussian", (0.0, 0.0)),
                                              (10, 100, "beta", (0.0, 0.0)), (4, 24, "gaussian", (0.05, 0.01)),
                                              (4, 24, "beta", (0.05, 0.01))])
def test_carla_mmd_iteration_lockstep(native, n, B, noise, const):
    """compute_cem_mmd, 20 iterations with the oracle synchronised to the GPU's
    carry before each one, at a small shape and at the timed configs[4] shape
    (n = 10: 100 mother rows, B = 100, H = 60, O = 3; bench.py's CARLA line).
    A free run cannot stay in lockstep (test_carla_mmd_free_run): the CARLA
    lane risk (weight 0.01) carries the beta-CEM's fp32 MMD values (GPU vs
    oracle ~1e-7 relative) into the CEM weights, so from the second iteration
    the populations differ in ulps, and the projection order of feasible
    candidates is rounding noise of those.  Given the same carry,
    every iteration's risks must agree (beta-CEM partings only at explaining
    near-ties) and every elite set exactly, or at a reported near-tie.
    noise = "beta": the mother rollouts draw Beta(2|u|, 5|u|) (C/opt/
    cem_helper.py:822-834); const = (acc_const_noise, steer_const_noise) added
    to both CARLA rollouts times the const normals (:783-784, :837-838)."""
    from parity import elite_equal
    tick, town, H, O, T = 60, "Town05", 60, 3, 20
    level = 0.1 if noise == "gaussian" else 0.3
    init, xo, yo, path = _tick(tick, O, H)
    ora = K.CarlaCEM(n, 1, O, level, H, noise, town, const[0], const[1], num_batch=B, maxiter_cem=T)
    nat = native.Handle(native.make_config(n, O, level, H, noise, const[0], const[1], num_batch=B, maxiter_cem=T,
                                           variant="carla_town05"))
    idx = 5
    draws = K.CarlaDraws.random(ora.prob, np.random.default_rng(7), idx_mpc=idx, with_beta_cem=True)
    nat.carla_begin("mmd_opt", idx, init, MEAN, COV, xo, yo, 10.0, path, draws)
    st = ora.init_carla("mmd_opt", init, MEAN, COV, path, draws)
    R = st["rows0"].shape[0]
    assert np.array_equal(nat.read("st0r").reshape(-1, 8)[:R, :5], st["rows0"]), "noisy initial rows differ"
    exact, parted = 0, {}
    for t in range(T):
        _sync_carry(nat, st, t, B)
        st0 = dict(st)
        pr, acc, steer = ora.front_carla(st, path)
        obs, lane, des, extra = ora.candidate_costs_carla("mmd_opt", st, acc, steer, xo, yo, path, draws, t)
        out, info = ora.select_carla("mmd_opt", st, t, pr, steer, obs, lane, des, np.float32(10.0), draws, extra)
        nat.iterate(t, 1)
        nat.sync()
        close(f"steer[{t}]", nat.read("steer").reshape(-1, 100)[:B], steer, rtol=0, atol=0)
        close(f"kappa[{t}]", nat.read("kappa_i").reshape(-1, 100)[:B], pr["kappa"], rtol=0, atol=0)
        close(f"res_norm[{t}]", nat.read("res_norm")[:B], pr["res_norm"], rtol=0, atol=0)
        obs_g, lane_g, des_g = nat.read("obs_cost")[:B], nat.read("lane_cost")[:B], nat.read("lane_des")[:B]
        ok = np.abs(obs_g - obs) <= 1e-2 + 1e-4 * np.abs(obs)
        ok &= np.abs(lane_g - lane) <= 1e-2 + 1e-4 * np.abs(lane)
        ok &= np.abs(des_g - des) <= 1e-2 + 1e-4 * np.abs(des)
        res_g = nat.read("res_beta").reshape(-1, 20)[:B]
        inner = np.all(np.abs(res_g - extra["res_beta"]) <= 1e-4 * np.abs(extra["res_beta"]) + 1e-6, axis=1)
        inner &= np.abs(nat.read("sigma")[:B] - extra["sigma"]) <= 1e-6 * np.abs(extra["sigma"])
        if not inner.all():
            acc_g = nat.read("acc").reshape(-1, 100)[:B]
            esum_g = nat.read("btrace").reshape(-1, 20)[:B]
            for b in np.nonzero(~inner)[0]:
                _, tie, detail = beta_near_tie(_beta_trace_carla(ora, st0, acc_g[b], steer[b], draws, t), res_g[b],
                                               esum_g[b])
                assert tie, f"iteration {t} candidate {b}: beta-CEM differs without a near-tie ({detail})"
                parted[(t, int(b))] = detail
        bad = np.nonzero(~ok)[0]
        assert all((t, int(b)) in parted for b in bad), f"iteration {t}: risks of {bad} differ, beta-CEM equal"
        tp = nat.read("tr_proj", np.int32).reshape(T, B)[t]
        to = nat.read("tr_obs", np.int32).reshape(T, 20)[t]
        tc = nat.read("tr_cem", np.int32).reshape(T, 5)[t]
        assert np.array_equal(tp, info["perm"]), f"iteration {t}: projection order differs (same carry)"
        if not elite_equal(f"elite_obs[{t}]", to, info["elite_obs"], obs):
            continue
        if not elite_equal(f"elite_cem[{t}]", tc, info["elite_cem"], info["cost20"]):
            continue
        exact += 1
        close(f"mean[{t}]", nat.read("mean")[:8], st["mean"], rtol=1e-4, atol=1e-5)
        close(f"res_steer[{t}]", nat.read("res_steer").reshape(-1, 100)[t], out["steer"], rtol=1e-4, atol=1e-6)
        res = nat.read("results").reshape(T, -1)[t]
        close(f"result_cx[{t}]", res[:11], out["cx"], atol=1e-4)
        close(f"result_cy[{t}]", res[11:22], out["cy"], atol=1e-4)
    assert exact >= 15, f"only {exact}/20 iterations had identical elite sets"
    got = nat.finish()
    assert got["v_best"].shape == (100,) and np.all(np.isfinite(got["steering"]))
    print(f"CARLA mmd_opt n={n} B={B} {noise} const {const}: {exact}/20 iterations with identical elite sets; "
          f"partings {parted}")


@pytest.mark.parametrize("cost,n,B,tick,town,noise,const", [
    ("cvar", 16, 100, 60, "Town05", "gaussian", (0.0, 0.0)),
    ("cvar", 12, 100, 170, "Town10HD", "gaussian", (0.0, 0.0)),
    ("cvar", 12, 100, 60, "Town05", "beta", (0.0, 0.0)),
    ("cvar", 12, 100, 60, "Town05", "gaussian", (0.05, 0.01)),
    ("cvar", 260, 20, 60, "Town05", "gaussian", (0.0, 0.0))])
def test_carla_tick_lockstep(native, cost, n, B, tick, town, noise, const):
    """compute_cem_cvar, 20 free-running iterations in lockstep with the oracle.
    Beta noise (main_carla.py --noises beta; C/opt/cem_helper.py:768-777): both
    sides draw Beta(2|u|, 5|u|) from the same Philox streams, the CARLA
    variant's combine in fp64 rounded once (rng.hpp: beta_combine_cr), so the
    draws, rollouts and risks are the oracle's bit for bit, as for Gaussian
    noise (a draw a few ulp off would move a risk by a Frenet path step).
    const: acc / steer const noise (C/opt/cem_helper.py:783-784).  n = 260
    rows (> 256): k_risk_carla's per-row maxima walk the rows with a stride."""
    H, O, T = 60, 3, 20
    level = 0.1 if noise == "gaussian" else 0.3
    init, xo, yo, path = _tick(tick, O, H)
    ora = K.CarlaCEM(n, 1, O, level, H, noise, town, const[0], const[1], num_batch=B, maxiter_cem=T)
    variant = "carla_town10hd" if town == "Town10HD" else "carla_town05"
    nat = native.Handle(native.make_config(n, O, level, H, noise, const[0], const[1], num_batch=B, maxiter_cem=T,
                                           variant=variant))
    idx = 5
    draws = K.CarlaDraws.random(ora.prob, np.random.default_rng(7), idx_mpc=idx, with_beta_cem=(cost == "mmd_opt"))
    trace = []
    ref = ora.solve_carla(cost, idx, init, MEAN, COV, xo, yo, 10.0, path, draws, trace=trace)
    nat.carla_begin(cost, idx, init, MEAN, COV, xo, yo, 10.0, path, draws)
    # the per-solve setup: noisy initial rows and the boundary vectors they give
    st0 = ora.init_carla(cost, init, MEAN, COV, path, draws)
    R = st0["rows0"].shape[0]
    assert np.array_equal(nat.read("st0r").reshape(-1, 8)[:R, :5], st0["rows0"]), "noisy initial rows differ"
    parted = {}
    for t in range(T):
        nat.iterate(t, 1)
        nat.sync()
        tr = trace[t]
        # bit-exact while the carries are (cvar; mmd_opt's first iteration).  From
        # mmd_opt's second iteration on the population carries the beta-CEM's
        # fp32 MMD costs (GPU vs oracle ~1e-7 relative) through the CEM weights
        tol = (0.0, 0.0) if cost == "cvar" or t == 0 else (1e-4, 1e-6)
        close(f"steer[{t}]", nat.read("steer").reshape(-1, 100)[:B], tr["steer"], rtol=tol[0], atol=tol[1])
        close(f"kappa[{t}]", nat.read("kappa_i").reshape(-1, 100)[:B], tr["kappa"], rtol=tol[0], atol=tol[1])
        obs_g, lane_g, des_g = nat.read("obs_cost")[:B], nat.read("lane_cost")[:B], nat.read("lane_des")[:B]
        fl = 1e-2 if cost == "mmd_opt" else 1e-5
        ok = np.abs(obs_g - tr["obs"]) <= fl + 1e-4 * np.abs(tr["obs"])
        ok &= np.abs(lane_g - tr["lane"]) <= fl + 1e-4 * np.abs(tr["lane"])
        ok &= np.abs(des_g - tr["des"]) <= fl + 1e-4 * np.abs(tr["des"])
        if cost == "mmd_opt":
            res_g = nat.read("res_beta").reshape(-1, 20)[:B]
            inner = np.all(np.abs(res_g - tr["res_beta"]) <= 1e-4 * np.abs(tr["res_beta"]) + 1e-6, axis=1)
            inner &= np.abs(nat.read("sigma")[:B] - tr["sigma"]) <= 1e-6 * np.abs(tr["sigma"])
            if not inner.all():
                acc = nat.read("acc").reshape(-1, 100)[:B]
                steer = nat.read("steer").reshape(-1, 100)[:B]
                esum_g = nat.read("btrace").reshape(-1, 20)[:B]
                for b in np.nonzero(~inner)[0]:
                    _, tie, detail = beta_near_tie(_beta_trace_carla(ora, st0, acc[b], steer[b], draws, t), res_g[b],
                                                   esum_g[b])
                    assert tie, f"iteration {t} candidate {b}: beta-CEM differs without a near-tie ({detail})"
                    parted[(t, int(b))] = detail
            bad = np.nonzero(~ok)[0]
            assert all((t, int(b)) in parted for b in bad), f"iteration {t}: risks of {bad} differ, beta-CEM equal"
        else:
            assert ok.all(), (f"iteration {t}: candidates {np.nonzero(~ok)[0]} differ: obs {obs_g[~ok]} vs "
                              f"{tr['obs'][~ok]}, lane {lane_g[~ok]} vs {tr['lane'][~ok]}")
        tp = nat.read("tr_proj", np.int32).reshape(T, B)[t]
        to = nat.read("tr_obs", np.int32).reshape(T, 20)[t]
        tc = nat.read("tr_cem", np.int32).reshape(T, 5)[t]
        assert np.array_equal(tp, tr["perm"]), f"iteration {t}: projection order differs"
        assert np.array_equal(to, tr["elite_obs"]), f"iteration {t}: obstacle elites {to} vs {tr['elite_obs']}"
        assert np.array_equal(tc, tr["elite_cem"]), f"iteration {t}: cost elites {tc} vs {tr['elite_cem']}"
    got = nat.finish()
    cx, cy, v_best, steer_best, mean_param, out = ref
    close("cx", got["cx"], cx, rtol=1e-4, atol=1e-4)
    close("cy", got["cy"], cy, rtol=1e-4, atol=1e-4)
    close("v_best", got["v_best"], v_best, rtol=1e-4, atol=1e-4)
    close("steering", got["steering"], steer_best, rtol=1e-4, atol=1e-5)
    close("mean_param", got["mean_param"], mean_param, rtol=1e-4, atol=1e-4)
    print(f"CARLA {cost}/{noise} const {const} n={n} B={B} {town} tick {tick}: 20 iterations in lockstep; obs "
          f"{float(got['cost_obs'])} lane {float(got['cost_lane'])}; explained beta-CEM partings {parted}")


def test_carla_dropin_interface(native):
    """The drop-in class with the reference's constructor and call signature
    (carla/main_carla.py:186-194, 378-382) returns the reference's tuple."""
    cem = importlib.import_module(carla_package() + ".cem")
    prob = cem.CEM(4, 1, 3, 0.1, 60, "gaussian", "Town05", 0.0, 0.0)
    init, xo, yo, path = _tick(40, 3, 60)
    for fn in (prob.compute_cem_mmd, prob.compute_cem_cvar, prob.compute_cem_det):
        cx, cy, v, steer, mean = fn(1, init, MEAN, COV, xo, yo, 10.0, path["x_path"], path["y_path"],
                                    path["arc_vec"], path["Fx_dot"], path["Fy_dot"], path["kappa"])
        assert cx.shape == (11,) and cy.shape == (11,) and v.shape == (100,) and steer.shape == (100,)
        assert mean.shape == (8,) and np.all(np.isfinite(cx)) and np.all(np.isfinite(steer))
        assert np.all(np.abs(steer) < np.pi / 2)
    # cem.py:161-166: only "Town10HD" selects its constants (Town10HD_Opt gets Town05's)
    opt = cem.CEM(4, 1, 3, 0.1, 60, "gaussian", "Town10HD_Opt", 0.0, 0.0)
    assert (opt.y_lb, opt.y_ub, opt.y_des_2) == (-3.8, 0.3, -3.5)


@pytest.mark.parametrize("n,B,tick,town", [(10, 100, 60, "Town05"), (10, 100, 170, "Town10HD")])
def test_carla_det_lockstep(native, n, B, tick, town):
    """compute_cem_det (carla/optimizer/cem.py:633-790) against the oracle's
    restatement of it and of projection_det.py, 20 free-running iterations at
    the configs[4] shape (H = 60, B = 100, 3 obstacles): the projection with
    its obstacle terms live, then the elites of the projection order with
    zero risk terms.  Every iteration's projection order, elites and cost
    elites exact; res_norm, steering, curvature and the multipliers within
    fp32 rounding; the returned tuple within 1e-4."""
    H, O, T, level = 60, 3, 20, 0.1
    init, xo, yo, path = _tick(tick, O, H)
    ora = K.CarlaCEM(n, 1, O, level, H, "gaussian", town, 0.0, 0.0, num_batch=B, maxiter_cem=T)
    variant = "carla_town10hd" if town == "Town10HD" else "carla_town05"
    cfg = native.make_config(n, O, level, H, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=T, variant=variant)
    for xy in ("x", "y"):   # the det KKT inverse (A_obs^T A_obs in the cost) bit-identical to the oracle's
        assert np.array_equal(native.host_constant(cfg, f"det_kinv_{xy}"),
                              ora.prob.det_kinv()[0 if xy == "x" else 1].reshape(-1))
    nat = native.Handle(cfg)
    idx = 5
    draws = K.CarlaDraws.random(ora.prob, np.random.default_rng(11), idx_mpc=idx, with_beta_cem=False)
    trace = []
    ref = ora.solve_det(idx, init, MEAN, COV, xo, yo, 10.0, path, draws, trace=trace)
    nat.carla_begin("det", idx, init, MEAN, COV, xo, yo, 10.0, path, draws)
    st0 = ora.init_carla("det", init, MEAN, COV, path, draws)
    assert np.array_equal(nat.read("st0r").reshape(-1, 8)[:1, :5], st0["rows0"]), "noisy initial state differs"
    for t in range(T):
        nat.iterate(t, 1)
        nat.sync()
        tr = trace[t]
        close(f"res_norm[{t}]", nat.read("res_norm")[:B], tr["res_norm"], rtol=1e-5, atol=1e-6)
        close(f"steer[{t}]", nat.read("steer").reshape(-1, 100)[:B], tr["steer"], rtol=1e-4, atol=1e-5)
        close(f"kappa[{t}]", nat.read("kappa_i").reshape(-1, 100)[:B], tr["kappa"], rtol=1e-4, atol=1e-6)
        close(f"lam_x[{t}]", nat.read("lam_x").reshape(-1, 11)[:B], tr["lam_x"], rtol=1e-4, atol=1e-3)
        close(f"lam_y[{t}]", nat.read("lam_y").reshape(-1, 11)[:B], tr["lam_y"], rtol=1e-4, atol=1e-3)
        tp = nat.read("tr_proj", np.int32).reshape(T, B)[t]
        to = nat.read("tr_obs", np.int32).reshape(T, 20)[t]
        tc = nat.read("tr_cem", np.int32).reshape(T, 5)[t]
        assert np.array_equal(tp, tr["perm"]), f"iteration {t}: projection order differs"
        assert np.array_equal(to, tr["perm"][:20]) and np.array_equal(to, tr["elite_obs"]), \
            f"iteration {t}: det elites are the projection order's first 20"
        assert np.array_equal(tc, tr["elite_cem"]), f"iteration {t}: cost elites {tc} vs {tr['elite_cem']}"
        close(f"mean[{t}]", nat.read("mean")[:8], tr["mean"], rtol=1e-4, atol=1e-5)
    got = nat.finish()
    cx, cy, v_best, steer_best, mean_param, out = ref
    close("cx", got["cx"], cx, rtol=1e-4, atol=1e-4)
    close("cy", got["cy"], cy, rtol=1e-4, atol=1e-4)
    close("v_best", got["v_best"], v_best, rtol=1e-4, atol=1e-4)
    close("steering", got["steering"], steer_best, rtol=1e-4, atol=1e-5)
    close("mean_param", got["mean_param"], mean_param, rtol=1e-4, atol=1e-4)
    assert float(got["cost_obs"]) == 0.0 and float(got["cost_lane"]) == 0.0
    print(f"CARLA det n={n} B={B} {town} tick {tick}: 20 iterations in lockstep; res_norm range "
          f"{float(trace[-1]['res_norm'].min()):.3f}..{float(trace[-1]['res_norm'].max()):.3f}")


@pytest.mark.parametrize("tick,town", [(60, "Town05"), (170, "Town10HD")])
def test_carla_mmd_free_run(native, tick, town):
    """compute_cem_mmd at the timed configs[4] shape (n = 10, B = 100, H = 60,
    O = 3), GPU and oracle each on their own carry for all 20 iterations (no
    state copied between them).  While the populations are bit-equal, every
    iteration is checked as in the lockstep test (risks, elite sets; beta-CEM
    partings only at explaining near-ties).  The first iteration after which
    the populations differ is the parting: it must come from the CEM weights
    (the mean and covariance agree to fp32 rounding there: the lane / obstacle
    MMD values are fp32 sums of v_exp_f32 terms, ~1e-7 relative from the
    oracle's), and it is reported.  Without a parting the returned (cx, cy,
    v_best, steering, mean_param) must agree within 1e-4.  After a parting the
    bound is the oracle's own sensitivity at that point (tests/carla_ensemble.py):
    sixteen oracle runs resume from the oracle's carry at the parting iteration
    with that iteration's risks shifted by 1-2 ulp per candidate (the size of
    the GPU-vs-oracle difference).  Per returned quantity the GPU's distance
    from the oracle must be within 1.25 x the ensemble's diameter, and its
    plan must cost (compute_cost, C/opt/cem_helper.py:522-556, on the
    noise-free plan: oracle/carla.py plan_cost) no more than the ensemble's
    worst widened by half the ensemble's cost range (carla_ensemble.py says
    why the bounds are widened)."""
    import carla_ensemble as E
    n, B, H, O, T, level = 10, 100, 60, 3, 20, 0.1
    init, xo, yo, path = _tick(tick, O, H)
    ora = K.CarlaCEM(n, 1, O, level, H, "gaussian", town, 0.0, 0.0, num_batch=B, maxiter_cem=T)
    variant = "carla_town10hd" if town == "Town10HD" else "carla_town05"
    nat = native.Handle(native.make_config(n, O, level, H, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=T,
                                           variant=variant))
    idx = 9
    draws = K.CarlaDraws.random(ora.prob, np.random.default_rng(13), idx_mpc=idx, with_beta_cem=True)
    trace, snaps = [], []
    ref = ora.solve_carla("mmd_opt", idx, init, MEAN, COV, xo, yo, 10.0, path, draws, trace=trace, snapshots=snaps)
    nat.carla_begin("mmd_opt", idx, init, MEAN, COV, xo, yo, 10.0, path, draws)
    st0 = ora.init_carla("mmd_opt", init, MEAN, COV, path, draws)
    parting, beta_parted = None, {}
    for t in range(T):
        nat.iterate(t, 1)
        nat.sync()
        if parting is not None:
            continue
        tr = trace[t]
        pop_g = nat.read("pop")[((t + 1) & 1) * B * 8:((t + 1) & 1) * B * 8 + B * 8].reshape(B, 8)
        res_g = nat.read("res_beta").reshape(-1, 20)[:B]
        inner = np.all(np.abs(res_g - tr["res_beta"]) <= 1e-4 * np.abs(tr["res_beta"]) + 1e-6, axis=1)
        if not inner.all():
            acc_g = nat.read("acc").reshape(-1, 100)[:B]
            esum_g = nat.read("btrace").reshape(-1, 20)[:B]
            for b in np.nonzero(~inner)[0]:
                _, tie, detail = beta_near_tie(_beta_trace_carla(ora, st0, acc_g[b], tr["steer"][b], draws, t),
                                               res_g[b], esum_g[b])
                assert tie, f"iteration {t} candidate {b}: beta-CEM differs without a near-tie ({detail})"
                beta_parted[(t, int(b))] = detail
        tp = nat.read("tr_proj", np.int32).reshape(T, B)[t]
        to = nat.read("tr_obs", np.int32).reshape(T, 20)[t]
        assert np.array_equal(tp, tr["perm"]), f"iteration {t}: projection order differs on equal populations"
        if not np.array_equal(to, tr["elite_obs"]):
            from parity import elite_equal
            elite_equal(f"elite_obs[{t}]", to, tr["elite_obs"], tr["obs"])   # only at a near-tie
        if not np.array_equal(pop_g, tr["pop"]):   # the population of iteration t + 1 (after the CEM update)
            parting = t
            close(f"mean at the parting ({t})", nat.read("mean")[:8], tr["mean"], rtol=1e-5, atol=1e-6)
    got = nat.finish()
    cx, cy, v_best, steer_best, mean_param, out = ref
    dv = float(np.max(np.abs(got["v_best"] - v_best)))
    dy = float(np.max(np.abs(got["cy"] - cy)))
    dm = float(np.max(np.abs(got["mean_param"] - mean_param)))
    print(f"CARLA mmd free run n={n} B={B} {town} tick {tick}: parting after iteration {parting}; "
          f"beta-CEM near-tie partings {beta_parted}; final |dv_best| {dv:.3g} |dcy| {dy:.3g} |dmean| {dm:.3g}")
    if parting is None:
        close("cx", got["cx"], cx, rtol=1e-4, atol=1e-4)
        close("cy", got["cy"], cy, rtol=1e-4, atol=1e-4)
        close("v_best", got["v_best"], v_best, rtol=1e-4, atol=1e-4)
        close("steering", got["steering"], steer_best, rtol=1e-4, atol=1e-5)
        close("mean_param", got["mean_param"], mean_param, rtol=1e-4, atol=1e-4)
        return
    # the oracle's sensitivity to an ulp at the parting iteration (carla_ensemble.py)
    members = E.run((n, B, H, O, T, level, town, idx, 13), (init, xo, yo, path), parting, snaps[parting])
    members.append(dict(cx=cx, cy=cy, v_best=v_best, steering=steer_best, mean_param=mean_param,
                        cost=K.plan_cost(ora.prob, "mmd_opt", cx, cy, steer_best, xo, yo, path, 10.0)))
    refd = members.pop()
    rep = E.spread_check(got, refd, members)
    cost_gpu = K.plan_cost(ora.prob, "mmd_opt", got["cx"], got["cy"], got["steering"], xo, yo, path, 10.0)
    costs = [m["cost"] for m in members] + [refd["cost"]]
    print(f"  ensemble of {len(members)} + oracle (parting iteration {parting}): GPU distance / ensemble "
          f"diameter { {k: (round(d, 4), round(w, 4)) for k, (d, w) in rep.items()} }; plan cost GPU "
          f"{cost_gpu:.6g}, ensemble {min(costs):.6g}..{max(costs):.6g}")
    for k, (d, diam) in rep.items():
        assert d <= 1.25 * diam + 1e-4, (f"{k}: the GPU solve is {d:.4g} from the oracle's, beyond the oracle's own "
                                         f"ulp-sensitivity (ensemble diameter {diam:.4g}) at the parting "
                                         f"iteration {parting}")
    assert cost_gpu <= E.cost_bound(costs), \
        f"the GPU plan costs {cost_gpu}, above the ensemble's {min(costs)}..{max(costs)}"
