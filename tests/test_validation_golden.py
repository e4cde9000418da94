"""Monte-Carlo validation pinned to the REFERENCE's own numbers.

tests/golden/validation_ref.npz was produced by executing the reference's
pure-NumPy functions of S/validation.py:21-171 (and D/validation.py:21-165)
on four cases (static / dynamic obstacles, gaussian / beta noise), with the
reference's own RNG (np.random.seed(key) + multivariate_normal / beta);
tests/golden/make_validation_golden.py is the generating script.

CPU: the oracle's restatement (controls, the draw sequence, the fp64
rollouts, the counts) reproduces the reference's controls and rollouts to
~1e-9 and its counts exactly.
GPU: the drop-in optimizer.validation entry points (mpcmmd_validate), fed
the same NumPy draws, return the reference's counts bit for bit.
Also the stats-file writer (S/validation.py:279-302, 459-464): key layout
and the set-intersection selection of configurations.
"""
import os

import numpy as np
import pytest

import oracle
from oracle import costs as Co
from oracle import helper as Hh
from oracle import validation as V
from oracle.problem import Problem

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "validation_ref.npz")


def _cases():
    d = np.load(GOLD)
    H, O = int(d["num_prime"]), int(d["num_obs"])
    out = []
    for name in d["cases"]:
        g = {k[len(name) + 1:]: d[k] for k in d.files if k.startswith(str(name) + "_")}
        g = {k: (v.item() if v.ndim == 0 else v) for k, v in g.items()}
        out.append((str(name), g, H, O))
    return out


CASES = _cases()
IDS = [c[0] for c in CASES]


@pytest.mark.parametrize("name,g,H,O", CASES, ids=IDS)
def test_oracle_pinned_to_reference(name, g, H, O):
    prob = Problem(10, O, g["level"], H, g["noise"], g["acc_c"], g["steer_c"], variant=g["variant"])
    acc, steer = V.controls(prob, g["cx"], g["cy"])
    np.testing.assert_allclose(acc, g["acc"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(steer, g["steer"], rtol=1e-12, atol=1e-14)
    draws = V.draws_numpy(g["noise"], acc, steer, 1000, H, g["key"])
    c, cl, xr, yr = V.compute_stats(prob, g["cx"], g["cy"], g["init_state"], g["x_obs_traj"], g["y_obs_traj"],
                                    g["noise"], g["level"], g["acc_c"], g["steer_c"], draws, return_rollouts=True)
    np.testing.assert_allclose(xr, g["x_roll"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(yr, g["y_roll"], rtol=0, atol=1e-9)
    assert (c, cl) == (g["count"], g["count_lane"])


@pytest.mark.gpu
@pytest.mark.parametrize("name,g,H,O", CASES, ids=IDS)
def test_gpu_validate_pinned_to_reference(name, g, H, O):
    from optimizer import validation as DV
    from optimizer.cem import CEM
    prob = CEM(10, O, g["level"], H, g["noise"], g["acc_c"], g["steer_c"], variant=g["variant"])
    oprob = Problem(10, O, g["level"], H, g["noise"], g["acc_c"], g["steer_c"], variant=g["variant"])
    acc, steer = V.controls(oprob, g["cx"], g["cy"])
    draws = V.draws_numpy(g["noise"], acc, steer, 1000, H, g["key"])
    if g["variant"] == "static":
        got = DV.compute_stats(prob, g["cx"], g["cy"], g["init_state"], g["x_obs"], g["y_obs"], g["vx_obs"],
                               g["vy_obs"], H, g["level"], g["noise"], O, g["key"], draws=draws)
    else:
        got = DV.compute_stats_tracks(prob, g["cx"], g["cy"], g["init_state"], g["x_obs_traj"], g["y_obs_traj"], H,
                                      g["level"], g["noise"], O, g["key"], draws=draws)
    prob.handle.close()
    assert got == (g["count"], g["count_lane"])


def _hot_path_rollouts(g, H, O):
    """The OPTIMIZER's fp32 noise injection and rollout (oracle/helper.py:
    inject_noise, rollout; cem_helper.py:380-464) driven by the reference's
    own controls and NumPy draws of the fixture case."""
    prob = Problem(1000, O, g["level"], H, g["noise"], g["acc_c"], g["steer_c"], variant=g["variant"])
    draws = V.draws_numpy(g["noise"], g["acc"], g["steer"], 1000, H, g["key"])
    acc = np.asarray(g["acc"][:H], np.float32)[None]
    steer = np.asarray(g["steer"][:H], np.float32)[None]
    na, ns, nc = (np.asarray(d, np.float32) for d in draws)
    if g["noise"] == "gaussian":
        acc_n, steer_n = Hh.inject_noise(prob, acc, steer, na, ns, nc)
    else:
        acc_n, steer_n = Hh.inject_noise(prob, acc, steer, None, None, nc, beta_acc=na[None], beta_steer=ns[None])
    xr, yr = Hh.rollout(prob, acc_n, steer_n, Hh.initial_state5(g["init_state"]))
    return prob, draws, xr[0], yr[0]


@pytest.mark.parametrize("name,g,H,O", CASES, ids=IDS)
def test_hot_path_oracle_pinned_to_reference(name, g, H, O):
    """The fp32 hot-path restatement that every GPU parity test checks
    against (compute_controls, the noise injection, the bicycle scan,
    compute_f_bar, compute_lane_bar, the CVaR reducer) reproduces the
    REFERENCE-executed controls, rollouts and residuals of
    S/validation.py:21-132 (the same formulas as S/opt/cem_helper.py:380-464,
    540-551 and S/opt/costs.py:50-71) within fp32 rounding."""
    prob, draws, xr, yr = _hot_path_rollouts(g, H, O)
    # controls from the saved coefficients, fp32 like the optimizer (Pdot_jax . c)
    f = lambda M, c: (M.astype(np.float64) @ np.asarray(c, np.float64)).astype(np.float32)[None]
    acc, steer = Hh.compute_controls(prob, f(prob.Pdot, g["cx"]), f(prob.Pdot, g["cy"]), f(prob.Pddot, g["cx"]),
                                     f(prob.Pddot, g["cy"]))
    np.testing.assert_allclose(acc[0], g["acc"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(steer[0], g["steer"], rtol=1e-4, atol=1e-5)
    # rollouts: fp32 scan vs the reference's fp64 one over 20 steps
    np.testing.assert_allclose(xr, g["x_roll"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(yr, g["y_roll"], rtol=1e-5, atol=1e-4)
    # per-element collision residual and lane bars
    xo = np.asarray(g["x_obs_traj"], np.float32)[:, :H]
    yo = np.asarray(g["y_obs_traj"], np.float32)[:, :H]
    fb = Co.compute_f_bar(prob, xr, yr, xo, yo)
    np.testing.assert_allclose(fb, g["f_bar"], rtol=0, atol=1e-4)
    # only elements at the ellipse boundary may change sides
    flip = (fb > 0) != (g["f_bar"] > 0)
    assert np.all(np.abs(g["f_bar"][flip]) < 1e-4), np.abs(g["f_bar"][flip]).max()
    lb, ub = Co.lane_bar(prob, yr)
    np.testing.assert_allclose(lb, g["lane_lb"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(ub, g["lane_ub"], rtol=0, atol=1e-4)
    # the risk reducers over those residuals (costs.py:206-234)
    cb_ref = g["f_bar"].max(axis=(0, 2)).astype(np.float32)
    cb = Co.compute_f_bar_max(prob, xr, yr, xo, yo)
    assert abs(float(Co.cvar(prob, cb)) - float(Co.cvar(prob, cb_ref))) < 1e-4
    assert abs(float(Co.saa(prob, cb)) - float(Co.saa(prob, cb_ref))) <= 2e-3


def test_static_scenarios_pinned_to_reference():
    """The sweep's scenario generator is the reference driver's, executed:
    compute_obs_data(num_obs, k) of S/main_mpc.py:10-21 and the idx_mpc
    np.random.randint(1, 10000) drawn after it (:114), k < 200."""
    from optimizer.sweep import static_obstacles
    d = np.load(GOLD)
    for O in (2, 4, 9):
        for k in range(200):
            ob = static_obstacles(k, O)
            assert np.array_equal(ob["x"], d[f"obs_{O}_x"][k]), (O, k)
            assert np.array_equal(ob["y"], d[f"obs_{O}_y"][k]), (O, k)
            assert ob["idx_mpc"] == d[f"obs_{O}_idx"][k], (O, k)


GAUSS = [c for c in CASES if c[1]["noise"] == "gaussian"]


@pytest.mark.gpu
@pytest.mark.parametrize("cost", ["cvar", "saa"])
@pytest.mark.parametrize("name,g,H,O", GAUSS, ids=[c[0] for c in GAUSS])
def test_gpu_risk_pinned_to_reference(native, name, g, H, O, cost):
    """k_risk_baseline (S = 1000 noisy rollouts, H = 20, O = 4) fed the
    reference's controls and NumPy normals returns the CVaR / SAA of the
    REFERENCE's own residual rows: obs = reducer(max_{o,t} f_bar), lane =
    reducer(max_t lb) + reducer(max_t ub) (costs.py:137-171, 206-234)."""
    B = 20
    cfg = native.make_config(1000, O, g["level"], H, "gaussian", g["acc_c"], g["steer_c"], num_batch=B,
                             variant=g["variant"], maxiter_cem=1)
    nat = native.Handle(cfg)
    prob = Problem(1000, O, g["level"], H, "gaussian", g["acc_c"], g["steer_c"], num_batch=B, variant=g["variant"],
                   maxiter_cem=1)
    draws = oracle.Draws.random(prob, np.random.default_rng(0), idx_mpc=int(g["key"]))
    draws.roll = np.asarray(V.draws_numpy("gaussian", g["acc"], g["steer"], 1000, H, g["key"]), np.float32)[None]
    mean = np.array([15] * 4 + [0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    nat.begin(cost, int(g["key"]), np.asarray(g["init_state"], np.float32), mean, cov, g["x_obs_traj"],
              g["y_obs_traj"], 15.0, draws)
    nat.write("acc", np.tile(np.asarray(g["acc"][:100], np.float32), B))
    nat.write("steer", np.tile(np.asarray(g["steer"][:100], np.float32), B))
    nat.run_stage(2, 0)
    obs, lane = nat.read("obs_cost")[:B], nat.read("lane_cost")[:B]
    nat.close()
    cb = g["f_bar"].max(axis=(0, 2)).astype(np.float32)
    lb, ub = g["lane_lb"].max(axis=1).astype(np.float32), g["lane_ub"].max(axis=1).astype(np.float32)
    if cost == "cvar":
        want_obs, want_lane = Co.cvar(prob, cb), Co.cvar(prob, lb) + Co.cvar(prob, ub)
        tol = 1e-4
    else:
        want_obs, want_lane = Co.saa(prob, cb), Co.saa_lane(prob, g["y_roll"].astype(np.float32))
        tol = 2e-3   # a sample whose residual sits at the ellipse boundary may change sides
    assert np.all(np.abs(obs - want_obs) <= tol), (obs[0], want_obs)
    assert np.all(np.abs(lane - want_lane) <= tol * max(1.0, abs(float(want_lane)))), (lane[0], want_lane)
    assert np.all(obs == obs[0]) and float(want_obs) > 0.0


SCRIPT_POINTS = [(str(n), float(l)) for n, l in zip(np.load(GOLD)["script_points"], np.load(GOLD)["script_levels"])]


def _script_files(noise):
    d = np.load(GOLD)
    pre = f"script_{noise}_"
    files = {cost: {k: d[pre + cost + "_" + k] for k in ("cx", "cy", "init_state", "x_obs", "y_obs", "vx_obs", "vy_obs")}
             for cost in ("cvar", "mmd_opt")}
    want = {k: d[pre + k] for k in ("coll_cvar", "coll_cvar_lane", "coll_mmd_opt", "coll_mmd_opt_lane")}
    return files, want, int(d["script_num_prime"]), int(d["script_num_obs"]), int(d["script_num_reduced"])


@pytest.mark.parametrize("noise,level", SCRIPT_POINTS)
def test_script_draws_and_selection_pinned_to_reference(noise, level):
    """The drop-in script's own pieces -- the configuration intersection and
    keys (validate_files) and the host draws it makes by default
    (optimizer.validation.reference_draws: np.random.seed(k) + NumPy
    multivariate_normal / beta, S/validation.py:42-84) -- with the oracle's
    fp64 counter in place of the GPU reproduce the coll_* arrays of the
    REFERENCE's main loop executed on the same data files (:224-464)."""
    import types
    from optimizer import validation as DV
    files, want, H, O, n = _script_files(noise)
    oprob = Problem(n, O, level, H, noise, 0.0, 0.0)
    nsprob = types.SimpleNamespace(Pdot_jax=oprob.Pdot, Pddot_jax=oprob.Pddot, t=0.15, wheel_base=2.5, beta_a=2,
                                   beta_b=5)

    def stats_fn(d, idx, keys):
        out = []
        for j, k in zip(idx, keys):
            draws = DV.reference_draws(nsprob, d["cx"][j], d["cy"][j], H, noise, int(k))
            xt, yt, _ = Hh.compute_obs_trajectories(oprob, d["x_obs"][j], d["y_obs"][j], d["vx_obs"][j], d["vy_obs"][j],
                                                    np.zeros(O))
            out.append(V.compute_stats(oprob, d["cx"][j], d["cy"][j], d["init_state"][j], xt, yt, noise, level, 0.0,
                                       0.0, draws))
        return np.array([o[0] for o in out], np.float64), np.array([o[1] for o in out], np.float64)

    got = DV.validate_files(None, files["cvar"], files["mmd_opt"], noise, level, H, O, "static", stats_fn=stats_fn)
    for k, v in want.items():
        assert np.array_equal(got[k], v), (k, got[k], v)


@pytest.mark.gpu
@pytest.mark.parametrize("noise,level", SCRIPT_POINTS)
def test_gpu_script_pinned_to_reference(tmp_path, noise, level):
    """``python -m optimizer.validation`` (default rng = the reference's NumPy
    draws) on the fixture's data files writes the coll_* arrays of the
    REFERENCE's script executed on the same files, bit for bit."""
    from optimizer import validation as DV
    files, want, H, O, n = _script_files(noise)
    root, stats = tmp_path / "data", tmp_path / "stats"
    for cost in ("cvar", "mmd_opt", "mmd_random"):
        dst = DV.data_path(str(root), noise, level, H, cost, n, O)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        np.savez(dst, **files["cvar" if cost == "mmd_random" else cost])
    DV.main(["--noise_levels", str(level), "--num_reduced_sets", str(n), "--num_obs", str(O), "--num_prime", str(H),
             "--noises", noise, "--acc_const_noise", "0", "--steer_const_noise", "0", "--root", str(root),
             "--stats_root", str(stats)])
    got = np.load(DV.stats_path(str(stats), noise, level, H, n, O))
    for k, v in want.items():
        assert np.array_equal(got[k], v), (k, got[k], v)


def _results_file(rs, ids, O, dynamic):
    """A results npz of S/main_mpc.py:130-135 layout for configuration ids."""
    d = dict(cx=rs.normal(size=(len(ids), 11)), cy=rs.normal(size=(len(ids), 11)),
             init_state=np.tile([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], (len(ids), 1)),
             x_obs=np.array([[35.0 + 5 * ((k + j) % 9) for j in range(O)] for k in ids]),
             y_obs=np.array([[1.75 if (k >> j) & 1 else -1.75 for j in range(O)] for k in ids]),
             vx_obs=np.zeros((len(ids), O)), vy_obs=np.zeros((len(ids), O)))
    if dynamic:
        d.update(psi_obs=np.zeros((len(ids), O)), x_obs_traj=rs.normal(size=(len(ids), O, 100)),
                 y_obs_traj=rs.normal(size=(len(ids), O, 100)))
    return d


@pytest.mark.parametrize("variant", ["static", "dynamic"])
def test_stats_writer_layout(tmp_path, variant):
    from optimizer import validation as DV
    O = 3
    rs = np.random.RandomState(0)
    d_cvar = _results_file(rs, [0, 2, 3, 5, 8], O, variant == "dynamic")
    d_opt = _results_file(rs, [1, 2, 3, 5, 7, 8], O, variant == "dynamic")
    rows = DV.common_configs(d_cvar, d_opt, O)
    # the reference's selection: configurations in both files, in the set-intersection order
    mat = lambda d: np.hstack((d["init_state"], d["x_obs"], d["y_obs"], d["vx_obs"], d["vy_obs"]))
    cset = set(tuple(x) for x in mat(d_cvar))
    dset = set(tuple(x) for x in mat(d_opt))
    eset = [np.array(x) for x in cset & dset]
    assert len(rows) == len(eset) == 4
    for (ic, im), e in zip(rows, eset):
        assert np.array_equal(mat(d_cvar)[ic], e) and np.array_equal(mat(d_opt)[im], e)
    seen = []

    def stats_fn(d, idx, keys):
        seen.append((d is d_opt, list(idx), list(keys)))
        return np.arange(len(idx)) * 10.0, np.arange(len(idx)) * 1.0

    out = DV.validate_files(None, d_cvar, d_opt, "gaussian", 0.1, 30, O, variant, stats_fn=stats_fn)
    assert [s[0] for s in seen] == [True, False]                      # mmd_opt first, then cvar
    assert seen[0][1] == [m for _, m in rows] and seen[1][1] == [c for c, _ in rows]
    assert seen[0][2] == list(range(4))                               # key = position k (:328)
    dst = DV.stats_path(str(tmp_path), "gaussian", 0.1, 30, 22, O)
    assert dst.endswith("gaussian_noise/noise_10/ts_30/22_samples_3_obs.npz")
    os.makedirs(os.path.dirname(dst))
    np.savez(dst, **out)
    f = np.load(dst)
    assert sorted(f.files) == ["coll_cvar", "coll_cvar_lane", "coll_mmd_opt", "coll_mmd_opt_lane",
                               "coll_mmd_random", "coll_mmd_random_lane"]
    assert f["coll_mmd_opt"].dtype == np.float64 and f["coll_mmd_random"].shape == (0,)
    assert DV.data_path("./data", "beta", 0.3, 30, "cvar", 500, 10) == \
        "./data/beta_noise/noise_30/ts_30/cvar_500_samples_10_obs.npz"
