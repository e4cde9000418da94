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
