"""Regression test for the handle-creation race of round 2 (fixed in
e19bbf7): the buffers of a new handle were zeroed by null-stream memsets that
are not ordered before the constant uploads on the handle's non-blocking
stream, so a zeroing could land after an upload and wipe a constant
(configs[2] full-shape front check: cx[3:] wrong for every candidate,
gpurun_out/gpu_tests_g.log:71 of that round).

Several handles of the BASELINE shapes are created and destroyed back to back;
straight after each mpcmmd_create the device constants are read back
(mpcmmd_read) and compared with the host's (mpcmmd_host_constant), and one
front stage runs against the oracle.
"""
import numpy as np
import pytest

import oracle
from parity import DEFAULT_COV, DEFAULT_INIT, DEFAULT_MEAN, close, scenario
from oracle.helper import compute_obs_trajectories
from test_gpu_parity_baseline import _sync_state

pytestmark = pytest.mark.gpu

SHAPES = [  # (cost, noise, n, O, H, B): configs[2], configs[1], configs[3]-like, the reference's B = 100
    ("cvar", "beta", 500, 10, 30, 1024),
    ("mmd_opt", "gaussian", 22, 10, 30, 1024),
    ("mmd_opt", "gaussian", 32, 20, 50, 256),
    ("cvar", "gaussian", 50, 4, 20, 100),
]


def _host_constants(native, cfg):
    P = [native.host_constant(cfg, k).reshape(100, 11).astype(np.float32) for k in ("P", "Pdot", "Pddot")]
    return np.concatenate([p.reshape(-1) for p in P]), native.host_constant(cfg, "fit")


def test_constants_right_after_create(native):
    for rep in range(2):
        for cost, noise, n, O, H, B in SHAPES:
            cfg = native.make_config(n, O, 0.1 if noise == "gaussian" else 0.3, H, noise, 0.0, 0.0, num_batch=B,
                                     maxiter_cem=1)
            h = native.Handle(cfg)
            basis, fit = _host_constants(native, cfg)
            assert np.array_equal(h.read("basis")[:basis.size], basis), f"basis wiped ({cost} n={n} B={B} rep {rep})"
            assert np.array_equal(h.read("fit", np.float64)[:fit.size], fit), f"fit wiped ({cost} n={n} B={B})"
            pm = h.read("proj_m", np.float64).reshape(2, 11, 11)
            for xy, name, k in ((0, "proj_kinv_x", 14), (1, "proj_kinv_y", 15)):
                kinv = native.host_constant(cfg, name).reshape(k, k)
                assert np.array_equal(pm[xy], kinv[:11, :11]), f"{name} wiped ({cost} n={n} B={B})"
            assert np.abs(h.read("guess_g", np.float64)).max() > 0.0
            # every other buffer of a fresh handle is zero
            for name in ("lam_x", "lam_y", "s_lane", "obs_cost", "res_norm"):
                assert not h.read(name).any(), f"{name} not zeroed"
            h.close()


@pytest.mark.parametrize("shape", SHAPES[:2], ids=["configs2", "configs1"])
def test_front_stage_after_create(native, shape):
    """A front stage straight after creating the handle (no other handle
    alive), all candidates against the oracle: catches any constant that is
    still being written when the first kernel runs."""
    cost, noise, n, O, H, B = shape
    level = 0.1 if noise == "gaussian" else 0.3
    ora = oracle.CEM(n, O, level, H, noise, 0.0, 0.0, num_batch=B, maxiter_cem=1)
    nat = native.Handle(native.make_config(n, O, level, H, noise, 0.0, 0.0, num_batch=B, maxiter_cem=1))
    x, y, vx, vy, psi = scenario(O, 3)
    xo, yo, _ = compute_obs_trajectories(ora.prob, x, y, vx, vy, psi)
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(4), idx_mpc=5, with_beta_cem=(cost == "mmd_opt"))
    nat.begin(cost, 5, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
    st = ora.init_state(DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, draws)
    _sync_state(nat, st, B)
    nat.run_stage(1, 0)
    pr, _, _ = ora.front(st)
    close("cx", nat.read("cx").reshape(B, 11), pr["c_x"], atol=1e-4)
    close("cy", nat.read("cy").reshape(B, 11), pr["c_y"], atol=1e-4)
    nat.close()


def test_handle_info(native, monkeypatch):
    """mpcmmd_handle_info reports the handle's implementation choices: the
    beta-CEM generator variant follows the handle's capacity (<= 512
    candidates and n <= 24: one wave per block), so the same problem can carry
    different bits on handles of 512 and 1024 candidates; MPCMMD_GENWAVE pins
    it."""
    def info(B, **env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        h = native.Handle(native.make_config(22, 10, 0.1, 30, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=2))
        out = {k: h.info(k) for k in ("gen_wave", "select_prep", "fused_small", "groups", "capacity")}
        h.close()
        for k in env:
            monkeypatch.delenv(k)
        return out
    a, b = info(512), info(1024)
    assert (a["gen_wave"], b["gen_wave"]) == (1, 0)
    assert (a["capacity"], b["capacity"]) == (512, 1024)
    assert b["groups"] == 2 and a["select_prep"] == 1
    assert info(512, MPCMMD_GENWAVE="0")["gen_wave"] == 0
    assert info(1024, MPCMMD_SELECT_PREP="0")["select_prep"] == 0
    h = native.Handle(native.make_config(8, 3, 0.1, 10, "gaussian", 0.0, 0.0, num_batch=32, maxiter_cem=2))
    with pytest.raises(native.NativeError, match="unknown handle_info"):
        h.info("nonsense")
    h.close()
