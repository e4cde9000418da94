"""Concurrent sweep (optimizer.sweep.run_block_concurrent): configurations in
flight on separate HIP streams give bit-identical rows to one-at-a-time
solving through the drop-in CEM (the per-configuration RNG is keyed by its own
idx_mpc), at the reference's num_batch = 100.  Both scenario variants: the
dynamic one changes y_lb / y_ub / K_steer on the device and feeds the
library's QP obstacle tracks (synthetic_dynamic_obs/main_mpc.py:116-135)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["static", "dynamic"])
@pytest.mark.parametrize("cost,n", [("cvar", 32), ("mmd_opt", 8)])
def test_concurrent_equals_sequential(cost, n, variant):
    from optimizer import _native
    from optimizer.cem import CEM
    from optimizer.sweep import run_block, run_block_concurrent
    prob = CEM(n, 4, 0.1, 20, "gaussian", 0.0, 0.0, num_batch=100, device=0, variant=variant)
    init = np.array([0.0, 1.75 if variant == "static" else -1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
    mean = np.array([15.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    ids = range(5)
    seq = run_block(prob, cost, ids, init, mean, cov, variant=variant)
    hs = [prob.handle] + [_native.Handle(prob._cfg) for _ in range(2)]
    con = run_block_concurrent(prob, hs, cost, ids, init, mean, cov, variant=variant)
    assert np.array_equal(seq, con)
    assert np.all(np.isfinite(seq[:, 1:25]))


@pytest.mark.parametrize("variant", ["static", "dynamic"])
@pytest.mark.parametrize("cost,n,noise", [("cvar", 32, "gaussian"), ("mmd_opt", 8, "gaussian"), ("cvar", 24, "beta"),
                                          ("mmd_random", 16, "gaussian")])
def test_batch_equals_sequential(cost, n, noise, variant):
    """mpcmmd_solve_batch (one launch per stage over configuration x
    candidate): rows bit-identical to one-configuration solves, including a
    last batch that is only partly filled (7 configurations, batches of 3)."""
    from optimizer import _native
    from optimizer.cem import CEM
    from optimizer.sweep import run_block, run_block_batch
    prob = CEM(n, 4, 0.1 if noise == "gaussian" else 0.3, 20, noise, 0.0, 0.0, num_batch=100, device=0,
               variant=variant)
    init = np.array([0.0, 1.75 if variant == "static" else -1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
    mean = np.array([15.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    ids = range(7)
    seq = run_block(prob, cost, ids, init, mean, cov, variant=variant)
    hb = _native.Handle(prob._cfg, max_configs=3)
    bat = run_block_batch(prob, hb, cost, ids, init, mean, cov, variant=variant)
    hb.close()
    assert np.array_equal(seq, bat), np.argwhere(seq != bat)[:5]


def test_batch_two_groups_equals_sequential():
    """A batch of 12 configurations x num_batch 100 (1200 candidates) runs its
    beta-CEM as two candidate groups on two streams, the group boundary
    inside a configuration (mpcmmd.hip: run_beta_cem) -- the production
    path of `optimizer.sweep --batch 32`: rows bit-identical to one
    configuration at a time."""
    from optimizer import _native
    from optimizer.cem import CEM
    from optimizer.sweep import run_block, run_block_batch
    prob = CEM(6, 3, 0.1, 12, "gaussian", 0.0, 0.0, num_batch=100, device=0, maxiter_cem=4)
    init = np.array([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
    mean = np.array([15.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    ids = range(12)
    seq = run_block(prob, "mmd_opt", ids, init, mean, cov)
    hb = _native.Handle(prob._cfg, max_configs=12)
    bat = run_block_batch(prob, hb, "mmd_opt", ids, init, mean, cov)
    hb.close()
    assert np.array_equal(seq, bat), np.argwhere(seq != bat)[:5]
