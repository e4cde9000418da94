"""optimizer.sweep.batch_handle retries handle creation
with half the configurations after the device refuses the buffers.  A failed
hipMalloc leaves the runtime's last-error state set; mpcmmd_create_batch
clears it on its failure path, so the retried (smaller) handle's first launch
check does not report the stale out-of-memory error.  The refusal here is a
real HIP out-of-memory error: MPCMMD_MAX_HANDLE_BYTES makes the library ask
for an impossible allocation once a handle's buffers pass the cap."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_batch_handle_halving_after_real_oom(monkeypatch):
    from optimizer import _native
    from optimizer.cem import CEM
    from optimizer.sweep import batch_handle, run_block, run_block_batch
    prob = CEM(6, 3, 0.1, 12, "gaussian", 0.0, 0.0, num_batch=100, device=0, maxiter_cem=3)
    one = _native.Handle(prob._cfg, max_configs=1)
    per_cfg = one.buffer_bytes("*")
    one.close()
    # room for a little over 3 configurations: 32 -> 16 -> 8 -> 4 fail, 2 fits
    monkeypatch.setenv("MPCMMD_MAX_HANDLE_BYTES", str(int(3.2 * per_cfg)))
    h = batch_handle(prob, 32)
    monkeypatch.delenv("MPCMMD_MAX_HANDLE_BYTES")
    assert 1 <= h.max_configs < 4, h.max_configs
    init = np.array([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
    mean = np.array([15.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    ids = range(3)
    bat = run_block_batch(prob, h, "mmd_opt", ids, init, mean, cov)
    h.close()
    seq = run_block(prob, "mmd_opt", ids, init, mean, cov)
    assert np.array_equal(seq, bat)
