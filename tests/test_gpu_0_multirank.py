"""The config-sharded sweep with REAL library handles on the one GPU of the
box (the 8-GPU run is the driver's): two freshly spawned ranks, gloo for the
gather, each solving its shard(...) block through run_block_batch
(mpcmmd_solve_batch), then gather_rows -- the rows must equal a one-process
solve of all configurations bit for bit (S/main_mpc.py:106-135 is the loop
being sharded).  The parent touches the GPU only after the ranks have exited
(the ranks are fresh processes that initialise HIP themselves), which is why
this file sorts before every other GPU test.

The one-process solve holds 12 configurations x num_batch 100 = 1200
candidates, so its beta-CEM runs as two candidate groups on two streams
(mpcmmd.hip: run_beta_cem), while each rank's 6-configuration batches run as
one: the rows must not depend on the grouping either."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_CFG, B, N_RED, O, H = 12, 100, 6, 3, 12
INIT = np.array([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
MEAN = np.array([15.0] * 4 + [0.0] * 4, np.float32)
COV = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, cost, out_path):
    import torch.distributed as dist

    from optimizer import _native, sweep
    from optimizer.cem import CEM
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = CEM(N_RED, O, 0.1, H, "gaussian", 0.0, 0.0, num_batch=B, device=0, maxiter_cem=4)
    ids = sweep.shard(N_CFG, world, rank)
    hb = _native.Handle(prob._cfg, max_configs=len(ids))
    rows = sweep.run_block_batch(prob, hb, cost, ids, INIT, MEAN, COV)
    hb.close()
    prob.handle.close()
    allr = sweep.gather_rows(rows, N_CFG)
    if rank == 0:
        np.save(out_path, allr)
    dist.destroy_process_group()


@pytest.mark.parametrize("cost", ["mmd_opt", "cvar"])
def test_two_rank_sweep_equals_one_process(tmp_path, cost):
    out = str(tmp_path / f"rows_{cost}.npy")
    mp.start_processes(_rank, args=(2, _free_port(), cost, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    from optimizer import _native, sweep
    from optimizer.cem import CEM
    prob = CEM(N_RED, O, 0.1, H, "gaussian", 0.0, 0.0, num_batch=B, device=0, maxiter_cem=4)
    hb = _native.Handle(prob._cfg, max_configs=N_CFG)
    ref = sweep.run_block_batch(prob, hb, cost, range(N_CFG), INIT, MEAN, COV)
    hb.close()
    assert got.shape == ref.shape == (N_CFG, sweep.row_width(N_RED))
    assert np.array_equal(got[:, 0], np.arange(N_CFG))
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]
    assert np.all(np.isfinite(got[:, 1:25]))
