"""Config sharding and the final gather of the multi-GPU sweep,
on CPU with the gloo backend at world size 2 (the GPU path differs only in the
backend: RCCL).  The solver is a deterministic stand-in: what is tested is the
partition, the packing and the gather, which must give the single-process
result bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from optimizer import sweep


class _Prob:
    num_obs = 4
    num_reduced = 6


def _fake_solve(k, ob):
    rng = np.random.default_rng(k)
    cx, cy = rng.normal(size=11).astype(np.float32), rng.normal(size=11).astype(np.float32)
    cost_obs = np.float32(-1000.0 if k % 3 else 5.0)
    return (cx, cy, np.float32(-2000.0), cost_obs, rng.random(6).astype(np.float32), np.float32(0.3 + k),
            np.arange(20, dtype=np.float32) * k)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = sweep.shard(n, world, rank)
    rows = sweep.run_block(_Prob(), "mmd_opt", ids, None, None, None, solve=_fake_solve)
    allr = sweep.gather_rows(rows, n)
    if rank == 0:
        np.save(out_path, allr)
    dist.destroy_process_group()


def test_shard_partition():
    for n in (1, 7, 200):
        for world in (1, 2, 3, 8):
            blocks = [list(sweep.shard(n, world, r)) for r in range(world)]
            assert sum(blocks, []) == list(range(n))
            assert max(map(len, blocks)) - min(map(len, blocks)) <= 1


def test_static_obstacles_match_reference_generator():
    """For num_obs <= 9 the draws are S/main_mpc.py:10-21 + :114 exactly."""
    for k in (0, 5, 199):
        np.random.seed(k)
        x = np.random.choice(np.array([35, 40, 45, 50, 55, 60, 65, 70, 75]), (4,), replace=False)
        y = np.random.choice(np.array([-1.75, 1.75]), (4,))
        idx = np.random.randint(1, 10000)
        ob = sweep.static_obstacles(k, 4)
        assert np.array_equal(ob["x"], x) and np.array_equal(ob["y"], y) and ob["idx_mpc"] == idx
    ob = sweep.static_obstacles(3, 10)           # BASELINE num_obs=10 needs the extended grid
    assert len(set(ob["x"])) == 10


@pytest.mark.parametrize("n", [7, 12])
def test_gloo_world2_gather_equals_single_process(tmp_path, n):
    out = str(tmp_path / "rows.npy")
    mp.start_processes(_worker, args=(2, _free_port(), n, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    ref = sweep.run_block(_Prob(), "mmd_opt", range(n), None, None, None, solve=_fake_solve)
    assert np.array_equal(got, ref)
    # npz in the reference's layout, successful configs only (cost_obs <= -999)
    nok = sweep.save_npz(str(tmp_path / "d" / "mmd_opt_6_samples_4_obs"), got, "mmd_opt", 4, np.zeros(6))
    d = np.load(str(tmp_path / "d" / "mmd_opt_6_samples_4_obs.npz"))
    assert nok == sum(1 for k in range(n) if k % 3) == d["cx"].shape[0]
    assert sorted(d.files) == ["cx", "cy", "init_state", "vx_obs", "vy_obs", "x_obs", "y_obs"]


def test_dynamic_variant_rows_and_npz(tmp_path):
    """synthetic_dynamic_obs sweep (BASELINE configs[3] shape: num_obs = 20):
    obstacle tracks from the library's QP flow into the solve, and the npz
    carries the dynamic driver's extra keys (D/main_mpc.py:150-156)."""
    seen = {}

    def solve(k, ob):
        seen[k] = ob["x_traj"]
        return _fake_solve(k, ob)

    class P(_Prob):
        num_obs = 20

    rows = sweep.run_block(P(), "mmd_opt", range(4), None, None, None, solve=solve, variant="dynamic")
    assert rows.shape[0] == 4 and all(v.shape == (20, 100) for v in seen.values())
    nok = sweep.save_npz(str(tmp_path / "dyn"), rows, "mmd_opt", 20, np.zeros(6), "dynamic")
    d = np.load(str(tmp_path / "dyn.npz"))
    assert nok == d["x_obs_traj"].shape[0] and d["x_obs_traj"].shape[1:] == (20, 100)
    assert "psi_obs" in d and "y_obs_traj" in d
