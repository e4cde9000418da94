"""Config-sharded sweeps over the GPUs of one node.

The reference driver (S/main_mpc.py:106-135) solves 200 independent obstacle
configurations one after another.  Here config k goes to rank
``shard(num_configs, world, rank)`` (contiguous blocks), each rank solves its
block on its own GPU with its own handle, and one all-gather over RCCL
(``torch.distributed`` backend "nccl"; "gloo" on CPU for tests) collects the
fixed-size result rows.  There is no other collective: configurations share
nothing (mean/cov are re-passed unchanged per config, S/main_mpc.py:114), and
results do not depend on the world size (RNG keyed by config, not rank).

    torchrun --nproc-per-node 8 -m optimizer.sweep --cost mmd_opt --num-reduced 22 ...

Rank 0 writes the reference's npz (S/main_mpc.py:130-135 keys) for the
configurations that meet the reference's success threshold.
"""
from __future__ import annotations

import argparse
import os

import numpy as np

NV = 11


def shard(num_configs: int, world: int, rank: int) -> range:
    """Contiguous block of config ids for ``rank`` (sizes differ by <= 1)."""
    base, extra = divmod(num_configs, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def static_obstacles(k: int, num_obs: int):
    """``compute_obs_data(num_obs, k)`` (S/main_mpc.py:10-21) followed by the
    driver's ``np.random.randint(1, 10000)`` (:114).  The x grid is extended
    to {35, 40, ...} with >= num_obs slots (the reference's 9 slots cannot
    place more than 9 obstacles); for num_obs <= 9 the draws are
    the reference's own."""
    rs = np.random.RandomState(k)
    grid = np.arange(35, 35 + 5 * max(9, num_obs), 5)
    x = rs.choice(grid, (num_obs,), replace=False).astype(np.float64)
    y = rs.choice(np.array([-1.75, 1.75]), (num_obs,))
    z = np.zeros(num_obs)
    idx_mpc = int(rs.randint(1, 10000))
    return dict(x=x, y=y, vx=z, vy=z.copy(), psi=z.copy(), idx_mpc=idx_mpc)


def obstacles(variant: str, k: int, num_obs: int):
    """Configuration k of the static (S/main_mpc.py:10-21) or dynamic
    (synthetic_dynamic_obs/main_mpc.py:108-126, QP obstacle tracks in
    ``x_traj``/``y_traj``) driver."""
    if variant == "dynamic":
        from .obs_data_generate_dynamic import dynamic_obstacles
        return dynamic_obstacles(k, num_obs)
    return static_obstacles(k, num_obs)


def tracks(prob, ob):
    """x_obs_traj, y_obs_traj [O][100] of one configuration."""
    if "x_traj" in ob:
        return ob["x_traj"], ob["y_traj"]
    xo, yo, _ = prob.cem_helper.compute_obs_trajectories(ob["x"], ob["y"], ob["vx"], ob["vy"], ob["psi"])
    return xo, yo


def row_width(num_reduced: int) -> int:
    # id, cx, cy, cost_lane, cost_obs, sigma, res_beta[20], beta[n]
    return 1 + 2 * NV + 3 + 20 + num_reduced


def pack(k: int, out: tuple, num_reduced: int) -> np.ndarray:
    """The compute_cem_* return tuple of config k as one fp32 row."""
    r = np.zeros(row_width(num_reduced), np.float32)
    r[0] = k
    r[1:1 + NV] = out[0]
    r[1 + NV:1 + 2 * NV] = out[1]
    r[1 + 2 * NV] = out[2]
    r[2 + 2 * NV] = out[3]
    if len(out) == 7:  # mmd_opt: beta, sigma, res_beta
        r[3 + 2 * NV] = out[5]
        r[4 + 2 * NV:24 + 2 * NV] = out[6]
        r[24 + 2 * NV:] = np.asarray(out[4])[:num_reduced]
    return r


def gather_rows(rows: np.ndarray, num_configs: int, device=None) -> np.ndarray:
    """All-gather of every rank's rows -> [num_configs, D] ordered by config id.
    Ranks hold blocks of unequal size: pad to the largest block."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return rows[np.argsort(rows[:, 0], kind="stable")]
    world = dist.get_world_size()
    D = rows.shape[1]
    cap = -(-num_configs // world)
    buf = np.full((cap, D), np.nan, np.float32)
    buf[:rows.shape[0]] = rows
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    allr = torch.cat(parts).cpu().numpy()
    allr = allr[~np.isnan(allr[:, 0])]
    allr = allr[np.argsort(allr[:, 0], kind="stable")]
    if allr.shape[0] != num_configs:
        raise RuntimeError(f"gathered {allr.shape[0]} rows, expected {num_configs}")
    return allr


def threshold(cost: str, ker_wt: float = 1000.0) -> float:
    """Success threshold on cost_obs (S/main_mpc.py:86-97)."""
    return -ker_wt + 1.0 if cost in ("mmd_opt", "mmd_random") else 1e-5


def run_block(prob, cost, ids, init_state, mean, cov, v_des=15.0, solve=None, variant="static"):
    """Solve configs ``ids`` on this rank; ``solve(k, obs) -> out tuple``
    defaults to ``prob.compute_cem_<cost>``."""
    fn = solve
    if fn is None:
        meth = getattr(prob, f"compute_cem_{cost}")

        def fn(k, ob):
            xo, yo = tracks(prob, ob)
            return meth(ob["idx_mpc"], init_state, mean, cov, xo, yo, v_des)
    rows = [pack(k, fn(k, obstacles(variant, k, prob.num_obs)), prob.num_reduced) for k in ids]
    return np.stack(rows) if rows else np.zeros((0, row_width(prob.num_reduced)), np.float32)


def result_tuple(cost, r, num_reduced):
    """Handle.finish() dict -> the compute_cem_* return tuple (cem.py:333 / 462)."""
    if cost == "mmd_opt":
        return (r["cx"], r["cy"], r["cost_lane"], r["cost_obs"], r["beta"][:num_reduced].copy(), r["sigma"],
                r["res_beta"])
    return r["cx"], r["cy"], r["cost_lane"], r["cost_obs"]


def run_block_concurrent(prob, handles, cost, ids, init_state, mean, cov, v_des=15.0, variant="static"):
    """Solve configs ``ids`` with len(handles) configurations in flight at
    once (handles: native handles of prob's configuration, e.g. prob.handle
    plus more).  Each handle owns its device buffers and a non-blocking HIP
    stream; begin + iterate only enqueue work, so the kernels of up to G
    configurations overlap on the GPU (the reference's num_batch = 100 fills
    only 100 of the 256 CUs per launch).  Rows are identical to run_block's:
    every configuration's RNG is keyed by its own idx_mpc."""
    rows = []
    G = len(handles)
    ids = list(ids)
    for g0 in range(0, len(ids), G):
        group = ids[g0:g0 + G]
        for h, k in zip(handles, group):
            ob = obstacles(variant, k, prob.num_obs)
            xo, yo = tracks(prob, ob)
            h.begin(cost, ob["idx_mpc"], init_state, mean, cov, xo, yo, v_des)
            h.iterate(0, h.cfg.maxiter_cem)
        for h, k in zip(handles, group):
            rows.append(pack(k, result_tuple(cost, h.finish(), prob.num_reduced), prob.num_reduced))
    return np.stack(rows) if rows else np.zeros((0, row_width(prob.num_reduced)), np.float32)


def batch_handle(prob, G):
    """A batch handle for up to ``G`` configurations, halving ``G`` while the
    device refuses the buffers (the mmd_opt buffers grow with G * B * M^2:
    n = 50 at B = 100 is ~25 MB per candidate).  A failed create frees what it
    allocated (mpcmmd_create_batch), so retrying in this process is safe."""
    from . import _native
    while True:
        try:
            return _native.Handle(prob._cfg, max_configs=G)
        except _native.NativeError:
            if G <= 1:
                raise
            G //= 2


def run_block_batch(prob, handle, cost, ids, init_state, mean, cov, v_des=15.0, variant="static"):
    """Solve configs ``ids`` with handle.max_configs configurations per
    batch (mpcmmd_solve_batch: every kernel is one launch over
    configuration x candidate).  Rows are identical to run_block's: every
    configuration's RNG is keyed by its own idx_mpc."""
    rows = []
    G = handle.max_configs
    ids = list(ids)
    for g0 in range(0, len(ids), G):
        group = ids[g0:g0 + G]
        obs = [obstacles(variant, k, prob.num_obs) for k in group]
        tr = [tracks(prob, ob) for ob in obs]
        res = handle.solve_batch(cost, [ob["idx_mpc"] for ob in obs], init_state, mean, cov,
                                 np.stack([t[0] for t in tr]), np.stack([t[1] for t in tr]), v_des)
        for k, r in zip(group, res):
            rows.append(pack(k, result_tuple(cost, r, prob.num_reduced), prob.num_reduced))
    return np.stack(rows) if rows else np.zeros((0, row_width(prob.num_reduced)), np.float32)


def save_npz(path, rows, cost, num_obs, init_state, variant="static"):
    """Successful configs in the reference's layout (S/main_mpc.py:130-135;
    dynamic: D/main_mpc.py:150-156 adds psi_obs, x_obs_traj, y_obs_traj)."""
    ok = rows[:, 2 + 2 * NV] <= threshold(cost)
    ks = rows[ok, 0].astype(int)
    obs = [obstacles(variant, int(k), num_obs) for k in ks]
    stack = lambda key: np.array([o[key] for o in obs]).reshape(len(obs), num_obs)
    extra = {}
    if variant == "dynamic":
        extra = dict(psi_obs=stack("psi"),
                     x_obs_traj=np.array([o["x_traj"] for o in obs]).reshape(len(obs), num_obs, 100),
                     y_obs_traj=np.array([o["y_traj"] for o in obs]).reshape(len(obs), num_obs, 100))
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    np.savez(path, cx=rows[ok, 1:1 + NV].astype(np.float64), cy=rows[ok, 1 + NV:1 + 2 * NV].astype(np.float64),
             init_state=np.tile(np.asarray(init_state, np.float64), (len(ks), 1)),
             x_obs=stack("x"), y_obs=stack("y"), vx_obs=stack("vx"), vy_obs=stack("vy"), **extra)
    return int(ok.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cost", default="mmd_opt", choices=["mmd_opt", "mmd_random", "cvar", "saa"])
    ap.add_argument("--num-reduced", type=int, default=22)
    ap.add_argument("--num-obs", type=int, default=10)
    ap.add_argument("--num-prime", type=int, default=30)
    ap.add_argument("--noise", default="gaussian")
    ap.add_argument("--noise-level", type=float, default=0.1)
    ap.add_argument("--num-batch", type=int, default=100)
    ap.add_argument("--num-configs", type=int, default=200)
    ap.add_argument("--acc-const-noise", type=float, default=0.0)
    ap.add_argument("--steer-const-noise", type=float, default=0.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--batch", type=int, default=32,
                    help="configurations per batched solve (mpcmmd_solve_batch; 0 = use --streams)")
    ap.add_argument("--streams", type=int, default=1, help="with --batch 0: configurations in flight on streams")
    ap.add_argument("--variant", default="static", choices=["static", "dynamic"])
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from .cem import CEM

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    prob = CEM(a.num_reduced, a.num_obs, a.noise_level, a.num_prime, a.noise, a.acc_const_noise,
               a.steer_const_noise, num_batch=a.num_batch, device=local, variant=a.variant)
    y0 = 1.75 if a.variant == "static" else -1.75                      # D/main_mpc.py:34-42
    init = np.array([0.0, y0, 5.0, 0.0, 0.0, 0.0], np.float32)          # S/main_mpc.py:46-54
    mean = np.array([15.0] * 4 + [0.0] * 4, np.float32)                 # :56-71
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)          # :69-74
    ids = shard(a.num_configs, world, rank)
    if a.batch > 0:
        from . import _native
        G = max(1, min(a.batch, len(ids), 65535 // a.num_batch))
        hb = batch_handle(prob, G)
        rows = run_block_batch(prob, hb, a.cost, ids, init, mean, cov, variant=a.variant)
        hb.close()
    elif a.streams > 1:
        from . import _native
        hs = [prob.handle] + [_native.Handle(prob._cfg) for _ in range(a.streams - 1)]
        rows = run_block_concurrent(prob, hs, a.cost, ids, init, mean, cov, variant=a.variant)
    else:
        rows = run_block(prob, a.cost, ids, init, mean, cov, variant=a.variant)
    allr = gather_rows(rows, a.num_configs, device if world > 1 else None)
    if rank == 0:
        out = a.out or "./data/{}_noise/noise_{}/ts_{}/{}_{}_samples_{}_obs".format(
            a.noise, int(a.noise_level * 100), a.num_prime, a.cost, a.num_reduced, a.num_obs)
        nok = save_npz(out, allr, a.cost, a.num_obs, init, a.variant)
        print(f"{a.cost}: {nok}/{a.num_configs} configs meet the threshold -> {out}.npz")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
