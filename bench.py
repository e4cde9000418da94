#!/usr/bin/env python3
"""Throughput bench of the CEM-projection optimizer hot path (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload mmd_opt|cvar]

One step = one outer CEM iteration (cem.py:221-315 body: initial guess,
projection, controls, noisy rollouts, risk reducer (beta-CEM for mmd_opt),
elite sorts, CEM update) over the whole batch, on device-resident inputs, with
the library's internal Philox noise.  Every 20 steps a new solve starts
(mpcmmd_begin: boundary vectors, initial population, obstacle upload), as in
the reference's 20-iteration compute_cem_* call; that host work is inside the
timed region.

N > 1: one process per GPU (torchrun).  Each rank solves its own obstacle
configuration (config k = rank, seeded like S/main_mpc.py:12,114), so per-GPU
work is fixed ("scaling": "weak"); RCCL is used for the barrier, the max of
the elapsed times and the final gather of the per-config results (§8e).

Extra fields: "roofline" for the dominant kernel (HIP-event durations of the
library's launches on its stream, during a profiled pass of the same steps)
and "cpu_baseline" (the NumPy oracle on a bounded sample of the same
workload, rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "mpc-mmd_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

kF = 22  # beta-CEM features per mother row (cx | cy)
METRIC = "MPC optimizer steps/s (batch=1024,H=30,obs_samp=500) @1/2/4/8 GPU; % HBM roofline"

# BASELINE.json configs[1] (headline), configs[2] and configs[3] (per GPU: one configuration per rank)
WORKLOADS = {
    "mmd_opt": dict(desc="static obs, mmd_opt, batch=1024 rollouts, H=30, num_obs=10, obs_samples=484 (n=22, M=n^2)",
                    cost="mmd_opt", num_reduced=22, num_obs=10, num_prime=30, noise="gaussian", level=0.1,
                    num_batch=1024),
    "cvar": dict(desc="static obs, cvar, batch=1024 rollouts, H=30, num_obs=10, obs_samples=500, beta noise 0.3",
                 cost="cvar", num_reduced=500, num_obs=10, num_prime=30, noise="beta", level=0.3,
                 num_batch=1024),
    "dynamic": dict(desc="dynamic obs, mmd_opt, batch=1024 rollouts, H=50, num_obs=20, obs_samples=1024 (n=32, M=n^2)",
                    cost="mmd_opt", num_reduced=32, num_obs=20, num_prime=50, noise="gaussian", level=0.1,
                    num_batch=1024, variant="dynamic"),
}

# MI355X peaks (MI355X_MICROARCH.md): fp32 vector 157.3 TFLOP/s = 78.6 T lane-ops/s
# (one fp32 op per lane per cycle at full packing); HBM3E 8 TB/s
VALU_PEAK_TOPS = 78.6
VALU64_PEAK_TOPS = 39.3   # fp64 vector 78.6 TFLOP/s = 39.3 T lane-ops/s
HBM_PEAK_GBS = 8000.0


def kernel_work(w, name, launches, stats):
    """Algorithmic work of the profiled launches of kernel `name`, in fp32
    lane-operations (Kernels):
      bdist     per candidate and outer iteration: M x M distances x 22
                features x 2 (sub, abs-add)
      bkernel   per candidate and beta-iteration: the (sample, row) pairs
                summed (counted by the kernel, stats[1]; 100 x n on the first
                beta-iteration, 89 x n after) x (M exp terms + (n-1)/2 K_red
                entries) x 3 (scale, exp, add)
      risk_baseline  B x S rollouts x H steps x (bicycle step 40 + 9 per obstacle)
    Returns (kind, ops) or None when no model is defined."""
    B, H, O = w["num_batch"], w["num_prime"], w["num_obs"]
    n = w["num_reduced"]
    M = n * n
    if name == "bkernel":
        # pairs summed (stats[1]) x (M exp terms + (n-1)/2 K_red entries on average) x 3 (scale, exp, add)
        return "ops", stats[1] * (M + (n - 1) / 2) * 3
    if name == "bdist":
        return "ops", launches * B * M * M * kF * 2
    if name == "beta_planes":
        # B x S x H x 2 Beta draws; per draw 2 gammas x (table transform 9 + log 1 + squeeze 5) + la/lb 4
        # + exp 1 + ratio 2 = 37 fp64 lane-ops (a transcendental / divide / sqrt counted as 1)
        return "ops64", launches * B * n * H * 2 * 37
    if name == "risk_baseline":
        beta = 2 * 160 if w["noise"] == "beta" else 0
        return "ops", launches * B * n * H * (40 + O * 9 + beta)
    return None


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` in `workload` from the committed PMC
    passes (profiles/r01_pmc_traffic.json, {workload: {kernel: bytes}}:
    2 x FETCH_SIZE + WRITE_SIZE per the MI355X guide's gfx950 correction),
    or None."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload, {}).get(kernel)
    except (OSError, ValueError, AttributeError):
        return None


def make_workload(w, rank):
    """Obstacle configuration k = rank: x without replacement from the
    extended grid {35, 40, ...}, y in {-1.75, 1.75} (S/main_mpc.py:10-21,
    SURVEY §8d), then idx_mpc = randint(1, 10000) (S/main_mpc.py:114)."""
    from optimizer.cem_helper import Helper  # noqa: F401  (drop-in package import check)
    O = w["num_obs"]
    init = np.array([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], np.float32)          # S/main_mpc.py:46-54
    mean = np.array([15] * 4 + [0] * 4, np.float32)                       # S/main_mpc.py:58-71
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    if w.get("variant") == "dynamic":
        # synthetic_dynamic_obs/main_mpc.py:34-41,106-129 (ego in the right lane; QP obstacle tracks)
        from optimizer.obs_data_generate_dynamic import dynamic_obstacles
        d = dynamic_obstacles(rank, O)
        init = np.array([0.0, -1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
        return dict(idx_mpc=d["idx_mpc"], init=init, mean=mean, cov=cov, xo=d["x_traj"], yo=d["y_traj"],
                    v_des=15.0)
    rs = np.random.RandomState(rank)
    xs = np.arange(35, 35 + 5 * max(9, O), 5, dtype=np.float64)
    x = rs.choice(xs, O, replace=False)
    y = rs.choice(np.array([-1.75, 1.75]), O)
    idx_mpc = int(rs.randint(1, 10000))
    # static obstacles: constant position over the 100-point plan (cem_helper.py:366-378 with v = 0)
    xo = np.repeat(x[:, None], 100, axis=1).astype(np.float32)
    yo = np.repeat(y[:, None], 100, axis=1).astype(np.float32)
    return dict(idx_mpc=idx_mpc, init=init, mean=mean, cov=cov, xo=xo, yo=yo, v_des=15.0)


def cpu_baseline(w, inst, seconds):
    """NumPy oracle (the CPU restatement of the reference) on a bounded sample
    of one step of the same workload: the batch-wide stages (guess +
    projection + controls, elite sorts + CEM update) on all B candidates and
    the per-candidate risk stage on the first c candidates, scaled to B."""
    import oracle
    try:
        from threadpoolctl import threadpool_info
        threads = max([d.get("num_threads", 1) for d in threadpool_info()] + [1])
    except Exception:
        threads = 1
    B = w["num_batch"]
    ora = oracle.CEM(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                     num_batch=B, maxiter_cem=1, variant=w.get("variant", "static"))
    draws = oracle.Draws.philox(ora.prob, inst["idx_mpc"], seed=0, with_beta_cem=(w["cost"] == "mmd_opt"))
    st = ora.init_state(inst["init"], inst["mean"], inst["cov"], draws)
    t0 = time.perf_counter()
    pr, acc, steer = ora.front(st)
    t_front = time.perf_counter() - t0
    # risk on growing candidate counts until the time budget is spent
    c, t_risk = 0, 0.0
    obs = np.zeros(B, np.float32)
    lane = np.zeros(B, np.float32)
    while c < B and t_risk < seconds:
        step = 1 if w["cost"] == "mmd_opt" else min(B - c, 64)
        t0 = time.perf_counter()
        o, l, _ = ora.candidate_costs(w["cost"], st, acc[c:c + step], steer[c:c + step], inst["xo"], inst["yo"],
                                      draws, 0)
        t_risk += time.perf_counter() - t0
        obs[c:c + step], lane[c:c + step] = o, l
        c += step
    t0 = time.perf_counter()
    n = w["num_reduced"]
    extra = dict(beta=np.full((B, n), np.float32(1.0 / n)), sigma=np.full(B, np.float32(0.01)),
                 res_beta=np.zeros((B, 20), np.float32))
    ora.select(w["cost"], st, 0, pr, steer, obs, lane, np.float32(inst["v_des"]), draws, extra)
    t_select = time.perf_counter() - t0
    t_step = t_front + t_risk * (B / c) + t_select
    return {"value": 1.0 / t_step, "unit": "steps/s", "cores": int(threads), "kind": "port",
            "sample": (f"oracle (NumPy restatement of the reference) one CEM step: front+select on all {B} "
                       f"candidates ({t_front + t_select:.2f} s), risk stage on {c} of {B} candidates "
                       f"({t_risk:.1f} s) scaled x{B / c:.1f}; BLAS threads {threads}")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="mmd_opt", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--profile-steps", type=int, default=20)
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    from optimizer import _native

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world} (launch N>1 with torchrun)")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    w = WORKLOADS[a.workload]
    inst = make_workload(w, rank)
    T = 20
    cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                              num_batch=w["num_batch"], maxiter_cem=T, device=local, seed=rank,
                              variant=w.get("variant", "static"))
    h = _native.Handle(cfg)
    stream = torch.cuda.current_stream()
    h.set_stream(stream.cuda_stream)

    def run(k0, count):
        for i in range(k0, k0 + count):
            t = i % T
            if t == 0:
                h.begin(w["cost"], inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"],
                        inst["v_des"])
            h.iterate(t, 1)

    run(0, a.warmup)
    h.sync()
    torch.cuda.synchronize()
    # timed region: K steps, fresh solve boundaries every 20 steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    run(0, a.steps)
    ev1.record(stream)
    h.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    if world > 1:
        el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
        dist.barrier()
    res = h.finish()
    # profiled pass (same steps, HIP events around every launch on the library's stream)
    h.write("stats", np.zeros(8, np.uint64))
    h.profile(True)
    run(0, a.profile_steps)
    h.sync()
    kt = h.kernel_times()
    h.profile(False)
    stats = h.read("stats", np.uint64).astype(np.int64)
    # final gather of per-config results over RCCL (§8e)
    vec = np.concatenate([res["cx"], res["cy"], [res["cost_lane"], res["cost_obs"]]]).astype(np.float32)
    if world > 1:
        vt = torch.from_numpy(vec).cuda()
        allv = [torch.empty_like(vt) for _ in range(world)]
        dist.all_gather(allv, vt)
        gathered = torch.stack(allv).cpu().numpy()
    else:
        gathered = vec[None]
    if rank == 0:
        steps_total = a.steps * world
        value = steps_total / elapsed
        busy = {k: v for k, v in kt.items() if v[0] > 0}
        dom = max(busy, key=lambda k: busy[k][1])
        launches, tot_ms = busy[dom]
        avg_s = tot_ms / launches / 1e3
        model = kernel_work(w, dom, launches, stats)
        peak = VALU64_PEAK_TOPS if model is not None and model[0] == "ops64" else VALU_PEAK_TOPS
        roof = {"bound": "valu", "achieved": None, "peak": peak, "unit": "Tops/s", "frac": None}
        if model is not None:
            roof["achieved"] = model[1] / launches / avg_s / 1e12
            roof["frac"] = roof["achieved"] / peak
            if model[0] == "ops64":
                roof["bound"] = "valu-fp64"
        roof["traffic"] = pmc_traffic(a.workload, dom)
        roof["kernel"] = dom
        roof["avg_us"] = avg_s * 1e6
        line = {
            "metric": METRIC, "value": value, "unit": "steps/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic ({w.get('variant', 'static')} obstacle configs k=rank, internal Philox noise)",
            "config": {"workload": w["desc"], "cost": w["cost"], "global_batch": w["num_batch"] * world,
                       "num_batch": w["num_batch"], "num_prime": w["num_prime"], "num_obs": w["num_obs"],
                       "num_reduced": w["num_reduced"], "noise": w["noise"], "noise_level": w["level"],
                       "parallelism": f"config-sharded x{world}", "solves_per_s": value / T},
            "roofline": roof,
            "kernels_ms_per_step": {k: v[1] / a.profile_steps for k, v in busy.items()},
            "event_ms_rank0": ev_ms,
            "results_gathered": int(gathered.shape[0]),
        }
        if world == 1 and a.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(w, inst, a.cpu_seconds)
        print(json.dumps(line), flush=True)
    h.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
