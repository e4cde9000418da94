#!/usr/bin/env python3
"""Per-workgroup lifetimes of k_front's last launch (MPCMMD_STAMPW slots 0:
entry, 1: after the basis staging, 2: exit; s_memrealtime, 100 MHz) after a
few steps of a workload (GPU box):  python tools/front_wg.py [workload]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
os.environ["MPCMMD_STAMPW"] = "1"
import bench  # noqa: E402
from optimizer import _native  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cvar"
w = bench.WORKLOADS[name]
inst = bench.make_workload(w, 0)
cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                          num_batch=w["num_batch"], maxiter_cem=20, variant=w.get("variant", "static"))
h = _native.Handle(cfg)
h.begin(w["cost"], inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"], inst["v_des"])
for t in range(3):
    h.run_stage(1, t)   # front only for the last launch's stamps: run full iterations first
    h.run_stage(2, t)
    h.run_stage(3, t)
h.run_stage(1, 3)
d = h.read("dbgw", np.uint64).astype(np.int64).reshape(65536, 8)
h.close()
nwg = (w["num_batch"] + 3) // 4
d = d[:nwg, :3]
t0 = d[:, 0].min()
us = lambda x: x / 100.0  # noqa: E731
life = us(d[:, 2] - d[:, 0])
stage = us(d[:, 1] - d[:, 0])
start = us(d[:, 0] - t0)
end = us(d[:, 2] - t0)
print(f"{name}: {nwg} workgroups, span {end.max():.1f} us; start spread {start.max():.1f} us; "
      f"lifetime mean {life.mean():.1f} p50 {np.median(life):.1f} p90 {np.percentile(life, 90):.1f} max {life.max():.1f}; "
      f"basis staging mean {stage.mean():.2f} max {stage.max():.2f}")
order = np.argsort(end)
print("last 8 workgroups (start, lifetime):", [(int(i), round(float(start[i]), 1), round(float(life[i]), 1)) for i in order[-8:]])
print("start histogram (us):", np.histogram(start, bins=8)[0].tolist(), np.round(np.histogram(start, bins=8)[1], 1).tolist())
