#!/usr/bin/env python3
"""Per-workgroup phases of k_risk_baseline's last launch (MPCMMD_STAMPW slots
0: entry, 1: obstacles staged and sorted, 2: rollouts done, 3: exit;
s_memrealtime, 100 MHz) on the cvar workload (GPU box):
    python tools/risk_wg.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
os.environ["MPCMMD_STAMPW"] = "1"
import bench  # noqa: E402
from optimizer import _native  # noqa: E402

w = bench.WORKLOADS["cvar"]
inst = bench.make_workload(w, 0)
cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                          num_batch=w["num_batch"], maxiter_cem=20)
h = _native.Handle(cfg)
h.begin(w["cost"], inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"], inst["v_des"])
for t in range(3):
    for st in (1, 2, 3):
        h.run_stage(st, t)
d = h.read("dbgw", np.uint64).astype(np.int64).reshape(65536, 8)
h.close()
B = w["num_batch"]
prep = 1 + (B + 7) // 8
d = d[prep:prep + B, :4]
t0 = d[:, 0].min()
us = lambda x: x / 100.0  # noqa: E731
start, end = us(d[:, 0] - t0), us(d[:, 3] - t0)
ph = [us(d[:, k + 1] - d[:, k]) for k in range(3)]
print(f"{B} risk workgroups, span {end.max():.1f} us, start spread {start.max():.1f} us, lifetime mean "
      f"{(end - start).mean():.1f} max {(end - start).max():.1f}")
for name, x in zip(("staging+sort", "rollouts", "reducer"), ph):
    print(f"  {name}: mean {x.mean():.2f} p90 {np.percentile(x, 90):.2f} max {x.max():.2f} us")
print("start histogram:", np.histogram(start, bins=8)[0].tolist(), np.round(np.histogram(start, bins=8)[1], 1).tolist())
