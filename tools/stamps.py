#!/usr/bin/env python3
"""Phase stamps (s_memrealtime, 100 MHz) of workgroup 0 of the last launch of
each beta-CEM kernel, after a few steps of a bench workload (GPU box):
    python tools/stamps.py [workload]
Slots: 0-1 k_bsample, 16 k_bkernel start, 17 setup done, 18-19 (kernel
specific), 20 end."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]

import bench  # noqa: E402
from optimizer import _native  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "mmd_opt"
    w = bench.WORKLOADS[name]
    inst = bench.make_workload(w, 0)
    cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                              num_batch=w["num_batch"], maxiter_cem=20, variant=w.get("variant", "static"))
    h = _native.Handle(cfg)
    h.begin(w["cost"], inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"], inst["v_des"])
    for t in range(3):
        h.iterate(t, 1)
    h.sync()
    d = h.read("dbg", np.uint64).astype(np.int64)
    wgt = h.read("wgt", np.uint64).astype(np.int64).reshape(-1, 2)
    h.close()
    wgt = wgt[(wgt[:, 0] > 0) & (wgt[:, 1] > wgt[:, 0])]
    if len(wgt):  # -DMPCMMD_WGT build: every k_bkernel workgroup's (start, end)
        t0 = wgt[:, 0].min()
        st, en = (wgt[:, 0] - t0) / 100.0, (wgt[:, 1] - t0) / 100.0
        dur = en - st
        ev = sorted([(x, 1) for x in st] + [(x, -1) for x in en])
        cur = peak = 0
        for _, e in ev:
            cur += e
            peak = max(peak, cur)
        print(f"bkernel workgroups {len(wgt)}: span {en.max():.1f} us, duration min/median/max "
              f"{dur.min():.1f}/{np.median(dur):.1f}/{dur.max():.1f} us, peak concurrency {peak}, "
              f"started by 5 us {int((st < 5).sum())}, start quantiles {np.percentile(st, [25, 50, 75, 100]).round(1)}")
    us = lambda a, b: (d[b] - d[a]) / 100.0  # noqa: E731  (100 MHz ticks -> us)
    print(f"{name}: bsample {us(0, 1):.1f} us")
    print(f"bkernel: setup {us(16, 17):.1f} us, rows {us(17, 20):.1f} us, total {us(16, 20):.1f} us")
    for s in (18, 19):
        if d[s] > d[16]:
            print(f"  slot {s}: +{us(16, s):.1f} us")


if __name__ == "__main__":
    main()
