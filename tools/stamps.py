#!/usr/bin/env python3
"""Phase stamps (s_memrealtime, 100 MHz) of workgroup 0 of the last launch of
each beta-CEM kernel, after a few steps of a bench workload (GPU box):
    python tools/stamps.py [workload]
Slots: 0-1 k_bsample; k_bkernel 16 start, 19 series pairs done, 17 setup
done, 18 K_red done, 20 end; k_front 40-46."""
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
    h.close()
    us = lambda a, b: (d[b] - d[a]) / 100.0  # noqa: E731  (100 MHz ticks -> us)
    print(f"{name}: bsample {us(0, 1):.1f} us")
    print(f"bkernel: series {us(16, 19):.1f} us, scan/order {us(19, 17):.1f} us, K_red {us(17, 18):.1f} us, "
          f"direct {us(18, 20):.1f} us, total {us(16, 20):.1f} us")
    # k_front (workgroup 0): 40 staged, 41 guess + atan2, 42 unwrap, 43 initial multipliers (+ det sums),
    # 44 compute_x, 45 compute_alph_d + multipliers, 46 controls + stores
    names = ["guess+atan2", "unwrap", "polar+adj", "compute_x", "alph_d+adj", "controls+stores"]
    print("front: " + ", ".join(f"{nm} {us(40 + i, 41 + i):.2f}" for i, nm in enumerate(names)) +
          f"; total {us(40, 46):.2f} us")


if __name__ == "__main__":
    main()
