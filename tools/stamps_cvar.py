#!/usr/bin/env python3
"""Phase stamps (s_memrealtime, 100 MHz) of workgroup 0 of k_front (slots
40-46) and k_select (32-37) after a few steps of a workload (GPU box):
    python tools/stamps_cvar.py [workload]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]

import bench  # noqa: E402
from optimizer import _native  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cvar"
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
    us = lambda a, b: (d[b] - d[a]) / 100.0  # noqa: E731
    print("front:  " + "  ".join(f"{a}->{a + 1} {us(a, a + 1):.2f}" for a in range(40, 46)) + f"  total {us(40, 46):.2f} us")
    print("select: " + "  ".join(f"{a}->{a + 1} {us(a, a + 1):.2f}" for a in range(32, 37)) + f"  total {us(32, 37):.2f} us")


if __name__ == "__main__":
    main()
