"""Phase timestamps of workgroup 0 (s_memrealtime, 100 MHz) for the mmd_opt
kernels at the bench shape: a profiling helper, not a test."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
import bench  # noqa: E402
from optimizer import _native  # noqa: E402

w = bench.WORKLOADS["mmd_opt"]
inst = bench.make_workload(w, 0)
cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                          num_batch=w["num_batch"], maxiter_cem=20, device=0, seed=0)
h = _native.Handle(cfg)
h.begin("mmd_opt", inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"], 15.0)
h.run_stage(0, 0)
h.run_stage(1, 0)
h.run_stage(4, 0)
for tb in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    for st in (5, 6, 7):
        h.write("dbg", np.zeros(64, np.uint64))
        h.run_stage(st, tb)
        d = h.read("dbg", np.uint64).astype(np.int64)
        nz = np.nonzero(d)[0]
        if len(nz):
            t0 = d[nz[0]]
            print(f"tb={tb} stage={st} " + " ".join(f"{i}:{(d[i] - t0) / 100:.1f}" for i in nz), flush=True)
