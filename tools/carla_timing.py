"""CARLA tick timing variants (GPU box): launch-bound or GPU-bound?
    python tools/carla_timing.py [n] [ticks]
Per variant: wall ms per tick of compute_cem_mmd + compute_cem_cvar on the
synthetic replay, the CPU time spent enqueueing (iterate returns before the
GPU finishes), with and without whole-solve graphs, and with the two solves
on two handles (two streams) at once."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    cem, rep = bench._carla_modules()
    w = bench.CARLA_WORKLOAD
    rec = rep.record_synthetic(ticks=ticks * 5 + 1)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    mean = np.array([10.0] * 4 + [0.0] * 4, np.float32)
    p1 = cem.CEM(n, 1, 3, 0.1, 60, "gaussian", "Town05", 0.0, 0.0)
    p2 = cem.CEM(n, 1, 3, 0.1, 60, "gaussian", "Town05", 0.0, 0.0)
    ins = [rep.tick_inputs(rec, k * 5, p1.cem_helper, 3) for k in range(ticks)]
    for graphs in (False, True):
        for h in (p1.handle, p2.handle):
            h.set_graphs(graphs)
        for mode in ("sequential", "two-streams"):
            rows = []
            for rep_i in range(2):  # first pass warms up (and captures the graphs)
                for (init, xo, yo, path) in ins:
                    t0 = time.perf_counter()
                    h1 = p1.handle
                    h2 = p1.handle if mode == "sequential" else p2.handle
                    h1.carla_begin("mmd_opt", 3, init, mean, cov, xo, yo, 10.0, path)
                    h1.iterate(0, 20)
                    t1 = time.perf_counter()
                    if mode == "sequential":
                        h1.finish()
                    h2.carla_begin("cvar", 3, init, mean, cov, xo, yo, 10.0, path)
                    h2.iterate(0, 20)
                    t2 = time.perf_counter()
                    if mode != "sequential":
                        h1.finish()
                    h2.finish()
                    t3 = time.perf_counter()
                    if rep_i == 1:
                        rows.append((t1 - t0, t2 - t1, t3 - t0))
            a = np.array(rows) * 1e3
            print(f"n={n} graphs={graphs} {mode}: tick {a[:, 2].mean():.2f} ms (median {np.median(a[:, 2]):.2f}); "
                  f"mmd enqueue {a[:, 0].mean():.2f} ms", flush=True)


if __name__ == "__main__":
    main()
