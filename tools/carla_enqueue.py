#!/usr/bin/env python3
"""Host enqueue time vs device completion of one CARLA compute_cem_mmd solve
(GPU box):  python tools/carla_enqueue.py [num_reduced] [ticks]
Prints per solve: begin (host), iterate's enqueue time (host returns), and the
wait until the stream drains -- a solve whose enqueue takes as long as the
whole solve is bound by the host's launch rate, not by the kernels."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    w = dict(bench.CARLA_WORKLOAD, num_reduced=n)
    cem, rep = bench._carla_modules()
    prob = cem.CEM(n, 1, w["num_obs"], w["level"], w["num_prime"], w["noise"], w["town"], 0.0, 0.0, device=0)
    rec = rep.record_synthetic(ticks=ticks * 5 + 1, town=w["town"])
    mean0 = np.array([10.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    h = prob.handle
    for i in range(ticks):
        init, xo, yo, path = rep.tick_inputs(rec, i * 5, prob.cem_helper, w["num_obs"])
        t0 = time.perf_counter()
        h.carla_begin("mmd_opt", i, init, mean0, cov, xo, yo, 10.0, path)
        t1 = time.perf_counter()
        h.iterate(0, prob.maxiter_cem)
        t2 = time.perf_counter()
        h.sync()
        t3 = time.perf_counter()
        print(f"n={n} tick {i}: begin {1e3 * (t1 - t0):.2f} ms, enqueue {1e3 * (t2 - t1):.2f} ms, "
              f"drain {1e3 * (t3 - t2):.2f} ms, solve {1e3 * (t3 - t0):.2f}")


if __name__ == "__main__":
    main()
