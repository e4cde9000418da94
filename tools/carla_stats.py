#!/usr/bin/env python3
"""k_bkernel / k_bdirect work counters of one CARLA compute_cem_mmd solve
(GPU box): distinct direct rows, direct pairs, series pairs, K_red entries.
    python tools/carla_stats.py [num_reduced_set]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    w = dict(bench.CARLA_WORKLOAD)
    cem, rep = bench._carla_modules()
    prob = cem.CEM(n, 1, w["num_obs"], w["level"], w["num_prime"], w["noise"], w["town"], 0.0, 0.0, device=0)
    rec = rep.record_synthetic(ticks=12, town=w["town"])
    mean0 = np.array([10.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    init, xo, yo, path = rep.tick_inputs(rec, 5, prob.cem_helper, w["num_obs"])
    args = (path["x_path"], path["y_path"], path["arc_vec"], path["Fx_dot"], path["Fy_dot"], path["kappa"])
    prob.compute_cem_mmd(5, init, mean0, cov, xo, yo, 10.0, *args)
    h = prob.handle
    h.write("stats", np.zeros(8, np.uint64))
    prob.compute_cem_mmd(5, init, mean0, cov, xo, yo, 10.0, *args)
    st = h.read("stats", np.uint64).astype(np.int64)
    pairs = st[1] + st[2]
    print(f"n={n}: direct rows {st[0]}, direct pairs {st[1]} ({st[1] / max(pairs, 1):.1%} of {pairs}), "
          f"series pairs {st[2]}, K_red entries {st[3]}")


if __name__ == "__main__":
    main()
