#!/usr/bin/env python3
"""Phase stamps of k_bcem_small (beta-iteration 5 of the last launch) after
one CARLA compute_cem_mmd solve (GPU box):
    python tools/stamp_small.py [num_reduced]
Slots: 0 start, 1 samples, 2 selection, 3 K_red, 4 direct sums, 5 QPs,
6 elites, 7 generators."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
os.environ["MPCMMD_STAMPW"] = "1"

import bench  # noqa: E402

NAMES = ["sample", "select", "kred", "direct", "qp", "elite", "gen"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    w = dict(bench.CARLA_WORKLOAD, num_reduced=n)
    cem, rep = bench._carla_modules()
    prob = cem.CEM(n, 1, w["num_obs"], w["level"], w["num_prime"], w["noise"], w["town"], 0.0, 0.0, device=0)
    rec = rep.record_synthetic(ticks=3, town=w["town"])
    mean0 = np.array([10.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    init, xo, yo, path = rep.tick_inputs(rec, 0, prob.cem_helper, w["num_obs"])
    args = (path["x_path"], path["y_path"], path["arc_vec"], path["Fx_dot"], path["Fy_dot"], path["kappa"])
    prob.compute_cem_mmd(0, init, mean0, cov, xo, yo, 10.0, *args)
    d = prob.handle.read("dbgw", np.uint64).astype(np.int64).reshape(65536, 8)[32768:49152]
    live = d[:, 0] > 0
    d = d[live]
    dt = np.diff(d, axis=1) / 100.0
    print(f"n={n}: {live.sum()} workgroups; beta-iteration 5 span mean {(d[:, 7] - d[:, 0]).mean() / 100:.2f} us")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:7s} mean {dt[:, i].mean():7.2f} us  p90 {np.percentile(dt[:, i], 90):7.2f} us")
    # bkernel_body's own stamps (rows = workgroups, the last beta-iteration)
    k = prob.handle.read("dbgw", np.uint64).astype(np.int64).reshape(65536, 8)[:100, :5]
    k = k[k[:, 0] > 0]
    kd = np.diff(k, axis=1) / 100.0
    print("  kred sub-phases (last beta-iteration): setup+union %.2f, records+series %.2f, table %.2f, "
          "entries %.2f us" % tuple(kd.mean(axis=0)))


if __name__ == "__main__":
    main()
