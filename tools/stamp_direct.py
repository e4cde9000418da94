#!/usr/bin/env python3
"""Per-workgroup phase stamps of k_bkernel (slots 0-4) and k_bdirect (slots
5 start, 6 setup done, 7 rows done) of the last beta-iteration after one CARLA
compute_cem_mmd solve on the per-iteration kernels (GPU box):
    python tools/stamp_direct.py [num_reduced]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
os.environ["MPCMMD_STAMPW"] = "1"
os.environ["MPCMMD_FUSED"] = "0"

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    w = dict(bench.CARLA_WORKLOAD, num_reduced=n)
    cem, rep = bench._carla_modules()
    prob = cem.CEM(n, 1, w["num_obs"], w["level"], w["num_prime"], w["noise"], w["town"], 0.0, 0.0, device=0)
    rec = rep.record_synthetic(ticks=3, town=w["town"])
    mean0 = np.array([10.0] * 4 + [0.0] * 4, np.float32)
    cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
    init, xo, yo, path = rep.tick_inputs(rec, 0, prob.cem_helper, w["num_obs"])
    args = (path["x_path"], path["y_path"], path["arc_vec"], path["Fx_dot"], path["Fy_dot"], path["kappa"])
    h = prob.handle
    h.write("stats", np.zeros(8, np.uint64))
    prob.compute_cem_mmd(0, init, mean0, cov, xo, yo, 10.0, *args)
    st = h.read("stats", np.uint64).astype(np.int64)
    d = h.read("dbgw", np.uint64).astype(np.int64).reshape(65536, 8)[:4096]
    print(f"n={n}: stats direct rows {st[0]}, direct pairs {st[1]}, series pairs {st[2]}, K_red entries {st[3]} "
          f"({100.0 * st[1] / max(1, st[1] + st[2]):.2f}% of pairs direct)")
    for name, sl in (("k_bkernel", slice(0, 5)), ("k_bdirect", slice(5, 8))):
        x = d[:, sl]
        live = np.all(x > 0, axis=1)
        live &= x[:, 0] >= x[:, 0].max() - 100 * 300   # the last launch (earlier launches' rows: older stamps)
        x = x[live]
        if not len(x):
            print(f"  {name}: no stamps")
            continue
        t0 = x[:, 0].min()
        print(f"  {name}: {live.sum()} workgroups, span {(x.max() - t0) / 100:.1f} us, start spread "
              f"{(x[:, 0].max() - t0) / 100:.1f} us, lifetime mean {(x[:, -1] - x[:, 0]).mean() / 100:.1f} us")
        dt = np.diff(x, axis=1) / 100.0
        print("    phases mean " + " ".join(f"{v:.2f}" for v in dt.mean(axis=0)) + " us; p90 "
              + " ".join(f"{v:.2f}" for v in np.percentile(dt, 90, axis=0)))


if __name__ == "__main__":
    main()
