#!/usr/bin/env python3
"""Per-workgroup phase stamps (MPCMMD_STAMPW, s_memrealtime at 100 MHz) of the
last launch of the instrumented kernel after a few bench steps (GPU box):
    python tools/stampsw.py [workload] [steps] [slots]
Prints the launch span, the workgroup lifetimes and each phase's mean
duration over the workgroups that wrote both of its stamps."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]

import bench  # noqa: E402
from optimizer import _native  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "mmd_opt"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    nslot = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    w = bench.WORKLOADS[name]
    inst = bench.make_workload(w, 0)
    os.environ.setdefault("MPCMMD_GROUPS", "1")
    os.environ["MPCMMD_STAMPW"] = "1"  # the handle allocates the stamp buffer only when asked
    cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                              num_batch=w["num_batch"], maxiter_cem=20, variant=w.get("variant", "static"))
    h = _native.Handle(cfg)
    h.begin(w["cost"], inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"], inst["v_des"])
    for t in range(steps):
        h.iterate(t, 1)
    h.sync()
    d = h.read("dbgw", np.uint64).astype(np.int64).reshape(65536, 8)[:, :nslot]
    h.close()
    live = d[:, 0] > 0
    d = d[live]
    t0 = d[:, 0].min()
    end = d.max(axis=1)
    print(f"{name}: {live.sum()} workgroups, launch span {(end.max() - t0) / 100:.1f} us, "
          f"start spread {(d[:, 0].max() - t0) / 100:.1f} us, lifetime mean {(end - d[:, 0]).mean() / 100:.1f} us "
          f"max {(end - d[:, 0]).max() / 100:.1f} us")
    for a in range(nslot - 1):
        for b in range(a + 1, nslot):
            ok = (d[:, a] >= t0) & (d[:, b] >= d[:, a])
            if ok.sum() > 0:
                dt = (d[ok, b] - d[ok, a]) / 100
                print(f"  slot {a} -> {b}: {ok.sum()} WGs, mean {dt.mean():.2f} us, p90 {np.percentile(dt, 90):.2f} us")
                break


if __name__ == "__main__":
    main()
