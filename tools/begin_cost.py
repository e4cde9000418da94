#!/usr/bin/env python3
"""Per-step event times of a bench workload split by whether the step opens
a solve (mpcmmd_begin on the host, t = 0) or not, plus begin's host time
(GPU box):  python tools/begin_cost.py [workload] [steps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from optimizer import _native  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cvar"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    w = bench.WORKLOADS[name]
    inst = bench.make_workload(w, 0)
    cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                              num_batch=w["num_batch"], maxiter_cem=20, variant=w.get("variant", "static"))
    h = _native.Handle(cfg)
    stream = torch.cuda.Stream()
    h.set_stream(stream.cuda_stream)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    tb = []
    for rep in range(2):
        evs[0].record(stream)
        for i in range(steps):
            if i % 20 == 0:
                t0 = time.perf_counter()
                h.begin(w["cost"], inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"],
                        inst["v_des"])
                tb.append(time.perf_counter() - t0)
            h.iterate(i % 20, 1)
            evs[i + 1].record(stream)
        h.sync()
        torch.cuda.synchronize()
    ms = np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(steps)])
    first = ms[0::20]
    rest = np.delete(ms, np.arange(0, steps, 20))
    print(f"{name}: step mean {ms.mean():.4f} ms, median {np.median(ms):.4f}; solve-opening steps mean "
          f"{first.mean():.4f} (n={first.size}), others mean {rest.mean():.4f}; begin host {1e3 * np.mean(tb[5:]):.3f} ms "
          f"(max {1e3 * np.max(tb[5:]):.3f})")
    h.close()


if __name__ == "__main__":
    main()
