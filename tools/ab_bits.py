"""Bit comparison of two library builds on the bench workloads (GPU box):
    python tools/ab_bits.py LIB_A LIB_B [workload ...]
Each build runs one full solve (T = 20 iterations) of every workload in its
own process (MPCMMD_LIB), every output array of mpcmmd_finish is saved, and
the two sets are compared bit for bit."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, numpy as np
sys.path.insert(0, "{root}")
import bench
from optimizer import _native
out = {{}}
for name in {names!r}:
    w = bench.WORKLOADS[name]
    inst = bench.make_workload(w, 0)
    cfg = _native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                              num_batch=w["num_batch"], maxiter_cem=20, device=0, seed=0, variant=w.get("variant", "static"))
    h = _native.Handle(cfg)
    h.begin(w["cost"], inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"], inst["v_des"])
    h.iterate(0, 20)
    res = h.finish(trace=True)
    for k, v in res.items():
        out[name + "/" + k] = np.asarray(v)
    out[name + "/pop"] = h.read("pop").copy()
    h.close()
np.savez("{path}", **out)
'''


def run(lib, names, path):
    env = dict(os.environ, MPCMMD_LIB=lib)
    code = CHILD.format(root=ROOT, names=names, path=path)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, cwd=ROOT)
    return dict(np.load(path))


def main():
    a, b = sys.argv[1], sys.argv[2]
    names = sys.argv[3:] or ["cvar", "mmd_opt"]
    ra = run(a, names, "/tmp/ab_bits_a.npz")
    rb = run(b, names, "/tmp/ab_bits_b.npz")
    bad = [k for k in ra if not np.array_equal(ra[k], rb[k], equal_nan=True)]
    print("arrays", len(ra), "differ", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
