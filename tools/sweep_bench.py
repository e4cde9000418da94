"""Wall time of a configuration sweep at the reference's num_batch = 100 (the
S/main_mpc.py loop): one configuration at a time, G in flight on streams, and
batches of Gb configurations per launch (mpcmmd_solve_batch):
    python tools/sweep_bench.py [num_configs] [G] [Gb]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]
from optimizer import _native  # noqa: E402
from optimizer.cem import CEM  # noqa: E402
from optimizer.sweep import run_block, run_block_batch, run_block_concurrent  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
G = int(sys.argv[2]) if len(sys.argv) > 2 else 4
GB = int(sys.argv[3]) if len(sys.argv) > 3 else 32
init = np.array([0.0, 1.75, 5.0, 0.0, 0.0, 0.0], np.float32)
mean = np.array([15.0] * 4 + [0.0] * 4, np.float32)
cov = np.diag([20.0] * 4 + [100.0] * 4).astype(np.float32)
for cost, n in (("mmd_opt", 22), ("cvar", 500)):
    prob = CEM(n, 10, 0.1, 30, "gaussian", 0.0, 0.0, num_batch=100, device=0)
    hs = [prob.handle] + [_native.Handle(prob._cfg) for _ in range(G - 1)]
    hb = _native.Handle(prob._cfg, max_configs=GB)
    run_block_concurrent(prob, hs, cost, range(G), init, mean, cov)  # warm-up
    run_block_batch(prob, hb, cost, range(GB), init, mean, cov)
    t0 = time.perf_counter()
    seq = run_block(prob, cost, range(K), init, mean, cov)
    t1 = time.perf_counter()
    con = run_block_concurrent(prob, hs, cost, range(K), init, mean, cov)
    t2 = time.perf_counter()
    bat = run_block_batch(prob, hb, cost, range(K), init, mean, cov)
    t3 = time.perf_counter()
    print(f"{cost} n={n} B=100 H=30 O=10, {K} configs: one at a time {K / (t1 - t0):.1f} solves/s; "
          f"{G} streams {K / (t2 - t1):.1f} solves/s; batches of {GB} {K / (t3 - t2):.1f} solves/s; "
          f"identical rows: {np.array_equal(seq, con) and np.array_equal(seq, bat)}", flush=True)
    for x in hs[1:] + [hb]:
        x.close()
