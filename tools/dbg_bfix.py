"""Debug: the share of Beta draws k_beta_planes defers to k_beta_fix (GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "mpc-mmd_amd")]
import oracle  # noqa: E402
from parity import DEFAULT_COV, DEFAULT_INIT, DEFAULT_MEAN, make_pair  # noqa: E402
from optimizer import _native  # noqa: E402

B, N_S, O, H, T = 256, 100, 3, 30, 4
ora, nat, xo, yo = make_pair(_native, "cvar", "beta", n=N_S, O=O, H=H, B=B, T=T, acc_c=0.05, steer_c=0.01)
draws = oracle.Draws.random(ora.prob, np.random.default_rng(3), idx_mpc=123, seed=0, with_beta_cem=False)
nat.begin("cvar", 123, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
for t in range(T):
    nat.run_stage(1, t)
    nat.run_stage(2, t)
    n = int(nat.read("bfix_n", np.uint32, (4,))[0])
    print(f"t={t} deferred {n} of {B * N_S * H} ({n / (B * N_S * H):.4%})")
    nat.run_stage(3, t)
