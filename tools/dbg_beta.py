"""Debug: the Beta draws of the fused rollouts that miss the oracle (GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "mpc-mmd_amd")]
os.environ["MPCMMD_BETA_DUMP"] = "1"
import oracle  # noqa: E402
from oracle.rng import (STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B,  # noqa
                        beta_draws, iteration_key, philox4x32_10, _u01)
from parity import DEFAULT_COV, DEFAULT_INIT, DEFAULT_MEAN, make_pair  # noqa: E402
from optimizer import _native  # noqa: E402

B, N_S, O, H, T = 32, 24, 3, 12, 3
ora, nat, xo, yo = make_pair(_native, "cvar", "beta", n=N_S, O=O, H=H, B=B, T=T, acc_c=0.05, steer_c=0.01)
draws = oracle.Draws.random(ora.prob, np.random.default_rng(3), idx_mpc=123, seed=0, with_beta_cem=False)
nat.begin("cvar", 123, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
p = ora.prob
t = 0
nat.run_stage(1, t)
nat.run_stage(2, t)
acc = nat.read("acc").reshape(B, 100)[:, :H]
steer = nat.read("steer").reshape(B, 100)[:, :H]
planes = nat.read("bplane", np.float32, (B, 2, H, N_S))
key = iteration_key(123, t, draws.seed)
elem = np.arange(N_S, dtype=np.uint64)[:, None] * np.uint64(H) + np.arange(H, dtype=np.uint64)[None, :]
elem = np.broadcast_to(elem, (B, N_S, H))
for kk, (ctl, sa, sb) in enumerate([(acc, STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B),
                                    (steer, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B)]):
    c = np.broadcast_to(np.abs(ctl)[:, None, :], (B, N_S, H))
    a_ = (np.float32(p.beta_a) * c).astype(np.float64)
    b_ = (np.float32(p.beta_b) * c).astype(np.float64)
    ref = beta_draws(a_, b_, key, sa, sb, elem)
    got = planes[:, kk].transpose(0, 2, 1)
    err = np.abs(got.astype(np.float64) - ref)
    bad = np.argwhere(err > 3e-7 + 1e-5 * np.abs(ref))
    print("plane", kk, "bad", len(bad))
    for (bi, ri, hi) in bad[:12]:
        e = int(elem[bi, ri, hi])
        print(f"  b={bi} r={ri} h={hi} got={got[bi, ri, hi]:.7g} ref={ref[bi, ri, hi]:.7g} a={a_[bi, ri, hi]:.6g}")
        for stream, al in ((sa, a_[bi, ri, hi]), (sb, b_[bi, ri, hi])):
            a1 = al + 1 if al < 1 else al
            d = a1 - 1 / 3
            cc = 1 / np.sqrt(9 * d)
            for k in range(4):
                u = philox4x32_10((np.uint64(e), k, stream, 1), key)
                rr = np.sqrt(-2.0 * np.log(_u01(u[0])))
                x = float(rr * np.cos((2.0 * np.pi) * _u01(u[1])))
                v = 1 + cc * x
                uu = float(_u01(u[2]))
                sq = uu < 1.0 - 0.0331 * x ** 4
                v3 = v ** 3 if v > 0 else 1.0
                lt = np.log(uu) - (0.5 * x * x + d - d * v3 + d * np.log(v3))
                vf = np.float32(1) + np.float32(cc) * np.float32(x)
                print(f"    stream {stream} alpha {al:.6g} k={k} x={x:.6g} v={v:.6g} vf={vf:.8g} sq={sq} "
                      f"logtest margin={lt:.3g}")
                if v > 0 and (sq or lt < 0):
                    break
