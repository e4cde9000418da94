"""GPU diagnostic: CARLA compute_cem_cvar with Beta noise -- the Beta planes
of iterations 0..2 against the oracle's draws on the GPU's own controls;
prints the elements outside tolerance with their Beta parameters."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpc-mmd_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
os.environ["MPCMMD_BETA_DUMP"] = "1"
from optimizer import _native as native  # noqa: E402
from oracle import carla as K  # noqa: E402
from oracle.rng import (STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B, STREAM_GAMMA_STEER_A,  # noqa: E402
                        STREAM_GAMMA_STEER_B, beta_draws, iteration_key)
import test_gpu_carla as T  # noqa: E402

n, B, H, O, level = 12, 100, 60, 3, 0.3
init, xo, yo, path = T._tick(60, O, H)
ora = K.CarlaCEM(n, 1, O, level, H, "beta", "Town05", 0.0, 0.0, num_batch=B, maxiter_cem=20)
nat = native.Handle(native.make_config(n, O, level, H, "beta", 0.0, 0.0, num_batch=B, maxiter_cem=20,
                                       variant="carla_town05"))
draws = K.CarlaDraws.random(ora.prob, np.random.default_rng(7), idx_mpc=5, with_beta_cem=False)
nat.carla_begin("cvar", 5, init, T.MEAN, T.COV, xo, yo, 10.0, path, draws)
p = ora.prob
for t in range(3):
    nat.iterate(t, 1)
    nat.sync()
    acc = nat.read("acc").reshape(-1, 100)[:B, :H]
    steer = nat.read("steer").reshape(-1, 100)[:B, :H]
    planes = nat.read("bplane", np.float32, (B, 2, H, n))
    key = iteration_key(5, t, draws.seed)
    elem = np.arange(n, dtype=np.uint64)[:, None] * np.uint64(H) + np.arange(H, dtype=np.uint64)[None, :]
    elem = np.broadcast_to(elem, (B, n, H))
    for k, (ctl, sa, sb) in enumerate([(acc, STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B),
                                       (steer, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B)]):
        c = np.broadcast_to(np.abs(ctl)[:, None, :], (B, n, H))
        ref = beta_draws((np.float32(p.beta_a) * c).astype(np.float64), (np.float32(p.beta_b) * c).astype(np.float64),
                         key, sa, sb, elem)
        got = planes[:, k].transpose(0, 2, 1)[:, :, :H - 1]
        ref = ref[:, :, :H - 1]
        err = np.abs(got.astype(np.float64) - ref)
        bad = np.argwhere(~(err <= 1e-5 + 1e-4 * np.abs(ref)))
        print(f"t={t} plane {'acc' if k == 0 else 'steer'}: {len(bad)} elements outside; worst {np.nanmax(err):.3g}")
        for (bb, r, h) in bad[:12]:
            print(f"   cand {bb} row {r} step {h}: |u| {c[bb, r, h]:.3e} got {got[bb, r, h]!r} ref {ref[bb, r, h]!r}")
