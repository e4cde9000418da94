"""Monte-Carlo validation (oracle side; TEST INFRASTRUCTURE ONLY, see
``oracle/__init__.py``).

NumPy restatement of ``synthetic_static_obs/validation.py``:
``compute_controls`` (:122-132), ``compute_rollout_complete`` (:42-101),
``compute_rollout_one_step`` (:21-40), ``compute_f_bar_temp`` (:103-110),
``compute_lane_bar`` (:112-120) and the counting of ``compute_stats``
(:134-171), all in fp64 like the original, vectorised over the rollouts.
Draws are explicit ([3][R][H]: acc, steer, const -- the Beta draws for
beta noise) or the library's Philox streams (streams 24-30, keyed by the
configuration key and the seed; csrc/k_validate.hip).
"""
from __future__ import annotations

import numpy as np

from . import rng
from .problem import Problem

F64 = np.float64
STREAM_VAL_ACC, STREAM_VAL_STEER, STREAM_VAL_CONST = 24, 25, 26
STREAM_VAL_GAMMA = (27, 28, 29, 30)  # acc A, acc B, steer A, steer B


def controls(prob, cx, cy):
    """compute_controls on the saved coefficients (:122-132, :140-145)."""
    Pd = prob.Pdot.astype(np.float32).astype(F64)
    Pdd = prob.Pddot.astype(np.float32).astype(F64)
    cx = np.asarray(cx, F64)
    cy = np.asarray(cy, F64)
    xd, xdd = Pd @ cx, Pdd @ cx
    yd, ydd = Pd @ cy, Pdd @ cy
    v = np.sqrt(xd ** 2 + yd ** 2)
    v = np.hstack((v, v[-1]))
    acc = np.diff(v) / 0.15
    acc = np.hstack((acc, acc[-1]))
    curv = (ydd * xd - yd * xdd) / ((xd ** 2 + yd ** 2) ** 1.5)
    return acc, np.arctan(curv * 2.5)


def _beta64(a, b, key, sa, sb, elem):
    ga, ua = rng._log_gamma_parts(a, key, sa, elem)
    gb, ub = rng._log_gamma_parts(b, key, sb, elem)
    sa_ = np.where(a > 0, a, 1.0)
    sb_ = np.where(b > 0, b, 1.0)
    la = np.where(a < 1.0, ga + ua / sa_, ga)
    lb = np.where(b < 1.0, gb + ub / sb_, gb)
    with np.errstate(over="ignore", invalid="ignore"):   # np.where evaluates both branches
        out = np.where(la > lb, 1.0 / (1.0 + np.exp(lb - la)), np.exp(la - lb) / (np.exp(la - lb) + 1.0))
    lim = np.where(ua * 5.0 > ub * 2.0, 1.0, 0.0)
    return np.where((a == 0.0) & (b == 0.0), lim, out)


def draws_philox(prob, acc, steer, noise, R, H, key, seed=0):
    k = (int(key) & 0xFFFFFFFF, int(seed) & 0xFFFFFFFF)
    n = R * H
    def normals(stream):  # fp64 Box-Muller values (the device does not round them)
        nblk = (n + 3) // 4
        j = np.arange(nblk, dtype=np.uint64)
        u = rng.philox4x32_10((j, 0, stream, 0), k)
        z0, z1 = rng._box_muller(u[0], u[1])
        z2, z3 = rng._box_muller(u[2], u[3])
        return np.stack([z0, z1, z2, z3], axis=1).reshape(-1)[:n].reshape(R, H)
    nc = normals(STREAM_VAL_CONST)
    if noise == "gaussian":
        return np.stack([normals(STREAM_VAL_ACC), normals(STREAM_VAL_STEER), nc])
    elem = (np.arange(R, dtype=np.uint64)[:, None] * np.uint64(H) + np.arange(H, dtype=np.uint64)[None, :])
    fa = np.abs(acc[:H])[None, :] * np.ones((R, 1))
    fs = np.abs(steer[:H])[None, :] * np.ones((R, 1))
    ba = _beta64(2.0 * fa, 5.0 * fa, k, STREAM_VAL_GAMMA[0], STREAM_VAL_GAMMA[1], elem)
    bs = _beta64(2.0 * fs + 1e-5, 5.0 * fs + 1e-5, k, STREAM_VAL_GAMMA[2], STREAM_VAL_GAMMA[3], elem)
    return np.stack([ba, bs, nc])


def draws_numpy(noise, acc, steer, R, H, key):
    """The reference's own draws of compute_rollout_complete (:42-92):
    ``np.random.seed(key)``, then NumPy multivariate_normal (gaussian) or
    beta draws for acc and steer, then the const-noise normals -- as the
    [3][R][H] array ``compute_stats`` / the GPU kernel take (for beta noise
    rows 0 and 1 are the Beta samples themselves)."""
    np.random.seed(key)
    acc = np.asarray(acc, F64)[:H]
    steer = np.asarray(steer, F64)[:H]
    if noise == "gaussian":
        na = np.random.multivariate_normal(np.zeros(H), np.eye(H), (R,))
        ns = np.random.multivariate_normal(np.zeros(H), np.eye(H), (R,))
    else:
        na = np.random.beta(2 * np.abs(acc), 5 * np.abs(acc), (R, H))
        ns = np.random.beta(2 * np.abs(steer) + 1e-5, 5 * np.abs(steer) + 1e-5, (R, H))
    nc = np.random.multivariate_normal(np.zeros(H), np.eye(H), (R,))
    return np.stack([na, ns, nc])


def compute_stats(prob: Problem, cx, cy, init_state, x_obs_traj, y_obs_traj, noise, noise_level, acc_const,
                  steer_const, draws, return_rollouts=False):
    """(count, count_lane) of one configuration (:134-171).  x_obs_traj,
    y_obs_traj [O][100] fp32; draws [3][R][H].  With return_rollouts also
    the [R][H] x / y rollouts (:148-149)."""
    H = prob.num_prime
    acc, steer = controls(prob, cx, cy)
    acc, steer = acc[:H], steer[:H]
    na, ns, nc = (np.asarray(d, F64) for d in draws)
    R = na.shape[0]
    if noise == "gaussian":
        acc_pert = noise_level * np.abs(acc) * na                     # :81-82
        steer_pert = noise_level * np.abs(steer) * ns
    else:
        acc_pert = noise_level * (2 * na - 1)                         # :91-92
        steer_pert = prob.K_steer * noise_level * (2 * ns - 1)
    acc_n = acc + acc_pert + acc_const * nc                           # :97-98
    steer_n = steer + steer_pert + steer_const * nc
    st = np.asarray(init_state, F64).reshape(-1)
    x = np.full(R, st[0])
    y = np.full(R, st[1])
    vx = np.full(R, st[2])
    vy = np.full(R, st[3])
    psi = np.full(R, np.arctan2(st[3], st[2]))
    xr = np.zeros((R, H))
    yr = np.zeros((R, H))
    for h in range(H):                                                # :94-99
        xr[:, h], yr[:, h] = x, y
        v = np.sqrt(vx ** 2 + vy ** 2)
        v = v + acc_n[:, h] * 0.15
        psidot = v * np.tan(steer_n[:, h]) / 2.5
        psi = psi + psidot * 0.15
        vx = v * np.cos(psi)
        vy = v * np.sin(psi)
        x = x + vx * 0.15
        y = y + vy * 0.15
    xo = np.asarray(x_obs_traj, np.float32)[:, :H].astype(F64)
    yo = np.asarray(y_obs_traj, np.float32)[:, :H].astype(F64)
    wc = xr[None] - xo[:, None]
    ws = yr[None] - yo[:, None]
    cost = -(wc ** 2) / (4.25 ** 2) - (ws ** 2) / (2.75 ** 2) + 1.0   # :106-108
    count = int(np.max(np.count_nonzero(np.maximum(0.0, cost), axis=1)))
    lb = np.maximum(0.0, -yr + prob.y_lb)
    ub = np.maximum(0.0, yr - prob.y_ub)
    count_lane = int(np.max(np.count_nonzero(lb, axis=0)) + np.max(np.count_nonzero(ub, axis=0)))
    if return_rollouts:
        return count, count_lane, xr, yr
    return count, count_lane
