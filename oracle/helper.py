"""Restatement of ``S/opt/cem_helper.py`` (class ``Helper``), vectorised over
the candidate batch.  fp32 elementwise in reference order; small dense algebra
accumulated in fp64 and rounded to fp32 (see ``oracle/__init__.py``).
Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

from .rng import STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B
from .rng import beta_draws, iteration_key

F32 = np.float32
F64 = np.float64


def f32(x):
    return np.asarray(x, dtype=F64).astype(F32)


def sort_key(x):
    """Total order used by jnp.argsort on fp32: -0 == +0, NaN last (all NaNs
    equal).  Returns uint64 keys (ascending == reference order)."""
    x = np.asarray(x, dtype=F32).copy()
    x[x == 0] = F32(0.0)
    nan = np.isnan(x)
    b = x.view(np.uint32).astype(np.uint64)
    neg = (b >> np.uint64(31)) == 1
    k = np.where(neg, np.uint64(0xFFFFFFFF) - b, b | np.uint64(0x80000000))
    k = np.where(nan, np.uint64(0xFFFFFFFF), k)
    return k


def argsort_stable(x):
    """``jnp.argsort`` (stable, ascending, NaN last)."""
    return np.argsort(sort_key(x), kind="stable")


def chol64(a):
    return np.linalg.cholesky(np.asarray(a, dtype=F64))


def mvn_rows(mean, cov, z):
    """``jax.random.multivariate_normal`` with method='cholesky' applied to
    injected standard normals: mean + L z (fp64, rounded to fp32)."""
    L = chol64(cov)
    return f32(np.asarray(mean, F64) + np.asarray(z, F64) @ L.T)


def clip_v(pop, prob):
    """clip v_des_1..4 to [v_min, v_max] (cem_helper.py:138-145, 304-307)."""
    pop = pop.copy()
    pop[:, 0:4] = np.clip(pop[:, 0:4], F32(prob.v_min), F32(prob.v_max))
    return pop


def sampling_param(prob, mean, cov, z):
    """``Helper.sampling_param`` (cem_helper.py:122-150): B MVN draws, fixed key."""
    return clip_v(mvn_rows(mean, cov, z), prob)


def compute_boundary_vec(prob, init_state):
    """``Helper.compute_boundary_vec`` (cem_helper.py:152-167); b_eq shared by
    every candidate, returned un-broadcast: b_eq_x [3], b_eq_y [4]."""
    x0, y0, vx0, vy0, ax0, ay0 = (F32(v) for v in init_state)
    return np.array([x0, vx0, ax0], F32), np.array([y0, vy0, ay0, 0.0], F32)


def compute_x_guess(prob, b_eq_x, b_eq_y, pop):
    """``Helper.compute_x_guess`` (cem_helper.py:169-230): 4-segment PD-tracking
    QP.  lincost_x = -sum_k A_vd_k^T b_vd_k with b_vd_k = -k_p_v v_k 1, so the
    KKT solution is affine in the 8 parameters: c_bar = G v + h with the
    batch-invariant G = Kinv[:11,:11] (-k_p colsum) and h = Kinv[:11,11:] b_eq
    (fp64, fixed summation order; reference: fp32 LU per call)."""
    p = pop.astype(F64)
    out = []
    for xy, (kinv, b, cols) in enumerate(((prob.guess_kinv_x, b_eq_x, slice(0, 4)),
                                          (prob.guess_kinv_y, b_eq_y, slice(4, 8)))):
        s = np.broadcast_to(prob.kkt_rhs_const(kinv, b), (pop.shape[0], 11)).copy()
        v = p[:, cols]
        for j in range(4):
            s = s + prob.guess_G[xy][:, j][None, :] * v[:, j:j + 1]
        out.append(f32(s))
    return out[0], out[1]


def cr(fn, *args):
    """Correctly rounded fp32 transcendental: evaluate in fp64, round once.
    Used by the projection / controls stage on both the oracle and the GPU
    (DESIGN.md Numerics: the feasible candidates' res_norm is rounding noise,
    so its order is only reproducible with reproducible transcendentals)."""
    return fn(*(np.asarray(a, F32).astype(F64) for a in args)).astype(F32)


def compute_controls(prob, xd, yd, xdd, ydd):
    """``Helper.compute_controls`` (cem_helper.py:540-551).  Returns acc
    [B, 101] and steer [B, 100] exactly as the reference shapes them."""
    v = np.sqrt(xd * xd + yd * yd)
    v = np.hstack([v, v[:, -1:]])
    acc = np.diff(v, axis=1) / F32(prob.t)
    acc = np.hstack([acc, acc[:, -1:]])
    s2 = xd * xd + yd * yd
    curv = (ydd * xd - yd * xdd) / cr(lambda a: np.power(a, 1.5), s2)
    steer = cr(np.arctan, curv * F32(prob.wheel_base))
    return acc.astype(F32), steer.astype(F32)


def compute_obs_trajectories(prob, x_obs, y_obs, vx_obs, vy_obs, psi_obs):
    """``Helper.compute_obs_trajectories`` (cem_helper.py:366-378)."""
    tt = prob.tot_time.astype(F32)[:, None]
    xo = (np.asarray(x_obs, F32) + np.asarray(vx_obs, F32) * tt).T
    yo = (np.asarray(y_obs, F32) + np.asarray(vy_obs, F32) * tt).T
    po = np.tile(np.asarray(psi_obs, F32), (prob.num, 1)).T
    return xo.astype(F32), yo.astype(F32), po.astype(F32)


def noisy_controls(prob, acc, steer, draws, t, rows):
    """Noise injection shared by ``compute_rollout_complete_baseline`` and
    ``_opt`` (cem_helper.py:405-443 / 469-508).

    acc, steer: [B, H] (first H controls of each candidate).  ``rows`` noise
    rows per candidate share one realisation (vmap key in_axes=None, Q2).
    Returns acc_n, steer_n [B, rows, H] fp32.
    """
    B, H = acc.shape
    n_a, n_s, n_c = draws.roll[t, 0], draws.roll[t, 1], draws.roll[t, 2]
    assert n_c.shape == (rows, H)
    nba = nbs = None
    if prob.noise != "gaussian":
        a = np.abs(acc[:, None, :])
        s = np.abs(steer[:, None, :])
        key = iteration_key(draws.idx_mpc, t, draws.seed)
        elem = (np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(H)
                + np.arange(H, dtype=np.uint64)[None, :])
        elem = np.broadcast_to(elem, (B, rows, H))
        aa = np.broadcast_to(a, (B, rows, H))
        ss = np.broadcast_to(s, (B, rows, H))
        nba = beta_draws((F32(prob.beta_a) * aa).astype(F64), (F32(prob.beta_b) * aa).astype(F64),
                         key, STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B, elem)
        nbs = beta_draws((F32(prob.beta_a) * ss).astype(F64), (F32(prob.beta_b) * ss).astype(F64),
                         key, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B, elem)
    return inject_noise(prob, acc, steer, n_a, n_s, n_c, nba, nbs)


def inject_noise(prob, acc, steer, n_a, n_s, n_c, beta_acc=None, beta_steer=None):
    """The perturbation itself (cem_helper.py:405-443): gaussian
    ``a + sigma |a| n_a + c_a n_c``; beta ``a + sigma (2 b_a - 1) + c_a n_c``
    and ``s + K_steer sigma (2 b_s - 1) + c_s n_c`` with the Beta draws given
    ([B, rows, H]).  acc, steer [B, H]; n_* [rows, H]."""
    a = acc[:, None, :]
    s = steer[:, None, :]
    if prob.noise == "gaussian":
        acc_pert = (F32(prob.sigma_acc) * np.abs(a)) * np.asarray(n_a, F32)[None]
        steer_pert = (F32(prob.sigma_steer) * np.abs(s)) * np.asarray(n_s, F32)[None]
    else:
        acc_pert = F32(prob.sigma_acc) * (F32(2) * np.asarray(beta_acc, F32) - F32(1))
        steer_pert = F32(prob.K_steer * prob.sigma_steer) * (F32(2) * np.asarray(beta_steer, F32) - F32(1))
    n_c = np.asarray(n_c, F32)[None]
    acc_n = (a + acc_pert) + prob.acc_const_noise * n_c
    steer_n = (s + steer_pert) + prob.steer_const_noise * n_c
    return acc_n.astype(F32), steer_n.astype(F32)


def initial_state5(init_state):
    x0, y0, vx0, vy0 = (F32(init_state[i]) for i in range(4))
    return np.array([x0, y0, vx0, vy0, np.arctan2(vy0, vx0)], F32)


def rollout(prob, acc_n, steer_n, st0):
    """H-step kinematic bicycle scan (cem_helper.py:380-400, 445-461).
    acc_n/steer_n [..., H]; returns x_roll, y_roll [..., H] (state before each
    step; the last step's output is never recorded)."""
    H = acc_n.shape[-1]
    t = F32(prob.t)
    wb = F32(prob.wheel_base)
    shp = acc_n.shape[:-1]
    x = np.full(shp, st0[0], F32)
    y = np.full(shp, st0[1], F32)
    vx = np.full(shp, st0[2], F32)
    vy = np.full(shp, st0[3], F32)
    psi = np.full(shp, st0[4], F32)
    xr = np.empty(acc_n.shape, F32)
    yr = np.empty(acc_n.shape, F32)
    for h in range(H):
        xr[..., h] = x
        yr[..., h] = y
        v = np.sqrt(vx * vx + vy * vy)
        v = v + acc_n[..., h] * t
        psidot = (v * np.tan(steer_n[..., h])) / wb
        psi = psi + psidot * t
        vx = v * np.cos(psi)
        vy = v * np.sin(psi)
        x = x + vx * t
        y = y + vy * t
    return xr, yr


def mother_controls(acc_n, steer_n):
    """jnp.repeat(acc, n, 0) / jnp.tile(steer, (n, 1)) (cem_helper.py:510-511):
    mother row m = (acc row m // n, steer row m % n)."""
    n = acc_n.shape[-2]
    acc_m = np.repeat(acc_n, n, axis=-2)
    steer_m = np.tile(steer_n, (1,) * (steer_n.ndim - 2) + (n, 1))
    return acc_m, steer_m


def compute_coeff(prob, x, y):
    """``Helper.compute_coeff`` (cem_helper.py:553-564): ridge fit to the
    horizon basis, c = (P'^T P' + 0.05 I)^-1 P'^T x.  The batch-invariant
    matrix Fit = (P'^T P' + 0.05 I)^-1 P'^T [11, H] is built once
    (problem.py) and applied in fp64, sequentially over the horizon (the GPU
    folds it into the rollout scan in the same order)."""
    fit = prob.fit
    cx = np.zeros(x.shape[:-1] + (11,))
    cy = np.zeros(y.shape[:-1] + (11,))
    xd = np.asarray(x, F64)
    yd = np.asarray(y, F64)
    for h in range(x.shape[-1]):
        cx = cx + fit[:, h] * xd[..., h:h + 1]
        cy = cy + fit[:, h] * yd[..., h:h + 1]
    return f32(cx), f32(cy)


def _norm(x):
    x = np.asarray(x, F64)
    return np.sqrt((x * x).sum(axis=-1))


def compute_cost(prob, cost_obs, cost_lane, y, res, xd, yd, xdd, ydd, v_des, steer):
    """``Helper.compute_cost`` (cem_helper.py:232-262); each norm in fp64, the
    weighted sum in fp64, rounded once.  0*x terms are kept (NaN propagates)."""
    v_des = F32(v_des)
    des = _norm(y - F32(prob.y_des_1))
    c_st = _norm(steer)
    sv = np.diff(steer, axis=1)
    c_sv = _norm(sv)
    sa = np.diff(sv, axis=1)
    c_sa = _norm(sa)
    v = np.sqrt(xd * xd + yd * yd)
    c_sp = _norm(np.maximum(F32(0), np.abs(steer) - F32(prob.steer_max)))
    c_svp = _norm(np.maximum(F32(0), np.abs(sv) - F32(0.05)))
    tot = (np.asarray(res, F64) + 0.1 * _norm(v - v_des) + 0.1 * (c_st + c_sv + c_sa)
           + 0.1 * (c_sp + c_svp) + 0.02 * _norm(ydd) + 0.02 * _norm(xdd)
           + 0.0 * des + np.asarray(cost_obs, F64) + 0.0 * np.asarray(cost_lane, F64))
    return f32(tot)


def compute_shifted_samples(prob, pop_elite, cost_sorted5, mean_prev, cov_prev, z):
    """``Helper.compute_shifted_samples`` (cem_helper.py:280-314).

    pop_elite [5, 8] (already cost-sorted), cost_sorted5 [5].  Weighted
    mean/cov EMA in fp64 (state kept fp32), B-5 MVN draws, v clipped."""
    c = np.asarray(cost_sorted5, F64)
    w = np.exp(-(1.0 / prob.lamda) * (c - c.min()))
    sw = w.sum()
    e = pop_elite.astype(F64)
    mean = f32((1 - prob.alpha_mean) * mean_prev.astype(F64) + prob.alpha_mean * (w[:, None] * e).sum(0) / sw)
    d = e - mean.astype(F64)
    prod = (w[:, None, None] * d[:, :, None] * d[:, None, :]).sum(0)
    cov = f32((1 - prob.alpha_cov) * cov_prev.astype(F64) + prob.alpha_cov * prod / sw + 0.01 * np.eye(8))
    new = clip_v(mvn_rows(mean, cov, z), prob)
    pop = np.vstack([pop_elite.astype(F32), new])
    return mean, cov, pop
