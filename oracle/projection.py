"""Restatement of ``S/opt/projection.py`` (class ``Projection``), one ADMM
iteration (``maxiter = 1``, ``S/opt/cem.py:88``), vectorised over candidates.
Obstacle terms (alpha_obs, d_obs, A_obs) are dead in the reference (commented
out of cost / lincost / residual / lambda) and are not computed.
Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

from .helper import cr

F32 = np.float32
F64 = np.float64


def f32(x):
    return np.asarray(x, dtype=F64).astype(F32)


def basis_eval(M, c):
    """jnp.dot(M, c.T).T with fp64 accumulation (sequential over the 11
    coefficients, the GPU's order): [B, 11] -> [B, rows]."""
    M = np.asarray(M, F64)
    c = np.asarray(c, F64)
    s = np.zeros((c.shape[0], M.shape[0]))
    for k in range(M.shape[1]):
        s = s + M[:, k][None, :] * c[:, k:k + 1]
    return f32(s)


def basis_adj(M, r):
    """jnp.dot(M.T, r.T).T with fp64 accumulation: [B, rows] -> [B, 11]."""
    return f32(np.asarray(r, F64) @ np.asarray(M, F64))


def unwrap(p):
    """``jnp.unwrap`` along the last axis (period 2 pi, discont pi), fp32;
    the correction cumsum is sequential."""
    pi = F32(np.pi)
    two_pi = F32(2 * np.pi)
    dd = np.diff(p, axis=-1)
    ddmod = np.mod(dd + pi, two_pi) - pi
    ddmod = np.where((ddmod == -pi) & (dd > 0), pi, ddmod).astype(F32)
    ph = np.where(np.abs(dd) < pi, F32(0), ddmod - dd).astype(F32)
    csum = np.empty_like(ph)
    acc = np.zeros(ph.shape[:-1], F32)
    for i in range(ph.shape[-1]):
        acc = (acc + ph[..., i]).astype(F32)
        csum[..., i] = acc
    out = p.copy()
    out[..., 1:] = p[..., 1:] + csum
    return out.astype(F32)


def _kkt_apply(prob, kinv, lin, b_eq):
    """fp64, sequential over the 11 right-hand-side rows (the GPU's order)."""
    s = np.broadcast_to(prob.kkt_rhs_const(kinv, b_eq), lin.shape).copy()
    neg = -lin.astype(F64)
    for j in range(11):
        s = s + kinv[:11, j][None, :] * neg[:, j:j + 1]
    return f32(s)


def _polar(wx, wy, lo, hi, unwrap_alpha):
    """alpha = atan2(wy, wx); d = clip((wx cos + wy sin)/(cos^2 + sin^2), lo, hi)
    (projection.py:75-98 and :217-243)."""
    alpha = cr(np.arctan2, wy, wx)
    if unwrap_alpha:
        alpha = unwrap(alpha)
    ca = cr(np.cos, alpha)
    sa = cr(np.sin, alpha)
    c1 = F32(1.0) * (ca * ca + sa * sa)
    c2 = F32(1.0) * (wx * ca + wy * sa)
    d = np.clip(c2 / c1, F32(lo), F32(hi))
    return alpha, d, ca, sa


def compute_projection(prob, b_eq_x, b_eq_y, lam_x, lam_y, cxb, cyb, s_lane):
    """``Projection.compute_projection`` (projection.py:276-323) =
    ``initial_alpha_d_obs`` (:52-121) -> ``compute_x`` (:123-185) ->
    ``compute_alph_d`` (:193-274).  Returns a dict of fp32 arrays."""
    P, Pd, Pdd = prob.P, prob.Pdot, prob.Pddot
    # guess trajectories (:282-289)
    xg, yg = basis_eval(P, cxb), basis_eval(P, cyb)
    xdg, ydg = basis_eval(Pd, cxb), basis_eval(Pd, cyb)
    xddg, yddg = basis_eval(Pdd, cxb), basis_eval(Pdd, cyb)
    del xg, yg
    # initial_alpha_d_obs (:73-119)
    alpha_v, d_v, cav, sav = _polar(xdg, ydg, prob.v_min, prob.v_max, True)
    alpha_a, d_a, caa, saa = _polar(xddg, yddg, 0.0, prob.a_max, True)
    res_ax = xddg - d_a * caa
    res_ay = yddg - d_a * saa
    res_vx = xdg - d_v * cav
    res_vy = ydg - d_v * sav
    lam_x = (lam_x - basis_adj(Pdd, res_ax)) - basis_adj(Pd, res_vx)
    lam_y = (lam_y - basis_adj(Pdd, res_ay)) - basis_adj(Pd, res_vy)

    # compute_x (:127-183)
    nm1 = prob.num - 1
    b_lane = np.concatenate([np.full(nm1, F32(prob.gamma * prob.y_ub)),
                             np.full(nm1, F32(-prob.gamma * prob.y_lb))]).astype(F32)
    b_lane_aug = b_lane[None, :] - s_lane
    b_ax, b_ay = d_a * caa, d_a * saa
    b_vx, b_vy = d_v * cav, d_v * sav
    lin_x = ((-lam_x - cxb) - basis_adj(Pdd, b_ax)) - basis_adj(Pd, b_vx)
    lin_y = (((-lam_y - cyb) - basis_adj(Pdd, b_ay)) - basis_adj(Pd, b_vy)) \
        - basis_adj(prob.A_lane, b_lane_aug)
    # KKT solve (:154-168) as c = Kinv[:11,:11] (-lincost) + Kinv[:11,11:] b_eq
    c_x = _kkt_apply(prob, prob.proj_kinv_x, lin_x, b_eq_x)
    c_y = _kkt_apply(prob, prob.proj_kinv_y, lin_y, b_eq_y)
    x, y = basis_eval(P, c_x), basis_eval(P, c_y)
    xd, yd = basis_eval(Pd, c_x), basis_eval(Pd, c_y)
    xdd, ydd = basis_eval(Pdd, c_x), basis_eval(Pdd, c_y)
    Ac = basis_eval(prob.A_lane, c_y)
    s_lane = np.maximum(F32(0), -Ac + b_lane[None, :])
    res_lane = (Ac - b_lane[None, :]) + s_lane

    # compute_alph_d (:217-272), no unwrap (Q13)
    alpha_v, d_v, cav, sav = _polar(xd, yd, prob.v_min, prob.v_max, False)
    alpha_a, d_a, caa, saa = _polar(xdd, ydd, 0.0, prob.a_max, False)
    res_ax = xdd - d_a * caa
    res_ay = ydd - d_a * saa
    res_vx = xd - d_v * cav
    res_vy = yd - d_v * sav

    def nrm(*parts):
        s = sum((np.asarray(p, F64) ** 2).sum(axis=1) for p in parts)
        return f32(np.sqrt(s))

    res_norm = (nrm(res_ax, res_ay) + nrm(res_vx, res_vy)) + nrm(res_lane)
    lam_x = (lam_x - basis_adj(Pdd, res_ax)) - basis_adj(Pd, res_vx)
    lam_y = ((lam_y - basis_adj(Pdd, res_ay)) - basis_adj(Pd, res_vy)) \
        - basis_adj(prob.A_lane, res_lane)
    return dict(c_x=c_x, c_y=c_y, x=x, y=y, xd=xd, yd=yd, xdd=xdd, ydd=ydd,
                res_norm=res_norm.astype(F32), lam_x=lam_x.astype(F32),
                lam_y=lam_y.astype(F32), s_lane=s_lane.astype(F32))


# ------------------------------------------------- CARLA det projection
def _obstacle_polar(prob, wc, ws):
    """alpha_obs, cos, sin and d_temp of ``C/opt/projection_det.py:69-73`` /
    ``:210-214`` on [..., O, 100] offsets wc = x - x_obs, ws = y - y_obs (fp32,
    the reference's operation order; transcendentals correctly rounded)."""
    a, b = F32(prob.a_obs), F32(prob.b_obs)
    alpha = cr(np.arctan2, ws * a, wc * b)
    ca = cr(np.cos, alpha)
    sa = cr(np.sin, alpha)
    c1 = F32(prob.a_obs ** 2) * (ca * ca) + F32(prob.b_obs ** 2) * (sa * sa)
    c2 = (a * wc) * ca + (b * ws) * sa
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        d_temp = (c2 / c1).astype(F32)
    return alpha, ca, sa, d_temp


def obs_adj(P, r):
    """jnp.dot(A_obs.T, r.T).T with A_obs = tile(P, (O, 1)): r [B, O, 100] ->
    [B, 11], fp64 accumulation rounded once."""
    B = r.shape[0]
    A = np.tile(np.asarray(P, F64), (r.shape[1], 1))
    return f32(np.asarray(r, F64).reshape(B, -1) @ A)


def compute_projection_det(prob, b_eq_x, b_eq_y, lam_x, lam_y, cxb, cyb, s_lane, x_obs, y_obs):
    """``Projection_det.compute_projection`` (C/opt/projection_det.py:279-336,
    ``C/`` = carla/): the projection of ``compute_projection`` with the
    obstacle terms live -- alpha_obs / d_obs on the guess (:60-74), the
    rho_obs A_obs terms in the KKT cost and linear cost (:143-169), the
    obstacle residual in res_norm and the multipliers (:201-274).  x_obs,
    y_obs: the Frenet obstacle tracks [O, 100].  Returns compute_projection's
    dict."""
    P, Pd, Pdd = prob.P, prob.Pdot, prob.Pddot
    xo = np.asarray(x_obs, F32)[None]
    yo = np.asarray(y_obs, F32)[None]
    kinv_x, kinv_y = prob.det_kinv()
    xg, yg = basis_eval(P, cxb), basis_eval(P, cyb)
    xdg, ydg = basis_eval(Pd, cxb), basis_eval(Pd, cyb)
    xddg, yddg = basis_eval(Pdd, cxb), basis_eval(Pdd, cyb)
    # initial_alpha_d_obs (:60-123): obstacle polar forms on the guess; the
    # multiplier update has no obstacle term there (:119-123)
    wc = xg[:, None, :] - xo
    ws = yg[:, None, :] - yo
    _, ca_o, sa_o, d_temp = _obstacle_polar(prob, wc, ws)
    d_obs0 = np.maximum(F32(1), d_temp)
    alpha_v, d_v, cav, sav = _polar(xdg, ydg, prob.v_min, prob.v_max, True)
    alpha_a, d_a, caa, saa = _polar(xddg, yddg, 0.0, prob.a_max, True)
    lam_x = (lam_x - basis_adj(Pdd, xddg - d_a * caa)) - basis_adj(Pd, xdg - d_v * cav)
    lam_y = (lam_y - basis_adj(Pdd, yddg - d_a * saa)) - basis_adj(Pd, ydg - d_v * sav)

    # compute_x (:128-189)
    nm1 = prob.num - 1
    b_lane = np.concatenate([np.full(nm1, F32(prob.gamma * prob.y_ub)),
                             np.full(nm1, F32(-prob.gamma * prob.y_lb))]).astype(F32)
    b_lane_aug = b_lane[None, :] - s_lane
    b_obs_x = xo + (d_obs0 * ca_o) * F32(prob.a_obs)
    b_obs_y = yo + (d_obs0 * sa_o) * F32(prob.b_obs)
    lin_x = (((-lam_x - cxb) - basis_adj(Pdd, d_a * caa)) - basis_adj(Pd, d_v * cav)) - obs_adj(P, b_obs_x)
    lin_y = ((((-lam_y - cyb) - basis_adj(Pdd, d_a * saa)) - basis_adj(Pd, d_v * sav))
             - basis_adj(prob.A_lane, b_lane_aug)) - obs_adj(P, b_obs_y)
    c_x = _kkt_apply(prob, kinv_x, lin_x, b_eq_x)
    c_y = _kkt_apply(prob, kinv_y, lin_y, b_eq_y)
    x, y = basis_eval(P, c_x), basis_eval(P, c_y)
    xd, yd = basis_eval(Pd, c_x), basis_eval(Pd, c_y)
    xdd, ydd = basis_eval(Pdd, c_x), basis_eval(Pdd, c_y)
    Ac = basis_eval(prob.A_lane, c_y)
    s_lane = np.maximum(F32(0), -Ac + b_lane[None, :])
    res_lane = (Ac - b_lane[None, :]) + s_lane

    # compute_alph_d (:198-276): d_obs >= 1 + (1 - gamma_obs)(d_obs_prev - 1)
    # with the previous d_obs shifted one step (comp_d_obs_prev, :192-195)
    wc = x[:, None, :] - xo
    ws = y[:, None, :] - yo
    _, ca_o, sa_o, d_temp = _obstacle_polar(prob, wc, ws)
    prev = np.concatenate([np.ones(d_obs0.shape[:-1] + (1,), F32), d_obs0[..., :-1]], axis=-1)
    with np.errstate(invalid="ignore"):
        lo = F32(1) + F32(1.0 - 1.0) * (prev - F32(1))     # gamma_obs = 1 (C/opt/cem.py:125)
    d_obs = np.maximum(lo, d_temp)
    res_xo = wc - (F32(prob.a_obs) * d_obs) * ca_o
    res_yo = ws - (F32(prob.b_obs) * d_obs) * sa_o
    alpha_v, d_v, cav, sav = _polar(xd, yd, prob.v_min, prob.v_max, False)
    alpha_a, d_a, caa, saa = _polar(xdd, ydd, 0.0, prob.a_max, False)
    res_ax = xdd - d_a * caa
    res_ay = ydd - d_a * saa
    res_vx = xd - d_v * cav
    res_vy = yd - d_v * sav

    def nrm(*parts):
        s = sum((np.asarray(p, F64) ** 2).reshape(p.shape[0], -1).sum(axis=1) for p in parts)
        return f32(np.sqrt(s))

    res_norm = ((nrm(res_ax, res_ay) + nrm(res_vx, res_vy)) + nrm(res_lane)) + nrm(res_xo, res_yo)
    lam_x = ((lam_x - basis_adj(Pdd, res_ax)) - basis_adj(Pd, res_vx)) - obs_adj(P, res_xo)
    lam_y = (((lam_y - basis_adj(Pdd, res_ay)) - basis_adj(Pd, res_vy)) - basis_adj(prob.A_lane, res_lane)) \
        - obs_adj(P, res_yo)
    return dict(c_x=c_x, c_y=c_y, x=x, y=y, xd=xd, yd=yd, xdd=xdd, ydd=ydd,
                res_norm=res_norm.astype(F32), lam_x=lam_x.astype(F32),
                lam_y=lam_y.astype(F32), s_lane=s_lane.astype(F32))
