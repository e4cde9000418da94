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
