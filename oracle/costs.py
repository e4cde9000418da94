"""Restatement of ``S/opt/costs.py`` (class ``Costs``) and
``S/kernel_computation.py`` (class ``kernel_matrix``).
Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
F64 = np.float64


def f32(x):
    return np.asarray(x, dtype=F64).astype(F32)


def compute_f_bar(prob, x, y, x_obs, y_obs):
    """``compute_f_bar`` (costs.py:50-60) per (obstacle, sample, step).

    x, y [..., H]; x_obs, y_obs [O, H] -> f_bar [O, ..., H] fp32.
    cost = (-(dx^2)/a^2 - dy^2/b^2) + 1, then max(0, cost).
    """
    a2 = F32(prob.a_obs ** 2)
    b2 = F32(prob.b_obs ** 2)
    out = []
    for o in range(x_obs.shape[0]):
        wc = x - x_obs[o]
        ws = y - y_obs[o]
        c = ((-(wc * wc)) / a2 - (ws * ws) / b2) + F32(1)
        out.append(np.maximum(F32(0), c))
    return np.stack(out).astype(F32)


def compute_f_bar_max(prob, x, y, x_obs, y_obs):
    """``compute_f_bar`` reduced by max over (obstacle, time) as every caller
    does (costs.py:177-180, 195, 210-213, 227-230): costbar [...] fp32."""
    out = np.zeros(x.shape[:-1], F32)
    for c in compute_f_bar(prob, x, y, x_obs, y_obs):
        out = np.maximum(out, c.max(axis=-1))
    return out


def lane_bar(prob, y):
    """``compute_lane_bar`` (costs.py:62-71) per (sample, step): (lb, ub)."""
    lb = np.maximum(F32(0), -y + F32(prob.y_lb))
    ub = np.maximum(F32(0), y - F32(prob.y_ub))
    return lb.astype(F32), ub.astype(F32)


def lane_bar_max(prob, y):
    """``compute_lane_bar`` max-reduced over time (costs.py:126-127, 142, 150,
    165, 168): returns (lb, ub) [...]."""
    lb, ub = lane_bar(prob, y)
    return lb.max(axis=-1), ub.max(axis=-1)


def quantile_linear(x, q):
    """``jnp.quantile(x, q)`` (linear interpolation) with JAX's fp32 weights:
    pos = q*(n-1) in fp32, low = floor, w = pos - low."""
    x = np.asarray(x, F32)
    n = x.shape[-1]
    pos = F32(q) * F32(n - 1)
    lo = np.floor(pos)
    hi = np.ceil(pos)
    hw = F32(pos - lo)
    lw = F32(F32(1) - hw)
    lo_i = int(min(max(lo, 0), n - 1))
    hi_i = int(min(max(hi, 0), n - 1))
    xs = np.sort(x, axis=-1)   # NaN last, like lax.sort
    return (xs[..., lo_i] * lw + xs[..., hi_i] * hw).astype(F32)


def cvar(prob, costbar):
    """CVaR_0.98 of ``costbar`` [..., S] (costs.py:215-219): VaR by linear
    quantile, mean of the samples >= VaR (fp64 sum), 0 if none."""
    var = quantile_linear(costbar, prob.alpha_quant)
    m = (costbar >= var[..., None]) & ~np.isnan(costbar)
    cnt = m.sum(axis=-1)
    s = np.where(m, costbar.astype(F64), 0.0).sum(axis=-1)
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.where(cnt > 0, s / np.maximum(cnt, 1), 0.0)
    return f32(r)


def saa(prob, costbar):
    """SAA (costs.py:230-234): fraction of samples with costbar > 0."""
    n = costbar.shape[-1]
    cnt = (costbar > F32(0)).sum(axis=-1)
    return (cnt.astype(F32) / F32(n)).astype(F32)


def mmd(prob, beta, cost, sigma):
    """``kernel_matrix.compute_mmd`` (kernel_computation.py:67-87) with the
    Laplace kernel of ``compute_kernel_matrix`` (:33-39) on 1-D costs and a
    Dirac-at-0 target: ker_wt*(b^T K_aa b - 2 b^T K_ab b_del), K_bb dropped.

    beta, cost [..., n]; sigma [...] -> [...] fp32.  Kernel entries fp32,
    quadratic forms fp64.
    """
    beta = np.asarray(beta, F32)
    cost = np.asarray(cost, F32)
    n = cost.shape[-1]
    sig = np.asarray(sigma, F32)[..., None, None]
    d_aa = np.abs(cost[..., :, None] - cost[..., None, :])
    K_aa = np.exp((-d_aa) / sig).astype(F32)
    d_ab = np.abs(cost - F32(0))
    K_ab = np.exp((-d_ab) / sig[..., 0]).astype(F32)            # [..., n] (all columns equal)
    b = beta.astype(F64)
    bdel = F64(F32(1.0 / n))
    q1 = np.einsum("...i,...ij,...j->...", b, K_aa.astype(F64), b)
    q2 = np.einsum("...i,...i->...", b, K_ab.astype(F64) * (n * bdel))
    return f32(prob.ker_wt * (q1 - 2.0 * q2))


def mmd_lane(prob, beta, sigma, y_red):
    """``Costs.compute_mmd_lane`` (costs.py:121-135)."""
    lb, ub = lane_bar_max(prob, y_red)
    return (mmd(prob, beta, lb, sigma) + mmd(prob, beta, ub, sigma)).astype(F32)


def cvar_lane(prob, y):
    """``Costs.compute_cvar_lane`` (costs.py:137-158)."""
    lb, ub = lane_bar_max(prob, y)
    return (cvar(prob, lb) + cvar(prob, ub)).astype(F32)


def saa_lane(prob, y):
    """``Costs.compute_saa_lane`` (costs.py:160-171)."""
    lb, ub = lane_bar_max(prob, y)
    n = y.shape[-2]
    cnt = (lb > 0).sum(axis=-1) + (ub > 0).sum(axis=-1)
    return (cnt.astype(F32) / F32(n)).astype(F32)
