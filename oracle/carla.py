"""Restatement of the CARLA optimizer variant (``C/optimizer/*.py``; ``C/`` =
``carla/``, ``C/opt/`` = ``carla/optimizer/``): the Frenet-frame CEM of
``C/main_carla.py`` with its path helpers.  Test infrastructure only (see
``oracle/__init__.py``).

What differs from the static optimizer (``S/opt``), all restated here:
  * constants (``C/opt/cem.py:25-36,152-182``; ``oracle/problem.py`` variant
    "carla_town05" / "carla_town10hd");
  * noisy initial states (``C/opt/cem_helper.py:660-715``): one per rollout row,
    their Frenet transforms averaged into the boundary vectors
    (``C/opt/cem.py:248-264, 476-492``);
  * the projection also interpolates the path curvature at the Frenet
    station and returns a steering angle (``C/opt/projection.py:307-319``);
  * rollouts run in the (ego-shifted) global frame from the noisy initial
    states and are mapped to Frenet coordinates by an argmin over the path
    (``C/opt/cem_helper.py:206-242``) before the collision / lane costs;
  * lane and desired-lane costs with non-zero weights, and a cost with a
    desired-lane and a centripetal term (``C/opt/costs.py:70-153``,
    ``C/opt/cem_helper.py:522-556``);
  * the solve returns (cx, cy, v, steering, mean_param) (``C/opt/cem.py:413-441``).

Numerics (shared with the HIP library): as for the static path, plus
  * ``jnp.interp`` restated from jax 0.3.23 (``requirements.txt:1``; third
    party, not vendored, so this is its published formula, unpinned):
    f = fp[i-1] + ((x - xp[i-1]) / dx[i-1]) * df[i-1], i = clip(searchsorted
    (xp, x, 'right'), 1, P-1), fp[0] / fp[-1] outside the grid;
  * rollout transcendentals (tan, sin, cos) and the projection's steering
    (sin, cos, atan) evaluated in fp64 and rounded once on both sides, so the
    rollouts - and with them the Frenet argmins, whose near-ties would
    otherwise flip on ulp-level differences - are reproducible;
  * path smoothing (``C/opt/cem_helper.py:112-131,279-318,391-410``): the
    601 x 601 KKT matrix inverted once in fp64 by the fixed-order Gauss-Jordan
    of ``problem.gauss_jordan_inverse`` (the reference: jnp.linalg.inv, fp32)
    and applied as fp64 GEMVs; the arc-length cumsum in fp64 (the reference's
    fp32 parallel prefix rounds differently).
"""
from __future__ import annotations

import numpy as np

from . import beta_cem as bc
from . import costs as C
from . import helper as H
from .cem import CEM
from .helper import cr
from .projection import basis_adj, basis_eval, _kkt_apply, _polar, unwrap  # noqa: F401
from .rng import STREAM_INIT_EPS, Draws, philox_normals

F32 = np.float32
F64 = np.float64
# C/opt/cem.py:161-166: only the exact name "Town10HD" selects its constants
# (Town10HD_Opt and any other town get Town05's)
TOWNS = {"Town05": "carla_town05", "Town10HD": "carla_town10hd"}


def f32(x):
    return np.asarray(x, dtype=F64).astype(F32)


# ---------------------------------------------------------------- jnp.interp
def interp(x, xp, fp):
    """``jnp.interp(x, xp, fp)`` (jax 0.3.23), fp32, x of any shape."""
    x = np.asarray(x, F32)
    xp = np.asarray(xp, F32)
    fp = np.asarray(fp, F32)
    P = xp.shape[0]
    df = (fp[1:] - fp[:-1]).astype(F32)
    dx = (xp[1:] - xp[:-1]).astype(F32)
    i = np.clip(np.searchsorted(xp, x, side="right"), 1, P - 1)
    delta = (x - xp[i - 1]).astype(F32)
    eps = np.spacing(np.finfo(F32).eps)
    d = dx[i - 1]
    dx0 = np.abs(d) <= eps
    with np.errstate(invalid="ignore", divide="ignore"):
        f = np.where(dx0, fp[i - 1], fp[i - 1] + (delta / np.where(dx0, F32(1), d)) * df[i - 1]).astype(F32)
    f = np.where(x < xp[0], fp[0], f)
    f = np.where(x > xp[-1], fp[-1], f)
    return f.astype(F32)


# ------------------------------------------------------------- Frenet frame
def closest_index(x, y, xp, yp, chunk=8192):
    """argmin(sqrt((xp - x)^2 + (yp - y)^2)) per point (first minimum, first
    NaN), fp32 (``C/opt/cem_helper.py:174, 214, 351``)."""
    x = np.asarray(x, F32)
    y = np.asarray(y, F32)
    xf, yf = x.reshape(-1), y.reshape(-1)
    out = np.empty(xf.shape[0], np.int64)
    for a in range(0, xf.shape[0], chunk):
        dx = xp[None, :] - xf[a:a + chunk, None]
        dy = yp[None, :] - yf[a:a + chunk, None]
        d = np.sqrt(dx * dx + dy * dy)
        nan = np.isnan(d)
        idx = np.argmin(np.where(nan, -np.inf, d), axis=1)
        out[a:a + chunk] = idx
    return out.reshape(x.shape)


def frenet_points(x, y, path):
    """``global_to_frenet_trajs`` (C/opt/cem_helper.py:206-242) point-wise:
    (s, d) of global points (any shape)."""
    xp, yp, arc, Fxd, Fyd = (np.asarray(path[k], F32) for k in ("x_path", "y_path", "arc_vec", "Fx_dot", "Fy_dot"))
    idx = closest_index(x, y, xp, yp)
    s = arc[idx]
    Fx = interp(s, arc, Fxd)
    Fy = interp(s, arc, Fyd)
    nx, ny = -Fy, Fx
    nrm = np.sqrt(nx * nx + ny * ny)
    vx = np.asarray(x, F32) - xp[idx]
    vy = np.asarray(y, F32) - yp[idx]
    d = (F32(1) / nrm) * (nx * vx + ny * vy)
    return s.astype(F32), d.astype(F32)


def global_to_frenet(path, x, y, v, vdot, psi, psidot):
    """``Helper.global_to_frenet`` (C/opt/cem_helper.py:348-388) for arrays of
    states.  Returns x, y, vx, vy, ax, ay, psi (Frenet)."""
    x, y, v, vdot, psi, psidot = (np.asarray(a, F32) for a in (x, y, v, vdot, psi, psidot))
    xp, yp, arc = (np.asarray(path[k], F32) for k in ("x_path", "y_path", "arc_vec"))
    kap = np.asarray(path["kappa"], F32)
    idx = closest_index(x, y, xp, yp)
    s = arc[idx]
    k_i = interp(s, arc, kap)
    k_p = interp((s + F32(0.001)).astype(F32), arc, kap)
    k_prime = (k_p - k_i) / F32(0.001)
    Fx = interp(s, arc, path["Fx_dot"])
    Fy = interp(s, arc, path["Fy_dot"])
    nx, ny = -Fy, Fx
    nrm = np.sqrt(nx * nx + ny * ny)
    d = (F32(1) / nrm) * (nx * (x - xp[idx]) + ny * (y - yp[idx]))
    pf = psi - cr(np.arctan2, Fy, Fx)
    pf = cr(np.arctan2, cr(np.sin, pf), cr(np.cos, pf))
    cp, sp = cr(np.cos, pf), cr(np.sin, pf)
    om = F32(1) - d * k_i
    vx = v * cp / om
    vy = v * sp
    pd = psidot - k_i * vx
    ay = vdot * sp + v * cp * pd
    ax1 = vdot * cp - v * sp * pd
    ax2 = -vy * k_i - d * k_prime * vx
    ax = (ax1 * om - (v * cp) * ax2) / (om * om)
    return tuple(a.astype(F32) for a in (s, d, vx, vy, ax, ay, pf))


def global_to_frenet_obs(path, x_obs, y_obs, vx_obs, vy_obs, psi_obs):
    """``Helper.global_to_frenet_obs`` (C/opt/cem_helper.py:171-200): the
    obstacles' Frenet states (x, y, vx, vy, psi)."""
    vx_obs, vy_obs = np.asarray(vx_obs, F32), np.asarray(vy_obs, F32)
    v = np.sqrt(vx_obs * vx_obs + vy_obs * vy_obs)
    s, d, vx, vy, _, _, pf = global_to_frenet(path, x_obs, y_obs, v, np.zeros_like(v), psi_obs, np.zeros_like(v))
    return s, d, vx, vy, pf


def frenet_to_global(y_frenet, ref_x, ref_y, dx_by_ds, dy_by_ds):
    """``Helper.frenet_to_global`` (C/opt/cem_helper.py:154-168)."""
    nx = F32(-1) * np.asarray(dy_by_ds, F32)
    ny = np.asarray(dx_by_ds, F32)
    nrm = np.sqrt(nx * nx + ny * ny)
    gx = np.asarray(ref_x, F32) + np.asarray(y_frenet, F32) * ((F32(1) / nrm) * nx)
    gy = np.asarray(ref_y, F32) + np.asarray(y_frenet, F32) * ((F32(1) / nrm) * ny)
    psi = cr(np.arctan2, np.diff(gy), np.diff(gx))
    return gx.astype(F32), gy.astype(F32), psi


# ------------------------------------------------------- path preprocessing
_SMOOTH_INV = {}


def smoothing_inverse(num_path=600):
    """inv([[20 D3^T D3 + I, e0^T], [e0, 0]]) (C/opt/cem_helper.py:115-129),
    fp64 fixed-order Gauss-Jordan (csrc: the same operation order)."""
    if num_path not in _SMOOTH_INV:
        n = num_path
        D3 = np.diff(np.eye(n), 3, axis=0)
        cost = 20.0 * (D3.T @ D3) + np.eye(n)
        kkt = np.zeros((n + 1, n + 1))
        kkt[:n, :n] = cost
        kkt[n, 0] = kkt[0, n] = 1.0
        _SMOOTH_INV[num_path] = gauss_jordan_vec(kkt)
    return _SMOOTH_INV[num_path]


def gauss_jordan_vec(a):
    """``problem.gauss_jordan_inverse`` with each column's row updates done as
    one array operation (the same per-element operations, so the same bits)."""
    a = np.array(a, dtype=F64)
    n = a.shape[0]
    inv = np.eye(n)
    for c in range(n):
        piv = c + int(np.argmax(np.abs(a[c:, c])))   # first maximal |a| (strict > in the loop form)
        if a[piv, c] == 0.0:
            raise np.linalg.LinAlgError("singular")
        if piv != c:
            a[[c, piv]] = a[[piv, c]]
            inv[[c, piv]] = inv[[piv, c]]
        d = a[c, c]
        a[c] = a[c] / d
        inv[c] = inv[c] / d
        f = a[:, c].copy()
        f[c] = 0.0
        a = a - f[:, None] * a[c][None, :]
        inv = inv - f[:, None] * inv[c][None, :]
    return inv


def _gemv_seq(M, v):
    """M @ v in fp64, sequential over the columns (the library's order)."""
    out = np.zeros(M.shape[0])
    for j in range(M.shape[1]):
        out = out + M[:, j] * v[j]
    return out


def custom_path_smoothing(x_wp, y_wp, threshold, maxiter=10):
    """``Helper.custom_path_smoothing`` (C/opt/cem_helper.py:279-318, 391-410):
    10 ADMM iterations of the jerk-smoothing QP with the waypoints as a
    distance-bounded target.  fp32 state, fp64 KKT products."""
    x_wp = np.asarray(x_wp, F32)
    y_wp = np.asarray(y_wp, F32)
    n = x_wp.shape[0]
    inv = smoothing_inverse(n)
    thr = F32(threshold)
    alpha = np.zeros(n, F32)
    d = np.full(n, thr, F32)
    lx = np.zeros(n, F32)
    ly = np.zeros(n, F32)
    xs, ys = x_wp, y_wp
    for _ in range(maxiter):
        bx = x_wp + d * cr(np.cos, alpha)
        by = y_wp + d * cr(np.sin, alpha)
        lin_x = -lx - bx
        lin_y = -ly - by
        rx = np.concatenate([-lin_x.astype(F64), [F64(x_wp[0])]])
        ry = np.concatenate([-lin_y.astype(F64), [F64(y_wp[0])]])
        xs = f32(_gemv_seq(inv, rx)[:n])
        ys = f32(_gemv_seq(inv, ry)[:n])
        wc = xs - x_wp
        ws = ys - y_wp
        alpha = cr(np.arctan2, ws, wc)
        ca, sa = cr(np.cos, alpha), cr(np.sin, alpha)
        c1 = ca * ca + sa * sa
        c2 = wc * ca + ws * sa
        d = np.minimum(c2 / c1, thr)
        lx = lx - (wc - d * ca)
        ly = ly - (ws - d * sa)
    return xs.astype(F32), ys.astype(F32)


def compute_path_parameters(x_path, y_path):
    """``Helper.compute_path_parameters`` (C/opt/cem_helper.py:321-345).
    Returns Fx_dot, Fy_dot, Fx_ddot, Fy_ddot, arc_vec, kappa, arc_length."""
    x = np.asarray(x_path, F32)
    y = np.asarray(y_path, F32)
    Fxd = np.diff(x)
    Fyd = np.diff(y)
    Fxd = np.concatenate([Fxd[:1], Fxd]).astype(F32)
    Fyd = np.concatenate([Fyd[:1], Fyd]).astype(F32)
    Fxdd = np.diff(Fxd)
    Fydd = np.diff(Fyd)
    Fxdd = np.concatenate([Fxdd[:1], Fxdd]).astype(F32)
    Fydd = np.concatenate([Fydd[:1], Fydd]).astype(F32)
    seg = np.sqrt(Fxd * Fxd + Fyd * Fyd).astype(F32)
    arc = f32(np.cumsum(seg.astype(F64)))
    arc_vec = np.concatenate([[F32(0)], arc[:-1]]).astype(F32)
    s2 = Fxd * Fxd + Fyd * Fyd
    kappa = (Fydd * Fxd - Fxdd * Fyd) / cr(lambda a: np.power(a, 1.5), s2)
    return Fxd, Fyd, Fxdd, Fydd, arc_vec, kappa.astype(F32), arc_vec[-1]


def make_path(x_path, y_path):
    Fxd, Fyd, Fxdd, Fydd, arc, kap, _ = compute_path_parameters(x_path, y_path)
    return dict(x_path=np.asarray(x_path, F32), y_path=np.asarray(y_path, F32), arc_vec=arc, Fx_dot=Fxd,
                Fy_dot=Fyd, kappa=kap)


# ------------------------------------------------------------- the optimizer
def rollout_cr(prob, acc_n, steer_n, st0):
    """compute_rollout_one_step scan (C/opt/cem_helper.py:732-751, 792-803) with
    per-row initial states st0 [..., 5] (broadcast against the rows) and the
    fp64-evaluated transcendentals of the numerics contract."""
    Hh = acc_n.shape[-1]
    t = F32(prob.t)
    wb = F32(prob.wheel_base)
    shp = acc_n.shape[:-1]
    st0 = np.broadcast_to(np.asarray(st0, F32), shp + (5,))
    x, y, vx, vy, psi = (st0[..., k].copy() for k in range(5))
    xr = np.empty(acc_n.shape, F32)
    yr = np.empty(acc_n.shape, F32)
    for h in range(Hh):
        xr[..., h] = x
        yr[..., h] = y
        v = np.sqrt(vx * vx + vy * vy)
        v = v + acc_n[..., h] * t
        psidot = (v * cr(np.tan, steer_n[..., h])) / wb
        psi = psi + psidot * t
        vx = v * cr(np.cos, psi)
        vy = v * cr(np.sin, psi)
        x = x + vx * t
        y = y + vy * t
    return xr, yr


def lane_des_bar(prob, y):
    """The constant costbar of ``compute_lane_des_{mmd,cvar}``
    (C/opt/costs.py:70-100): max(0, ||y - y_des_1||_F ||y - y_des_2||_F - 0.3)
    over the rows x steps of one candidate, broadcast to every row."""
    y = np.asarray(y, F64)
    n1 = np.sqrt(((y - F64(F32(prob.y_des_1))) ** 2).sum(axis=(-2, -1)))
    n2 = np.sqrt(((y - F64(F32(prob.y_des_2))) ** 2).sum(axis=(-2, -1)))
    c = np.maximum(F32(0), f32(f32(n1) * f32(n2)) - F32(prob.gamma_lane_des))
    return np.broadcast_to(c[..., None], y.shape[:-1]).astype(F32)


def compute_cost_carla(prob, cost_obs_w, cost_lane_w, cost_des_w, y, res, xd, yd, xdd, ydd, v_des, steer, kappa):
    """``Helper.compute_cost`` (C/opt/cem_helper.py:522-556) on the 20 elites:
    norms in fp64, the weighted sum in fp64 rounded once (the static
    compute_cost's convention); the risk terms arrive already weighted in fp32
    (C/opt/cem.py:373-375)."""
    def nrm(a):
        a = np.asarray(a, F64)
        return np.sqrt((a * a).sum(axis=-1))
    des = nrm(y - F32(prob.y_des_1)) * nrm(y - F32(prob.y_des_2))
    c_st = nrm(steer)
    sv = np.diff(steer, axis=1)
    c_sv = nrm(sv)
    sa = np.diff(sv, axis=1)
    c_sa = nrm(sa)
    v = np.sqrt(xd * xd + yd * yd)
    c_sp = nrm(np.maximum(F32(0), np.abs(steer) - F32(prob.steer_max)))
    c_svp = nrm(np.maximum(F32(0), np.abs(sv) - F32(0.05)))
    centr = np.abs((xd * xd) * kappa)
    c_centr = nrm(np.maximum(F32(0), centr - F32(prob.a_centr)))
    tot = (np.asarray(res, F64) + 0.1 * nrm(v - F32(v_des)) + 0.1 * (c_st + c_sv + c_sa) + 0.1 * (c_sp + c_svp)
           + 0.02 * nrm(ydd) + 0.02 * nrm(xdd) + 0.01 * des + 0.1 * c_centr) \
        + np.asarray(cost_obs_w, F64) + np.asarray(cost_lane_w, F64) + np.asarray(cost_des_w, F64)
    return f32(tot)


def plan_cost(prob, cost, cx, cy, steer, x_obs, y_obs, path, v_des):
    """The CEM cost of ``Helper.compute_cost`` (C/opt/cem_helper.py:522-556)
    evaluated on a returned plan (cx, cy, steering_best) as a noise-free
    trajectory: the collision / lane / desired-lane bars of the nominal Frenet
    path over the rollout horizon stand in for the risks (weighted as the
    solve weights them, C/opt/cem.py:373-375), the projection residual is 0.
    Test infrastructure: it ranks two solutions of the same problem (the
    sensitivity-ensemble check of tests/test_gpu_carla.py), it is not a step of
    the reference's algorithm."""
    p = prob
    Hh = p.num_prime
    cx = np.asarray(cx, F32)[None]
    cy = np.asarray(cy, F32)[None]
    x = basis_eval(p.P, cx)
    y = basis_eval(p.P, cy)
    xd, yd = basis_eval(p.Pdot, cx), basis_eval(p.Pdot, cy)
    xdd, ydd = basis_eval(p.Pddot, cx), basis_eval(p.Pddot, cy)
    arc = np.asarray(path["arc_vec"], F32)
    kap = interp(np.clip(x, F32(0), arc[-1]), arc, path["kappa"])
    xs, ys = x[:, None, :Hh], y[:, None, :Hh]
    cb = C.compute_f_bar_max(p, xs, ys, np.asarray(x_obs, F32)[:, :Hh], np.asarray(y_obs, F32)[:, :Hh])[:, 0]
    lb, ub = C.lane_bar_max(p, ys)
    des = lane_des_bar(p, ys)[:, 0]
    w_obs, w_lane, w_des = {"mmd_opt": (p.weight_mmd_obs, p.weight_mmd_lane, p.weight_mmd_lane_des)}.get(
        cost, (p.weight_cvar_obs, p.weight_cvar_lane, p.weight_cvar_lane_des))
    tot = compute_cost_carla(p, F32(w_obs) * cb, F32(w_lane) * (lb[:, 0] + ub[:, 0]), F32(w_des) * des, y,
                             np.zeros(1, F32), xd, yd, xdd, ydd, F32(v_des), np.asarray(steer, F32)[None], kap)
    return float(tot[0])


class CarlaDraws:
    """``rng.Draws`` plus the noisy-initial-state normals ``init_eps``
    [R, 4] (``C/opt/cem_helper.py:665``: MVN(0, I_4) = standard normals; R =
    n^2 rows for compute_cem_mmd, n for compute_cem_cvar)."""

    def __init__(self, base, init_eps):
        self.base = base
        self.init_eps = np.ascontiguousarray(init_eps, F32)

    def __getattr__(self, k):
        return getattr(self.__dict__["base"], k)

    @classmethod
    def random(cls, prob, rng, idx_mpc=0, seed=0, with_beta_cem=True):
        base = Draws.random(prob, rng, idx_mpc=idx_mpc, seed=seed, with_beta_cem=with_beta_cem)
        return cls(base, rng.standard_normal((prob.num_reduced ** 2, 4)).astype(F32))

    @classmethod
    def philox(cls, prob, idx_mpc, seed=0, with_beta_cem=True):
        """The library's internal streams (init_eps: stream STREAM_INIT_EPS,
        key (idx_mpc, seed), the reference's PRNGKey(idx_mpc))."""
        base = Draws.philox(prob, idx_mpc, seed, with_beta_cem=with_beta_cem)
        R = prob.num_reduced ** 2
        eps = philox_normals((int(idx_mpc) & 0xFFFFFFFF, int(seed) & 0xFFFFFFFF), STREAM_INIT_EPS, 0, R * 4)
        return cls(base, eps.reshape(R, 4))


class CarlaCEM(CEM):
    """``C/opt/cem.py`` class ``CEM(num_reduced_sqrt, num_mother, num_obs,
    noise_level, num_prime, noise, town, acc_const_noise, steer_const_noise)``
    with ``compute_cem_mmd`` (:217-441) and ``compute_cem_cvar`` (:444-629).
    ``num_mother`` is unused by the reference (Q15: the mother set is
    num_reduced_sqrt^2)."""

    def __init__(self, num_reduced_sqrt, num_mother, num_obs, noise_level, num_prime, noise, town,
                 acc_const_noise, steer_const_noise, num_batch=100, maxiter_cem=20):
        super().__init__(num_reduced_sqrt, num_obs, noise_level, num_prime, noise, acc_const_noise,
                         steer_const_noise, num_batch=num_batch, variant=TOWNS.get(town, "carla_town05"),
                         maxiter_cem=maxiter_cem)
        self.town = town
        self.num_mother_arg = num_mother

    # -- per-solve setup (C/opt/cem.py:248-264, 476-492) -------------------
    def rows(self, cost):
        """Noisy initial states: n^2 (compute_noisy_init_state), n (_baseline)
        or 1 (_det) (C/opt/cem_helper.py:661-715)."""
        p = self.prob
        return {"mmd_opt": p.num_reduced ** 2, "det": 1}.get(cost, p.num_reduced)

    def noisy_init(self, init_state, eps):
        """compute_noisy_init_state(_baseline) (C/opt/cem_helper.py:660-715):
        rows [R, 5] = (x + eps_x, y + eps_y, vx, vy, atan2(vy, vx))."""
        p = self.prob
        x0, y0, v0, _, psi0, _ = (F32(v) for v in init_state)
        vx = v0 * cr(np.cos, psi0)
        vy = v0 * cr(np.sin, psi0)
        eps = np.asarray(eps, F32)
        ex = eps[:, 0] * F32(p.init_sigma[0]) + F32(p.init_mu[0])
        ey = eps[:, 1] * F32(p.init_sigma[1]) + F32(p.init_mu[1])
        R = eps.shape[0]
        st = np.empty((R, 5), F32)
        st[:, 0] = x0 + ex
        st[:, 1] = y0 + ey
        st[:, 2] = vx
        st[:, 3] = vy
        st[:, 4] = cr(np.arctan2, vy, vx)
        return st

    def boundary(self, path, init_state, st):
        """b_eq from the mean Frenet state of the noisy rows (C/opt/cem.py:255-264)."""
        v = np.sqrt(st[:, 2] * st[:, 2] + st[:, 3] * st[:, 3])
        R = st.shape[0]
        fs = global_to_frenet(path, st[:, 0], st[:, 1], v, np.full(R, F32(init_state[3])), st[:, 4],
                              np.full(R, F32(init_state[5])))
        # sequential fp64 sums (the library's order; jnp.mean in the reference)
        m = [f32(np.cumsum(np.asarray(a, F64))[-1] / R) for a in fs[:6]]
        return np.array([m[0], m[2], m[4]], F32), np.array([m[1], m[3], m[5], 0.0], F32)

    def init_carla(self, cost, init_state, mean, cov, path, draws):
        p = self.prob
        B = p.num_batch
        st = dict(pop=H.sampling_param(p, np.asarray(mean, F32), np.asarray(cov, F32), draws.pop0),
                  mean=np.asarray(mean, F32).copy(), cov=np.asarray(cov, F32).copy(),
                  lam_x=np.zeros((B, 11), F32), lam_y=np.zeros((B, 11), F32),
                  s_lane=np.zeros((B, 2 * (p.num - 1)), F32))
        st["rows0"] = self.noisy_init(init_state, draws.init_eps[:self.rows(cost)])
        st["b_eq_x"], st["b_eq_y"] = self.boundary(path, init_state, st["rows0"])
        return st

    # -- per iteration ------------------------------------------------------
    def front_carla(self, st, path, det_obs=None):
        """compute_x_guess + the CARLA projection (C/opt/projection.py:279-336)
        + compute_controls' acc (C/opt/cem.py:307-309).  det_obs = (x_obs,
        y_obs): the det projection instead (C/opt/projection_det.py:279-336,
        obstacle terms live; compute_cem_det, C/opt/cem.py:689-693)."""
        p = self.prob
        cxb, cyb = H.compute_x_guess(p, st["b_eq_x"], st["b_eq_y"], st["pop"])
        from .projection import compute_projection, compute_projection_det
        if det_obs is None:
            pr = compute_projection(p, st["b_eq_x"], st["b_eq_y"], st["lam_x"], st["lam_y"], cxb, cyb, st["s_lane"])
        else:
            pr = compute_projection_det(p, st["b_eq_x"], st["b_eq_y"], st["lam_x"], st["lam_y"], cxb, cyb,
                                        st["s_lane"], det_obs[0], det_obs[1])
        st["lam_x"], st["lam_y"], st["s_lane"] = pr["lam_x"], pr["lam_y"], pr["s_lane"]
        arc = np.asarray(path["arc_vec"], F32)
        xs = np.clip(pr["x"], F32(0), arc[-1])
        kap = interp(xs, arc, path["kappa"])
        # steering (:314-315) from compute_alph_d's polar forms (no unwrap)
        al_v, d_v, ca_v, _ = _polar(pr["xd"], pr["yd"], p.v_min, p.v_max, False)
        al_a, d_a, _, _ = _polar(pr["xdd"], pr["ydd"], 0.0, p.a_max, False)
        curv = (d_a * cr(np.sin, (al_a - al_v).astype(F32))) / (d_v * d_v)
        steer = cr(np.arctan, ((curv + (kap * ca_v) / (F32(1) - pr["y"] * kap)) * F32(p.wheel_base)).astype(F32))
        acc, _ = H.compute_controls(p, pr["xd"], pr["yd"], pr["xdd"], pr["ydd"])
        pr["kappa"] = kap
        return pr, acc, steer.astype(F32)

    def candidate_costs_carla(self, cost, st, acc, steer, x_obs, y_obs, path, draws, t):
        """Risk per candidate (un-permuted): obs [B], lane [B] (lb + ub risk),
        lane_des [B] and for mmd beta / sigma / res_beta / sel."""
        p = self.prob
        n = p.num_reduced
        Hh = p.num_prime
        xo, yo = x_obs[:, :Hh], y_obs[:, :Hh]
        acc_n, steer_n = H.noisy_controls(p, acc[:, :Hh], steer[:, :Hh], draws, t, n)
        B = acc.shape[0]
        extra = {}
        if cost == "mmd_opt":
            acc_m, steer_m = H.mother_controls(acc_n, steer_n)
            xm, ym = rollout_cr(p, acc_m, steer_m, st["rows0"][None, :, :])
            cxm, cym = H.compute_coeff(p, xm, ym)
            # every candidate's beta-CEM, stacked and on a thread pool (the same
            # bits as bc.compute_cem per candidate)
            beta, res_beta, sigma, sel = bc.compute_cem_many(p, cxm, cym, draws.beta_z0, draws.beta_z, threads=4)
            xr = np.take_along_axis(xm, sel[:, :, None], axis=1)
            yr = np.take_along_axis(ym, sel[:, :, None], axis=1)
            sf, df = frenet_points(xr, yr, path)
            cb = C.compute_f_bar_max(p, sf, df, xo, yo)
            obs = C.mmd(p, beta, cb, sigma)
            lane = C.mmd_lane(p, beta, sigma, df)
            des = C.mmd(p, beta, lane_des_bar(p, df), sigma)
            extra = dict(beta=beta, sigma=sigma, res_beta=res_beta, sel=sel, frenet=(sf, df))
        else:
            xr, yr = rollout_cr(p, acc_n, steer_n, st["rows0"][None, :, :])
            sf, df = frenet_points(xr, yr, path)
            cb = C.compute_f_bar_max(p, sf, df, xo, yo)
            obs = C.cvar(p, cb)
            lane = C.cvar_lane(p, df)
            des = C.cvar(p, lane_des_bar(p, df))
            extra = dict(frenet=(sf, df))
        return obs, lane, des, extra

    def weights3(self, cost):
        p = self.prob
        if cost == "mmd_opt":
            return p.weight_mmd_obs, p.weight_mmd_lane, p.weight_mmd_lane_des
        if cost == "det":                     # 0 * the zero risks (C/opt/cem.py:750)
            return 0.0, 0.0, 0.0
        return p.weight_cvar_obs, p.weight_cvar_lane, p.weight_cvar_lane_des

    def select_carla(self, cost, st, t, pr, steer, obs, lane, des, v_des, draws, extra):
        p = self.prob
        perm = H.argsort_stable(pr["res_norm"])                              # C/opt/cem.py:287
        idx_obs = H.argsort_stable(obs[perm])[:p.ellite_num_cost]            # :329
        el = perm[idx_obs]
        w_obs, w_lane, w_des = self.weights3(cost)
        cost20 = compute_cost_carla(p, (F32(w_obs) * obs[el]).astype(F32), (F32(w_lane) * lane[el]).astype(F32),
                                    (F32(w_des) * des[el]).astype(F32), pr["y"][el], pr["res_norm"][el],
                                    pr["xd"][el], pr["yd"][el], pr["xdd"][el], pr["ydd"][el], v_des, steer[el],
                                    pr["kappa"][el])
        idx_cem = H.argsort_stable(cost20)
        pop_el = st["pop"][el[idx_cem[:p.ellite_num]]]
        cost5 = cost20[idx_cem[:p.ellite_num]]
        st["mean"], st["cov"], st["pop"] = H.compute_shifted_samples(
            p, pop_el, cost5, st["mean"], st["cov"], draws.resample[t])
        imin = bc.argmin_nan(cost5)
        e = el[imin]
        out = dict(cx=pr["c_x"][e], cy=pr["c_y"][e], steer=steer[e], lane=lane[e], obs=obs[e])
        if cost == "mmd_opt":
            out.update(beta=extra["beta"][e], sigma=extra["sigma"][e], res_beta=extra["res_beta"][e])
        info = dict(perm=perm, elite_obs=el, cost20=cost20, elite_cem=idx_cem[:p.ellite_num])
        return out, info

    def solve_carla(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, path, draws, trace=None,
                    iters=None, start=None, perturb=None, snapshots=None):
        """compute_cem_mmd / compute_cem_cvar (C/opt/cem.py:217-441, 444-629).
        Returns (cx, cy, v_best [100], steering [100], mean_param [8]).

        Test hooks (none changes the algorithm): ``snapshots`` (a list)
        receives a copy of the carry before every iteration; ``start`` = (t0,
        carry) resumes from such a copy at iteration t0; ``perturb(t, obs, lane,
        des)`` may replace an iteration's risks before the elite selection (the
        sensitivity ensembles of tests/test_gpu_carla.py)."""
        p = self.prob
        x_obs = np.asarray(x_obs, F32)
        y_obs = np.asarray(y_obs, F32)
        if start is None:
            t0, st = 0, self.init_carla(cost, init_state, mean, cov, path, draws)
        else:
            t0, st = start[0], {k: np.array(v, copy=True) for k, v in start[1].items()}
        out = None
        for t in range(t0, p.maxiter_cem if iters is None else iters):
            if snapshots is not None:
                snapshots.append({k: np.array(v, copy=True) for k, v in st.items()})
            pr, acc, steer = self.front_carla(st, path)
            obs, lane, des, extra = self.candidate_costs_carla(cost, st, acc, steer, x_obs, y_obs, path, draws, t)
            if perturb is not None:
                obs, lane, des = perturb(t, obs, lane, des)
            out, info = self.select_carla(cost, st, t, pr, steer, obs, lane, des, F32(v_des), draws, extra)
            if trace is not None:
                trace.append(dict(res_norm=pr["res_norm"], obs=obs, lane=lane, des=des, steer=steer,
                                  kappa=pr["kappa"], acc=acc, pop=st["pop"].copy(), mean=st["mean"].copy(),
                                  **info, **{k: v for k, v in extra.items() if k != "frenet"}))
        xd = basis_eval(p.Pdot, out["cx"][None])[0]
        yd = basis_eval(p.Pdot, out["cy"][None])[0]
        v_best = np.sqrt(xd * xd + yd * yd).astype(F32)
        return out["cx"], out["cy"], v_best, out["steer"].astype(F32), st["mean"].copy(), out

    # -- compute_cem_det (C/opt/cem.py:633-790) --------------------------------
    def select_det(self, st, t, pr, steer, v_des, draws):
        """The det iteration after the projection (C/opt/cem.py:695-772): no
        rollouts; the obstacle "cost" is zeros, so its stable argsort keeps the
        projection order and the elites are its first 20 (:720-722); the cost
        has zero risk terms (:750)."""
        p = self.prob
        B = pr["res_norm"].shape[0]
        z = np.zeros(B, F32)
        return self.select_carla("det", st, t, pr, steer, z, z, z, v_des, draws, {})

    def solve_det(self, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, path, draws, trace=None, iters=None):
        """compute_cem_det: (cx, cy, v_best [100], steering [100], mean_param [8], out)."""
        p = self.prob
        x_obs = np.asarray(x_obs, F32)
        y_obs = np.asarray(y_obs, F32)
        st = self.init_carla("det", init_state, mean, cov, path, draws)
        out = None
        for t in range(p.maxiter_cem if iters is None else iters):
            pr, acc, steer = self.front_carla(st, path, det_obs=(x_obs, y_obs))
            out, info = self.select_det(st, t, pr, steer, F32(v_des), draws)
            if trace is not None:
                trace.append(dict(res_norm=pr["res_norm"], steer=steer, kappa=pr["kappa"], acc=acc,
                                  pop=st["pop"].copy(), mean=st["mean"].copy(), c_x=pr["c_x"], c_y=pr["c_y"],
                                  lam_x=st["lam_x"].copy(), lam_y=st["lam_y"].copy(), **info))
        xd = basis_eval(p.Pdot, out["cx"][None])[0]
        yd = basis_eval(p.Pdot, out["cy"][None])[0]
        v_best = np.sqrt(xd * xd + yd * yd).astype(F32)
        return out["cx"], out["cy"], v_best, out["steer"].astype(F32), st["mean"].copy(), out
