"""``carla/optimizer/cem_helper.py`` (class Helper): the per-tick path and
frame helpers ``carla/main_carla.py`` calls through ``prob.cem_helper``
(``:275, 286, 345, 364-376, 387-392``).

* ``path_spline`` / ``waypoint_generator`` (cem_helper.py:244-276) are NumPy /
  SciPy in the reference too (cubic splines of the route by arc length);
  pinned bit for bit to the reference's own functions executed on fixed
  routes (tests/golden/make_carla_path_golden.py).
* ``custom_path_smoothing``, ``compute_path_parameters``, the Frenet
  transforms run in libmpcmmd.so (host C++, the same operations as its
  kernels; include/mpcmmd.h).
* ``jax_interp`` / ``frenet_to_global`` / ``compute_obs_trajectories`` are the
  small post-processing of one trajectory (100 points), fp32 NumPy in the
  jitted reference's operation order.
"""
from __future__ import annotations

import numpy as np

from ._lib import native

F32 = np.float32


def _path(x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa):
    return dict(x_path=x_path, y_path=y_path, arc_vec=arc_vec, Fx_dot=Fx_dot, Fy_dot=Fy_dot, kappa=kappa)


def interp(x, xp, fp):
    """``jnp.interp`` (jax 0.3.23): fp[i-1] + ((x - xp[i-1]) / dx) * df with
    i = clip(searchsorted(xp, x, 'right'), 1, P-1); fp[0] / fp[-1] outside."""
    x = np.asarray(x, F32)
    xp = np.asarray(xp, F32)
    fp = np.asarray(fp, F32)
    P = xp.shape[0]
    i = np.clip(np.searchsorted(xp, x, side="right"), 1, P - 1)
    dx = (xp[i] - xp[i - 1]).astype(F32)
    df = (fp[i] - fp[i - 1]).astype(F32)
    dlt = (x - xp[i - 1]).astype(F32)
    small = np.abs(dx) <= np.spacing(np.finfo(F32).eps)
    with np.errstate(invalid="ignore", divide="ignore"):
        f = np.where(small, fp[i - 1], fp[i - 1] + (dlt / np.where(small, F32(1), dx)) * df).astype(F32)
    return np.where(x < xp[0], fp[0], np.where(x > xp[-1], fp[-1], f)).astype(F32)


class Helper:
    def __init__(self, cem=None, num_prime=30):
        self._cem = cem
        self.num_path = 600
        self.num = 100
        self.num_prime = cem.num_prime if cem is not None else num_prime
        self.t = 15 / 100
        self.tot_time = np.linspace(0, 15, self.num)
        self.maxiter_smoothing = 10

    # -- route (NumPy / SciPy in the reference as well) -----------------------
    def path_spline(self, x_path, y_path):
        """Cubic splines of x, y and the unwrapped heading over a uniform
        arc-length grid of the route (cem_helper.py:244-262)."""
        from scipy.interpolate import CubicSpline
        x_path = np.asarray(x_path, np.float64)
        y_path = np.asarray(y_path, np.float64)
        dx, dy = np.diff(x_path), np.diff(y_path)
        heading = np.unwrap(np.arctan2(dy, dx))
        heading = np.concatenate([heading[:1], heading])
        arc_length = np.cumsum(np.sqrt(dx ** 2 + dy ** 2))[-1]   # the reference's formula (not hypot: last-bit)
        arc_vec = np.linspace(0.0, arc_length, x_path.shape[0])
        return (CubicSpline(arc_vec, x_path), CubicSpline(arc_vec, y_path), CubicSpline(arc_vec, heading),
                arc_length, arc_vec)

    def waypoint_generator(self, x_global_init, y_global_init, x_path_data, y_path_data, arc_vec, cs_x_path,
                           cs_y_path, cs_phi_path, arc_length):
        """num_path waypoints over the 300 m ahead of the route point closest
        to the ego (cem_helper.py:264-276)."""
        d = np.sqrt((x_global_init - np.asarray(x_path_data)) ** 2 + (y_global_init - np.asarray(y_path_data)) ** 2)
        s0 = arc_vec[int(np.argmin(d))]
        look = np.linspace(s0, s0 + 300.0, self.num_path)
        return cs_x_path(look), cs_y_path(look), cs_phi_path(look)

    # -- libmpcmmd ------------------------------------------------------------
    def custom_path_smoothing(self, x_waypoints, y_waypoints, threshold):
        """cem_helper.py:391-410 (mpcmmd_path_smoothing)."""
        return native().path_smoothing(x_waypoints, y_waypoints, threshold)

    def compute_path_parameters(self, x_path, y_path):
        """cem_helper.py:321-345 -> Fx_dot, Fy_dot, Fx_ddot, Fy_ddot, arc_vec, kappa, arc_length."""
        return native().path_parameters(x_path, y_path)

    def global_to_frenet(self, x_path, y_path, initial_state, arc_vec, Fx_dot, Fy_dot, kappa):
        """cem_helper.py:348-388 for one state (x, y, v, vdot, psi, psidot):
        x, y, vx, vy, ax, ay, psi, psi_fin (0), psidot."""
        x, y, v, vdot, psi, psidot = (np.float32(u) for u in initial_state)
        out = native().global_to_frenet(_path(x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa), x, y, v, vdot,
                                        psi, psidot)
        xi, yi, vx, vy, ax, ay, pf = (o[0] for o in out)
        ki = interp(xi, arc_vec, kappa)
        return xi, yi, vx, vy, ax, ay, pf, np.float32(0.0), np.float32(psidot - ki * vx)

    def global_to_frenet_obs_vmap(self, x_obs, y_obs, vx_obs, vy_obs, psi_obs, x_path, y_path, arc_vec, Fx_dot,
                                  Fy_dot, kappa):
        """cem_helper.py:171-200, vmapped over the obstacles: x, y, vx, vy, psi."""
        vx_obs = np.asarray(vx_obs, F32)
        vy_obs = np.asarray(vy_obs, F32)
        v = np.sqrt(vx_obs * vx_obs + vy_obs * vy_obs)
        z = np.zeros_like(v)
        xi, yi, vx, vy, _, _, pf = native().global_to_frenet(_path(x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa),
                                                             x_obs, y_obs, v, z, psi_obs, z)
        return xi, yi, vx, vy, pf

    # -- post-processing of one trajectory -------------------------------------
    def jax_interp(self, x, xp, fp):
        return interp(x, xp, fp)

    def interp_vmap(self, x, xp, fp):
        return interp(x, xp, fp)

    def frenet_to_global(self, y_frenet, ref_x, ref_y, dx_by_ds, dy_by_ds):
        """cem_helper.py:154-168: points at offset y_frenet along the unit
        normal (-dy/ds, dx/ds); heading of the resulting polyline."""
        nx = -np.asarray(dy_by_ds, F32)
        ny = np.asarray(dx_by_ds, F32)
        inv = F32(1) / np.sqrt(nx * nx + ny * ny)
        yf = np.asarray(y_frenet, F32)
        gx = (np.asarray(ref_x, F32) + yf * (inv * nx)).astype(F32)
        gy = (np.asarray(ref_y, F32) + yf * (inv * ny)).astype(F32)
        psi = np.arctan2(np.diff(gy).astype(np.float64), np.diff(gx).astype(np.float64)).astype(F32)
        return gx, gy, psi

    def compute_obs_trajectories(self, x_obs, y_obs, vx_obs, vy_obs, psi_obs):
        """cem_helper.py:717-729: constant-velocity tracks on the 100-point grid."""
        tt = self.tot_time.astype(F32)[:, None]
        x = (np.asarray(x_obs, F32) + np.asarray(vx_obs, F32) * tt).T
        y = (np.asarray(y_obs, F32) + np.asarray(vy_obs, F32) * tt).T
        psi = np.tile(np.asarray(psi_obs, F32), (self.num, 1)).T
        return np.ascontiguousarray(x, F32), np.ascontiguousarray(y, F32), np.ascontiguousarray(psi, F32)
