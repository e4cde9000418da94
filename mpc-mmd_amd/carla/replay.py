"""Replay format for the CARLA optimizer (BASELINE configs[4]) and a synthetic
recording of it.

The reference drives its CARLA optimizer from a live simulator
(``carla/main_carla.py:329-457``) and writes no traces, so a replay format
is defined here.  One file (``.npz``) holds what the optimizer sees each
simulator tick, in the simulator's global frame:

    version        int                        1
    town           str                        "Town05" / "Town10HD" (y_lb, y_ub, y_des)
    num_path       int                        waypoints per tick (reference: 600)
    dt             float                      tick length (reference: 1/20 s, carla_simulation.py:20)
    ego            [T, 6] float32             x, y, v, vdot, psi, psidot  (main_carla.py:352-353)
    waypoints      [T, 2, num_path] float32   x, y: waypoint_generator output (main_carla.py:345)
    obstacles      [T, total_obs, 5] float32  x, y, vx, vy, psi of every spawned vehicle (compute_obs_data)
    route          [2, R] float64             the (extended) route the waypoints follow

``tick_inputs`` turns tick k into the arguments of ``compute_cem_mmd`` /
``compute_cem_cvar`` exactly as main_carla.py:345-382 does: waypoints shifted
to the ego, ``custom_path_smoothing``, ``compute_path_parameters``, the
nearest ``num_obs`` obstacles (``compute_obs_data``, main_carla.py:74-150)
mapped to the Frenet frame and extended to constant-velocity tracks.

``record_synthetic`` makes a recording without CARLA: a Town05-like route
(straight, 90-degree left bend, straight, sampled every 0.25 m like the
route planner, carla_simulation.py:72), extended past its end as
main_carla.py:261-271 does, vehicles spawned at the reference's offsets along
it (carla_simulation.py:53-61, held at zero velocity, :232-238), and an ego
that follows the route at a speed ramp to 10 m/s (v_des, main_carla.py:302),
moving to the free lane around blocking vehicles.  The ego motion is scripted
(no simulator physics), so a recording is deterministic and needs no GPU.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32

# carla_simulation.py:53-61 (distance along the route, lane offset)
SPAWN = {"Town05": (np.array([50, 70, 95, 105, 130, 150, 160, 170, 180, 190], float), (0.0, -3.5)),
         "Town10HD": (np.array([70, 105, 120, 140, 175, 210, 245, 280], float), (0.0, 3.5))}
NUM_PATH = 600


def synthetic_route(spacing=0.25):
    """Town05-like route: 60 m straight, a 90-degree left bend of radius
    40 m, 200 m straight; points every ``spacing`` m (x, y float64)."""
    r = 40.0
    L1, L2 = 60.0, np.pi / 2 * r
    s = np.arange(0.0, L1 + L2 + 200.0, spacing)
    x = np.empty_like(s)
    y = np.empty_like(s)
    a = s <= L1
    x[a], y[a] = s[a], 0.0
    b = (s > L1) & (s <= L1 + L2)
    th = (s[b] - L1) / r
    x[b], y[b] = L1 + r * np.sin(th), r * (1.0 - np.cos(th))
    c = s > L1 + L2
    x[c], y[c] = L1 + r, r + (s[c] - L1 - L2)
    return x, y


def extend_route(x, y, num_p=20000, length=5000.0):
    """main_carla.py:261-271: a straight extension past the route's end so the
    300 m waypoint window never runs out."""
    dx, dy = x[-1] - x[-2], y[-1] - y[-2]
    u = np.hypot(dx, dy)
    t = np.linspace(0.0, length, num_p)[1:]
    return np.concatenate([x, x[-1] + dx / u * t]), np.concatenate([y, y[-1] + dy / u * t])


class Route:
    """Arc-length parametrised route with headings and left normals."""

    def __init__(self, x, y):
        self.x, self.y = np.asarray(x, float), np.asarray(y, float)
        seg = np.hypot(np.diff(self.x), np.diff(self.y))
        self.s = np.concatenate([[0.0], np.cumsum(seg)])
        self.psi = np.unwrap(np.arctan2(np.gradient(self.y), np.gradient(self.x)))

    def at(self, s, d=0.0):
        x = np.interp(s, self.s, self.x)
        y = np.interp(s, self.s, self.y)
        psi = np.interp(s, self.s, self.psi)
        return x - d * np.sin(psi), y + d * np.cos(psi), psi


def _lane_offset(s, obs_s, obs_d, lane_free):
    """Scripted lateral offset of the ego: move to the free lane 25 m before
    a vehicle in its lane, come back 10 m after it (15 m cosine ramps)."""
    d = np.zeros_like(s)
    for so, do in zip(obs_s, obs_d):
        if do != 0.0:
            continue
        a0, a1, b0, b1 = so - 40.0, so - 25.0, so + 10.0, so + 25.0
        w = np.clip((s - a0) / (a1 - a0), 0, 1) * np.clip((b1 - s) / (b1 - b0), 0, 1)
        d = np.minimum(d, lane_free * 0.5 * (1 - np.cos(np.pi * w))) if lane_free < 0 else \
            np.maximum(d, lane_free * 0.5 * (1 - np.cos(np.pi * w)))
    return d


def record_synthetic(ticks=200, town="Town05", dt=0.05, v_des=10.0, num_path=NUM_PATH):
    """A deterministic recording (see the module docstring)."""
    from scipy.interpolate import CubicSpline
    offs, lanes = SPAWN["Town10HD" if town.startswith("Town10") else "Town05"]
    rx, ry = synthetic_route()
    rt = Route(rx, ry)
    obs_s = offs.copy()
    obs_d = np.array([lanes[i % 2] for i in range(offs.size)])
    ox, oy, opsi = rt.at(obs_s, obs_d)
    obstacles = np.zeros((offs.size, 5), F32)
    obstacles[:, 0], obstacles[:, 1], obstacles[:, 4] = ox, oy, np.arctan2(np.sin(opsi), np.cos(opsi))
    ex, ey = extend_route(rx, ry)
    # waypoints: splines over the extended route's arc length (path_spline / waypoint_generator)
    seg = np.hypot(np.diff(ex), np.diff(ey))
    es = np.concatenate([[0.0], np.cumsum(seg)])
    csx, csy = CubicSpline(es, ex), CubicSpline(es, ey)
    # ego: speed ramp to v_des, scripted lane changes
    t = np.arange(ticks) * dt
    v = np.minimum(v_des, 0.1 + 2.0 * t)
    s = np.concatenate([[0.0], np.cumsum(0.5 * (v[1:] + v[:-1]) * dt)])
    d = _lane_offset(s, obs_s, obs_d, lanes[1])
    x, y, psi = rt.at(s, d)
    dd = np.gradient(d, s + 1e-9 * np.arange(ticks)) if ticks > 1 else np.zeros(1)
    psi = psi + np.arctan(dd)
    psi = np.arctan2(np.sin(psi), np.cos(psi))
    vdot = np.zeros_like(v)  # main_carla.py:296: vdot_global_init = 0.0 is never updated in the loop
    psidot = np.gradient(np.unwrap(psi), dt) if ticks > 1 else np.zeros(1)
    ego = np.stack([x, y, v, vdot, psi, psidot], axis=1).astype(F32)
    wps = np.empty((ticks, 2, num_path), F32)
    for k in range(ticks):
        i = int(np.argmin(np.hypot(ex - x[k], ey - y[k])))
        look = np.linspace(es[i], es[i] + 300.0, num_path)
        wps[k, 0], wps[k, 1] = csx(look), csy(look)
    return dict(version=np.int32(1), town=np.array(town), num_path=np.int32(num_path), dt=np.float32(dt), ego=ego,
                waypoints=wps, obstacles=np.repeat(obstacles[None], ticks, axis=0), route=np.stack([ex, ey]))


def save(path, rec):
    np.savez_compressed(path, **rec)


def load(path):
    with np.load(path, allow_pickle=False) as z:
        rec = {k: z[k] for k in z.files}
    if int(rec["version"]) != 1:
        raise ValueError(f"replay version {int(rec['version'])} (expected 1)")
    rec["town"] = str(rec["town"])
    return rec


def nearest_obstacles(obs, ego, num_obs):
    """compute_obs_data (main_carla.py:74-150): vehicles not behind the ego
    (angle to the heading <= 150 degrees, :87-90), padded by repeating the last
    (or 300 m away when none, :113-134), the num_obs nearest (:137-147)."""
    x0, y0, v0, _, psi0, _ = (float(u) for u in ego)
    rel = obs[:, :2].astype(np.float64) - np.array([x0, y0])
    h = v0 * np.array([np.cos(psi0), np.sin(psi0)])
    theta = np.arccos(np.clip(rel @ h, -1.0, 1.0))
    keep = obs[theta <= 5 * np.pi / 6]
    if keep.shape[0] == 0:
        keep = np.zeros((num_obs, 5), F32)
        keep[:, 0] = keep[:, 1] = 300.0
    while keep.shape[0] < num_obs:
        keep = np.vstack([keep, keep[-1:]])
    dist = (x0 - keep[:, 0].astype(np.float64)) ** 2 + (y0 - keep[:, 1].astype(np.float64)) ** 2
    return keep[np.argsort(dist, kind="stable")[:num_obs]].astype(F32)


def tick_inputs(rec, k, helper, num_obs, threshold=0.1):
    """Arguments of compute_cem_* for tick k (main_carla.py:345-382) through
    ``helper`` (``prob.cem_helper`` of the drop-in, the library's helpers):
    (init_state_global, x_obs_traj, y_obs_traj, path dict)."""
    ego = rec["ego"][k]
    x0, y0 = float(ego[0]), float(ego[1])
    h = helper
    xw = (rec["waypoints"][k, 0].astype(np.float64) - x0).astype(F32)
    yw = (rec["waypoints"][k, 1].astype(np.float64) - y0).astype(F32)
    x_path, y_path = h.custom_path_smoothing(xw, yw, threshold)
    Fxd, Fyd, _, _, arc, kap, _ = h.compute_path_parameters(x_path, y_path)
    ob = nearest_obstacles(rec["obstacles"][k], ego, num_obs)
    xs = (ob[:, 0].astype(np.float64) - x0).astype(F32)
    ys = (ob[:, 1].astype(np.float64) - y0).astype(F32)
    xi, yi, vxi, vyi, pi = h.global_to_frenet_obs_vmap(xs, ys, ob[:, 2], ob[:, 3], ob[:, 4], x_path, y_path, arc,
                                                       Fxd, Fyd, kap)
    xo, yo, _ = h.compute_obs_trajectories(xi, yi, vxi, vyi, pi)
    init = np.array([0.0, 0.0, ego[2], ego[3], ego[4], ego[5]], F32)   # x_global_shifted = y_global_shifted = 0
    path = dict(x_path=x_path, y_path=y_path, arc_vec=arc, Fx_dot=Fxd, Fy_dot=Fyd, kappa=kap)
    return init, xo, yo, path
