"""Drop-in replacement of the reference's ``carla/optimizer/cem.py`` (class
CEM of the CARLA experiments).  ``carla/main_carla.py`` does::

    sys.path.insert(1, 'path/to/optimizer'); from optimizer import cem
    prob = cem.CEM(num_reduced, 1, num_obs, noise_level, num_prime, noise, town,
                   acc_const_noise, steer_const_noise)                # main_carla.py:186-187
    cx, cy, v, steering, mean_param = prob.compute_cem_mmd(
        i, init_state_global, mean_param, cov_param, x_obs_traj, y_obs_traj, v_des,
        x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa)              # :378-382

With ``mpc-mmd_amd/carla`` on sys.path the same calls run on the MI355X
through libmpcmmd.so (mpcmmd_carla_begin / iterate / finish; no JAX).
``compute_cem_mmd``, ``compute_cem_cvar`` and ``compute_cem_det`` (the
deterministic baseline with the obstacle-constrained projection of
projection_det.py) are built, so every ``--costs`` of main_carla.py:188-194
runs.  Extra keyword-only options:
``num_batch`` (reference: 100, cem.py:138), ``maxiter_cem``, ``device``,
``seed``; per call ``draws`` (explicit standard normals incl. ``init_eps``,
include/mpcmmd.h) and ``trace``.
"""
from __future__ import annotations

import os

import numpy as np

from ._lib import native
from .cem_helper import Helper

# cem.py:161-166 tests town == "Town10HD" only: every other name, Town10HD_Opt
# included, gets the Town05 lane bounds and desired lanes
_TOWN = {"Town10HD": "carla_town10hd"}


class CEM:
    def __init__(self, num_reduced_sqrt, num_mother, num_obs, noise_level, num_prime, noise, town,
                 acc_const_noise, steer_const_noise, *, num_batch=100, maxiter_cem=20, device=None, seed=0):
        N = native()
        if noise not in N.NOISE:
            raise ValueError("noise must be 'gaussian' or 'beta'")
        self.town = town
        self.noise = noise
        self.acc_const_noise = acc_const_noise
        self.steer_const_noise = steer_const_noise
        # scalars the driver reads (cem.py:25-182)
        self.beta_a, self.beta_b = 2, 5
        self.a_obs, self.b_obs = 4.5, 3
        self.wheel_base = 2.875
        self.kappa_max, self.a_centr = 0.230, 1.5
        self.v_max, self.v_min, self.a_max = 30.0, 0.1, 18.0
        self.num_obs = int(num_obs)
        self.steer_max = 0.6
        self.steer_rate_max = 0.6
        self.t_fin, self.num = 15, 100
        self.num_prime = int(num_prime)
        self.t = self.t_fin / self.num
        self.tot_time = np.linspace(0, self.t_fin, self.num)
        self.maxiter, self.maxiter_cem = 1, int(maxiter_cem)
        self.num_params = 8
        self.num_batch = int(num_batch)
        self.ellite_num, self.ellite_num_projection, self.ellite_num_cost = 5, self.num_batch, 20
        self.num_mother = num_mother                      # unused by the reference
        self.num_reduced_sqrt = int(num_reduced_sqrt)
        self.num_reduced = self.num_reduced_sqrt ** 2
        self.variant = _TOWN.get(town, "carla_town05")
        if self.variant == "carla_town10hd":
            self.y_lb, self.y_ub, self.y_des_1, self.y_des_2 = -0.3, 3.8, 0.0, 3.5
        else:
            self.y_lb, self.y_ub, self.y_des_1, self.y_des_2 = -3.8, 0.3, 0.0, -3.5
        self.alpha_quant = self.alpha_quant_lane = 0.98
        self.weight_mmd_lane_des, self.weight_mmd_lane, self.weight_mmd_obs = 0.0, 0.01, 0.1
        self.weight_cvar_lane_des, self.weight_cvar_lane, self.weight_cvar_obs = 0.0, 25, 100
        self.sigma_ker, self.ker_wt = 1e-2, 1000
        self.sigma_acc = self.sigma_steer = noise_level
        self.gamma_lane_des = 0.3
        dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else device
        self._cfg = N.make_config(num_reduced_sqrt, num_obs, noise_level, num_prime, noise, acc_const_noise,
                                  steer_const_noise, num_batch, self.variant, maxiter_cem, dev, seed)
        sh = (self.num, 11)
        self.P = N.host_constant(self._cfg, "P64").reshape(sh)
        self.Pdot = N.host_constant(self._cfg, "Pdot64").reshape(sh)
        self.Pddot = N.host_constant(self._cfg, "Pddot64").reshape(sh)
        self.P_jax, self.Pdot_jax, self.Pddot_jax = (a.astype(np.float32) for a in (self.P, self.Pdot, self.Pddot))
        self.nvar = 11
        self.cem_helper = Helper(self)
        self._h = N.Handle(self._cfg)

    def _solve(self, cost, idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj, y_obs_traj,
               v_des, x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa, draws=None, trace=False):
        path = dict(x_path=x_path, y_path=y_path, arc_vec=arc_vec, Fx_dot=Fx_dot, Fy_dot=Fy_dot, kappa=kappa)
        r = self._h.carla_solve(cost, idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj,
                                y_obs_traj, v_des, path, draws, trace)
        self.last_result = r
        return r["cx"], r["cy"], r["v_best"].copy(), r["steering"].copy(), r["mean_param"]

    def compute_cem_mmd(self, idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj, y_obs_traj,
                        v_des, x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa, **kw):
        """cem.py:217-441 -> (cx_best, cy_best, v_best, steering_best, mean_param)."""
        return self._solve("mmd_opt", idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj,
                           y_obs_traj, v_des, x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa, **kw)

    def compute_cem_cvar(self, idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj, y_obs_traj,
                         v_des, x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa, **kw):
        """cem.py:444-629 -> (cx_best, cy_best, v_best, steering_best, mean_param)."""
        return self._solve("cvar", idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj,
                           y_obs_traj, v_des, x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa, **kw)

    def compute_cem_det(self, idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj, y_obs_traj,
                        v_des, x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa, **kw):
        """cem.py:633-790, the deterministic baseline: one noisy initial state
        (cem_helper.py:680-696), the projection with its obstacle terms live
        (projection_det.py), no rollouts and no risk terms ->
        (cx_best, cy_best, v_best, steering_best, mean_param)."""
        return self._solve("det", idx_mpc, init_state_global, mean_param_init, cov_param_init, x_obs_traj,
                           y_obs_traj, v_des, x_path, y_path, arc_vec, Fx_dot, Fy_dot, kappa, **kw)

    @property
    def handle(self):
        return self._h
