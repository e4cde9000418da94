"""Drop-in replacement of ``synthetic_static_obs/optimizer/cem.py`` (class CEM).

The reference drivers do::

    sys.path.insert(1, 'path/to/optimizer'); from optimizer import cem
    prob = cem.CEM(num_reduced, num_obs, noise_level, num_prime, noise,
                   acc_const_noise, steer_const_noise)            # cem.py:17-18
    prob.compute_cem_mmd_opt(idx_mpc, init_state, mean_param, cov_param,
                             x_obs_traj, y_obs_traj, v_des)          # cem.py:201-204

With ``path/to/optimizer`` pointing at ``mpc-mmd_amd`` the same code runs on
the MI355X through libmpcmmd.so (no JAX).  Constructor and methods keep the
reference's names, argument meaning and return tuples; extra keyword-only
options: ``num_batch`` (reference hard-codes 100, cem.py:137), ``variant``
("static" / "dynamic": the two constants that differ in
synthetic_dynamic_obs), ``maxiter_cem``, ``device``, ``seed``; per call
``draws`` (explicit standard normals, see include/mpcmmd.h) and ``trace``.
"""
from __future__ import annotations

import os

import numpy as np

from . import _native
from .cem_helper import Helper


def _default_device():
    return int(os.environ.get("LOCAL_RANK", "0"))


class CEM:
    def __init__(self, num_reduced, num_obs, noise_level, num_prime, noise, acc_const_noise,
                 steer_const_noise, *, num_batch=100, variant="static", maxiter_cem=20, device=None,
                 seed=0):
        if noise not in _native.NOISE:
            raise ValueError("noise must be 'gaussian' or 'beta'")
        self.noise = noise
        self.acc_const_noise = acc_const_noise
        self.steer_const_noise = steer_const_noise
        # scalar attributes read by the drivers / validation (cem.py:24-171)
        self.beta_a, self.beta_b = 2, 5
        self.a_obs, self.b_obs = 4.25, 2.75
        self.wheel_base = 2.5
        self.v_max, self.v_min, self.a_max = 30.0, 0.1, 18.0
        self.num_obs = int(num_obs)
        self.steer_max = 0.6
        self.t_fin, self.num = 15, 100
        self.t = self.t_fin / self.num
        self.tot_time = np.linspace(0, self.t_fin, self.num)
        self.num_prime = int(num_prime)
        self.maxiter = 1
        self.maxiter_cem = int(maxiter_cem)
        self.num_params = 8
        self.num_batch = int(num_batch)
        self.ellite_num = 5
        self.ellite_num_projection = self.num_batch
        self.ellite_num_cost = 20
        self.num_reduced = int(num_reduced)
        self.num_mother = self.num_reduced ** 2
        self.variant = variant
        self.y_lb, self.y_ub = (-2.25, 2.25) if variant == "static" else (-2.25, -1.25)
        self.y_des_1, self.y_des_2 = -1.75, 1.75
        self.alpha_quant = self.alpha_quant_lane = 0.98
        self.weight_mmd_lane, self.weight_mmd_obs = 0.0, 1e3
        self.weight_cvar_lane, self.weight_cvar_obs = 0.0, 1e3
        self.weight_saa_lane, self.weight_saa_obs = 1e6, 1e6
        self.ker_wt = 1000.0
        self.sigma_acc = self.sigma_steer = noise_level
        self._cfg = _native.make_config(num_reduced, num_obs, noise_level, num_prime, noise,
                                        acc_const_noise, steer_const_noise, num_batch, variant,
                                        maxiter_cem, _default_device() if device is None else device, seed)
        # bases: fp64 self.P (the reference's NumPy arrays) and fp32 *_jax (cem.py:46-48)
        sh = (self.num, 11)
        self.P = _native.host_constant(self._cfg, "P64").reshape(sh)
        self.Pdot = _native.host_constant(self._cfg, "Pdot64").reshape(sh)
        self.Pddot = _native.host_constant(self._cfg, "Pddot64").reshape(sh)
        self.P_jax = self.P.astype(np.float32)
        self.Pdot_jax = self.Pdot.astype(np.float32)
        self.Pddot_jax = self.Pddot.astype(np.float32)
        self.nvar = 11
        self.cem_helper = Helper(self)
        self._h = _native.Handle(self._cfg)

    # ------------------------------------------------------------------
    def _solve(self, cost, idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj, y_obs_traj,
               v_des, draws=None, trace=False):
        r = self._h.solve(cost, idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                          y_obs_traj, v_des, draws, trace)
        self.last_trace = r if trace else None
        if cost == "mmd_opt":
            return (r["cx"], r["cy"], r["cost_lane"], r["cost_obs"], r["beta"][:self.num_reduced].copy(),
                    r["sigma"], r["res_beta"])
        return r["cx"], r["cy"], r["cost_lane"], r["cost_obs"]

    def compute_cem_mmd_opt(self, idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                            y_obs_traj, v_des, **kw):
        """cem.py:201-333 -> (cx_best, cy_best, mmd_lane, mmd_obs, beta, sigma, res_beta)."""
        return self._solve("mmd_opt", idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                           y_obs_traj, v_des, **kw)

    def compute_cem_mmd_random(self, idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                               y_obs_traj, v_des, **kw):
        """cem.py:335-462 -> (cx_best, cy_best, mmd_lane, mmd_obs)."""
        return self._solve("mmd_random", idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                           y_obs_traj, v_des, **kw)

    def compute_cem_cvar(self, idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                         y_obs_traj, v_des, **kw):
        """cem.py:464-588 -> (cx_best, cy_best, cvar_lane, cvar_obs)."""
        return self._solve("cvar", idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                           y_obs_traj, v_des, **kw)

    def compute_cem_saa(self, idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                        y_obs_traj, v_des, **kw):
        """cem.py:590-714 -> (cx_best, cy_best, saa_lane, saa_obs)."""
        return self._solve("saa", idx_mpc, init_state, mean_param_init, cov_param_init, x_obs_traj,
                           y_obs_traj, v_des, **kw)

    @property
    def handle(self):
        """The underlying native handle (stage access, streams, profiling)."""
        return self._h
