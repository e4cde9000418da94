"""The host-side pieces of ``optimizer/cem_helper.py`` (class Helper) that the
reference drivers call directly: ``compute_obs_trajectories``
(cem_helper.py:366-378, used at S/main_mpc.py:109) and ``K_steer``
(cem_helper.py:24, read by S/validation.py).  Everything on the hot path runs
inside libmpcmmd.so.
"""
from __future__ import annotations

import numpy as np


class Helper:
    def __init__(self, cem):
        self._cem = cem
        self.K_steer = 0.01 if cem.variant == "static" else 0.05
        self.num_prime = cem.num_prime
        self.num = cem.num
        self.tot_time = cem.tot_time
        self.t = cem.t

    def compute_obs_trajectories(self, x_obs, y_obs, vx_obs, vy_obs, psi_obs):
        """Constant-velocity obstacle tracks on the 100-point grid, fp32 like
        the jitted reference: returns x, y, psi, each [num_obs, 100]."""
        tt = self.tot_time.astype(np.float32)[:, None]
        x = (np.asarray(x_obs, np.float32) + np.asarray(vx_obs, np.float32) * tt).T
        y = (np.asarray(y_obs, np.float32) + np.asarray(vy_obs, np.float32) * tt).T
        psi = np.tile(np.asarray(psi_obs, np.float32), (self.num, 1)).T
        return (np.ascontiguousarray(x, np.float32), np.ascontiguousarray(y, np.float32),
                np.ascontiguousarray(psi, np.float32))
