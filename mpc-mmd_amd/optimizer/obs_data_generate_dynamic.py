"""Drop-in for synthetic_dynamic_obs/obs_data_generate_dynamic.py (class
``obs_data``), the dynamic-obstacle scenario generator of the dynamic driver
(synthetic_dynamic_obs/main_mpc.py:9,106-126).

The trajectory QP (``compute_obs_guess``, :73-109) runs in libmpcmmd.so
(``mpcmmd_obs_dynamic_traj``: fp64 KKT inverted once, fp32 output).  The
random draws of the reference are JAX threefry streams (``jax.random.choice``
without replacement, :136-148; ``jax.random.normal``, :111-133), which cannot
be reproduced without JAX: here they come from ``numpy.random.RandomState``
keyed by the same seeds (parity unpinned for the draws; the QP is parity-
tested against the oracle on identical inputs).  The vx pool of the reference
(15 values, drawn without replacement) is extended to >= num_obs values so
num_obs = 20 (BASELINE configs[3]) is defined; for num_obs <= 15 it is the
reference's pool.
"""
from __future__ import annotations

import numpy as np

from . import _native


class obs_data:  # noqa: N801  (reference class name)
    def __init__(self, _num_batch):
        self._num_batch = int(_num_batch)
        self.num = 100
        self.v_mu = 6.0       # :45
        self.v_sigma = 0.1    # :46

    def compute_boundary_vec(self, x_init, vx_init, ax_init, y_init, vy_init, ay_init):
        """:56-71 -> b_eq_x [B,3], b_eq_y [B,4] (last column 0)."""
        B = self._num_batch
        b_eq_x = np.tile(np.array([x_init, vx_init, ax_init], np.float32), (B, 1))
        b_eq_y = np.tile(np.array([y_init, vy_init, ay_init, 0.0], np.float32), (B, 1))
        return b_eq_x, b_eq_y

    def sampling_param(self, seed):
        """:111-133: v_des = 6 + 0.1 N(0,1) per batch row."""
        z = np.random.RandomState(int(seed) & 0xFFFFFFFF).standard_normal(self._num_batch).astype(np.float32)
        return z * np.float32(self.v_sigma) + np.float32(self.v_mu)

    def compute_obs_guess(self, b_eq_x, b_eq_y, y_samples, seed):
        """:73-109 -> x, y [B,100].  The reference's QP has zero initial
        acceleration rows in b_eq (the driver passes ax = ay = 0); non-zero
        accelerations are rejected rather than silently dropped."""
        b_eq_x = np.asarray(b_eq_x, np.float32).reshape(self._num_batch, 3)
        b_eq_y = np.asarray(b_eq_y, np.float32).reshape(self._num_batch, 4)
        if np.any(b_eq_x[:, 2] != 0) or np.any(b_eq_y[:, 2:] != 0):
            raise ValueError("compute_obs_guess: only zero initial acceleration / terminal lateral speed")
        y_des = np.broadcast_to(np.asarray(y_samples, np.float32).reshape(-1), (self._num_batch,))
        if np.any(y_des != y_des[0]):
            raise ValueError("compute_obs_guess: one lane target per call")
        v_des = self.sampling_param(seed)
        return _native.obs_dynamic_traj(b_eq_x[:, 0], b_eq_y[:, 0], b_eq_x[:, 1], b_eq_y[:, 1], v_des,
                                        float(y_des[0]))

    def compute_obs_data(self, num_obs, seed):
        """:136-148 (cut-in scenario: y = 1.75, vy = 0, psi = 0)."""
        return dynamic_obstacle_states(int(num_obs), int(seed))


def dynamic_obstacle_states(num_obs: int, seed: int):
    rs = np.random.RandomState(seed)
    x = rs.choice(np.linspace(15, 45, 30), (num_obs,), replace=False)
    vx = rs.choice(np.linspace(0.5, 5, max(15, num_obs)), (num_obs,), replace=False)
    z = np.zeros(num_obs)
    return x, 1.75 * np.ones(num_obs), vx, z, z.copy()


def dynamic_obstacles(k: int, num_obs: int):
    """One configuration of the dynamic driver (synthetic_dynamic_obs/
    main_mpc.py:108-126): obstacle states, then per obstacle the QP trajectory
    seeded 43k + 11tt + 5 with y target -1.75; then np.random.seed(k) and the
    driver's idx_mpc = randint(1, 10000) (:112, :129)."""
    gen = obs_data(1)
    x, y, vx, vy, psi = gen.compute_obs_data(num_obs, k)
    xt = np.zeros((num_obs, 100), np.float32)
    yt = np.zeros((num_obs, 100), np.float32)
    for tt in range(num_obs):
        bx, by = gen.compute_boundary_vec(x[tt], vx[tt], 0.0, y[tt], vy[tt], 0.0)
        a, b = gen.compute_obs_guess(bx, by, -1.75 * np.ones(1), 43 * k + 11 * tt + 5)
        xt[tt], yt[tt] = a[0], b[0]
    idx_mpc = int(np.random.RandomState(k).randint(1, 10000))
    return dict(x=x, y=y, vx=vx, vy=vy, psi=psi, x_traj=xt, y_traj=yt, idx_mpc=idx_mpc)
