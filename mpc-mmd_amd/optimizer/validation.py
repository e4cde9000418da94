"""Monte-Carlo collision statistics of saved optima on the GPU -- the
reference's outcome metric, synthetic_static_obs/validation.py (and the
synthetic_dynamic_obs copy): ``compute_stats`` (:134-171) replays each saved
(cx, cy) with 1000 noisy rollouts and counts collisions and lane violations;
the script then stores them as ``coll_<cost>`` / ``coll_<cost>_lane``
(:459-464).  Here the per-configuration work runs in libmpcmmd.so
(``mpcmmd_validate``: one workgroup per configuration, fp64 rollouts like
the NumPy original), all configurations of a results file in one launch.

Random draws: the reference seeds ``np.random.seed(key)`` per configuration
and draws with NumPy's multivariate_normal / beta; those streams are not
reproduced (parity is defined on injected draws, ``draws=``); without them
the library's Philox streams keyed by (key, seed) are used.
"""
from __future__ import annotations

import numpy as np

from . import _native

NUM_ROLLOUTS = 1000  # _num_batch (validation.py:173)


def compute_stats(prob, cx, cy, init_state, x_obs, y_obs, vx_obs, vy_obs, num_prime, noise_level, noise, num_obs,
                  key, draws=None, num_rollouts=NUM_ROLLOUTS):
    """Same arguments as the reference's compute_stats (validation.py:134);
    returns (count, count_lane).  ``prob`` is the drop-in ``CEM`` (for the
    obstacle tracks, the const-noise levels and the scenario variant)."""
    c, l = compute_stats_batch(prob, np.atleast_2d(cx), np.atleast_2d(cy), np.atleast_2d(init_state),
                               np.atleast_2d(x_obs), np.atleast_2d(y_obs), np.atleast_2d(vx_obs),
                               np.atleast_2d(vy_obs), num_prime, noise_level, noise, [key],
                               None if draws is None else np.asarray(draws)[None], num_rollouts)
    return int(c[0]), int(l[0])


def compute_stats_batch(prob, cx, cy, init_state, x_obs, y_obs, vx_obs, vy_obs, num_prime, noise_level, noise, keys,
                        draws=None, num_rollouts=NUM_ROLLOUTS):
    """All configurations of a results file (the npz keys of S/main_mpc.py:130-135)
    at once: arrays with a leading configuration axis."""
    K = len(keys)
    xt = np.zeros((K, prob.num_obs, 100), np.float32)
    yt = np.zeros((K, prob.num_obs, 100), np.float32)
    for k in range(K):
        vx = np.asarray(vx_obs[k], np.float64).reshape(-1)
        vy = np.asarray(vy_obs[k], np.float64).reshape(-1)
        xt[k], yt[k], _ = prob.cem_helper.compute_obs_trajectories(
            np.asarray(x_obs[k]).reshape(-1), np.asarray(y_obs[k]).reshape(-1), vx, vy, np.arctan2(vy, vx))
    return _native.validate(cx, cy, init_state, xt, yt, keys, num_prime, noise, noise_level,
                            prob.acc_const_noise, prob.steer_const_noise, num_rollouts, prob.variant, draws,
                            device=prob._cfg.device)
