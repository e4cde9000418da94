"""Monte-Carlo collision statistics of saved optima on the GPU -- the
reference's outcome metric, ``synthetic_static_obs/validation.py`` and its
``synthetic_dynamic_obs`` copy.

``compute_stats`` (S/validation.py:134-171) replays one saved (cx, cy) with
1000 noisy rollouts and counts collisions and lane violations; the static
variant rebuilds the obstacle tracks from (x, y, vx, vy) with
``compute_obs_trajectories``, the dynamic one takes the saved QP tracks
``x_obs_traj`` / ``y_obs_traj`` as they are (D/validation.py:129-165).  Here
every configuration of a results file runs in ONE ``mpcmmd_validate``
launch (one workgroup per configuration, fp64 rollouts like the NumPy
original).

``python -m optimizer.validation`` is the script itself (S/validation.py:202-464):
for each sweep point it loads the ``data/`` npz files of mmd_opt and cvar
(and mmd_random for the static variant, as the reference does), intersects
the configurations the two costs solved (the reference's set intersection,
:284-302), validates them with key = position in that intersection, and
writes ``stats/<noise>_noise/noise_<100 sigma>/ts_<H>/<n>_samples_<O>_obs.npz``
with the ``coll_*`` keys (:459-464).

Random draws: the reference seeds ``np.random.seed(key)`` per configuration
and draws with NumPy's multivariate_normal / beta (S/validation.py:42-84).
By default (``rng="numpy"``) the same NumPy draws are made here on the host
(``reference_draws``: a ``RandomState(key)`` gives the stream of the seeded
global generator) and handed to the GPU, so the counts are the reference's
own (tests/golden pins them).  ``rng="philox"`` (``--rng philox``) uses the
library's counter-based Philox streams keyed by (key, seed) instead: no host
work, other numbers.
"""
from __future__ import annotations

import argparse
import os

import numpy as np

from . import _native

NUM_ROLLOUTS = 1000  # _num_batch (validation.py:173)
RNGS = ("numpy", "philox")


def _controls(prob, cx, cy):
    """compute_controls of a saved optimum, fp64 on the fp32 basis
    (S/validation.py:122-132, 140-146): acc [101], steer [100]."""
    cx = np.asarray(cx, np.float64).reshape(-1)
    cy = np.asarray(cy, np.float64).reshape(-1)
    xd, xdd = np.dot(prob.Pdot_jax, cx), np.dot(prob.Pddot_jax, cx)
    yd, ydd = np.dot(prob.Pdot_jax, cy), np.dot(prob.Pddot_jax, cy)
    v = np.sqrt(xd ** 2 + yd ** 2)
    v = np.hstack((v, v[-1]))
    acc = np.diff(v) / prob.t
    acc = np.hstack((acc, acc[-1]))
    curv = (ydd * xd - yd * xdd) / ((xd ** 2 + yd ** 2) ** 1.5)
    return acc, np.arctan(curv * prob.wheel_base)


def reference_draws(prob, cx, cy, num_prime, noise, key, num_rollouts=NUM_ROLLOUTS):
    """The draws of compute_rollout_complete (S/validation.py:42-84) for one
    saved optimum: np.random.seed(key), then acc / steer noise (gaussian:
    multivariate_normal; beta: Beta(2|acc|, 5|acc|) and Beta(2|steer| + 1e-5,
    5|steer| + 1e-5) of the optimum's controls), then the const-noise
    normals.  Returns [3][R][H] fp64 as mpcmmd_validate takes them."""
    H, R = int(num_prime), int(num_rollouts)
    acc, steer = _controls(prob, cx, cy)
    acc, steer = acc[:H], steer[:H]
    rs = np.random.RandomState(int(key))
    if noise == "gaussian":
        na = rs.multivariate_normal(np.zeros(H), np.eye(H), (R,))
        ns = rs.multivariate_normal(np.zeros(H), np.eye(H), (R,))
    else:
        na = rs.beta(prob.beta_a * np.abs(acc), prob.beta_b * np.abs(acc), (R, H))
        ns = rs.beta(prob.beta_a * np.abs(steer) + 1e-5, prob.beta_b * np.abs(steer) + 1e-5, (R, H))
    nc = rs.multivariate_normal(np.zeros(H), np.eye(H), (R,))
    return np.stack([na, ns, nc])


def _tracks(prob, x_obs, y_obs, vx_obs, vy_obs):
    """Constant-velocity tracks of every configuration (S/validation.py:151)."""
    K = len(x_obs)
    xt = np.zeros((K, prob.num_obs, 100), np.float32)
    yt = np.zeros((K, prob.num_obs, 100), np.float32)
    for k in range(K):
        vx = np.asarray(vx_obs[k], np.float64).reshape(-1)
        vy = np.asarray(vy_obs[k], np.float64).reshape(-1)
        xt[k], yt[k], _ = prob.cem_helper.compute_obs_trajectories(
            np.asarray(x_obs[k]).reshape(-1), np.asarray(y_obs[k]).reshape(-1), vx, vy, np.arctan2(vy, vx))
    return xt, yt


def compute_stats(prob, cx, cy, init_state, x_obs, y_obs, vx_obs, vy_obs, num_prime, noise_level, noise, num_obs,
                  key, draws=None, num_rollouts=NUM_ROLLOUTS, rng="numpy"):
    """S/validation.py:134 (static variant: obstacle state, constant-velocity
    tracks); returns (count, count_lane)."""
    xt, yt = _tracks(prob, [x_obs], [y_obs], [vx_obs], [vy_obs])
    return compute_stats_tracks(prob, cx, cy, init_state, xt[0], yt[0], num_prime, noise_level, noise, num_obs, key,
                                draws, num_rollouts, rng)


def compute_stats_tracks(prob, cx, cy, init_state, x_obs_traj, y_obs_traj, num_prime, noise_level, noise, num_obs,
                         key, draws=None, num_rollouts=NUM_ROLLOUTS, rng="numpy"):
    """D/validation.py:129 (dynamic variant: the saved [num_obs, 100] QP
    tracks are used as they are); returns (count, count_lane)."""
    c, l = compute_stats_batch(prob, np.atleast_2d(cx), np.atleast_2d(cy), np.atleast_2d(init_state), None, None,
                               None, None, num_prime, noise_level, noise, [key],
                               None if draws is None else np.asarray(draws)[None], num_rollouts,
                               x_obs_traj=np.asarray(x_obs_traj, np.float32).reshape(1, num_obs, 100),
                               y_obs_traj=np.asarray(y_obs_traj, np.float32).reshape(1, num_obs, 100), rng=rng)
    return int(c[0]), int(l[0])


def compute_stats_batch(prob, cx, cy, init_state, x_obs, y_obs, vx_obs, vy_obs, num_prime, noise_level, noise, keys,
                        draws=None, num_rollouts=NUM_ROLLOUTS, x_obs_traj=None, y_obs_traj=None, rng="numpy"):
    """All configurations of a results file at once (leading configuration
    axis).  Pass ``x_obs_traj`` / ``y_obs_traj`` [K, O, 100] for the dynamic
    variant (saved tracks); otherwise the tracks are rebuilt from the
    obstacle states like the static script.  Without ``draws`` the
    reference's NumPy draws are made per configuration (``rng="numpy"``) or
    the library's Philox streams are used (``rng="philox"``)."""
    if rng not in RNGS:
        raise ValueError(f"rng must be one of {RNGS}")
    if x_obs_traj is None:
        xt, yt = _tracks(prob, x_obs, y_obs, vx_obs, vy_obs)
    else:
        xt = np.asarray(x_obs_traj, np.float32).reshape(len(keys), prob.num_obs, 100)
        yt = np.asarray(y_obs_traj, np.float32).reshape(len(keys), prob.num_obs, 100)
    if draws is None and rng == "numpy":
        cx2, cy2 = np.atleast_2d(cx), np.atleast_2d(cy)
        draws = np.stack([reference_draws(prob, cx2[k], cy2[k], num_prime, noise, keys[k], num_rollouts)
                          for k in range(len(keys))])
    return _native.validate(cx, cy, init_state, xt, yt, keys, num_prime, noise, noise_level,
                            prob.acc_const_noise, prob.steer_const_noise, num_rollouts, prob.variant, draws,
                            device=prob._cfg.device)


# --------------------------------------------------------------------------
# the validation script (S/validation.py:202-464, D/validation.py)

def data_path(root, noise, noise_level, num_prime, cost, num_reduced, num_obs):
    """S/validation.py:235-245 (and S/main_mpc.py:130-135, which writes it)."""
    return os.path.join(root, "{}_noise/noise_{}/ts_{}/{}_{}_samples_{}_obs.npz".format(
        noise, int(noise_level * 100), num_prime, cost, num_reduced, num_obs))


def stats_path(root, noise, noise_level, num_prime, num_reduced, num_obs):
    """S/validation.py:459-461 (np.savez adds .npz)."""
    return os.path.join(root, "{}_noise/noise_{}/ts_{}/{}_samples_{}_obs.npz".format(
        noise, int(noise_level * 100), num_prime, num_reduced, num_obs))


def _config_matrix(d, num_obs):
    """Rows identifying a configuration (S/validation.py:284-294)."""
    return np.hstack((np.asarray(d["init_state"]), np.asarray(d["x_obs"])[:, 0:num_obs],
                      np.asarray(d["y_obs"])[:, 0:num_obs], np.asarray(d["vx_obs"])[:, 0:num_obs],
                      np.asarray(d["vy_obs"])[:, 0:num_obs]))


def common_configs(d_cvar, d_mmd_opt, num_obs):
    """The configurations both costs solved, in the reference's order: the
    iteration order of the Python set intersection ``cset & dset``
    (S/validation.py:299-302), and for each the first matching row of each
    file (:309-320)."""
    cm = _config_matrix(d_cvar, num_obs)
    dm = _config_matrix(d_mmd_opt, num_obs)
    cset = set([tuple(x) for x in cm])
    dset = set([tuple(x) for x in dm])
    eset = np.array([x for x in cset & dset])
    rows = []
    for k in range(eset.shape[0]):
        i_c = int(np.where(np.all(eset[k] == cm, axis=1))[0][0])
        i_m = int(np.where(np.all(eset[k] == dm, axis=1))[0][0])
        rows.append((i_c, i_m))
    return rows


def validate_files(prob, d_cvar, d_mmd_opt, noise, noise_level, num_prime, num_obs, variant="static",
                   stats_fn=None, num_rollouts=NUM_ROLLOUTS, rng="numpy"):
    """coll_* arrays of one sweep point (S/validation.py:279-364): both costs'
    optima of every common configuration k, validated with key k.
    ``stats_fn(d, idx, keys)`` -> (count, count_lane) replaces the GPU call
    (CPU tests)."""
    rows = common_configs(d_cvar, d_mmd_opt, num_obs)
    keys = np.arange(len(rows))

    def run(d, idx):
        if not len(idx):
            return np.zeros(0), np.zeros(0)
        if stats_fn is not None:
            return stats_fn(d, idx, keys)
        g = lambda name: np.asarray(d[name])[idx]
        if variant == "dynamic":
            c, l = compute_stats_batch(prob, g("cx"), g("cy"), g("init_state"), None, None, None, None, num_prime,
                                       noise_level, noise, keys, num_rollouts=num_rollouts,
                                       x_obs_traj=g("x_obs_traj"), y_obs_traj=g("y_obs_traj"), rng=rng)
        else:
            c, l = compute_stats_batch(prob, g("cx"), g("cy"), g("init_state"), g("x_obs"), g("y_obs"), g("vx_obs"),
                                       g("vy_obs"), num_prime, noise_level, noise, keys, num_rollouts=num_rollouts,
                                       rng=rng)
        return np.asarray(c, np.float64), np.asarray(l, np.float64)

    c_opt, l_opt = run(d_mmd_opt, [m for _, m in rows])
    c_cvar, l_cvar = run(d_cvar, [c for c, _ in rows])
    # np.append onto [] (S/validation.py:355-362) gives float64 arrays; the
    # mmd_random lists stay empty (their compute_stats is commented out, :336-342)
    return dict(coll_cvar=c_cvar, coll_cvar_lane=l_cvar, coll_mmd_opt=c_opt, coll_mmd_opt_lane=l_opt,
                coll_mmd_random=np.zeros(0), coll_mmd_random_lane=np.zeros(0))


def main(argv=None):
    ap = argparse.ArgumentParser(description="Monte-Carlo validation of saved optima (S/validation.py)")
    ap.add_argument("--noise_levels", type=float, nargs="+", required=True)
    ap.add_argument("--num_reduced_sets", type=int, nargs="+", required=True)
    ap.add_argument("--num_obs", type=int, nargs="+", required=True)
    ap.add_argument("--num_prime", type=int, nargs="+", required=True)
    ap.add_argument("--noises", type=str, nargs="+", required=True)
    ap.add_argument("--acc_const_noise", type=float, required=True)
    ap.add_argument("--steer_const_noise", type=float, required=True)
    ap.add_argument("--variant", default="static", choices=["static", "dynamic"])
    ap.add_argument("--root", default="./data")
    ap.add_argument("--stats_root", default="./stats")
    ap.add_argument("--rng", default="numpy", choices=RNGS,
                    help="numpy: the reference's np.random.seed(k) draws (default); philox: the library's streams")
    a = ap.parse_args(argv)
    from .cem import CEM
    for noise in a.noises:
        for noise_level in a.noise_levels:
            for num_prime in a.num_prime:
                for num_obs in a.num_obs:
                    for num_reduced in a.num_reduced_sets:
                        prob = CEM(num_reduced, num_obs, noise_level, num_prime, noise, a.acc_const_noise,
                                   a.steer_const_noise, variant=a.variant)
                        load = lambda cost: np.load(data_path(a.root, noise, noise_level, num_prime, cost,
                                                              num_reduced, num_obs))
                        d_opt, d_cvar = load("mmd_opt"), load("cvar")
                        if a.variant == "static":
                            load("mmd_random")  # the static script requires the file (:243-245), unused
                        out = validate_files(prob, d_cvar, d_opt, noise, noise_level, num_prime, num_obs, a.variant,
                                             rng=a.rng)
                        dst = stats_path(a.stats_root, noise, noise_level, num_prime, num_reduced, num_obs)
                        os.makedirs(os.path.dirname(dst), exist_ok=True)
                        np.savez(dst, **out)
                        print(f"{dst}: {len(out['coll_cvar'])} common configurations")
                        prob.handle.close()


if __name__ == "__main__":
    main()
