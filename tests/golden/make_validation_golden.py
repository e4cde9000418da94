"""Generate tests/golden/validation_ref.npz by EXECUTING the reference's own
pure-NumPy Monte-Carlo functions (S/validation.py:21-171 and the dynamic copy
D/validation.py:21-165): ``compute_rollout_one_step``,
``compute_rollout_complete`` (seeded with ``np.random.seed(key)`` exactly as
the reference does), ``compute_f_bar_temp``, ``compute_lane_bar``,
``compute_controls`` and ``compute_stats``.

The modules themselves cannot be imported (they import jax and run argparse
at import time), so only those function definitions are taken from the
reference's source (parsed with ``ast``, executed in a namespace of their
own; nothing from the reference is written to the repository).  The
namespace provides what the functions read from globals:
  * ``prob``: the Appendix-B constants (t = 0.15, wheel_base = 2.5,
    a_obs / b_obs, y_lb / y_ub, beta_a / beta_b, the const-noise levels,
    cem_helper.K_steer) and ``Pdot_jax`` / ``Pddot_jax`` = fp32 casts of
    the basis produced by IMPORTING the reference's
    bernstein_coeff_order10_arbitinterval.py (as ``jnp.asarray`` does,
    S/opt/cem.py:46-48);
  * ``prob.cem_helper.compute_obs_trajectories`` (static variant only): the
    oracle's restatement of S/opt/cem_helper.py:366-378 (JAX, not
    executable here) -- the fixture's obstacles are static, so the tracks
    are constant rows;
  * ``_num_batch = 1000`` (S/validation.py:173).

Outputs per case: inputs, the controls, the 1000 x H rollouts and the
(count, count_lane) the reference computes.  The draws are NumPy's own
(np.random.seed(key) + multivariate_normal / beta), so the oracle's
restatement of that call sequence (oracle.validation.draws_numpy) and the
GPU kernel fed with those draws are pinned to the reference's numbers.

Run in the build container only (``/root/reference`` does not exist on the
GPU box):  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_validation_golden.py
"""
import ast
import importlib.util
import os
import sys
import types

import numpy as np

REF = "/root/reference"
FUNCS = ("compute_rollout_one_step", "compute_rollout_complete", "compute_f_bar_temp", "compute_lane_bar",
         "compute_controls", "compute_stats")
H = 20          # num_prime
O = 4           # num_obs


def load_functions(path, ns):
    """Execute the named function definitions of a reference script in ns."""
    tree = ast.parse(open(path).read(), path)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in FUNCS]
    assert sorted(d.name for d in defs) == sorted(FUNCS), [d.name for d in defs]
    exec(compile(ast.Module(body=defs, type_ignores=[]), path, "exec"), ns)
    return ns


def reference_basis():
    spec = importlib.util.spec_from_file_location(
        "ref_bernstein", os.path.join(REF, "synthetic_static_obs/bernstein_coeff_order10_arbitinterval.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    t = np.linspace(0, 15, 100).reshape(-1, 1)
    P, Pd, Pdd = mod.bernstein_coeff_order10_new(10, t[0], t[-1], t)
    return P, Pd.astype(np.float32), Pdd.astype(np.float32)


def make_prob(variant, acc_c, steer_c, Pd, Pdd):
    from oracle.helper import compute_obs_trajectories
    from oracle.problem import Problem
    y_lb, y_ub = (-2.25, 2.25) if variant == "static" else (-2.25, -1.25)   # S/opt/cem.py:155, D/opt/cem.py:155
    K_steer = 0.01 if variant == "static" else 0.05                          # cem_helper.py:24
    ora = Problem(10, O, 0.1, H, "gaussian", acc_c, steer_c, variant=variant)
    helper = types.SimpleNamespace(K_steer=K_steer,
                                   compute_obs_trajectories=lambda *a: compute_obs_trajectories(ora, *a))
    return types.SimpleNamespace(t=15 / 100, wheel_base=2.5, a_obs=4.25, b_obs=2.75, y_lb=y_lb, y_ub=y_ub,
                                 beta_a=2, beta_b=5, acc_const_noise=acc_c, steer_const_noise=steer_c, num=100,
                                 Pdot_jax=Pd, Pddot_jax=Pdd, cem_helper=helper)


def saved_optimum(P, y0, y1, a):
    """Bernstein coefficients of a lane change from y0 to y1 while
    accelerating (least squares on the planning grid), like a saved optimum."""
    t = np.linspace(0, 15, 100)
    x = 5.0 * t + 0.5 * a * t ** 2
    s = np.clip((t - 0.5) / 4.0, 0.0, 1.0)
    y = y0 + (y1 - y0) * (3 * s ** 2 - 2 * s ** 3)
    cx = np.linalg.lstsq(P, x, rcond=None)[0]
    cy = np.linalg.lstsq(P, y, rcond=None)[0]
    return cx, cy


CASES = [
    # name, variant, noise, level, acc_c, steer_c, y0, y1, accel, key
    ("static_gauss", "static", "gaussian", 0.1, 0.05, 0.01, 1.75, -1.75, 1.0, 3),
    ("static_beta", "static", "beta", 0.3, 0.0, 0.0, 1.75, -1.75, 1.5, 5),
    ("dynamic_gauss", "dynamic", "gaussian", 0.2, 0.1, 0.02, -1.75, -1.75, 0.8, 7),
    ("dynamic_beta", "dynamic", "beta", 0.3, 0.05, 0.0, -1.75, -1.75, 1.2, 11),
]


def main():
    sys.dont_write_bytecode = True
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(os.path.dirname(here)))   # repo root: oracle
    P, Pd, Pdd = reference_basis()
    out = {"cases": np.array([c[0] for c in CASES]), "num_prime": H, "num_obs": O}
    for name, variant, noise, level, acc_c, steer_c, y0, y1, accel, key in CASES:
        prob = make_prob(variant, acc_c, steer_c, Pd, Pdd)
        sub = "synthetic_static_obs" if variant == "static" else "synthetic_dynamic_obs"
        ns = load_functions(os.path.join(REF, sub, "validation.py"), {"np": np, "prob": prob, "_num_batch": 1000})
        cx, cy = saved_optimum(P, y0, y1, accel)
        init = np.array([0.0, y0, 5.0, 0.0, 0.0, 0.0])
        # obstacles just outside the NOMINAL (noise-free) rollout at its last
        # recorded steps, where the noisy rollouts spread most: only the
        # rollouts that drift towards an obstacle collide (partial counts)
        xd, xdd = np.dot(Pd, cx), np.dot(Pdd, cx)
        yd, ydd = np.dot(Pd, cy), np.dot(Pdd, cy)
        acc, steer = ns["compute_controls"](xd, yd, xdd, ydd)
        st = np.array([[init[0], init[1], init[2], init[3], np.arctan2(init[3], init[2])]])
        nom = []
        for h in range(H):
            nom.append(st[0, :2].copy())
            st = ns["compute_rollout_one_step"](acc[h], steer[h], st)
        nom = np.array(nom)
        tt = np.linspace(0, 15, 100)
        vx = np.zeros(O) if variant == "static" else np.array([1.0, 0.5, 3.0, 0.0])
        vy = np.zeros(O) if variant == "static" else np.array([0.0, -0.02, 0.0, 0.01])
        at = [(H - 1, 0.0, 2.75 + 0.03), (H - 1, 4.25 + 0.05, 0.0), (H - 4, 0.0, -(2.75 + 0.02)), (0, 60.0, 0.0)]
        xo = np.array([nom[h, 0] + dx - vx[i] * tt[h] for i, (h, dx, dy) in enumerate(at)])
        yo = np.array([nom[h, 1] + dy - vy[i] * tt[h] for i, (h, dx, dy) in enumerate(at)])
        if variant == "static":
            res = ns["compute_stats"](cx, cy, init, xo, yo, vx, vy, H, level, noise, O, key)
            xt, yt = res[4], res[5]
        else:
            xt = (xo[:, None] + vx[:, None] * tt).astype(np.float32)
            yt = (yo[:, None] + vy[:, None] * tt).astype(np.float32)
            res = ns["compute_stats"](cx, cy, init, xt, yt, H, level, noise, O, key)
        count, count_lane, x_roll, y_roll = res[:4]
        print(f"{name}: count {count} count_lane {count_lane}")
        assert 0 < count < 1000, "the case should collide for some rollouts only"
        pre = name + "_"
        out.update({pre + "variant": variant, pre + "noise": noise, pre + "level": level, pre + "acc_c": acc_c,
                    pre + "steer_c": steer_c, pre + "key": key, pre + "cx": cx, pre + "cy": cy,
                    pre + "init_state": init, pre + "x_obs": xo, pre + "y_obs": yo, pre + "vx_obs": vx,
                    pre + "vy_obs": vy, pre + "x_obs_traj": np.asarray(xt, np.float32),
                    pre + "y_obs_traj": np.asarray(yt, np.float32), pre + "acc": acc, pre + "steer": steer,
                    pre + "x_roll": x_roll, pre + "y_roll": y_roll, pre + "count": int(count),
                    pre + "count_lane": int(count_lane)})
    dst = os.path.join(here, "validation_ref.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst)


if __name__ == "__main__":
    main()
