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

Outputs per case: inputs, the controls, the 1000 x H rollouts, their
per-element collision residuals f_bar [O][1000][H] and lane bars, and the
(count, count_lane) the reference computes.  Also the static driver's scenario
sequence: ``compute_obs_data`` of S/main_mpc.py:10-21 executed for k < 200.  The draws are NumPy's own
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


def load_functions(path, ns, names=FUNCS):
    """Execute the named function definitions of a reference script in ns."""
    tree = ast.parse(open(path).read(), path)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert sorted(d.name for d in defs) == sorted(names), [d.name for d in defs]
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


def make_prob(variant, acc_c, steer_c, Pd, Pdd, H_=H, O_=O):
    from oracle.helper import compute_obs_trajectories
    from oracle.problem import Problem
    y_lb, y_ub = (-2.25, 2.25) if variant == "static" else (-2.25, -1.25)   # S/opt/cem.py:155, D/opt/cem.py:155
    K_steer = 0.01 if variant == "static" else 0.05                          # cem_helper.py:24
    ora = Problem(10, O_, 0.1, H_, "gaussian", acc_c, steer_c, variant=variant)
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


OBS_COUNTS = (2, 4, 9)   # num_obs <= 9: the reference's grid (S/main_mpc.py:13) places at most 9
OBS_CONFIGS = 200        # S/main_mpc.py:76


def obstacle_configs():
    """The static driver's scenario sequence, executed: for k < 200,
    ``compute_obs_data(num_obs, k)`` (S/main_mpc.py:10-21) and the
    ``np.random.randint(1, 10000)`` idx_mpc the driver draws right after it
    (:114) -> obs_<O>_{x,y,idx} [200][O] / [200]."""
    ns = load_functions(os.path.join(REF, "synthetic_static_obs", "main_mpc.py"), {"np": np},
                        names=("compute_obs_data",))
    out = {}
    for O_ in OBS_COUNTS:
        xs, ys, idx = [], [], []
        for k in range(OBS_CONFIGS):
            x, y, vx, vy, psi = ns["compute_obs_data"](O_, k)
            assert not (vx.any() or vy.any() or psi.any())
            xs.append(x)
            ys.append(y)
            idx.append(np.random.randint(1, 10000))
        out.update({f"obs_{O_}_x": np.array(xs, np.float64), f"obs_{O_}_y": np.array(ys),
                    f"obs_{O_}_idx": np.array(idx, np.int64)})
    return out


# The validation SCRIPT (S/validation.py:224-464) on small data files of the
# S/main_mpc.py:130-135 layout: configurations k from compute_obs_data, the
# cvar file holding k in CVAR_K, the mmd_opt file k in OPT_K (the drivers
# save only the configurations each cost solved, so the files differ)
SCRIPT_POINTS = [("gaussian", 0.1), ("beta", 0.3)]
SCRIPT_H, SCRIPT_O, SCRIPT_N = 50, 4, 10
CVAR_K = (0, 2, 3, 5, 8, 11)
OPT_K = (1, 2, 3, 5, 7, 8, 11)


def script_cases(P, Pd, Pdd):
    """For each sweep point: the two data files and the coll_* arrays the
    reference's main loop computes from them -- the loop of :284-362
    restated (set intersection, first matching row, key = position k) around
    the EXECUTED compute_stats."""
    obs_ns = load_functions(os.path.join(REF, "synthetic_static_obs", "main_mpc.py"), {"np": np},
                            names=("compute_obs_data",))
    out = {}
    for noise, level in SCRIPT_POINTS:
        prob = make_prob("static", 0.0, 0.0, Pd, Pdd, H_=SCRIPT_H, O_=SCRIPT_O)
        ns = load_functions(os.path.join(REF, "synthetic_static_obs", "validation.py"),
                            {"np": np, "prob": prob, "_num_batch": 1000})
        files = {}
        for cost, ks in (("cvar", CVAR_K), ("mmd_opt", OPT_K)):
            d = {key: [] for key in ("cx", "cy", "init_state", "x_obs", "y_obs", "vx_obs", "vy_obs")}
            for k in ks:
                x, y, vx, vy, _ = obs_ns["compute_obs_data"](SCRIPT_O, k)
                # an optimum-like plan per (cost, k): lane change or lane keeping, some acceleration
                y1 = -1.75 if (k + (cost == "cvar")) % 2 else 1.75
                cx, cy = saved_optimum(P, 1.75, y1, 0.6 + 0.15 * (k % 5))
                for key, v in (("cx", cx), ("cy", cy), ("init_state", [0.0, 1.75, 5.0, 0.0, 0.0, 0.0]), ("x_obs", x),
                               ("y_obs", y), ("vx_obs", vx), ("vy_obs", vy)):
                    d[key].append(np.asarray(v, np.float64))
            files[cost] = {key: np.array(v) for key, v in d.items()}
        mat = lambda d: np.hstack((d["init_state"], d["x_obs"][:, 0:SCRIPT_O], d["y_obs"][:, 0:SCRIPT_O],
                                   d["vx_obs"][:, 0:SCRIPT_O], d["vy_obs"][:, 0:SCRIPT_O]))
        cvar_matrix, opt_matrix = mat(files["cvar"]), mat(files["mmd_opt"])
        cset = set([tuple(x) for x in cvar_matrix])
        dset = set([tuple(x) for x in opt_matrix])
        eset = np.array([x for x in cset & dset])
        coll = {key: [] for key in ("coll_cvar", "coll_cvar_lane", "coll_mmd_opt", "coll_mmd_opt_lane")}
        for k in range(eset.shape[0]):
            for cost, m in (("mmd_opt", opt_matrix), ("cvar", cvar_matrix)):
                i = np.where(np.all(eset[k] == m, axis=1))[0]
                if len(i) > 1:
                    i = i[0]
                f = files[cost]
                c, cl = ns["compute_stats"](f["cx"][i], f["cy"][i], f["init_state"][i], f["x_obs"][i], f["y_obs"][i],
                                            f["vx_obs"][i], f["vy_obs"][i], SCRIPT_H, level, noise, SCRIPT_O, k)[:2]
                coll[f"coll_{cost}"] = np.append(coll[f"coll_{cost}"], c)
                coll[f"coll_{cost}_lane"] = np.append(coll[f"coll_{cost}_lane"], cl)
        pre = f"script_{noise}_"
        for cost, f in files.items():
            out.update({pre + cost + "_" + key: v for key, v in f.items()})
        out.update({pre + key: np.asarray(v, np.float64) for key, v in coll.items()})
        print(f"script {noise}: {eset.shape[0]} common configurations, coll_cvar {coll['coll_cvar']}, "
              f"coll_mmd_opt {coll['coll_mmd_opt']}")
    out.update(script_points=np.array([p[0] for p in SCRIPT_POINTS]), script_levels=np.array([p[1] for p in SCRIPT_POINTS]),
               script_num_prime=SCRIPT_H, script_num_obs=SCRIPT_O, script_num_reduced=SCRIPT_N)
    return out


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
        # the reference's per-element residuals of those rollouts (what
        # compute_stats counts): f_bar [O][R][H], lane bars [R][H]
        f_bar = ns["compute_f_bar_temp"](np.asarray(xt, np.float64), np.asarray(yt, np.float64), x_roll, y_roll, H, O)
        lane_lb, lane_ub = ns["compute_lane_bar"](y_roll, H)
        print(f"{name}: count {count} count_lane {count_lane}")
        assert 0 < count < 1000, "the case should collide for some rollouts only"
        pre = name + "_"
        out.update({pre + "variant": variant, pre + "noise": noise, pre + "level": level, pre + "acc_c": acc_c,
                    pre + "steer_c": steer_c, pre + "key": key, pre + "cx": cx, pre + "cy": cy,
                    pre + "init_state": init, pre + "x_obs": xo, pre + "y_obs": yo, pre + "vx_obs": vx,
                    pre + "vy_obs": vy, pre + "x_obs_traj": np.asarray(xt, np.float32),
                    pre + "y_obs_traj": np.asarray(yt, np.float32), pre + "acc": acc, pre + "steer": steer,
                    pre + "x_roll": x_roll, pre + "y_roll": y_roll, pre + "count": int(count),
                    pre + "count_lane": int(count_lane), pre + "f_bar": f_bar, pre + "lane_lb": lane_lb,
                    pre + "lane_ub": lane_ub})
    out.update(obstacle_configs())
    out.update(script_cases(P, Pd, Pdd))
    dst = os.path.join(here, "validation_ref.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst)


if __name__ == "__main__":
    main()
