"""Generate tests/golden/carla_path_ref.npz by EXECUTING the reference's own
NumPy / SciPy route helpers of the CARLA optimizer,
``Helper.path_spline`` and ``Helper.waypoint_generator``
(carla/optimizer/cem_helper.py:244-276), on fixed routes.

``carla/optimizer/cem_helper.py`` cannot be imported (it imports jax at the
top), so only those two method definitions are taken from its source (parsed
with ``ast``, executed in a namespace holding ``np`` and SciPy's
``CubicSpline``, as the module's own imports provide; ``self`` is a
namespace with ``num_path = 600``, cem_helper.py's value).  Nothing from the
reference is written to the repository: the npz holds the inputs and the
outputs only.

Routes (float64, as main_carla.py:238-286 builds them from the route
planner): the synthetic Town05-like route of mpc-mmd_amd/carla/replay.py
(0.25 m spacing, a 90-degree bend), the same extended by replay.extend_route,
and a loop whose heading crosses +-pi (np.unwrap's correction).  Per route:
arc_length, arc_vec, the three splines evaluated at 997 arc positions, and
waypoint_generator's (x, y, phi) for several ego positions (on and off the
route).

Run in the build container only:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_carla_path_golden.py
"""
import ast
import importlib.util
import os
import types

import numpy as np
from scipy.interpolate import CubicSpline

REF = "/root/reference/carla/optimizer/cem_helper.py"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "carla_path_ref.npz")


def load_methods(path, names=("path_spline", "waypoint_generator")):
    tree = ast.parse(open(path).read(), path)
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Helper"][0]
    defs = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert sorted(d.name for d in defs) == sorted(names)
    ns = {"np": np, "CubicSpline": CubicSpline}
    exec(compile(ast.Module(body=defs, type_ignores=[]), path, "exec"), ns)
    return ns


def routes():
    spec = importlib.util.spec_from_file_location("replay", os.path.join(ROOT, "mpc-mmd_amd", "carla", "replay.py"))
    R = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(R)
    rx, ry = R.synthetic_route()
    ex, ey = R.extend_route(rx, ry, num_p=2000, length=500.0)
    th = np.linspace(0.0, 2.6 * np.pi, 1500)            # a loop: the heading passes +-pi
    lx, ly = 30.0 * np.cos(th) + 0.05 * th ** 2, 30.0 * np.sin(th)
    return {"town05": (rx, ry), "extended": (ex, ey), "loop": (lx, ly)}


def main():
    ns = load_methods(REF)
    self = types.SimpleNamespace(num_path=600)
    out = {}
    for name, (x, y) in routes().items():
        csx, csy, csphi, arc_length, arc_vec = ns["path_spline"](self, x, y)
        s = np.linspace(0.0, arc_length, 997)
        out[f"{name}_x"], out[f"{name}_y"] = x, y
        out[f"{name}_arc_length"] = np.float64(arc_length)
        out[f"{name}_arc_vec"] = arc_vec
        out[f"{name}_s"] = s
        out[f"{name}_csx"], out[f"{name}_csy"], out[f"{name}_csphi"] = csx(s), csy(s), csphi(s)
        ego = np.stack([x[[0, len(x) // 3, len(x) // 2]] + np.array([0.0, 1.3, -2.1]),
                        y[[0, len(x) // 3, len(x) // 2]] + np.array([0.0, -0.7, 3.4])], axis=1)
        wps = [ns["waypoint_generator"](self, e[0], e[1], x, y, arc_vec, csx, csy, csphi, arc_length) for e in ego]
        out[f"{name}_ego"] = ego
        out[f"{name}_wp"] = np.array([np.stack(w) for w in wps])     # [ego, 3 (x, y, phi), 600]
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items() if k.endswith("_wp")})


if __name__ == "__main__":
    main()
