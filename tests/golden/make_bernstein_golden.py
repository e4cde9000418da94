"""Generate tests/golden/bernstein_ref.npz by IMPORTING the reference's own
``synthetic_static_obs/bernstein_coeff_order10_arbitinterval.py`` (the only
reference module importable here: NumPy + SciPy, no JAX).

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_bernstein_golden.py

Grids follow the reference call sites: the planning grid
``linspace(0, 15, 100)`` (S/opt/cem.py:42-46) and the rollout-horizon grids
``linspace(0, 0.15*H, H)`` (S/opt/cem_helper.py:112-116).
"""
import importlib.util
import os
import sys

import numpy as np

REF = "/root/reference/synthetic_static_obs/bernstein_coeff_order10_arbitinterval.py"
HORIZONS = (8, 20, 30, 50, 60)


def main():
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("ref_bernstein", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    t = np.linspace(0, 15, 100).reshape(-1, 1)
    P, Pd, Pdd = mod.bernstein_coeff_order10_new(10, t[0], t[-1], t)
    out.update(grid100_t=t.ravel(), grid100_P=P, grid100_Pdot=Pd, grid100_Pddot=Pdd)
    for H in HORIZONS:
        t = np.linspace(0, H * (15 / 100), H).reshape(-1, 1)
        P, Pd, Pdd = mod.bernstein_coeff_order10_new(10, t[0], t[-1], t)
        out.update({f"h{H}_t": t.ravel(), f"h{H}_P": P, f"h{H}_Pdot": Pd, f"h{H}_Pddot": Pdd})
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bernstein_ref.npz")
    np.savez(dst, **out)
    print("wrote", dst, sorted(out))


if __name__ == "__main__":
    main()
