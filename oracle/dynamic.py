"""Dynamic-obstacle trajectory QP (oracle side; TEST INFRASTRUCTURE ONLY, see
``oracle/__init__.py``).

Restates ``synthetic_dynamic_obs/obs_data_generate_dynamic.py``:
``obs_data.__init__`` (:10-54: basis on linspace(0, 15, 100), weights 100,
k_p_v = k_p = 2, rho = 1, A_eq rows), ``compute_boundary_vec`` (:56-71) and
``compute_obs_guess`` (:73-109).  Written the reference's way -- the full
KKT matrix assembled with dense products and solved per right-hand side with
``numpy.linalg.solve`` (LU), fp64 here where JAX uses fp32 -- so it is an
independent check of the library's once-inverted fp64 KKT
(``csrc/host_constants.cpp: build_dyn_obs_consts``).  The fp32 basis is the
reference's (jnp.asarray of the fp64 NumPy basis, :18).
"""
from __future__ import annotations

import numpy as np

from .problem import bernstein_order10

F32 = np.float32
F64 = np.float64


def obs_guess(x0, y0, vx0, vy0, v_des, y_des=-1.75):
    """Per obstacle (rows of the inputs): x, y [O][100] fp32."""
    t = np.linspace(0, 15, 100)
    P, Pd, Pdd = (m.astype(F32).astype(F64) for m in bernstein_order10(t[0], t[-1], t))
    k_p_v = k_p = 2.0
    A_vd = Pdd - k_p_v * Pd                                    # :79
    A_pd = Pdd - k_p * P                                       # :82
    cost_x = 100 * Pdd.T @ Pdd + A_vd.T @ A_vd                 # :85-89
    cost_y = 100 * Pdd.T @ Pdd + A_pd.T @ A_pd
    A_eq_x = np.vstack((P[0], Pd[0], Pdd[0]))                  # :33
    A_eq_y = np.vstack((P[0], Pd[0], Pdd[0], Pd[-1]))          # :34
    K_x = np.block([[cost_x, A_eq_x.T], [A_eq_x, np.zeros((3, 3))]])   # :91
    K_y = np.block([[cost_y, A_eq_y.T], [A_eq_y, np.zeros((4, 4))]])   # :92
    O = len(x0)
    xs = np.zeros((O, 100), F32)
    ys = np.zeros((O, 100), F32)
    for o in range(O):
        b_vd = -k_p_v * np.ones(100) * F64(F32(v_des[o]))      # :80
        b_pd = -k_p * np.ones(100) * F64(F32(y_des))           # :83
        b_eq_x = np.array([x0[o], vx0[o], 0.0], F32).astype(F64)            # :66
        b_eq_y = np.array([y0[o], vy0[o], 0.0, 0.0], F32).astype(F64)       # :67
        sol_x = np.linalg.solve(K_x, np.hstack((A_vd.T @ b_vd, b_eq_x)))    # :94-98
        sol_y = np.linalg.solve(K_y, np.hstack((A_pd.T @ b_pd, b_eq_y)))
        cx = sol_x[:11].astype(F32).astype(F64)
        cy = sol_y[:11].astype(F32).astype(F64)
        xs[o] = (P @ cx).astype(F32)                           # :104
        ys[o] = (P @ cy).astype(F32)                           # :105
    return xs, ys
