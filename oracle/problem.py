"""Problem constants and batch-invariant matrices (oracle side).

Follows ``S/opt/cem.py:17-199`` (``CEM.__init__``), ``S/opt/cem_helper.py:10-120``
(``Helper.__init__``) and ``S/bernstein_coeff_order10_arbitinterval.py:13-103``.
Test infrastructure only (see ``oracle/__init__.py``).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
F64 = np.float64


def _binom(n: int, k: int) -> float:
    if k < 0 or k > n:
        return 0.0
    r = 1
    for i in range(1, k + 1):
        r = r * (n - k + i) // i
    return float(r)


def _bern(n: int, i: int, s: np.ndarray, oms: np.ndarray) -> np.ndarray:
    """C(n,i) (1-s)^(n-i) s^i with powers by repeated multiplication (the C++
    host in ``csrc/host_constants.cpp`` evaluates the identical sequence)."""
    if i < 0 or i > n:
        return np.zeros_like(s)
    a = np.ones_like(s)
    for _ in range(n - i):
        a = a * oms
    b = np.ones_like(s)
    for _ in range(i):
        b = b * s
    return (_binom(n, i) * a) * b


def bernstein_order10(tmin: float, tmax: float, t: np.ndarray):
    """Degree-10 Bernstein basis and first/second time derivatives (fp64).

    Restates ``S/bernstein_coeff_order10_arbitinterval.py:13-103`` with the
    standard derivative identities dB_{i,n}/ds = n (B_{i-1,n-1} - B_{i,n-1}).
    Values agree with the reference's expanded polynomials to ~1e-15; after the
    fp32 cast the reference applies (``S/opt/cem.py:48``) a handful of entries
    differ by 1 ulp (pinned in tests/test_oracle_golden.py).
    """
    n = 10
    t = np.asarray(t, dtype=F64).reshape(-1)
    l = F64(tmax) - F64(tmin)
    s = (t - F64(tmin)) / l
    oms = 1.0 - s
    P = np.stack([_bern(n, i, s, oms) for i in range(n + 1)], axis=1)
    Pd = np.stack([n * (_bern(n - 1, i - 1, s, oms) - _bern(n - 1, i, s, oms)) for i in range(n + 1)], axis=1) / l
    Pdd = np.stack([n * (n - 1) * ((_bern(n - 2, i - 2, s, oms) - 2.0 * _bern(n - 2, i - 1, s, oms))
                                   + _bern(n - 2, i, s, oms)) for i in range(n + 1)], axis=1) / (l * l)
    return P, Pd, Pdd


class Problem:
    """All reference constants (Appendix B of SURVEY.md) plus derived matrices.

    ``variant`` = "static" (``S/``) or "dynamic" (``synthetic_dynamic_obs/``):
    the only differences are ``y_lb,y_ub`` (``D/opt/cem.py:155``) and
    ``K_steer`` (``D/opt/cem_helper.py:24``).
    """

    def __init__(self, num_reduced, num_obs, noise_level, num_prime, noise,
                 acc_const_noise, steer_const_noise, num_batch=100, variant="static",
                 maxiter_cem=20):
        if noise not in ("gaussian", "beta"):
            raise ValueError("noise must be 'gaussian' or 'beta'")
        self.variant = variant
        self.noise = noise
        self.acc_const_noise = F32(acc_const_noise)
        self.steer_const_noise = F32(steer_const_noise)
        # S/opt/cem.py:24-40
        self.beta_a, self.beta_b = 2.0, 5.0
        self.a_obs, self.b_obs = 4.25, 2.75
        self.wheel_base = 2.5
        self.v_max, self.v_min, self.a_max = 30.0, 0.1, 18.0
        self.num_obs = int(num_obs)
        self.steer_max = 0.6
        self.t_fin, self.num = 15.0, 100
        self.t = self.t_fin / self.num                       # dt = 0.15 (cem.py:40)
        self.tot_time = np.linspace(0, self.t_fin, self.num)  # cem.py:42
        P, Pd, Pdd = bernstein_order10(self.tot_time[0], self.tot_time[-1], self.tot_time)
        self.P64, self.Pd64, self.Pdd64 = P, Pd, Pdd
        # jnp.asarray casts the fp64 basis to fp32 (cem.py:48)
        self.P, self.Pdot, self.Pddot = P.astype(F32), Pd.astype(F32), Pdd.astype(F32)
        self.nvar = 11
        self.num_prime = int(num_prime)
        self.maxiter = 1                  # cem.py:88
        self.maxiter_cem = int(maxiter_cem)  # cem.py:89
        self.k_p_v = 2.0                  # cem.py:91
        self.k_p = 2.0                    # cem.py:94
        self.num_partial = 25             # cem.py:112
        self.alpha_mean, self.alpha_cov, self.lamda = 0.6, 0.6, 0.9  # cem.py:118-121
        self.gamma = 1.0
        self.num_params = 8
        self.num_batch = int(num_batch)   # cem.py:137 (hard-coded 100 there)
        self.ellite_num = 5
        self.ellite_num_projection = self.num_batch   # cem.py:139 (Q6)
        self.ellite_num_cost = 20
        self.num_reduced = int(num_reduced)
        self.num_mother = self.num_reduced ** 2      # cem.py:143
        self.y_des_1, self.y_des_2 = -1.75, 1.75
        self.carla = variant.startswith("carla")
        if variant == "static":
            self.y_lb, self.y_ub = -2.25, 2.25        # S/opt/cem.py:155
            self.K_steer = 0.01                       # S/opt/cem_helper.py:24
        elif variant == "dynamic":
            self.y_lb, self.y_ub = -2.25, -1.25       # D/opt/cem.py:155
            self.K_steer = 0.05                       # D/opt/cem_helper.py:24
        elif variant in ("carla_town05", "carla_town10hd"):
            # C/opt/cem.py:25-36, 152-178: CARLA constants (the optimizer of
            # C/main_carla.py; C/ = carla/, C/opt/ = carla/optimizer/)
            self.a_obs, self.b_obs = 4.5, 3.0          # :26
            self.wheel_base = 2.875                    # :27
            self.a_centr = 1.5                         # :29
            if variant == "carla_town10hd":            # :161-166
                self.y_lb, self.y_ub = -0.3, 3.8
                self.y_des_1, self.y_des_2 = 0.0, 3.5
            else:
                self.y_lb, self.y_ub = -3.8, 0.3
                self.y_des_1, self.y_des_2 = 0.0, -3.5
            self.K_steer = 1.0                         # beta steer noise sigma (2b - 1) (C/opt/cem_helper.py:777)
            self.init_mu, self.init_sigma = (0.3, 0.0), (0.05, 0.1)   # :152-153 (noisy init states)
            self.gamma_lane_des = 0.3                  # :182
        else:
            raise ValueError("variant must be 'static', 'dynamic', 'carla_town05' or 'carla_town10hd'")
        self.alpha_quant = 0.98
        self.weight_mmd_lane, self.weight_mmd_obs = 0.0, 1e3
        self.weight_cvar_lane, self.weight_cvar_obs = 0.0, 1e3
        self.weight_saa_lane, self.weight_saa_obs = 1e6, 1e6
        self.weight_mmd_lane_des = self.weight_cvar_lane_des = 0.0
        if self.carla:                                 # C/opt/cem.py:171-174
            self.weight_mmd_lane_des, self.weight_mmd_lane, self.weight_mmd_obs = 0.0, 0.01, 0.1
            self.weight_cvar_lane_des, self.weight_cvar_lane, self.weight_cvar_obs = 0.0, 25.0, 100.0
            self.weight_saa_lane, self.weight_saa_obs = 1000.0, 1000.0
        self.ker_wt = 1000.0
        self.sigma_acc = float(noise_level)
        self.sigma_steer = float(noise_level)
        # beta_cem (S/compute_beta.py:14-29)
        self.num_samples_cem = 100
        self.maxiter_beta_cem = 20
        self.num_ellite_beta = max(int(0.1 * self.num_samples_cem) + 1, 3)   # = 11
        self.sigma_clip = 0.01
        # rollout-horizon basis (cem_helper.py:112-116)
        self.t_fin_prime = self.num_prime * self.t
        tp = np.linspace(0, self.t_fin_prime, self.num_prime)
        Pp, _, _ = bernstein_order10(tp[0], tp[-1], tp)
        self.P_prime = Pp.astype(F32)
        self._build_matrices()

    # ------------------------------------------------------------------
    def _build_matrices(self):
        """Batch-invariant matrices, assembled in fp64 from the fp32 basis.

        Assembly loops and the Gauss-Jordan inverse repeat the fixed operation
        order of ``csrc/host_constants.cpp`` so the oracle and the library hold
        bit-identical constants (the guess KKT has condition ~1e5: two
        different fp64 solvers disagree in the 11th digit, enough to flip fp32
        roundings of the coefficients)."""
        P = self.P.astype(F64)
        Pd = self.Pdot.astype(F64)
        Pdd = self.Pddot.astype(F64)
        nv = self.nvar
        self.A_eq_x = np.stack([P[0], Pd[0], Pdd[0]])               # cem.py:55
        self.A_eq_y = np.stack([P[0], Pd[0], Pdd[0], Pd[-1]])       # cem.py:56
        # lane bound (cem.py:126-134, gamma = 1 so A_ub = P[1:], A_lb = -P[1:])
        self.A_lane = np.vstack([P[1:], -P[1:]])                     # [198, 11]

        def kkt(cost, A_eq):
            ne = A_eq.shape[0]
            return np.block([[cost, A_eq.T], [A_eq, np.zeros((ne, ne))]])

        # ---- initial-guess QP (cem_helper.py:183-217)
        seg = self.num_partial
        sm = _atb(Pdd, Pdd)
        cx = 100.0 * sm
        cy = 100.0 * sm
        self.guess_colsum_x = np.zeros((4, nv))
        self.guess_colsum_y = np.zeros((4, nv))
        for k in range(4):
            sl = slice(k * seg, (k + 1) * seg)
            A_vd = Pdd[sl] - self.k_p_v * Pd[sl]
            A_pd = Pdd[sl] - self.k_p * P[sl]
            for r in range(seg):
                self.guess_colsum_x[k] = self.guess_colsum_x[k] + A_vd[r]
                self.guess_colsum_y[k] = self.guess_colsum_y[k] + A_pd[r]
            cx = cx + _atb(A_vd, A_vd)
            cy = cy + _atb(A_pd, A_pd)
        self.guess_kkt_x = kkt(cx, self.A_eq_x)     # 14x14
        self.guess_kkt_y = kkt(cy, self.A_eq_y)     # 15x15
        self.guess_kinv_x = gauss_jordan_inverse(self.guess_kkt_x)
        self.guess_kinv_y = gauss_jordan_inverse(self.guess_kkt_y)
        # c_bar = G v + h  (G[k][j] = sum_i Kinv[k][i] (-k_p colsum_j[i]), sequential i)
        self.guess_G = np.zeros((2, nv, 4))
        for xy, (Ki, cs, kp) in enumerate(((self.guess_kinv_x, self.guess_colsum_x, self.k_p_v),
                                           (self.guess_kinv_y, self.guess_colsum_y, self.k_p))):
            acc = np.zeros((nv, 4))
            for i in range(nv):
                acc = acc + Ki[:nv, i][:, None] * (-kp * cs[:, i])[None, :]
            self.guess_G[xy] = acc

        # ---- projection KKT (projection.py:145-156), rho_* = 1, A_projection = I
        base = (np.eye(nv) + _atb(Pdd, Pdd)) + _atb(Pd, Pd)
        self.proj_kkt_x = kkt(base, self.A_eq_x)
        self.proj_kkt_y = kkt(base + _atb(self.A_lane, self.A_lane), self.A_eq_y)
        self.proj_kinv_x = gauss_jordan_inverse(self.proj_kkt_x)
        self.proj_kinv_y = gauss_jordan_inverse(self.proj_kkt_y)

        # ---- Bernstein fit on the rollout horizon (cem_helper.py:553-564)
        Pp = self.P_prime.astype(F64)
        g = _atb(Pp, Pp) + 0.05 * np.eye(nv)
        self.fit_cost = g
        gi = gauss_jordan_inverse(g)
        fit = np.zeros((nv, self.num_prime))
        for k in range(nv):
            fit = fit + gi[:, k][:, None] * Pp[:, k][None, :]
        self.fit = fit                                               # [11, H]

    def det_kinv(self):
        """KKT inverses of the CARLA det projection (``C/opt/projection_det.py:
        149-160``): the cost matrices gain ``rho_obs A_obs^T A_obs`` with
        ``A_obs = tile(P, (num_obs, 1))`` (``C/opt/cem.py:66``), accumulated row
        by row over the O x 100 rows (host_constants.cpp: det_projection_kinv).
        Returns (kinv_x [14, 14], kinv_y [15, 15]); cached."""
        if getattr(self, "_det_kinv", None) is None:
            P = self.P.astype(F64)
            nv = self.nvar
            A_obs = np.tile(P, (self.num_obs, 1))
            obs = _atb(A_obs, A_obs)
            base = (np.eye(nv) + _atb(self.Pddot.astype(F64), self.Pddot.astype(F64))) \
                + _atb(self.Pdot.astype(F64), self.Pdot.astype(F64))
            ne_x, ne_y = self.A_eq_x.shape[0], self.A_eq_y.shape[0]
            kx = np.block([[base + obs, self.A_eq_x.T], [self.A_eq_x, np.zeros((ne_x, ne_x))]])
            ky = np.block([[(base + _atb(self.A_lane, self.A_lane)) + obs, self.A_eq_y.T],
                           [self.A_eq_y, np.zeros((ne_y, ne_y))]])
            self._det_kinv = (gauss_jordan_inverse(kx), gauss_jordan_inverse(ky))
        return self._det_kinv

    def kkt_rhs_const(self, kinv, b):
        """Kinv[:11, 11:] @ b_eq, sequential over the equality rows."""
        out = np.zeros(self.nvar)
        for e in range(len(b)):
            out = out + kinv[:self.nvar, self.nvar + e] * F64(b[e])
        return out


def _atb(A, B):
    """A^T B accumulated row by row (host_constants.cpp: atb)."""
    C = np.zeros((A.shape[1], B.shape[1]))
    for r in range(A.shape[0]):
        C = C + np.outer(A[r], B[r])
    return C


def gauss_jordan_inverse(a):
    """Gauss-Jordan with partial pivoting, the operation order of
    host_constants.cpp: invert()."""
    a = np.array(a, dtype=F64)
    n = a.shape[0]
    inv = np.eye(n)
    for c in range(n):
        piv = c
        for r in range(c + 1, n):
            if abs(a[r, c]) > abs(a[piv, c]):
                piv = r
        if a[piv, c] == 0.0:
            raise np.linalg.LinAlgError("singular")
        if piv != c:
            a[[c, piv]] = a[[piv, c]]
            inv[[c, piv]] = inv[[piv, c]]
        d = a[c, c]
        a[c] = a[c] / d
        inv[c] = inv[c] / d
        for r in range(n):
            if r == c:
                continue
            f = a[r, c]
            if f == 0.0:
                continue
            a[r] = a[r] - f * a[c]
            inv[r] = inv[r] - f * inv[c]
    return inv
