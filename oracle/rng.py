"""Random draws for the oracle: explicit containers + the Philox streams.

The reference draws from jax.random (threefry2x32): ``multivariate_normal`` at
``S/opt/cem_helper.py:126,292,406-441,470-505`` and ``S/compute_beta.py:46,63``,
``beta`` at ``S/opt/cem_helper.py:427-433,492-498``.  Those streams are not
reproducible here (JAX absent), so parity is defined on injected draws:
``Draws`` carries every standard-normal tensor the algorithm consumes.  The
structure of the reference's keys is kept:

* the initial population and the beta-CEM tables use a *fixed* key, identical
  for every call and candidate (``S/opt/cem_helper.py:86,125``,
  ``S/compute_beta.py:25,108,131``);
* per outer iteration ``t`` the key is ``3*idx_mpc + 5*t + 7``
  (``S/opt/cem.py:225``), shared by all candidates (Q2);
* Beta noise needs draws that depend on the controls, so it is always produced
  from the counter-based streams below (never injected).

Internal streams: Philox4x32-10 (Salmon et al., SC'11; Random123 constants),
Box-Muller in fp64, Marsaglia-Tsang gamma in fp64.  ``csrc/rng.hpp`` implements
the identical counter layout on the GPU.
Test infrastructure only (see ``oracle/__init__.py``).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
U32 = np.uint32
M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF

# stream identifiers (counter word 2); keep in sync with csrc/rng.hpp
STREAM_ROLL_ACC, STREAM_ROLL_STEER, STREAM_ROLL_CONST = 0, 1, 2
STREAM_RESAMPLE = 3
STREAM_GAMMA_ACC_A, STREAM_GAMMA_ACC_B, STREAM_GAMMA_STEER_A, STREAM_GAMMA_STEER_B = 4, 5, 6, 7
STREAM_POP0, STREAM_BETA_Z0, STREAM_BETA_Z = 16, 17, 18
STREAM_INIT_EPS = 19   # CARLA noisy initial states, key (idx_mpc, seed)
FIXED_KEY0 = 0xFFFFFFFF
GAMMA_MAX_ATTEMPTS = 32
BETA_A_RATIO, BETA_B_RATIO = 2.0, 5.0   # beta_a, beta_b (S/opt/cem.py:24)
BOOST_LIN_MIN = -600.0                  # csrc/rng.hpp: kBoostLinMin


def philox4x32_10(ctr, key):
    """Vectorised Philox4x32-10.  ctr: 4 uint arrays (broadcastable), key: 2."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK for c in ctr)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.asarray(key[0], dtype=np.uint64) & MASK
    k1 = np.asarray(key[1], dtype=np.uint64) & MASK
    for _ in range(10):
        p0 = np.uint64(M0) * c0
        p1 = np.uint64(M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & np.uint64(MASK), lo1, (hi0 ^ c3 ^ k1) & np.uint64(MASK), lo0
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK)
    return c0.astype(U32), c1.astype(U32), c2.astype(U32), c3.astype(U32)


def _u01(u):
    """uint32 -> fp64 uniform strictly inside (0, 1)."""
    return (u.astype(np.float64) + 0.5) * (1.0 / 4294967296.0)


def _box_muller(u0, u1):
    r = np.sqrt(-2.0 * np.log(_u01(u0)))
    th = (2.0 * np.pi) * _u01(u1)
    return r * np.cos(th), r * np.sin(th)


def philox_normals(key, stream, word1, count):
    """``count`` standard normals (fp32) of stream ``(stream, word1)``.

    Element e lives in counter (e // 4, word1, stream, 0): the four Philox
    words give two Box-Muller pairs -> normals 4j..4j+3.
    """
    nblk = (count + 3) // 4
    j = np.arange(nblk, dtype=np.uint64)
    u = philox4x32_10((j, word1, stream, 0), key)
    z0, z1 = _box_muller(u[0], u[1])
    z2, z3 = _box_muller(u[2], u[3])
    z = np.stack([z0, z1, z2, z3], axis=1).reshape(-1)[:count]
    return z.astype(F32)


def iteration_key(idx_mpc, t, seed):
    """Per-iteration key: the reference's PRNGKey(3*idx_mpc + 5*idx + 7)."""
    return ((3 * int(idx_mpc) + 5 * int(t) + 7) & MASK, int(seed) & MASK)


def fixed_key(seed):
    return (FIXED_KEY0, int(seed) & MASK)


def _log_gamma_parts(alpha, key, stream, elem, linear=False):
    """Marsaglia-Tsang core for Gamma(alpha') with alpha' = alpha + 1 when
    alpha < 1 (boost), in fp64.  Returns (log G', log U_boost).

    Attempt k uses counter (elem, k, stream, 1): words 0,1 -> Box-Muller normal
    (cos branch), word 2 -> acceptance uniform (squeeze, then log test), word
    3 -> boost uniform.  The GPU reads attempts 0..3 from a per-iteration
    table of these same values (csrc/rng.hpp: k_gamma_tab); that is caching,
    not a different stream.
    Not accepted after GAMMA_MAX_ATTEMPTS -> G' = d (never observed).
    ``linear=True`` returns G' itself instead of log G'.
    """
    alpha = np.asarray(alpha, dtype=np.float64)
    elem = np.asarray(elem, dtype=np.uint64)
    a1 = np.where(alpha < 1.0, alpha + 1.0, alpha)
    d = a1 - 1.0 / 3.0
    c = 1.0 / np.sqrt(9.0 * d)
    out = d.copy() if linear else np.log(d)
    logub = np.zeros(alpha.shape)
    done = np.zeros(alpha.shape, dtype=bool)
    for k in range(GAMMA_MAX_ATTEMPTS):
        u = philox4x32_10((elem, k, stream, 1), key)
        r = np.sqrt(-2.0 * np.log(_u01(u[0])))
        x = r * np.cos((2.0 * np.pi) * _u01(u[1]))
        v = 1.0 + c * x
        vpos = v > 0.0
        v3 = np.where(vpos, v * v * v, 1.0)
        uu = _u01(u[2])
        lu = np.log(uu)
        # squeeze first, exact log test when it fails (Marsaglia & Tsang 2000;
        # csrc/rng.hpp: mt_accept evaluates the same two tests)
        squeeze = uu < 1.0 - 0.0331 * (x * x) * (x * x)
        acc = vpos & (squeeze | (lu < 0.5 * x * x + d - d * v3 + d * np.log(v3)))
        newly = acc & ~done
        out = np.where(newly, d * v3 if linear else np.log(d * v3), out)
        logub = np.where(newly, np.log(_u01(u[3])), logub)
        done = done | acc
        if done.all():
            break
    return out, logub


def beta_draws(a, b, key, stream_a, stream_b, elem):
    """Beta(a, b) = Ga / (Ga + Gb) (fp64 -> fp32), G = G' U^(1/alpha) for
    alpha < 1 (boost).  Evaluated in linear space while both boost factors
    log(U)/alpha exceed -600 (no underflow), else in log space -- the same
    two-branch formula as csrc/rng.hpp: beta_draw_tab.  For a = b = 0
    (|control| == 0 exactly) the reference's Beta(0, 0) is NaN;
    with the reference's fp32 solves the controls are never exactly zero, so
    we take the alpha -> 0+ limit of the same draw instead: 1 if
    log(U_a)/a_ratio > log(U_b)/b_ratio else 0 (Numerics).
    """
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    ga, ua = _log_gamma_parts(a, key, stream_a, elem, linear=True)
    gb, ub = _log_gamma_parts(b, key, stream_b, elem, linear=True)
    zero = (a == 0.0) & (b == 0.0)
    sa = np.where(a > 0, a, 1.0)
    sb = np.where(b > 0, b, 1.0)
    ba = np.where(a < 1.0, ua / sa, 0.0)
    bb = np.where(b < 1.0, ub / sb, 0.0)
    with np.errstate(over="ignore", under="ignore", divide="ignore", invalid="ignore"):
        Ga = ga * np.where(a < 1.0, np.exp(ba), 1.0)
        Gb = gb * np.where(b < 1.0, np.exp(bb), 1.0)
        lin = Ga / (Ga + Gb)
        la = np.log(ga) + ba
        lb = np.log(gb) + bb
        lm = np.maximum(la, lb)
        ea = np.exp(la - lm)
        eb = np.exp(lb - lm)
        logsp = ea / (ea + eb)
    out = np.where((ba > BOOST_LIN_MIN) & (bb > BOOST_LIN_MIN), lin, logsp)
    lim = np.where(ua * BETA_B_RATIO > ub * BETA_A_RATIO, 1.0, 0.0)
    return np.where(zero, lim, out).astype(F32)


class Draws:
    """Every standard-normal tensor a solve consumes.

    pop0      [B, 8]             initial population z (fixed key)
    roll      [T, 3, S, H]       rollout noise rows: acc, steer, const
                                 (S = num_reduced; for mmd_opt S = n rows)
    resample  [T, B-5, 8]        CEM resample z
    beta_z0   [100, M+1]         beta-CEM initial z (mmd_opt only)
    beta_z    [20, 89, M+1]      beta-CEM resample z (mmd_opt only)
    idx_mpc, seed                keys of the (always internal) Beta streams
    """

    def __init__(self, pop0, roll, resample, beta_z0=None, beta_z=None, idx_mpc=0, seed=0):
        self.pop0 = np.ascontiguousarray(pop0, dtype=F32)
        self.roll = np.ascontiguousarray(roll, dtype=F32)
        self.resample = np.ascontiguousarray(resample, dtype=F32)
        self.beta_z0 = None if beta_z0 is None else np.ascontiguousarray(beta_z0, dtype=F32)
        self.beta_z = None if beta_z is None else np.ascontiguousarray(beta_z, dtype=F32)
        self.idx_mpc = int(idx_mpc)
        self.seed = int(seed)

    @staticmethod
    def shapes(prob, with_beta_cem):
        B, S, H, T = prob.num_batch, prob.num_reduced, prob.num_prime, prob.maxiter_cem
        M1 = prob.num_mother + 1
        K, E, Tb = prob.num_samples_cem, prob.num_ellite_beta, prob.maxiter_beta_cem
        d = {"pop0": (B, 8), "roll": (T, 3, S, H), "resample": (T, B - 5, 8)}
        if with_beta_cem:
            d["beta_z0"] = (K, M1)
            d["beta_z"] = (Tb, K - E, M1)
        return d

    @classmethod
    def random(cls, prob, rng, idx_mpc=0, seed=0, with_beta_cem=True):
        """External draws from a NumPy Generator (test fixtures)."""
        sh = cls.shapes(prob, with_beta_cem)
        arrs = {k: rng.standard_normal(v).astype(F32) for k, v in sh.items()}
        return cls(idx_mpc=idx_mpc, seed=seed, **arrs)

    @classmethod
    def philox(cls, prob, idx_mpc, seed=0, with_beta_cem=True):
        """The internal streams (what the library generates when no external
        draws are passed)."""
        sh = cls.shapes(prob, with_beta_cem)
        fk = fixed_key(seed)
        pop0 = philox_normals(fk, STREAM_POP0, 0, int(np.prod(sh["pop0"]))).reshape(sh["pop0"])
        T = prob.maxiter_cem
        roll = np.empty(sh["roll"], dtype=F32)
        res = np.empty(sh["resample"], dtype=F32)
        n_roll = int(np.prod(sh["roll"][2:]))
        n_res = int(np.prod(sh["resample"][1:]))
        for t in range(T):
            ik = iteration_key(idx_mpc, t, seed)
            for s in range(3):
                roll[t, s] = philox_normals(ik, STREAM_ROLL_ACC + s, 0, n_roll).reshape(sh["roll"][2:])
            res[t] = philox_normals(ik, STREAM_RESAMPLE, 0, n_res).reshape(sh["resample"][1:])
        kw = {}
        if with_beta_cem:
            kw["beta_z0"] = philox_normals(fk, STREAM_BETA_Z0, 0, int(np.prod(sh["beta_z0"]))).reshape(sh["beta_z0"])
            bz = np.empty(sh["beta_z"], dtype=F32)
            n_bz = int(np.prod(sh["beta_z"][1:]))
            for t in range(sh["beta_z"][0]):
                bz[t] = philox_normals(fk, STREAM_BETA_Z, t, n_bz).reshape(sh["beta_z"][1:])
            kw["beta_z"] = bz
        return cls(pop0, roll, res, idx_mpc=idx_mpc, seed=seed, **kw)
