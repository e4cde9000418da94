"""Pin the oracle (CPU restatement) against the reference's golden vectors and
known-answer tests.  CPU only.

* Bernstein basis: tests/golden/bernstein_ref.npz, produced by importing the
  reference's own S/bernstein_coeff_order10_arbitinterval.py (the only
  reference module importable here; script committed beside it).
* Philox4x32-10: the Random123 known-answer vectors.
* Derived KATs of the reference semantics: partition of unity,
  KKT equalities, MMD floor -1000 (kernel_computation.py:82-87), f_bar = 1 at
  an obstacle centre (costs.py:50-60), CVaR of constants, quantile weights.
"""
import os

import numpy as np
import pytest

import oracle
from oracle import beta_cem as bc
from oracle import costs as C
from oracle import helper as H
from oracle.problem import Problem, bernstein_order10
from oracle.projection import unwrap
from oracle.rng import beta_draws, philox4x32_10, philox_normals

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "bernstein_ref.npz"))
F32 = np.float32


def ulps(a, b):
    """fp32 ulp distance (monotone integer map of the bit patterns)."""
    def key(x):
        i = np.asarray(x, F32).view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    return np.abs(key(a) - key(b))


@pytest.mark.parametrize("grid", ["grid100", "h8", "h20", "h30", "h50", "h60"])
def test_bernstein_matches_reference(grid):
    t = GOLD[f"{grid}_t"]
    P, Pd, Pdd = bernstein_order10(t[0], t[-1], t)
    for name, mine in (("P", P), ("Pdot", Pd), ("Pddot", Pdd)):
        ref = GOLD[f"{grid}_{name}"]
        scale = np.abs(ref).max()
        np.testing.assert_allclose(mine, ref, rtol=0, atol=1e-12 * scale, err_msg=name)
        # after the fp32 cast the reference applies (cem.py:48): bit-equal,
        # except entries whose exact value is 0 where the reference's expanded
        # polynomials leave cancellation noise (|ref| ~ 3e-17, 4 entries of
        # the 100-point Pddot); those are covered by the absolute check above
        d = ulps(mine.astype(F32), ref.astype(F32))
        sig = np.abs(ref) > 1e-12 * scale
        assert d[sig].max() == 0, f"{grid} {name}: {d[sig].max()} ulp"
        assert (~sig & (d > 0)).sum() <= 4


def test_problem_basis_is_fp32_of_reference():
    p = Problem(10, 3, 0.1, 30, "gaussian", 0.0, 0.0)
    assert np.array_equal(p.P, GOLD["grid100_P"].astype(F32))
    assert np.array_equal(p.Pdot, GOLD["grid100_Pdot"].astype(F32))
    assert np.array_equal(p.P_prime, GOLD["h30_P"].astype(F32))


def test_partition_of_unity_and_endpoints():
    t = np.linspace(0, 15, 100)
    P, Pd, Pdd = bernstein_order10(0.0, 15.0, t)
    np.testing.assert_allclose(P.sum(1), 1.0, atol=1e-14)
    np.testing.assert_allclose(Pd.sum(1), 0.0, atol=1e-12)
    np.testing.assert_allclose(Pdd.sum(1), 0.0, atol=1e-11)
    assert P[0, 0] == 1.0 and P[-1, -1] == 1.0


@pytest.mark.parametrize("variant", ["static", "dynamic"])
def test_kkt_inverses(variant):
    p = Problem(10, 3, 0.1, 20, "gaussian", 0.0, 0.0, variant=variant)
    for K, Ki in ((p.guess_kkt_x, p.guess_kinv_x), (p.guess_kkt_y, p.guess_kinv_y),
                  (p.proj_kkt_x, p.proj_kinv_x), (p.proj_kkt_y, p.proj_kinv_y)):
        np.testing.assert_allclose(K @ Ki, np.eye(K.shape[0]), atol=1e-6)
    # the projection solution satisfies the boundary equalities exactly (KKT rows)
    b = np.array([0.0, 5.0, 0.0])
    c = p.proj_kinv_x[:11, :11] @ np.random.default_rng(0).normal(size=11) + p.kkt_rhs_const(p.proj_kinv_x, b)
    np.testing.assert_allclose(p.A_eq_x @ c, b, atol=1e-6)


def test_fit_reproduces_polynomials():
    """compute_coeff (cem_helper.py:553-564) is a ridge fit: a trajectory that
    is exactly P' c is recovered up to the 0.05 ridge shrinkage."""
    p = Problem(10, 3, 0.1, 30, "gaussian", 0.0, 0.0)
    c = np.random.default_rng(1).normal(size=(4, 11))
    x = c @ p.P_prime.astype(np.float64).T
    cx, _ = H.compute_coeff(p, x, x)
    G = p.P_prime.astype(np.float64).T @ p.P_prime.astype(np.float64)
    expect = np.linalg.solve(G + 0.05 * np.eye(11), G @ c.T).T
    np.testing.assert_allclose(cx, expect, rtol=1e-4, atol=1e-4)


def test_philox_known_answers():
    """Random123 KAT vectors for philox4x32_10."""
    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, want in kat:
        got = tuple(int(w) for w in philox4x32_10(ctr, key))
        assert got == want, (ctr, [hex(g) for g in got])


def test_normals_and_beta_statistics():
    z = philox_normals((5, 0), 0, 0, 200000).astype(np.float64)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    n = 40000
    elem = np.arange(n, dtype=np.uint64)
    b = beta_draws(np.full(n, 2.0), np.full(n, 5.0), (9, 0), 4, 5, elem)
    assert abs(b.mean() - 2 / 7) < 0.005                     # Beta(2, 5) mean
    assert abs(b.var() - 10 / (49 * 8)) < 0.003              # ab / ((a+b)^2 (a+b+1))
    # alpha, beta -> 0+ (|acc| == 0): the Beta(0, 0) limit is Bernoulli on {0, 1}
    b0 = beta_draws(np.zeros(1000), np.zeros(1000), (9, 0), 4, 5, np.arange(1000, dtype=np.uint64))
    assert set(np.unique(b0)) <= {0.0, 1.0}


def test_sort_key_order():
    x = np.array([np.nan, 1.0, -0.0, 0.0, -1.0, np.inf, -np.inf], F32)
    order = H.argsort_stable(x)
    assert list(order) == [6, 4, 2, 3, 1, 5, 0]              # -0 == +0 (stable), NaN last


def test_select_top_is_argsort_tail():
    rng = np.random.default_rng(2)
    s = rng.normal(size=(7, 50)).astype(F32)
    s[0, 3] = s[0, 9] = 5.0                                  # exact tie: larger index ranks later
    top = bc.select_top(s, 49, 5)
    for k in range(7):
        ref = np.argsort(H.sort_key(np.abs(s[k, :49])), kind="stable")[-5:]
        assert np.array_equal(top[k], ref)
    assert list(top[0][-2:]) == [3, 9]


def test_unwrap_matches_numpy():
    rng = np.random.default_rng(3)
    p = np.cumsum(rng.normal(scale=1.5, size=(4, 100)), axis=1)
    p = (np.mod(p + np.pi, 2 * np.pi) - np.pi).astype(F32)
    np.testing.assert_allclose(unwrap(p), np.unwrap(p.astype(np.float64)), atol=2e-4)


def test_fbar_center_and_mmd_floor():
    p = Problem(10, 1, 0.1, 5, "gaussian", 0.0, 0.0)
    x = np.full((1, 5), 40.0, F32)
    y = np.full((1, 5), 1.75, F32)
    cb = C.compute_f_bar_max(p, x, y, np.full((1, 5), 40.0, F32), np.full((1, 5), 1.75, F32))
    assert cb[0] == 1.0
    # MMD of a collision-free sample set against the Dirac at 0: -ker_wt for any
    # weights summing to one (K_bb dropped, kernel_computation.py:82-87)
    beta = np.full((1, 10), F32(0.1))
    assert C.mmd(p, beta, np.zeros((1, 10), F32), np.array([0.5], F32))[0] == np.float32(-1000.0)
    w = np.random.default_rng(4).dirichlet(np.ones(10))[None].astype(F32)
    assert abs(C.mmd(p, w, np.zeros((1, 10), F32), np.array([0.5], F32))[0] + 1000.0) < 1e-3


def test_cvar_and_quantile():
    p = Problem(10, 1, 0.1, 5, "gaussian", 0.0, 0.0)
    assert C.cvar(p, np.full((1, 500), F32(0.25)))[0] == F32(0.25)
    x = np.random.default_rng(5).random((3, 500)).astype(F32)
    np.testing.assert_allclose(C.quantile_linear(x, 0.98), np.quantile(x, 0.98, axis=1), rtol=1e-6)
    v = C.quantile_linear(x, 0.98)
    ref = np.array([x[i][x[i] >= v[i]].astype(np.float64).mean() for i in range(3)])
    np.testing.assert_allclose(C.cvar(p, x), ref, rtol=1e-6)
    assert C.saa(p, np.array([[0, 0.5, 0, 1]], F32))[0] == F32(0.5)


def test_rollout_straight_line():
    """Zero steer, zero acceleration: constant-speed straight line."""
    p = Problem(4, 1, 0.1, 10, "gaussian", 0.0, 0.0)
    st0 = np.array([0.0, 1.75, 5.0, 0.0, 0.0], F32)
    x, y = H.rollout(p, np.zeros((1, 10), F32), np.zeros((1, 10), F32), st0)
    np.testing.assert_allclose(x[0], 0.75 * np.arange(10), rtol=1e-6)
    assert np.all(y == F32(1.75))


def test_draw_shapes_and_philox_determinism():
    p = Problem(5, 2, 0.1, 10, "gaussian", 0.0, 0.0, num_batch=32)
    d1 = oracle.Draws.philox(p, 17, seed=3)
    d2 = oracle.Draws.philox(p, 17, seed=3)
    for k, shp in oracle.Draws.shapes(p, True).items():
        a = getattr(d1, k)
        assert a.shape == shp and np.array_equal(a, getattr(d2, k))
