"""Monte-Carlo validation (SURVEY §8f-2, S/validation.py:134-171): the
oracle's known answers on CPU, and the GPU kernel (mpcmmd_validate) against
the oracle -- injected draws (bit-exact counts) and the internal Philox
streams (gaussian and Beta)."""
import numpy as np
import pytest

from oracle import validation as V
from oracle.problem import Problem

H, O, R = 30, 10, 1000


def _trajectory(rs, y0):
    """Saved-optimum-like Bernstein coefficients: accelerating, drifting
    laterally (nonzero acc / steer so the noise matters)."""
    j = np.arange(11) / 10.0
    cx = 15.0 * (5.0 * j + 3.0 * j * j) + rs.normal(0, 0.2, 11)
    cy = y0 + rs.normal(0, 0.4, 11)
    cy[:3] = y0
    return cx, cy


def _case(seed, K=6):
    rs = np.random.RandomState(seed)
    prob = Problem(10, O, 0.1, H, "gaussian", 0.05, 0.01)
    cx, cy, st, xo, yo = [], [], [], [], []
    for k in range(K):
        a, b = _trajectory(rs, 1.75)
        cx.append(a), cy.append(b)
        st.append([0.0, 1.75, 5.0, 0.0, 0.0, 0.0])
        # obstacles spread along the lane so some rollouts graze them
        xs = rs.choice(np.arange(15, 80, 5.0), O, replace=False)
        ys = rs.choice([-1.75, 1.75, 3.5], O)
        xo.append(np.repeat(xs[:, None], 100, 1).astype(np.float32))
        yo.append(np.repeat(ys[:, None], 100, 1).astype(np.float32))
    return prob, np.array(cx), np.array(cy), np.array(st), np.array(xo), np.array(yo)


def test_oracle_known_answers():
    prob = Problem(10, 1, 0.1, H, "gaussian", 0.0, 0.0)
    cx = 5.0 * 15.0 * np.arange(11) / 10.0     # x = 5 t, straight
    cy = np.full(11, 1.75)
    acc, steer = V.controls(prob, cx, cy)
    np.testing.assert_allclose(acc[:H], 0.0, atol=1e-3)   # fp32 basis
    np.testing.assert_allclose(steer[:H], 0.0, atol=1e-6)
    z = np.zeros((3, 50, H))
    st = [0.0, 1.75, 5.0, 0.0, 0.0, 0.0]
    on = np.full((1, 100), 10.0, np.float32), np.full((1, 100), 1.75, np.float32)
    far = np.full((1, 100), 500.0, np.float32), np.full((1, 100), -1.75, np.float32)
    assert V.compute_stats(prob, cx, cy, st, *on, "gaussian", 0.1, 0.0, 0.0, z)[0] == 50
    assert V.compute_stats(prob, cx, cy, st, *far, "gaussian", 0.1, 0.0, 0.0, z) == (0, 0)
    cy3 = np.full(11, 3.0)                     # above y_ub = 2.25 for every rollout
    assert V.compute_stats(prob, cx, cy3, [0, 3.0, 5.0, 0, 0, 0], *far, "gaussian", 0.1, 0.0, 0.0, z)[1] == 50


@pytest.mark.gpu
def test_gpu_injected_draws_exact():
    from optimizer import _native
    prob, cx, cy, st, xo, yo = _case(0)
    K = cx.shape[0]
    rs = np.random.RandomState(1)
    draws = rs.standard_normal((K, 3, R, H))
    got_c, got_l = _native.validate(cx, cy, st, xo, yo, np.arange(K), H, "gaussian", 0.1, 0.05, 0.01,
                                    num_rollouts=R, draws=draws)
    ref = [V.compute_stats(prob, cx[k], cy[k], st[k], xo[k], yo[k], "gaussian", 0.1, 0.05, 0.01, draws[k])
           for k in range(K)]
    assert np.any(got_c > 0) and np.any(got_c < R), got_c   # the case exercises partial collisions
    assert got_c.tolist() == [r[0] for r in ref]
    assert got_l.tolist() == [r[1] for r in ref]


@pytest.mark.gpu
@pytest.mark.parametrize("noise,level", [("gaussian", 0.1), ("beta", 0.3)])
def test_gpu_internal_streams(noise, level):
    """Library Philox streams vs the oracle's restatement of them: counts may
    differ only through ulp-level differences of fp64 transcendentals at a
    boundary -- within 1% of the rollouts."""
    from optimizer import _native
    prob, cx, cy, st, xo, yo = _case(2, K=4)
    K = cx.shape[0]
    keys = np.array([11, 12, 13, 14])
    got_c, got_l = _native.validate(cx, cy, st, xo, yo, keys, H, noise, level, 0.05, 0.01, num_rollouts=R,
                                    seed=7)
    for k in range(K):
        acc, steer = V.controls(prob, cx[k], cy[k])
        d = V.draws_philox(prob, acc, steer, noise, R, H, keys[k], seed=7)
        rc, rl = V.compute_stats(prob, cx[k], cy[k], st[k], xo[k], yo[k], noise, level, 0.05, 0.01, d)
        assert abs(int(got_c[k]) - rc) <= R // 100, (k, got_c[k], rc)
        assert abs(int(got_l[k]) - rl) <= R // 100, (k, got_l[k], rl)
