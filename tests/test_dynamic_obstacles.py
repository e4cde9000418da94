"""Dynamic-obstacle generator: the library's host QP
(mpcmmd_obs_dynamic_traj) against the oracle's LU restatement of
synthetic_dynamic_obs/obs_data_generate_dynamic.py:73-109, plus the known
answers of the QP and the drop-in generator class.  Host code only: CPU."""
import numpy as np
import pytest

from oracle.dynamic import obs_guess


@pytest.fixture(scope="module")
def nat():
    from optimizer import _native
    return _native


def test_matches_oracle(nat):
    rs = np.random.RandomState(3)
    O = 20
    x0 = rs.choice(np.linspace(15, 45, 30), O, replace=False)
    vx0 = rs.choice(np.linspace(0.5, 5, 20), O, replace=False)
    y0 = np.full(O, 1.75)
    vy0 = rs.uniform(-0.5, 0.5, O)
    v_des = 6.0 + 0.1 * rs.standard_normal(O)
    got = nat.obs_dynamic_traj(x0, y0, vx0, vy0, v_des)
    ref = obs_guess(x0, y0, vx0, vy0, v_des)
    for g, r in zip(got, ref):
        # fp32 outputs; KKT condition ~1e5 -> tolerance 1e-5 relative
        np.testing.assert_allclose(g, r, rtol=1e-5, atol=1e-4)


def test_known_answers(nat):
    # boundary equalities: x(0) = x0, y(0) = y0
    x, y = nat.obs_dynamic_traj([20.0, 30.0], [1.75, 1.75], [2.0, 4.0], [0.0, 0.0], [6.0, 6.0])
    np.testing.assert_allclose(x[:, 0], [20.0, 30.0], atol=1e-4)
    np.testing.assert_allclose(y[:, 0], [1.75, 1.75], atol=1e-5)
    # lane change -1.75 <- 1.75: converges to the target lane, x monotone
    assert abs(y[0, -1] + 1.75) < 0.1 and np.all(np.diff(x[0]) > 0)
    # already on target: constant speed at v_des in lane y_des is the exact optimum
    t = np.linspace(0, 15, 100)
    x, y = nat.obs_dynamic_traj([10.0], [-1.75], [6.0], [0.0], [6.0])
    np.testing.assert_allclose(x[0], 10.0 + 6.0 * t, rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(y[0], -1.75, atol=1e-4)


def test_generator_class(nat):
    from optimizer.obs_data_generate_dynamic import obs_data, dynamic_obstacles
    gen = obs_data(1)
    bx, by = gen.compute_boundary_vec(20.0, 3.0, 0.0, 1.75, 0.0, 0.0)
    assert bx.shape == (1, 3) and by.shape == (1, 4) and by[0, 3] == 0
    x, y = gen.compute_obs_guess(bx, by, -1.75 * np.ones(1), 5)
    v = gen.sampling_param(5)
    rx, ry = obs_guess([20.0], [1.75], [3.0], [0.0], v)
    np.testing.assert_allclose(x, rx, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(y, ry, rtol=1e-5, atol=1e-4)
    cfg = dynamic_obstacles(7, 20)     # BASELINE configs[3]: num_obs = 20 (pool extended)
    assert cfg["x_traj"].shape == (20, 100) and len(set(cfg["vx"])) == 20
    assert len(set(cfg["x"])) == 20 and 1 <= cfg["idx_mpc"] < 10000
    with pytest.raises(ValueError):
        gen.compute_obs_guess(np.array([[0.0, 1.0, 0.5]]), by, -1.75, 1)
