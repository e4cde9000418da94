"""k_bcem_small -- the 20 beta-iterations of a candidate in one workgroup, the
small-batch path (num_batch <= 512, num_reduced <= 16: the reference's
num_batch = 100, BASELINE configs[4]) -- against the per-iteration kernels it
replaces (MPCMMD_FUSED=0): every phase is the same device code, so a solve
must give the same bits: per outer iteration the beta-CEM outputs (beta,
sigma, res_beta, the elite-cost trace), the obstacle / lane costs, the elite
index sets, and the returned result."""
import numpy as np
import pytest

from parity import DEFAULT_COV, DEFAULT_INIT, DEFAULT_MEAN, make_pair

pytestmark = pytest.mark.gpu


def _run(native, monkeypatch, fused, cost, n, B, H, O, T, xo=None, yo=None, carla=None, keys=()):
    monkeypatch.setenv("MPCMMD_FUSED", "1" if fused else "0")
    if carla is None:
        ora, nat, xo_, yo_ = make_pair(native, cost, n=n, O=O, H=H, B=B, T=T)
        xo, yo = (xo_, yo_) if xo is None else (xo, yo)
        nat.begin(cost, 7, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0)
    else:
        init, xo, yo, path, variant = carla
        nat = native.Handle(native.make_config(n, O, 0.1, H, "gaussian", 0.0, 0.0, num_batch=B, maxiter_cem=T,
                                               variant=variant))
        mean = np.array([10.0] * 4 + [0.0] * 4, np.float32)
        nat.carla_begin(cost, 7, init, mean, DEFAULT_COV, xo, yo, 10.0, path)
    out = []
    for t in range(T):
        nat.iterate(t, 1)
        nat.sync()
        out.append({k: nat.read(k).copy() for k in ("beta", "sigma", "res_beta", "btrace", "obs_cost", "lane_cost")
                    + tuple(keys)})
        out[-1]["tr"] = (nat.read("tr_proj", np.int32).copy(), nat.read("tr_obs", np.int32).copy(),
                         nat.read("tr_cem", np.int32).copy())
    res = nat.finish()
    nat.close()
    return out, res


@pytest.mark.parametrize("n,B,H,O", [(6, 32, 10, 3), (10, 100, 30, 4), (16, 100, 30, 10)])
def test_fused_bits_static(native, monkeypatch, n, B, H, O):
    T = 3
    ref, rr = _run(native, monkeypatch, False, "mmd_opt", n, B, H, O, T)
    got, rg = _run(native, monkeypatch, True, "mmd_opt", n, B, H, O, T)
    for t in range(T):
        for k in ref[t]:
            if k == "tr":
                assert all(np.array_equal(a, b) for a, b in zip(got[t][k], ref[t][k])), f"iteration {t}: elites"
            else:
                assert np.array_equal(got[t][k], ref[t][k], equal_nan=True), f"iteration {t}: {k} differs"
    for k, v in rr.items():
        assert np.array_equal(np.asarray(rg[k]), np.asarray(v), equal_nan=True), k


def test_fused_bits_carla(native, monkeypatch):
    from test_gpu_carla import _tick
    init, xo, yo, path = _tick(60, 3, 60)
    carla = (init, xo, yo, path, "carla_town05")
    T = 3
    ref, rr = _run(native, monkeypatch, False, "mmd_opt", 10, 100, 60, 3, T, carla=carla)
    got, rg = _run(native, monkeypatch, True, "mmd_opt", 10, 100, 60, 3, T, carla=carla)
    for t in range(T):
        for k in ref[t]:
            if k == "tr":
                assert all(np.array_equal(a, b) for a, b in zip(got[t][k], ref[t][k])), f"iteration {t}: elites"
            else:
                assert np.array_equal(got[t][k], ref[t][k], equal_nan=True), f"iteration {t}: {k} differs"
    for k in ("cx", "cy", "steering", "v_best", "mean_param"):
        assert np.array_equal(rg[k], rr[k]), k


@pytest.mark.parametrize("case", ["static-22", "carla-22", "static-50"])
def test_direct_pairs_same_bits(native, monkeypatch, case):
    """The direct row sums from k_bkernel's pair list (a wave per 8 listed
    pairs; MPCMMD_DIR_PAIRS=1, the default: k_bdirect_pairs on the
    per-iteration kernels of launches <= 256 candidates) against bdirect_body (pairs counting-sorted by mother row in
    LDS): the same per-lane terms and the same reduction tree for every slot,
    so the direct row sums (brow) and every output carry the same bits."""
    kind, n = case.split("-")[:2]
    fused = case.endswith("fused")
    n = int(n)
    T = 2
    carla = None
    B, H, O = (100, 20, 4) if n == 50 else (100, 30, 10)
    if kind == "carla":
        from test_gpu_carla import _tick
        init, xo, yo, path = _tick(60, 3, 60)
        carla = (init, xo, yo, path, "carla_town05")
        H, O = 60, 3
    runs = []
    for pairs in ("0", "1"):
        monkeypatch.setenv("MPCMMD_DIR_PAIRS", pairs)
        runs.append(_run(native, monkeypatch, fused, "mmd_opt", n, B, H, O, T, carla=carla, keys=("brow",)))
    (ref, rr), (got, rg) = runs
    for t in range(T):
        for k in ref[t]:
            if k == "tr":
                assert all(np.array_equal(a, b) for a, b in zip(got[t][k], ref[t][k])), f"iteration {t}: elites"
            else:
                assert np.array_equal(got[t][k], ref[t][k], equal_nan=True), f"iteration {t}: {k} differs"
    for k in ("cx", "cy"):
        assert np.array_equal(np.asarray(rg[k]), np.asarray(rr[k])), k
