"""k_bmoment_rows (a distance row per 16-lane DPP row, the default) against
k_bmoment (a wave per row, MPCMMD_MOM_ROWS=0) and against NumPy: the series
records of every distance row (kernel_computation.py:33-39 row sums through
the moments P_k = sum_j t_j^k, t_j = D[r][j] / R - 1, R = max_j D[r][j] / 2)
and the first beta-iteration's direct row sums (the pairs whose a = R / sigma
exceeds the series' range, compute_beta.py:75).  The two kernels sum in
different orders, so the moments and direct sums agree to fp32 rounding; the
row maximum R, the record's M slot and the set of direct pairs are exact."""
import numpy as np
import pytest

import oracle

from parity import DEFAULT_COV, DEFAULT_INIT, DEFAULT_MEAN, make_pair

pytestmark = pytest.mark.gpu

F32, F64 = np.float32, np.float64


def _moments(native, monkeypatch, rows, n, B, H, O, level=None):
    monkeypatch.setenv("MPCMMD_MOM_ROWS", rows)
    ora, nat, xo, yo = make_pair(native, "mmd_opt", n=n, O=O, H=H, B=B, T=2, level=level)
    # explicit noise tables (the mother rows' noise), as test_gpu_parity_mmdopt
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(1), idx_mpc=11, seed=0, with_beta_cem=True)
    nat.begin("mmd_opt", 11, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
    nat.run_stage(1, 0)
    nat.sync()
    brow0 = np.full(nat.read("brow").shape, np.nan, F32)
    nat.write("brow", brow0)  # sentinel: entries the moment kernel does not write stay NaN
    nat.run_stage(4, 0)
    nat.sync()
    out = {k: nat.read(k).copy() for k in ("bmom", "brow", "bdist")}
    nat.close()
    return out


@pytest.mark.parametrize("n,B,H,O,level", [(6, 24, 12, 3, None), (10, 20, 30, 4, None), (22, 21, 30, 10, None),
                                           (32, 20, 20, 4, None), (22, 20, 30, 4, 30.0)])
def test_moment_rows(native, monkeypatch, n, B, H, O, level):
    M = n * n
    Md = (M + 255) & ~255
    old = _moments(native, monkeypatch, "0", n, B, H, O, level)
    new = _moments(native, monkeypatch, "1", n, B, H, O, level)
    assert np.array_equal(old["bdist"], new["bdist"])
    D = new["bdist"].reshape(B * M, Md)[:, :M].astype(F64)
    assert D.max() > 0 and (D == 0).mean() < 1.0 / M + 0.01, "degenerate mother rows"  # zeros: the diagonal
    ro = old["bmom"].reshape(B * M, 16)
    rn = new["bmom"].reshape(B * M, 16)
    # exact: the M slot, R (a maximum) and the unused slots
    assert np.array_equal(rn[:, 0], ro[:, 0]) and np.all(rn[:, 0] == M)
    R = (F32(0.5) * D.max(axis=1).astype(F32)).astype(F32)
    assert np.array_equal(rn[:, 12], R) and np.array_equal(ro[:, 12], R)
    assert np.all(rn[:, 13:] == 0) and np.all(ro[:, 13:] == 0)
    # moments: fp64 sums of the fp32 t_j powers; bound |P_k| <= M, fp32 sums of M terms
    invR = np.where(R > 0, F32(1) / np.where(R > 0, R, F32(1)), F32(0)).astype(F32)
    t = (D.astype(F32) * invR[:, None] - F32(1)).astype(F64)  # fma(d, 1/R, -1) up to one rounding
    tol = 4e-7 * M
    for k in range(1, 12):
        ref = (t ** k).sum(axis=1)
        for name, rec in (("rows", rn), ("wave", ro)):
            err = np.abs(rec[:, k].astype(F64) - ref)
            assert err.max() <= tol * k, f"P_{k} ({name}): {err.max()} > {tol * k}"
        d = np.abs(rn[:, k].astype(F64) - ro[:, k].astype(F64))
        assert d.max() <= tol, f"P_{k}: rows vs wave {d.max()}"
    # the first-iteration direct sums: the same pairs written, values to fp32 rounding
    wo, wn = ~np.isnan(old["brow"]), ~np.isnan(new["brow"])
    assert np.array_equal(wo, wn), "different direct pairs"
    if wo.any():
        a, b = new["brow"][wn].astype(F64), old["brow"][wo].astype(F64)
        assert np.all(np.abs(a - b) <= 2e-5 * np.abs(b)), "direct sums"
    print(f"n={n}: {int((~np.isnan(new['brow'])).sum())} direct first-iteration sums")


@pytest.mark.parametrize("n,B", [(10, 20), (22, 21)])
def test_moment_rows_direct_sums(native, monkeypatch, n, B):
    """Every first-iteration pair sent to the direct sums (MPCMMD_MOM_AMAX=0:
    the direct test is a > 0; at the BASELINE shapes a <= 1 for nearly every
    pair, so the default tests write none): both kernels write the same pairs,
    each sum_j exp(-D[r][j] / sigma) to fp32 rounding of NumPy's."""
    monkeypatch.setenv("MPCMMD_MOM_AMAX", "0")
    H, O, M = 30, 4, n * n
    Md = (M + 255) & ~255
    old = _moments(native, monkeypatch, "0", n, B, H, O)
    new = _moments(native, monkeypatch, "1", n, B, H, O)
    wo, wn = ~np.isnan(old["brow"]), ~np.isnan(new["brow"])
    assert np.array_equal(wo, wn) and wn.all(), "every (sample, row) pair written by both"
    a, b = new["brow"].astype(F64), old["brow"].astype(F64)
    assert np.all(np.abs(a - b) <= 2e-5 * np.abs(b)), "direct sums"
