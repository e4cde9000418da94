"""k_select's preparation -- the stable argsort of the projection residuals
(cem.py:233-248) and compute_cost's eleven norms (cem_helper.py:232-262) --
runs in leading workgroups of the risk launch where that is k_risk_baseline
(cost.hpp: select_prep), or, with MPCMMD_SELECT_PREP=0 (and on every other
path), in k_select (sort.hpp's merge sort) and k_front.  Both must give the
same bits: every iteration's residual order, obstacle / cost elites and the
result rows of whole solves, for batches that take the one-key-per-thread
merge sort (B <= 1024) and the LDS bitonic network (B > 1024)."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


def _solve(native, monkeypatch, prep, cost, noise, B, S):
    monkeypatch.setenv("MPCMMD_SELECT_PREP", prep)  # read when the handle is created
    w = dict(bench.WORKLOADS["cvar"], cost=cost, noise=noise, num_batch=B, num_reduced=S)
    inst = bench.make_workload(w, 0)
    cfg = native.make_config(w["num_reduced"], w["num_obs"], w["level"], w["num_prime"], w["noise"], 0.0, 0.0,
                             num_batch=B, maxiter_cem=6)
    h = native.Handle(cfg)
    try:
        h.begin(cost, inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"], inst["v_des"])
        h.iterate(0, 6)
        h.sync()
        out = {k: h.read(k, np.int32) for k in ("tr_proj", "tr_obs", "tr_cem")}
        out["results"] = h.read("results")
        out["cnorm"] = h.read("cnorm", np.float64)
    finally:
        h.close()
    return out


@pytest.mark.parametrize("cost,noise,B,S", [("cvar", "beta", 256, 100), ("saa", "gaussian", 1024, 64),
                                            ("mmd_random", "gaussian", 2048, 32)])
def test_select_prep_same_bits(native, monkeypatch, cost, noise, B, S):
    a = _solve(native, monkeypatch, "1", cost, noise, B, S)
    b = _solve(native, monkeypatch, "0", cost, noise, B, S)
    for k in ("tr_proj", "tr_obs", "tr_cem"):
        assert np.array_equal(a[k], b[k]), f"{k} differs between the two select preparations"
    assert np.array_equal(a["results"], b["results"], equal_nan=True), "results differ"
    assert np.array_equal(a["cnorm"], b["cnorm"], equal_nan=True), "cost norms differ"


@pytest.mark.parametrize("B", [100, 300, 520, 600, 777, 1000])
def test_residual_argsort_ragged_batches(native, monkeypatch, B):
    """k_select's one-key-per-thread merge sort (sort.hpp: merge_sort_reg)
    for batches that are not a power of two, where padding keys fill both runs
    of a merge pair (B = 300: the runs [256, 320) and [320, 384); B = 520 ..
    1000 in the 1024-key sort): the permutation written to tr_proj must be
    jnp.argsort's (stable, -0 == +0, NaN last; cem.py:233-248) on residuals
    with many ties, both zeros and NaNs."""
    monkeypatch.setenv("MPCMMD_SELECT_PREP", "0")   # the sort runs in k_select (stage 3)
    w = dict(bench.WORKLOADS["cvar"], num_batch=B, num_reduced=16)
    inst = bench.make_workload(w, 0)
    cfg = native.make_config(16, w["num_obs"], w["level"], w["num_prime"], "gaussian", 0.0, 0.0,
                             num_batch=B, maxiter_cem=2)
    h = native.Handle(cfg)
    try:
        assert h.info("select_prep") == 0
        h.begin("cvar", inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"],
                inst["v_des"])
        rng = np.random.default_rng(B)
        for t in range(2):
            h.run_stage(0, t)
            h.run_stage(1, t)
            h.run_stage(2, t)
            r = rng.choice(np.array([0.0, -0.0, 1e-6, 2.5e-6, 3.0, np.nan, 1e-30], np.float32), size=B)
            r = np.where(rng.random(B) < 0.5, r, rng.random(B).astype(np.float32))
            h.write("res_norm", r.astype(np.float32))
            h.run_stage(3, t)
            h.sync()
            got = h.read("tr_proj", np.int32)[t * B:(t + 1) * B]
            want = np.argsort(r, kind="stable")
            assert np.array_equal(got, want), f"B={B} t={t}: first difference at {np.argmax(got != want)}"
    finally:
        h.close()


def test_stage3_needs_stage2_with_select_prep(native, monkeypatch):
    """With the select preparation in the risk launch (the default for cvar),
    stage 3 right after stage 1 would read stale residual ranks and cost norms:
    the library refuses it instead of running on them."""
    monkeypatch.setenv("MPCMMD_SELECT_PREP", "1")
    w = dict(bench.WORKLOADS["cvar"], num_batch=128, num_reduced=16)
    inst = bench.make_workload(w, 0)
    cfg = native.make_config(16, w["num_obs"], w["level"], w["num_prime"], "gaussian", 0.0, 0.0,
                             num_batch=128, maxiter_cem=2)
    h = native.Handle(cfg)
    try:
        assert h.info("select_prep") == 1
        h.begin("cvar", inst["idx_mpc"], inst["init"], inst["mean"], inst["cov"], inst["xo"], inst["yo"],
                inst["v_des"])
        h.run_stage(0, 0)
        h.run_stage(1, 0)
        with pytest.raises(native.NativeError, match="stage 3 needs stage 2"):
            h.run_stage(3, 0)
        h.run_stage(2, 0)
        h.run_stage(3, 0)   # now in order
        h.sync()
    finally:
        h.close()
