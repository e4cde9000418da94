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
