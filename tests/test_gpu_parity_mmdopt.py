"""GPU parity of the mmd_opt path (nested beta-CEM) against the oracle.

Sub-stage lockstep (run_stage 4-8): the oracle is fed the GPU's inputs of
each sub-stage and must reproduce its outputs:
  mother    noisy rows + mother rollouts + Bernstein fit  -> ctrl_n, feat
  bsample   samples (elites of the previous iteration + mean + L z with the
            dense fp64 Cholesky of jnp.cov + 0.05 I) -> top-n |beta| rows, sigma
  bkernel   Laplace kernels, reduced QP, QP cost          -> btop, bcost
  belite    elite 11 by cost                              -> elite sample rows
  mmdfinal  reduced rollouts + MMD obs / lane             -> obs_cost, lane_cost
Selections (integer index sets) must agree exactly unless the compared keys
are a near-tie; floating outputs within tolerances stated per check.
"""
import numpy as np
import pytest

import oracle
from oracle import beta_cem as bc
from oracle import costs as C
from oracle import helper as Hh
from parity import DEFAULT_COV, DEFAULT_INIT, DEFAULT_MEAN, close, elite_equal, make_pair

pytestmark = pytest.mark.gpu

F32, F64 = np.float32, np.float64
SQRT20 = np.sqrt(20.0)


def _samples_from_elites(E, z_t, M, clip=0.01):
    """Rows 11..99 of the next samples from the 11 elite rows E [11, M+1]
    (compute_beta.py:51-68): mean, jnp.cov + 0.05 I, dense Cholesky."""
    El = E.astype(F64)
    mean64 = El.mean(axis=0)
    mean32 = mean64.astype(F32)
    D = El - mean64
    cov = D.T @ D / 10.0 + 0.05 * np.eye(M + 1)
    L = Hh.chol64(cov)
    new = (mean32.astype(F64) + z_t.astype(F64) @ L.T).astype(F32)
    new[:, M] = np.maximum(new[:, M], F32(clip))
    return new


def _check_selection(name, got, samples, M, n):
    ref = bc.select_top(samples, M, n)
    keys = np.abs(samples[:, :M]).astype(F64)
    for s in range(samples.shape[0]):
        if not np.array_equal(got[s], ref[s]):
            elite_equal(f"{name}[{s}]", got[s], ref[s], keys[s], tol=1e-6)


def _run_mother(native, n, B, H, O, noise, seed, variant="static"):
    ora, nat, xo, yo = make_pair(native, "mmd_opt", noise, n=n, O=O, H=H, B=B, T=2, acc_c=0.05, steer_c=0.01,
                                 variant=variant)
    if variant == "dynamic":   # synthetic_dynamic_obs scenario (obs_data_generate_dynamic.py, library QP)
        from optimizer.obs_data_generate_dynamic import dynamic_obstacles
        dyn = dynamic_obstacles(seed, O)
        xo, yo = dyn["x_traj"], dyn["y_traj"]
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(seed), idx_mpc=11, seed=0, with_beta_cem=True)
    nat.begin("mmd_opt", 11, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
    st = ora.init_state(DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, draws)
    nat.run_stage(1, 0)
    nat.run_stage(4, 0)
    acc = nat.read("acc").reshape(B, 100)
    steer = nat.read("steer").reshape(B, 100)
    return ora, nat, xo, yo, draws, st, acc, steer


@pytest.mark.parametrize("noise", ["gaussian", "beta"])
def test_mother_features(native, noise):
    n, B, H, O = 6, 24, 12, 3
    ora, nat, xo, yo, draws, st, acc, steer = _run_mother(native, n, B, H, O, noise, 1)
    p = ora.prob
    acc_n, steer_n = Hh.noisy_controls(p, acc[:, :H], steer[:, :H], draws, 0, n)
    ctrl = nat.read("ctrl_n").reshape(B, 2, n, H)
    frac = 0.05 if noise == "beta" else 0.0
    close("acc_n", ctrl[:, 0], acc_n, atol=1e-5, frac_ok=frac)
    close("steer_n", ctrl[:, 1], steer_n, atol=1e-6, frac_ok=frac)
    # features from the GPU's noisy rows (isolates the rollout + fit)
    acc_m, steer_m = Hh.mother_controls(ctrl[:, 0], ctrl[:, 1])
    xm, ym = Hh.rollout(p, acc_m, steer_m, st["st0"])
    cxm, cym = Hh.compute_coeff(p, xm, ym)
    feat = nat.read("feat").reshape(B, 22, n * n)
    close("feat_cx", feat[:, :11].transpose(0, 2, 1), cxm, rtol=1e-4, atol=2e-4)
    close("feat_cy", feat[:, 11:].transpose(0, 2, 1), cym, rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("n,B,H,O,variant,check,qp_iters", [
    (5, 20, 10, 3, "static", None, None), (12, 20, 10, 3, "static", [0, 7, 19], None),
    (22, 20, 10, 3, "static", [0, 19], None),
    # BASELINE configs[3] shape: dynamic obstacles, H = 50, O = 20, n = 32 (M = 1024 mother rollouts)
    (32, 20, 50, 20, "dynamic", [0, 19], None),
    # BASELINE configs[0] shape: n = 50 (M = 2500), B = 100, H = 20, O = 4 (the wave-per-QP path, n > 32);
    # the oracle QP (100 x 50 x 2500 kernel entries per sample set) is checked on three iterations
    (50, 100, 20, 4, "static", [0, 99], (0, 1, 19))])
def test_beta_cem_lockstep(native, n, B, H, O, variant, check, qp_iters):
    ora, nat, xo, yo, draws, st, acc, steer = _run_mother(native, n, B, H, O, "gaussian", 2, variant)
    p = ora.prob
    M = n * n
    M1 = M + 1
    cand = list(range(B)) if check is None else check
    feat = nat.read("feat").reshape(B, 22, M)
    Fb = {b: np.ascontiguousarray(feat[b].T) for b in cand}        # [M, 22]
    Db = {b: bc.distance_matrix(Fb[b]) for b in cand} if M > 256 else {b: None for b in cand}
    z0, z = draws.beta_z0, draws.beta_z
    samples = {}
    for b in cand:
        s0 = (SQRT20 * z0.astype(F64)).astype(F32)
        s0[:, M] = np.maximum(s0[:, M], F32(0.01))
        samples[b] = s0
    res_ref = {b: np.zeros(20, F32) for b in cand}
    qp_rel, qp_worst = 0.0, None   # largest relative difference of a QP cost on identical inputs (sizes parity.TIE_REL)
    for tb in range(20):
        nat.run_stage(5, tb)
        bsel = nat.read("bsel", np.int32).reshape(B, 100, n)
        bsig = nat.read("bsig").reshape(B, 100)
        for b in cand:
            _check_selection(f"bsel[tb={tb},b={b}]", bsel[b], samples[b], M, n)
            close(f"bsig[{tb},{b}]", bsig[b], samples[b][:, M], rtol=1e-6, atol=0)
        nat.run_stage(6, tb)
        btop = nat.read("btop").reshape(B, 100, n)
        bcost = nat.read("bcost").reshape(B, 100)
        brow = nat.read("brow", F32, (B, 100, n))
        kred = nat.read("bkred", F32, (B, 100, (n * (n - 1) // 2 + 3) // 4 * 4))[:, :, :n * (n - 1) // 2]
        lo = np.tril_indices(n, -1)   # k_bkernel's K_red layout: entry (k, kk < k) at k (k - 1) / 2 + kk
        s_lo = 11 if tb > 0 else 0    # later iterations: rows 0..10 are the carried elites
        for b in cand if qp_iters is None or tb in qp_iters else []:
            beta, cost, K_red, rowsum = bc.reduced_qp(p, Fb[b], bsel[b].astype(np.int64), bsig[b], M, Db[b])
            # K_mixed row sums (fp32 terms, fp32 partial sums on the GPU vs fp64 in the oracle) and K_red
            close(f"brow[{tb},{b}]", brow[b, s_lo:], rowsum[s_lo:], rtol=1e-5, atol=0)
            close(f"kred[{tb},{b}]", kred[b, s_lo:], K_red[s_lo:, lo[0], lo[1]], rtol=1e-6, atol=1e-7)
            close(f"btop[{tb},{b}]", btop[b], beta, rtol=1e-3, atol=1e-4)
            close(f"bcost[{tb},{b}]", bcost[b], cost, rtol=1e-4, atol=1e-4)
            # relative to the elite boundary's magnitude (the 11th smallest cost): what
            # orders the elites (parity.beta_trace measures its gaps the same way)
            scale = max(abs(float(np.sort(cost.astype(F64))[10])), 1e-6)
            rel = np.abs(bcost[b, s_lo:].astype(F64) - cost[s_lo:]) / np.maximum(np.abs(cost[s_lo:]), scale)
            if rel.max() > qp_rel:
                w = int(np.argmax(rel)) + s_lo
                qp_rel, qp_worst = float(rel.max()), (tb, b, w, float(bcost[b, w]), float(cost[w]),
                                                      float(np.sort(cost)[0]), float(bsig[b, w]))
        nat.run_stage(7, tb)
        bel = nat.read("belite").reshape(2, B, 11, M1)[(tb + 1) & 1]
        res_beta = nat.read("res_beta").reshape(B, 20)
        for b in cand:
            idx_e = Hh.argsort_stable(bcost[b])[:11]
            close(f"elites[{tb},{b}]", bel[b], samples[b][idx_e], rtol=1e-6, atol=1e-6)
            assert res_beta[b, tb] == np.min(bcost[b])
            nxt = np.vstack([bel[b], _samples_from_elites(bel[b], z[tb], M)]).astype(F32)
            if tb == 19:
                imin = bc.argmin_nan(bcost[b])
                beta_g = nat.read("beta").reshape(B, n)[b]
                sel_g = nat.read("bestsel", np.int32).reshape(B, n)[b]
                sig_g = nat.read("sigma")[b]
                assert np.array_equal(sel_g, bsel[b, imin])
                assert np.array_equal(beta_g, btop[b, imin])
                close(f"sigma_best[{b}]", sig_g, nxt[imin, M], rtol=1e-6, atol=0)
            samples[b] = nxt
    from parity import TIE_REL
    print(f"n={n}: QP costs GPU vs oracle on identical inputs agree to {qp_rel:.3g} relative (TIE_REL {TIE_REL}); "
          f"worst (beta-iteration, candidate, sample, GPU, oracle, min cost, sigma) {qp_worst}")
    assert qp_rel <= TIE_REL / 2, f"QP cost agreement {qp_rel:.3g} too coarse for the near-tie threshold {TIE_REL}"
    # final reduced-set MMD on the GPU's beta-CEM outputs
    nat.run_stage(8, 0)
    ctrl = nat.read("ctrl_n").reshape(B, 2, n, H)
    sel = nat.read("bestsel", np.int32).reshape(B, n)
    beta = nat.read("beta").reshape(B, n)
    sigma = nat.read("sigma")[:B]
    acc_m, steer_m = Hh.mother_controls(ctrl[:, 0], ctrl[:, 1])
    acc_r = np.take_along_axis(acc_m, sel[:, :, None].astype(np.int64), axis=1)
    steer_r = np.take_along_axis(steer_m, sel[:, :, None].astype(np.int64), axis=1)
    xr, yr = Hh.rollout(p, acc_r, steer_r, st["st0"])
    cb = C.compute_f_bar_max(p, xr, yr, xo[:, :H], yo[:, :H])
    obs = C.mmd(p, beta, cb, sigma)
    lane = C.mmd_lane(p, beta, sigma, yr)
    close("mmd_obs", nat.read("obs_cost")[:B], obs, rtol=1e-4, atol=1e-2)
    close("mmd_lane", nat.read("lane_cost")[:B], lane, rtol=1e-4, atol=1e-2)


def test_mmdopt_iteration_lockstep(native):
    """20 full GPU mmd_opt iterations (noise, front, mother, 20 x beta-CEM,
    final MMD, select).  Before each, the oracle is synchronised to the GPU's
    carry and runs the same iteration.  Per candidate: obs / lane costs
    within 1e-4 relative and the beta-CEM outputs (beta, sigma, res_beta)
    equal; a candidate may differ only where its beta-CEM took another path
    at a reported near-tie of QP costs.  Elite index sets (projection
    permutation, obstacle elites, cost elites) exact unless a near-tie."""
    from parity import beta_cem_trace, beta_near_tie
    from test_gpu_parity_baseline import _sync_state
    n, B, H, O, Tf = 6, 32, 10, 3, 20
    ora, nat, xo, yo = make_pair(native, "mmd_opt", "gaussian", n=n, O=O, H=H, B=B, T=Tf)
    draws = oracle.Draws.random(ora.prob, np.random.default_rng(4), idx_mpc=3, with_beta_cem=True)
    nat.begin("mmd_opt", 3, DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, xo, yo, 15.0, draws)
    st = ora.init_state(DEFAULT_INIT, DEFAULT_MEAN, DEFAULT_COV, draws)
    exact, explained = 0, []
    for t in range(Tf):
        _sync_state(nat, st, B)
        st["pop"] = nat.read("pop")[(t & 1) * B * 8:(t & 1) * B * 8 + B * 8].reshape(B, 8).copy()
        out = ora.iteration("mmd_opt", st, t, xo, yo, np.float32(15.0), draws, trace := [])
        tr = trace[0]
        nat.iterate(t, 1)
        nat.sync()
        close(f"res_norm[{t}]", nat.read("res_norm")[:B], tr["res_norm"], atol=1e-5)
        obs_g, lane_g = nat.read("obs_cost")[:B], nat.read("lane_cost")[:B]
        res_g = nat.read("res_beta").reshape(B, 20)
        esum_g = nat.read("btrace").reshape(B, 20)
        beta_g, sig_g = nat.read("beta").reshape(B, n), nat.read("sigma")[:B]
        cost_ok = np.abs(obs_g - tr["obs"]) <= 1e-2 + 1e-4 * np.abs(tr["obs"])
        cost_ok &= np.abs(lane_g - tr["lane"]) <= 1e-2 + 1e-4 * np.abs(tr["lane"])
        ok = cost_ok & np.all(np.abs(res_g - tr["res_beta"]) <= 1e-4 * np.abs(tr["res_beta"]) + 1e-6, axis=1)
        ok &= np.all(np.abs(beta_g - tr["beta"]) <= 1e-3 * np.abs(tr["beta"]) + 1e-4, axis=1)
        ok &= np.abs(sig_g - tr["sigma"]) <= 1e-6 * np.abs(tr["sigma"])
        if not ok.all():
            acc, steer = nat.read("acc").reshape(B, 100), nat.read("steer").reshape(B, 100)
            for b in np.nonzero(~ok)[0]:
                t0, tie, detail = beta_near_tie(beta_cem_trace(ora, st, acc[b], steer[b], draws, t), res_g[b],
                                                esum_g[b])
                print(f"iteration {t} candidate {b}: obs {obs_g[b]} / {tr['obs'][b]}, sigma {sig_g[b]} / "
                      f"{tr['sigma'][b]}; {detail}")
                assert tie, f"iteration {t} candidate {b}: beta-CEM differs without a near-tie ({detail})"
                explained.append((t, int(b)))
        if not cost_ok.all():
            continue  # obstacle / lane costs moved: the elite sets may legitimately differ; the next iteration re-syncs
        tp = nat.read("tr_proj", np.int32).reshape(Tf, B)[t]
        to = nat.read("tr_obs", np.int32).reshape(Tf, 20)[t]
        tc = nat.read("tr_cem", np.int32).reshape(Tf, 5)[t]
        if not elite_equal(f"elite_proj[{t}]", tp, tr["perm"], tr["res_norm"], tol=1e-3):
            continue
        if not elite_equal(f"elite_obs[{t}]", to, tr["elite_obs"], tr["obs"]):
            continue
        if not elite_equal(f"elite_cem[{t}]", tc, tr["elite_cem"], tr["cost20"]):
            continue
        exact += 1
        nxt = ((t + 1) & 1) * B * 8
        close(f"pop[{t}]", nat.read("pop")[nxt:nxt + B * 8].reshape(B, 8), st["pop"], rtol=1e-4, atol=1e-4)
        res = nat.read("results").reshape(Tf, -1)[t]
        close(f"result_cx[{t}]", res[:11], out["cx"], atol=1e-3)
        close(f"result_cy[{t}]", res[11:22], out["cy"], atol=1e-3)
        close(f"result_obs[{t}]", res[23], out["obs"], rtol=1e-4, atol=1e-2)
        if ok[to[0]]:  # the result's beta-CEM outputs (unless that candidate's beta-CEM parted at a near-tie)
            close(f"result_sigma[{t}]", res[24], out["sigma"], rtol=1e-6, atol=0)
            close(f"result_res_beta[{t}]", res[25:45], out["res_beta"], rtol=1e-4, atol=1e-4)
            close(f"result_beta[{t}]", res[45:45 + n], out["beta"], rtol=1e-3, atol=1e-4)
    print(f"{exact}/{Tf} iterations exact; beta-CEM near-tie divergences {explained}")
    assert exact >= 15, f"only {exact}/{Tf} iterations had identical elite sets"
