"""Restatement of ``S/compute_beta.py`` (class ``beta_cem``): the nested CEM
that picks the reduced sample set and the MMD weights beta for one candidate.
Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

from .helper import argsort_stable, chol64, sort_key

F32 = np.float32
F64 = np.float64


def f32(x):
    return np.asarray(x, dtype=F64).astype(F32)


def l1_dist(a, b):
    """sum_f |a_f - b_f| over the 22 features, sequential fp32 (the order the
    GPU uses, so equal features give bit-equal distances).
    a [..., 22] broadcast against b [..., 22]."""
    acc = np.abs(a[..., 0] - b[..., 0])
    for f in range(1, a.shape[-1]):
        acc = acc + np.abs(a[..., f] - b[..., f])
    return acc.astype(F32)


def argmin_nan(x):
    """jnp.argmin: first NaN if any, else first minimum."""
    nan = np.isnan(x)
    if nan.any():
        return int(np.argmax(nan))
    return int(np.argmin(x))


def select_top(samples, M, n):
    """idx_beta_top = argsort(|beta[:, :M]|, axis=1)[:, M-n:] (compute_beta.py:117-118)."""
    keys = sort_key(np.abs(samples[:, :M]))
    return np.argsort(keys, axis=1, kind="stable")[:, M - n:]


def distance_matrix(F):
    """All L1 distances of the mother features [M, M] (the rows
    ``reduced_qp`` gathers; bit-identical to computing them per sample)."""
    return l1_dist(F[:, None, :], F[None, :, :])


def reduced_qp(prob, F, top, sigma, M, D=None):
    """Kernels (compute_beta.py:120-127, kernel_computation.py:19-65) and the
    equality-constrained QP ``compute_beta_reduced`` (compute_beta.py:70-91)
    for every sample.  Returns beta_top [K, n] fp32, cost [K] fp32,
    K_red [K, n, n] fp32, rowsum [K, n] fp64.  ``D``: the precomputed
    ``distance_matrix(F)`` (large M: gathered instead of recomputed)."""
    K, n = top.shape
    if D is None:
        A = F[top]                                            # [K, n, 22]
        D_red = l1_dist(A[:, :, None, :], A[:, None, :, :])    # [K, n, n]
        D_mix = l1_dist(A[:, :, None, :], F[None, None, :, :])  # [K, n, M]
    else:
        D_mix = D[top]                                         # [K, n, M]
        D_red = np.take_along_axis(D_mix, top[:, None, :], axis=2)
    sig = sigma.astype(F32)[:, None, None]
    K_red = np.exp((-D_red) / sig).astype(F32)
    K_mix = np.exp((-D_mix) / sig).astype(F32)
    rowsum = K_mix.astype(F64).sum(axis=2)
    inv_m = F64(F32(1.0 / M))
    g = rowsum * inv_m                                     # -lincost
    C = (K_red + F32(0.05) * np.eye(n, dtype=F32)).astype(F64)
    kkt = np.zeros((K, n + 1, n + 1))
    kkt[:, :n, :n] = C
    kkt[:, :n, n] = 1.0
    kkt[:, n, :n] = 1.0
    rhs = np.concatenate([g, np.ones((K, 1))], axis=1)
    beta = f32(np.linalg.solve(kkt, rhs[:, :, None])[:, :n, 0])
    b = beta.astype(F64)
    q = -2.0 * g
    cost = f32(np.einsum("si,sij,sj->s", b, K_red.astype(F64), b) + np.einsum("si,si->s", q, b))
    return beta, cost, K_red, rowsum


def compute_cem(prob, cx_m, cy_m, z0, z, trace=None):
    """``beta_cem.compute_cem`` (compute_beta.py:93-157) for ONE candidate.

    cx_m, cy_m [M, 11] mother Bernstein coefficients; z0 [100, M+1] and
    z [20, 89, M+1] the fixed-key normals (identical for every candidate, Q3).
    Returns (beta_best [n], res [20], sigma_best, sel_best [n]).
    ``sel_best`` are mother-row indices in the reference's argsort order; the
    caller gathers x_red/y_red with them.
    """
    M = cx_m.shape[0]
    n = prob.num_reduced
    E = prob.num_ellite_beta
    T = prob.maxiter_beta_cem
    F = np.concatenate([cx_m, cy_m], axis=1).astype(F32)   # B = dstack(cx, cy) (:124)
    # initial samples: MVN(0, 20 I) (:41-49, :108-110)
    samples = f32(np.sqrt(20.0) * z0.astype(F64))
    samples[:, M] = np.maximum(samples[:, M], F32(prob.sigma_clip))
    res = np.zeros(T, F32)
    out = None
    Dm = distance_matrix(F)   # gathered per sample: the same bits as recomputing them (reduced_qp)
    for t in range(T):
        sigma = samples[:, M].copy()
        top = select_top(samples, M, n)
        beta, cost, K_red, _ = reduced_qp(prob, F, top, sigma, M, Dm)
        # compute_mean_cov_beta (:51-68)
        idx_e = argsort_stable(cost)[:E]
        El = samples[idx_e].astype(F64)
        mean64 = El.mean(axis=0)
        mean32 = f32(mean64)
        D = El - mean64
        cov = D.T @ D / (E - 1) + 0.05 * np.eye(M + 1)
        L = chol64(cov)
        new = f32(mean32.astype(F64) + z[t].astype(F64) @ L.T)
        samples_next = np.vstack([samples[idx_e], new]).astype(F32)
        samples_next[:, M] = np.maximum(samples_next[:, M], F32(prob.sigma_clip))
        imin = argmin_nan(cost)
        res[t] = np.min(cost) if not np.isnan(cost).any() else np.nan
        out = (beta[imin].copy(), samples_next[imin, M], top[imin].copy())
        if trace is not None:
            trace.append(dict(top=top, sigma=sigma, cost=cost, beta=beta, elite=idx_e,
                              imin=imin, samples=samples))
        samples = samples_next
    beta_best, sigma_best, sel_best = out
    return beta_best, res, F32(sigma_best), sel_best


def compute_cem_batch(prob, cx_m, cy_m, z0, z):
    """``compute_cem`` for a batch of candidates at once (cx_m, cy_m [B, M,
    11]): the same per-candidate operations, stacked (tests compare it with the
    one-candidate form).  Returns beta [B, n], res [B, 20], sigma [B], sel
    [B, n]."""
    Bc, M = cx_m.shape[0], cx_m.shape[1]
    n = prob.num_reduced
    E = prob.num_ellite_beta
    T = prob.maxiter_beta_cem
    F = np.concatenate([cx_m, cy_m], axis=2).astype(F32)            # [B, M, 22]
    Dm = l1_dist(F[:, :, None, :], F[:, None, :, :])                 # [B, M, M]
    s0 = f32(np.sqrt(20.0) * z0.astype(F64))
    s0[:, M] = np.maximum(s0[:, M], F32(prob.sigma_clip))
    samples = np.broadcast_to(s0, (Bc,) + s0.shape).copy()          # [B, K, M+1]
    K = samples.shape[1]
    res = np.zeros((Bc, T), F32)
    bi = np.arange(Bc)[:, None]
    eye_n = F32(0.05) * np.eye(n, dtype=F32)
    inv_m = F64(F32(1.0 / M))
    out = None
    for t in range(T):
        sigma = samples[:, :, M].copy()                              # [B, K]
        keys = sort_key(np.abs(samples[:, :, :M]))
        top = np.argsort(keys, axis=2, kind="stable")[:, :, M - n:]  # [B, K, n]
        D_mix = Dm[bi[:, :, None], top]                              # [B, K, n, M]
        D_red = np.take_along_axis(D_mix, top[:, :, None, :], axis=3)
        sig = sigma.astype(F32)[:, :, None, None]
        K_red = np.exp((-D_red) / sig).astype(F32)
        K_mix = np.exp((-D_mix) / sig).astype(F32)
        g = K_mix.astype(F64).sum(axis=3) * inv_m                    # [B, K, n]
        kkt = np.zeros((Bc, K, n + 1, n + 1))
        kkt[:, :, :n, :n] = (K_red + eye_n).astype(F64)
        kkt[:, :, :n, n] = 1.0
        kkt[:, :, n, :n] = 1.0
        rhs = np.concatenate([g, np.ones((Bc, K, 1))], axis=2)
        beta = f32(np.linalg.solve(kkt.reshape(-1, n + 1, n + 1), rhs.reshape(-1, n + 1, 1))[:, :n, 0]
                   ).reshape(Bc, K, n)
        b = beta.astype(F64)
        quad = np.einsum("ksi,ksij,ksj->ks", b, K_red.astype(F64), b)
        cost = f32(quad + np.einsum("ksi,ksi->ks", -2.0 * g, b))
        idx_e = np.argsort(sort_key(cost), axis=1, kind="stable")[:, :E]   # [B, E]
        El = samples[bi, idx_e].astype(F64)                                # [B, E, M+1]
        mean64 = El.mean(axis=1)
        Dd = El - mean64[:, None, :]
        cov = np.matmul(Dd.transpose(0, 2, 1), Dd) / (E - 1) + 0.05 * np.eye(M + 1)
        L = np.linalg.cholesky(cov)
        new = f32(f32(mean64).astype(F64)[:, None, :] + np.matmul(z[t].astype(F64)[None], L.transpose(0, 2, 1)))
        samples_next = np.concatenate([samples[bi, idx_e], new], axis=1).astype(F32)
        samples_next[:, :, M] = np.maximum(samples_next[:, :, M], F32(prob.sigma_clip))
        nan = np.isnan(cost)
        imin = np.where(nan.any(axis=1), np.argmax(nan, axis=1), np.argmin(np.where(nan, np.inf, cost), axis=1))
        res[:, t] = np.where(nan.any(axis=1), np.nan, cost.min(axis=1))
        out = (beta[np.arange(Bc), imin], samples_next[np.arange(Bc), imin, M], top[np.arange(Bc), imin])
        samples = samples_next
    beta_best, sigma_best, sel_best = out
    return beta_best.copy(), res, sigma_best.astype(F32), sel_best.copy()


def compute_cem_many(prob, cx_m, cy_m, z0, z, threads=8):
    """``compute_cem_batch`` over candidate chunks on a thread pool (NumPy
    releases the GIL in its array kernels; no processes, so nothing is forked
    from a process that holds the GPU).  Same bits as one call."""
    Bc = cx_m.shape[0]
    k = max(1, min(threads, Bc))
    if k == 1:
        return compute_cem_batch(prob, cx_m, cy_m, z0, z)
    from concurrent.futures import ThreadPoolExecutor
    cuts = np.linspace(0, Bc, k + 1).astype(int)
    with ThreadPoolExecutor(k) as ex:
        parts = list(ex.map(lambda i: compute_cem_batch(prob, cx_m[cuts[i]:cuts[i + 1]], cy_m[cuts[i]:cuts[i + 1]],
                                                        z0, z), range(k)))
    return tuple(np.concatenate([p[j] for p in parts]) for j in range(4))
