"""Restatement of ``S/opt/cem.py`` (class ``CEM``): the 20-iteration outer
CEM for the four cost variants, built on the oracle's helper / projection /
costs / beta_cem modules.  Test infrastructure only.

``CEM`` mirrors the reference constructor (``S/opt/cem.py:17-18``) and the
``compute_cem_{mmd_opt,mmd_random,cvar,saa}`` entry points (``:201-714``),
with the RNG made explicit (``draws``) and an optional ``trace`` list that
records per-iteration elite index sets for parity tests.
"""
from __future__ import annotations

import numpy as np

from . import beta_cem as bc
from . import costs as C
from . import helper as H
from .problem import Problem
from .projection import compute_projection
from .rng import Draws

F32 = np.float32
F64 = np.float64
COSTS = ("mmd_opt", "mmd_random", "cvar", "saa")


class CEM:
    def __init__(self, num_reduced, num_obs, noise_level, num_prime, noise,
                 acc_const_noise, steer_const_noise, num_batch=100, variant="static",
                 maxiter_cem=20):
        self.prob = Problem(num_reduced, num_obs, noise_level, num_prime, noise,
                            acc_const_noise, steer_const_noise, num_batch, variant, maxiter_cem)

    def __getattr__(self, name):       # expose reference attribute names
        return getattr(self.__dict__["prob"], name)

    # ------------------------------------------------------------------
    def init_state(self, init_state, mean, cov, draws):
        """Carry initialisation (cem.py:206-219)."""
        p = self.prob
        B = p.num_batch
        st = dict(
            pop=H.sampling_param(p, np.asarray(mean, F32), np.asarray(cov, F32), draws.pop0),
            mean=np.asarray(mean, F32).copy(), cov=np.asarray(cov, F32).copy(),
            lam_x=np.zeros((B, 11), F32), lam_y=np.zeros((B, 11), F32),
            s_lane=np.zeros((B, 2 * (p.num - 1)), F32))
        st["b_eq_x"], st["b_eq_y"] = H.compute_boundary_vec(p, init_state)
        st["st0"] = H.initial_state5(init_state)
        return st

    def candidate_costs(self, cost, st, acc, steer, x_obs, y_obs, draws, t):
        """Obstacle + lane risk per candidate (un-permuted order).

        Returns obs [B], lane [B] and, for mmd_opt, beta [B, n], sigma [B],
        res_beta [B, 20].  The reference computes lane costs for the 20
        obstacle elites only; every candidate's value is identical, so the
        elites' entries are taken afterwards.
        """
        p = self.prob
        n = p.num_reduced
        Hh = p.num_prime
        xo, yo = x_obs[:, :Hh], y_obs[:, :Hh]
        acc_n, steer_n = H.noisy_controls(p, acc[:, :Hh], steer[:, :Hh], draws, t, n)
        extra = {}
        if cost == "mmd_opt":
            B = acc.shape[0]
            acc_m, steer_m = H.mother_controls(acc_n, steer_n)                # [B, M, H]
            xm, ym = H.rollout(p, acc_m, steer_m, st["st0"])
            cxm, cym = H.compute_coeff(p, xm, ym)
            beta = np.empty((B, n), F32)
            sigma = np.empty(B, F32)
            res_beta = np.empty((B, p.maxiter_beta_cem), F32)
            sel = np.empty((B, n), np.int64)
            for b in range(B):
                beta[b], res_beta[b], sigma[b], sel[b] = bc.compute_cem(
                    p, cxm[b], cym[b], draws.beta_z0, draws.beta_z)
            xr = np.take_along_axis(xm, sel[:, :, None], axis=1)
            yr = np.take_along_axis(ym, sel[:, :, None], axis=1)
            cb = C.compute_f_bar_max(p, xr, yr, xo, yo)
            obs = C.mmd(p, beta, cb, sigma)
            lane = C.mmd_lane(p, beta, sigma, yr)
            extra = dict(beta=beta, sigma=sigma, res_beta=res_beta, sel=sel)
        else:
            xr, yr = H.rollout(p, acc_n, steer_n, st["st0"])                # [B, S, H]
            cb = C.compute_f_bar_max(p, xr, yr, xo, yo)
            if cost == "mmd_random":
                B = acc.shape[0]
                beta = np.full((B, n), F32(1.0 / n))                         # cem.py:355
                sigma = np.full(B, F32(0.01))                                # cem.py:356
                obs = C.mmd(p, beta, cb, sigma)
                lane = np.zeros(B, F32)                                      # cem.py:427
            elif cost == "cvar":
                obs = C.cvar(p, cb)
                lane = C.cvar_lane(p, yr)
            else:
                obs = C.saa(p, cb)
                lane = C.saa_lane(p, yr)
        return obs, lane, extra

    def front(self, st):
        """Guess + projection + controls (cem.py:227-252).  Updates the
        positional carries in ``st`` and returns (pr, acc, steer)."""
        p = self.prob
        cxb, cyb = H.compute_x_guess(p, st["b_eq_x"], st["b_eq_y"], st["pop"])
        pr = compute_projection(p, st["b_eq_x"], st["b_eq_y"], st["lam_x"], st["lam_y"],
                                cxb, cyb, st["s_lane"])
        # carries are positional, never permuted (cem.py:230, 313)
        st["lam_x"], st["lam_y"], st["s_lane"] = pr["lam_x"], pr["lam_y"], pr["s_lane"]
        acc, steer = H.compute_controls(p, pr["xd"], pr["yd"], pr["xdd"], pr["ydd"])
        pr["cxb"], pr["cyb"] = cxb, cyb
        return pr, acc, steer

    def weights(self, cost):
        p = self.prob
        w_obs = {"mmd_opt": p.weight_mmd_obs, "mmd_random": p.weight_mmd_obs,
                 "cvar": p.weight_cvar_obs, "saa": p.weight_saa_obs}[cost]
        w_lane = {"mmd_opt": p.weight_mmd_lane, "mmd_random": p.weight_mmd_lane,
                  "cvar": p.weight_cvar_lane, "saa": p.weight_saa_lane}[cost]
        return w_obs, w_lane

    def select(self, cost, st, t, pr, steer, obs, lane, v_des, draws, extra=None):
        """argsorts, compute_cost, elites, compute_shifted_samples
        (cem.py:233-315).  Mutates ``st`` (pop, mean, cov); returns
        (out, info)."""
        p = self.prob
        perm = H.argsort_stable(pr["res_norm"])                              # cem.py:233
        idx_obs = H.argsort_stable(obs[perm])[:p.ellite_num_cost]            # cem.py:264
        el = perm[idx_obs]
        w_obs, w_lane = self.weights(cost)
        obs_el = obs[el]
        lane_el = lane[el]
        cost20 = H.compute_cost(p, (F32(w_obs) * obs_el).astype(F32),
                                (F32(w_lane) * lane_el).astype(F32),
                                pr["y"][el], pr["res_norm"][el], pr["xd"][el], pr["yd"][el],
                                pr["xdd"][el], pr["ydd"][el], v_des, steer[el])
        idx_cem = H.argsort_stable(cost20)                                   # cem_helper.py:267
        pop_el = st["pop"][el[idx_cem[:p.ellite_num]]]
        cost5 = cost20[idx_cem[:p.ellite_num]]
        st["mean"], st["cov"], st["pop"] = H.compute_shifted_samples(
            p, pop_el, cost5, st["mean"], st["cov"], draws.resample[t])
        imin = bc.argmin_nan(cost5)                                           # cem.py:308 (== 0)
        e = el[imin]
        out = dict(cx=pr["c_x"][e], cy=pr["c_y"][e], lane=lane_el[imin], obs=obs_el[imin])
        if cost == "mmd_opt":
            out.update(beta=extra["beta"][e], sigma=extra["sigma"][e], res_beta=extra["res_beta"][e])
        info = dict(perm=perm, elite_obs=el, cost20=cost20, elite_cem=idx_cem[:p.ellite_num])
        return out, info

    def iteration(self, cost, st, t, x_obs, y_obs, v_des, draws, trace=None):
        """One ``lax_cem`` body (cem.py:221-315 and the three siblings).
        Mutates ``st`` (the scan carry) and returns the per-iteration output
        tuple (cem.py:314-315)."""
        pr, acc, steer = self.front(st)
        obs, lane, extra = self.candidate_costs(cost, st, acc, steer, x_obs, y_obs, draws, t)
        out, info = self.select(cost, st, t, pr, steer, obs, lane, v_des, draws, extra)
        if trace is not None:
            trace.append(dict(res_norm=pr["res_norm"], obs=obs, lane=lane, cx=pr["c_x"], cy=pr["c_y"],
                              pop=st["pop"].copy(), mean=st["mean"].copy(), cov=st["cov"].copy(),
                              **info, **extra))
        return out

    def solve(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, draws=None,
              seed=0, trace=None):
        if cost not in COSTS:
            raise ValueError(cost)
        p = self.prob
        if draws is None:
            draws = Draws.philox(p, idx_mpc, seed, with_beta_cem=(cost == "mmd_opt"))
        x_obs = np.asarray(x_obs, F32)
        y_obs = np.asarray(y_obs, F32)
        st = self.init_state(init_state, mean, cov, draws)
        out = None
        for t in range(p.maxiter_cem):
            out = self.iteration(cost, st, t, x_obs, y_obs, F32(v_des), draws, trace)
        # result[...][-1]: the last iteration's elite-0 (cem.py:324-333, Q1)
        if cost == "mmd_opt":
            return (out["cx"], out["cy"], out["lane"], out["obs"], out["beta"], out["sigma"],
                    out["res_beta"])
        return out["cx"], out["cy"], out["lane"], out["obs"]

    # reference entry-point names (S/opt/cem.py:201, 335, 464, 590)
    def compute_cem_mmd_opt(self, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw):
        return self.solve("mmd_opt", idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw)

    def compute_cem_mmd_random(self, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw):
        return self.solve("mmd_random", idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw)

    def compute_cem_cvar(self, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw):
        return self.solve("cvar", idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw)

    def compute_cem_saa(self, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw):
        return self.solve("saa", idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, **kw)
