// Device pieces shared by the rollout kernels (baseline risk and mmd_opt).
#pragma once
#include "common.hpp"
#include "kernels.hpp"
#include "rng.hpp"

namespace mpcmmd {

constexpr float kDt = 0.15f;         // cem.py:40
constexpr float kWheelBase = 2.5f;   // cem.py:26
constexpr float kObsA = 4.25f;       // a_obs (cem.py:25)

// The two Beta draws of (candidate controls a, s; row r, step h)
// (cem_helper.py:427-433): Beta(2|a|, 5|a|), Beta(2|s|, 5|s|).  mc: the four
// Marsaglia-Tsang constants of (2|a|, 5|a|, 2|s|, 5|s|) when the caller
// shares them across rows (else computed here).
DEVI void beta_pair(const Params& p, const Cfg& cf, int t, int r, int h, float a, float s, float& nba, float& nbs,
                    const MtConst* mc = nullptr) {
  const int S = p.S, H = p.H;
  const uint32_t k0 = iteration_key0(cf.idx_mpc, t), k1 = p.seed;
  const size_t sl = size_t(kGammaTabAttempts) * 4 * S * H;  // one stream's table
  const float fa = fabsf(a), fs = fabsf(s);
  const double aa = double(2.0f * fa), ab = double(5.0f * fa), sa = double(2.0f * fs), sb = double(5.0f * fs);
  MtConst m[4];
  if (mc) {
    for (int i = 0; i < 4; ++i) m[i] = mc[i];
  } else {
    m[0] = mt_const(aa), m[1] = mt_const(ab), m[2] = mt_const(sa), m[3] = mt_const(sb);
  }
  nba = beta_draw_tab(aa, ab, 2.0, 5.0, m[0], m[1], cf.gtab, cf.gtab + sl, S, H, r, h, k0, k1, kStreamGammaAccA,
                      kStreamGammaAccB, p.carla != 0);
  nbs = beta_draw_tab(sa, sb, 2.0, 5.0, m[2], m[3], cf.gtab + 2 * sl, cf.gtab + 3 * sl, S, H, r, h, k0, k1,
                      kStreamGammaSteerA, kStreamGammaSteerB, p.carla != 0);
}

// Noisy controls of noise row r at step h of outer iteration t
// (cem_helper.py:405-443 baseline / 469-508 opt; one realisation shared by
// every candidate, Q2).  Gaussian rows come from p.roll [T][3][H][S]; Beta
// draws from the Philox gamma streams (elements r*H + h) through the
// iteration's attempt table p.gtab (k_gamma_tab).
// kPlanes: Beta draws read from bpl (k_beta_planes) instead of sampled here.
template <bool kPlanes = false>
DEVI void noisy_control(const Params& p, const Cfg& cf, int t, int r, int h, float a, float s, float& an, float& sn,
                        const float* bpl = nullptr) {
  const int S = p.S, H = p.H;
  const float* roll = cf.roll + size_t(t) * 3 * H * S;
  const float nc = roll[(2 * H + h) * S + r];
  float ap, sp;
  if (p.noise == 0) {
    ap = (p.sigma_acc * fabsf(a)) * roll[(0 * H + h) * S + r];
    sp = (p.sigma_steer * fabsf(s)) * roll[(1 * H + h) * S + r];
  } else {
    float nba, nbs;
    if constexpr (kPlanes) {  // precomputed by k_beta_planes: [2][H][S] of this candidate
      nba = bpl[size_t(h) * S + r];
      nbs = bpl[(size_t(H) + h) * S + r];
    } else {
      beta_pair(p, cf, t, r, h, a, s, nba, nbs);
    }
    ap = p.sigma_acc * (2.0f * nba - 1.0f);
    sp = p.K_steer * (2.0f * nbs - 1.0f);  // K_steer holds float32(K_steer * sigma_steer)
  }
  an = (a + ap) + p.acc_const * nc;
  sn = (s + sp) + p.steer_const * nc;
}

// The same perturbation from the step's noise values already in registers:
// gaussian n0, n1 = the acc / steer normals, beta n0, n1 = the two Beta
// draws; n2 = the const-noise normal (identical arithmetic to noisy_control)
DEVI void noisy_from(const Params& p, float a, float s, float n0, float n1, float n2, float& an, float& sn) {
  float ap, sp;
  if (p.noise == 0) {
    ap = (p.sigma_acc * fabsf(a)) * n0;
    sp = (p.sigma_steer * fabsf(s)) * n1;
  } else {
    ap = p.sigma_acc * (2.0f * n0 - 1.0f);
    sp = p.K_steer * (2.0f * n1 - 1.0f);  // K_steer holds float32(K_steer * sigma_steer)
  }
  an = (a + ap) + p.acc_const * n2;
  sn = (s + sp) + p.steer_const * n2;
}

// compute_rollout_one_step (cem_helper.py:380-400), fp32 in reference order.
// psidot = v tan(steer) / 2.5: division by 2.5 via the exact fma form.
DEVI void bicycle_step(float& x, float& y, float& vx, float& vy, float& psi, float an, float sn) {
  float v = sqrtf(vx * vx + vy * vy);
  v = v + an * kDt;
  const float psidot = div_rc(v * tanf(sn), kWheelBase, 1.0f / kWheelBase);
  psi = psi + psidot * kDt;
  float sp, cp;
  sincosf(psi, &sp, &cp);  // one argument reduction for both (OCML: the values of sinf / cosf)
  vx = v * cp;
  vy = v * sp;
  x = x + vx * kDt;
  y = y + vy * kDt;
}

// The CARLA variant's step (carla/optimizer/cem_helper.py:732-751): wheel
// base 2.875, true division, tan / cos / sin evaluated in fp64 and rounded
// once (oracle/carla.py: rollout_cr), so rollouts - and the Frenet argmins
// taken on them - are reproducible bit for bit.
// Here with tn = float(tan(double(steer))) computed by the caller (it does
// not depend on the state: off the step chain), cos / sin from one fp64
// sincos (OCML: one argument reduction, the values of cos and sin).
DEVI void bicycle_step_cr_t(float& x, float& y, float& vx, float& vy, float& psi, float an, float tn, float wb) {
  float v = sqrtf(vx * vx + vy * vy);
  v = v + an * kDt;
  const float psidot = (v * tn) / wb;
  psi = psi + psidot * kDt;
  double sp, cp;
  sincos(double(psi), &sp, &cp);
  vx = v * float(cp);
  vy = v * float(sp);
  x = x + vx * kDt;
  y = y + vy * kDt;
}

// compute_f_bar (costs.py:50-60): ((-(dx^2))/a^2 - dy^2/b^2) + 1
DEVI float f_bar(float x, float y, float xo, float yo) {
  constexpr float kA2 = 18.0625f, kB2 = 7.5625f;  // 4.25^2, 2.75^2 (exact in fp32)
  const float wc = x - xo, ws = y - yo;
  return (-div_rc(wc * wc, kA2, 1.0f / kA2) - div_rc(ws * ws, kB2, 1.0f / kB2)) + 1.0f;
}

}  // namespace mpcmmd

namespace mpcmmd {
// compute_f_bar with the CARLA ellipse (carla/optimizer/costs.py:48-57, a =
// 4.5, b = 3): true divisions by a^2 = 20.25, b^2 = 9
DEVI float f_bar_ab(float x, float y, float xo, float yo, float a2, float b2) {
  const float wc = x - xo, ws = y - yo;
  return ((-(wc * wc)) / a2 - (ws * ws) / b2) + 1.0f;
}
}  // namespace mpcmmd
