// Counter-based RNG streams of the library (host + device).
// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123 round
// constants), Box-Muller in fp64, Marsaglia-Tsang gamma in fp64, Beta as a
// log-space gamma ratio.  The counter layout mirrors the reference's key
// structure (fixed key for the initial population and the beta-CEM tables,
// key 3*idx_mpc + 5*t + 7 per outer iteration: cem.py:225, cem_helper.py:86,
// compute_beta.py:25) and is restated by oracle/rng.py for the parity tests.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

namespace mpcmmd {

enum Stream : uint32_t {
  kStreamRollAcc = 0,
  kStreamRollSteer = 1,
  kStreamRollConst = 2,
  kStreamResample = 3,
  kStreamGammaAccA = 4,
  kStreamGammaAccB = 5,
  kStreamGammaSteerA = 6,
  kStreamGammaSteerB = 7,
  kStreamValAcc = 24,  // validation (k_validate): normals acc / steer / const, Beta gammas
  kStreamValSteer = 25,
  kStreamValConst = 26,
  kStreamValGammaAccA = 27,
  kStreamValGammaAccB = 28,
  kStreamValGammaSteerA = 29,
  kStreamValGammaSteerB = 30,
  kStreamPop0 = 16,
  kStreamBetaZ0 = 17,
  kStreamBetaZ = 18,
  kStreamInitEps = 19,  // CARLA noisy initial states, key (idx_mpc, seed) (carla/optimizer/cem_helper.py:662-665)
};
constexpr uint32_t kFixedKey0 = 0xFFFFFFFFu;
constexpr int kGammaMaxAttempts = 32;

struct U4 {
  uint32_t x, y, z, w;
};

HDI U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = uint64_t(M0) * c.x;
    const uint64_t p1 = uint64_t(M1) * c.z;
    const uint32_t hi0 = uint32_t(p0 >> 32), lo0 = uint32_t(p0);
    const uint32_t hi1 = uint32_t(p1 >> 32), lo1 = uint32_t(p1);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

HDI uint32_t iteration_key0(int32_t idx_mpc, int32_t t) { return uint32_t(3 * idx_mpc + 5 * t + 7); }

HDI double u01(uint32_t u) { return (double(u) + 0.5) * (1.0 / 4294967296.0); }

// 4 normals of block j of stream (stream, word1): counter (j, word1, stream, 0)
HDI void philox_normals4(uint32_t k0, uint32_t k1, uint32_t stream, uint32_t word1, uint32_t j, double out[4]) {
  const U4 u = philox4x32_10(U4{j, word1, stream, 0u}, k0, k1);
  const double two_pi = 6.283185307179586;
  double r0 = sqrt(-2.0 * log(u01(u.x)));
  double t0 = two_pi * u01(u.y);
  double r1 = sqrt(-2.0 * log(u01(u.z)));
  double t1 = two_pi * u01(u.w);
  out[0] = r0 * cos(t0);
  out[1] = r0 * sin(t0);
  out[2] = r1 * cos(t1);
  out[3] = r1 * sin(t1);
}

// Marsaglia-Tsang acceptance of attempt (x, u, log u) for d, v3 = (1 + c x)^3:
// the squeeze u < 1 - 0.0331 x^4 first, the exact log test only when it
// fails (Marsaglia & Tsang 2000; oracle/rng.py:_log_gamma_parts applies the
// identical two tests in the identical order).
// The exact test lu < 0.5 x^2 + d - d v3 + d log(v3) is first decided in
// fp32 (v_log_f32) and re-evaluated in fp64 only when the two sides lie
// within a bound far above the fp32 evaluation error: the same decision as
// the fp64 test, without an fp64 log (a ~50-instruction expansion) per attempt.
HDI bool mt_log_test(double x, double lu, double d, double v3) {
#ifdef __HIP_DEVICE_COMPILE__
  const float xf = float(x), df = float(d), v3f = float(v3), luf = float(lu);
  const float q = 0.5f * xf * xf, dv = df * v3f, dl = df * (__builtin_amdgcn_logf(v3f) * 0.693147180559945309f);
  const float rhs = ((q + df) - dv) + dl;
  const float tol = 1e-5f * (1.0f + fabsf(luf) + q + fabsf(df) + fabsf(dv) + fabsf(dl));
  if (luf < rhs - tol) return true;
  if (luf > rhs + tol) return false;
#endif
  return lu < 0.5 * x * x + d - d * v3 + d * log(v3);
}
HDI bool mt_accept(double x, double u, double lu, double d, double v3) {
  if (u < 1.0 - 0.0331 * (x * x) * (x * x)) return true;
  return mt_log_test(x, lu, d, v3);
}

// One Marsaglia-Tsang attempt from the Philox counter (elem, k, stream, 1):
// words 0,1 -> Box-Muller normal (cos branch), word 2 -> acceptance uniform,
// word 3 -> boost uniform.
struct GammaAttempt {
  double x, u, lu, lw;
};
HDI GammaAttempt gamma_attempt(uint32_t k0, uint32_t k1, uint32_t stream, uint32_t elem, int k) {
  const U4 w = philox4x32_10(U4{elem, uint32_t(k), stream, 1u}, k0, k1);
  const double two_pi = 6.283185307179586;
  const double r = sqrt(-2.0 * log(u01(w.x)));
  GammaAttempt a;
  a.x = r * cos(two_pi * u01(w.y));
  a.u = u01(w.z);
  a.lu = log(a.u);
  a.lw = log(u01(w.w));
  return a;
}

// Attempt table of one outer iteration: the Philox-derived (x, u, log u,
// +-log w) of attempts 0..kGammaTabAttempts-1 for every (stream, row r, step h).
// The squeeze test u < 1 - 0.0331 x^4 does not depend on alpha, so it is
// evaluated once when the table is built and stored as the sign of the
// log w field (log w < 0 always): negative = the squeeze accepts.
// The uniforms of the Beta noise depend only on (key, stream, r, h) -- the
// same realisation for every candidate (cem_helper.py:110, Q2) -- so they
// are drawn once per iteration instead of once per candidate; each
// candidate applies only its own (alpha-dependent) transform.  Layout
// [stream 0..3][k][field 0..3][h][r] (r fastest: coalesced per sample row).
constexpr int kGammaTabAttempts = 4;
constexpr int kGammaTabStreams = 4;  // acc A, acc B, steer A, steer B
HDI size_t gamma_tab_size(int S, int H) { return size_t(kGammaTabStreams) * kGammaTabAttempts * 4 * S * H; }

// G' for alpha' = alpha (+1 when alpha < 1) and the boost log-uniform,
// from the table (attempts < kGammaTabAttempts) then Philox directly.
struct MtConst {
  double d, c;
};
HDI MtConst mt_const(double alpha) {
  const double a1 = alpha < 1.0 ? alpha + 1.0 : alpha;
  const double d = a1 - 1.0 / 3.0;
  return MtConst{d, 1.0 / sqrt(9.0 * d)};
}
// One tabulated attempt (fields x, log u, +-log w; the uniform u itself is
// only needed by the squeeze, whose decision the sign of log w holds):
// Marsaglia-Tsang acceptance with the stored squeeze decision
struct TabAtt {
  double x, lu, lw;
};
DEVI TabAtt tab_load(const double* t, size_t plane) { return TabAtt{t[0], t[2 * plane], t[3 * plane]}; }
DEVI bool tab_try(MtConst mc, const TabAtt& a, double& g, double& lub) {
  const double v = 1.0 + mc.c * a.x;
  if (v > 0.0) {
    const double v3 = v * v * v;
    if (a.lw < 0.0 || mt_log_test(a.x, a.lu, mc.d, v3)) {
      g = mc.d * v3;
      lub = -fabs(a.lw);
      return true;
    }
  }
  return false;
}
DEVI bool tab_attempt(MtConst mc, const double* t, size_t plane, double& g, double& lub) {
  return tab_try(mc, tab_load(t, plane), g, lub);
}
DEVI void gamma_parts_tab(MtConst mc, const double* tab, int S, int H, int r, int h, uint32_t k0, uint32_t k1,
                          uint32_t stream, uint32_t elem, double& g, double& lub) {
  const double d = mc.d, c = mc.c;
  const size_t plane = size_t(S) * H, at = size_t(h) * S + r;
  g = d;
  lub = 0.0;
  for (int k = 0; k < kGammaTabAttempts; ++k) {
    if (tab_attempt(mc, tab + size_t(k) * 4 * plane + at, plane, g, lub)) return;
  }
  for (int k = kGammaTabAttempts; k < kGammaMaxAttempts; ++k) {
    const GammaAttempt ga = gamma_attempt(k0, k1, stream, elem, k);
    const double v = 1.0 + c * ga.x;
    if (v > 0.0) {
      const double v3 = v * v * v;
      if (mt_accept(ga.x, ga.u, ga.lu, d, v3)) {
        g = d * v3;
        lub = ga.lw;
        return;
      }
    }
  }
}

// Beta(a, b) = Ga / (Ga + Gb) from the two gammas' G' and boost log-uniforms
// (G = G' U^(1/alpha) for alpha < 1):  1 / (1 + 2^d) with
//   d = log2 Gb - log2 Ga = log2 gb - log2 ga + log2(e) (ub/b - ua/a).
// The boost difference (two large, close terms for a small control) is
// formed in fp64 as one fraction (ub a - ua b) / (a b) and rounded once (a
// huge |d| saturates the draw at 0 or 1 through inf, as the fp64 form does); the
// rest is fp32 (v_log_f32, v_exp_f32, v_rcp_f32).  Versus the oracle's fp64
// evaluation (oracle/rng.py:beta_draws) the draw differs by a few ulp where it
// is not saturated at 0 or 1 (tests/test_gpu_parity_baseline.py states the
// tolerance); the accept / reject decisions of the gammas stay fp64 and exact.
DEVI float beta_combine(double a, double b, double ra, double rb, double ga, double ua, double gb, double ub) {
  if (a == 0.0 && b == 0.0) return (ua * rb > ub * ra) ? 1.0f : 0.0f;
  const bool ka = a < 1.0, kb = b < 1.0;
  const double fa = ka ? a : 1.0, fb = kb ? b : 1.0;
  const double num = (kb ? ub : 0.0) * fa - (ka ? ua : 0.0) * fb;
  const float e = float(num * __builtin_amdgcn_rcp(fa * fb));  // v_rcp_f64: fp64 range for tiny controls
  const float d = (__builtin_amdgcn_logf(float(gb)) - __builtin_amdgcn_logf(float(ga))) +
                  1.44269504088896340736f * e;
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(d));
}

// beta_combine in fp64, rounded once (the CARLA variant, Params::carla):
// oracle/rng.py:beta_draws' formula -- G = G' exp(log U / alpha) and Ga / (Ga
// + Gb) while both boost exponents exceed -600, else the same ratio in log
// space -- so a draw is the oracle's float32 value but where the two fp64
// evaluations straddle a float32 rounding boundary.  The CARLA risk takes
// the closest path point of every rollout point (a discontinuous map): a
// draw a few ulp off moves a candidate's risk by a path step, where the
// static variant's risks move by ulps.
constexpr double kBoostLinMin = -600.0;
DEVI float beta_combine_cr(double a, double b, double ra, double rb, double ga, double ua, double gb, double ub) {
  if (a == 0.0 && b == 0.0) return (ua * rb > ub * ra) ? 1.0f : 0.0f;
  const double ba = a < 1.0 ? ua / (a > 0.0 ? a : 1.0) : 0.0;
  const double bb = b < 1.0 ? ub / (b > 0.0 ? b : 1.0) : 0.0;
  double out;
  if (ba > kBoostLinMin && bb > kBoostLinMin) {
    const double Ga = ga * (a < 1.0 ? exp(ba) : 1.0), Gb = gb * (b < 1.0 ? exp(bb) : 1.0);
    out = Ga / (Ga + Gb);
  } else {
    const double la = log(ga) + ba, lb = log(gb) + bb, lm = la > lb ? la : lb;
    const double ea = exp(la - lm), eb = exp(lb - lm);
    out = ea / (ea + eb);
  }
  return float(out);
}

// Beta(a, b) with a = ra*s, b = rb*s (s = |control|); s == 0 takes the
// alpha -> 0+ limit (oracle/rng.py:beta_draws, DESIGN.md Numerics).  tab_a,
// tab_b: the attempt-table slices of the two gamma streams.
// mc_a, mc_b: mt_const(a), mt_const(b) (shared by every row r of a step).
// cr: the fp64 combine (beta_combine_cr, the CARLA variant).
DEVI float beta_draw_tab(double a, double b, double ra, double rb, MtConst mc_a, MtConst mc_b,
                         const double* tab_a, const double* tab_b, int S, int H, int r, int h, uint32_t k0,
                         uint32_t k1, uint32_t stream_a, uint32_t stream_b, bool cr = false) {
  const uint32_t elem = uint32_t(r) * uint32_t(H) + uint32_t(h);
  double ga, ua, gb, ub;
  gamma_parts_tab(mc_a, tab_a, S, H, r, h, k0, k1, stream_a, elem, ga, ua);
  gamma_parts_tab(mc_b, tab_b, S, H, r, h, k0, k1, stream_b, elem, gb, ub);
  return cr ? beta_combine_cr(a, b, ra, rb, ga, ua, gb, ub) : beta_combine(a, b, ra, rb, ga, ua, gb, ub);
}

// Table-only path for the hot plane kernel: attempts k0 .. kGammaTabAttempts
// - 1 of the table; false when a gamma needs more (rare: the caller defers
// the element to the full beta_draw_tab, identical arithmetic)
DEVI bool gamma_tab_from(MtConst mc, const double* tab, size_t plane, size_t at, int k0, double& g, double& lub) {
  for (int k = k0; k < kGammaTabAttempts; ++k)
    if (tab_attempt(mc, tab + size_t(k) * 4 * plane + at, plane, g, lub)) return true;
  return false;
}
}  // namespace mpcmmd
