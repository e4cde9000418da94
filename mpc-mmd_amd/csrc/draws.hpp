// Internal draws of one outer iteration as per-item device functions, shared
// by their own launches (k_noise, k_gamma_tab) and by k_select, which draws
// iteration t + 1's items in spare workgroups while its one workgroup per
// configuration ranks iteration t (k_select alone occupies G CUs for ~30 us;
// the draws are independent of the ranking).
#pragma once

#include "kernels.hpp"
#include "rng.hpp"

namespace mpcmmd {

// roll [3][H][S] (Philox normals, 4 per item) and resample [B-5][8]
HDI int noise_items(const Params& p) { return 3 * ((p.S * p.H + 3) / 4) + ((p.B - kElite) * 8 + 3) / 4; }

__device__ inline void noise_item(const Params& p, int t, const Cfg& cf, int j) {
  const int S = p.S, H = p.H;
  const uint32_t k0 = iteration_key0(cf.idx_mpc, t), k1 = p.seed;
  const int nroll = (S * H + 3) / 4;
  const int nres = ((p.B - kElite) * 8 + 3) / 4;
  float* roll = const_cast<float*>(cf.roll) + size_t(t) * 3 * H * S;
  float* res = const_cast<float*>(cf.resample) + size_t(t) * (p.B - kElite) * 8;
  if (j < 3 * nroll) {
    const int st = j / nroll, jb = j % nroll;
    double z[4];
    philox_normals4(k0, k1, kStreamRollAcc + st, 0u, uint32_t(jb), z);
    for (int q = 0; q < 4; ++q) {
      const int e = 4 * jb + q;
      if (e >= S * H) break;
      const int s = e / H, h = e % H;
      roll[(size_t(st) * H + h) * S + s] = float(z[q]);
    }
  } else if (j < 3 * nroll + nres) {
    const int jb = j - 3 * nroll;
    double z[4];
    philox_normals4(k0, k1, kStreamResample, 0u, uint32_t(jb), z);
    for (int q = 0; q < 4; ++q) {
      const int e = 4 * jb + q;
      if (e < (p.B - kElite) * 8) res[e] = float(z[q]);
    }
  }
}

// Beta-noise attempt table (rng.hpp): one item per (stream, attempt, r, h).
// Item 0 of configuration 0 also clears k_beta_planes' deferred-list count.
HDI int gamma_items(const Params& p) { return kGammaTabStreams * kGammaTabAttempts * p.S * p.H; }

__device__ inline void gamma_item(const Params& p, int t, const Cfg& cf, int idx) {
  const int S = p.S, H = p.H;
  const int plane = S * H;
  if (idx == 0 && cf.g == 0) *p.bfix_n = 0u;
  const int e = idx % plane, sk = idx / plane;
  const int k = sk % kGammaTabAttempts, st = sk / kGammaTabAttempts;
  const int h = e / S, r = e - h * S;
  const uint32_t k0 = iteration_key0(cf.idx_mpc, t), k1 = p.seed;
  const GammaAttempt g = gamma_attempt(k0, k1, kStreamGammaAccA + uint32_t(st), uint32_t(r) * uint32_t(H) + h, k);
  double* o = cf.gtab + (size_t(sk) * 4) * plane + e;
  o[0] = g.x;
  o[plane] = g.u;
  o[2 * size_t(plane)] = g.lu;
  const bool squeeze = g.u < 1.0 - 0.0331 * (g.x * g.x) * (g.x * g.x);  // alpha-independent (rng.hpp)
  o[3 * size_t(plane)] = squeeze ? g.lw : -g.lw;
}

// which draws a k_select launch produces ahead (bit mask)
constexpr int kAheadNoise = 1, kAheadGamma = 2;
HDI int ahead_items(const Params& p, int kind) {
  return ((kind & kAheadNoise) ? noise_items(p) : 0) + ((kind & kAheadGamma) ? gamma_items(p) : 0);
}
// item i of the ahead draws of iteration t (all G configurations)
__device__ inline void ahead_item(const Params& p, int t, int kind, int i) {
  const int per = ahead_items(p, kind);
  const int g = i / per, j = i - g * per;
  if (g >= p.G) return;
  const Cfg cf = cfg_of(p, g);
  const int nn = (kind & kAheadNoise) ? noise_items(p) : 0;
  if (j < nn)
    noise_item(p, t, cf, j);
  else
    gamma_item(p, t, cf, j - nn);
}

}  // namespace mpcmmd
