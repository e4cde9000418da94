// Device pieces of the CARLA variant's Frenet frame (carla/optimizer/
// cem_helper.py:171-242, projection.py:307): jnp.interp and the closest-point
// transform, on path arrays staged in LDS.  Same fp32 operations as the host
// (carla_host.cpp) and the oracle (oracle/carla.py).
#pragma once
#include "common.hpp"

namespace mpcmmd {

// jnp.interp(x, xp, fp) (jax 0.3.23): fp[i-1] + ((x - xp[i-1]) / dx) * df,
// i = clip(searchsorted(xp, x, 'right'), 1, P - 1); fp[0] / fp[P-1] outside.
DEVI float interp_jnp(float x, const float* xp, const float* fp, int P) {
  int lo = 0, hi = P;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (xp[m] <= x) lo = m + 1;
    else hi = m;
  }
  const int i = lo < 1 ? 1 : (lo > P - 1 ? P - 1 : lo);
  const float dx = xp[i] - xp[i - 1];
  const float df = fp[i] - fp[i - 1];
  const float delta = x - xp[i - 1];
  float f = fabsf(dx) <= 1.4210855e-14f ? fp[i - 1] : fp[i - 1] + (delta / dx) * df;
  if (x < xp[0]) f = fp[0];
  if (x > xp[P - 1]) f = fp[P - 1];
  return f;
}

// global_to_frenet_trajs (cem_helper.py:206-242) of one point on a quad of
// lanes: the first path point minimising sqrt(dx^2 + dy^2) (the first NaN if
// any), s = its arc length, d = the signed distance along the interpolated
// path normal.  Lane q of the quad scans path points [q Pq, (q + 1) Pq);
// pxy: the path as float2 (x, y) in LDS, padded with +inf to 4 Pq points
// (Pq a multiple of 8: eight points per batch of LDS reads).
//
// The scan compares squares: sqrtf is monotone, so pass 1 finds the first
// minimum bq of dx^2 + dy^2 (no square root per point), and the reference's
// answer -- the first point whose sqrtf equals sqrtf(bq) -- is the first
// point with a square <= hi, the largest float whose sqrtf is sqrtf(bq)
// (pass 2, over the points before the minimum; ties within an ulp or two of
// sqrtf are the only ones it finds).  Same index as comparing sqrtf point by
// point.  Every lane of the quad returns the same (s, d).
constexpr int kFrenetBatch = 8;
HDI int frenet_quarter(int P) { return (((P + 3) / 4) + kFrenetBatch - 1) / kFrenetBatch * kFrenetBatch; }

DEVI int quad_min_i(int v) {
  v = min(v, __shfl_xor(v, 1));
  return min(v, __shfl_xor(v, 2));
}

DEVI void frenet_point_quad(float x, float y, const float2* pxy, const float* arc, const float* Fxd, const float* Fyd,
                            int P, int Pq, float& s, float& d) {
  constexpr int kNone = 0x7fffffff;
  const int q = threadIdx.x & 3, j0 = q * Pq;
  const float4* p4 = reinterpret_cast<const float4*>(pxy + j0);
  const float inf = __int_as_float(0x7f800000);
  // squares of the batch of points c .. c + 7 of the lane's quarter
  auto batch = [&](int c, float (&sq)[kFrenetBatch]) {
    float4 v[kFrenetBatch / 2];
#pragma unroll
    for (int u = 0; u < kFrenetBatch / 2; ++u) v[u] = p4[(c >> 1) + u];
#pragma unroll
    for (int u = 0; u < kFrenetBatch / 2; ++u) {
      const float dx0 = v[u].x - x, dy0 = v[u].y - y, dx1 = v[u].z - x, dy1 = v[u].w - y;
      sq[2 * u] = dx0 * dx0 + dy0 * dy0;
      sq[2 * u + 1] = dx1 * dx1 + dy1 * dy1;
    }
  };
  float bq = inf;
  int bj = kNone, nanj = kNone;
  for (int c = 0; c < Pq; c += kFrenetBatch) {
    float sq[kFrenetBatch];
    batch(c, sq);
#pragma unroll
    for (int e = 0; e < kFrenetBatch; ++e) {
      const int j = j0 + c + e;
      nanj = min(nanj, sq[e] != sq[e] && j < P ? j : kNone);
      const bool lt = sq[e] < bq;
      bq = lt ? sq[e] : bq;
      bj = lt ? j : bj;
    }
  }
  // the quad's first minimum: the smaller square, equal squares the smaller index
#pragma unroll
  for (int m = 1; m <= 2; m <<= 1) {
    const float oq = __shfl_xor(bq, m);
    const int oj = __shfl_xor(bj, m);
    const bool take = oq < bq || (oq == bq && oj < bj);
    bq = take ? oq : bq;
    bj = take ? oj : bj;
  }
  nanj = quad_min_i(nanj);
  int best;
  if (nanj != kNone) {
    best = nanj;
  } else if (!(bq < inf)) {
    best = 0;  // no finite distance: no sqrtf is below the initial +inf
  } else {
    const float m = sqrtf(bq);
    float hi = bq;
    for (int it = 0; it < 8; ++it) {  // a sqrtf value has at most ~4 squares
      const float nx = __int_as_float(__float_as_int(hi) + 1);
      if (sqrtf(nx) != m) break;
      hi = nx;
    }
    int fj = bj;
    const int end = min(bj - j0, Pq);
    for (int c = 0; c < end; c += kFrenetBatch) {
      float sq[kFrenetBatch];
      batch(c, sq);
#pragma unroll
      for (int e = 0; e < kFrenetBatch; ++e) {
        const int j = j0 + c + e;
        fj = min(fj, j < bj && sq[e] <= hi ? j : kNone);
      }
    }
    best = quad_min_i(fj);
  }
  s = arc[best];
  const float Fx = interp_jnp(s, arc, Fxd, P);
  const float Fy = interp_jnp(s, arc, Fyd, P);
  const float nx = -Fy, ny = Fx;
  const float nrm = sqrtf(nx * nx + ny * ny);
  const float2 c = pxy[best];
  d = (1.0f / nrm) * (nx * (x - c.x) + ny * (y - c.y));
}

}  // namespace mpcmmd
