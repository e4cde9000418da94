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

// global_to_frenet_trajs (cem_helper.py:206-242) of one point: the first
// path point minimising sqrt(dx^2 + dy^2) (first NaN if any), s = its arc
// length, d = the signed distance along the interpolated path normal.
// pxy: the path as float2 (x, y) in LDS.
DEVI void frenet_point(float x, float y, const float2* pxy, const float* arc, const float* Fxd, const float* Fyd,
                       int P, float& s, float& d) {
  int best = 0;
  float bd = __int_as_float(0x7f800000);
  bool nan = false;
  for (int j = 0; j < P; ++j) {
    const float2 q = pxy[j];
    const float dx = q.x - x, dy = q.y - y;
    const float dist = sqrtf(dx * dx + dy * dy);
    if (dist != dist && !nan) {
      nan = true;
      best = j;
    }
    if (!nan && dist < bd) {
      bd = dist;
      best = j;
    }
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
