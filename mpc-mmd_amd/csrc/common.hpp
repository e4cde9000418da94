// Device helpers shared by the kernels (gfx950, wave64).
// Everything in this library is compiled with -ffp-contract=off: the fp32
// elementwise expressions follow the reference's operation order exactly and
// only explicit fmaf()/fma() fuse.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEVI __device__ __forceinline__
#define HDI __host__ __device__ __forceinline__

namespace mpcmmd {

// phase timestamp of workgroup 0 into dbg[slot] (profiling only)
#define MPCMMD_STAMP(p, slot)                                                   \
  do {                                                                          \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (p).dbg)                         \
      (p).dbg[(slot)] = __builtin_amdgcn_s_memrealtime();                       \
  } while (0)


constexpr int kWave = 64;

// ---- wave-wide reductions (result valid in every lane) ----------------------
DEVI double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
DEVI float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
DEVI int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
DEVI float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
DEVI unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, kWave);
    v = w > v ? w : v;
  }
  return v;
}
DEVI unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, kWave);
    v = w < v ? w : v;
  }
  return v;
}

DEVI float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// ---- ordering ----------------------------------------------------------------
// jnp.argsort total order on fp32: -0 == +0, every NaN equal and last.
HDI uint32_t sort_key(float x) {
  if (x == 0.0f) x = 0.0f;
  if (x != x) return 0xFFFFFFFFu;
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t u = __float_as_uint(x);
#else
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
#endif
  return (u >> 31) ? ~u : (u | 0x80000000u);
}

// ---- arithmetic --------------------------------------------------------------
// x / d for a divisor known in advance, r = RN(1/d): one FMA correction of
// RN(x r).  Bit-equal to IEEE division for every x when d = 2.5, and for
// d = 4.25^2, 2.75^2 wherever |x| >= 2^-117 (checked exhaustively on the host;
// below that the caller's "+ 1" absorbs any difference).  For run-time
// divisors it is within 1 ulp (used only where results are tolerance-checked).
DEVI float div_rc(float x, float d, float r) {
  float q = x * r;
  float e = fmaf(-q, d, x);
  return fmaf(e, r, q);
}

// NaN-propagating max (numpy.maximum semantics; v_max_f32 returns the non-NaN
// operand).
DEVI float max_nan(float a, float b) { return (a != a || b != b) ? __int_as_float(0x7fc00000) : fmaxf(a, b); }

}  // namespace mpcmmd
