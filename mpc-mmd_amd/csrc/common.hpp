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


// per-workgroup phase timestamp into dbgw[blockIdx.x][slot] (profiling only;
// the workgroups of one launch, slots 0..7)
#define MPCMMD_STAMPW(p, slot)                                                      \
  do {                                                                              \
    const unsigned wg_ = blockIdx.x + gridDim.x * blockIdx.y;                       \
    if (threadIdx.x == 0 && (p).dbgw && wg_ < 65536)                                \
      (p).dbgw[size_t(wg_) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)

constexpr int kWave = 64;

// ---- DPP helpers (gfx9 DPP controls) -----------------------------------------
// quad_perm(1,0,3,2) 0xB1, quad_perm(2,3,0,1) 0x4E, row_ror:4 0x124,
// row_ror:8 0x128, row_bcast:15 0x142, row_bcast:31 0x143.  Rows disabled by
// ROWS read 0.
// With every row enabled a lane without a source reads 0 through
// bound_ctrl, so no old value is needed (no register to initialise); with
// rows disabled those keep the old value 0.
template <int CTRL, int ROWS = 0xF>
DEVI int dpp_i(int v) {
  if constexpr (ROWS == 0xF)
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
  else
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, false);
}
template <int CTRL>
DEVI int dpp_full(int v) {
  return dpp_i<CTRL>(v);
}
template <int CTRL, int ROWS = 0xF>
DEVI double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_i<CTRL, ROWS>(int(b));
  const int hi = dpp_i<CTRL, ROWS>(int(b >> 32));
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
DEVI float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
DEVI double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(int(b), l);
  const int hi = __builtin_amdgcn_readlane(int(b >> 32), l);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// v_permlane32_swap (W = 32): lanes 32-63 of x <-> lanes 0-31 of y;
// v_permlane16_swap (W = 16): the odd 16-lane rows of x <-> the even rows of y.
// Inline asm: hipcc (ROCm 7.2) may commute the builtins' two operands, which
// exchanges the other halves.  s_nop 1: the VALU-write -> permlane hazard.
template <int W>
DEVI void permlane_swap(float& x, float& y) {
  if constexpr (W == 32)
    __asm__ volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  else
    __asm__ volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}

template <int W>
DEVI void permlane_swap(double& x, double& y) {
  const long long bx = __double_as_longlong(x), by = __double_as_longlong(y);
  float xl = __int_as_float(int(bx)), xh = __int_as_float(int(bx >> 32));
  float yl = __int_as_float(int(by)), yh = __int_as_float(int(by >> 32));
  permlane_swap<W>(xl, yl);
  permlane_swap<W>(xh, yh);
  x = __longlong_as_double((static_cast<long long>(__float_as_int(xh)) << 32) | static_cast<unsigned>(__float_as_int(xl)));
  y = __longlong_as_double((static_cast<long long>(__float_as_int(yh)) << 32) | static_cast<unsigned>(__float_as_int(yl)));
}

// wave totals of up to 16 per-lane fp64 values (v[n..15] taken as 0): lane l
// ends with the total of v[l >> 2].  Each butterfly step halves the values a
// lane carries (permlane32 / permlane16 swaps, then row_mirror and
// row_half_mirror DPP keeping the half the pairing's lane bit selects, then
// the quad) -- about a third of the instructions of n separate wave_sum trees.
template <int n>
DEVI double wave_totals16_d(const double (&v)[n]) {
  static_assert(n <= 16, "at most 16 values");
  const int lane = threadIdx.x & 63;
  auto at = [&](int i) { return i < n ? v[i] : 0.0; };
  double w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // lanes < 32 keep values 0..7, lanes >= 32 values 8..15
    double a = at(i), b = at(i + 8);
    permlane_swap<32>(a, b);
    w[i] = a + b;
  }
  double x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // odd rows keep the upper four
    double a = w[i], b = w[i + 4];
    permlane_swap<16>(a, b);
    x[i] = a + b;
  }
  const bool b3 = lane & 8, b2 = lane & 4;
  double y[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // row_mirror pairs l with l ^ 15 (bit 3 flipped)
    const double keep = b3 ? x[i + 2] : x[i], send = b3 ? x[i] : x[i + 2];
    y[i] = keep + dpp_d<0x140>(send);
  }
  // row_half_mirror pairs l with l ^ 7 (bit 2 flipped)
  double z = (b2 ? y[1] : y[0]) + dpp_d<0x141>(b2 ? y[0] : y[1]);
  z += dpp_d<0xB1>(z);
  return z + dpp_d<0x4E>(z);
}

// ---- wave-wide reductions (wave-uniform result) --------------------------------
// Sums: quad and row butterflies by DPP, then the row broadcasts into lane 63
// and one readlane -- VALU only (a __shfl_xor butterfly is six LDS-crossbar
// round trips, ds_bpermute, per sum).
DEVI int wave_total(int v) {
  v += dpp_i<0xB1>(v);
  v += dpp_i<0x4E>(v);
  v += dpp_i<0x124>(v);
  v += dpp_i<0x128>(v);
  v += dpp_i<0x142, 0xA>(v);
  v += dpp_i<0x143, 0xC>(v);
  return __builtin_amdgcn_readlane(v, 63);
}
DEVI float wave_total(float v) {
  v += __int_as_float(dpp_i<0xB1>(__float_as_int(v)));
  v += __int_as_float(dpp_i<0x4E>(__float_as_int(v)));
  v += __int_as_float(dpp_i<0x124>(__float_as_int(v)));
  v += __int_as_float(dpp_i<0x128>(__float_as_int(v)));
  v += __int_as_float(dpp_i<0x142, 0xA>(__float_as_int(v)));
  v += __int_as_float(dpp_i<0x143, 0xC>(__float_as_int(v)));
  return readlane_f(v, 63);
}
DEVI double wave_total(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x124>(v);
  v += dpp_d<0x128>(v);
  v += dpp_d<0x142, 0xA>(v);
  v += dpp_d<0x143, 0xC>(v);
  return readlane_d(v, 63);
}
DEVI double wave_sum(double v) { return wave_total(v); }
DEVI float wave_sum(float v) { return wave_total(v); }
DEVI int wave_sum(int v) { return wave_total(v); }
// wave maximum (fmaxf: NaN ignored unless every lane is NaN), VALU only: quad
// and row butterflies, then the row broadcasts into lane 63 (rows a broadcast
// does not write keep their own value: old = v), one readlane
template <int CTRL, int ROWS = 0xF>
DEVI float dpp_keep_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWS, 0xF, false));
}
DEVI float wave_max(float v) {
  v = fmaxf(v, dpp_keep_f<0xB1>(v));
  v = fmaxf(v, dpp_keep_f<0x4E>(v));
  v = fmaxf(v, dpp_keep_f<0x124>(v));
  v = fmaxf(v, dpp_keep_f<0x128>(v));
  v = fmaxf(v, dpp_keep_f<0x142, 0xA>(v));
  v = fmaxf(v, dpp_keep_f<0x143, 0xC>(v));
  return readlane_f(v, 63);
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

// sort_key(fabsf(x)) in four VALU operations: |x| has no sign and no -0, so
// the key is its bit pattern with bit 31 set, or ~0 for a NaN (pattern above
// +inf's) -- the same value for every x
DEVI uint32_t sort_key_abs(float x) {
  const uint32_t u = __float_as_uint(x) & 0x7FFFFFFFu;
  return u > 0x7F800000u ? 0xFFFFFFFFu : (u | 0x80000000u);
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
