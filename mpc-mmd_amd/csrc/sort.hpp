// One-key-per-thread sorts of distinct 64-bit keys inside one workgroup
// (k_select's argsorts; tools/sort_bench.hip measures them).
#pragma once
#include "common.hpp"

namespace mpcmmd {

// The key of lane (lane ^ S), S < 64, by DPP / permlane moves (no LDS
// round trip): quad permutes for 1 and 2, row shifts for 4, the row rotate
// for 8, the permlane swaps for 16 and 32.
template <int S>
DEVI unsigned long long xor_partner(unsigned long long a) {
  int lo = int(a), hi = int(a >> 32);
  const int lane = threadIdx.x & 63;
  if constexpr (S == 1) {
    lo = dpp_i<0xB1>(lo);
    hi = dpp_i<0xB1>(hi);
  } else if constexpr (S == 2) {
    lo = dpp_i<0x4E>(lo);
    hi = dpp_i<0x4E>(hi);
  } else if constexpr (S == 4) {  // row_shl:4 (lane + 4) or row_shr:4 (lane - 4)
    const int l1 = dpp_i<0x104>(lo), h1 = dpp_i<0x104>(hi);
    const int l2 = dpp_i<0x114>(lo), h2 = dpp_i<0x114>(hi);
    const bool up = (lane & 4) != 0;
    lo = up ? l2 : l1;
    hi = up ? h2 : h1;
  } else if constexpr (S == 8) {  // row_ror:8
    lo = dpp_i<0x128>(lo);
    hi = dpp_i<0x128>(hi);
  } else {
    static_assert(S == 16 || S == 32, "xor stride");
    float xl = __int_as_float(lo), yl = xl, xh = __int_as_float(hi), yh = xh;
    permlane_swap<S>(xl, yl);
    permlane_swap<S>(xh, yh);
    // after the swap y holds the partner where the lane's S-bit is 0, x where it is 1
    const bool first = (lane & S) == 0;
    lo = __float_as_int(first ? yl : xl);
    hi = __float_as_int(first ? yh : xh);
  }
  return (static_cast<unsigned long long>(static_cast<unsigned>(hi)) << 32) | static_cast<unsigned>(lo);
}

// one compare-exchange stage of the bitonic network at stride S (in-wave)
template <int S>
DEVI unsigned long long cx_stage(unsigned long long a, bool up) {
  const unsigned long long b = xor_partner<S>(a);
  const bool lower = (threadIdx.x & S) == 0;
  const unsigned long long mn = a < b ? a : b, mx = a < b ? b : a;
  return lower == up ? mn : mx;
}

// the in-wave stages of a bitonic merge, strides top .. 1 (top <= 32)
DEVI unsigned long long wave_merge(unsigned long long a, int top, bool up) {
  if (top >= 32) a = cx_stage<32>(a, up);
  if (top >= 16) a = cx_stage<16>(a, up);
  if (top >= 8) a = cx_stage<8>(a, up);
  if (top >= 4) a = cx_stage<4>(a, up);
  if (top >= 2) a = cx_stage<2>(a, up);
  return cx_stage<1>(a, up);
}

// bitonic_sort_reg's network (ascending, N a power of two <= blockDim.x, key
// a of thread i; threads >= N hold ~0): the in-wave stages by DPP / permlane
// moves, the strides >= 64 through LDS k[N].  Returns thread i's sorted key.
DEVI unsigned long long bitonic_reg_dpp(unsigned long long a, int N, unsigned long long* k) {
  const int i = threadIdx.x;
  for (int size = 2; size <= N; size <<= 1) {
    const bool up = (i & size) == 0;
    for (int stride = size >> 1; stride >= 64; stride >>= 1) {
      __syncthreads();
      if (i < N) k[i] = a;
      __syncthreads();
      const unsigned long long b = i < N ? k[i ^ stride] : ~0ull;
      const bool lower = (i & stride) == 0;
      const unsigned long long mn = a < b ? a : b, mx = a < b ? b : a;
      a = lower == up ? mn : mx;
    }
    a = wave_merge(a, min(size >> 1, 32), up);
  }
  return a;
}

// Ascending sort of N distinct keys (N a power of two <= blockDim.x; key a of
// thread i, threads >= N hold ~0): every wave sorts its 64 keys (bitonic,
// DPP / permlane moves), then runs of L = 64, 128, .. are merged pairwise --
// a key's place in the merged run is its place in its own run plus the
// number of smaller keys in the partner run (a binary search in LDS; real
// keys are distinct, so no ties), one barrier per level (k: 2 x 1024 words,
// the levels alternate halves).  Returns a; idx = its position in the sorted
// order.  The padding keys (~0, threads B..N-1) are equal, so a search would
// give two pads of a pair of runs the same place and leave holes that a later
// level reads; they instead keep idx = i at every level: after the wave sort
// they sit at threads >= B, and the real keys of every merged pair of runs
// fill exactly its slots below B, so the pads' own slots are the rest.
DEVI unsigned long long merge_sort_reg(unsigned long long a, int& idx, int N, unsigned long long* k) {
  const int i = threadIdx.x, run = min(N, 64);
  for (int size = 2; size <= run; size <<= 1) a = wave_merge(a, size >> 1, size == run || (i & size) == 0);
  idx = i;
  int lvl = 0;
  for (int L = 64; L < N; L <<= 1, ++lvl) {
    unsigned long long* b = k + (lvl & 1) * 1024;
    if (i < N) b[idx] = a;
    __syncthreads();
    if (i < N && a != ~0ull) {
      const int r = idx / L, pos = idx & (L - 1);
      const unsigned long long* part = b + (r ^ 1) * L;
      int base = 0;
      for (int half = L >> 1; half > 0; half >>= 1) base += part[base + half - 1] < a ? half : 0;
      base += part[base] < a ? 1 : 0;
      idx = (r & ~1) * L + pos + base;
    }
  }
  return a;
}

}  // namespace mpcmmd
