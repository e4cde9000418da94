// Workgroup-level helpers: reductions, bitonic sort of 64-bit keys in LDS,
// and the CVaR / SAA / MMD reducers over an LDS-resident sample vector.
#pragma once
#include "common.hpp"

namespace mpcmmd {

// sum over the workgroup (blockDim.x multiple of 64); scratch: >= 16 doubles
DEVI double block_sum(double v, double* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  __syncthreads();
  return s;
}
DEVI int block_sum(int v, int* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  int s = 0;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

// ascending bitonic sort of N (power of two) 64-bit keys in LDS, whole block
DEVI void bitonic_sort(unsigned long long* k, int N) {
  for (int size = 2; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < (N >> 1); i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long a = k[lo], b = k[hi];
        if ((a > b) == up) {
          k[lo] = b;
          k[hi] = a;
        }
      }
    }
  }
  __syncthreads();
}

// The same network with one key per thread (N <= blockDim.x): the stages
// whose partner is in the same wave (stride < 64) exchange by lane shuffles,
// only the wider ones go through LDS with barriers (10 of 55 stages at
// N = 1024).  Same compare-exchanges, so the same result as bitonic_sort.
DEVI void bitonic_sort_reg(unsigned long long* k, int N) {
  const int i = threadIdx.x;
  __syncthreads();
  unsigned long long a = i < N ? k[i] : ~0ull;
  for (int size = 2; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      unsigned long long b;
      if (stride >= 64) {
        __syncthreads();
        if (i < N) k[i] = a;
        __syncthreads();
        b = i < N ? k[i ^ stride] : ~0ull;
      } else {
        b = __shfl_xor(a, stride, 64);
      }
      const bool up = (i & size) == 0, lower = (i & stride) == 0;
      const unsigned long long mn = a < b ? a : b, mx = a < b ? b : a;
      a = lower == up ? mn : mx;
    }
  }
  __syncthreads();
  if (i < N) k[i] = a;
  __syncthreads();
}

// block_sum of a double and an int together (one pair of barriers for both;
// each total in block_sum's order, so the same bits)
DEVI void block_sum2(double& v, int& c, double* sd, int* si) {
  v = wave_sum(v);
  c = wave_sum(c);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sd[w] = v;
    si[w] = c;
  }
  __syncthreads();
  double s = 0.0;
  int k = 0;
  for (int i = 0; i < nw; ++i) {
    s += sd[i];
    k += si[i];
  }
  __syncthreads();
  v = s;
  c = k;
}

struct ReduceScratch {
  double d[16];
  int i[16];
  int list_n;
  float v_lo, v_hi;
  unsigned long long t0;
  alignas(16) unsigned long long gm[128];  // 8-lane group maxima of block_cvar (blockDim <= 1024)
};

// largest 64-bit word over each group of 8 lanes (quad butterflies, then
// row_half_mirror pairs the two quads), in every lane of the group
DEVI unsigned long long max8_u64(unsigned long long v) {
  auto step = [](unsigned long long a, auto dpp) {
    const unsigned long long b = (static_cast<unsigned long long>(unsigned(dpp(int(a >> 32)))) << 32) |
                                 unsigned(dpp(int(a)));
    return b > a ? b : a;
  };
  v = step(v, [](int x) { return dpp_i<0xB1>(x); });
  v = step(v, [](int x) { return dpp_i<0x4E>(x); });
  return step(v, [](int x) { return dpp_i<0x141>(x); });
}

// smallest 64-bit word over each group of 8 lanes, in every lane of the group
DEVI unsigned long long min8_u64(unsigned long long v) {
  auto step = [](unsigned long long a, auto dpp) {
    const unsigned long long b = (static_cast<unsigned long long>(unsigned(dpp(int(a >> 32)))) << 32) |
                                 unsigned(dpp(int(a)));
    return b < a ? b : a;
  };
  v = step(v, [](int x) { return dpp_i<0xB1>(x); });
  v = step(v, [](int x) { return dpp_i<0x4E>(x); });
  return step(v, [](int x) { return dpp_i<0x141>(x); });
}

// The K smallest of B <= blockDim.x distinct 64-bit words (one per thread,
// w = ~0 for threads >= B), in ascending order: out(rank, w) for rank < K.
// Window as in block_cvar: T0 = the K-th smallest of the 8-lane group minima
// (the K groups whose minimum is <= T0 hold K words <= T0, so every one of
// the K smallest is <= T0, and at most K groups contribute), the words <= T0
// compacted into LDS and ranked exactly among themselves.  gm: B / 8 + 2
// words, list: 8 K + 2 words (16-byte aligned), cnt / t0: LDS scalars.
template <class Out>
DEVI void block_smallest(unsigned long long w, int B, int K, unsigned long long* gm, unsigned long long* list,
                         int& cnt, unsigned long long& t0, Out out) {
  const int tid = threadIdx.x, G = (B + 7) >> 3;
  const unsigned long long m = min8_u64(w);
  if ((tid & 7) == 0 && tid < 8 * G) gm[tid >> 3] = m;
  if (tid == 0) {
    cnt = 0;
    t0 = ~0ull;     // fewer than K groups: every word is in the window
    gm[G] = ~0ull;  // pads the pair reads (never smaller); slot G is no group's
  }
  // the list pre-filled with ~0 (never smaller): the pair reads past its
  // count need no pad written after the compaction
  for (int i = tid; i < 8 * K + 2; i += blockDim.x) list[i] = ~0ull;
  __syncthreads();
  if (G > K && tid < G) {
    const unsigned long long mg = gm[tid];  // group tid's minimum
    const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(gm);
    int r = 0;
#pragma unroll 8
    for (int q = 0; q < (G + 1) >> 1; ++q) {  // LDS broadcast reads, several in flight
      const ulonglong2 v = g2[q];
      r += int(v.x < mg) + int(v.y < mg);
    }
    if (r == K - 1) t0 = mg;
  }
  __syncthreads();
  const unsigned long long T0 = t0;
  if (tid < B && w <= T0) list[atomicAdd(&cnt, 1)] = w;
  __syncthreads();
  const int c = cnt;
  const ulonglong2* l2 = reinterpret_cast<const ulonglong2*>(list);
  for (int a = tid; a < c; a += blockDim.x) {
    const unsigned long long ka = list[a];
    int r = 0;
#pragma unroll 8
    for (int q = 0; q < (c + 1) >> 1; ++q) {
      const ulonglong2 v = l2[q];
      r += int(v.x < ka) + int(v.y < ka);
    }
    if (r < K) out(r, ka);
  }
  __syncthreads();
}

// jnp.quantile(x, 0.98) (linear, JAX fp32 weights) + mean of the tail
// (costs.py:215-219) over vals[0..S).  list: >= S 64-bit words of LDS.
// Sorted order = the jnp.argsort total order (ties by index): the words
// (sort key << 32 | index) are distinct and their unsigned order is it.
// Ascending positions lo <= hi lie among the top need = S - lo words, so
// only a window of the largest words is ranked: T0 = the need-th largest of
// the 8-lane group maxima (each of those need groups holds a word >= T0, so
// at least need words are >= T0, and at most need groups contribute), the
// words >= T0 are compacted into LDS and ranked exactly among themselves.
DEVI float block_cvar(const float* vals, int S, unsigned long long* list, ReduceScratch& rs) {
  const float pos = 0.98f * float(S - 1);
  const float flo = floorf(pos), fhi = ceilf(pos);
  const float hw = pos - flo;
  const float lw = 1.0f - hw;
  const int lo = min(max(int(flo), 0), S - 1), hi = min(max(int(fhi), 0), S - 1);
  const int need = S - lo, tid = threadIdx.x, G = blockDim.x >> 3;
  auto word = [&](int s) {
    return (static_cast<unsigned long long>(sort_key(vals[s])) << 32) | static_cast<unsigned>(s);
  };
  unsigned long long km = 0;  // below every word (sort keys are >= 0x007FFFFF)
  for (int s = tid; s < S; s += blockDim.x) {
    const unsigned long long k = word(s);
    km = k > km ? k : km;
  }
  km = max8_u64(km);
  if (tid == 0) {
    rs.list_n = 0;
    rs.t0 = 0;  // need > G: every word is in the window
    rs.v_lo = 0.0f;
    rs.v_hi = 0.0f;
  }
  if ((tid & 7) == 0) rs.gm[tid >> 3] = km;
  __syncthreads();
  if (need <= G && tid < G) {
    const unsigned long long g = rs.gm[tid];
    const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(rs.gm);
    int r = 0;
#pragma unroll 8
    for (int q = 0; q < (G >> 1); ++q) {  // LDS broadcast reads, several in flight (G even)
      const ulonglong2 v = g2[q];
      r += int(v.x > g) + int(v.y > g);
    }
    if (r == need - 1) rs.t0 = g;  // empty groups (0) share a rank: any of them writes 0
  }
  __syncthreads();
  const unsigned long long T0 = rs.t0;
  for (int s = tid; s < S; s += blockDim.x) {
    const unsigned long long k = word(s);
    if (k >= T0) list[atomicAdd(&rs.list_n, 1)] = k;
  }
  __syncthreads();
  const int c = rs.list_n;
  for (int a = tid; a < c; a += blockDim.x) {
    const unsigned long long ka = list[a];
    int r = 0;  // words above ka: its position from the top
#pragma unroll 8
    for (int q = 0; q < c; ++q) r += list[q] > ka;  // several broadcast reads in flight
    const int ia = int(ka & 0xFFFFFFFFull);
    if (r == S - 1 - lo) rs.v_lo = vals[ia];
    if (r == S - 1 - hi) rs.v_hi = vals[ia];
  }
  __syncthreads();
  const float var = rs.v_lo * lw + rs.v_hi * hw;
  double sum = 0.0;
  int cnt = 0;
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    const float v = vals[s];
    if (v >= var) {  // false for NaN
      sum += double(v);
      ++cnt;
    }
  }
  block_sum2(sum, cnt, rs.d, rs.i);
  return cnt > 0 ? float(sum / double(cnt)) : 0.0f;
}

// fraction of samples > 0 (costs.py:230-234, 160-171)
DEVI int block_count_pos(const float* vals, int S, ReduceScratch& rs) {
  int c = 0;
  for (int s = threadIdx.x; s < S; s += blockDim.x) c += vals[s] > 0.0f;
  return block_sum(c, rs.i);
}

// Laplace-kernel MMD against a Dirac at 0 (kernel_computation.py:67-87):
// ker_wt (b^T K_aa b - 2 b^T K_ab b_del) with K = exp(-|d| / sigma).
// beta == nullptr means uniform beta = float32(1/n) (mmd_random, cem.py:355).
DEVI float block_mmd(const float* c, const float* beta, int n, float sigma, float ker_wt, ReduceScratch& rs) {
  const float bdel = 1.0f / float(n);
  const float rs_sig = 1.0f / sigma;
  double q1 = 0.0, q2 = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float ci = c[i];
    double row = 0.0;
    for (int k = 0; k < n; ++k) {
      const float d = fabsf(ci - c[k]);
      const float kk = __expf(div_rc(-d, sigma, rs_sig));
      row += double(kk) * double(beta ? beta[k] : bdel);
    }
    const double bi = double(beta ? beta[i] : bdel);
    q1 += bi * row;
    const float kab = __expf(div_rc(-fabsf(ci - 0.0f), sigma, rs_sig));
    q2 += bi * (double(kab) * (double(n) * double(bdel)));
  }
  q1 = block_sum(q1, rs.d);
  q2 = block_sum(q2, rs.d);
  return float(double(ker_wt) * (q1 - 2.0 * q2));
}

}  // namespace mpcmmd
