// Stage "risk" for cost = mmd_opt: the mother rollouts, their Bernstein fit
// and the nested beta-CEM that picks the reduced set and the MMD weights,
// then the reduced-set MMD.  Per outer iteration:
//
//   k_mother    noisy control rows, n^2 mother rollouts (Cartesian product,
//               cem_helper.py:469-530) with the ridge fit folded into the scan
//               (compute_coeff, cem_helper.py:553-564) -> 22 features per row
//   20 x { k_bsample  new samples of the beta-CEM (compute_beta.py:51-68)
//          k_bselect  top-n |beta| rows and sigma per sample (compute_beta.py:41-49, 117-118)
//          k_bkernel  Laplace-kernel row sums over the mother set and K_red
//                     (kernel_computation.py:19-65, compute_beta.py:120-127)
//          k_bqp      the equality-constrained QP and its cost per sample
//                     (compute_beta.py:70-91, 129)
//          k_belite   elite 11, mean, structured Cholesky of
//                     cov = D D^T / 10 + 0.05 I, next generators (compute_beta.py:51-68, 133-145) }
//   k_mmdfinal  reduced-set rollouts, collision residual, MMD obs / lane
//               (costs.py:121-135, 173-186)
//
// k_bselect and k_bqp are latency-bound chains and run as many single-wave
// workgroups; the others use one workgroup per candidate (the candidate's beta-CEM
// is sequential over its 20 iterations; candidates are independent).
//
// The covariance of the beta-CEM is rank <= 10 plus 0.05 I
// (jnp.cov of 11 elites, compute_beta.py:61).  Its Cholesky factor is never
// formed: with U = (E - mean)^T / sqrt(10), Phi_j = I + U_{<j}^T U_{<j} / d,
// v_j = Phi_j^-1 u_j, L_jj = sqrt(d + u_j.v_j), w_j = v_j / L_jj, one has
// L_ij = u_i . w_j (i > j), so (L z)_i = L_ii z_i + u_i . sum_{j<i} w_j z_j.
// Same factor as chol(cov) in exact arithmetic, O(M r^2) instead of O(M^3).
#include "block.hpp"
#include "kernels.hpp"
#include "rng.hpp"
#include "rollout.hpp"

namespace mpcmmd {

namespace {

constexpr int kF = 22;                               // features: cx (11) | cy (11)
constexpr int kNew = kBetaSamples - kBetaElite;      // 89 resampled rows per iteration
constexpr int kThreads = 512;
constexpr double kSqrt20 = 4.47213595499957927704;   // chol(20 I) (compute_beta.py:24)
constexpr double kRidge = 0.05;                      // cov jitter (compute_beta.py:61)
constexpr double kInvRidge = 20.0;

#define kconst __attribute__((address_space(4)))
typedef float f2 __attribute__((ext_vector_type(2)));

// Intra-wave LDS hand-off: a wave's LDS operations execute in order, so only
// the compiler must be kept from reordering them (no memory-counter waits).
DEVI void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  __asm__ volatile("" ::: "memory");
}

// ------------------------------------------------------------------------
// k_mother
__global__ __launch_bounds__(kThreads) void k_mother(Params p, int t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = p.n, H = p.H, M = p.M, b = blockIdx.x;
  float* an = reinterpret_cast<float*>(smem);
  float* sn = an + n * H;
  float* gctrl = p.ctrl_n + size_t(b) * 2 * n * H;
  for (int idx = threadIdx.x; idx < n * H; idx += blockDim.x) {
    const int r = idx / H, h = idx % H;
    float a, s;
    noisy_control(p, t, r, h, p.acc[size_t(b) * 100 + h], p.steer[size_t(b) * 100 + h], a, s);
    an[idx] = a;
    sn[idx] = s;
    gctrl[idx] = a;
    gctrl[n * H + idx] = s;
  }
  __syncthreads();
  float* F = p.feat + size_t(b) * kF * M;
  for (int m = threadIdx.x; m < M; m += blockDim.x) {
    // jnp.repeat(acc, n, 0) / jnp.tile(steer, (n, 1)) (cem_helper.py:510-511)
    const float* ar = an + (m / n) * H;
    const float* sr = sn + (m % n) * H;
    float x = p.st0[0], y = p.st0[1], vx = p.st0[2], vy = p.st0[3], psi = p.st0[4];
    double cx[11], cy[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) cx[k] = cy[k] = 0.0;
    for (int h = 0; h < H; ++h) {
      const double dx = double(x), dy = double(y);
#pragma unroll
      for (int k = 0; k < 11; ++k) {
        const double f = p.fit[k * H + h];
        cx[k] = cx[k] + f * dx;
        cy[k] = cy[k] + f * dy;
      }
      if (h == H - 1) break;
      bicycle_step(x, y, vx, vy, psi, ar[h], sr[h]);
    }
#pragma unroll
    for (int k = 0; k < 11; ++k) {
      F[k * M + m] = float(cx[k]);
      F[(11 + k) * M + m] = float(cy[k]);
    }
  }
}

// ------------------------------------------------------------------------
// top-n of |v_j| (j < M) in jnp.argsort order, one wave.  out[k] (k < n) are
// the indices at sorted positions M-n+k (ascending by (|v|, j)).
// Lane holds NQ keys (j = lane + 64 q).  The n-th largest key is found by
// bisection on the key bits with ballot counts; the search stops as soon as
// exactly n keys lie above the candidate threshold (continuous data: ~10 of
// the 31 steps).  Ties at the threshold go to the largest indices.
// scratch: 2 * 32 ints of LDS owned by the wave.
template <int NQ, class V>
DEVI void load_keys(V val, int M, uint32_t* key) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int j = lane + 64 * q;
    const float v = val(min(j, M - 1));
    key[q] = j < M ? sort_key(fabsf(v)) : 0u;  // real keys have bit 31 set
  }
}

// Threshold search for NB samples at once (independent chains interleave):
// T[u] = the n-th largest key of sample u, or exact[u] when exactly n keys
// are >= T[u] (the search stops early for continuous data).
template <int NQ, int NB>
DEVI void find_thresholds(const uint32_t (*key)[NQ], int nb, int n, uint32_t* T, bool* exact) {
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    T[u] = 0x80000000u;  // real keys have bit 31 set, padding keys are 0
    exact[u] = u >= nb;
  }
  for (int bit = 30; bit >= 0; --bit) {
    bool all = true;
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if (exact[u]) continue;
      const uint32_t cand = T[u] | (1u << bit);
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < NQ; ++q) cnt += __popcll(__ballot(key[u][q] >= cand));
      if (cnt >= n) T[u] = cand;
      exact[u] = cnt == n;
      all = all && exact[u];
    }
    if (all) break;
  }
}

// Given the threshold, write the indices of the top n keys to out[0..n) in
// jnp.argsort order (ascending key, ties by index).  Ties at a non-exact
// threshold go to the largest indices.
template <int NQ>
DEVI void emit_top(const uint32_t* key, uint32_t T, bool exact, int n, int32_t* out, int* scratch) {
  const int lane = threadIdx.x & 63;
  int need = 0;
  unsigned long long eqm[NQ];
  if (!exact) {
    int gt = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) gt += __popcll(__ballot(key[q] > T));
    need = n - gt;
#pragma unroll
    for (int q = 0; q < NQ; ++q) eqm[q] = __ballot(key[q] == T);
  } else {
#pragma unroll
    for (int q = 0; q < NQ; ++q) eqm[q] = 0ull;
  }
  const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  int* lj = scratch;
  uint32_t* lk = reinterpret_cast<uint32_t*>(scratch + 32);
  int base = 0;
  int later_eq = 0;  // equal keys in q' > q
#pragma unroll
  for (int q = 0; q < NQ; ++q) later_eq += __popcll(eqm[q]);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    later_eq -= __popcll(eqm[q]);
    const int larger = later_eq + __popcll(eqm[q] & above);
    const bool sel = exact ? key[q] >= T : (key[q] > T || (key[q] == T && larger < need));
    const unsigned long long sm = __ballot(sel);
    if (sel) {
      const int pos = base + __popcll(sm & ((1ull << lane) - 1ull));
      lj[pos] = lane + 64 * q;
      lk[pos] = key[q];
    }
    base += __popcll(sm);
  }
  wave_sync();
  // compaction order is ascending index, so ties rank by lane
  const int j = lane < n ? lj[lane] : 0;
  const uint32_t k = lane < n ? lk[lane] : 0xFFFFFFFFu;
  int r = 0;
  for (int c = 0; c < n; ++c) {
    const uint32_t kc = __builtin_amdgcn_readlane(k, c);
    r += (kc < k) || (kc == k && c < lane);
  }
  if (lane < n) out[r] = j;
  wave_sync();
}

// Top-n selection for the samples s = first, first + stride, ... < last of
// one wave, NB at a time: keys of NB samples are loaded together and their
// threshold searches interleave.  row(s) -> values, out(s) -> int32[n].
template <int NQ, class Row, class Out>
DEVI void select_batch(Row row, Out out, int first, int last, int stride, int M, int n, int* scratch) {
  constexpr int NB = NQ <= 8 ? 4 : (NQ <= 12 ? 2 : 1);
  for (int s0 = first; s0 < last; s0 += NB * stride) {
    uint32_t key[NB][NQ];
    const int nb = min(NB, (last - s0 + stride - 1) / stride);
#pragma unroll
    for (int u = 0; u < NB; ++u)  // unconditional (clamped) loads: one memory latency
      load_keys<NQ>(row(min(s0 + u * stride, last - 1)), M, key[u]);
    uint32_t T[NB];
    bool exact[NB];
    find_thresholds<NQ, NB>(key, nb, n, T, exact);
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (u < nb) emit_top<NQ>(key[u], T[u], exact[u], n, out(s0 + u * stride), scratch);
  }
}

template <class Row, class Out>
DEVI void select_rows(Row row, Out out, int first, int last, int stride, int M, int n, int* scratch) {
  switch ((M + 63) >> 6) {
#define MPCMMD_SEL_CASE(q) \
  case q:                  \
    return select_batch<q>(row, out, first, last, stride, M, n, scratch);
    MPCMMD_SEL_CASE(1)
    MPCMMD_SEL_CASE(2)
    MPCMMD_SEL_CASE(3)
    MPCMMD_SEL_CASE(4)
    MPCMMD_SEL_CASE(5)
    MPCMMD_SEL_CASE(6)
    MPCMMD_SEL_CASE(7)
    MPCMMD_SEL_CASE(8)
    MPCMMD_SEL_CASE(9)
    MPCMMD_SEL_CASE(10)
    MPCMMD_SEL_CASE(11)
    MPCMMD_SEL_CASE(12)
    MPCMMD_SEL_CASE(13)
    MPCMMD_SEL_CASE(14)
    MPCMMD_SEL_CASE(15)
#undef MPCMMD_SEL_CASE
    default:
      return select_batch<16>(row, out, first, last, stride, M, n, scratch);
  }
}

// ------------------------------------------------------------------------
// k_bsample: the new samples of beta-CEM iteration tb >= 1.
//
// New samples (rows 11..99) use the structured Cholesky (file header):
// lanes = samples, waves = position blocks, two passes (block partial sums
// P = sum_j w_j z_j, then the scan y_j = m_j + L_jj z_j + u_j . S_j).  The
// candidate's generators (W, U, L_jj, m per position, 192 B) are staged in
// LDS once, so the serial chain over positions is LDS-broadcast bound.  The
// samples go to ygen (global, row per sample) for the selection and for
// k_belite's elite copy.
constexpr int kZChunk = 16;  // positions per register chunk of normals in the generation
HDI size_t bs_gbytes(int M1) { return (size_t(M1) * kGenStride * 8 + 15) & ~size_t(15); }
HDI size_t bs_pbytes() { return size_t(8) * 11 * 64 * 8; }
HDI size_t bs_lds(int M1) { return bs_gbytes(M1) + bs_pbytes(); }

__global__ __launch_bounds__(kThreads) void k_bsample(Params p, int tb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, M = p.M, M1 = M + 1;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6, lane = threadIdx.x & 63;
  double* Gl = reinterpret_cast<double*>(smem);
  double* Pbuf = reinterpret_cast<double*>(smem + bs_gbytes(M1));
  MPCMMD_STAMP(p, 0);
  // generators of iteration tb-1 -> LDS (W 0..10, U 11..21, L_jj 22, m 23)
  const double* G = p.gen + size_t(b) * M1 * kGenStride;
  const float* gm = p.genm + size_t(b) * M1;
#pragma unroll 4
  for (int i = threadIdx.x; i < M1 * kGenStride; i += blockDim.x) Gl[i] = G[i];
  __syncthreads();
  for (int j = threadIdx.x; j < M1; j += blockDim.x) Gl[j * kGenStride + 23] = double(gm[j]);
  __syncthreads();
  MPCMMD_STAMP(p, 1);
  // rows 11..99: mean + L z (compute_beta.py:63), 64 samples per round
  const float* z = p.beta_z + size_t(tb - 1) * M1 * kNew;  // device layout [M+1][89]
  const int ys = ygen_stride(M);
  float* Y = p.ygen + size_t(b) * kNew * ys;
  const int bs = (M1 + nw - 1) / nw;
  const int j0 = min(M1, w * bs), j1 = min(M1, j0 + bs);
  for (int r0 = 0; r0 < kNew; r0 += 64) {
    const int ns = min(64, kNew - r0);
    const bool act = lane < ns;
    const int sz = r0 + (act ? lane : 0);
    // standard normals of this wave's positions, register double-buffered in
    // chunks of 16 positions (the next chunk's loads fly during the FMAs)
    auto load = [&](float* zc, int c0) {
#pragma unroll
      for (int q = 0; q < kZChunk; ++q) {
        const int j = min(c0 + q, M);
        zc[q] = z[size_t(j) * kNew + sz];
      }
    };
    double P[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) P[k] = 0.0;
    auto passA = [&](const float* zc, int c0) {
#pragma unroll
      for (int q = 0; q < kZChunk; ++q) {
        if (c0 + q >= j1) break;
        const double zj = double(zc[q]);
        const double* g = Gl + (c0 + q) * kGenStride;
#pragma unroll
        for (int k = 0; k < 11; ++k) P[k] = fma(g[k], zj, P[k]);
      }
    };
    float za[kZChunk], zb[kZChunk];
    load(za, j0);
    for (int c0 = j0; c0 < j1; c0 += 2 * kZChunk) {
      load(zb, c0 + kZChunk);
      passA(za, c0);
      load(za, c0 + 2 * kZChunk);
      passA(zb, c0 + kZChunk);
    }
#pragma unroll
    for (int k = 0; k < 11; ++k) Pbuf[(w * 11 + k) * 64 + lane] = P[k];
    __syncthreads();
    double S[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) {
      double c = 0.0;
      for (int w2 = 0; w2 < w; ++w2) c = c + Pbuf[(w2 * 11 + k) * 64 + lane];
      S[k] = c;
    }
    float* yrow = Y + size_t(sz) * ys;
    auto passB = [&](const float* zc, int c0) {
#pragma unroll
      for (int q = 0; q < kZChunk; ++q) {
        const int j = c0 + q;
        if (j >= j1) break;
        const double zj = double(zc[q]);
        const double* g = Gl + j * kGenStride;
        double d = 0.0;
#pragma unroll
        for (int k = 0; k < 11; ++k) d = fma(g[11 + k], S[k], d);
        const double yv = fma(g[22], zj, g[23]) + d;
#pragma unroll
        for (int k = 0; k < 11; ++k) S[k] = fma(g[k], zj, S[k]);
        if (act) yrow[j] = j == M ? fmaxf(float(yv), 0.01f) : float(yv);
      }
    };
    load(za, j0);
    for (int c0 = j0; c0 < j1; c0 += 2 * kZChunk) {
      load(zb, c0 + kZChunk);
      passB(za, c0);
      load(za, c0 + 2 * kZChunk);
      passB(zb, c0 + kZChunk);
    }
    __syncthreads();  // Pbuf reuse in the next round
    MPCMMD_STAMP(p, 2 + (r0 >> 6));
  }
}

// ------------------------------------------------------------------------
// k_bselect: top-n |beta| rows (compute_beta.py:117-118) and sigma of the
// 100 samples.  Latency-bound per wave (ballot chains), so it runs as many
// single-wave workgroups: wave (b, g) handles samples g, g+25, g+50, g+75.
constexpr int kSelGroups = 25;

__global__ __launch_bounds__(64) void k_bselect(Params p, int tb) {
  __shared__ int scratch[64];
  const int b = blockIdx.x, g = blockIdx.y, M = p.M, M1 = M + 1, n = p.n;
  int32_t* sel = p.bsel + size_t(b) * kBetaSamples * n;
  float* sig = p.bsig + size_t(b) * kBetaSamples;
  const float* E = p.belite + (size_t(tb & 1) * p.B + b) * kBetaElite * M1;
  const int ys = ygen_stride(M);
  const float* Y = p.ygen + size_t(b) * kNew * ys;
  const float* z0 = p.beta_z0;
  // sample s: initial MVN(0, 20 I) draws (tb = 0, compute_beta.py:41-49), the
  // previous elites (rows 0..10) or this iteration's new samples
  auto row = [&](int s) {
    const float* r = tb == 0 ? z0 + size_t(s) * M1 : (s < kBetaElite ? E + size_t(s) * M1 : Y + size_t(s - kBetaElite) * ys);
    const bool scale = tb == 0;
    return [=](int j) { return scale ? float(kSqrt20 * double(r[j])) : r[j]; };
  };
  select_rows(row, [&](int s) { return sel + s * n; }, g, kBetaSamples, kSelGroups, M, n, scratch);
  if (threadIdx.x < 4) {
    const int s = g + threadIdx.x * kSelGroups;
    const float v = row(s)(M);
    sig[s] = tb == 0 ? fmaxf(v, 0.01f) : v;  // later rows are clipped when written
  }
}

// ------------------------------------------------------------------------
// k_bkernel: one workgroup (1024 threads) per candidate.
//
//   rows     the distinct mother rows any sample selected (union, ~150 of 484
//            on average; every K_mixed row is a row of the M x M mother
//            distance matrix, kernel_computation.py:33-39)
//   D chunk  rows of the L1 distance matrix in LDS, register-tiled: a thread
//            owns one column j (its 22 features in registers) and walks the
//            chunk's rows, whose features are LDS broadcasts
//   pairs    (sample, reduced row) pairs sorted by row; a 16-lane group sums
//            exp(-D[r][j] / sigma_s) over j (v_exp_f32 on d * (-log2 e / sigma))
//   QP       2 samples per wave, lane = row: K_red (strict lower triangle
//            spread over the half-wave), left-looking fp64 Cholesky of
//            C = K_red + 0.05 I with the lane's row in registers, two
//            triangular solves (g and 1), beta = x1 + ((1 - sum x1)/sum x2) x2,
//            cost = beta^T K beta - 2 g^T beta with beta^T C beta = |L^T beta|^2
constexpr int kKerThreads = 1024;
constexpr int kFr = 24;  // row-major feature stride (floats): 22 + pad for b128 reads

struct KerLds {
  size_t Fr, sel, csg, rowsum, cnt, start, fill, ulist, urank, pairs, pair_s, work, total;
  int rows;  // D-chunk rows
};


HDI KerLds ker_lds(int M, int n, size_t budget) {
  KerLds L{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = (o + bytes + 15) & ~size_t(15);
    return at;
  };
  L.Fr = take(size_t(M) * kFr * 4);
  L.sel = take(size_t(kBetaSamples) * n * 2);
  L.csg = take(size_t(kBetaSamples) * 4);
  L.rowsum = take(size_t(kBetaSamples) * n * 8);
  L.cnt = take(size_t(M) * 4);
  L.start = take(size_t(M) * 4);
  L.fill = take(size_t(M) * 4);
  L.ulist = take(size_t(M) * 4);
  L.urank = take(size_t(M) * 4);
  L.pairs = take(size_t(kBetaSamples) * n * 2);
  L.pair_s = take(size_t(kBetaSamples) * n);
  L.work = o;
  const size_t rest = budget > o ? budget - o : 0;
  const int Ms = (M + 1) & ~1;  // even row stride: float2 reads
  int rows = int(rest / (size_t(Ms) * 4));
  if (rows > 128) rows = 128;
  L.rows = rows;
  L.total = o + size_t(rows) * Ms * 4;
  return L;
}

constexpr size_t kLdsBudget = 160 * 1024 - 1024;
constexpr float kNegLog2e = -1.44269504088896340736f;

// value of lane j of this half-wave (lanes 0..31 | 32..63), via readlane
DEVI double bcast_half(double v, int j, int hw) {
  const long long bits = __double_as_longlong(v);
  const int lo = int(bits), hi = int(bits >> 32);
  const int l0 = __builtin_amdgcn_readlane(lo, j), h0 = __builtin_amdgcn_readlane(hi, j);
  const int l1 = __builtin_amdgcn_readlane(lo, j + 32), h1 = __builtin_amdgcn_readlane(hi, j + 32);
  const long long r0 = (static_cast<long long>(h0) << 32) | static_cast<unsigned>(l0);
  const long long r1 = (static_cast<long long>(h1) << 32) | static_cast<unsigned>(l1);
  return __longlong_as_double(hw ? r1 : r0);
}

// sum_f |a_f - b_f| over the 22 features, sequential (oracle l1_dist order)
DEVI float l1_22(const float* a, const float* b) {
  float d = fabsf(a[0] - b[0]);
#pragma unroll
  for (int f = 1; f < kF; ++f) d = d + fabsf(a[f] - b[f]);
  return d;
}

DEVI void load_row(const float* Fr, int r, float* out) {
  const float4* s = reinterpret_cast<const float4*>(Fr + r * kFr);
#pragma unroll
  for (int q = 0; q < kFr / 4; ++q) {
    const float4 v = s[q];
    out[4 * q] = v.x;
    out[4 * q + 1] = v.y;
    out[4 * q + 2] = v.z;
    out[4 * q + 3] = v.w;
  }
}

__global__ __launch_bounds__(kKerThreads) void k_bkernel(Params p, int tb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, M = p.M, n = p.n;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const KerLds C = ker_lds(M, n, kLdsBudget);
  float* Fr = reinterpret_cast<float*>(smem + C.Fr);
  short* sl = reinterpret_cast<short*>(smem + C.sel);
  float* csg = reinterpret_cast<float*>(smem + C.csg);
  double* rowsum = reinterpret_cast<double*>(smem + C.rowsum);
  int* cnt = reinterpret_cast<int*>(smem + C.cnt);
  int* start = reinterpret_cast<int*>(smem + C.start);
  int* fill = reinterpret_cast<int*>(smem + C.fill);
  int* ulist = reinterpret_cast<int*>(smem + C.ulist);
  int* urank = reinterpret_cast<int*>(smem + C.urank);
  short* pairs = reinterpret_cast<short*>(smem + C.pairs);
  unsigned char* pair_s = reinterpret_cast<unsigned char*>(smem + C.pair_s);
  float* Dl = reinterpret_cast<float*>(smem + C.work);
  const float* Fg = p.feat + size_t(b) * kF * M;
  MPCMMD_STAMP(p, 16);
  // features [22][M] (global) -> rows [M][24] (LDS)
#pragma unroll 4
  for (int i = tid; i < kF * M; i += kKerThreads) {
    const int f = i / M, j = i - f * M;
    Fr[j * kFr + f] = Fg[i];
  }
  for (int j = tid; j < M; j += kKerThreads) Fr[j * kFr + 22] = Fr[j * kFr + 23] = 0.0f;
  const int32_t* gsel = p.bsel + size_t(b) * kBetaSamples * n;
  for (int i = tid; i < kBetaSamples * n; i += kKerThreads) sl[i] = short(gsel[i]);
  for (int s = tid; s < kBetaSamples; s += kKerThreads) csg[s] = kNegLog2e / p.bsig[size_t(b) * kBetaSamples + s];
  for (int r = tid; r < M; r += kKerThreads) {
    cnt[r] = 0;
    fill[r] = 0;
  }
  __syncthreads();
  for (int i = tid; i < kBetaSamples * n; i += kKerThreads) atomicAdd(&cnt[sl[i]], 1);
  __syncthreads();
  if (w == 0) {  // exclusive scans of cnt and (cnt > 0), one wave
    const int per = (M + 63) / 64, a = lane * per, e = min(M, a + per);
    int s1 = 0, s2 = 0;
    for (int r = a; r < e; ++r) {
      s1 += cnt[r];
      s2 += cnt[r] > 0;
    }
    int x1 = s1, x2 = s2;
    for (int o = 1; o < 64; o <<= 1) {
      const int y1 = __shfl_up(x1, o, 64), y2 = __shfl_up(x2, o, 64);
      if (lane >= o) {
        x1 += y1;
        x2 += y2;
      }
    }
    x1 -= s1;
    x2 -= s2;
    for (int r = a; r < e; ++r) {
      start[r] = x1;
      urank[r] = x2;
      if (cnt[r] > 0) ulist[x2] = r;
      x1 += cnt[r];
      x2 += cnt[r] > 0;
    }
  }
  __syncthreads();
  const int U = urank[M - 1] + (cnt[M - 1] > 0);
  if (tid == 0) atomicAdd(&p.stats[0], static_cast<unsigned long long>(U));
  for (int i = tid; i < kBetaSamples * n; i += kKerThreads) {
    const int r = sl[i];
    const int pos = start[r] + atomicAdd(&fill[r], 1);
    pairs[pos] = short(i);  // i = s * n + k
    pair_s[pos] = static_cast<unsigned char>(i / n);
  }
  // ---- K_mixed row sums, chunk by chunk
  const int R = C.rows;
  const int half = tid >> 9, jt = tid & 511;  // two threads per column, alternate rows
  const int Ms = (M + 1) & ~1;
  float fj[kFr];
  if (jt < M) load_row(Fr, jt, fj);
  __syncthreads();
  MPCMMD_STAMP(p, 17);
  const int g = tid >> 3, gl = tid & 7, ng = kKerThreads >> 3;  // 8 lanes per pair
  const int ntri = n * (n - 1) / 2;
  for (int c0 = 0; c0 < U; c0 += R) {
    const int rc = min(R, U - c0);
    for (int u = half; u < rc; u += 2) {
      float fr[kFr];
      load_row(Fr, ulist[c0 + u], fr);  // wave-uniform address: LDS broadcast
      const float d = l1_22(fr, fj);
      if (jt < M) Dl[u * Ms + jt] = d;
      if (jt == M && (M & 1)) Dl[u * Ms + jt] = __builtin_inff();  // pad: exp2(-inf) = 0
    }
    __syncthreads();
    if (c0 == 0) MPCMMD_STAMP(p, 18);
    const int p0 = start[ulist[c0]];
    const int p1 = start[ulist[c0 + rc - 1]] + cnt[ulist[c0 + rc - 1]];
    const int J = Ms >> 1;
    for (int pi = p0 + g; pi < p1; pi += ng) {
      const int i = pairs[pi];
      const int s = pair_s[pi];
      const int k = i - s * n;
      const float cn = csg[s];
      const int u = urank[sl[i]] - c0;
      const f2* drow = reinterpret_cast<const f2*>(Dl + size_t(u) * Ms);
      const f2 c2 = {cn, cn};
      f2 a0 = {0.0f, 0.0f}, a1 = {0.0f, 0.0f};
      int j = gl;
      for (; j + 8 < J; j += 16) {
        const f2 t0 = drow[j] * c2, t1 = drow[j + 8] * c2;
        a0 += f2{__builtin_amdgcn_exp2f(t0.x), __builtin_amdgcn_exp2f(t0.y)};
        a1 += f2{__builtin_amdgcn_exp2f(t1.x), __builtin_amdgcn_exp2f(t1.y)};
      }
      if (j < J) {
        const f2 t0 = drow[j] * c2;
        a0 += f2{__builtin_amdgcn_exp2f(t0.x), __builtin_amdgcn_exp2f(t0.y)};
      }
      a0 += a1;
      // K_red[s][k][kk] for kk < k: row t_k of the distance matrix is in the chunk
      const float* dr = Dl + size_t(u) * Ms;
      float* kr = p.bkred + (size_t(b) * kBetaSamples + s) * ntri + k * (k - 1) / 2;
      for (int kk = gl; kk < k; kk += 8) kr[kk] = __builtin_amdgcn_exp2f(dr[sl[s * n + kk]] * cn);
      float a = a0.x + a0.y;
      a += __shfl_xor(a, 1, 8);
      a += __shfl_xor(a, 2, 8);
      a += __shfl_xor(a, 4, 8);
      if (gl == 0) rowsum[i] = double(a);
    }
    __syncthreads();
    if (c0 == 0) MPCMMD_STAMP(p, 19);
  }
  for (int i = tid; i < kBetaSamples * n; i += kKerThreads) p.brow[size_t(b) * kBetaSamples * n + i] = rowsum[i];
  MPCMMD_STAMP(p, 20);
}

// ------------------------------------------------------------------------
// k_bqp: compute_beta_reduced (compute_beta.py:70-91) for every sample, 2
// samples per single-wave workgroup (half-waves, lane = row): left-looking
// fp64 Cholesky of C = K_red + 0.05 I with the lane's row in registers (NP =
// n rounded up to 8; padding rows are identity, their right-hand sides 0),
// two triangular solves (g and 1), beta = x1 + ((1 - sum x1)/sum x2) x2,
// cost = beta^T K beta - 2 g^T beta with beta^T C beta = |L^T beta|^2.
// Latency-bound chains, hence many small workgroups.
template <int NP>
DEVI void bqp_solve(const Params& p, double* Lp, double* rinv) {
  const int b = blockIdx.x, M = p.M, n = p.n, lane = threadIdx.x;
  const int hw = lane >> 5, li = lane & 31;
  const int s = blockIdx.y * 2 + hw;
  const int ntri = n * (n - 1) / 2;
  const double inv_m = double(1.0f / float(M));
  const double delta = double(1.0f + 0.05f) - 1.0;  // C_ii - K_ii (K_ii = exp(0) = 1)
  const bool sok = s < kBetaSamples;
  const int sc = sok ? s : 0;
  const bool act = sok && li < n;
  const bool row_ok = li < NP;
  const float* kr = p.bkred + (size_t(b) * kBetaSamples + sc) * ntri;
  // own row of C in registers
  double r[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    double v = 0.0;
    if (k < li && li < n) v = double(kr[li * (li - 1) / 2 + k]);
    if (k == li) v = li < n ? double(1.0f + 0.05f) : 1.0;
    r[k] = v;
  }
  const double gi = act ? p.brow[(size_t(b) * kBetaSamples + s) * n + li] * inv_m : 0.0;
  double* myrow = Lp + li * NP;
  // left-looking Cholesky: row j of L is read from LDS (broadcast)
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const double* rj = Lp + j * NP;
    double q0 = 0.0, q1 = 0.0;
#pragma unroll
    for (int k = 0; k + 1 < j; k += 2) {
      q0 = fma(r[k], rj[k], q0);
      q1 = fma(r[k + 1], rj[k + 1], q1);
    }
    if (j & 1) q0 = fma(r[j - 1], rj[j - 1], q0);
    const double sv = r[j] - (q0 + q1);
    if (li == j) {  // 1/sqrt by v_rsq_f64 + two Newton steps (no fp64 division)
      double y = __builtin_amdgcn_rsq(sv);
      y = y * fma(-0.5 * sv, y * y, 1.5);
      y = y * fma(-0.5 * sv, y * y, 1.5);
      const double d = sv * y;
      r[j] = d;
      rinv[j] = y;
      myrow[j] = d;
    }
    wave_sync();
    if (row_ok && li > j) {
      r[j] = sv * rinv[j];
      myrow[j] = r[j];
    }
    wave_sync();
  }
  // forward: L y = (g, 1); y_j handed to the half-wave through LDS
  double2* xb = reinterpret_cast<double2*>(rinv + NP);
  double a1 = gi, a2 = act ? 1.0 : 0.0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    if (li == j) {
      a1 = a1 * rinv[j];
      a2 = a2 * rinv[j];
      xb[j] = double2{a1, a2};
    }
    wave_sync();
    if (li > j) {
      const double2 y = xb[j];
      a1 = fma(-r[j], y.x, a1);
      a2 = fma(-r[j], y.y, a2);
    }
  }
  // backward: L^T x = y (column li of L from LDS)
#pragma unroll
  for (int j = NP - 1; j >= 0; --j) {
    if (li == j) {
      a1 = a1 * rinv[j];
      a2 = a2 * rinv[j];
      xb[j] = double2{a1, a2};
    }
    wave_sync();
    if (li < j) {
      const double lji = Lp[j * NP + li];
      const double2 x = xb[j];
      a1 = fma(-lji, x.x, a1);
      a2 = fma(-lji, x.y, a2);
    }
  }
  double s1 = act ? a1 : 0.0, s2 = act ? a2 : 0.0;
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    s1 += __shfl_xor(s1, o, 32);
    s2 += __shfl_xor(s2, o, 32);
  }
  const float beta = act ? float(a1 + ((1.0 - s1) / s2) * a2) : 0.0f;
  // cost = |L^T beta|^2 - delta |beta|^2 - 2 g^T beta
  const double bd = double(beta);
  double* bl = reinterpret_cast<double*>(xb + NP);
  if (li < NP) bl[li] = bd;
  wave_sync();
  double lt = 0.0;
#pragma unroll
  for (int k = 0; k < NP; ++k)
    if (k >= li && li < NP) lt = fma(Lp[k * NP + li], bl[k], lt);
  double c1 = act ? lt * lt : 0.0, c2 = act ? bd * bd : 0.0, c3 = act ? gi * bd : 0.0;
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    c1 += __shfl_xor(c1, o, 32);
    c2 += __shfl_xor(c2, o, 32);
    c3 += __shfl_xor(c3, o, 32);
  }
  if (act) p.btop[(size_t(b) * kBetaSamples + s) * n + li] = beta;
  if (sok && li == 0) p.bcost[size_t(b) * kBetaSamples + s] = float((c1 - delta * c2) - 2.0 * c3);
}

HDI int qp_np(int n) { return (n + 7) & ~7; }
// per half-wave: L rows (NP x NP doubles), 1/L_jj (NP), solve hand-off (2 NP), beta (NP)
HDI size_t qp_slot(int np) { return size_t(np) * np + 4 * np; }
HDI size_t ker_qp_bytes(int n) { return size_t(2) * qp_slot(qp_np(n)) * 8; }

__global__ __launch_bounds__(64) void k_bqp(Params p, int tb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int np = qp_np(p.n), hw = threadIdx.x >> 5;
  double* Lp = reinterpret_cast<double*>(smem) + size_t(hw) * qp_slot(np);
  double* rinv = Lp + np * np;
  switch (np) {
    case 8: return bqp_solve<8>(p, Lp, rinv);
    case 16: return bqp_solve<16>(p, Lp, rinv);
    case 24: return bqp_solve<24>(p, Lp, rinv);
    default: return bqp_solve<32>(p, Lp, rinv);
  }
}

// ------------------------------------------------------------------------
// k_belite: elites, mean, next generators; on the last iteration the outputs
// (beta_best, sigma_best with the post-update quirk Q4, the reduced set).
struct EliteLds {
  size_t U, Gb, misc, total;
};
HDI EliteLds elite_lds(int M1) {
  EliteLds L{};
  const int nblk = (M1 + 15) / 16;
  L.U = 0;
  L.Gb = (size_t(M1) * 11 * 8 + 15) & ~size_t(15);
  L.misc = L.Gb + ((size_t(nblk) * 66 * 8 + 15) & ~size_t(15));
  L.total = L.misc + 1024;
  return L;
}

// packed upper index of (a <= c) in an 11 x 11 symmetric matrix
HDI int sym11(int a, int c) { return a * 11 - a * (a - 1) / 2 + (c - a); }

__global__ __launch_bounds__(kThreads) void k_belite(Params p, int tb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, M = p.M, M1 = M + 1, n = p.n, tid = threadIdx.x;
  const EliteLds C = elite_lds(M1);
  double* Ul = reinterpret_cast<double*>(smem + C.U);
  double* Gb = reinterpret_cast<double*>(smem + C.Gb);
  int* elite = reinterpret_cast<int*>(smem + C.misc);    // [11]
  int* info = elite + 16;                                 // [0] imin, [1] any NaN
  float* cst = reinterpret_cast<float*>(info + 16);       // [100]
  const float* costs = p.bcost + size_t(b) * kBetaSamples;
  if (tid < kBetaSamples) cst[tid] = costs[tid];
  if (tid == 0) {
    info[0] = -1;
    info[1] = 0;
  }
  __syncthreads();
  if (tid < kBetaSamples) {
    const uint32_t ks = sort_key(cst[tid]);
    int r = 0;
    for (int k = 0; k < kBetaSamples; ++k) {
      const uint32_t kk = sort_key(cst[k]);
      r += (kk < ks) || (kk == ks && k < tid);
    }
    if (r < kBetaElite) elite[r] = tid;
    if (cst[tid] != cst[tid]) {
      atomicOr(&info[1], 1);
      atomicMin(reinterpret_cast<unsigned*>(&info[0]), unsigned(tid));  // first NaN (-1 == max)
    }
  }
  __syncthreads();
  const int imin = info[1] ? info[0] : elite[0];  // jnp.argmin: first NaN, else first minimum
  if (tid == 0) p.res_beta[size_t(b) * kBetaIters + tb] = info[1] ? __int_as_float(0x7fc00000) : cst[elite[0]];
  // ---- E_new = the 11 elite sample vectors (rows 0..10 of the next samples):
  // previous elites, this iteration's new samples (ygen), or at tb = 0 the
  // initial samples
  const float* Eold = p.belite + (size_t(tb & 1) * p.B + b) * kBetaElite * M1;
  float* Enew = p.belite + (size_t((tb + 1) & 1) * p.B + b) * kBetaElite * M1;
  const int ys = ygen_stride(M);
  const float* Y = p.ygen + size_t(b) * kNew * ys;
  for (int i = tid; i < kBetaElite * M1; i += blockDim.x) {
    const int q = i / M1, j = i - q * M1;
    const int e = elite[q];
    float v;
    if (tb == 0) {
      v = float(kSqrt20 * double(p.beta_z0[size_t(e) * M1 + j]));
      if (j == M) v = fmaxf(v, 0.01f);
    } else if (e < kBetaElite) {
      v = Eold[size_t(e) * M1 + j];
    } else {
      v = Y[size_t(e - kBetaElite) * ys + j];
    }
    Enew[i] = v;
  }
  __syncthreads();
  // ---- outputs of the beta-CEM on its last iteration (compute_beta.py:152-157)
  const bool last = tb == kBetaIters - 1;
  // ---- mean, U = (E - mean) / sqrt(10), generators of the next iteration
  const double rs10 = 1.0 / sqrt(10.0);
  double* gen = p.gen + size_t(b) * M1 * kGenStride;
  for (int j = tid; j < M1; j += blockDim.x) {
    double s = 0.0;
    for (int q = 0; q < kBetaElite; ++q) s = s + double(Enew[size_t(q) * M1 + j]);
    const double m = s / double(kBetaElite);
    for (int q = 0; q < kBetaElite; ++q) Ul[j * 11 + q] = (double(Enew[size_t(q) * M1 + j]) - m) * rs10;
    p.genm[size_t(b) * M1 + j] = float(m);
  }
  __syncthreads();
  // level 1: block sums of u u^T over 16 positions (66 packed entries)
  const int nblk = (M1 + 15) / 16;
  for (int i = tid; i < nblk * 66; i += blockDim.x) {
    const int blk = i / 66, e = i - blk * 66;
    int a = 0, c = e;
    while (c >= 11 - a) {
      c -= 11 - a;
      ++a;
    }
    c += a;
    double s = 0.0;
    const int k1 = min(M1, blk * 16 + 16);
    for (int k = blk * 16; k < k1; ++k) s += Ul[k * 11 + a] * Ul[k * 11 + c];
    Gb[i] = s;
  }
  __syncthreads();
  // block prefix: Gb[blk] <- Phi at the start of blk = I + sum_{<blk} / d
  if (tid < 66) {
    int a = 0, c = tid;
    while (c >= 11 - a) {
      c -= 11 - a;
      ++a;
    }
    c += a;
    double acc = a == c ? 1.0 : 0.0;
    for (int blk = 0; blk < nblk; ++blk) {
      const double g = Gb[blk * 66 + tid];
      Gb[blk * 66 + tid] = acc;
      acc = fma(g, kInvRidge, acc);
    }
  }
  __syncthreads();
  // level 2: per position Phi_j, Cholesky, v = Phi^-1 u_j, L_jj, w_j
  for (int j = tid; j < M1; j += blockDim.x) {
    const int blk = j >> 4;
    double A[66];
#pragma unroll
    for (int e = 0; e < 66; ++e) A[e] = Gb[blk * 66 + e];
    for (int k = blk * 16; k < j; ++k) {
      double uk[11];
#pragma unroll
      for (int a = 0; a < 11; ++a) uk[a] = Ul[k * 11 + a];
#pragma unroll
      for (int a = 0; a < 11; ++a) {
        const double ua = uk[a] * kInvRidge;
#pragma unroll
        for (int c = a; c < 11; ++c) A[sym11(a, c)] = fma(ua, uk[c], A[sym11(a, c)]);
      }
    }
    // Cholesky A = R^T R (R upper, stored in A; rinv = 1 / diag)
    double rinv[11];
#pragma unroll
    for (int a = 0; a < 11; ++a) {
      double d = A[sym11(a, a)];
#pragma unroll
      for (int k = 0; k < a; ++k) d = fma(-A[sym11(k, a)], A[sym11(k, a)], d);
      d = sqrt(d);
      A[sym11(a, a)] = d;
      rinv[a] = 1.0 / d;
#pragma unroll
      for (int c = a + 1; c < 11; ++c) {
        double s = A[sym11(a, c)];
#pragma unroll
        for (int k = 0; k < a; ++k) s = fma(-A[sym11(k, a)], A[sym11(k, c)], s);
        A[sym11(a, c)] = s * rinv[a];
      }
    }
    double u[11], v[11];
#pragma unroll
    for (int a = 0; a < 11; ++a) u[a] = Ul[j * 11 + a];
    // R^T y = u
#pragma unroll
    for (int a = 0; a < 11; ++a) {
      double s = u[a];
#pragma unroll
      for (int k = 0; k < a; ++k) s = fma(-A[sym11(k, a)], v[k], s);
      v[a] = s * rinv[a];
    }
    // R v = y
#pragma unroll
    for (int a = 10; a >= 0; --a) {
      double s = v[a];
#pragma unroll
      for (int k = a + 1; k < 11; ++k) s = fma(-A[sym11(a, k)], v[k], s);
      v[a] = s * rinv[a];
    }
    double uv = 0.0;
#pragma unroll
    for (int a = 0; a < 11; ++a) uv = fma(u[a], v[a], uv);
    const double ljj = sqrt(kRidge + uv);
    const double rl = 1.0 / ljj;
    double* g = gen + size_t(j) * kGenStride;
#pragma unroll
    for (int a = 0; a < 11; ++a) {
      g[a] = v[a] * rl;
      g[11 + a] = u[a];
    }
    g[22] = ljj;
  }
  if (!last) return;
  __syncthreads();
  // last iteration: beta_best / reduced set of argmin (pre-update), sigma_best
  // from the post-update samples at the same row (Q4, compute_beta.py:133-145)
  const int* bsel = p.bsel + (size_t(b) * kBetaSamples + imin) * n;
  for (int i = tid; i < n; i += blockDim.x) {
    p.bestsel[size_t(b) * n + i] = bsel[i];
    p.beta[size_t(b) * n + i] = p.btop[(size_t(b) * kBetaSamples + imin) * n + i];
  }
  if (imin < kBetaElite) {
    if (tid == 0) p.sigma[b] = Enew[size_t(imin) * M1 + M];
  } else {
    // sigma coordinate of new sample imin-11 drawn with the NEW generators:
    // y_M = mean_M + L_MM z_M + u_M . sum_{j<M} w_j z_j
    double* red = reinterpret_cast<double*>(smem + C.Gb);  // reuse
    const float* z = p.beta_z + size_t(tb) * M1 * kNew;
    const int si = imin - kBetaElite;
    double part[11];
#pragma unroll
    for (int a = 0; a < 11; ++a) part[a] = 0.0;
    for (int j = tid; j < M; j += blockDim.x) {
      const double zj = double(z[size_t(j) * kNew + si]);
#pragma unroll
      for (int a = 0; a < 11; ++a) part[a] += gen[size_t(j) * kGenStride + a] * zj;
    }
#pragma unroll
    for (int a = 0; a < 11; ++a) {
      part[a] = wave_sum(part[a]);
    }
    __syncthreads();
    if ((tid & 63) == 0)
#pragma unroll
      for (int a = 0; a < 11; ++a) red[(tid >> 6) * 11 + a] = part[a];
    __syncthreads();
    if (tid == 0) {
      const double* g = gen + size_t(M) * kGenStride;
      double d = 0.0;
      for (int a = 0; a < 11; ++a) {
        double sa = 0.0;
        for (int w2 = 0; w2 < (int)(blockDim.x >> 6); ++w2) sa += red[w2 * 11 + a];
        d += g[11 + a] * sa;
      }
      const double zM = double(z[size_t(M) * kNew + si]);
      const float yM = float((double(p.genm[size_t(b) * M1 + M]) + g[22] * zM) + d);
      p.sigma[b] = fmaxf(yM, 0.01f);
    }
  }
}

// ------------------------------------------------------------------------
// k_mmdfinal: x_red / y_red of the best reduced set (compute_beta.py:465),
// compute_mmd_obs (costs.py:173-186) and compute_mmd_lane (costs.py:121-135).
__global__ __launch_bounds__(64) void k_mmdfinal(Params p, int t) {
  __shared__ float cb[kMaxReduced], lb[kMaxReduced], ub[kMaxReduced], bt[kMaxReduced];
  __shared__ ReduceScratch rs;
  const int b = blockIdx.x, n = p.n, H = p.H, O = p.O, lane = threadIdx.x;
  const float* ctrl = p.ctrl_n + size_t(b) * 2 * n * H;
  if (lane < n) {
    const int m = p.bestsel[size_t(b) * n + lane];
    const float* ar = ctrl + (m / n) * H;
    const float* sr = ctrl + n * H + (m % n) * H;
    float x = p.st0[0], y = p.st0[1], vx = p.st0[2], vy = p.st0[3], psi = p.st0[4];
    float c = 0.0f, l = 0.0f, u = 0.0f;
    bool nan = false;
    for (int h = 0; h < H; ++h) {
      for (int o = 0; o < O; ++o) {
        const float f = f_bar(x, y, p.obs[o * H + h], p.obs[O * H + o * H + h]);
        nan |= (f != f);
        c = fmaxf(c, f);
      }
      nan |= (y != y);
      l = fmaxf(l, -y + p.y_lb);
      u = fmaxf(u, y - p.y_ub);
      if (h == H - 1) break;
      bicycle_step(x, y, vx, vy, psi, ar[h], sr[h]);
    }
    const float qnan = __int_as_float(0x7fc00000);
    cb[lane] = nan ? qnan : c;
    lb[lane] = nan ? qnan : l;
    ub[lane] = nan ? qnan : u;
    bt[lane] = p.beta[size_t(b) * n + lane];
  }
  __syncthreads();
  const float sigma = p.sigma[b];
  const float obs = block_mmd(cb, bt, n, sigma, 1000.0f, rs);
  const float ml = block_mmd(lb, bt, n, sigma, 1000.0f, rs);
  const float mu = block_mmd(ub, bt, n, sigma, 1000.0f, rs);
  if (lane == 0) {
    p.obs_cost[b] = obs;
    p.lane_cost[b] = ml + mu;
  }
}



}  // namespace

bool mmdopt_supported(int n, int H, int O, std::string* why) {
  const int M = n * n;
  if (n > kMaxReduced) {
    if (why) *why = "mmd_opt needs num_reduced <= 32";
    return false;
  }
  const KerLds k = ker_lds(M, n, kLdsBudget);
  if (k.rows < 1 || k.total > kLdsBudget) {
    if (why) *why = "mmd_opt: num_reduced^2 too large for the LDS-resident kernel-sum stage";
    return false;
  }
  const EliteLds e = elite_lds(M + 1);
  if (bs_lds(M + 1) > kLdsBudget) {
    if (why) *why = "mmd_opt: num_reduced^2 too large for the sampling stage";
    return false;
  }
  if (e.total > kLdsBudget) {
    if (why) *why = "mmd_opt: num_reduced^2 too large for the elite stage";
    return false;
  }
  (void)H;
  (void)O;
  return true;
}

void launch_mother(const Params& p, int t, hipStream_t s) {
  hipLaunchKernelGGL(k_mother, dim3(p.B), dim3(kThreads), size_t(2) * p.n * p.H * 4, s, p, t);
}

void launch_bsample(const Params& p, int tb, hipStream_t s) {
  hipLaunchKernelGGL(k_bsample, dim3(p.B), dim3(kThreads), bs_lds(p.M + 1), s, p, tb);
}

void launch_bselect(const Params& p, int tb, hipStream_t s) {
  hipLaunchKernelGGL(k_bselect, dim3(p.B, kSelGroups), dim3(64), 0, s, p, tb);
}

void launch_bqp(const Params& p, int tb, hipStream_t s) {
  hipLaunchKernelGGL(k_bqp, dim3(p.B, kBetaSamples / 2), dim3(64), ker_qp_bytes(p.n), s, p, tb);
}

void launch_bkernel(const Params& p, int tb, hipStream_t s) {
  const KerLds k = ker_lds(p.M, p.n, kLdsBudget);
  hipLaunchKernelGGL(k_bkernel, dim3(p.B), dim3(kKerThreads), k.total, s, p, tb);
}

void launch_belite(const Params& p, int tb, hipStream_t s) {
  const EliteLds e = elite_lds(p.M + 1);
  hipLaunchKernelGGL(k_belite, dim3(p.B), dim3(kThreads), e.total, s, p, tb);
}

void launch_mmdfinal(const Params& p, int t, hipStream_t s) {
  hipLaunchKernelGGL(k_mmdfinal, dim3(p.B), dim3(64), 0, s, p, t);
}

}  // namespace mpcmmd
