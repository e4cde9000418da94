// Stage "risk" for cost = mmd_opt: the mother rollouts, their Bernstein fit
// and the nested beta-CEM that picks the reduced set and the MMD weights,
// then the reduced-set MMD.  Per outer iteration:
//
//   k_mother    noisy control rows, n^2 mother rollouts (Cartesian product,
//               cem_helper.py:469-530) with the ridge fit folded into the scan
//               (compute_coeff, cem_helper.py:553-564) -> 22 features per row
//   k_bdist     the M x M L1 distance matrix of the features (once)
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
// The beta-iteration kernels work on a candidate range [p.b0, p.b0 + p.nb):
// the host splits the batch into groups, each on its own stream, so the
// kernels of different groups (bound by different units: MFMA, exp, fp64
// FMA latency, LDS) run side by side.  Every supported size n <= 64
// (M = n^2 <= 4096) takes the same kernels; the LDS-resident pieces are sized
// at launch (ker_lds, dir_lds, elite_lds).
//
// The covariance of the beta-CEM is rank <= 10 plus 0.05 I
// (jnp.cov of 11 elites, compute_beta.py:61).  Its Cholesky factor is never
// formed: with U = (E - mean)^T / sqrt(10), Phi_j = I + U_{<j}^T U_{<j} / d,
// v_j = Phi_j^-1 u_j, L_jj = sqrt(d + u_j.v_j), w_j = v_j / L_jj, one has
// L_ij = u_i . w_j (i > j), so (L z)_i = L_ii z_i + u_i . sum_{j<i} w_j z_j.
// Same factor as chol(cov) in exact arithmetic, O(M r^2) instead of O(M^3).
#include <cstdlib>

#include "block.hpp"
#include "kernels.hpp"
#include "rng.hpp"
#include "rollout.hpp"

namespace mpcmmd {

namespace {

// The thread's index.  The small-batch fused kernel (k_bcem_small.hip, which
// compiles this file with MPCMMD_FUSED_TU) runs every phase inside one loop
// over the beta-iterations; there each read is opaque, so nothing computed
// from the index is hoisted out of the loop and held in registers across the
// other phases (spills).  The per-iteration kernels read threadIdx.x.
#ifdef MPCMMD_FUSED_TU
DEVI unsigned tidx() {
  unsigned t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
#else
DEVI unsigned tidx() { return threadIdx.x; }
#endif

constexpr int kF = 22;                               // features: cx (11) | cy (11)
constexpr int kNew = kBetaSamples - kBetaElite;      // 89 resampled rows per iteration
constexpr int kThreads = 512;
constexpr double kSqrt20 = 4.47213595499957927704;   // chol(20 I) (compute_beta.py:24)
constexpr double kRidge = 0.05;                      // cov jitter (compute_beta.py:61)
constexpr double kInvRidge = 20.0;

// first sample a beta-iteration processes: from the second iteration on,
// samples 0..10 are the previous iteration's elites, unchanged, and k_belite
// carries their top-n rows, sigma, QP solution and cost
HDI int first_sample(int tb) { return tb > 0 ? kBetaElite : 0; }

#define kconst __attribute__((address_space(4)))
typedef float f2 __attribute__((ext_vector_type(2)));

// Intra-wave LDS hand-off: a wave's LDS operations execute in order, so only
// the compiler must be kept from reordering them (no memory-counter waits).
DEVI void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  __asm__ volatile("" ::: "memory");
}

// sum over each row of 16 lanes (every lane of the row holds it)
DEVI double row16_sum(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x124>(v);
  return v + dpp_d<0x128>(v);
}

// Negative-control builds (tools/perturb_kred.sh): a deliberately wrong K_red
// entry, so the parity tests can be shown to catch a kernel error.  Entry 0
// of every sample: MPCMMD_PERTURB_KRED=1 scales it by 1.001, =2 flips its
// mantissa bit 10 (a 1.2e-4 relative change).  Off in every product build.
DEVI float kred_perturb(float v, int e) {
#if defined(MPCMMD_PERTURB_KRED) && MPCMMD_PERTURB_KRED == 1
  return e == 0 ? v * 1.001f : v;
#elif defined(MPCMMD_PERTURB_KRED) && MPCMMD_PERTURB_KRED == 2
  return e == 0 ? __int_as_float(__float_as_int(v) ^ (1 << 10)) : v;
#else
  (void)e;
  return v;
#endif
}

// ------------------------------------------------------------------------
// k_mother
#ifndef MPCMMD_FUSED_TU
// CARLA (the fp64 tan / per-row initial states) and the static rollouts as two
// instantiations: the static one's registers no longer carry the CARLA path
// (166 -> fewer VGPRs, SGPR spills gone: two 512-thread workgroups per CU)
#ifndef MPCMMD_MOTHER_WAVES
#define MPCMMD_MOTHER_WAVES 1
#endif
template <bool CARLA>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(CARLA ? 1 : MPCMMD_MOTHER_WAVES))) void k_mother(Params p, int t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = p.n, H = p.H, M = p.M, b = blockIdx.x;
  const Cfg cf = cfg_of(p, b / p.B);
  float* an = reinterpret_cast<float*>(smem);
  float* sn = an + n * H;
  float* tn = sn + n * H;  // CARLA: float(tan(double(steer))) of each control, off the rows' step chains
  // the Bernstein fit rows by step, [H][11] doubles: a step's eleven factors as
  // LDS broadcasts, not a scalar-load latency inside every step of the chain
  double* fitl = reinterpret_cast<double*>(smem + ((size_t(3) * n * H * 4 + 15) & ~size_t(15)));
  for (int idx = tidx(); idx < 11 * H; idx += blockDim.x) {
    const int h = idx / 11, k = idx - h * 11;
    fitl[idx] = p.fit[k * H + h];
  }
  float* gctrl = p.ctrl_n + size_t(b) * 2 * n * H;
  for (int idx = tidx(); idx < n * H; idx += blockDim.x) {
    const int r = idx / H, h = idx % H;
    float a, s;
    noisy_control(p, cf, t, r, h, p.acc[size_t(b) * 100 + h], p.steer[size_t(b) * 100 + h], a, s);
    an[idx] = a;
    sn[idx] = s;
    if constexpr (CARLA) tn[idx] = float(tan(double(s)));
    gctrl[idx] = a;
    gctrl[n * H + idx] = s;
  }
  __syncthreads();
  float* F = p.feat + size_t(b) * kF * M;
  for (int m = tidx(); m < M; m += blockDim.x) {
    // jnp.repeat(acc, n, 0) / jnp.tile(steer, (n, 1)) (cem_helper.py:510-511)
    const float* ar = an + (m / n) * H;
    const float* sr = sn + (m % n) * H;
    const float* tr = tn + (m % n) * H;
    // CARLA: every mother row starts from its own noisy initial state
    // (carla/optimizer/cem.py:251-253, cem_helper.py:846)
    const float* st = CARLA ? p.st0r + (size_t(cf.g) * p.R0 + m) * 8 : cf.st0;
    float x = st[0], y = st[1], vx = st[2], vy = st[3], psi = st[4];
    double cx[11], cy[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) cx[k] = cy[k] = 0.0;
    for (int h = 0; h < H; ++h) {
      const double dx = double(x), dy = double(y);
#pragma unroll
      for (int k = 0; k < 11; ++k) {
        const double f = fitl[h * 11 + k];
        cx[k] = cx[k] + f * dx;
        cy[k] = cy[k] + f * dy;
      }
      if (h == H - 1) break;
      if constexpr (CARLA) bicycle_step_cr_t(x, y, vx, vy, psi, ar[h], tr[h], p.wheel_base);
      else bicycle_step(x, y, vx, vy, psi, ar[h], sr[h]);
    }
    float fr[kFeatStride];
#pragma unroll
    for (int k = 0; k < 11; ++k) {
      fr[k] = float(cx[k]);
      fr[11 + k] = float(cy[k]);
      F[k * M + m] = fr[k];
      F[(11 + k) * M + m] = fr[11 + k];
    }
    fr[22] = fr[23] = 0.0f;
    float4* Fr = reinterpret_cast<float4*>(p.featr + (size_t(b) * M + m) * kFeatStride);
#pragma unroll
    for (int q = 0; q < kFeatStride / 4; ++q) Fr[q] = make_float4(fr[4 * q], fr[4 * q + 1], fr[4 * q + 2], fr[4 * q + 3]);
  }
}
#endif

// ------------------------------------------------------------------------
// k_bdist: the L1 distance matrix of the mother features,
// D[a][b] = sum_f |F_a,f - F_b,f| (kernel_computation.py:33-39 with the
// 22-dim features of compute_beta.py:120-124), once per outer iteration.
// Every K_mixed / K_red entry the 20 beta-iterations need is exp(-D[a][b] /
// sigma) for a selected row a, so the rows are computed once here instead
// of 20 times.  Workgroup = (candidate, tile of kDistRows rows); a thread
// owns one column (its 22 features in registers), the tile's row features
// are LDS broadcasts; the feature sum is sequential (the oracle's order).
// Pad columns M..Md-1 hold +inf so exp2(-inf) = 0 in the row sums (written
// once per handle by k_dist_pad).
constexpr int kDistRows = 32;
constexpr int kDistThreads = 256;

// XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs by
// linear id, so id L runs on XCD L % 8.  Candidate b's row tiles get ids
// ((b / 8) * T + tile) * 8 + b % 8: all on one XCD and launched together, so
// the candidate's column features (42 KB) are read from HBM once and then
// hit that XCD's L2, instead of once per tile.
constexpr int kXcds = 8;
constexpr int kCUs = 256;  // MI355X compute units (launch sizing only)

// The matrix is symmetric and |a - b| == |b - a| exactly, so a tile of rows
// computes only the columns from its own first row on and also writes the
// mirrored entries D[j][r0 .. r0 + 31] of every later column j: half the
// VALU work of the full matrix, same bits.  The mirrored 32-entry pieces go
// through LDS, so each store instruction writes whole 128-byte rows (eight
// lanes per row) instead of 16 bytes to 64 rows.
constexpr int kMirrorPitch = kDistRows + 4;  // floats per staged row (16-byte aligned, spreads banks)

#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(kDistThreads) void k_bdist(Params p) {
  __shared__ __attribute__((aligned(16))) float Fr[kDistRows][kF + 2];
  __shared__ __attribute__((aligned(16))) float Tm[kDistThreads * kMirrorPitch];
  const int M = p.M, Md = dist_stride(M), T = (M + kDistRows - 1) / kDistRows;
  const int L = blockIdx.x, q = L / kXcds;
  const int b = (q / T) * kXcds + L % kXcds, r0 = (q % T) * kDistRows;
  if (b >= p.Bt) return;
  const int tid = tidx();
  const float* Fg = p.feat + size_t(b) * kF * M;
  for (int i = tid; i < kDistRows * kF; i += kDistThreads) {
    const int r = i / kF, f = i - r * kF;
    Fr[r][f] = r0 + r < M ? Fg[f * M + r0 + r] : 0.0f;
  }
  __syncthreads();
  const int rn = min(kDistRows, M - r0);
  float* Db = p.bdist + size_t(b) * M * Md;
  float* D = Db + size_t(r0) * Md;
  // a later real column exists only if this tile is full (r0 + 32 < M)
  for (int j0 = r0; j0 < Md; j0 += kDistThreads) {  // wave-uniform trip count
    const int j = j0 + tid;
    if (j < Md) {
      float fj[kF];
      const int jc = min(j, M - 1);
#pragma unroll
      for (int f = 0; f < kF; ++f) fj[f] = Fg[f * M + jc];
      for (int rg = 0; rg < kDistRows / 4; ++rg) {
        float dv[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = 4 * rg + rr;
          if (r < rn) {
            const float* fr = Fr[r];  // wave-uniform: LDS broadcast
            // the differences two features at a time (v_pk_add_f32: the same
            // roundings as two v_sub_f32), the sum sequential as before
            static_assert(kF % 2 == 0, "feature pairs");
            f2 df = f2{fr[0], fr[1]} - f2{fj[0], fj[1]};
            float d = fabsf(df.x);
            d = d + fabsf(df.y);
#pragma unroll
            for (int f = 2; f < kF; f += 2) {
              df = f2{fr[f], fr[f + 1]} - f2{fj[f], fj[f + 1]};
              d = d + fabsf(df.x);
              d = d + fabsf(df.y);
            }
#if defined(MPCMMD_BDIST_VARIANT) && MPCMMD_BDIST_VARIANT == 2
            if (d == -1.0f) D[size_t(r) * Md + j] = d;  // timing build: no row stores
#else
            if (j < M) D[size_t(r) * Md + j] = d;  // pad columns: +inf once per handle (k_dist_pad)
#endif
            dv[rr] = d;
          }
        }
        *reinterpret_cast<float4*>(&Tm[tid * kMirrorPitch + 4 * rg]) = make_float4(dv[0], dv[1], dv[2], dv[3]);
      }
    }
#if defined(MPCMMD_BDIST_VARIANT) && MPCMMD_BDIST_VARIANT >= 1
    continue;  // timing builds (tools/bdist_variants.sh): no mirror phase
#endif
    __syncthreads();
    // rows j0 + c (c < 256) of the mirror: 8 lanes per row, 16 bytes each
    for (int i = tid; i < kDistThreads * (kDistRows / 4); i += kDistThreads) {
      const int c = i >> 3, part = i & 7, jj = j0 + c;
      if (jj >= r0 + kDistRows && jj < M)
        *reinterpret_cast<float4*>(Db + size_t(jj) * Md + r0 + 4 * part) =
            *reinterpret_cast<const float4*>(&Tm[c * kMirrorPitch + 4 * part]);
    }
    __syncthreads();
  }
}
#endif

// ------------------------------------------------------------------------
// k_bmoment: the series record of every distance row (once per outer
// iteration, after k_bdist).  A K_mixed row sum of sample s over the mother
// set (kernel_computation.py:33-39, 45; compute_beta.py:75) is
//   S(r, c) = sum_j exp(-c D[r][j]),  c = 1 / sigma_s.
// With R = max_j D[r][j] / 2, t_j = D[r][j] / R - 1 in [-1, 1] and a = c R,
//   S = exp(-a) sum_j exp(-a t_j) = exp(-a) sum_{k < 12} (-a)^k / k! P_k + E,
//   P_k = sum_j t_j^k,   |E| / S <= e^{2a} a^12 / 12!
// (each term's Taylor remainder is <= a^12 e^a / 12! while each term is
// >= e^-a), i.e. <= 1.5e-8 for a <= 1: below half an fp32 ulp, so the
// series is as exact as the reference's fp32 exponentials and sum.  P_k
// depends on the row only; k_bkernel then pays a 12-term Horner sum per
// (sample, row) pair instead of M exponentials (pairs with a > 1 are summed
// directly).  One wave per row: the row as float4s in registers, the row max
// by DPP, t and its powers in packed fp32 (the column pairs of a float4 as
// one v_pk_* operand), one wave sum per moment.  Pad columns (+inf) count 0.
// The first beta-iteration's pairs of the row (Params::rp0, the handle's
// table) whose a > 1 are summed here directly, from the row already in
// registers, instead of re-reading it in k_bdirect.
constexpr int kMomRowsPerBlock = 4;
constexpr double kSeriesAMaxRow = 1.0;                     // == kSeriesAMax (k_bkernel)
constexpr float kNegLog2eRow = -1.44269504088896340736f;   // == kNegLog2e

// wave totals of 16 per-lane values: lane l ends with the total of v[l >> 2].
// Each butterfly step halves the values a lane carries (permlane32 / permlane16
// swaps, then row_mirror and row_half_mirror DPP with the kept half chosen by
// the lane bit the pairing flips, then the quad), ~35 VALU for all 16 totals
// instead of a 7-step reduction per value.
DEVI float wave_totals16(const float (&v)[16]) {
  const int lane = tidx() & 63;
  float w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // lanes < 32 keep values 0..7, lanes >= 32 values 8..15
    float a = v[i], b = v[i + 8];
    permlane_swap<32>(a, b);
    w[i] = a + b;
  }
  float x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // odd rows keep the upper four
    float a = w[i], b = w[i + 4];
    permlane_swap<16>(a, b);
    x[i] = a + b;
  }
  const bool b3 = lane & 8, b2 = lane & 4;
  float y[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // row_mirror pairs l with l ^ 15 (bit 3 flipped)
    const float keep = b3 ? x[i + 2] : x[i], send = b3 ? x[i] : x[i + 2];
    y[i] = keep + __int_as_float(dpp_i<0x140>(__float_as_int(send)));
  }
  // row_half_mirror pairs l with l ^ 7 (bit 2 flipped)
  float z = (b2 ? y[1] : y[0]) + __int_as_float(dpp_i<0x141>(__float_as_int(b2 ? y[0] : y[1])));
  z += __int_as_float(dpp_i<0xB1>(__float_as_int(z)));
  return z + __int_as_float(dpp_i<0x4E>(__float_as_int(z)));
}

// one distance row (global row index gw over the launch's candidates) held in x
// Its first-iteration pairs: rpair0[q0 .. q1), lane L's record of the first 64
// (pr) loaded with the row, ahead of it.
struct RowPairs {
  int q0, q1;
  int2 pr;
};

DEVI RowPairs load_row_pairs(const Params& p, int r) {
  const int lane = tidx() & 63;
  RowPairs rp;
  rp.q0 = p.rp0[r];
  rp.q1 = p.rp0[r + 1];
  rp.pr = p.rpair0[max(min(rp.q0 + lane, rp.q1 - 1), 0)];  // a row without pairs reads a valid record, unused
  return rp;
}

template <int NV4>
DEVI void bmoment_row(const Params& p, int gw, const float4 (&x)[NV4], const RowPairs& rq) {
  const int lane = tidx() & 63;
  const int M = p.M;
  const int b = gw / M, r = gw - b * M;
  // columns j = 4 (lane + 64 t) + c; pad columns j >= M
  auto valid = [&](int t, int c) { return 4 * (lane + 64 * t) + c < M; };
  float mx = 0.0f;
#pragma unroll
  for (int t = 0; t < NV4; ++t) {
    if (valid(t, 0)) mx = fmaxf(mx, x[t].x);
    if (valid(t, 1)) mx = fmaxf(mx, x[t].y);
    if (valid(t, 2)) mx = fmaxf(mx, x[t].z);
    if (valid(t, 3)) mx = fmaxf(mx, x[t].w);
  }
  const float R = 0.5f * wave_max(mx);
  const float invR = R > 0.0f ? 1.0f / R : 0.0f;  // R = 0: every t = -1, every a = 0
  f2 acc[kMom - 1];
#pragma unroll
  for (int k = 0; k < kMom - 1; ++k) acc[k] = f2{0.0f, 0.0f};
#pragma unroll
  for (int t = 0; t < NV4; ++t) {
    const float e[4] = {x[t].x, x[t].y, x[t].z, x[t].w};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float t0 = valid(t, 2 * h) ? fmaf(e[2 * h], invR, -1.0f) : 0.0f;
      const float t1 = valid(t, 2 * h + 1) ? fmaf(e[2 * h + 1], invR, -1.0f) : 0.0f;
      const f2 tt = {t0, t1};
      f2 pw = tt;
#pragma unroll
      for (int k = 0; k < kMom - 1; ++k) {
        acc[k] += pw;
        if (k + 1 < kMom - 1) pw *= tt;
      }
    }
  }
  static_assert(kMomStride == 16 && kMomR < 16 && kMom == kMomR, "record slots");
  float v[16];  // slot k + 1 of the record: P_{k+1}
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = k >= 1 && k < kMom ? acc[k - 1].x + acc[k - 1].y : 0.0f;
  const int slot = lane >> 2;  // lanes 4 s .. 4 s + 3 hold slot s
  float rec = wave_totals16(v);
  if (slot == 0) rec = float(M);
  if (slot == kMomR) rec = R;
  if ((lane & 3) == 0) p.bmom[(size_t(b) * M + r) * kMomStride + slot] = rec;
  // first-iteration pairs of this row that the series does not cover (the
  // test is k_bkernel's, on the same R and sigma)
  const int n = p.n;
  float* rowsum = p.brow + size_t(b) * kBetaSamples * n;
  const int q0 = rq.q0, q1 = rq.q1;
  for (int c0 = q0; c0 < q1; c0 += 64) {  // one (index, sigma) record per lane
    const int2 pr = c0 == q0 ? rq.pr : p.rpair0[min(c0 + lane, q1 - 1)];
    const int il = pr.x;
    const float sl = __int_as_float(pr.y);
    const bool dl = !(double(R) * (1.0 / double(sl)) <= p.mom_amax) && c0 + lane < q1;
    unsigned long long todo = __ballot(dl);
    while (todo) {  // wave-uniform
      const int j = __builtin_ctzll(todo);
      todo &= todo - 1;
      const int i = __builtin_amdgcn_readlane(il, j);
      const float sg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sl), j));
      const float cs = kNegLog2eRow / sg;
      const f2 c2 = {cs, cs};
      f2 acc2 = {0.0f, 0.0f};
#pragma unroll
      for (int t = 0; t < NV4; ++t) {  // pad columns: +inf * cs = -inf -> 0
        const f2 t0 = f2{x[t].x, x[t].y} * c2, t1 = f2{x[t].z, x[t].w} * c2;
        acc2 += f2{__builtin_amdgcn_exp2f(t0.x), __builtin_amdgcn_exp2f(t0.y)};
        acc2 += f2{__builtin_amdgcn_exp2f(t1.x), __builtin_amdgcn_exp2f(t1.y)};
      }
      const float sum = wave_total(acc2.x + acc2.y);
      if (lane == 0) rowsum[i] = sum;
    }
  }
}

// rows per wave: the next row's loads are issued before the current row is
// processed (a wave no longer waits one full memory latency per row)
template <int NV4>
constexpr int mom_rows_per_wave() { return NV4 <= 2 ? 4 : (NV4 <= 4 ? 2 : 1); }

#ifndef MPCMMD_FUSED_TU
template <int NV4>
__global__ __launch_bounds__(64 * kMomRowsPerBlock) void k_bmoment(Params p) {
  constexpr int RPW = mom_rows_per_wave<NV4>();
  const int lane = tidx() & 63;
  const int total = p.Bt * p.M, Md = dist_stride(p.M);
  const int g0 = (blockIdx.x * kMomRowsPerBlock + (tidx() >> 6)) * RPW;
  if (g0 >= total) return;  // wave-uniform
  auto load = [&](float4 (&x)[NV4], int g) {
    const float4* row = reinterpret_cast<const float4*>(p.bdist + size_t(g) * Md) + lane;  // rows of all candidates are consecutive
#pragma unroll
    for (int t = 0; t < NV4; ++t) x[t] = row[64 * t];
  };
  const int M = p.M;
  float4 x[NV4], xn[NV4];
  RowPairs rq = load_row_pairs(p, g0 % M), rqn;
  load(x, g0);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int g = g0 + i;
    if (g >= total) break;  // wave-uniform
    if (i + 1 < RPW) {  // the next row's pair records, then its distances
      const int gn = min(g + 1, total - 1);
      rqn = load_row_pairs(p, gn % M);
      load(xn, gn);
    }
    bmoment_row<NV4>(p, g, x, rq);
    if (i + 1 < RPW) {
      rq = rqn;
#pragma unroll
      for (int t = 0; t < NV4; ++t) x[t] = xn[t];
    }
  }
}
#endif

// k_bmoment_rows: the same series records (and first-iteration direct sums)
// with a distance row on one 16-lane DPP row instead of a whole wave: four
// rows per wave, NV float4s (4 NV columns) per lane.  The per-row work that
// does not scale with the row length -- the maximum, the division, the
// totals of the eleven moments, the record store -- is then shared by four
// times the columns per lane: 16-lane reductions (two quad_perm and two
// row_ror DPP steps) instead of 64-lane ones, and the eleven totals by one
// transposing butterfly over the row (row_mirror, row_half_mirror and the
// two quad pairings: lane l ends with slot l of the record).  Same values as
// bmoment_row up to the summation order of the moments and direct sums.
// Columns j = 4 (l + 16 t) + c, l = lane & 15.
DEVI float row16_max(float v) {
  v = fmaxf(v, dpp_keep_f<0xB1>(v));
  v = fmaxf(v, dpp_keep_f<0x4E>(v));
  v = fmaxf(v, dpp_keep_f<0x124>(v));
  return fmaxf(v, dpp_keep_f<0x128>(v));
}
DEVI float row16_total(float v) {
  v += __int_as_float(dpp_i<0xB1>(__float_as_int(v)));
  v += __int_as_float(dpp_i<0x4E>(__float_as_int(v)));
  v += __int_as_float(dpp_i<0x124>(__float_as_int(v)));
  return v + __int_as_float(dpp_i<0x128>(__float_as_int(v)));
}
// 16 per-lane values -> lane l (of each 16-lane row) holds the row total of v[l & 15]
DEVI float row16_totals16(const float (&v)[16]) {
  const int lane = tidx() & 15;
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  float y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // row_mirror: l <-> 15 - l (bit 3 flipped)
    const float keep = b3 ? v[i + 8] : v[i], send = b3 ? v[i] : v[i + 8];
    y[i] = keep + __int_as_float(dpp_i<0x140>(__float_as_int(send)));
  }
  float z[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // row_half_mirror: l <-> l ^ 7 (bit 2 flipped)
    const float keep = b2 ? y[i + 4] : y[i], send = b2 ? y[i] : y[i + 4];
    z[i] = keep + __int_as_float(dpp_i<0x141>(__float_as_int(send)));
  }
  float w[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // quad_perm(2,3,0,1): l <-> l ^ 2
    const float keep = b1 ? z[i + 2] : z[i], send = b1 ? z[i] : z[i + 2];
    w[i] = keep + __int_as_float(dpp_i<0x4E>(__float_as_int(send)));
  }
  const float keep = b0 ? w[1] : w[0], send = b0 ? w[0] : w[1];  // quad_perm(1,0,3,2): l <-> l ^ 1
  return keep + __int_as_float(dpp_i<0xB1>(__float_as_int(send)));
}

template <int NV>
DEVI void bmoment_row16(const Params& p, int g, bool live, const float4 (&x)[NV], int q0, int q1) {
  const int l = tidx() & 15, grp = (tidx() & 63) >> 4;
  const int M = p.M;
  const int b = g / M;
  // M > dist_stride(M) - 256, so the columns of t < NV - 4 are all real; only
  // the last four float4s of a lane can hold pad columns (+inf)
  auto sure = [](int t) { return t < NV - 4; };
  auto valid = [&](int t, int c) { return sure(t) || 4 * (l + 16 * t) + c < M; };
  // the row maximum on the bit patterns: distances are >= +0 (sums of fabsf),
  // where unsigned order is float order (and no canonicalising v_max per
  // element).  A NaN distance (NaN features) now makes R NaN where fmaxf
  // skipped it; its row's sums are NaN either way (t = NaN for that column)
  auto key = [](float v) { return __float_as_uint(v); };
  uint32_t mb = 0u;
#pragma unroll
  for (int t = 0; t < NV; ++t) {
    const float e[4] = {x[t].x, x[t].y, x[t].z, x[t].w};
#pragma unroll
    for (int c = 0; c < 4; ++c) mb = max(mb, valid(t, c) ? key(e[c]) : 0u);
  }
  const float R = 0.5f * row16_max(__uint_as_float(mb));
  const float invR = R > 0.0f ? 1.0f / R : 0.0f;  // R = 0: every t = -1, every a = 0
  f2 acc[kMom - 1];
#pragma unroll
  for (int k = 0; k < kMom - 1; ++k) acc[k] = f2{0.0f, 0.0f};
#pragma unroll
  for (int t = 0; t < NV; ++t) {
    const float e[4] = {x[t].x, x[t].y, x[t].z, x[t].w};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float t0 = valid(t, 2 * h) ? fmaf(e[2 * h], invR, -1.0f) : 0.0f;
      const float t1 = valid(t, 2 * h + 1) ? fmaf(e[2 * h + 1], invR, -1.0f) : 0.0f;
      const f2 tt = {t0, t1};
      f2 pw = tt;
#pragma unroll
      for (int k = 0; k < kMom - 1; ++k) {
        acc[k] += pw;
        if (k + 1 < kMom - 1) pw *= tt;
      }
      // one column pair's powers at a time (left to itself the scheduler
      // interleaves all of them: 230 VGPRs)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float v[16];  // slot k + 1 of the record: P_{k+1}
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = k >= 1 && k < kMom ? acc[k - 1].x + acc[k - 1].y : 0.0f;
  float rec = row16_totals16(v);
  if (l == 0) rec = float(M);
  if (l == kMomR) rec = R;
  if (live) p.bmom[size_t(g) * kMomStride + l] = rec;
  // first-iteration pairs of this row that the series does not cover (k_bkernel's
  // test, on the same R and sigma: about 3/4 of the pairs on real distances),
  // each 16-lane row on its own records, one distinct sigma per round, the
  // wave looping while any row has one left (a whole wave per pair would need
  // the rows in LDS: 32-64 KB per workgroup, measured slower)
  const int n = p.n;
  float* rowsum = p.brow + size_t(b) * kBetaSamples * n;
  int nmax = q1 - q0;
  nmax = max(nmax, __shfl_xor(nmax, 16));
  nmax = max(nmax, __shfl_xor(nmax, 32));
  for (int c0 = 0; c0 < nmax; c0 += 16) {  // wave-uniform
    const int c = q0 + c0 + l;
    const bool have = c < q1;
    const int2 pr = p.rpair0[have ? c : max(q0, 0)];
    const int il = pr.x;
    const float sl = __int_as_float(pr.y);
    bool todo = have && !(double(R) * (1.0 / double(sl)) <= p.mom_amax);
    while (__ballot(todo)) {  // wave-uniform
      const unsigned field = unsigned(__ballot(todo) >> (16 * grp)) & 0xFFFFu;
      const int j = field ? __builtin_ctz(field) : 0;
      const int src = 16 * grp + j;
      const float sg = __int_as_float(__shfl(__float_as_int(sl), src));
      const float cs = kNegLog2eRow / sg;
      const f2 c2 = {cs, cs};
      f2 acc2 = {0.0f, 0.0f};
#pragma unroll
      for (int t = 0; t < NV; ++t) {  // pad columns: +inf * cs = -inf -> 0
        const f2 t0 = f2{x[t].x, x[t].y} * c2, t1 = f2{x[t].z, x[t].w} * c2;
        acc2 += f2{__builtin_amdgcn_exp2f(t0.x), __builtin_amdgcn_exp2f(t0.y)};
        acc2 += f2{__builtin_amdgcn_exp2f(t1.x), __builtin_amdgcn_exp2f(t1.y)};
      }
      const float sum = row16_total(acc2.x + acc2.y);
      // every pair of the row with this sigma (the first iteration's samples
      // share sigma = 0.01, the clip, about half of them) takes the same sum
      const bool same = todo && __float_as_uint(sl) == __float_as_uint(sg);
      if (field && same) rowsum[il] = sum;
      if (field && same) todo = false;
    }
  }
}

constexpr int kMomRowWaves = 4;  // waves per k_bmoment_rows workgroup

#ifndef MPCMMD_FUSED_TU
// four rows per wave and nothing else: measured against 2-16 four-row passes
// per wave with the next pass's rows in flight (0.306 vs 0.318-0.363 ms per
// configs[1] step), more resident waves hide the row loads better than a
// prefetch within each
template <int NV>
__global__ __launch_bounds__(64 * kMomRowWaves) void k_bmoment_rows(Params p) {
  const int l = tidx() & 15;
  const int total = p.Bt * p.M, Md = dist_stride(p.M), M = p.M;
  const int w = blockIdx.x * kMomRowWaves + (tidx() >> 6);
  if (w * 4 >= total) return;  // wave-uniform
  // position gp of the candidates' rows in pair-count order (Params::rperm): the
  // wave's four rows carry nearly the same number of first-iteration pairs
  const int gp = w * 4 + ((tidx() & 63) >> 4);
  // positions past the end (the last wave's) compute on a clamped row, store nothing
  const bool live = gp < total;
  const int gpc = live ? gp : total - 1, bc = gpc / M, r = p.rperm[gpc - bc * M], gc = bc * M + r;
  const float4* row = reinterpret_cast<const float4*>(p.bdist + size_t(gc) * Md) + l;
  float4 x[NV];
#pragma unroll
  for (int t = 0; t < NV; ++t) x[t] = row[16 * t];
  const int q0 = live ? p.rp0[r] : 0, q1 = live ? p.rp0[r + 1] : 0;
  bmoment_row16<NV>(p, gc, live, x, q0, q1);
}
#endif

// ------------------------------------------------------------------------
// top-n of |v_j| (j < M) in jnp.argsort order, one wave.  out[k] (k < n) are
// the indices at sorted positions M-n+k (ascending by (|v|, j)).
// Lane holds NQ keys (j = lane + 64 q).  The n-th largest key is found by
// bisection on the key bits; the counts are VALU (per-lane compares, then a
// DPP reduction of two samples' counts packed in 16-bit halves), so the
// search does not serialise on the CU's scalar unit.  The search stops as
// soon as exactly n keys lie above the candidate threshold (continuous data:
// well before the 31 steps).  Ties at the threshold go to the largest
// indices.  scratch: 2 * 64 ints of LDS owned by the wave.
template <int NQ, class V>
DEVI void load_keys(V val, int M, uint32_t* key) {
  const int lane = tidx() & 63;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int j = lane + 64 * q;
    const float v = val(min(j, M - 1));
    key[q] = j < M ? sort_key_abs(v) : 0u;  // real keys have bit 31 set
  }
}

// Threshold search for NB samples at once (independent chains interleave):
// T[u] = the n-th largest key of sample u, or exact[u] when exactly n keys
// are >= T[u].
template <int NQ, int NB>
DEVI void find_thresholds(const uint32_t (*key)[NQ], int nb, int n, uint32_t* T, bool* exact) {
  constexpr int NP = (NB + 1) / 2;
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    T[u] = 0x80000000u;  // real keys have bit 31 set, padding keys are 0
    exact[u] = u >= nb;
  }
  for (int bit = 30; bit >= 0; --bit) {
    int packed[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) packed[i] = 0;
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if (exact[u]) continue;  // wave-uniform
      const uint32_t cand = T[u] | (1u << bit);
      int c = 0;
#pragma unroll
      for (int q = 0; q < NQ; ++q) c += key[u][q] >= cand;
      packed[u >> 1] += c << (16 * (u & 1));
    }
    bool all = true;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int tot = wave_total(packed[i]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int u = 2 * i + h;
        if (u >= NB || exact[u]) continue;
        const int cnt = (tot >> (16 * h)) & 0xFFFF;
        if (cnt >= n) T[u] |= 1u << bit;
        exact[u] = cnt == n;
        all = all && exact[u];
      }
    }
    if (all) break;
  }
}

// Given the threshold, write the indices of the top n keys to out[0..n) in
// jnp.argsort order (ascending key, ties by index).  Ties at a non-exact
// threshold go to the largest indices.
template <int NQ>
DEVI void emit_top(const uint32_t* key, uint32_t T, bool exact, int n, int32_t* out, int* scratch) {
  const int lane = tidx() & 63;
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
  uint32_t* lk = reinterpret_cast<uint32_t*>(scratch + 64);
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

// Window top-n.  Given a threshold T with n <= c = #{keys >= T}, the keys
// >= T are compacted into LDS as 64-bit words (key << 32 | j), whose unsigned
// order is the jnp.argsort order (ascending |v|, ties by index); if c <= 64 R
// each lane ranks R of them exactly (one broadcast LDS read and one 64-bit
// compare per candidate, no scalar-unit chains) and the top n go to out[] in
// argsort order (out[n - 1 - rank], rank 0 = largest).  Returns false (and
// writes nothing) when c > 64 R.
template <int NQ, int R>
DEVI bool emit_window(const uint32_t* key, uint32_t T, int n, int32_t* out, unsigned long long* cand) {
  constexpr int cap = 64 * R;
  const int lane = tidx() & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  int c = 0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const bool sel = key[q] >= T;
    const unsigned long long m = __ballot(sel);
    const int pos = c + __popcll(m & below);
    // unconditional store: overflow and unselected lanes write the dump slot
    cand[sel && pos < cap ? pos : cap + 3] = (static_cast<unsigned long long>(key[q]) << 32) | uint32_t(lane + 64 * q);
    c += __popcll(m);
  }
  if (c > cap) return false;
  if (lane < 8) cand[c + lane] = 0ull;  // pad the reads past c (rank nothing: real keys have bit 31 set)
  wave_sync();
  unsigned long long mine[R];
  int rank[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    mine[r] = cand[lane + 64 * r];  // slots >= c are stale; never emitted
    rank[r] = 0;
  }
  const ulonglong2* c2 = reinterpret_cast<const ulonglong2*>(cand);
  for (int e = 0; e < c; e += 8) {  // four broadcast reads in flight, not one LDS latency per pair
    ulonglong2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = c2[(e >> 1) + u];  // wave-uniform address: LDS broadcast
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) rank[r] += int(v[u].x > mine[r]) + int(v[u].y > mine[r]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (lane + 64 * r < c && rank[r] < n) out[n - 1 - rank[r]] = int32_t(uint32_t(mine[r]));
  wave_sync();
  return true;
}

// wave minimum (VALU: quad / row butterflies, then the row broadcasts into
// lane 63; rows a broadcast does not write keep the identity)
template <int CTRL, int ROWS = 0xF>
DEVI uint32_t dpp_umin_src(uint32_t v) {
  return uint32_t(__builtin_amdgcn_update_dpp(-1, int(v), CTRL, ROWS, 0xF, false));
}
DEVI uint32_t wave_min_u32(uint32_t v) {
  v = min(v, dpp_umin_src<0xB1>(v));
  v = min(v, dpp_umin_src<0x4E>(v));
  v = min(v, dpp_umin_src<0x124>(v));
  v = min(v, dpp_umin_src<0x128>(v));
  v = min(v, dpp_umin_src<0x142, 0xA>(v));
  v = min(v, dpp_umin_src<0x143, 0xC>(v));
  return uint32_t(__builtin_amdgcn_readlane(int(v), 63));
}

// A threshold T0 with #{keys >= T0} >= n and few keys above it: the n-th
// largest of the G group maxima (groups of 64 / G lanes; each of the n groups
// whose maximum is >= T0 holds a key >= T0).  For the top 22 of 484 keys in
// 32 lane pairs about 37 keys lie above it.  Ranks by broadcast LDS reads,
// the pick by a wave minimum; lm: G words of the wave's LDS.
template <int NQ, int G>
DEVI uint32_t group_max_threshold(const uint32_t* key, int n, uint32_t* lm) {
  const int lane = tidx() & 63;
  uint32_t m = key[0];
#pragma unroll
  for (int q = 1; q < NQ; ++q) m = max(m, key[q]);
  if constexpr (G == 32) m = max(m, uint32_t(__builtin_amdgcn_update_dpp(0, int(m), 0xB1, 0xF, 0xF, false)));
  if (lane % (64 / G) == 0) lm[lane / (64 / G)] = m;
  wave_sync();
  int gt = 0;
  const uint4* l4 = reinterpret_cast<const uint4*>(lm);
#pragma unroll
  for (int e = 0; e < G / 4; ++e) {
    const uint4 v = l4[e];  // broadcast
    gt += int(v.x > m) + int(v.y > m) + int(v.z > m) + int(v.w > m);
  }
  const uint32_t t = wave_min_u32(gt < n ? m : 0xFFFFFFFFu);
  wave_sync();
  return t;
}

// Top-n of the samples s = first, first + stride, ... < last, one wave, the
// next sample's keys in flight while one is ranked.  With M <= 64 R every key
// is a candidate; otherwise the window threshold comes from the group maxima
// (G = 32 lane pairs for n <= 24, 64 lanes for n <= 48).  Larger n, and ties
// so massive that the window overflows, take the exact bit bisection
// (find_thresholds) and the ballot emission (emit_top).
template <int NQ, int R, int G, class Row, class Out>
DEVI void select_walk(Row row, Out out, int first, int last, int stride, int M, int n, unsigned long long* cand,
                      uint32_t* lm, int* scratch) {
  uint32_t key[NQ], nxt[NQ];
  load_keys<NQ>(row(first), M, key);
  for (int s = first; s < last; s += stride) {
    load_keys<NQ>(row(min(s + stride, last - 1)), M, nxt);  // next sample's keys in flight
    bool done = false;
    if (M <= 64 * R)
      done = emit_window<NQ, R>(key, 0x80000000u, n, out(s), cand);  // real keys have bit 31 set
    else if (G > 0 && n <= G * 3 / 4)
      done = emit_window<NQ, R>(key, group_max_threshold<NQ, (G > 0 ? G : 64)>(key, n, lm), n, out(s), cand);
    if (!done) {
      uint32_t Tn[1];
      bool ex[1];
      find_thresholds<NQ, 1>(&key, 1, n, Tn, ex);
      emit_top<NQ>(key, Tn[0], ex[0], n, out(s), scratch);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) key[q] = nxt[q];
  }
}

// The first beta-iteration's selection from the handle's table (Params::sel0,
// sig0: k_bselect's output for the shared initial samples, computed once per
// table) into every candidate's bsel / bsig.
#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(256) void k_bsel0(Params p) {
  const int n = p.n, per = kBetaSamples * n + kBetaSamples;
  for (size_t x = size_t(blockIdx.x) * 256 + tidx(); x < size_t(p.nb) * per; x += size_t(gridDim.x) * 256) {
    const int c = int(x / per), e = int(x - size_t(c) * per), b = p.b0 + c;
    if (e < kBetaSamples * n)
      p.bsel[size_t(b) * kBetaSamples * n + e] = p.sel0[e];
    else
      p.bsig[size_t(b) * kBetaSamples + e - kBetaSamples * n] = p.sig0[e - kBetaSamples * n];
  }
}
#endif

// ------------------------------------------------------------------------
// k_bsample: the new samples of beta-CEM iteration tb >= 1 (rows 11..99,
// mean + L z, compute_beta.py:51-68) with the structured factor of the file
// header, as fp64 MFMA (v_mfma_f64_16x16x4_f64) over blocks of 16 positions:
//
//   Y_c = m_c + T_c Z_c + U_c S_c,   S_{c+1} = S_c + W_c^T Z_c
//
// Z_c [16 positions x 16 samples] the normals, S_c [11 x 16] the prefix
// sum_{j < 16c} w_j z_j, U_c / W_c [16 x 11] the generators u_j / w_j and
// T_c [16 x 16] = strict_lower(U_c W_c^T) + diag(L_jj) (itself one MFMA
// product, masked).  A wave owns kTilesPerWave tiles of 16 samples and walks
// the blocks in order; S lives in accumulator registers and is, by the
// 16x16x4 f64 layouts, directly the B operand of U_c S_c.  All in fp64 (the
// oracle's dense fp64 Cholesky agrees to ~1e-15 before the fp32 rounding).
//
// f64 16x16x4 layouts (lane l, r = l & 15, h = l >> 4):
//   A: A[r][h]   B: B[h][r]   C/D register i: C[h + 4 i][r]
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kSampleTiles = kBzCols / 16;  // 6 tiles of 16 sample columns (89 used)
static_assert(kBzCols >= kNew, "sample tiles");
// TPW = sample tiles per wave: 6 (one wave per candidate: the generator
// operands loaded once) when the batch fills the chip; small batches -- the
// reference's num_batch = 100 -- take k_bsample_chunks (one tile per wave,
// the blocks split into chunks walked in parallel).
//
// The prefix is kept as S = S_pre + S_loc: S_loc accumulates W^T Z from zero
// within a chunk of sample_chunk(nblk) blocks and is folded into S_pre at the
// chunk's end.  The chunking depends only on M, so one wave walking every
// chunk (k_bsample) and one wave per chunk (k_bsample_chunks, S_pre from the
// earlier chunks' sums) compute the same bits: a configuration's samples do
// not depend on the batch it is solved in.
constexpr int kChunkWavesMax = 12;
HDI int sample_chunk(int nblk) {
  int cl = nblk <= 8 ? 4 : 8;  // two chunks at M = 100 (k_bcem_small walks them in parallel)
  while ((nblk + cl - 1) / cl > kChunkWavesMax) cl <<= 1;
  return cl;
}
template <int TPW>
constexpr int sample_waves() {
  static_assert(kSampleTiles % TPW == 0, "tiles per wave");
  return kSampleTiles / TPW;
}

DEVI d4 mfma64(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// Operands of one block, loaded unconditionally (generators and normals are
// zero padded to whole blocks and tiles), so the loop has no branches and the
// compiler can count outstanding loads exactly.  Generator rows (k_belite,
// k_bgen): W plane = w_0..w_10 and a zero slot 11, U plane = u_0..u_10 and the
// position's mean in slot 11, genm = L_jj.  With row 11 of S_pre held at 1
// (and row 11 of S_loc exactly 0, W's slot 11 being 0), U S carries the mean
// as its twelfth term: no mean operand, no accumulator initialisation.
template <int TPW>
struct SampleBlock {
  double wA[4];  // W[p0 + 4k + h][r]        (A of W^T Z; r = feature)
  double wX[3];  // W[p0 + r][4i + h]        (A of W U^T; 4i + h = feature)
  double uX[3];  // U[p0 + r][4i + h]        (B of W U^T, A of U S; feature 11 = mean)
  double L;      // L_jj of position p0 + r
  float z[TPW][4];   // Z[p0 + 4k + h][sample of (tile t, lane r)] (sample_of); fp32 normals, widened at use
};

template <int TPW>
DEVI void load_block(SampleBlock<TPW>& q, const double* G, const double* GU, const double* gm, const float* z, int p0,
                     int s0, int r, int h) {
#pragma unroll
  for (int k = 0; k < 4; ++k) q.wA[k] = G[size_t(p0 + 4 * k + h) * kGenRow + kGenW + r];  // rows > 11 of S unused
  const double* g = G + size_t(p0 + r) * kGenRow;
  const double* gu = GU + size_t(p0 + r) * kGenRow;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    q.wX[i] = g[kGenW + 4 * i + h];  // W's zero slot 11 times U's mean: X gets no mean term
    q.uX[i] = gu[4 * i + h];
  }
  q.L = gm[p0 + r];
  // tiles in pairs: lane r of tiles 2u, 2u + 1 takes samples 32u + 2r, 32u +
  // 2r + 1 -- the lane image of bz_index, six float4 loads per block (one
  // tile per wave: lane r takes sample s0 + r, scalar loads)
  static_assert(TPW == 1 || TPW == kSampleTiles, "tile pairing of the normals' layout");
  if constexpr (TPW == 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) q.z[0][k] = z[bz_index(p0 + 4 * k + h, s0 + r)];
  } else {
    const float4* zb = reinterpret_cast<const float4*>(z + size_t(p0 >> 4) * (16 * kBzCols)) + r + 16 * h;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const float4 f = zb[64 * c];
      const float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int idx = 4 * c + w, k = idx / 6, t = idx % 6;  // t = 2 u + e
        q.z[t][k] = fv[w];
      }
    }
  }
}

// load_block<kSampleTiles> as raw buffer loads: the lane parts of the offsets
// are fixed for the launch (four VGPRs), the block part p0 goes in SGPRs, so
// a block's 17 loads need no per-lane address arithmetic and no 64-bit
// address registers (the walker runs at 1 wave per SIMD, where every VALU
// instruction and register counts).  Same addresses as load_block.
struct SampleRsrc {
  __amdgpu_buffer_rsrc_t gen, genm, z;
  int vA, vX, vL, vZ;  // lane offsets (bytes): W^T rows, W / U rows, L_jj, normals
  int uplane;          // bytes from the W plane to the U plane
};
DEVI SampleRsrc sample_rsrc(const double* G, const double* gm, const float* z, int Pp, int r, int h) {
  SampleRsrc s;
  s.gen = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(G), short(0), Pp * kGenStride * 8, 0x00020000);
  s.genm = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(gm), short(0), Pp * 8, 0x00020000);
  s.z = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(z), short(0), Pp * kBzCols * 4, 0x00020000);
  s.vA = (h * kGenRow + kGenW + r) * 8;
  s.vX = (r * kGenRow + h) * 8;
  s.vL = r * 8;
  s.vZ = (r + 16 * h) * 16;
  s.uplane = Pp * kGenRow * 8;
  return s;
}
DEVI double buf_ld_d(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}
DEVI void load_block_buf(SampleBlock<kSampleTiles>& q, const SampleRsrc& s, int p0) {
  const int sg = p0 * kGenRow * 8;
#pragma unroll
  for (int k = 0; k < 4; ++k) q.wA[k] = buf_ld_d(s.gen, s.vA + k * 4 * kGenRow * 8, sg);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    q.wX[i] = buf_ld_d(s.gen, s.vX + 32 * i, sg);
    q.uX[i] = buf_ld_d(s.gen, s.vX + 32 * i, sg + s.uplane);
  }
  q.L = buf_ld_d(s.genm, s.vL, p0 * 8);
  const int szz = (p0 >> 4) * (16 * kBzCols * 4);
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f f = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(s.z, s.vZ + 1024 * (c % 3), szz + 3072 * (c / 3), 0));
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int idx = 4 * c + w, k = idx / 6, t = idx % 6;
      q.z[t][k] = f[w];
    }
  }
}

// One block's MFMAs for the wave's tiles, all accumulating in place:
//   Y  = U S              (3 per tile from a zero C operand; the mean is
//                          U's feature 11 times row 11 of S_pre, which is 1)
//   S += W^T Z            (4 per tile; after U S has read S)
//   Y += T Z              (4 per tile; T from X = W U^T, built meanwhile)
// The Y products are formed transposed, Y^T = S^T U^T + Z^T T^T (the same
// operand registers with A and B exchanged), so register i of lane (r, h)
// holds sample row h + 4i of the tile at position p0 + r: a store covers
// four sample rows x 16 consecutive positions, no transpose before it.
// Tiles are interleaved, so every accumulator chain has 6 MFMAs between
// dependent steps.  No VALU work on the accumulators: the pipe never waits
// for a vector add between blocks.
template <int TPW>
DEVI void block_mfma(const SampleBlock<TPW>& cur, d4* S, const d4* Sp, d4* Y, int r, int h) {
  double zd[TPW][4];  // the fp32 normals widened once (exact), used by two MFMA chains
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int k = 0; k < 4; ++k) zd[t][k] = double(cur.z[t][k]);
  d4 X = d4{0.0, 0.0, 0.0, 0.0};  // X = W_c U_c^T: register i holds w_{h+4i} . u_r = T[row r][col h + 4i]
#pragma unroll
  for (int i = 0; i < 3; ++i) X = mfma64(cur.wX[i], cur.uX[i], X);
  const d4 zero = d4{0.0, 0.0, 0.0, 0.0};
  // B operand of U S: S_pre + S_loc (rows 0..11 of S: registers 0..2)
  double St[TPW][3];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int k = 0; k < 3; ++k) St[t][k] = Sp[t][k] + S[t][k];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int t = 0; t < TPW; ++t) Y[t] = mfma64(St[t][k], cur.uX[k], k == 0 ? zero : Y[t]);
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int t = 0; t < TPW; ++t) S[t] = mfma64(cur.wA[k], zd[t][k], S[t]);
  double T[4];  // B operand of (T Z)^T, k-step i: T[r][4i + h]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = h + 4 * i;
    T[i] = k < r ? X[i] : (k == r ? cur.L : 0.0);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int t = 0; t < TPW; ++t) Y[t] = mfma64(zd[t][k], T[k], Y[t]);
}

// the finished block's samples to fp32 (the sigma coordinate M clipped).
// Lane (r, h), register i of tile t: sample row rho = h + 4i of the tile
// (sample s0 + rho for one tile per wave; 32 (t / 2) + 2 rho + t % 2 for the
// paired tiles of the one-wave walker), position p0 + r; per store, four
// sample rows x 64 contiguous bytes.  Blocks wholly past the sigma coordinate
// and the padding samples >= kNew are not stored (k_bselect never reads them).
HDI_CONST int tile_sample(int TPW, int s0, int t, int rho) { return TPW == 1 ? s0 + rho : 32 * (t >> 1) + 2 * rho + (t & 1); }
template <int TPW>
DEVI void block_store(const d4* Yv, float* plane, int p0, int M, int ys, int s0, int r, int h) {
  if (p0 > M) return;
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = tile_sample(TPW, s0, t, h + 4 * i);
      const float v = float(Yv[t][i]);
      if (s < kNew) plane[size_t(s) * ys + p0 + r] = p0 + r == M ? fmaxf(v, 0.01f) : v;
    }
}

// k_bsample's store of a finished block that does not hold the sigma
// coordinate M: block_store<kSampleTiles> without the clip's selects and
// without per-block address arithmetic (on gfx950 a wave's VALU work does not
// run in the shadow of its fp64 MFMAs -- tools/mfma_overlap.hip: +6..8
// clocks per VALU instruction between MFMAs).  Raw buffer stores over the
// candidate's sample plane: the lane part of the offset (vl = row 2h,
// position r) is fixed for the launch, the block, tile and register parts go
// in an SGPR.  Tiles 0-3 hold real samples only; in tiles 4 and 5 register 3
// holds samples 88 + 2h + t % 2 >= kNew but for (t = 4, h = 0) -- that store
// takes v43, out of range (dropped by the buffer unit) for h > 0, and tile
// 5's register 3 is not stored.
DEVI __amdgpu_buffer_rsrc_t ygen_rsrc(float* plane, int ys) {
  return __builtin_amdgcn_make_buffer_rsrc(plane, short(0), kBzCols * ys * 4, 0x00020000);
}
constexpr int kDropOffset = 0x7FFFFF00;  // out of range for any plane
static_assert(kNew == 89, "tile 4 / 5 register 3 validity below");
DEVI void block_store_rows(const d4* Yv, __amdgpu_buffer_rsrc_t yr, int p0, int ys, int vl, int v43) {
#pragma unroll
  for (int t = 0; t < kSampleTiles; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (t == 5 && i == 3) continue;
      const int soff = ((32 * (t >> 1) + (t & 1) + 8 * i) * ys + p0) * 4;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(float(Yv[t][i])), yr, t == 4 && i == 3 ? v43 : vl, soff, 0);
    }
}

// S_pre += S_loc, S_loc = 0 (a chunk's end)
DEVI void fold_chunk(d4& Sp, d4& S) {
#pragma unroll
  for (int k = 0; k < 3; ++k) Sp[k] = Sp[k] + S[k];
  S = d4{0.0, 0.0, 0.0, 0.0};
}

#ifndef MPCMMD_FUSED_TU
template <int TPW>
__global__ __launch_bounds__(64 * sample_waves<TPW>()) void k_bsample(Params p, int tb) {
  const int b = p.b0 + blockIdx.x, M = p.M, Pp = pos_pad(M);
  const int lane = tidx() & 63, w = tidx() >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int s0 = w * TPW * 16;
  MPCMMD_STAMP(p, 0);
  const double* G = p.gen + size_t(b) * Pp * kGenStride;
  const double* gm = p.genm + size_t(b) * Pp;
  const float* z = p.beta_z + size_t(tb - 1) * Pp * kBzCols;
  const int ys = ygen_stride(M);
  float* plane = p.ygen + size_t(b) * kBzCols * ys;
  d4 S[TPW], Sp[TPW], Ya[TPW], Yb[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    S[t] = Sp[t] = d4{0.0, 0.0, 0.0, 0.0};
    Sp[t][2] = h == 3 ? 1.0 : 0.0;  // row 11 of S_pre: the mean's coefficient
  }
  const int nblk = Pp >> 4, cl = sample_chunk(nblk);
  const __amdgpu_buffer_rsrc_t yr = ygen_rsrc(plane, ys);
  const int vl = (2 * h * ys + r) * 4, v43 = h == 0 ? vl : kDropOffset;
  auto store = [&](const d4* Yv, int q0) {
    if (TPW == kSampleTiles && q0 + 15 < M)  // block-uniform
      block_store_rows(Yv, yr, q0, ys, vl, v43);
    else
      block_store<TPW>(Yv, plane, q0, M, ys, s0, r, h);
  };
  // blocks in pairs, operands and outputs ping-ponged: the next block's loads
  // are in flight and its MFMAs issued while the previous block's samples
  // are converted and stored (the last prefetch re-reads a block; nblk and
  // the chunk length are even; sched barriers keep that order)
  SampleBlock<TPW> qa, qb;
  const SampleRsrc srs = sample_rsrc(G, gm, z, Pp, r, h);
  auto load = [&](SampleBlock<TPW>& q, int q0) {
    if constexpr (TPW == kSampleTiles)
      load_block_buf(q, srs, q0);
    else
      load_block(q, G, G + gen_uplane(Pp), gm, z, q0, s0, r, h);
  };
  load(qa, 0);
  for (int c = 0; c < nblk; c += 2) {
    const int p0 = c << 4;
    load(qb, p0 + 16);
    __builtin_amdgcn_sched_barrier(0);
    block_mfma(qa, S, Sp, Ya, r, h);
    __builtin_amdgcn_sched_barrier(0);
    if (c > 0) store(Yb, p0 - 16);
    __builtin_amdgcn_sched_barrier(0);
    load(qa, min(p0 + 32, Pp - 16));
    __builtin_amdgcn_sched_barrier(0);
    block_mfma(qb, S, Sp, Yb, r, h);
    if ((c + 2) % cl == 0)
#pragma unroll
      for (int t = 0; t < TPW; ++t) fold_chunk(Sp[t], S[t]);
    __builtin_amdgcn_sched_barrier(0);
    store(Ya, p0);
    __builtin_amdgcn_sched_barrier(0);
  }
  store(Yb, Pp - 16);
  MPCMMD_STAMP(p, 1);
}
#endif

// k_bsample_chunks: the samples of k_bsample for small batches, workgroup =
// (candidate, tile of 16 samples), one wave per chunk of blocks.  Phase 1:
// each wave but the last sums W^T Z over its chunk (the MFMAs of the walker's
// S_loc, from zero) into LDS; phase 2: S_pre = the earlier chunks' sums in
// order (the walker's folds), then the chunk's blocks as in k_bsample.
#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(64 * kChunkWavesMax) void k_bsample_chunks(Params p, int tb) {
  __shared__ double dS[kChunkWavesMax - 1][3][64];
  const int b = p.b0 + blockIdx.x, M = p.M, Pp = pos_pad(M), nblk = Pp >> 4;
  const int lane = tidx() & 63, k = tidx() >> 6, P = blockDim.x >> 6;
  const int r = lane & 15, h = lane >> 4, s0 = blockIdx.y * 16;
  const int cl = sample_chunk(nblk), c0 = k * cl, c1 = min(nblk, c0 + cl);
  MPCMMD_STAMP(p, 0);
  const double* G = p.gen + size_t(b) * Pp * kGenStride;
  const double* gm = p.genm + size_t(b) * Pp;
  const float* z = p.beta_z + size_t(tb - 1) * Pp * kBzCols;
  const int ys = ygen_stride(M);
  float* plane = p.ygen + size_t(b) * kBzCols * ys;
  if (k < P - 1) {
    // operands of W^T Z for block c: W[p0 + 4 kk + h][r], Z[p0 + 4 kk + h][s0 + r]
    auto ld = [&](double (&wa)[4], double (&zz)[4], int c) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const size_t pos = size_t(c) * 16 + 4 * kk + h;
        wa[kk] = G[pos * kGenRow + kGenW + r];
        zz[kk] = double(z[bz_index(int(pos), s0 + r)]);
      }
    };
    d4 Sl = d4{0.0, 0.0, 0.0, 0.0};
    double wa[4], zz[4], wn[4], zn[4];
    ld(wa, zz, c0);
    for (int c = c0; c < c1; ++c) {
      ld(wn, zn, min(c + 1, c1 - 1));
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) Sl = mfma64(wa[kk], zz[kk], Sl);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        wa[kk] = wn[kk];
        zz[kk] = zn[kk];
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) dS[k][i][lane] = Sl[i];
  }
  __syncthreads();
  d4 S[1] = {d4{0.0, 0.0, 0.0, 0.0}}, Sp[1] = {d4{0.0, 0.0, 0.0, 0.0}}, Ya[1], Yb[1];
  Sp[0][2] = h == 3 ? 1.0 : 0.0;  // row 11 of S_pre: the mean's coefficient (the chunks' row 11 sums are 0)
  for (int j = 0; j < k; ++j)
#pragma unroll
    for (int i = 0; i < 3; ++i) Sp[0][i] = Sp[0][i] + dS[j][i][lane];
  SampleBlock<1> qa, qb;
  const int pend = c1 << 4;
  load_block(qa, G, G + gen_uplane(Pp), gm, z, c0 << 4, s0, r, h);
  for (int c = c0; c < c1; c += 2) {
    const int p0 = c << 4;
    load_block(qb, G, G + gen_uplane(Pp), gm, z, p0 + 16, s0, r, h);
    __builtin_amdgcn_sched_barrier(0);
    block_mfma(qa, S, Sp, Ya, r, h);
    __builtin_amdgcn_sched_barrier(0);
    if (c > c0) block_store<1>(Yb, plane, p0 - 16, M, ys, s0, r, h);
    __builtin_amdgcn_sched_barrier(0);
    load_block(qa, G, G + gen_uplane(Pp), gm, z, min(p0 + 32, pend - 16), s0, r, h);
    __builtin_amdgcn_sched_barrier(0);
    block_mfma(qb, S, Sp, Yb, r, h);
    __builtin_amdgcn_sched_barrier(0);
    block_store<1>(Ya, plane, p0, M, ys, s0, r, h);
    __builtin_amdgcn_sched_barrier(0);
  }
  block_store<1>(Yb, plane, pend - 16, M, ys, s0, r, h);
  MPCMMD_STAMP(p, 1);
}
#endif

// k_bcem_small's sampler, from an LDS copy of the candidate's generators (lg:
// W plane, U plane, genm, as in global memory; its workgroup just wrote them).
// Two passes:
//   bsample_tblocks  every block's T = strict_lower(W U^T) + diag(L_jj) (the
//                    X MFMAs of block_mfma), once per block into LDS (Tl)
//                    instead of once per tile
//   bsample_unit_lds one (tile of 16 samples, chunk of blocks) per wave: the
//                    earlier chunks' W^T Z sums first (S_pre, folded chunk by
//                    chunk as the walker folds), then the chunk's blocks --
//                    so the chunks of a tile run on separate waves
// Per block the operands and MFMAs of block_mfma in its order, so the samples
// are the per-iteration kernels' bits.  The normals (global, shared by every
// candidate) come kZAhead blocks ahead in registers.
constexpr int kZAhead = 4;
HDI size_t gen_lds_bytes(int M) { return size_t(pos_pad(M)) * (2 * kGenRow + 1) * 8 + 16 * 8; }  // + wA's overreach
HDI size_t tblk_lds_bytes(int M) { return size_t(pos_pad(M) >> 4) * 4 * 64 * 8; }

DEVI void bsample_tblocks(const Params& p, const double* lg, double* Tl, int w, int W) {
  const int M = p.M, Pp = pos_pad(M), nblk = Pp >> 4;
  const int lane = tidx() & 63, r = lane & 15, h = lane >> 4;
  for (int blk = w; blk < nblk; blk += W) {
    const int p0 = blk * 16;
    const double* g = lg + size_t(p0 + r) * kGenRow;
    const double* gu = lg + gen_uplane(Pp) + size_t(p0 + r) * kGenRow;
    double wX[3], uX[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      wX[i] = g[kGenW + 4 * i + h];
      uX[i] = gu[4 * i + h];
    }
    const double L = lg[2 * gen_uplane(Pp) + p0 + r];
    d4 X = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 3; ++i) X = mfma64(wX[i], uX[i], X);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = h + 4 * i;
      Tl[(size_t(blk) * 4 + i) * 64 + lane] = k < r ? X[i] : (k == r ? L : 0.0);
    }
  }
}

DEVI void bsample_unit_lds(const Params& p, int tb, int b, int tile, int chunk, const double* lg, const double* Tl) {
  const int M = p.M, Pp = pos_pad(M), nblk = Pp >> 4, cl = sample_chunk(nblk);
  const int c0 = chunk * cl, c1 = min(nblk, c0 + cl);
  const int lane = tidx() & 63, r = lane & 15, h = lane >> 4, s0 = tile * 16;
  const double* LW = lg;
  const double* LU = lg + gen_uplane(Pp);
  const float* z = p.beta_z + size_t(tb - 1) * Pp * kBzCols;
  const int ys = ygen_stride(M);
  float* plane = p.ygen + size_t(b) * kBzCols * ys;
  d4 S = d4{0.0, 0.0, 0.0, 0.0}, Sp = d4{0.0, 0.0, 0.0, 0.0};
  Sp[2] = h == 3 ? 1.0 : 0.0;  // row 11 of S_pre: the mean's coefficient
  auto zload = [&](float (&zz)[4], int c) {
#pragma unroll
    for (int k = 0; k < 4; ++k) zz[k] = z[bz_index(c * 16 + 4 * k + h, s0 + r)];
  };
  float zr[kZAhead][4];
#pragma unroll
  for (int u = 0; u < kZAhead; ++u) zload(zr[u], min(u, c1 - 1));
  const d4 zero = d4{0.0, 0.0, 0.0, 0.0};
  for (int c = 0; c < c1; c += kZAhead) {
#pragma unroll
    for (int u = 0; u < kZAhead; ++u) {
      const int cb = c + u;
      if (cb < c1) {  // wave-uniform
        const int p0 = cb * 16;
        double zd[4], wA[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          zd[k] = double(zr[u][k]);
          wA[k] = LW[size_t(p0 + 4 * k + h) * kGenRow + kGenW + r];
        }
        zload(zr[u], min(cb + kZAhead, c1 - 1));
        if (cb >= c0) {  // the chunk's block: Y = U S + T Z (block_mfma)
          double uX[3], T[4];
#pragma unroll
          for (int i = 0; i < 3; ++i) uX[i] = LU[size_t(p0 + r) * kGenRow + 4 * i + h];
#pragma unroll
          for (int i = 0; i < 4; ++i) T[i] = Tl[(size_t(cb) * 4 + i) * 64 + lane];
          double St[3];
#pragma unroll
          for (int k = 0; k < 3; ++k) St[k] = Sp[k] + S[k];
          d4 Y = zero;
#pragma unroll
          for (int k = 0; k < 3; ++k) Y = mfma64(St[k], uX[k], k == 0 ? zero : Y);
#pragma unroll
          for (int k = 0; k < 4; ++k) S = mfma64(wA[k], zd[k], S);
#pragma unroll
          for (int k = 0; k < 4; ++k) Y = mfma64(zd[k], T[k], Y);
          block_store<1>(&Y, plane, p0, M, ys, s0, r, h);
        } else {  // an earlier chunk's block: its W^T Z into S_loc only
#pragma unroll
          for (int k = 0; k < 4; ++k) S = mfma64(wA[k], zd[k], S);
        }
        if ((cb + 1) % cl == 0) fold_chunk(Sp, S);  // the walker's fold after a chunk's last block
      }
    }
  }
}

// ------------------------------------------------------------------------
// k_bselect: top-n |beta| rows (compute_beta.py:117-118) and sigma of the
// 100 samples.  Single-wave workgroups, W = gridDim.y waves per candidate;
// wave (b, g) walks samples g, g + W, g + 2W, ... (select_walk).
// NQ = keys per lane (M <= 64 NQ), R = window capacity / 64, G = groups for
// the window threshold (0: bisection): one instantiation per size, so each
// has its own register allocation
// the samples g, g + W, ... of candidate b on the calling wave; cand [64 R +
// 8], lm [64], scratch [128]: the wave's LDS
template <int NQ, int R, int G>
DEVI void bselect_wave(const Params& p, int tb, int b, int g, int W, unsigned long long* cand, uint32_t* lm,
                       int* scratch) {
  const int M = p.M, M1 = M + 1, n = p.n;
  int32_t* sel = p.bsel + size_t(b) * kBetaSamples * n;
  float* sig = p.bsig + size_t(b) * kBetaSamples;
  const float* E = p.belite + (size_t(tb & 1) * p.Bt + b) * kBetaElite * M1;
  const int ys = ygen_stride(M);
  const float* Y = p.ygen + size_t(b) * kBzCols * ys;
  const float* z0 = p.beta_z0;
  // sample s: initial MVN(0, 20 I) draws (tb = 0, compute_beta.py:41-49), the
  // previous elites (rows 0..10) or this iteration's new samples
  auto row = [&](int s) {
    const float* r = tb == 0 ? z0 + size_t(s) * M1 : (s < kBetaElite ? E + size_t(s) * M1 : Y + size_t(s - kBetaElite) * ys);
    const bool scale = tb == 0;
    return [=](int j) { return scale ? float(kSqrt20 * double(r[j])) : r[j]; };
  };
  // samples 0..10 of iteration tb >= 1 are the previous elites, whose rows
  // and sigma k_belite carried over
  const int s_lo = first_sample(tb);
  if (s_lo + g >= kBetaSamples) return;
  select_walk<NQ, R, G>(row, [&](int s) { return sel + s * n; }, s_lo + g, kBetaSamples, W, M, n, cand, lm, scratch);
  const int lane = tidx() & 63;
  for (int s = s_lo + g + lane * W; lane < 16 && s < kBetaSamples; s += 16 * W) {
    const float v = row(s)(M);
    sig[s] = tb == 0 ? fmaxf(v, 0.01f) : v;  // later rows are clipped when written
  }
}

#ifndef MPCMMD_FUSED_TU
template <int NQ, int R, int G>
__global__ __launch_bounds__(64) void k_bselect(Params p, int tb) {
  __shared__ __attribute__((aligned(16))) unsigned long long cand[64 * R + 8];
  __shared__ __attribute__((aligned(16))) uint32_t lm[64];
  __shared__ int scratch[128];
  // this beta-iteration's direct-pair list starts empty (k_bkernel appends)
  if (blockIdx.y == 0 && tidx() == 0) p.bdlcount[size_t(p.b0 + blockIdx.x) * kBetaIters + tb] = 0;
  bselect_wave<NQ, R, G>(p, tb, p.b0 + blockIdx.x, blockIdx.y, gridDim.y, cand, lm, scratch);
}
#endif

// ------------------------------------------------------------------------
// k_bkernel + k_bdirect: kernel_computation.py:19-65 / compute_beta.py:120-127
// for every sample of the iteration: the K_mixed row sums and K_red.
//
// k_bkernel, workgroup = (candidate, part of its samples):
//   union    the distinct mother rows the iteration's samples select (LDS
//            flags, scan): their rank and their series records (k_bmoment),
//            staged in LDS
//   series   every (sample s, reduced position k) pair whose a = R_r / sigma_s
//            is <= 1: row sum = exp(-a) * a 12-term Horner sum over the row's
//            moments, fp64, one thread per pair; the other pairs are flagged
//            for k_bdirect (Params::bdflag, a count per part in bdcount)
//   K_red    exp(-D[sel_k][sel_kk] / sigma_s), kk < k, the distances
//            recomputed from the feature rows (Params::featr) in k_bdist's
//            sequential feature order (bit-equal to D's entries), consecutive
//            entries stored by consecutive lanes.  When the pairwise distances
//            of the union fit the LDS budget (after the first few
//            beta-iterations the samples concentrate: ~40-150 distinct rows
//            of 484 at n = 22) they are computed once (a lane per row a, the
//            rows b < a as LDS broadcasts) and each sample's entries are
//            exponentials of table lookups (a wave per sample, the lookups of
//            all its entries in flight together); otherwise a wave per sample
//            stages its n feature rows in LDS and forms its n (n - 1) / 2
//            distances, one lane per entry.
// k_bdirect, workgroup = (candidate, part of its rows), only when a candidate
// has flagged pairs (a > 1: mostly the first beta-iteration, whose samples
// clipped to sigma = 0.01 have a ~ 100): the flagged pairs counting-sorted by
// mother row r (LDS); a wave takes the next distinct row (LDS counter,
// heaviest first) and holds its distance row (k_bdist) in registers (lane L:
// float4s L + 64 t; for short rows the next row's loads are issued before the
// current one is summed).  The row's pairs are summed 8 at a time: per lane
// and pair the lane's terms exp2(D[r][j] * (-log2 e / sigma_s)) (v_exp_f32,
// packed scale / add), then one transposing cross-lane reduction (permlane32
// / permlane16 swaps, DPP) leaves pair j's row sum in lane 8 j + 4.
// From the second beta-iteration on, samples 0..10 are the previous elites:
// their selection, kernels and QP are unchanged, k_belite carried them, and
// only samples 11..99 are processed here.
constexpr int kKerWaves = 16;
constexpr int kDirWaves = 4;
constexpr int kLptBins = 128;        // pair counts per distinct row (<= 100 samples)
constexpr double kSeriesAMax = kSeriesAMaxRow;  // k_bmoment's error bound holds for a <= 1
constexpr size_t kLdsBudget = 160 * 1024 - 1024;

struct LdsTake {  // consecutive 16-byte aligned LDS pieces
  size_t o = 0;
  HDI size_t operator()(size_t bytes) {
    const size_t at = o;
    o = (o + bytes + 15) & ~size_t(15);
    return at;
  }
};

// k_bkernel LDS.  persistent: sel (short; union ranks once the records are
// staged), -log2 e / sigma, 1 / sigma, the entry table (k | kk << 8), union
// rank of a row, row of a rank; scratch (`scratch` bytes, chosen at launch):
// the union flags, then the union's series records, then the distance table
// and the union's feature rows, or the waves' per-sample feature rows
struct KerLds {
  size_t sel, csg, csd, tri, urank, urow, misc, scratch, total;
};
HDI KerLds ker_lds(int M, int n, size_t scratch) {
  KerLds L{};
  LdsTake take;
  L.sel = take(size_t(kBetaSamples) * n * 2);
  L.csg = take(size_t(kBetaSamples) * 4);
  L.csd = take(size_t(kBetaSamples) * 8);
  L.tri = take(size_t(n) * (n - 1));
  L.urank = take(size_t(M) * 2);
  L.urow = take(size_t(M) * 2);
  L.misc = take(32 * 4);  // [0] union rows, [1] series pairs, [2] direct pairs, [16..] wave totals
  L.scratch = take(scratch);
  L.total = take.o;
  return L;
}
HDI size_t ker_sample_bytes(int n, int nw = kKerWaves) { return size_t(nw) * n * kFeatStride * 4; }
HDI size_t ker_tab_bytes(int U) { return ((size_t(U) * (U - 1) / 2 * 4 + 15) & ~size_t(15)) + size_t(U) * kFeatStride * 4; }
constexpr size_t kKerTabBytes = 55 * 1024;  // the table of a union of <= 144 rows
// scratch: the series records of every mother row (up to kKerRecBytes;
// larger unions read them from global memory), and the union table (up to
// kKerTabBytes) from the second beta-iteration on (the first one's 100 fresh
// samples select nearly every mother row)
constexpr size_t kKerRecBytes = 64 * 1024;
HDI size_t ker_scratch(int M, int n, int tb, int nw = kKerWaves) {
  size_t sc = ker_sample_bytes(n, nw);
  size_t rec = size_t(M) * kMomStride * 4;
  if (rec > kKerRecBytes) rec = kKerRecBytes;
  if (rec > sc) sc = rec;
  if (tb > 0 && kKerTabBytes > sc) sc = kKerTabBytes;
  return sc;
}

// k_bdirect LDS.  persistent: sel (short), -log2 e / sigma, the direct pairs
// sorted by row, the distinct direct rows and their first pair, the grab
// order; scratch: the setup's counts / fill / scan (10 M bytes)
struct DirLds {
  size_t sel, csg, pairs, ulist, ustart, order, bins, misc, scratch, total;
};
HDI DirLds dir_lds(int M, int n) {
  DirLds L{};
  LdsTake take;
  L.sel = take(size_t(kBetaSamples) * n * 2);
  L.csg = take(size_t(kBetaSamples) * 4);
  L.pairs = take(size_t(kBetaSamples) * n * 2);
  L.ulist = take(size_t(M) * 2);
  L.ustart = take(size_t(M + 1) * 2);
  L.order = take(size_t(M) * 2);
  L.bins = take(kLptBins * 4);
  L.misc = take(32 * 4);  // [0] next row, [1] distinct rows, [16..] wave totals
  L.scratch = take(size_t(M) * 10);
  L.total = take.o;
  return L;
}

constexpr float kNegLog2e = kNegLog2eRow;

DEVI float dpp_f_ror8(float v) { return __int_as_float(dpp_i<0x128>(__float_as_int(v))); }

// v[j] per lane -> lanes 8 j + 4..7 hold the 64-lane sum of v[j] (row_ror:4
// moves lane i - 4 into lane i, so the 8-lane group's total lands in its upper quad)
DEVI float transpose_sum8(const float (&v)[8]) {
  const int lane = tidx() & 63;
  float a[4], c2[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // lanes 0-31: slots 0..3, lanes 32-63: slots 4..7
    float x = v[i], y = v[4 + i];
    permlane_swap<32>(x, y);
    a[i] = x + y;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // lane bit 4 picks slot 4 h + 2 b4 + i
    float x = a[i], y = a[2 + i];
    permlane_swap<16>(x, y);
    c2[i] = x + y;
  }
  const bool b3 = lane & 8;  // lane bit 3 picks slot 4 h + 2 b4 + b3 = lane >> 3
  const float y0 = dpp_f_ror8(c2[0]), y1 = dpp_f_ror8(c2[1]);
  float x = b3 ? c2[1] + y1 : c2[0] + y0;
  x += __int_as_float(dpp_i<0xB1>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x4E>(__float_as_int(x)));
  return x + __int_as_float(dpp_i<0x124>(__float_as_int(x)));
}

// 1 / (k + 1) for the Horner steps of the series
__constant__ double kInvK[kMom] = {1.0,       1.0 / 2,  1.0 / 3,  1.0 / 4,  1.0 / 5,  1.0 / 6,
                                   1.0 / 7,   1.0 / 8,  1.0 / 9,  1.0 / 10, 1.0 / 11, 1.0 / 12};

// row sum of one pair by the series: q = the row's record, na = -a.  The
// Horner sum in fp64; exp(-a) by v_exp_f32 (~1 ulp: the sum is rounded to
// fp32 anyway, as the reference's fp32 terms are)
DEVI float series_sum(const float4 (&q)[3], double na) {
  const double P[kMom] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y,
                          q[1].z, q[1].w, q[2].x, q[2].y, q[2].z, q[2].w};
  double h = P[kMom - 1];
#pragma unroll
  for (int k = kMom - 2; k >= 0; --k) h = fma(h, na * kInvK[k], P[k]);  // P_k + (-a / (k + 1)) h
  constexpr double kLog2e = 1.44269504088896340736;
  return float(double(__builtin_amdgcn_exp2f(float(na * kLog2e))) * h);
}
static_assert(kMomR == 12 && kMom == 12, "record layout: P_0..P_11 in float4s 0..2, R in float4 3");

// The body of k_bkernel for part `part` of candidate `cand` (of `split`),
// NW waves (k_bkernel: 16; the small-batch fused kernel k_bcem_small: 8)
// mom_l / feat_l: LDS copies of the candidate's series records and feature
// rows (k_bcem_small, which keeps them for its 20 beta-iterations), else null
// (read from global memory)
template <int NW, bool kList = false>
DEVI void bkernel_body(const Params& p, int tb, int cand, int part, int split, int scratch, char* smem,
                       const float4* mom_l = nullptr, const float4* feat_l = nullptr) {
  constexpr int kKerWaves = NW;
  constexpr int NT = 64 * kKerWaves, Q = kFeatStride / 4;
  const int b = p.b0 + cand, M = p.M, n = p.n;
  const int tid = tidx(), lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const KerLds C = ker_lds(M, n, size_t(scratch));
  short* sl = reinterpret_cast<short*>(smem + C.sel);
  float* csg = reinterpret_cast<float*>(smem + C.csg);
  double* csd = reinterpret_cast<double*>(smem + C.csd);
  unsigned short* tri = reinterpret_cast<unsigned short*>(smem + C.tri);
  unsigned short* urank = reinterpret_cast<unsigned short*>(smem + C.urank);
  unsigned short* urow = reinterpret_cast<unsigned short*>(smem + C.urow);
  int* misc = reinterpret_cast<int*>(smem + C.misc);
  unsigned char* uflag = reinterpret_cast<unsigned char*>(smem + C.scratch);  // setup only
  const int ntri = tri_stride(n), nent = n * (n - 1) / 2;
  const int s_lo = first_sample(tb);
  const int i_lo = s_lo * n, i_hi = kBetaSamples * n;
  MPCMMD_STAMP(p, 16);
  MPCMMD_STAMPW(p, 0);
  const int32_t* gsel = p.bsel + size_t(b) * kBetaSamples * n;
  for (int i = i_lo + tid; i < i_hi; i += NT) sl[i] = short(gsel[i]);
  for (int s = s_lo + tid; s < kBetaSamples; s += NT) {
    const float sg = p.bsig[size_t(b) * kBetaSamples + s];
    csg[s] = kNegLog2e / sg;
    csd[s] = 1.0 / double(sg);
  }
  for (int k = 1 + w; k < n; k += kKerWaves)  // entry k (k - 1) / 2 + kk of the strict lower triangle
    for (int kk = lane; kk < k; kk += 64) tri[k * (k - 1) / 2 + kk] = (unsigned short)(k | kk << 8);
  for (int r = tid; r < M; r += NT) uflag[r] = 0;
  if (tid < 3) misc[tid] = 0;
  __syncthreads();
  for (int i = i_lo + tid; i < i_hi; i += NT) uflag[sl[i]] = 1;
  __syncthreads();
  {  // union ranks: exclusive scan of the flags (thread runs, wave scans, wave totals)
    const int per = (M + NT - 1) / NT, a = tid * per, e = min(M, a + per);
    int sq = 0;
    for (int r = a; r < e; ++r) sq += uflag[r];
    int y = sq;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int yo = __shfl_up(y, o, 64);
      if (lane >= o) y += yo;
    }
    if (lane == 63) misc[16 + w] = y;
    __syncthreads();
    int base = 0;
    for (int v = 0; v < w; ++v) base += misc[16 + v];
    y += base - sq;
    if (tid == NT - 1) misc[0] = y + sq;
    for (int r = a; r < e; ++r) {
      if (uflag[r]) {
        urank[r] = (unsigned short)y;
        urow[y] = (unsigned short)r;
        ++y;
      }
    }
  }
  __syncthreads();  // the flags are dead: the scratch now holds the union's records
  MPCMMD_STAMPW(p, 1);
  const int Uu = misc[0];
  {
    // the union's records: staged in LDS when they fit, else read in place
    const float4* mom = mom_l ? mom_l : reinterpret_cast<const float4*>(p.bmom + size_t(b) * M * kMomStride);
    const bool staged = !mom_l && size_t(Uu) * kMomStride * 4 <= size_t(scratch);  // block-uniform
    float4* lrec = reinterpret_cast<float4*>(smem + C.scratch);
    if (staged)
      for (int i = tid; i < Uu * 4; i += NT) lrec[i] = mom[size_t(urow[i >> 2]) * 4 + (i & 3)];
    for (int i = i_lo + tid; i < i_hi; i += NT) sl[i] = short(urank[sl[i]]);  // rows -> union ranks
    __syncthreads();
    const float4* rec = staged ? lrec : mom;
    // series pairs of this part's samples; the others flagged for k_bdirect
    float* rowsum = p.brow + size_t(b) * kBetaSamples * n;
    unsigned char* dflag = p.bdflag + size_t(b) * kBetaSamples * n;
    int nd = 0;
    const int ns = (kBetaSamples - s_lo - part + split - 1) / split;
    for (int j = tid; j < ns * n; j += NT) {
      const int sj = j / n, s = s_lo + part + split * sj, i = s * n + (j - sj * n);
      const float4* q = rec + 4 * (staged ? int(sl[i]) : int(urow[sl[i]]));
      const double na = -double(q[3].x) * csd[s];  // -a, a = R / sigma
      const bool series = -na <= kSeriesAMax;     // NaN sigma: direct (NaN sum, as the reference)
      if (series) {
        const float4 qq[3] = {q[0], q[1], q[2]};
        rowsum[i] = series_sum(qq, na);
      }
      const bool direct = !series && tb > 0;  // first iteration: k_bmoment summed them
      dflag[i] = direct ? 1 : 0;
      nd += direct ? 1 : 0;
      if (kList) {  // the direct-pair list (its order is free: every pair's sum is its own)
        const unsigned long long m = __ballot(direct);  // one atomic per wave
        if (m) {
          const int ld = __builtin_ctzll(m);
          int at = 0;
          if (lane == ld) at = atomicAdd(&p.bdlcount[size_t(b) * kBetaIters + tb], __popcll(m));
          at = __shfl(at, ld, 64) + __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
          if (direct && at < kBetaSamples * n) p.bdlist[size_t(b) * kBetaSamples * n + at] = i;
        }
      }
    }
    nd = wave_total(nd);
    if (lane == 0) atomicAdd(&misc[2], nd);
    __syncthreads();  // the records are dead
    if (tid == 0) {
      p.bdcount[size_t(b) * kMaxSplit + part] = misc[2];
      atomicAdd(&p.stats[2], static_cast<unsigned long long>(ns * n - misc[2]));
      if (part == 0) atomicAdd(&p.stats[3], static_cast<unsigned long long>((kBetaSamples - s_lo) * nent));
    }
  }
  MPCMMD_STAMP(p, 17);
  MPCMMD_STAMPW(p, 2);
  const float4* fg = feat_l ? feat_l : reinterpret_cast<const float4*>(p.featr + size_t(b) * M * kFeatStride);
  float* kbase = p.bkred + size_t(b) * kBetaSamples * ntri;
  if (ker_tab_bytes(Uu) <= size_t(scratch)) {  // block-uniform
    float* T = reinterpret_cast<float*>(smem + C.scratch);
    float4* Fu = reinterpret_cast<float4*>(smem + C.scratch + ((size_t(Uu) * (Uu - 1) / 2 * 4 + 15) & ~size_t(15)));
    for (int i = tid; i < Uu * Q; i += NT) {
      const int u = i / Q;
      Fu[i] = fg[size_t(urow[u]) * Q + (i - u * Q)];
    }
    __syncthreads();
    // work items: (block of 64 rows a, chunk of 16 rows b below the block's last row)
    const int nab = (Uu + 63) >> 6;
    auto chunks = [&](int ab) { return (min(64 * ab + 63, Uu - 1) + 15) >> 4; };
    int items = 0;
    for (int ab = 0; ab < nab; ++ab) items += chunks(ab);
    for (int it = w; it < items; it += kKerWaves) {
      int ab = 0, c = it;
      while (c >= chunks(ab)) c -= chunks(ab++);
      const int a = 64 * ab + lane;
      float fa[kF];
      {
        const float4* src = Fu + min(a, Uu - 1) * Q;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const float4 v = src[q];
          fa[4 * q] = v.x;
          fa[4 * q + 1] = v.y;
          if (q < Q - 1) {
            fa[4 * q + 2] = v.z;
            fa[4 * q + 3] = v.w;
          }
        }
      }
      const int b_end = min(16 * c + 16, min(64 * ab + 63, Uu - 1));
      float* Ta = T + a * (a - 1) / 2;
#pragma unroll 2
      for (int bb = 16 * c; bb < b_end; ++bb) {
        const float4* fb = Fu + bb * Q;  // wave-uniform: LDS broadcast
        float dd = 0.0f;
#pragma unroll
        for (int q = 0; q < Q; ++q) {  // differences as packed pairs, the sum in feature order
          const float4 y = fb[q];
          const f2 d0 = f2{fa[4 * q], fa[4 * q + 1]} - f2{y.x, y.y};
          dd = q == 0 ? fabsf(d0.x) : dd + fabsf(d0.x);
          dd = dd + fabsf(d0.y);
          if (q < Q - 1) {
            const f2 d1 = f2{fa[4 * q + 2], fa[4 * q + 3]} - f2{y.z, y.w};
            dd = dd + fabsf(d1.x);
            dd = dd + fabsf(d1.y);
          }
        }
        if (bb < a && a < Uu) Ta[bb] = dd;
      }
    }
    __syncthreads();
    MPCMMD_STAMPW(p, 3);
#ifdef MPCMMD_FUSED_TU
    // k_bcem_small: the (sample, entry) items spread over every thread, kJ
    // items per thread in flight together (a wave per sample leaves most
    // lanes idle at small n: 45 entries at n = 10)
    constexpr int kJ = 4;
    const int ns = (kBetaSamples - s_lo - part + split - 1) / split, nitems = ns * nent;
    for (int i0 = tid; i0 < nitems; i0 += NT * kJ) {
      int s[kJ], e[kJ], t[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const int i = min(i0 + NT * j, nitems - 1), sj = i / nent;
        s[j] = s_lo + part + split * sj;
        e[j] = i - sj * nent;
        t[j] = tri[e[j]];
      }
      int u0[kJ], u1[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        u0[j] = sl[s[j] * n + (t[j] & 0xFF)];
        u1[j] = sl[s[j] * n + (t[j] >> 8)];
      }
      float dv[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const int hi = max(u0[j], u1[j]), lo = min(u0[j], u1[j]);
        dv[j] = T[hi * (hi - 1) / 2 + lo];
      }
#pragma unroll
      for (int j = 0; j < kJ; ++j)
        if (i0 + NT * j < nitems)
          kbase[size_t(s[j]) * ntri + e[j]] = kred_perturb(__builtin_amdgcn_exp2f(dv[j] * csg[s[j]]), e[j]);
    }
#else
    // a wave per sample of this part, all its lookups in flight together
    // (entries lane + 64 j, j < kJ covers n <= 23; larger n loop)
    constexpr int kJ = 4;
    for (int s = s_lo + part + split * w; s < kBetaSamples; s += split * kKerWaves) {
      const short* su = sl + s * n;
      const float cs = csg[s];
      float* kr = kbase + size_t(s) * ntri;
      for (int e0 = 0; e0 < nent; e0 += 64 * kJ) {
        int t[kJ];
#pragma unroll
        for (int j = 0; j < kJ; ++j) t[j] = tri[min(e0 + lane + 64 * j, nent - 1)];
        int u0[kJ], u1[kJ];
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
          u0[j] = su[t[j] & 0xFF];
          u1[j] = su[t[j] >> 8];
        }
        float dv[kJ];
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
          const int hi = max(u0[j], u1[j]), lo = min(u0[j], u1[j]);
          dv[j] = T[hi * (hi - 1) / 2 + lo];
        }
#pragma unroll
        for (int j = 0; j < kJ; ++j)
          if (e0 + lane + 64 * j < nent)
            kr[e0 + lane + 64 * j] = kred_perturb(__builtin_amdgcn_exp2f(dv[j] * cs), e0 + lane + 64 * j);
      }
    }
#endif
  } else {
    // per-sample: the union records are dead, sl holds union ranks (urow maps back)
    float4* Fw = reinterpret_cast<float4*>(smem + C.scratch) + size_t(w) * n * Q;
    for (int s = s_lo + part + split * w; s < kBetaSamples; s += split * kKerWaves) {
      for (int k = lane; k < n; k += 64) {
        const float4* src = fg + size_t(urow[sl[s * n + k]]) * Q;
#pragma unroll
        for (int q = 0; q < Q; ++q) Fw[k * Q + q] = src[q];
      }
      wave_sync();  // one wave's LDS operations run in order
      const float cs = csg[s];
      float* kr = kbase + size_t(s) * ntri;
      for (int e = lane; e < nent; e += 64) {
        const int kk2 = tri[e];
        const float4* A = Fw + (kk2 & 0xFF) * Q;
        const float4* Bv = Fw + (kk2 >> 8) * Q;
        float dd = 0.0f;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const float4 x = A[q], y = Bv[q];
          dd = q == 0 ? fabsf(x.x - y.x) : dd + fabsf(x.x - y.x);
          dd = dd + fabsf(x.y - y.y);
          if (q < Q - 1) {  // features 22, 23 are padding
            dd = dd + fabsf(x.z - y.z);
            dd = dd + fabsf(x.w - y.w);
          }
        }
        kr[e] = kred_perturb(__builtin_amdgcn_exp2f(dd * cs), e);
      }
      wave_sync();  // the reads are done before the next sample's rows overwrite them
    }
  }
  MPCMMD_STAMP(p, 18);
  MPCMMD_STAMPW(p, 4);
}

// two workgroups per CU: 8 waves per SIMD, which needs <= 64 VGPRs and <= 80
// SGPRs (MI355X_MICROARCH.md residency rules: 90 SGPRs admitted one)
#ifndef MPCMMD_FUSED_TU
template <bool kList>
__global__ __launch_bounds__(64 * kKerWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_bkernel(Params p, int tb, int split, int scratch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cand = blockIdx.x / split, part = blockIdx.x - cand * split;
  bkernel_body<kKerWaves, kList>(p, tb, cand, part, split, scratch, smem);
}
#endif

// flagged pairs of candidate b (k_bkernel's parts): k_bdirect's work
DEVI int bdirect_total(const Params& p, int b, int kparts) {
  int total = 0;
  for (int k = 0; k < kparts; ++k) total += p.bdcount[size_t(b) * kMaxSplit + k];
  return total;
}

// The body of k_bdirect for part `part` of candidate `cand` with `total` > 0
// flagged pairs, NW waves (k_bdirect: 4; k_bcem_small: 8)
template <int NV4, int NW>
DEVI void bdirect_body(const Params& p, int tb, int split, int lpt, int cand, int part, int total, char* smem) {
  constexpr int kDirWaves = NW;
  constexpr bool kPrefetch = NV4 <= 4;
  constexpr int NT = 64 * kDirWaves;
  const int b = p.b0 + cand, M = p.M, n = p.n, Md = dist_stride(M);
  const int tid = tidx(), lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const DirLds C = dir_lds(M, n);
  short* sl = reinterpret_cast<short*>(smem + C.sel);
  float* csg = reinterpret_cast<float*>(smem + C.csg);
  unsigned short* pairs = reinterpret_cast<unsigned short*>(smem + C.pairs);
  unsigned short* ulist = reinterpret_cast<unsigned short*>(smem + C.ulist);
  unsigned short* ustart = reinterpret_cast<unsigned short*>(smem + C.ustart);
  unsigned short* order = reinterpret_cast<unsigned short*>(smem + C.order);
  int* bins = reinterpret_cast<int*>(smem + C.bins);
  int* misc = reinterpret_cast<int*>(smem + C.misc);
  int* cnt = reinterpret_cast<int*>(smem + C.scratch);  // setup only
  int* fill = cnt + M;
  unsigned short* start = reinterpret_cast<unsigned short*>(fill + M);
  float* rowsum = p.brow + size_t(b) * kBetaSamples * n;
  const unsigned char* dflag = p.bdflag + size_t(b) * kBetaSamples * n;
  const int s_lo = first_sample(tb);
  const int i_lo = s_lo * n, i_hi = kBetaSamples * n;
  const int32_t* gsel = p.bsel + size_t(b) * kBetaSamples * n;
  MPCMMD_STAMPW(p, 5);
  // direct pairs keep their row; the others get row -1
  for (int i = i_lo + tid; i < i_hi; i += NT) sl[i] = dflag[i] ? short(gsel[i]) : short(-1);
  for (int s = s_lo + tid; s < kBetaSamples; s += NT) csg[s] = kNegLog2e / p.bsig[size_t(b) * kBetaSamples + s];
  for (int r = tid; r < M; r += NT) {
    cnt[r] = 0;
    fill[r] = 0;
  }
  if (tid == 0) misc[0] = 0;
  for (int c = tid; c < kLptBins; c += NT) bins[c] = 0;
  __syncthreads();
  for (int i = i_lo + tid; i < i_hi; i += NT)
    if (sl[i] >= 0) atomicAdd(&cnt[sl[i]], 1);
  __syncthreads();
  {  // exclusive scans of cnt and (cnt > 0), packed as cnt | (cnt > 0) << 16
     // (totals <= 6400 pairs, <= 4096 rows): thread runs, wave scans, wave totals
    const int per = (M + NT - 1) / NT, a = tid * per, e = min(M, a + per);
    int sp = 0;
    for (int r = a; r < e; ++r) {
      const int c = cnt[r];
      sp += c | (c > 0) << 16;
    }
    int x = sp;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) misc[16 + w] = x;
    __syncthreads();
    int base = 0;
    for (int v = 0; v < w; ++v) base += misc[16 + v];
    x += base - sp;  // exclusive prefix of this thread's run
    if (tid == NT - 1) {
      const int tot = x + sp;
      misc[1] = tot >> 16;
      ustart[tot >> 16] = (unsigned short)(tot & 0xFFFF);
    }
    for (int r = a; r < e; ++r) {
      const int c = cnt[r], x1 = x & 0xFFFF, x2 = x >> 16;
      start[r] = (unsigned short)x1;
      if (c > 0) {
        ulist[x2] = (unsigned short)r;
        ustart[x2] = (unsigned short)x1;
      }
      x += c | (c > 0) << 16;
    }
  }
  __syncthreads();
  const int U = misc[1];
  if (tid == 0 && part == 0) {
    atomicAdd(&p.stats[0], static_cast<unsigned long long>(U));
    atomicAdd(&p.stats[1], static_cast<unsigned long long>(total));
  }
  for (int i = i_lo + tid; i < i_hi; i += NT) {
    const int r = sl[i];
    if (r >= 0) pairs[start[r] + atomicAdd(&fill[r], 1)] = (unsigned short)i;
  }
  // grab order: heaviest rows (most pairs) first, so no wave starts a long
  // row while the others run dry (bucket sort by pair count; the order within
  // a bucket is arbitrary -- every row's outputs are independent of it -- so
  // only for a candidate in one workgroup: parts of a split candidate must
  // agree on the order)
  if (lpt && split == 1) {
    for (int u = tid; u < U; u += NT) atomicAdd(&bins[kLptBins - 1 - min(ustart[u + 1] - ustart[u], kLptBins - 1)], 1);
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the 128 bins, two per lane
      const int a = bins[2 * tid], c = bins[2 * tid + 1];
      int x = a + c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (tid >= o) x += y;
      }
      bins[2 * tid] = x - a - c;
      bins[2 * tid + 1] = x - c;
    }
    __syncthreads();
    for (int u = tid; u < U; u += NT)
      order[atomicAdd(&bins[kLptBins - 1 - min(ustart[u + 1] - ustart[u], kLptBins - 1)], 1)] = (unsigned short)u;
  } else {
    for (int u = tid; u < U; u += NT) order[u] = (unsigned short)u;
  }
  __syncthreads();
  MPCMMD_STAMP(p, 19);
  MPCMMD_STAMPW(p, 6);
  const float4* Dg = reinterpret_cast<const float4*>(p.bdist + size_t(b) * M * Md);
  // this part's rows order[part + split q], q from the workgroup's counter
  // (U: past the end)
  auto grab = [&]() {
    int q = 0;
    if (lane == 0) q = atomicAdd(&misc[0], 1);
    const int i = part + split * __builtin_amdgcn_readfirstlane(q);
    return i < U ? int(order[i]) : U;
  };
  auto load = [&](float4 (&x)[NV4], int u) {
    const float4* src = Dg + size_t(ulist[u]) * (Md >> 2) + lane;
#pragma unroll
    for (int t = 0; t < NV4; ++t) x[t] = src[64 * t];
  };
  // one distinct row u held in x: its pairs 8 at a time
  auto do_row = [&](const float4 (&x)[NV4], int u) {
    const int pb = ustart[u], pc = ustart[u + 1] - pb;
    for (int c0 = 0; c0 < pc; c0 += 64) {  // (rows with more than 64 pairs: chunks)
      // lane l holds pair c0 + l and its scale; batches broadcast them by readlane
      const int cc = min(64, pc - c0);
      const int pl = pairs[pb + c0 + min(lane, cc - 1)];
      const float cl = csg[pl / n];
      for (int j0 = 0; j0 < cc; j0 += 8) {
        float v[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          v[jj] = 0.0f;
          if (j0 + jj < cc) {
            const float cn = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cl), j0 + jj));
            const f2 c2 = {cn, cn};
            f2 a0, a1;
#pragma unroll
            for (int t = 0; t < NV4; ++t) {
              const f2 t0 = f2{x[t].x, x[t].y} * c2, t1 = f2{x[t].z, x[t].w} * c2;
              const f2 e0 = {__builtin_amdgcn_exp2f(t0.x), __builtin_amdgcn_exp2f(t0.y)};
              const f2 e1 = {__builtin_amdgcn_exp2f(t1.x), __builtin_amdgcn_exp2f(t1.y)};
              a0 = t == 0 ? e0 : a0 + e0;
              a1 = t == 0 ? e1 : a1 + e1;
            }
            a0 += a1;
            v[jj] = a0.x + a0.y;
          }
        }
        const float sum = transpose_sum8(v);
        // lane group j = lane >> 3 takes pair j0 + j
        const int jg = j0 + (lane >> 3);
        const int pj = __shfl(pl, jg, 64);
        if ((lane & 7) == 4 && jg < cc) rowsum[pj] = sum;
      }
    }
  };
  float4 d[NV4];
  int u = grab();
  if (kPrefetch) {
    // ping-pong: the next row's loads are issued (unconditionally, a past-the-
    // end index clamped to the current row) before the current row is summed,
    // so the memory-counter waits are exact and the loads overlap the exps
    float4 dn[NV4];
    if (u < U) load(d, u);
    while (u < U) {
      const int un = grab();
      load(dn, un < U ? un : u);
      do_row(d, u);
      if (un >= U) break;
      const int unn = grab();
      load(d, unn < U ? unn : un);
      do_row(dn, un);
      u = unn;
    }
  } else {
    for (; u < U; u = grab()) {
      load(d, u);
      do_row(d, u);
    }
  }
  MPCMMD_STAMP(p, 20);
  MPCMMD_STAMPW(p, 7);
}

#ifndef MPCMMD_FUSED_TU
template <int NV4, int NW>
__global__ __launch_bounds__(64 * NW) void k_bdirect(Params p, int tb, int kparts, int split, int lpt) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cand = blockIdx.x / split, part = blockIdx.x - cand * split;
  const int total = bdirect_total(p, p.b0 + cand, kparts);
  if (total == 0) return;  // block-uniform
  bdirect_body<NV4, NW>(p, tb, split, lpt, cand, part, total, smem);
}
#endif

// Direct row sums from k_bkernel's list of flagged pairs (k_bdirect_pairs),
// no per-candidate setup (bdirect_body counting-sorts the
// pairs by mother row in LDS first, which at the reference's num_batch = 100
// -- CARLA, where about half of all pairs are direct at every beta-iteration
// -- costs more than the sums).  A wave takes PJ listed pairs, issues all
// their distance-row loads (lane L: float4s L + 64 t of row sel[i]) before the
// first exponential, forms each pair's per-lane terms exactly as
// bdirect_body's do_row (packed scale, v_exp_f32, the same pairwise order),
// and reduces the PJ slots by one transpose_sum8, whose tree is the same for
// every slot: the bits of bdirect_body.
// Groups g0, g0 + gs, .. of PJ listed pairs of candidate b (cnt pairs) on the
// calling wave.
template <int NV4, int PJ>
DEVI void direct_pairs_wave(const Params& p, int b, int cnt, int g0, int gs) {
  static_assert(PJ >= 1 && PJ <= 8, "pairs per wave");
  const int M = p.M, n = p.n, Md = dist_stride(M);
  const int lane = tidx() & 63;
  const int groups = (cnt + PJ - 1) / PJ;
  const int32_t* list = p.bdlist + size_t(b) * kBetaSamples * n;
  const int32_t* gsel = p.bsel + size_t(b) * kBetaSamples * n;
  const float* gsig = p.bsig + size_t(b) * kBetaSamples;
  float* rowsum = p.brow + size_t(b) * kBetaSamples * n;
  const float4* Dg = reinterpret_cast<const float4*>(p.bdist + size_t(b) * M * Md);
  for (int g = g0; g < groups; g += gs) {
    int pi[PJ];
    float cs[PJ];
    float4 x[PJ][NV4];
#pragma unroll
    for (int j = 0; j < PJ; ++j) {  // a past-the-end slot repeats the group's first pair (not stored)
      const int k = g * PJ + j < cnt ? g * PJ + j : g * PJ;
      pi[j] = list[k];
    }
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const float4* src = Dg + size_t(gsel[pi[j]]) * (Md >> 2) + lane;
#pragma unroll
      for (int t = 0; t < NV4; ++t) x[j][t] = src[64 * t];
      cs[j] = kNegLog2e / gsig[pi[j] / n];
    }
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.0f;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const f2 c2 = {cs[j], cs[j]};
      f2 a0, a1;
#pragma unroll
      for (int t = 0; t < NV4; ++t) {
        const f2 t0 = f2{x[j][t].x, x[j][t].y} * c2, t1 = f2{x[j][t].z, x[j][t].w} * c2;
        const f2 e0 = {__builtin_amdgcn_exp2f(t0.x), __builtin_amdgcn_exp2f(t0.y)};
        const f2 e1 = {__builtin_amdgcn_exp2f(t1.x), __builtin_amdgcn_exp2f(t1.y)};
        a0 = t == 0 ? e0 : a0 + e0;
        a1 = t == 0 ? e1 : a1 + e1;
      }
      a0 += a1;
      v[j] = a0.x + a0.y;
    }
    const float sum = transpose_sum8(v);  // slot j's total in lanes 8 j + 4..7
    const int j = lane >> 3;
    int pj = pi[0];
#pragma unroll
    for (int q = 1; q < PJ; ++q) pj = j == q ? pi[q] : pj;
    if ((lane & 7) == 4 && j < PJ && g * PJ + j < cnt) rowsum[pj] = sum;
  }
}

// pairs per wave of the pair-list direct sums: as many distance rows in flight
// as fit ~64 VGPRs of operands (NV4 float4s per lane and row)
HDI_CONST int direct_pj(int nv4) { return nv4 <= 2 ? 8 : (nv4 <= 4 ? 4 : (nv4 <= 8 ? 2 : 1)); }

#ifndef MPCMMD_FUSED_TU
// k_bdirect_pairs, workgroup = (candidate, part), kDirWaves waves each
template <int NV4, int PJ>
__global__ __launch_bounds__(64 * kDirWaves) void k_bdirect_pairs(Params p, int tb, int parts) {
  // a candidate's parts on blocks of one blockIdx % 8 (one XCD under the
  // observed round-robin dispatch, for L2 reuse of its distance rows; any
  // placement is correct): the grid is a multiple of 8, its block L of XCD
  // group x = blockIdx % 8 is the (x * grid / 8 + blockIdx / 8)-th (cand, part)
  const int per = gridDim.x >> 3, L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const int cand = L / parts, part = L - cand * parts;
  if (cand >= p.nb) return;
  const int b = p.b0 + cand, n = p.n;
  const int w = __builtin_amdgcn_readfirstlane(int(tidx()) >> 6);
  const int cnt = min(p.bdlcount[size_t(b) * kBetaIters + tb], kBetaSamples * n);
  if (part * kDirWaves >= (cnt + PJ - 1) / PJ) return;  // block-uniform
  if (part == 0 && tidx() == 0) atomicAdd(&p.stats[1], static_cast<unsigned long long>(cnt));
  direct_pairs_wave<NV4, PJ>(p, b, cnt, part * kDirWaves + w, parts * kDirWaves);
}
#endif

// ------------------------------------------------------------------------
// k_bqp: compute_beta_reduced (compute_beta.py:70-91) for every sample:
// C = K_red + 0.05 I, C x1 = g, C x2 = 1, beta = x1 + ((1 - sum x1) / sum x2) x2
// (the (n+1) KKT system).  The factorisation and the solves are fp32, the
// reference's precision (jnp.linalg.solve on fp32, compute_beta.py:79); the
// cost beta^T K beta - 2 g^T beta is accumulated in fp64 from the fp32 beta
// and the re-read K_red, so it carries no factorisation error.
//
// A quad (4 lanes) per QP, 16 QPs per wave: lane q owns rows i = 4t + q of
// the (padded to NP) matrix, in registers.  Right-looking Cholesky; the
// column entries every lane needs are quad broadcasts (DPP quad_perm, no
// LDS, no barriers); the triangular solves are a row sweep (forward, quad
// broadcast of y_j) and a column sweep (backward, quad sum of partials).
// Entries above the diagonal are kept at exactly 0, padding rows are
// identity with zero right-hand sides.
// value of quad lane l (0..3) in every lane of the quad; l is a constant
// after unrolling, so the switch folds
DEVI float quad_bcast(float v, int l) {
  const int b = __float_as_int(v);
  switch (l & 3) {
    case 0: return __int_as_float(dpp_full<0x00>(b));
    case 1: return __int_as_float(dpp_full<0x55>(b));
    case 2: return __int_as_float(dpp_full<0xAA>(b));
    default: return __int_as_float(dpp_full<0xFF>(b));
  }
}
DEVI double quad_bcast(double v, int l) {
  const long long b = __double_as_longlong(v);
  int lo = int(b), hi = int(b >> 32);
  switch (l & 3) {
    case 0: lo = dpp_full<0x00>(lo), hi = dpp_full<0x00>(hi); break;
    case 1: lo = dpp_full<0x55>(lo), hi = dpp_full<0x55>(hi); break;
    case 2: lo = dpp_full<0xAA>(lo), hi = dpp_full<0xAA>(hi); break;
    default: lo = dpp_full<0xFF>(lo), hi = dpp_full<0xFF>(hi); break;
  }
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
// sum over the quad, bit-identical in its 4 lanes
DEVI float quad_sum(float v) {
  v = v + __int_as_float(dpp_full<0xB1>(__float_as_int(v)));  // quad_perm(1,0,3,2)
  return v + __int_as_float(dpp_full<0x4E>(__float_as_int(v)));  // quad_perm(2,3,0,1)
}
DEVI double quad_sum(double v) {
  auto sw = [](double x, auto f) {
    const long long b = __double_as_longlong(x);
    return __longlong_as_double((static_cast<long long>(f(int(b >> 32))) << 32) | static_cast<unsigned>(f(int(b))));
  };
  v = v + sw(v, [](int x) { return dpp_full<0xB1>(x); });
  return v + sw(v, [](int x) { return dpp_full<0x4E>(x); });
}
// 1 / sqrt(x): v_rsq_f32 and one Newton step
DEVI float rsqrt_nr(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
  return y * fmaf(-0.5f * x, y * y, 1.5f);
}

// zero floats after the staged triangles (bqp_solve's padding rows and
// reads past a row end: at most NP - 1 <= 31 floats past a triangle)
constexpr int kQpZeros = 64;

// K_red of the workgroup's QPs is staged in LDS first (consecutive
// threads copy consecutive entries of one QP's triangle: coalesced), so the
// per-lane row gathers of the factorisation and the cost read LDS, not
// scattered global lines.
DEVI void bqp_stage(const Params& p, int tb, float* kl) {
  const int n = p.n;
  const int s_lo = first_sample(tb), per = kBetaSamples - s_lo;
  const int ntri = tri_stride(n), n4 = ntri >> 2;
  const int nq = blockDim.x >> 2, q0 = blockIdx.x * nq, total = p.nb * per;
  {  // the workgroup's K_red rows as float4s, consecutive threads on consecutive
     // float4s, every thread's loads issued before its first LDS store (one
     // memory latency, not one per four rows).  QP g = q0 + j (clamped to the
     // last) is sample s0 + j of candidate c0 while s0 + j < per, else sample
     // s0 + j - per of candidate c0 + 1 (nq < per): its triangle is the
     // (j + (j >= jw ? s_lo : 0))-th past the first one's.  Float4 (j, r) of
     // the staging advances by (T / n4, T % n4) per round of T threads.
    const int c0 = q0 / per, s0 = q0 - c0 * per, jw = per - s0, jmax = min(nq, total - q0) - 1;
    const float4* src = reinterpret_cast<const float4*>(p.bkred + (size_t(p.b0 + c0) * kBetaSamples + s_lo + s0) * ntri);
    float4* kl4 = reinterpret_cast<float4*>(kl);
    const int T = blockDim.x, dj = T / n4, dr = T - dj * n4;
    int j = int(tidx()) / n4, r = int(tidx()) - j * n4;
    constexpr int kU = 16;  // float4s per thread and round: 32 QPs x 58 float4s fit one round at n = 22
    for (int i0 = 0; i0 < nq * n4; i0 += kU * T) {
      float4 v[kU];
      int jj[kU], rr[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        jj[u] = j;
        rr[u] = r;
        const int jc = min(j, jmax);
        v[u] = src[(jc + (jc >= jw ? s_lo : 0)) * n4 + r];
        j += dj;
        r += dr;
        if (r >= n4) {
          r -= n4;
          ++j;
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (jj[u] < nq) kl4[jj[u] * n4 + rr[u]] = v[u];
    }
    if (int(tidx()) < kQpZeros) kl[nq * ntri + tidx()] = 0.0f;  // the padding rows' zeros
    __syncthreads();
  }
}

// QP of sample s of candidate b on the calling quad (lane q = tidx() & 3),
// its K_red strict lower triangle at kr (LDS staging); zr: kQpZeros zero
// floats (the padding rows' entries), placed right after the last staged
// triangle, so every read past a row end -- masked, never used -- lands on
// K_red entries or zeros; ok = false: compute on the clamped inputs, store
// nothing
template <int NP>
DEVI void bqp_solve(const Params& p, int b, int s, bool ok, const float* kr, const float* zr) {
  constexpr int T4 = NP / 4;
  const int n = p.n, M = p.M, q = tidx() & 3;
  const float* br = p.brow + (size_t(b) * kBetaSamples + s) * n;
  const double inv_m = double(1.0f / float(M));
  const float cdiag = 1.0f + 0.05f;
  // row i = 4t+q of K_red (k_bkernel's strict lower triangle: entry (i, k < i)
  // at i (i-1)/2 + k), read at constant offsets k <= 4t+3 past the row start
  // (entries k >= i are the next row's or zeros, masked); padding rows i >= n
  // read zeros
  const float* rowp[T4];
#pragma unroll
  for (int t = 0; t < T4; ++t) {
    const int i = 4 * t + q;
    rowp[t] = i < n ? kr + i * (i - 1) / 2 : zr;
  }
  // own rows: A[t][k] = C[4t+q][k], k <= 4t+3; loaded as K_red (every load
  // unconditional, so they are all in flight together), factored in place
  float A[T4][NP];
  float a1[T4], a2[T4], rin[T4];
#pragma unroll
  for (int t = 0; t < T4; ++t) {
#pragma unroll
    for (int k = 0; k < NP; ++k)
      if (k <= 4 * t + 3) A[t][k] = rowp[t][k];
    const int i = 4 * t + q;
    const float g = float(double(br[min(i, n - 1)]) * inv_m);
    a1[t] = i < n ? g : 0.0f;
    a2[t] = i < n ? 1.0f : 0.0f;
    rin[t] = 0.0f;
  }
#if defined(MPCMMD_QP_VARIANT) && MPCMMD_QP_VARIANT >= 2
  // PMC attribution builds (tools/qp_variants.sh; results are garbage):
  // 2 = staging + the row loads only, 3 = staging only
  {
    float acc = 0.0f;
#if MPCMMD_QP_VARIANT == 2
#pragma unroll
    for (int t = 0; t < T4; ++t)
#pragma unroll
      for (int k = 0; k < NP; ++k)
        if (k <= 4 * t + 3) acc += A[t][k];
#endif
    if (ok && acc == 12345.0f) p.bcost[size_t(b) * kBetaSamples + s] = acc;
    return;
  }
#endif
  // C in place: strict lower part from K_red, the diagonal 1.05 (1 for the
  // padding rows), entries above the diagonal 0
#pragma unroll
  for (int t = 0; t < T4; ++t)
#pragma unroll
    for (int k = 0; k <= 4 * t + 3; ++k) {
      const int i = 4 * t + q;
      float v = k < i ? A[t][k] : 0.0f;  // padding rows: zeros
      if (k == i) v = i < n ? cdiag : 1.0f;
      A[t][k] = v;
    }
  // Cholesky, right-looking: column k scaled by 1 / sqrt(C_kk), then the
  // trailing columns c > k updated (every update of a step independent)
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int tk = k >> 2, qk = k & 3;
    const float sv = quad_bcast(A[tk][k], qk);  // the pivot, from the lane owning row k
    const float y = rsqrt_nr(sv);
    if (q == qk) rin[tk] = y;
#pragma unroll
    for (int t = tk; t < T4; ++t) {
      const float v = A[t][k] * y;
      A[t][k] = t > tk ? v : (q > qk ? v : (q == qk ? sv * y : 0.0f));
    }
#pragma unroll
    for (int c = k + 1; c < NP; ++c) {
      const int tc = c >> 2;
      const float lck = quad_bcast(A[tc][k], c & 3);  // L_ck from the lane owning row c
      // rows (t, t + 1), t even, as packed pairs (v_pk_fma_f32: two fmaf)
      int t = tc;
      if (t & 1) {
        A[t][c] = fmaf(-A[t][k], lck, A[t][c]);
        ++t;
      }
#pragma unroll
      for (; t + 1 < T4; t += 2) {
        const f2 x = __builtin_elementwise_fma(f2{-A[t][k], -A[t + 1][k]}, f2{lck, lck}, f2{A[t][c], A[t + 1][c]});
        A[t][c] = x.x;
        A[t + 1][c] = x.y;
      }
      if (t < T4) A[t][c] = fmaf(-A[t][k], lck, A[t][c]);
    }
  }
  // forward: L y = (g, 1)
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int tj = j >> 2, qj = j & 3;
    const float y1 = a1[tj] * rin[tj], y2 = a2[tj] * rin[tj];
    if (q == qj) {
      a1[tj] = y1;
      a2[tj] = y2;
    }
    const float b1 = quad_bcast(y1, qj), b2 = quad_bcast(y2, qj);
#pragma unroll
    for (int t = tj; t < T4; ++t) {
      const float lij = (t == tj && q <= qj) ? 0.0f : A[t][j];
      a1[t] = fmaf(-lij, b1, a1[t]);
      a2[t] = fmaf(-lij, b2, a2[t]);
    }
  }
  // C^-1 = L^-T L^-1, so with y1 = L^-1 g, y2 = L^-1 1: sum x1 = y2 . y1,
  // sum x2 = |y2|^2 and beta = L^-T (y1 + alpha y2) -- one backward sweep
  float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
  for (int t = 0; t < T4; ++t) {  // padding rows hold y = 0
    s1 = fmaf(a2[t], a1[t], s1);
    s2 = fmaf(a2[t], a2[t], s2);
  }
  s1 = quad_sum(s1);
  s2 = quad_sum(s2);
  const float alpha = (1.0f - s1) / s2;
#pragma unroll
  for (int t = 0; t < T4; ++t) a1[t] = fmaf(alpha, a2[t], a1[t]);
  // backward: L^T beta = y1 + alpha y2 (beta overwrites it row by row, last row first)
#pragma unroll
  for (int j = NP - 1; j >= 0; --j) {
    const int tj = j >> 2, qj = j & 3;
    float p1 = 0.0f;
#pragma unroll
    for (int t = tj; t < T4; ++t) {
      const float lij = (t == tj && q <= qj) ? 0.0f : A[t][j];
      p1 = fmaf(lij, a1[t], p1);
    }
    p1 = quad_sum(p1);
    if (q == qj) a1[tj] = (a1[tj] - p1) * rin[tj];
  }
  float bf[T4];
#pragma unroll
  for (int t = 0; t < T4; ++t) bf[t] = 4 * t + q < n ? a1[t] : 0.0f;
#if defined(MPCMMD_QP_VARIANT) && MPCMMD_QP_VARIANT == 1
  // PMC attribution build: no cost phase (the K_red re-read)
  if (ok && q == 0) p.bcost[size_t(b) * kBetaSamples + s] = bf[0];
  return;
#endif
  // cost = beta^T K beta - 2 g^T beta in fp64, K = K_red re-read (unit
  // diagonal): r_i = sum_{k<i} K_ik beta_k by columns k, column k + 1's
  // entries in flight while column k is summed (two columns live, not the
  // whole triangle); row i contributes beta_i (beta_i + 2 r_i).  An entry
  // outside the triangle is a zero (padding rows) or masked to zero (k >= i
  // in the diagonal block), and fma(0, beta_k, r) = r: the masked sum's bits
  double r[T4];
  float kc[T4], kn[T4];
#pragma unroll
  for (int t = 0; t < T4; ++t) {
    r[t] = 0.0;
    kc[t] = rowp[t][0];
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) {
#pragma unroll
    for (int t = (k + 1) >> 2; t < T4; ++t) kn[t] = rowp[t][min(k + 1, NP - 1)];
    __builtin_amdgcn_sched_barrier(0);
    const double bk = double(quad_bcast(bf[k >> 2], k & 3));
#pragma unroll
    for (int t = k >> 2; t < T4; ++t) {
      const float kv = t == (k >> 2) && !(k < 4 * t + q) ? 0.0f : kc[t];
      r[t] = fma(double(kv), bk, r[t]);
      kc[t] = kn[t];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  double c1 = 0.0, c3 = 0.0;
#pragma unroll
  for (int t = 0; t < T4; ++t) {
    const int i = 4 * t + q;
    const double bi = double(bf[t]);
    c1 = fma(bi, fma(2.0, r[t], bi), c1);
    c3 = fma(i < n ? double(br[min(i, n - 1)]) * inv_m : 0.0, bi, c3);
  }
  c1 = quad_sum(c1);
  c3 = quad_sum(c3);
  if (!ok) return;
  float* bt = p.btop + (size_t(b) * kBetaSamples + s) * n;
#pragma unroll
  for (int t = 0; t < T4; ++t)
    if (4 * t + q < n) bt[4 * t + q] = bf[t];
  if (q == 0) p.bcost[size_t(b) * kBetaSamples + s] = float(c1 - 2.0 * c3);
}

template <int NP>
DEVI void bqp_quad(const Params& p, int tb, float* kl) {
  const int s_lo = first_sample(tb), per = kBetaSamples - s_lo;
  const int gq = (blockIdx.x * blockDim.x + tidx()) >> 2;
  const bool ok = gq < p.nb * per;
  const int gqc = ok ? gq : 0;
  const int b = p.b0 + gqc / per, s = s_lo + gqc % per;
  bqp_stage(p, tb, kl);
  bqp_solve<NP>(p, b, s, ok, kl + (tidx() >> 2) * tri_stride(p.n), kl + (blockDim.x >> 2) * tri_stride(p.n));
}

// padded QP size (a multiple of 4: rows 4 t + q on quad lane q).  The
// padding rows are identity rows with zero right-hand sides, whose every
// contribution to the real rows is an exact zero: any NP >= n gives the same
// bits
HDI int qp_np(int n) {
  return n <= 8 ? 8 : (n <= 12 ? 12 : (n <= 16 ? 16 : (n <= 24 ? 24 : (n <= 32 ? 32 : (n <= 48 ? 48 : 64)))));
}
// threads per workgroup: 32 QPs (their K_red in LDS: 30 KB at n = 22), 16 QPs
// for n > 24 (32 KB at n = 32, so the LDS still admits 4 workgroups per CU)
HDI_CONST int qp_threads(int np) { return np > 24 ? 64 : 128; }

#ifndef MPCMMD_FUSED_TU
template <int NP>
__global__ __launch_bounds__(qp_threads(NP), NP == 24 ? 3 : (NP <= 16 ? 4 : 2)) void k_bqp(Params p, int tb) {
  extern __shared__ __attribute__((aligned(16))) float kl[];
  bqp_quad<NP>(p, tb, kl);
}
#endif

// k_bqp_wave: the same QP for 32 < n <= 64, one wave per QP, lane i owns
// row i of C (NP floats in registers).  Right-looking Cholesky with the
// column entries broadcast by v_readlane (entries above the diagonal are
// left stale and zeroed when their column is reached, never read); forward
// solves for g and 1 together; then, since C^-1 = L^-T L^-1,
//   sum x1 = y2.y1, sum x2 = |y2|^2, beta = L^-T (y1 + alpha y2),
// one backward solve (column sums as wave reductions).  fp32 like the quad
// kernel; the cost beta^T K beta - 2 g^T beta in fp64 on the fp32 beta with
// K_red re-read.
#ifndef MPCMMD_FUSED_TU
template <int NP>
__global__ __launch_bounds__(256) void k_bqp_wave(Params p, int tb) {
  const int lane = tidx() & 63;
  const int n = p.n, M = p.M;
  const int s_lo = first_sample(tb), per = kBetaSamples - s_lo;
  const int gq = blockIdx.x * 4 + (tidx() >> 6);
  if (gq >= p.nb * per) return;  // whole waves
  const int b = p.b0 + gq / per, s = s_lo + gq % per;
  const int ntri = tri_stride(n);
  const float* kr = p.bkred + (size_t(b) * kBetaSamples + s) * ntri;
  const float* br = p.brow + (size_t(b) * kBetaSamples + s) * n;
  const double inv_m = double(1.0f / float(M));
  const float cdiag = 1.0f + 0.05f;
  const bool real = lane < n;
  float A[NP];
  const int ic = min(lane, n - 1);
#pragma unroll
  for (int k = 0; k < NP; ++k) {  // unconditional loads (clamped entry), masked after
    const int e = ic > 0 ? ic * (ic - 1) / 2 + max(min(k, ic - 1), 0) : 0;
    A[k] = kr[e];
  }
  const double gd = real ? double(br[ic]) * inv_m : 0.0;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    float v = (k < lane && real) ? A[k] : 0.0f;
    if (k == lane) v = real ? cdiag : 1.0f;
    A[k] = v;
  }
  float rdiag = 1.0f;
  // Cholesky, column j
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const float djj = readlane_f(A[j], j);
    const float y = rsqrt_nr(djj);
    const float lij = A[j] * y;
    A[j] = lane > j ? lij : (lane == j ? djj * y : 0.0f);
    if (lane == j) rdiag = y;
#pragma unroll
    for (int k = j + 1; k < NP; ++k) A[k] = fmaf(-A[j], readlane_f(A[j], k), A[k]);
  }
  // forward: L y = (g, 1)
  float y1 = float(gd), y2 = real ? 1.0f : 0.0f;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const float t1 = readlane_f(y1 * rdiag, j), t2 = readlane_f(y2 * rdiag, j);
    y1 = lane == j ? t1 : fmaf(-A[j], t1, y1);
    y2 = lane == j ? t2 : fmaf(-A[j], t2, y2);
  }
  const float s1 = wave_total(y2 * y1), s2 = wave_total(y2 * y2);
  const float alpha = (1.0f - s1) / s2;
  const float wv = fmaf(alpha, y2, y1);
  // backward: L^T beta = w
  float bet = 0.0f;
#pragma unroll
  for (int j = NP - 1; j >= 0; --j) {
    const float r = wave_total(A[j] * bet);
    if (lane == j) bet = (wv - r) * rdiag;
  }
  const float bf = real ? bet : 0.0f;
  const double bd = double(bf);
  // cost = bd^T K bd - 2 g^T bd, K = K_red (unit diagonal)
  double kb = bd;
#pragma unroll 8
  for (int k = 0; k < NP; ++k) {
    const double bk = double(readlane_f(bf, k));
    if (k != lane && real && k < n) {
      const int e = k < lane ? lane * (lane - 1) / 2 + k : k * (k - 1) / 2 + lane;
      kb = fma(double(kr[e]), bk, kb);
    }
  }
  const double c1 = wave_total(bd * kb), c3 = wave_total(gd * bd);
  float* bt = p.btop + (size_t(b) * kBetaSamples + s) * n;
  if (real) bt[lane] = bf;
  if (lane == 0) p.bcost[size_t(b) * kBetaSamples + s] = float(c1 - 2.0 * c3);
}
#endif

// ------------------------------------------------------------------------
// k_belite: elites, mean, next generators; on the last iteration the outputs
// (beta_best, sigma_best with the post-update quirk Q4, the reduced set).
// Positions are thread-strided (lane = position), so a wave covers four
// whole 16-position blocks: mean and u_j stay in the thread's registers and
// the block sums of u u^T are row-of-16 DPP reductions.  LDS holds only the
// block sums (nblk x 66 fp64) and small bookkeeping.
struct EliteLds {
  size_t Gb, misc, carry, ublk, total;
};
constexpr int kUPitch = 12;  // doubles per position row of the per-wave u staging
HDI EliteLds elite_lds(int M1, int waves = kThreads / 64) {
  EliteLds L{};
  const int nblk = (M1 + 15) / 16;
  L.Gb = 0;
  L.misc = (size_t(nblk) * 66 * 8 + 15) & ~size_t(15);
  L.carry = L.misc + 1024;
  L.ublk = (L.carry + size_t(kBetaElite) * (2 * kMaxReduced + 2) * 4 + 15) & ~size_t(15);
  L.total = L.ublk + size_t(waves) * 16 * kUPitch * 8;  // one 16-position block per wave
  return L;
}

// packed upper index of (a <= c) in an 11 x 11 symmetric matrix
HDI int sym11(int a, int c) { return a * 11 - a * (a - 1) / 2 + (c - a); }

// The body of k_belite for candidate b (any whole number of waves)
DEVI void belite_body(const Params& p, int tb, int b, char* smem) {
  const int M = p.M, M1 = M + 1, n = p.n, tid = tidx();
  const EliteLds C = elite_lds(M1, blockDim.x >> 6);
  double* Gb = reinterpret_cast<double*>(smem + C.Gb);
  int* elite = reinterpret_cast<int*>(smem + C.misc);    // [11]
  int* info = elite + 16;                                 // [0] imin, [1] any NaN
  float* cst = reinterpret_cast<float*>(info + 16);       // [100]
  float* sig_new = cst + kBetaSamples;                    // [11] sigma of the new elite rows
  uint32_t* ckey = reinterpret_cast<uint32_t*>(sig_new + 12);  // [100] sort keys of the costs (16-byte aligned)
  const float* costs = p.bcost + size_t(b) * kBetaSamples;
  if (tid < kBetaSamples) {
    const float c = costs[tid];
    cst[tid] = c;
    ckey[tid] = sort_key(c);
  }
  if (tid == 0) {
    info[0] = -1;
    info[1] = 0;
  }
  __syncthreads();
  if (tid < kBetaSamples) {
    // stable rank: 25 broadcast reads of four keys each, all in flight
    const uint32_t ks = ckey[tid];
    const uint4* k4 = reinterpret_cast<const uint4*>(ckey);
    int r = 0;
#pragma unroll
    for (int k = 0; k < kBetaSamples / 4; ++k) {
      const uint4 v = k4[k];
      r += int(v.x < ks || (v.x == ks && 4 * k < tid)) + int(v.y < ks || (v.y == ks && 4 * k + 1 < tid)) +
           int(v.z < ks || (v.z == ks && 4 * k + 2 < tid)) + int(v.w < ks || (v.w == ks && 4 * k + 3 < tid));
    }
    if (r < kBetaElite) elite[r] = tid;
    if (cst[tid] != cst[tid]) {
      atomicOr(&info[1], 1);
      atomicMin(reinterpret_cast<unsigned*>(&info[0]), unsigned(tid));  // first NaN (-1 == max)
    }
  }
  __syncthreads();
  const int imin = info[1] ? info[0] : elite[0];  // jnp.argmin: first NaN, else first minimum
  if (tid == 0) {
    p.res_beta[size_t(b) * kBetaIters + tb] = info[1] ? __int_as_float(0x7fc00000) : cst[elite[0]];
    double es = 0.0;  // elite costs in rank order (the parity trace; tests/parity.py)
    for (int q = 0; q < kBetaElite; ++q) es += double(cst[elite[q]]);
    p.btrace[size_t(b) * kBetaIters + tb] = float(es);
  }
  // the elites are samples 0..10 of the next iteration, unchanged: carry
  // their top-n rows, sigma, QP solution and cost there (first_sample)
  if (tb < kBetaIters - 1) {
    int* csel = reinterpret_cast<int*>(smem + C.carry);
    float* ctop = reinterpret_cast<float*>(csel + kBetaElite * n);
    float* csig = ctop + kBetaElite * n;
    float* ccost = csig + kBetaElite;
    const size_t rb = size_t(b) * kBetaSamples;
    for (int i = tid; i < kBetaElite * n; i += blockDim.x) {
      const int q = i / n, k = i - q * n;
      const size_t src = (rb + elite[q]) * n + k;
      csel[i] = p.bsel[src];
      ctop[i] = p.btop[src];
    }
    if (tid < kBetaElite) {
      csig[tid] = p.bsig[rb + elite[tid]];
      ccost[tid] = cst[elite[tid]];
    }
    __syncthreads();
    for (int i = tid; i < kBetaElite * n; i += blockDim.x) {
      p.bsel[rb * n + i] = csel[i];
      p.btop[rb * n + i] = ctop[i];
    }
    if (tid < kBetaElite) {
      p.bsig[rb + tid] = csig[tid];
      p.bcost[rb + tid] = ccost[tid];
    }
  }
  // ---- per position j: E_new column (the 11 elite sample values: previous
  // elites, this iteration's new samples (ygen) or, at tb = 0, the initial
  // samples), mean, u = (E - mean) / sqrt(10), block sums of u u^T
  const float* Eold = p.belite + (size_t(tb & 1) * p.Bt + b) * kBetaElite * M1;
  float* Enew = p.belite + (size_t((tb + 1) & 1) * p.Bt + b) * kBetaElite * M1;
  const int ys = ygen_stride(M);
  const float* Y = p.ygen + size_t(b) * kBzCols * ys;
  const double rs10 = 1.0 / sqrt(10.0);
  double* gen = p.gen + size_t(b) * pos_pad(M) * kGenStride;
  const int nblk = (M1 + 15) / 16;
  const int span = ((nblk * 16 + 63) / 64) * 64;  // whole waves
  for (int j = tid; j < span; j += blockDim.x) {
    const bool valid = j < M1;
    double u[kBetaElite], mean;
    {
      float v[kBetaElite];
      double s = 0.0;
      const int jc = min(j, M);
      // the 11 loads are unconditional (clamped position, source row chosen
      // by pointer) so they are in flight together
#pragma unroll
      for (int q = 0; q < kBetaElite; ++q) {
        const int e = elite[q];
        const float* src = tb == 0 ? p.beta_z0 + size_t(e) * M1
                                   : (e < kBetaElite ? Eold + size_t(e) * M1 : Y + size_t(e - kBetaElite) * ys);
        v[q] = src[jc];
      }
#pragma unroll
      for (int q = 0; q < kBetaElite; ++q) {
        float x = v[q];
        if (tb == 0) {
          x = float(kSqrt20 * double(x));
          if (j == M) x = fmaxf(x, 0.01f);
        }
        x = valid ? x : 0.0f;
        if (valid) {
          Enew[size_t(q) * M1 + j] = x;
          if (j == M) sig_new[q] = x;
        }
        v[q] = x;
        s = s + double(x);
      }
      const double m = s / double(kBetaElite);
#pragma unroll
      for (int q = 0; q < kBetaElite; ++q) u[q] = valid ? (double(v[q]) - m) * rs10 : 0.0;
      mean = valid ? double(float(m)) : 0.0;
    }
    // level 1: block sums G = U^T U of u u^T over each 16-position block (66
    // packed entries) on fp64 MFMA: the wave's four blocks one at a time, the
    // block's u rows staged in the wave's LDS slice, then 4 x
    // v_mfma_f64_16x16x4 with A = B = U (lane (r, h) of step s: feature r of
    // position 4 s + h; features 11..15 zero)
    double* ub = reinterpret_cast<double*>(smem + C.ublk) + (tid >> 6) * 16 * kUPitch;
    const int lane = tid & 63, r = lane & 15, h = lane >> 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int blk = (j >> 6) * 4 + k;  // wave-uniform
      if ((lane >> 4) == k) {
#pragma unroll
        for (int q = 0; q < kBetaElite; ++q) ub[(lane & 15) * kUPitch + q] = u[q];
        ub[(lane & 15) * kUPitch + kGenMean] = mean;  // the U row's slot 11 (the MFMA below masks it)
      }
      wave_sync();
      d4 G = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const double x = r < 11 ? ub[(4 * st + h) * kUPitch + r] : 0.0;
        G = mfma64(x, x, G);
      }
      // the block's u rows into gen from the same staging: consecutive lanes
      // on consecutive features of a row, so a store instruction covers ~6
      // position rows (a lane per position wrote 64 rows per instruction)
#pragma unroll
      for (int i = 0; i < 3; ++i) {  // whole rows: u_0..u_10 and the mean
        const int e = lane + 64 * i, row = e / kGenRow, q = e - row * kGenRow;
        const int pos = blk * 16 + row;
        if (pos < M1) gen[gen_uplane(pos_pad(M)) + size_t(pos) * kGenRow + q] = ub[row * kUPitch + q];
      }
      wave_sync();
      // register i: G[h + 4 i][r]; the packed upper triangle a <= c
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int a = h + 4 * i;
        if (blk < nblk && a <= r && r < 11) Gb[blk * 66 + sym11(a, r)] = G[i];
      }
    }
  }
  __syncthreads();
  // block prefix: phib[blk] <- Phi at the start of blk = I + sum_{<blk} / d
  if (tid < 66) {
    int a = 0, c = tid;
    while (c >= 11 - a) {
      c -= 11 - a;
      ++a;
    }
    c += a;
    double acc = a == c ? 1.0 : 0.0;
    double* ph = p.phib + size_t(b) * nblk * 66;
#pragma unroll 8
    for (int blk = 0; blk < nblk; ++blk) {  // the LDS reads of several blocks in flight
      const double g = Gb[blk * 66 + tid];
      ph[blk * 66 + tid] = acc;
      acc = fma(g, kInvRidge, acc);
    }
  }
  // last iteration: beta_best / reduced set of argmin (pre-update) and, when
  // argmin is a carried elite, sigma_best (Q4); k_bsigma handles a new sample
  if (tb == kBetaIters - 1) {
    const int* bsel = p.bsel + (size_t(b) * kBetaSamples + imin) * n;
    for (int i = tid; i < n; i += blockDim.x) {
      p.bestsel[size_t(b) * n + i] = bsel[i];
      p.beta[size_t(b) * n + i] = p.btop[(size_t(b) * kBetaSamples + imin) * n + i];
    }
    if (tid == 0) {
      p.bimin[b] = imin;
      if (imin < kBetaElite) p.sigma[b] = sig_new[imin];
    }
  }
}

#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(kThreads) void k_belite(Params p, int tb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  belite_body(p, tb, p.b0 + blockIdx.x, smem);
}
#endif

// k_bgen: level 2 of the generators, one quad (4 lanes) per (candidate,
// block of 16 positions).  The block prefix Phi_b (k_belite) is inverted
// once, A = Phi_b^-1; then, position by position through the block,
//   v_j = A u_j,  L_jj = sqrt(0.05 + u_j . v_j),  w_j = v_j / L_jj,
//   A <- A - w_j w_j^T      (= Phi_{j+1}^-1: Sherman-Morrison, since
//                            Phi_{j+1} = Phi_j + u_j u_j^T / 0.05)
// -- at most 15 rank-1 steps from an exactly inverted start, so the error
// stays at the level of one fp64 inversion.  Lane q of the quad owns rows
// q, q + 4, q + 8 of A (full rows, so A stays symmetric without a packed
// layout); the inverse is an in-place Gauss-Jordan sweep (Phi_b is SPD: no
// pivoting), its pivot rows and the w_j of each step quad broadcasts (DPP),
// so the chain per position is one 11-term dot product deep instead of the
// whole matrix-vector product, and the ~32 blocks x 4 lanes of a candidate
// give ~2 waves per SIMD at B = 1024 (one lane per block gave < 1).
HDI int sym11i(int a, int c) { return a <= c ? sym11(a, c) : sym11(c, a); }

// the generators of 16-position block blk of candidate b on the calling quad
// (lane q = tidx() & 3); live = false: compute, store nothing
DEVI void bgen_quad(const Params& p, int b, int blk, bool live) {
  const int M = p.M, M1 = M + 1, nblk = (M1 + 15) / 16;
  const int q = tidx() & 3;
  double* gen = p.gen + size_t(b) * pos_pad(M) * kGenStride;
  const double* Gb = p.phib + (size_t(b) * nblk + blk) * 66;
  // own rows a = q + 4 i; row 11 (q = 3, i = 2) is padding: an identity row
  // that no other row reads (column 11 does not exist)
  double A[3][11];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int a = q + 4 * i;
#pragma unroll
    for (int c = 0; c < 11; ++c) A[i][c] = a < 11 ? Gb[sym11i(a, c)] : 0.0;
  }
  // in-place Gauss-Jordan inversion
#pragma unroll
  for (int k = 0; k < 11; ++k) {
    const int ik = k >> 2, ok = k & 3;
    const double ip = 1.0 / quad_bcast(A[ik][k], ok);  // the pivot, from its owner lane
    double f[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) f[i] = A[i][k];
    // column by column: entry c of pivot row k (broadcast before its owner
    // overwrites it), scaled, then every own row's update
#pragma unroll
    for (int c = 0; c < 11; ++c) {
      const double rc = c == k ? ip : quad_bcast(A[ik][c], ok) * ip;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const bool pivot_row = q + 4 * i == k;
        A[i][c] = pivot_row ? rc : (c == k ? -f[i] * ip : fma(-f[i], rc, A[i][c]));
      }
    }
  }
  const int j0 = blk * 16, j1 = min(M1, j0 + 16);
  double un[11];  // the quad's four lanes load the same 88 bytes; the next
                  // position's u in flight while one is processed
  double uon[3];  // and the lane's own components u[q + 4 i] (slot 11, the
                  // mean, loaded and masked), so the dot u . v needs no
                  // lane-dependent register selects
  const double* ub = gen + gen_uplane(pos_pad(M));
#pragma unroll
  for (int c = 0; c < 11; ++c) un[c] = ub[size_t(j0) * kGenRow + c];
#pragma unroll
  for (int i = 0; i < 3; ++i) uon[i] = ub[size_t(j0) * kGenRow + q + 4 * i];
  for (int j = j0; j < j1; ++j) {
    double u[11], uo[3];
#pragma unroll
    for (int c = 0; c < 11; ++c) u[c] = un[c];
#pragma unroll
    for (int i = 0; i < 3; ++i) uo[i] = uon[i];
    const int jn = min(j + 1, j1 - 1);
#pragma unroll
    for (int c = 0; c < 11; ++c) un[c] = ub[size_t(jn) * kGenRow + c];
#pragma unroll
    for (int i = 0; i < 3; ++i) uon[i] = ub[size_t(jn) * kGenRow + q + 4 * i];
    double v[3], part = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < 11; ++c) s = fma(A[i][c], u[c], s);
      v[i] = s;
      const int a = q + 4 * i;
      part = fma(i < 2 || a < 11 ? uo[i] : 0.0, s, part);
    }
    const double uv = quad_sum(part);
    const double ljj = sqrt(kRidge + uv);
    const double rl = 1.0 / ljj;
    double w[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = v[i] * rl;
    double* g = gen + size_t(j) * kGenRow;
    if (live) {
#pragma unroll
      for (int i = 0; i < 3; ++i) g[kGenW + q + 4 * i] = q + 4 * i < 11 ? w[i] : 0.0;  // whole rows: slot 11 is 0
      if (q == 0) p.genm[size_t(b) * pos_pad(M) + j] = ljj;
    }
#pragma unroll
    for (int c = 0; c < 11; ++c) {
      const double wc = quad_bcast(w[c >> 2], c & 3);
#pragma unroll
      for (int i = 0; i < 3; ++i) A[i][c] = fma(-w[i], wc, A[i][c]);
    }
  }
}

#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_bgen(Params p) {
  const int nblk = (p.M + 1 + 15) / 16;
  const int gq = (blockIdx.x * blockDim.x + tidx()) >> 2;
  const bool live = gq < p.nb * nblk;  // quads stay whole: dead ones compute on a clamped block, store nothing
  const int gqc = live ? gq : p.nb * nblk - 1;
  bgen_quad(p, p.b0 + gqc / nblk, gqc % nblk, live);
}
#endif

// The generators of block blk of candidate b on one wave (Params::gen_wave:
// small batches, where k_bgen's chain of 11 pivots + 16 positions x (an
// 11-term dot product, sqrt, divide, 11 broadcasts) on one quad is the whole
// latency).  The same quantities in block form:
//   A = Phi_b^-1                    symmetric sweep of Phi_b (11 pivots, a
//                                   lane per matrix entry; -A after the sweep)
//   V = A U,  G = 0.05 I + U^T V    fp64 MFMA (3 + 3 of 16x16x4; U = the
//                                   block's 16 u_j as columns, features 11..
//                                   15 zero)
//   G = L L^T,  W = V L^-T          right-looking Cholesky of the 16 x 16 G,
//                                   V updated alongside (16 pivots)
// -- L_jj and w_j are k_bgen's (G_jj - sum_{i<j} L_ji^2 = 0.05 + u_j . A_j u_j
// with A_j = A - sum_{i<j} w_i w_i^T; w_j = (A u_j - sum_{i<j} w_i L_ji) /
// L_jj = A_j u_j / L_jj), summed in another order (fp64; ~1e-16 apart).
// Every matrix is in the f64 MFMA accumulator layout (lane (r, h), register
// i: row h + 4 i, column r); a pivot step publishes column k through the
// wave's 32 doubles of LDS (xl) and every lane updates its entries.  The
// sweep keeps A exactly symmetric (mirrored entries see the same products),
// so register s of A is also the A operand of step s of A U.
// 1 / d and 1 / sqrt(d) for d > 0: the hardware estimate and two Newton
// steps (a few ulp; the pivots' chain is these few dependent operations, not
// the IEEE divide and square root sequences)
DEVI double rcp_nr(double d) {
  double y = __builtin_amdgcn_rcp(d);
  y = fma(y, fma(-d, y, 1.0), y);
  return fma(y, fma(-d, y, 1.0), y);
}
DEVI double rsq_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double e = fma(-(d * y), y, 1.0);
    y = fma(0.5 * y, e, y);
  }
  return y;
}

// NB blocks blk0, blk0 + bstride, ... of candidate b on the calling wave, their
// pivot chains interleaved (independent: the same bits as one block per
// wave); blocks >= nblk compute on the last block and store nothing.  xl: the
// wave's 32 NB doubles of LDS.
template <int NB>
DEVI void bgen_wave(const Params& p, int b, int blk0, int bstride, double* xl) {
  const int M = p.M, M1 = M + 1, nblk = (M1 + 15) / 16, Pp = pos_pad(M);
  const int lane = tidx() & 63, r = lane & 15, h = lane >> 4;
  double* gen = p.gen + size_t(b) * Pp * kGenStride;
  double* gm = p.genm + size_t(b) * Pp;
  int j0[NB];
  bool live[NB];
  d4 A[NB];
  double U[NB][3];
#pragma unroll
  for (int t = 0; t < NB; ++t) {
    const int blk = blk0 + t * bstride;
    live[t] = blk < nblk;
    const int bc = live[t] ? blk : nblk - 1;
    j0[t] = bc * 16;
    const double* Gb = p.phib + (size_t(b) * nblk + bc) * 66;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a = h + 4 * i;
      A[t][i] = a < 11 && r < 11 ? Gb[sym11i(min(a, 10), min(r, 10))] : 0.0;
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int f = 4 * s + h;  // feature 11 is the mean's slot: zero here
      U[t][s] = f < 11 && j0[t] + r < M1 ? gen[gen_uplane(Pp) + size_t(j0[t] + r) * kGenRow + f] : 0.0;
    }
  }
  // sweep: A_kk <- -1/d, A_ik = A_ki <- A_ik / d, A_ij <- A_ij - A_ik A_kj / d
#pragma unroll
  for (int k = 0; k < 11; ++k) {
    if (r == k) {
#pragma unroll
      for (int t = 0; t < NB; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) xl[32 * t + h + 4 * i] = A[t][i];
    }
    wave_sync();
    double d[NB], cr[NB], ci[NB][4];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      d[t] = xl[32 * t + k];
      cr[t] = xl[32 * t + r];
#pragma unroll
      for (int i = 0; i < 4; ++i) ci[t][i] = xl[32 * t + h + 4 * i];
    }
    wave_sync();
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const double id = rcp_nr(d[t]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int a = h + 4 * i;
        A[t][i] = a == k ? (r == k ? -id : cr[t] * id) : (r == k ? ci[t][i] * id : A[t][i] - (ci[t][i] * cr[t]) * id);
      }
    }
  }
  const d4 zero = d4{0.0, 0.0, 0.0, 0.0};
  d4 V[NB], G[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) A[t][i] = -A[t][i];
    V[t] = zero;
    G[t] = zero;
#pragma unroll
    for (int s = 0; s < 3; ++s) V[t] = mfma64(A[t][s], U[t][s], V[t]);
#pragma unroll
    for (int s = 0; s < 3; ++s) G[t] = mfma64(U[t][s], V[t][s], G[t]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (h + 4 * i == r) G[t][i] = G[t][i] + kRidge;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (r == k) {
#pragma unroll
      for (int t = 0; t < NB; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          xl[32 * t + h + 4 * i] = G[t][i];
          xl[32 * t + 16 + h + 4 * i] = V[t][i];
        }
    }
    wave_sync();
    double d[NB], gr[NB], gi[NB][4], vi[NB][4];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      d[t] = xl[32 * t + k];
      gr[t] = xl[32 * t + r];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gi[t][i] = xl[32 * t + h + 4 * i];
        vi[t][i] = xl[32 * t + 16 + h + 4 * i];
      }
    }
    wave_sync();
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const double rl = rsq_nr(d[t]);
      const double lr = r > k ? gr[t] * rl : 0.0;
      double wk[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double li = h + 4 * i > k ? gi[t][i] * rl : 0.0;
        wk[i] = vi[t][i] * rl;
        G[t][i] = G[t][i] - li * lr;
        V[t][i] = V[t][i] - wk[i] * lr;
      }
      if (live[t] && r == k && j0[t] + k < M1) {
        double* g = gen + size_t(j0[t] + k) * kGenRow + kGenW;
#pragma unroll
        for (int i = 0; i < 3; ++i) g[h + 4 * i] = h + 4 * i < 11 ? wk[i] : 0.0;  // whole rows: slot 11 is 0
        if (h == 0) gm[j0[t] + k] = d[t] * rl;  // L_jj
      }
    }
  }
}

constexpr int kGenWaveWaves = 4;
#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(64 * kGenWaveWaves) void k_bgen_wave(Params p) {
  __shared__ double xl[kGenWaveWaves][32];
  const int nblk = (p.M + 1 + 15) / 16;
  const int w = tidx() >> 6, gw = blockIdx.x * kGenWaveWaves + w;
  if (gw >= p.nb * nblk) return;  // whole waves; no workgroup barrier below
  bgen_wave<1>(p, p.b0 + gw / nblk, gw % nblk, 0, xl[w]);
}
#endif

// k_bsigma (last beta-iteration only): sigma_best when argmin is a new
// sample -- its sigma coordinate drawn with the NEW generators (Q4,
// compute_beta.py:133-145): y_M = mean_M + L_MM z_M + u_M . sum_{j<M} w_j z_j
// the body of k_bsigma for candidate b when its argmin is a new sample;
// red: (kThreads / 64) * 11 doubles of LDS.  The sums are split over
// kThreads threads whatever the workgroup size (the threads beyond add
// nothing), so every caller forms the same bits.
DEVI void bsigma_body(const Params& p, int tb, int b, double* red) {
  const int M = p.M, tid = tidx();
  const int imin = p.bimin[b];
  const double* gen = p.gen + size_t(b) * pos_pad(M) * kGenStride;
  {
    const float* z = p.beta_z + size_t(tb) * pos_pad(M) * kBzCols;
    const int si = imin - kBetaElite;
    double part[11];
#pragma unroll
    for (int a = 0; a < 11; ++a) part[a] = 0.0;
    for (int j = tid; j < M && tid < kThreads; j += kThreads) {
      const double zj = double(z[bz_index(j, si)]);
#pragma unroll
      for (int a = 0; a < 11; ++a) part[a] += gen[size_t(j) * kGenRow + kGenW + a] * zj;
    }
#pragma unroll
    for (int a = 0; a < 11; ++a) {
      part[a] = wave_sum(part[a]);
    }
    __syncthreads();
    if ((tid & 63) == 0 && tid < kThreads)
#pragma unroll
      for (int a = 0; a < 11; ++a) red[(tid >> 6) * 11 + a] = part[a];
    __syncthreads();
    if (tid == 0) {
      const double* g = gen + size_t(M) * kGenRow;
      const double* gu = g + gen_uplane(pos_pad(M));
      double d = 0.0;
      for (int a = 0; a < 11; ++a) {
        double sa = 0.0;
        for (int w2 = 0; w2 < kThreads / 64; ++w2) sa += red[w2 * 11 + a];
        d += gu[a] * sa;
      }
      const double zM = z[bz_index(M, si)];
      const float yM = float((gu[kGenMean] + p.genm[size_t(b) * pos_pad(M) + M] * zM) + d);
      p.sigma[b] = fmaxf(yM, 0.01f);
    }
  }
}

#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(kThreads) void k_bsigma(Params p, int tb) {
  __shared__ double red[(kThreads / 64) * 11];
  const int b = p.b0 + blockIdx.x;
  if (p.bimin[b] < kBetaElite) return;  // k_belite wrote it
  bsigma_body(p, tb, b, red);
}
#endif

// ------------------------------------------------------------------------
// k_mmdfinal: x_red / y_red of the best reduced set (compute_beta.py:465),
// compute_mmd_obs (costs.py:173-186) and compute_mmd_lane (costs.py:121-135).
#ifndef MPCMMD_FUSED_TU
// Two phases: the n reduced rollouts a lane each, their states kept in LDS,
// then the n H O obstacle terms over all 64 lanes, a (row, step) pair per
// lane, the row maxima by LDS atomics on the bit patterns (every compared
// value is >= +0 after the max with the initial 0, where unsigned order is
// float order; a maximum is order-free, so the bits are the sequential
// loop's).  The sequential form held 22 of 64 lanes through H x O f_bar
// evaluations and their obstacle loads (62 us per configs[1] step).
__global__ __launch_bounds__(64) void k_mmdfinal(Params p, int t) {
  __shared__ float cb[kMaxReduced], lb[kMaxReduced], ub[kMaxReduced], bt[kMaxReduced];
  __shared__ uint32_t cbits[kMaxReduced], cnan[kMaxReduced];
  __shared__ ReduceScratch rs;
  extern __shared__ __attribute__((aligned(16))) float xy[];  // [2][n][H] rollout states, then [2][n][H] controls
  const int b = blockIdx.x, n = p.n, H = p.H, O = p.O, lane = tidx();
  const Cfg cf = cfg_of(p, b / p.B);
  // the candidate's noisy controls staged by all lanes (coalesced), so the
  // rollouts' per-step reads are LDS reads, not a global load latency per step
  float* ctrl = xy + 2 * n * H;
  for (int i = lane; i < 2 * n * H; i += 64) ctrl[i] = p.ctrl_n[size_t(b) * 2 * n * H + i];
  __syncthreads();
  if (lane < n) {
    const int m = p.bestsel[size_t(b) * n + lane];
    const float* ar = ctrl + (m / n) * H;
    const float* sr = ctrl + n * H + (m % n) * H;
    float x = cf.st0[0], y = cf.st0[1], vx = cf.st0[2], vy = cf.st0[3], psi = cf.st0[4];
    float l = 0.0f, u = 0.0f;
    bool nan = false;
    for (int h = 0; h < H; ++h) {
      xy[lane * H + h] = x;
      xy[(n + lane) * H + h] = y;
      nan |= (y != y);
      l = fmaxf(l, -y + p.y_lb);
      u = fmaxf(u, y - p.y_ub);
      if (h == H - 1) break;
      bicycle_step(x, y, vx, vy, psi, ar[h], sr[h]);
    }
    const float qnan = __int_as_float(0x7fc00000);
    cbits[lane] = 0u;
    cnan[lane] = nan ? 1u : 0u;
    lb[lane] = nan ? qnan : l;
    ub[lane] = nan ? qnan : u;
    bt[lane] = p.beta[size_t(b) * n + lane];
  }
  __syncthreads();
  for (int e = lane; e < n * H; e += 64) {
    const int k = e / H, h = e - k * H;
    const float x = xy[e], y = xy[n * H + e];
    float c = 0.0f;
    bool nan = false;
    for (int o = 0; o < O; ++o) {
      const float f = f_bar(x, y, cf.obs[o * H + h], cf.obs[O * H + o * H + h]);
      nan |= (f != f);
      c = fmaxf(c, f);
    }
    atomicMax(&cbits[k], __float_as_uint(c + 0.0f));  // -0 -> +0 (fmaxf may keep -0): unsigned order = float order
    if (nan) atomicOr(&cnan[k], 1u);
  }
  __syncthreads();
  if (lane < n) cb[lane] = cnan[lane] ? __int_as_float(0x7fc00000) : __uint_as_float(cbits[lane]);
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
#endif


// ------------------------------------------------------------------------
// k_bcem_small: the 20 beta-iterations of one candidate in one workgroup
// (small batches: the reference's num_batch = 100, BASELINE configs[4]'s
// CARLA solves).  At B = 100 the seven per-iteration kernels above run as
// one latency-bound launch each (10-27 us for a few microseconds of work per
// candidate, 140 launches per outer iteration); here the same phases follow
// each other inside one launch, separated by workgroup barriers, with the
// candidate's intermediates (samples, selections, K_red, generators) in
// global memory that this workgroup alone touches -- L2-resident at this
// size.  Every phase is the body of its multi-kernel counterpart (same
// operations, so the same bits): samples by bsample_unit_lds (a wave per tile
// and chunk), selection by bselect_wave, kernel sums / K_red by bkernel_body, direct row
// sums by bdirect_body, the QPs by bqp_solve (a quad each), elites by
// belite_body, generators by bgen_wave, sigma_best by bsigma_body.
// W = 16 waves (1024 threads, <= 128 VGPRs) for n <= 16, else 8 (the QPs of
// n > 16 need up to 256 VGPRs): small_waves.
HDI size_t small_sel_bytes(int R) { return size_t(64 * R + 8) * 8 + 64 * 4 + 128 * 4; }  // one wave's select LDS
HDI size_t small_lds(int M, int n, int R, int W) {
  size_t b = size_t(W) * small_sel_bytes(R) + size_t(kNew) * ygen_stride(M) * 4;  // + the staged sample rows
  const size_t k = ker_lds(M, n, ker_scratch(M, n, 1, W)).total;
  const size_t d = dir_lds(M, n).total, e = elite_lds(M + 1, W).total;
  const size_t q = (size_t(kBetaSamples) * tri_stride(n) + kQpZeros) * 4;  // the QPs' K_red and zeros
  const size_t g = size_t(W) * 4 * 32 * 8;                        // bgen_wave<4>'s pivot columns
  const size_t gl = ((gen_lds_bytes(M) + 15) & ~size_t(15)) + tblk_lds_bytes(M);  // the sampler's copy + T blocks
  b = b > q ? b : q;
  b = b > g ? b : g;
  b = b > gl ? b : gl;
  b = b > k ? b : k;
  b = b > d ? b : d;
  b = b > e ? b : e;
  return b;
}

// the persistent LDS copies (k_bcem_small's persist): after the phases' space
HDI size_t small_persist_off(int M, int n, int R, int W) { return (small_lds(M, n, R, W) + 15) & ~size_t(15); }
HDI size_t small_persist_bytes(int M) { return size_t(M) * (kMomStride + kFeatStride) * 4; }

// phase stamps of beta-iteration 5 (MPCMMD_STAMPW; rows 32768 + workgroup,
// apart from the kernel-sum body's own stamps): tools/stamp_small.py
#define SMALL_STAMP(p, slot)                                                             \
  do {                                                                                   \
    if (tidx() == 0 && (p).dbgw)                                                    \
      (p).dbgw[size_t(32768 + blockIdx.x) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

#ifdef MPCMMD_FUSED_TU
template <int NQ, int R, int G, int NP, int NV4, int GNB, int W>
__global__ __launch_bounds__(64 * W) void k_bcem_small(Params p0, int persist) {
  constexpr int kSmallWaves = W, kSmallThreads = 64 * W;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cand = blockIdx.x;
  const int tid = tidx();
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // persist: the candidate's series records and feature rows (fixed for the
  // outer iteration) copied once into LDS past the phases' space, for the
  // kernel-sum phase of every beta-iteration
  const float4* mom_l = nullptr;
  const float4* feat_l = nullptr;
  if (persist) {
    const int M = p0.M, b = p0.b0 + cand;
    float4* pm = reinterpret_cast<float4*>(smem + small_persist_off(M, p0.n, R, W));
    float4* pf = pm + M * (kMomStride / 4);
    const float4* gm = reinterpret_cast<const float4*>(p0.bmom + size_t(b) * M * kMomStride);
    const float4* gf = reinterpret_cast<const float4*>(p0.featr + size_t(b) * M * kFeatStride);
    for (int i = tid; i < M * (kMomStride / 4); i += kSmallThreads) pm[i] = gm[i];
    for (int i = tid; i < M * (kFeatStride / 4); i += kSmallThreads) pf[i] = gf[i];
    mom_l = pm;
    feat_l = pf;
    __syncthreads();
  }
  for (int tb = 0; tb < kBetaIters; ++tb) {
    // the launch's Params read through a pointer laundered per iteration: no
    // field (nor anything computed from one) is hoisted out of the loop
    typedef const Params __attribute__((address_space(4)))* KParams;
    KParams pk = (KParams)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(pk));
    const Params& p = *(const Params*)pk;
    const int b = p.b0 + cand, M = p.M, n = p.n;
    const int ntri = tri_stride(n);
    // samples of this iteration (compute_beta.py:51-68); the first ones are
    // the shared initial draws (Q3), taken from the handle's selection table
    if (tb > 0) {
      if (tb == 5) SMALL_STAMP(p, 0);
      {  // the generators into LDS (W and U planes, genm), then the walkers
        const int Pp = pos_pad(M);
        const double2* gsrc = reinterpret_cast<const double2*>(p.gen + size_t(b) * Pp * kGenStride);
        const double2* msrc = reinterpret_cast<const double2*>(p.genm + size_t(b) * Pp);
        double2* dst = reinterpret_cast<double2*>(smem);
        const int ng = Pp * kGenRow, nm = Pp >> 1;  // double2 counts
        for (int i = tid; i < ng + nm; i += kSmallThreads) dst[i] = i < ng ? gsrc[i] : msrc[i - ng];
        if (tid < 8) dst[ng + nm + tid] = double2{0.0, 0.0};
      }
      __syncthreads();
      {
        const double* lg = reinterpret_cast<const double*>(smem);
        double* Tl = reinterpret_cast<double*>(smem + ((gen_lds_bytes(M) + 15) & ~size_t(15)));
        bsample_tblocks(p, lg, Tl, w, kSmallWaves);
        __syncthreads();
        const int nblk = pos_pad(M) >> 4, units = kSampleTiles * ((nblk + sample_chunk(nblk) - 1) / sample_chunk(nblk));
        for (int u = w; u < units; u += kSmallWaves) bsample_unit_lds(p, tb, b, u % kSampleTiles, u / kSampleTiles, lg, Tl);
      }
      __syncthreads();
      if (tb == 5) SMALL_STAMP(p, 1);
      // the new samples' rows into LDS (after the waves' select scratch), so
      // each wave's top-n walk reads its keys at LDS latency: a wave's chain of
      // samples otherwise waits on one L2 round trip per sample.  Then
      // bselect_wave's walk (samples first_sample(tb) = 11 .. 99: the elites'
      // selections were carried) on the staged rows
      const int ys = ygen_stride(M);
      const float* Yl = reinterpret_cast<const float*>(smem + size_t(kSmallWaves) * small_sel_bytes(R));
      {
        const float4* src = reinterpret_cast<const float4*>(p.ygen + size_t(b) * kBzCols * ys);
        float4* dst = reinterpret_cast<float4*>(smem + size_t(kSmallWaves) * small_sel_bytes(R));
        for (int i = tid; i < kNew * (ys >> 2); i += kSmallThreads) dst[i] = src[i];
      }
      __syncthreads();
      char* sw = smem + size_t(w) * small_sel_bytes(R);
      unsigned long long* cand_l = reinterpret_cast<unsigned long long*>(sw);
      uint32_t* lm = reinterpret_cast<uint32_t*>(sw + size_t(64 * R + 8) * 8);
      int* scr = reinterpret_cast<int*>(sw + size_t(64 * R + 8) * 8 + 64 * 4);
      {
        int32_t* sel = p.bsel + size_t(b) * kBetaSamples * n;
        float* sig = p.bsig + size_t(b) * kBetaSamples;
        auto row = [&](int s) {
          const float* r = Yl + size_t(s - kBetaElite) * ys;
          return [=](int j) { return r[j]; };
        };
        const int s_lo = first_sample(tb), lane = tid & 63;
        if (s_lo + w < kBetaSamples) {
          select_walk<NQ, R, G>(row, [&](int s) { return sel + s * n; }, s_lo + w, kBetaSamples, kSmallWaves, M, n,
                                cand_l, lm, scr);
          for (int s2 = s_lo + w + lane * kSmallWaves; lane < 16 && s2 < kBetaSamples; s2 += 16 * kSmallWaves)
            sig[s2] = row(s2)(M);  // tb >= 1: rows are clipped when written
        }
      }
    } else {
      for (int e = tid; e < kBetaSamples * n; e += kSmallThreads) p.bsel[size_t(b) * kBetaSamples * n + e] = p.sel0[e];
      for (int e = tid; e < kBetaSamples; e += kSmallThreads) p.bsig[size_t(b) * kBetaSamples + e] = p.sig0[e];
    }
    __syncthreads();
    if (tb == 5) SMALL_STAMP(p, 2);
    // K_mixed row sums and K_red (compute_beta.py:120-127).  The direct sums
    // by rows (bdirect_body): a candidate's direct pairs share its M rows
    // several times over, and the pair-list form (direct_pairs_wave) measured
    // no faster here (CARLA n = 10: 24.2 vs 24.3 ms per solve)
    bkernel_body<kSmallWaves>(p, tb, cand, 0, 1, int(ker_scratch(M, n, tb, kSmallWaves)), smem, mom_l, feat_l);
    __syncthreads();
    if (tb == 5) SMALL_STAMP(p, 3);
    if (tb > 0) {
      const int total = bdirect_total(p, b, 1);  // block-uniform
      if (total > 0) {
        bdirect_body<NV4, kSmallWaves>(p, tb, 1, 1, cand, 0, total, smem);
        __syncthreads();
      }
    }
    if (tb == 5) SMALL_STAMP(p, 4);
    // the QPs (compute_beta.py:70-91), a quad each, the samples' K_red staged
    // in LDS (one contiguous copy: the candidate's triangles are consecutive)
    {
      const int s_lo = first_sample(tb), per = kBetaSamples - s_lo;
      const float4* src = reinterpret_cast<const float4*>(p.bkred + (size_t(b) * kBetaSamples + s_lo) * ntri);
      float4* kl4 = reinterpret_cast<float4*>(smem);
      for (int i = tid; i < per * (ntri >> 2); i += kSmallThreads) kl4[i] = src[i];
      if (tid < kQpZeros) reinterpret_cast<float*>(smem)[per * ntri + tid] = 0.0f;
      __syncthreads();
      static_assert(kSmallThreads / 4 >= kBetaSamples, "one quad per QP");
      const int g = tid >> 2;
      const bool ok = g < per;
      const int gc = ok ? g : 0;
      bqp_solve<NP>(p, b, s_lo + gc, ok, reinterpret_cast<const float*>(smem) + size_t(gc) * ntri,
                    reinterpret_cast<const float*>(smem) + size_t(per) * ntri);
    }
    __syncthreads();
    if (tb == 5) SMALL_STAMP(p, 5);
    // elites, mean, generator level 1 (compute_beta.py:51-68, 133-157)
    belite_body(p, tb, b, smem);
    __syncthreads();
    if (tb == 5) SMALL_STAMP(p, 6);
    // generator level 2, a wave per 16-position block
    {
      const int nblk = (M + 1 + 15) / 16;
      double* xl = reinterpret_cast<double*>(smem) + 32 * GNB * w;
      for (int blk = w; blk < nblk; blk += kSmallWaves * GNB) bgen_wave<GNB>(p, b, blk, kSmallWaves, xl);
    }
    __syncthreads();
    if (tb == 5) SMALL_STAMP(p, 7);
    if (tb == kBetaIters - 1 && p.bimin[b] >= kBetaElite) {  // block-uniform
      bsigma_body(p, tb, b, reinterpret_cast<double*>(smem));
      __syncthreads();
    }
  }
}
#endif

}  // namespace

#ifndef MPCMMD_FUSED_TU
bool mmdopt_supported(int n, int H, int O, std::string* why) {
  const int M = n * n;
  if (n > kMaxReduced) {
    if (why) *why = "mmd_opt needs num_reduced <= 64";
    return false;
  }
  if (dir_lds(M, n).total > kLdsBudget || ker_lds(M, n, ker_scratch(M, n, 1)).total > kLdsBudget) {
    if (why) *why = "mmd_opt: num_reduced^2 too large for the kernel-sum stage";
    return false;
  }
  const EliteLds e = elite_lds(M + 1);
  if (e.total > kLdsBudget) {
    if (why) *why = "mmd_opt: num_reduced^2 too large for the elite stage";
    return false;
  }
  (void)H;
  (void)O;
  return true;
}

void launch_mother(const Params& p, int t, hipStream_t s) {
  const size_t lds = ((size_t(3) * p.n * p.H * 4 + 15) & ~size_t(15)) + size_t(11) * p.H * 8;  // controls, fit rows
  if (p.carla)
    hipLaunchKernelGGL(k_mother<true>, dim3(p.Bt), dim3(kThreads), lds, s, p, t);
  else
    hipLaunchKernelGGL(k_mother<false>, dim3(p.Bt), dim3(kThreads), lds, s, p, t);
}

// the pad columns M..Md-1 of every distance row, +inf (exp(-inf) = 0 in the
// row sums): once per handle, k_bdist writes the real columns only
#ifndef MPCMMD_FUSED_TU
__global__ __launch_bounds__(256) void k_dist_pad(Params p, int cap) {
  const int M = p.M, Md = dist_stride(M), np = Md - M;
  const size_t total = size_t(cap) * M * np;
  for (size_t x = size_t(blockIdx.x) * 256 + tidx(); x < total; x += size_t(gridDim.x) * 256) {
    const size_t row = x / np;
    p.bdist[row * Md + M + (x - row * np)] = __builtin_inff();
  }
}
#endif

void launch_dist_pad(const Params& p, int cap, hipStream_t s) {
  if (dist_stride(p.M) == p.M) return;
  hipLaunchKernelGGL(k_dist_pad, dim3(2048), dim3(256), 0, s, p, cap);
}

void launch_bdist(const Params& p, hipStream_t s) {
  const int T = (p.M + kDistRows - 1) / kDistRows, groups = (p.Bt + kXcds - 1) / kXcds;
  hipLaunchKernelGGL(k_bdist, dim3(groups * T * kXcds), dim3(kDistThreads), 0, s, p);
}

template <int NV4>
void launch_bmoment_v(const Params& p, hipStream_t s) {
  const size_t rows = size_t(p.Bt) * p.M, per = size_t(kMomRowsPerBlock) * mom_rows_per_wave<NV4>();
  hipLaunchKernelGGL((k_bmoment<NV4>), dim3((rows + per - 1) / per),
                     dim3(64 * kMomRowsPerBlock), 0, s, p);
}

template <int NV>
void launch_bmoment_rows(const Params& p, hipStream_t s) {
  const size_t rows = size_t(p.Bt) * p.M, per = size_t(kMomRowWaves) * 4;
  hipLaunchKernelGGL((k_bmoment_rows<NV>), dim3((rows + per - 1) / per), dim3(64 * kMomRowWaves), 0, s, p);
}

void launch_bmoment(const Params& p, hipStream_t s) {
  if (p.mom_rows) {
    switch (dist_stride(p.M) >> 8) {  // 16 lanes x NV float4s = one row of dist_stride(M) columns
      case 1:
        return launch_bmoment_rows<4>(p, s);
      case 2:
        return launch_bmoment_rows<8>(p, s);
      case 3:
        return launch_bmoment_rows<12>(p, s);
      case 4:
        return launch_bmoment_rows<16>(p, s);
      default:
        break;
    }
  }
  switch (dist_stride(p.M) >> 8) {
#define MPCMMD_MOM_CASE(V) \
  case V:                  \
    return launch_bmoment_v<V>(p, s);
    MPCMMD_MOM_CASE(1) MPCMMD_MOM_CASE(2) MPCMMD_MOM_CASE(3) MPCMMD_MOM_CASE(4)
    MPCMMD_MOM_CASE(5) MPCMMD_MOM_CASE(6) MPCMMD_MOM_CASE(7) MPCMMD_MOM_CASE(8)
    MPCMMD_MOM_CASE(9) MPCMMD_MOM_CASE(10) MPCMMD_MOM_CASE(11) MPCMMD_MOM_CASE(12)
    MPCMMD_MOM_CASE(13) MPCMMD_MOM_CASE(14) MPCMMD_MOM_CASE(15)
    default:
      return launch_bmoment_v<16>(p, s);
#undef MPCMMD_MOM_CASE
  }
}

void launch_bsample(const Params& p, int tb, hipStream_t s) {
  // one wave per candidate when the launch alone holds >= ~half a wave per
  // SIMD; smaller batches one wave per (candidate, tile, chunk)
  if (p.nb >= 384) {
    hipLaunchKernelGGL((k_bsample<6>), dim3(p.nb), dim3(64 * sample_waves<6>()), 0, s, p, tb);
  } else {
    const int nblk = pos_pad(p.M) >> 4, cl = sample_chunk(nblk);
    hipLaunchKernelGGL(k_bsample_chunks, dim3(p.nb, kSampleTiles), dim3(64 * ((nblk + cl - 1) / cl)), 0, s, p, tb);
  }
}

// waves per candidate: ~16 single-wave workgroups per SIMD over the launch,
// at most 16 per candidate (B = 1024: 8 -> 16 measured -8.5%; the 512-candidate
// groups of the two-stream split: 25 -> 16 +1%)
void launch_bsel0(const Params& p, hipStream_t s) {
  const size_t total = size_t(p.nb) * (kBetaSamples * p.n + kBetaSamples);
  hipLaunchKernelGGL(k_bsel0, dim3(unsigned(std::min<size_t>((total + 255) / 256, 4096))), dim3(256), 0, s, p);
}

// (small launches, nb <= 128: up to Params::sel_cap waves per candidate --
// CARLA n = 22, B = 100: 16 -> 64 took 1.5 ms off a 49.5 ms solve)
int sel_waves(int nb, int cap) { return std::max(4, std::min(nb <= 128 ? cap : 16, 16384 / std::max(1, nb))); }

template <int NQ>
void launch_bselect_q(const Params& p, int tb, hipStream_t s) {
  const dim3 grid(p.nb, sel_waves(p.nb, p.sel_cap));
  if (p.n <= 24)
    hipLaunchKernelGGL((k_bselect<NQ, 1, 32>), grid, dim3(64), 0, s, p, tb);
  else if (p.n <= 48)
    hipLaunchKernelGGL((k_bselect<NQ, 2, 64>), grid, dim3(64), 0, s, p, tb);
  else
    hipLaunchKernelGGL((k_bselect<NQ, 2, 0>), grid, dim3(64), 0, s, p, tb);
}

void launch_bselect(const Params& p, int tb, hipStream_t s) {
  const int nq = (p.M + 63) >> 6;
  switch (nq) {
#define MPCMMD_SEL_CASE(q) \
  case q:                  \
    return launch_bselect_q<q>(p, tb, s);
    MPCMMD_SEL_CASE(1)
    MPCMMD_SEL_CASE(2)
    MPCMMD_SEL_CASE(4)
    MPCMMD_SEL_CASE(8)
    MPCMMD_SEL_CASE(16)
#undef MPCMMD_SEL_CASE
    default:
      break;
  }
  if (nq <= 4) return launch_bselect_q<4>(p, tb, s);
  if (nq <= 8) return launch_bselect_q<8>(p, tb, s);
  if (nq <= 12) return launch_bselect_q<12>(p, tb, s);
  if (nq <= 16) return launch_bselect_q<16>(p, tb, s);
  if (nq <= 24) return launch_bselect_q<24>(p, tb, s);
  if (nq <= 32) return launch_bselect_q<32>(p, tb, s);
  if (nq <= 40) return launch_bselect_q<40>(p, tb, s);
  if (nq <= 48) return launch_bselect_q<48>(p, tb, s);
  return launch_bselect_q<64>(p, tb, s);
}

template <int NP>
void launch_bqp_quad(const Params& p, int tb, int qps, hipStream_t s) {
  // threads per workgroup: qp_threads, or 64 (16 QPs) where the launch
  // would give the CUs barely one workgroup each (Params::qp_small)
  const int T = p.qp_small && (qps + 31) / 32 < 2 * kCUs ? 64 : qp_threads(NP);
  const size_t lds = (size_t(T / 4) * tri_stride(p.n) + kQpZeros) * 4;
  hipLaunchKernelGGL((k_bqp<NP>), dim3((qps * 4 + T - 1) / T), dim3(T), lds, s, p, tb);
}

void launch_bqp(const Params& p, int tb, hipStream_t s) {
  const int qps = p.nb * (kBetaSamples - first_sample(tb));
  const dim3 grid_wave((qps + 3) / 4);
  switch (qp_np(p.n)) {
    case 8:
      return launch_bqp_quad<8>(p, tb, qps, s);
    case 12:
      return launch_bqp_quad<12>(p, tb, qps, s);
    case 16:
      return launch_bqp_quad<16>(p, tb, qps, s);
    case 24:
      return launch_bqp_quad<24>(p, tb, qps, s);
    case 32:
      return launch_bqp_quad<32>(p, tb, qps, s);
    case 48:
      hipLaunchKernelGGL((k_bqp_wave<48>), grid_wave, dim3(256), 0, s, p, tb);
      return;
    default:
      hipLaunchKernelGGL((k_bqp_wave<64>), grid_wave, dim3(256), 0, s, p, tb);
      return;
  }
}

// parts per candidate: enough workgroups to fill the chip
int ker_split(int nb, int target) {
  int split = 1;
  while (split < kMaxSplit && nb * split < target) split <<= 1;
  return split;
}

// k_bdirect_pairs (and k_bkernel's pair list) for launches of <= 256
// candidates: at B = 100 the row-sorted k_bdirect's per-candidate setup
// dominates; at B = 1024 (few direct pairs) the list's atomics cost k_bkernel
// more than they save (mmd_opt 133 -> 129 steps/s), so k_bdirect stays there
bool use_pairs(const Params& p) { return p.dir_pairs && p.nb <= 256; }

void launch_bkernel(const Params& p, int tb, hipStream_t s) {
  const size_t sc = ker_scratch(p.M, p.n, tb);
  const dim3 grid(p.nb * ker_split(p.nb, p.ker_target)), block(64 * kKerWaves);
  const size_t lds = ker_lds(p.M, p.n, sc).total;
  if (use_pairs(p))
    hipLaunchKernelGGL(k_bkernel<true>, grid, block, lds, s, p, tb, ker_split(p.nb, p.ker_target), int(sc));
  else
    hipLaunchKernelGGL(k_bkernel<false>, grid, block, lds, s, p, tb, ker_split(p.nb, p.ker_target), int(sc));
}

template <int NV4>
void launch_bdirect_v(const Params& p, int tb, int split, hipStream_t s) {
  if (p.dir_waves >= 16)
    hipLaunchKernelGGL((k_bdirect<NV4, 16>), dim3(p.nb * split), dim3(64 * 16), dir_lds(p.M, p.n).total, s, p, tb,
                       ker_split(p.nb, p.ker_target), split, 1);
  else if (p.dir_waves >= 8)
    hipLaunchKernelGGL((k_bdirect<NV4, 8>), dim3(p.nb * split), dim3(64 * 8), dir_lds(p.M, p.n).total, s, p, tb,
                       ker_split(p.nb, p.ker_target), split, 1);
  else
    hipLaunchKernelGGL((k_bdirect<NV4, kDirWaves>), dim3(p.nb * split), dim3(64 * kDirWaves), dir_lds(p.M, p.n).total,
                       s, p, tb, ker_split(p.nb, p.ker_target), split, 1);
}

template <int NV4>
void launch_bdirect_pairs_v(const Params& p, int tb, hipStream_t s) {
  constexpr int PJ = direct_pj(NV4);
  const int parts = std::max(1, std::min(64, (p.dir_target + p.nb - 1) / p.nb));
  const int grid = (p.nb * parts + 7) & ~7;
  hipLaunchKernelGGL((k_bdirect_pairs<NV4, PJ>), dim3(grid), dim3(64 * kDirWaves), 0, s, p, tb, parts);
}

void launch_bdirect(const Params& p, int tb, hipStream_t s) {
  if (use_pairs(p)) {
    switch (dist_stride(p.M) >> 8) {
#define MPCMMD_PAIR_CASE(V) \
  case V:                   \
    return launch_bdirect_pairs_v<V>(p, tb, s);
      MPCMMD_PAIR_CASE(1) MPCMMD_PAIR_CASE(2) MPCMMD_PAIR_CASE(3) MPCMMD_PAIR_CASE(4)
      MPCMMD_PAIR_CASE(5) MPCMMD_PAIR_CASE(6) MPCMMD_PAIR_CASE(7) MPCMMD_PAIR_CASE(8)
      MPCMMD_PAIR_CASE(9) MPCMMD_PAIR_CASE(10) MPCMMD_PAIR_CASE(11) MPCMMD_PAIR_CASE(12)
      MPCMMD_PAIR_CASE(13) MPCMMD_PAIR_CASE(14) MPCMMD_PAIR_CASE(15)
      default:
        return launch_bdirect_pairs_v<16>(p, tb, s);
#undef MPCMMD_PAIR_CASE
    }
  }
  const int split = ker_split(p.nb, p.dir_target);
  switch (dist_stride(p.M) >> 8) {
#define MPCMMD_KER_CASE(V) \
  case V:                  \
    return launch_bdirect_v<V>(p, tb, split, s);
    MPCMMD_KER_CASE(1) MPCMMD_KER_CASE(2) MPCMMD_KER_CASE(3) MPCMMD_KER_CASE(4)
    MPCMMD_KER_CASE(5) MPCMMD_KER_CASE(6) MPCMMD_KER_CASE(7) MPCMMD_KER_CASE(8)
    MPCMMD_KER_CASE(9) MPCMMD_KER_CASE(10) MPCMMD_KER_CASE(11) MPCMMD_KER_CASE(12)
    MPCMMD_KER_CASE(13) MPCMMD_KER_CASE(14) MPCMMD_KER_CASE(15)
    default:
      return launch_bdirect_v<16>(p, tb, split, s);
#undef MPCMMD_KER_CASE
  }
}

void launch_belite(const Params& p, int tb, hipStream_t s) {
  const EliteLds e = elite_lds(p.M + 1);
  hipLaunchKernelGGL(k_belite, dim3(p.nb), dim3(kThreads), e.total, s, p, tb);
}

void launch_bgen(const Params& p, int tb, hipStream_t s) {
  const int nblk = (p.M + 1 + 15) / 16;
  if (p.gen_wave)
    hipLaunchKernelGGL(k_bgen_wave, dim3((p.nb * nblk + kGenWaveWaves - 1) / kGenWaveWaves), dim3(64 * kGenWaveWaves), 0,
                       s, p);
  else
    hipLaunchKernelGGL(k_bgen, dim3((p.nb * nblk * 4 + 255) / 256), dim3(256), 0, s, p);
  if (tb == kBetaIters - 1) hipLaunchKernelGGL(k_bsigma, dim3(p.nb), dim3(kThreads), 0, s, p, tb);
}

// (k_bcem_small's generators are bgen_wave's: handles with gen_wave only)
void launch_mmdfinal(const Params& p, int t, hipStream_t s) {
  hipLaunchKernelGGL(k_mmdfinal, dim3(p.Bt), dim3(64), size_t(4) * p.n * p.H * 4, s, p, t);
}

#else
// waves per workgroup: 16 while every phase fits 128 VGPRs (the QPs of n <=
// 16, NP <= 16), else 8 (256 VGPRs)
#ifndef MPCMMD_SMALL_W512
#define MPCMMD_SMALL_W512 8  // waves at 256 < M <= 512 (experiment builds: -DMPCMMD_SMALL_W512=16)
#endif
HDI int small_waves(int M) { return M <= 256 ? 16 : (M <= 512 ? MPCMMD_SMALL_W512 : 8); }

// M <= 256 (n <= 16): at n = 22 the per-iteration kernels, which spread each
// phase over the whole chip, measured faster (CARLA n = 22: 63.0 vs 70.9 ms
// per tick); the M > 256 instantiations stay for MPCMMD_FUSED experiments
bool bcem_small_ok(const Params& p) {
  return p.gen_wave && p.M <= 256 && p.nb <= 512 && small_lds(p.M, p.n, 1, small_waves(p.M)) <= kLdsBudget;
}

void launch_bcem_small(const Params& p, hipStream_t s) {
  const int n = p.n, M = p.M, W = small_waves(M);
  const dim3 grid(p.nb), block(64 * W);
  const size_t lp = small_persist_off(M, n, 1, W) + small_persist_bytes(M);
  const int persist = lp <= kLdsBudget;  // the records and features stay in LDS when they fit
  const size_t lds = persist ? lp : small_lds(M, n, 1, W);
  if (M <= 64)
    hipLaunchKernelGGL((k_bcem_small<1, 1, 32, 8, 1, 1, 16>), grid, block, lds, s, p, persist);
  else if (M <= 128)
    hipLaunchKernelGGL((k_bcem_small<2, 1, 32, 12, 1, 1, 16>), grid, block, lds, s, p, persist);
  else if (M <= 256)
    hipLaunchKernelGGL((k_bcem_small<4, 1, 32, 16, 1, 1, 16>), grid, block, lds, s, p, persist);
  else if (M <= 512)
    hipLaunchKernelGGL((k_bcem_small<8, 1, 32, 24, 2, 16 / MPCMMD_SMALL_W512, MPCMMD_SMALL_W512>), grid, block, lds, s,
                       p, persist);
  else
    hipLaunchKernelGGL((k_bcem_small<12, 1, 32, 24, 3, 2, 8>), grid, block, lds, s, p, persist);
}

#endif

}  // namespace mpcmmd
