// Stage "select": everything after the per-candidate risk, on one workgroup
// (the batch-global argsorts make this a single-CU step):
//
//   argsort(res_norm) (full permutation, ellite_num_projection = B, Q6)  cem.py:233-248
//   argsort(obs cost) over the permuted batch, top 20                   cem.py:264-289
//   compute_cost of the 20 elites (norms from k_front, cost.hpp)        cem_helper.py:232-262
//   compute_ellite_samples (top 5)                                      cem_helper.py:264-271
//   compute_shifted_samples (mean/cov EMA, 8x8 Cholesky, B-5 draws)     cem_helper.py:280-314
//   per-iteration result = elite 0 of the obstacle sort (Q1)            cem.py:308-315
//
// Plus stage "noise": the internal Philox draws of one outer iteration.
#include "block.hpp"
#include "cost.hpp"
#include "draws.hpp"
#include "kernels.hpp"
#include "rng.hpp"
#include "sort.hpp"

namespace mpcmmd {

namespace {

// Intra-wave LDS hand-off: one wave's LDS operations execute in order, so
// only the compiler must be kept from reordering them.
DEVI void wave_sync_lds() {
  __builtin_amdgcn_wave_barrier();
  __asm__ volatile("" ::: "memory");
}

constexpr int kMaxSortN = 4096;
constexpr int kN = 100;

// The stable argsort of configuration cf's projection residuals
// (cem.py:233-248) into perm (LDS) and cf.tr_proj[t]: the words
// (sort key << 32 | index) are distinct and their unsigned order is the
// stable order.  Up to blockDim.x candidates one word per thread
// (merge_sort_reg: wave bitonic + pairwise merges), beyond that the LDS
// bitonic network.
DEVI void sort_residuals(const Params& p, const Cfg& cf, int g0, int B, int t, unsigned long long* keys, int* perm) {
  int N = 1;
  while (N < B) N <<= 1;
  const int i = threadIdx.x;
  if (N <= int(blockDim.x)) {
    unsigned long long a = i < B ? ((unsigned long long)sort_key(p.res_norm[g0 + i]) << 32) | unsigned(i) : ~0ull;
    int idx;
    a = merge_sort_reg(a, idx, N, keys);
    if (i < B) {
      const int v = int(a & 0xFFFFFFFFu);
      perm[idx] = v;
      cf.tr_proj[size_t(t) * B + idx] = v;
    }
    return;
  }
  for (int j = i; j < N; j += blockDim.x)
    keys[j] = j < B ? ((unsigned long long)sort_key(p.res_norm[g0 + j]) << 32) | unsigned(j) : ~0ull;
  bitonic_sort(keys, N);
  for (int j = i; j < B; j += blockDim.x) {
    const int v = int(keys[j] & 0xFFFFFFFFu);
    perm[j] = v;
    cf.tr_proj[size_t(t) * B + j] = v;
  }
}

// Workgroups G.. (when kind != 0) draw iteration ahead_t's noise / gamma
// table items (draws.hpp) meanwhile.
__global__ __launch_bounds__(1024) void k_select(Params p, int t, int ahead_t, int kind) {
  __shared__ __attribute__((aligned(16))) unsigned long long keys[kMaxSortN];
  __shared__ int perm[kMaxSortN];
  __shared__ float ocost[1024];
  __shared__ int el[kEliteCost];
  __shared__ float cost20[kEliteCost];
  __shared__ int cem5[kElite];
  __shared__ float pe[kElite][8];
  __shared__ float pe20[kEliteCost][8];
  __shared__ double L[8][8];
  __shared__ double cvs[8][8];
  __shared__ float mean32[8];
  __shared__ int imin_s;
  if (int(blockIdx.x) >= p.G) {  // whole workgroups: no barrier below is reached
    ahead_item(p, ahead_t, kind, (int(blockIdx.x) - p.G) * 1024 + int(threadIdx.x));
    return;
  }
  const int B = p.B;
  const Cfg cf = cfg_of(p, blockIdx.x);  // one workgroup per configuration
  const int g0 = blockIdx.x * B;          // its first candidate
  int N = 1;
  while (N < B) N <<= 1;
  const int tid = threadIdx.x;
  const bool window = B <= int(blockDim.x) && B >= kEliteCost;

  MPCMMD_STAMP(p, 32);
  // ---- argsort(res_norm), stable ------------------------------------------
  const float oc = window && tid < B ? p.obs_cost[g0 + tid] : 0.0f;  // in flight during the sort
  if (p.select_prep) {  // sorted by the risk launch (cost.hpp: select_prep)
    for (int i = tid; i < B; i += blockDim.x) perm[i] = cf.tr_proj[size_t(t) * B + i];
  } else {
    sort_residuals(p, cf, g0, B, t, keys, perm);
  }
  if (window && tid < B) ocost[tid] = oc;
  __syncthreads();
  MPCMMD_STAMP(p, 33);
  // the mean / covariance entries of the update, loaded during the selection
  const float cov0 = tid < 64 ? cf.cov[tid] : 0.0f, mean0 = tid < 8 ? cf.mean[tid] : 0.0f;
  // ---- argsort(obs cost) over the permuted batch -------------------------
  if (window) {  // only the 20 smallest words are needed: a window selection
    __shared__ int wcnt;
    __shared__ unsigned long long wt0;
    const unsigned long long wv =
        tid < B ? ((unsigned long long)sort_key(ocost[perm[tid]]) << 32) | unsigned(tid) : ~0ull;
    block_smallest(wv, B, kEliteCost, keys, keys + 1024, wcnt, wt0, [&](int r, unsigned long long k) {
      const int e = perm[int(k & 0xFFFFFFFFu)];
      el[r] = e;  // candidate index within the configuration
      cf.tr_obs[size_t(t) * kEliteCost + r] = e;
    });
  } else {
    for (int i = tid; i < N; i += blockDim.x)
      keys[i] = i < B ? ((unsigned long long)sort_key(p.obs_cost[g0 + perm[i]]) << 32) | unsigned(i) : ~0ull;
    if (N <= int(blockDim.x)) bitonic_sort_reg(keys, N);
    else bitonic_sort(keys, N);
    if (tid < kEliteCost) {
      const int e = perm[int(keys[tid] & 0xFFFFFFFFu)];
      el[tid] = e;  // candidate index within the configuration
      cf.tr_obs[size_t(t) * kEliteCost + tid] = e;
    }
    __syncthreads();
  }
  MPCMMD_STAMP(p, 34);
  // ---- compute_cost of the 20 elites, from k_front's norms (Params::cnorm)
  if (tid < kEliteCost) {
    const int e = g0 + el[tid];
    double nk[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) nk[k] = p.cnorm[size_t(e) * kCnormStride + k];
    cost20[tid] = cost_total(p, e, nk);
  }
  const float* pop = p.pop + (size_t(t & 1) * p.Bt + g0) * 8;
  float* pop_next = p.pop + (size_t((t + 1) & 1) * p.Bt + g0) * 8;
  if (tid >= 64 && tid < 64 + kEliteCost * 8) {  // the 20 elites' rows: the top 5 are among them
    const int q = (tid - 64) >> 3, c = tid & 7;
    pe20[q][c] = pop[size_t(el[q]) * 8 + c];
  }
  __syncthreads();
  MPCMMD_STAMP(p, 35);
  // ---- top 5 by cost (stable) -------------------------------------------
  if (tid < kEliteCost) {
    const uint32_t kj = sort_key(cost20[tid]);
    int r = 0;
    for (int k = 0; k < kEliteCost; ++k) {
      const uint32_t kk = sort_key(cost20[k]);
      r += (kk < kj) || (kk == kj && k < tid);
    }
    if (r < kElite) cem5[r] = tid;
  }
  __syncthreads();
  if (tid < kElite * 8) {
    const int q = tid >> 3, c = tid & 7;
    pe[q][c] = pe20[cem5[q]][c];
  }
  __syncthreads();
  // ---- compute_shifted_samples (fp64): weights per thread, mean entry c on
  // thread c, covariance entry (a, c) on thread 8 a + c (each sum in the
  // reference's order), the 8x8 Cholesky on thread 0
  if (tid < 64) {
    double c5[kElite], wgt[kElite];
    for (int q = 0; q < kElite; ++q) c5[q] = double(cost20[cem5[q]]);
    double cmin = c5[0];
    for (int q = 1; q < kElite; ++q) cmin = c5[q] < cmin ? c5[q] : cmin;
    double sw = 0.0;
    for (int q = 0; q < kElite; ++q) {
      wgt[q] = exp(-(1.0 / 0.9) * (c5[q] - cmin));
      sw += wgt[q];
    }
    if (tid < 8) {
      const int c = tid;
      double s = 0.0;
      for (int q = 0; q < kElite; ++q) s += wgt[q] * double(pe[q][c]);
      mean32[c] = float((1.0 - 0.6) * double(mean0) + 0.6 * s / sw);  // mean0 = cf.mean[c]
    }
    wave_sync_lds();
    const int a = tid >> 3, c = tid & 7;
    const double ma = double(mean32[a]), mc = double(mean32[c]);
    double s = 0.0;
    for (int q = 0; q < kElite; ++q) s += wgt[q] * (double(pe[q][a]) - ma) * (double(pe[q][c]) - mc);
    const float v = float((1.0 - 0.6) * double(cov0) + 0.6 * s / sw + (a == c ? 0.01 : 0.0));  // cov0 = cf.cov[tid]
    cvs[a][c] = double(v);
    cf.cov[a * 8 + c] = v;
    if (tid < 8) cf.mean[tid] = mean32[tid];
    wave_sync_lds();
  }
  if (tid < 64) {
    // Cholesky (lower) of the fp32 covariance, in fp64: lane i < 8 holds row
    // i in registers; column j's pivot from lane j's row, broadcast by
    // readlane with row j's earlier entries, then the entries below on lanes
    // i > j (each entry's sum in the serial algorithm's order, so the same
    // bits); no LDS round trips between the columns
    const int i = tid & 7;
    double c[8], Lr[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      c[k] = cvs[i][k];
      Lr[k] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      double Ljk[8];
#pragma unroll
      for (int k = 0; k < j; ++k) Ljk[k] = readlane_d(Lr[k], j);
      double d = c[j];
#pragma unroll
      for (int k = 0; k < j; ++k) d -= Lr[k] * Lr[k];
      const double piv = readlane_d(sqrt(d), j);
      if (i == j) Lr[j] = piv;
      if (i > j) {
        double sm = c[j];
#pragma unroll
        for (int k = 0; k < j; ++k) sm -= Lr[k] * Ljk[k];
        Lr[j] = sm / piv;
      }
    }
    if (tid < 8)
#pragma unroll
      for (int k = 0; k < 8; ++k) L[tid][k] = Lr[k];
  }
  if (tid == 0) {
    // idx_min = argmin(cost_batch_temp) (== 0 unless NaN; jnp.argmin: first NaN)
    int im = 0;
    for (int q = 0; q < kElite; ++q) {
      const float cq = cost20[cem5[q]];
      if (cq != cq) {
        im = q;
        break;
      }
    }
    imin_s = im;
    for (int q = 0; q < kElite; ++q) cf.tr_cem[size_t(t) * kElite + q] = cem5[q];
  }
  __syncthreads();
  MPCMMD_STAMP(p, 36);
  // ---- new population: [elites; mean + L z], v columns clipped -----------
  const float* z = cf.resample + size_t(t) * (B - kElite) * 8;
  for (int i = tid; i < B; i += blockDim.x) {
    float row[8];
    if (i < kElite) {
      for (int c = 0; c < 8; ++c) row[c] = pe[i][c];
    } else {
      const float* zi = z + size_t(i - kElite) * 8;
      for (int a = 0; a < 8; ++a) {
        double s = double(mean32[a]);
        for (int c = 0; c <= a; ++c) s += L[a][c] * double(zi[c]);
        row[a] = float(s);
      }
      for (int c = 0; c < 4; ++c) row[c] = fminf(fmaxf(row[c], 0.1f), 30.0f);
    }
    for (int c = 0; c < 8; ++c) pop_next[size_t(i) * 8 + c] = row[c];
  }
  MPCMMD_STAMP(p, 37);
  // ---- per-iteration result (cem.py:314-315) ------------------------------
  if (p.carla && tid < kN)  // steering of the chosen elite (carla/optimizer/cem.py:398-399, 419)
    p.res_steer[(size_t(cf.g) * p.T + t) * kN + tid] = p.steer[size_t(g0 + el[imin_s]) * kN + tid];
  if (tid < kResultStride) {
    const int e = g0 + el[imin_s];
    float* r = cf.results + size_t(t) * kResultStride;
    float v = 0.0f;
    if (tid < 11) v = p.cx[size_t(e) * 11 + tid];
    else if (tid < 22) v = p.cy[size_t(e) * 11 + tid - 11];
    else if (tid == 22) v = p.lane_cost[e];
    else if (tid == 23) v = p.obs_cost[e];
    else if (tid == 24) v = p.cost == 0 ? p.sigma[e] : 0.0f;
    else if (tid < 45) v = p.cost == 0 ? p.res_beta[size_t(e) * kBetaIters + tid - 25] : 0.0f;
    else if (tid - 45 < p.n) v = p.cost == 0 ? p.beta[size_t(e) * p.n + tid - 45] : 0.0f;
    r[tid] = v;
  }
}

// internal draws of outer iteration t: roll [3][H][S] and resample [B-5][8]
__global__ __launch_bounds__(256) void k_noise(Params p, int t) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < noise_items(p)) noise_item(p, t, cfg_of(p, blockIdx.y), j);  // configuration blockIdx.y
}

}  // namespace

void launch_select(const Params& p, int t, hipStream_t s, int ahead_t, int kind) {
  const int extra = ahead_t >= 0 && kind ? (p.G * ahead_items(p, kind) + 1023) / 1024 : 0;
  hipLaunchKernelGGL(k_select, dim3(p.G + extra), dim3(1024), 0, s, p, t, ahead_t, extra ? kind : 0);
}

void launch_noise(const Params& p, int t, hipStream_t s) {
  const int total = noise_items(p);
  hipLaunchKernelGGL(k_noise, dim3((total + 255) / 256, p.G), dim3(256), 0, s, p, t);
}

}  // namespace mpcmmd
