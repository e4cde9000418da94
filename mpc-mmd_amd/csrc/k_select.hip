// Stage "select": everything after the per-candidate risk, on one workgroup
// (the batch-global argsorts make this a single-CU step):
//
//   argsort(res_norm) (full permutation, ellite_num_projection = B, Q6)  cem.py:233-248
//   argsort(obs cost) over the permuted batch, top 20                   cem.py:264-289
//   compute_cost of the 20 elites                                       cem_helper.py:232-262
//   compute_ellite_samples (top 5)                                      cem_helper.py:264-271
//   compute_shifted_samples (mean/cov EMA, 8x8 Cholesky, B-5 draws)     cem_helper.py:280-314
//   per-iteration result = elite 0 of the obstacle sort (Q1)            cem.py:308-315
//
// Plus stage "noise": the internal Philox draws of one outer iteration.
#include "block.hpp"
#include "draws.hpp"
#include "kernels.hpp"
#include "rng.hpp"

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

// Workgroups G.. (when kind != 0) draw iteration ahead_t's noise / gamma
// table items (draws.hpp) meanwhile.
__global__ __launch_bounds__(1024) void k_select(Params p, int t, int ahead_t, int kind) {
  __shared__ __attribute__((aligned(16))) unsigned long long keys[kMaxSortN];
  __shared__ int perm[kMaxSortN];
  __shared__ int el[kEliteCost];
  __shared__ float cost20[kEliteCost];
  __shared__ int cem5[kElite];
  __shared__ float pe[kElite][8];
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

  MPCMMD_STAMP(p, 32);
  // ---- argsort(res_norm), stable ------------------------------------------
  for (int i = tid; i < N; i += blockDim.x)
    keys[i] = i < B ? ((unsigned long long)sort_key(p.res_norm[g0 + i]) << 32) | unsigned(i) : ~0ull;
  if (N <= int(blockDim.x)) bitonic_sort_reg(keys, N);
  else bitonic_sort(keys, N);
  for (int i = tid; i < B; i += blockDim.x) {
    perm[i] = int(keys[i] & 0xFFFFFFFFu);
    cf.tr_proj[size_t(t) * B + i] = perm[i];
  }
  __syncthreads();
  MPCMMD_STAMP(p, 33);
  // ---- argsort(obs cost) over the permuted batch -------------------------
  if (B <= int(blockDim.x) && B >= kEliteCost) {  // only the 20 smallest words are needed: a window selection
    __shared__ int wcnt;
    __shared__ unsigned long long wt0;
    const unsigned long long wv =
        tid < B ? ((unsigned long long)sort_key(p.obs_cost[g0 + perm[tid]]) << 32) | unsigned(tid) : ~0ull;
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
  // ---- compute_cost of the 20 elites: one wave each ----------------------
  const int lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  for (int j = w; j < kEliteCost; j += nw) {
    const int e = g0 + el[j];
    const size_t plane = size_t(p.Bt) * kN, row = size_t(e) * kN;
    const int t0 = lane, t1 = lane + 64;
    const bool v1 = t1 < kN;
    const int t1c = v1 ? t1 : kN - 1;
    auto ld = [&](int k, int tt) { return p.traj[size_t(k) * plane + row + tt]; };
    float y[2] = {ld(1, t0), ld(1, t1c)}, xd[2] = {ld(2, t0), ld(2, t1c)}, yd[2] = {ld(3, t0), ld(3, t1c)};
    float xdd[2] = {ld(4, t0), ld(4, t1c)}, ydd[2] = {ld(5, t0), ld(5, t1c)};
    float st[2] = {p.steer[row + t0], p.steer[row + t1c]};
    // neighbours for the diffs
    const float st_d0 = __shfl_down(st[0], 1, kWave);
    const float st_f1 = readlane_f(st[1], 0);
    const float st_n1 = __shfl_down(st[1], 1, kWave);
    const float st_n0 = lane < 63 ? st_d0 : st_f1;
    const float sv[2] = {st_n0 - st[0], st_n1 - st[1]};  // valid for t < 99
    const float sv_d0 = __shfl_down(sv[0], 1, kWave);
    const float sv_f1 = readlane_f(sv[1], 0);
    const float sv_n1 = __shfl_down(sv[1], 1, kWave);
    const float sv_n0 = lane < 63 ? sv_d0 : sv_f1;
    const float sa[2] = {sv_n0 - sv[0], sv_n1 - sv[1]};  // valid for t < 98
    double n_des = 0, n_st = 0, n_sv = 0, n_sa = 0, n_v = 0, n_sp = 0, n_svp = 0, n_ydd = 0, n_xdd = 0;
    double n_des2 = 0, n_cen = 0;  // CARLA: second desired lane, centripetal penalty
    float kap[2] = {0.f, 0.f};
    if (p.carla) {
      kap[0] = p.kappa_i[row + t0];
      kap[1] = p.kappa_i[row + t1c];
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int tt = q == 0 ? t0 : t1;
      if (tt >= kN) continue;
      const double dd = double(y[q] - (p.carla ? p.y_des1 : -1.75f));
      n_des += dd * dd;
      if (p.carla) {  // carla/optimizer/cem_helper.py:529-544
        const double d2 = double(y[q] - p.y_des2);
        n_des2 += d2 * d2;
        const double c = double(fmaxf(0.0f, fabsf((xd[q] * xd[q]) * kap[q]) - p.a_centr));
        n_cen += c * c;
      }
      n_st += double(st[q]) * double(st[q]);
      const float v = sqrtf(xd[q] * xd[q] + yd[q] * yd[q]);
      const double dv = double(v - cf.v_des);
      n_v += dv * dv;
      const double sp = double(fmaxf(0.0f, fabsf(st[q]) - 0.6f));
      n_sp += sp * sp;
      n_ydd += double(ydd[q]) * double(ydd[q]);
      n_xdd += double(xdd[q]) * double(xdd[q]);
      if (tt < kN - 1) {
        n_sv += double(sv[q]) * double(sv[q]);
        const double svp = double(fmaxf(0.0f, fabsf(sv[q]) - 0.05f));
        n_svp += svp * svp;
      }
      if (tt < kN - 2) n_sa += double(sa[q]) * double(sa[q]);
    }
    {  // the eleven wave totals at once (lanes 4 k .. 4 k + 3 hold total k)
      const double nv[11] = {n_des, n_st, n_sv, n_sa, n_v, n_sp, n_svp, n_ydd, n_xdd, n_des2, n_cen};
      const double z = wave_totals16_d(nv);
      n_des = sqrt(readlane_d(z, 0));
      n_st = sqrt(readlane_d(z, 4));
      n_sv = sqrt(readlane_d(z, 8));
      n_sa = sqrt(readlane_d(z, 12));
      n_v = sqrt(readlane_d(z, 16));
      n_sp = sqrt(readlane_d(z, 20));
      n_svp = sqrt(readlane_d(z, 24));
      n_ydd = sqrt(readlane_d(z, 28));
      n_xdd = sqrt(readlane_d(z, 32));
      n_des2 = sqrt(readlane_d(z, 36));
      n_cen = sqrt(readlane_d(z, 40));
    }
    if (lane == 0) {
      const double cobs = double(p.w_obs * p.obs_cost[e]);
      const double clane = double(p.w_lane * p.lane_cost[e]);
      double tot;
      if (p.carla) {  // carla/optimizer/cem_helper.py:546-554; risk terms weighted in fp32 (cem.py:373-375)
        const double cdes = double(p.w_des * p.lane_des[e]);
        tot = (double(p.res_norm[e]) + 0.1 * n_v + 0.1 * (n_st + n_sv + n_sa) + 0.1 * (n_sp + n_svp) +
               0.02 * n_ydd + 0.02 * n_xdd + 0.01 * (n_des * n_des2) + 0.1 * n_cen) +
              cobs + clane + cdes;
      } else {
        tot = double(p.res_norm[e]) + 0.1 * n_v + 0.1 * (n_st + n_sv + n_sa) + 0.1 * (n_sp + n_svp) +
              0.02 * n_ydd + 0.02 * n_xdd + 0.0 * n_des + cobs + 0.0 * clane;
      }
      cost20[j] = float(tot);
    }
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
  const float* pop = p.pop + (size_t(t & 1) * p.Bt + g0) * 8;
  float* pop_next = p.pop + (size_t((t + 1) & 1) * p.Bt + g0) * 8;
  if (tid < kElite * 8) {
    const int q = tid >> 3, c = tid & 7;
    pe[q][c] = pop[size_t(el[cem5[q]]) * 8 + c];
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
      mean32[c] = float((1.0 - 0.6) * double(cf.mean[c]) + 0.6 * s / sw);
    }
    wave_sync_lds();
    const int a = tid >> 3, c = tid & 7;
    const double ma = double(mean32[a]), mc = double(mean32[c]);
    double s = 0.0;
    for (int q = 0; q < kElite; ++q) s += wgt[q] * (double(pe[q][a]) - ma) * (double(pe[q][c]) - mc);
    const float v = float((1.0 - 0.6) * double(cf.cov[a * 8 + c]) + 0.6 * s / sw + (a == c ? 0.01 : 0.0));
    cvs[a][c] = double(v);
    cf.cov[a * 8 + c] = v;
    if (tid < 8) cf.mean[tid] = mean32[tid];
    wave_sync_lds();
  }
  if (tid < 64) {
    // Cholesky (lower) of the fp32 covariance, in fp64: column j's pivot on
    // lane j, then its entries below on lanes i > j in parallel (each entry's
    // sum in the serial algorithm's order, so the same bits)
    for (int j = 0; j < 8; ++j) {
      if (tid == j) {
        double d = cvs[j][j];
        for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
        L[j][j] = sqrt(d);
      }
      wave_sync_lds();
      if (tid > j && tid < 8) {
        double s = cvs[tid][j];
        for (int k = 0; k < j; ++k) s -= L[tid][k] * L[j][k];
        L[tid][j] = s / L[j][j];
      }
      if (tid < j) L[tid][j] = 0.0;
      wave_sync_lds();
    }
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
