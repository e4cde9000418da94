// Stage "risk" for cost = mmd_opt: the mother rollouts, their Bernstein fit
// and the nested beta-CEM that picks the reduced set and the MMD weights,
// then the reduced-set MMD.  Per outer iteration:
//
//   k_mother    noisy control rows, n^2 mother rollouts (Cartesian product,
//               cem_helper.py:469-530) with the ridge fit folded into the scan
//               (compute_coeff, cem_helper.py:553-564) -> 22 features per row
//   20 x { k_bsample  samples of the beta-CEM and their top-n |beta| rows
//                     (compute_beta.py:41-49, 51-68, 117-118)
//          k_bkernel  Laplace-kernel row sums over the mother set, K_red, the
//                     equality-constrained QP and its cost per sample
//                     (kernel_computation.py:19-65, compute_beta.py:70-91, 120-129)
//          k_belite   elite 11, mean, structured Cholesky of
//                     cov = D D^T / 10 + 0.05 I, next generators (compute_beta.py:51-68, 133-145) }
//   k_mmdfinal  reduced-set rollouts, collision residual, MMD obs / lane
//               (costs.py:121-135, 173-186)
//
// All kernels: one 512-thread workgroup per candidate (the candidate's beta-CEM
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
constexpr int kMaxQ = 16;                            // M <= 1024 -> 16 values per lane
constexpr double kSqrt20 = 4.47213595499957927704;   // chol(20 I) (compute_beta.py:24)
constexpr double kRidge = 0.05;                      // cov jitter (compute_beta.py:61)

DEVI void wave_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

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
// scratch: 2 * 32 ints of LDS owned by the wave.
template <class V>
DEVI void select_top(V val, int M, int n, int32_t* out, int* scratch) {
  const int lane = threadIdx.x & 63;
  const int nq = (M + 63) >> 6;
  uint32_t key[kMaxQ];
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) {
    const int j = lane + 64 * q;
    key[q] = (q < nq && j < M) ? sort_key(fabsf(val(j))) : 0u;
  }
  // T = n-th largest key (bisection on the key bits)
  uint32_t T = 0u;
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t cand = T | (1u << bit);
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < kMaxQ; ++q)
      if (q < nq) cnt += __popcll(__ballot(key[q] >= cand));
    if (cnt >= n) T = cand;
  }
  int gt = 0;
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q)
    if (q < nq) gt += __popcll(__ballot(key[q] > T));
  const int need = n - gt;  // equal keys taken from the largest indices
  unsigned long long eqm[kMaxQ];
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) eqm[q] = q < nq ? __ballot(key[q] == T) : 0ull;
  const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  int* lj = scratch;
  uint32_t* lk = reinterpret_cast<uint32_t*>(scratch + 32);
  int base = 0;
  int later_eq = 0;  // equal keys in q' > q
  for (int q = nq - 1; q >= 0; --q) later_eq += __popcll(eqm[q]);
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) {
    if (q >= nq) break;
    later_eq -= __popcll(eqm[q]);
    const int larger = later_eq + __popcll(eqm[q] & above);
    const bool sel = key[q] > T || (key[q] == T && larger < need);
    const unsigned long long sm = __ballot(sel);
    if (sel) {
      const int pos = base + __popcll(sm & ((1ull << lane) - 1ull));
      lj[pos] = lane + 64 * q;
      lk[pos] = key[q];
    }
    base += __popcll(sm);
  }
  wave_sync();
  if (lane < n) {
    const int j = lj[lane];
    const uint32_t k = lk[lane];
    int r = 0;
    for (int c = 0; c < n; ++c) {
      const uint32_t kc = lk[c];
      const int jc = lj[c];
      r += (kc < k) || (kc == k && jc < j);
    }
    out[r] = j;
  }
  wave_sync();
}

// ------------------------------------------------------------------------
// New beta-CEM samples with the structured Cholesky (see file header).
// lanes = samples (sidx(lane) = new-sample index 0..88, or -1), waves =
// position blocks; two passes: block partial sums P = sum w_j z_j, then the
// scan.  emit(lane, j, y) receives fp32 y for every position j <= M.
// Pbuf: 8 * 11 * 64 doubles of LDS (may alias the emit target: a barrier
// separates its last read from the first emit).
template <class SIdx, class Emit>
DEVI void generate(const Params& p, int b, int tz, SIdx sidx, Emit emit, double* Pbuf) {
  const int M1 = p.M + 1, lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int bs = (M1 + nw - 1) / nw;
  const int j0 = min(M1, w * bs), j1 = min(M1, j0 + bs);
  const double* G = p.gen + size_t(b) * M1 * kGenStride;
  const float* gm = p.genm + size_t(b) * M1;
  const float* z = p.beta_z + size_t(tz) * M1 * kNew;  // device layout [M+1][89]
  const int si = sidx(lane);
  const bool act = si >= 0;
  const int sz = act ? si : 0;
  double P[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) P[k] = 0.0;
  for (int j = j0; j < j1; ++j) {
    const double zj = act ? double(z[size_t(j) * kNew + sz]) : 0.0;
    const double* g = G + size_t(j) * kGenStride;
#pragma unroll
    for (int k = 0; k < 11; ++k) P[k] = P[k] + g[k] * zj;
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
  __syncthreads();
  for (int j = j0; j < j1; ++j) {
    const double zj = act ? double(z[size_t(j) * kNew + sz]) : 0.0;
    const double* g = G + size_t(j) * kGenStride;
    double d = 0.0;
#pragma unroll
    for (int k = 0; k < 11; ++k) d = d + g[11 + k] * S[k];
    const double yv = (double(gm[j]) + g[22] * zj) + d;
#pragma unroll
    for (int k = 0; k < 11; ++k) S[k] = S[k] + g[k] * zj;
    if (act) emit(lane, j, float(yv));
  }
}

// ------------------------------------------------------------------------
// k_bsample: the 100 samples of beta-CEM iteration tb and their top-n rows.
__global__ __launch_bounds__(kThreads) void k_bsample(Params p, int tb, int spr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, M = p.M, M1 = M + 1, n = p.n;
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = threadIdx.x & 63;
  const int ys = spr + 1;
  float* ybuf = reinterpret_cast<float*>(smem);
  size_t ybytes = size_t(M1) * ys * 4;
  const size_t pbytes = size_t(8) * 11 * 64 * 8;
  if (ybytes < pbytes) ybytes = pbytes;
  int* wscr = reinterpret_cast<int*>(smem + ((ybytes + 15) & ~size_t(15))) + w * 64;
  int32_t* sel = p.bsel + size_t(b) * kBetaSamples * n;
  float* sig = p.bsig + size_t(b) * kBetaSamples;
  if (tb == 0) {
    // initial samples MVN(0, 20 I) with chol(20 I) = sqrt(20) I (compute_beta.py:41-49)
    for (int s = w; s < kBetaSamples; s += nw) {
      const float* z0 = p.beta_z0 + size_t(s) * M1;
      auto val = [&](int j) { return float(kSqrt20 * double(z0[j])); };
      select_top(val, M, n, sel + s * n, wscr);
      if (lane == 0) sig[s] = fmaxf(val(M), 0.01f);
    }
    return;
  }
  // rows 0..10: the previous iteration's elites (compute_beta.py:62)
  const float* E = p.belite + (size_t(tb & 1) * p.B + b) * kBetaElite * M1;
  for (int s = w; s < kBetaElite; s += nw) {
    const float* e = E + size_t(s) * M1;
    auto val = [&](int j) { return e[j]; };
    select_top(val, M, n, sel + s * n, wscr);
    if (lane == 0) sig[s] = e[M];
  }
  // rows 11..99: mean + L z (compute_beta.py:63), in rounds of spr samples
  for (int r0 = 0; r0 < kNew; r0 += spr) {
    const int ns = min(spr, kNew - r0);
    __syncthreads();
    generate(
        p, b, tb - 1, [&](int l) { return l < ns ? r0 + l : -1; },
        [&](int l, int j, float y) { ybuf[size_t(j) * ys + l] = y; }, reinterpret_cast<double*>(smem));
    __syncthreads();
    for (int sl = w; sl < ns; sl += nw) {
      auto val = [&](int j) { return ybuf[size_t(j) * ys + sl]; };
      const int s = kBetaElite + r0 + sl;
      select_top(val, M, n, sel + s * n, wscr);
      if (lane == 0) sig[s] = fmaxf(val(M), 0.01f);
    }
  }
}

// ------------------------------------------------------------------------
// k_bkernel LDS carve (host and device agree)
struct KerLds {
  size_t F, sel, rsig, rowsum, cnt, start, fill, ulist, urank, pairs, work, total;
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
  L.F = take(size_t(kF) * M * 4);
  L.sel = take(size_t(kBetaSamples) * n * 2);
  L.rsig = take(size_t(2) * kBetaSamples * 4);
  L.rowsum = take(size_t(kBetaSamples) * n * 8);
  L.cnt = take(size_t(M) * 4);
  L.start = take(size_t(M) * 4);
  L.fill = take(size_t(M) * 4);
  L.ulist = take(size_t(M) * 4);
  L.urank = take(size_t(M) * 4);
  L.pairs = take(size_t(kBetaSamples) * n * 2);
  L.work = o;
  // QP needs per wave: packed L (n(n+1)/2 doubles) + K [32][33] floats + beta [32] doubles
  const size_t qp = size_t(8) * ((size_t(n) * (n + 1) / 2) * 8 + 32 * 33 * 4 + 32 * 8 + 64);
  size_t rest = budget > o ? budget - o : 0;
  int rows = int(rest / (size_t(M) * 4));
  if (rows > 64) rows = 64;
  L.rows = rows;
  size_t work = size_t(rows) * M * 4;
  if (work < qp) work = qp;
  L.total = o + work;
  return L;
}

constexpr size_t kLdsBudget = 160 * 1024 - 1024;

__global__ __launch_bounds__(kThreads) void k_bkernel(Params p, int tb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, M = p.M, n = p.n;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const KerLds C = ker_lds(M, n, kLdsBudget);
  float* Fl = reinterpret_cast<float*>(smem + C.F);
  short* sl = reinterpret_cast<short*>(smem + C.sel);
  float* sg = reinterpret_cast<float*>(smem + C.rsig);
  float* rsg = sg + kBetaSamples;
  double* rowsum = reinterpret_cast<double*>(smem + C.rowsum);
  int* cnt = reinterpret_cast<int*>(smem + C.cnt);
  int* start = reinterpret_cast<int*>(smem + C.start);
  int* fill = reinterpret_cast<int*>(smem + C.fill);
  int* ulist = reinterpret_cast<int*>(smem + C.ulist);
  int* urank = reinterpret_cast<int*>(smem + C.urank);
  short* pairs = reinterpret_cast<short*>(smem + C.pairs);
  float* Dl = reinterpret_cast<float*>(smem + C.work);
  const float* Fg = p.feat + size_t(b) * kF * M;
  for (int i = tid; i < kF * M; i += blockDim.x) Fl[i] = Fg[i];
  const int32_t* sg_sel = p.bsel + size_t(b) * kBetaSamples * n;
  for (int i = tid; i < kBetaSamples * n; i += blockDim.x) sl[i] = short(sg_sel[i]);
  for (int s = tid; s < kBetaSamples; s += blockDim.x) {
    const float v = p.bsig[size_t(b) * kBetaSamples + s];
    sg[s] = v;
    rsg[s] = 1.0f / v;
  }
  for (int r = tid; r < M; r += blockDim.x) {
    cnt[r] = 0;
    fill[r] = 0;
  }
  __syncthreads();
  // ---- rows used by any sample (the reduced rows are mother rows, so every
  // K_mixed row is a row of the M x M mother distance matrix)
  for (int i = tid; i < kBetaSamples * n; i += blockDim.x) atomicAdd(&cnt[sl[i]], 1);
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
  for (int i = tid; i < kBetaSamples * n; i += blockDim.x) {
    const int r = sl[i];
    const int pos = start[r] + atomicAdd(&fill[r], 1);
    pairs[pos] = short(i);  // i = s * n + k
  }
  for (int i = tid; i < kBetaSamples * n; i += blockDim.x) rowsum[i] = 0.0;
  __syncthreads();
  // ---- K_mixed row sums: D rows of the union, chunk by chunk, in LDS
  const int R = C.rows;
  const int g = tid >> 4, gl = tid & 15, ng = blockDim.x >> 4;
  for (int c0 = 0; c0 < U; c0 += R) {
    const int rc = min(R, U - c0);
    for (int idx = tid; idx < rc * M; idx += blockDim.x) {
      const int u = idx / M, j = idx - u * M;
      const int r = ulist[c0 + u];
      float d = fabsf(Fl[r] - Fl[j]);
      for (int f = 1; f < kF; ++f) d = d + fabsf(Fl[f * M + r] - Fl[f * M + j]);
      Dl[idx] = d;
    }
    __syncthreads();
    const int p0 = start[ulist[c0]];
    const int p1 = start[ulist[c0 + rc - 1]] + cnt[ulist[c0 + rc - 1]];
    for (int pi = p0 + g; pi < p1; pi += ng) {
      const int i = pairs[pi];
      const int s = i / n;
      const int u = urank[sl[i]] - c0;
      const float sgm = sg[s], rs = rsg[s];
      const float* drow = Dl + size_t(u) * M;
      float acc = 0.0f;
      for (int j = gl; j < M; j += 16) acc += __expf(div_rc(-drow[j], sgm, rs));
      double a = double(acc);
      a += __shfl_xor(a, 1, 16);
      a += __shfl_xor(a, 2, 16);
      a += __shfl_xor(a, 4, 16);
      a += __shfl_xor(a, 8, 16);
      if (gl == 0) rowsum[i] = a;
    }
    __syncthreads();
  }
  // ---- K_red, QP (compute_beta_reduced) and cost, one wave per sample
  const size_t qpw = (size_t(n) * (n + 1) / 2) * 8 + 32 * 33 * 4 + 32 * 8 + 64;
  char* qbase = smem + C.work + size_t(w) * qpw;
  double* Lp = reinterpret_cast<double*>(qbase);                                      // packed lower
  float* Kl = reinterpret_cast<float*>(qbase + (size_t(n) * (n + 1) / 2) * 8);         // [32][33]
  double* bl = reinterpret_cast<double*>(qbase + (size_t(n) * (n + 1) / 2) * 8 + 32 * 33 * 4);
  const double inv_m = double(1.0f / float(M));
  for (int s = w; s < kBetaSamples; s += nw) {
    const float sgm = sg[s], rs = rsg[s];
    const int ti = lane < n ? sl[s * n + lane] : 0;
    if (lane < n) {
      const int rowoff = lane * (lane + 1) / 2;
      for (int k = 0; k < n; ++k) {
        const int tk = sl[s * n + k];
        float d = fabsf(Fl[ti] - Fl[tk]);
        for (int f = 1; f < kF; ++f) d = d + fabsf(Fl[f * M + ti] - Fl[f * M + tk]);
        const float kv = __expf(div_rc(-d, sgm, rs));
        Kl[lane * 33 + k] = kv;
        if (k <= lane) Lp[rowoff + k] = double(k == lane ? kv + 0.05f : kv);
      }
    }
    wave_sync();
    // left-looking Cholesky, lane = row
    for (int j = 0; j < n; ++j) {
      double sv = 0.0;
      if (lane >= j && lane < n) {
        const int ri = lane * (lane + 1) / 2, rj = j * (j + 1) / 2;
        sv = Lp[ri + j];
        for (int k = 0; k < j; ++k) sv -= Lp[ri + k] * Lp[rj + k];
        if (lane == j) Lp[ri + j] = sqrt(sv);
      }
      wave_sync();
      if (lane > j && lane < n) Lp[lane * (lane + 1) / 2 + j] = sv / Lp[j * (j + 1) / 2 + j];
      wave_sync();
    }
    // two right-hand sides: g = rowsum / M (= -lincost) and 1 (the constraint column)
    double a1 = lane < n ? rowsum[s * n + lane] * inv_m : 0.0, a2 = lane < n ? 1.0 : 0.0;
    for (int j = 0; j < n; ++j) {  // forward, column-oriented
      double y1 = 0.0, y2 = 0.0;
      if (lane == j) {
        const double dj = Lp[j * (j + 1) / 2 + j];
        y1 = a1 / dj;
        y2 = a2 / dj;
        a1 = y1;
        a2 = y2;
      }
      y1 = __shfl(y1, j, 64);
      y2 = __shfl(y2, j, 64);
      if (lane > j && lane < n) {
        const double lij = Lp[lane * (lane + 1) / 2 + j];
        a1 -= lij * y1;
        a2 -= lij * y2;
      }
    }
    for (int j = n - 1; j >= 0; --j) {  // backward with L^T
      double x1 = 0.0, x2 = 0.0;
      if (lane == j) {
        const double dj = Lp[j * (j + 1) / 2 + j];
        x1 = a1 / dj;
        x2 = a2 / dj;
        a1 = x1;
        a2 = x2;
      }
      x1 = __shfl(x1, j, 64);
      x2 = __shfl(x2, j, 64);
      if (lane < j) {
        const double lji = Lp[j * (j + 1) / 2 + lane];
        a1 -= lji * x1;
        a2 -= lji * x2;
      }
    }
    // beta = x1 + ((1 - sum x1) / sum x2) x2   (KKT with 1^T beta = 1)
    const double s1 = wave_sum(lane < n ? a1 : 0.0), s2 = wave_sum(lane < n ? a2 : 0.0);
    const float beta = lane < n ? float(a1 + ((1.0 - s1) / s2) * a2) : 0.0f;
    if (lane < n) bl[lane] = double(beta);
    wave_sync();
    double kb = 0.0, qb = 0.0;
    if (lane < n) {
      for (int k = 0; k < n; ++k) kb += double(Kl[lane * 33 + k]) * bl[k];
      kb *= double(beta);
      qb = (-2.0 * (rowsum[s * n + lane] * inv_m)) * double(beta);
    }
    const double cost = wave_sum(kb) + wave_sum(qb);
    if (lane < n) p.btop[(size_t(b) * kBetaSamples + s) * n + lane] = beta;
    if (lane == 0) p.bcost[size_t(b) * kBetaSamples + s] = float(cost);
    wave_sync();
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
  size_t u = size_t(M1) * 11 * 8;
  const size_t pbuf = size_t(8) * 11 * 64 * 8;  // generate() scratch aliases U
  if (u < pbuf) u = pbuf;
  L.U = 0;
  L.Gb = (u + 15) & ~size_t(15);
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
  // ---- E_new = the 11 elite sample vectors (rows 0..10 of the next samples)
  const float* Eold = p.belite + (size_t(tb & 1) * p.B + b) * kBetaElite * M1;
  float* Enew = p.belite + (size_t((tb + 1) & 1) * p.B + b) * kBetaElite * M1;
  for (int i = tid; i < kBetaElite * M1; i += blockDim.x) {
    const int q = i / M1, j = i - q * M1;
    const int e = elite[q];
    if (tb == 0) {
      float v = float(kSqrt20 * double(p.beta_z0[size_t(e) * M1 + j]));
      if (j == M) v = fmaxf(v, 0.01f);
      Enew[i] = v;
    } else if (e < kBetaElite) {
      Enew[i] = Eold[size_t(e) * M1 + j];
    }
  }
  if (tb > 0) {  // elites that were new samples: regenerate them (generators of tb-1)
    generate(
        p, b, tb - 1,
        [&](int l) { return (l < kBetaElite && elite[l] >= kBetaElite) ? elite[l] - kBetaElite : -1; },
        [&](int l, int j, float y) { Enew[size_t(l) * M1 + j] = j == M ? fmaxf(y, 0.01f) : y; },
        reinterpret_cast<double*>(smem + C.U));
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
      acc += g / kRidge;
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
      for (int a = 0; a < 11; ++a)
#pragma unroll
        for (int c = a; c < 11; ++c) A[sym11(a, c)] += uk[a] * uk[c] / kRidge;
    }
    // Cholesky A = R^T R (R upper, stored in A)
#pragma unroll
    for (int a = 0; a < 11; ++a) {
      double d = A[sym11(a, a)];
#pragma unroll
      for (int k = 0; k < a; ++k) d -= A[sym11(k, a)] * A[sym11(k, a)];
      d = sqrt(d);
      A[sym11(a, a)] = d;
#pragma unroll
      for (int c = a + 1; c < 11; ++c) {
        double s = A[sym11(a, c)];
#pragma unroll
        for (int k = 0; k < a; ++k) s -= A[sym11(k, a)] * A[sym11(k, c)];
        A[sym11(a, c)] = s / d;
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
      for (int k = 0; k < a; ++k) s -= A[sym11(k, a)] * v[k];
      v[a] = s / A[sym11(a, a)];
    }
    // R v = y
#pragma unroll
    for (int a = 10; a >= 0; --a) {
      double s = v[a];
#pragma unroll
      for (int k = a + 1; k < 11; ++k) s -= A[sym11(a, k)] * v[k];
      v[a] = s / A[sym11(a, a)];
    }
    double uv = 0.0;
#pragma unroll
    for (int a = 0; a < 11; ++a) uv += u[a] * v[a];
    const double ljj = sqrt(kRidge + uv);
    double* g = gen + size_t(j) * kGenStride;
#pragma unroll
    for (int a = 0; a < 11; ++a) {
      g[a] = v[a] / ljj;
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

int samples_per_round(int M1) { return size_t(M1) * 65 * 4 <= 140 * 1024 ? 64 : 32; }

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
  const int M1 = p.M + 1, spr = samples_per_round(M1);
  size_t ybytes = size_t(M1) * (spr + 1) * 4;
  const size_t pbytes = size_t(8) * 11 * 64 * 8;
  if (ybytes < pbytes) ybytes = pbytes;
  const size_t lds = ((ybytes + 15) & ~size_t(15)) + size_t(8) * 64 * 4;
  hipLaunchKernelGGL(k_bsample, dim3(p.B), dim3(kThreads), lds, s, p, tb, spr);
}

void launch_bkernel(const Params& p, int tb, hipStream_t s) {
  const KerLds k = ker_lds(p.M, p.n, kLdsBudget);
  hipLaunchKernelGGL(k_bkernel, dim3(p.B), dim3(kThreads), k.total, s, p, tb);
}

void launch_belite(const Params& p, int tb, hipStream_t s) {
  const EliteLds e = elite_lds(p.M + 1);
  hipLaunchKernelGGL(k_belite, dim3(p.B), dim3(kThreads), e.total, s, p, tb);
}

void launch_mmdfinal(const Params& p, int t, hipStream_t s) {
  hipLaunchKernelGGL(k_mmdfinal, dim3(p.B), dim3(64), 0, s, p, t);
}

}  // namespace mpcmmd
