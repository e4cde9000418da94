// The CARLA optimizer variant's risk stage (carla/optimizer/cem.py:311-356,
// 536-581 of the reference; "C/opt/" below):
//
//   k_roll_carla  rollouts of the candidate's rows from their own noisy
//                 initial states (cem_helper.py:754-805 baseline rows for cvar,
//                 mode 0; the beta-CEM's reduced set of mother rows for
//                 mmd_opt, mode 1, cem_helper.py:808-872), the recorded global
//                 points to Params::rxy
//   k_frenet      global_to_frenet_trajs (cem_helper.py:206-242): every
//                 recorded point to (s, d) by the closest of the P path points,
//                 a quad of lanes per point, the path staged in LDS
//   k_risk_carla  per candidate: collision residual in the Frenet frame
//                 (costs.py:48-57, a = 4.5, b = 3), lane and desired-lane bars,
//                 then CVaR (costs.py:133-153, 84-100, 184-198) or the MMD with
//                 the beta-CEM's beta / sigma (costs.py:116-130, 70-82, 168-181)
//
// Splitting the rollouts (sequential in the step) from the Frenet search
// (independent per point) keeps the search, the dominant cost, at a quad of
// lanes per point: B x rows x H x 4 threads instead of B x rows.
#include "block.hpp"
#include "frenet.hpp"
#include "kernels.hpp"
#include "rng.hpp"
#include "rollout.hpp"

namespace mpcmmd {

namespace {

constexpr int kN = 100;

// One wave per (candidate, 64 rows).  The step's control and tan(steer) do
// not depend on the state: every lane first computes (row, step) pairs of
// the wave's rows into LDS (tan off the step chain, spread over the wave's
// 64 lanes rather than the S < 64 live rows), then each row runs its chain of
// H - 1 steps with one fp64 sincos per step.
constexpr int kRollLds = 64 * 2 * kMaxH;  // floats: [h][row] controls and tan(steer)
__global__ __launch_bounds__(64) void k_roll_carla(Params p, int t, int mode) {
  __shared__ float ctl[kRollLds];
  const int b = blockIdx.x, S = p.S, H = p.H, n = p.n, lane = threadIdx.x;
  const int r0 = blockIdx.y * 64, rows = min(64, S - r0);
  const Cfg cf = cfg_of(p, b / p.B);
  float* an_l = ctl;             // [h][64]
  float* tn_l = ctl + 64 * kMaxH;
  const float* ctrl = p.ctrl_n + size_t(b) * 2 * n * H;
  const float* bpl = p.noise == 1 ? p.bplane + size_t(b) * 2 * H * S : nullptr;
  for (int e = lane; e < rows * (H - 1); e += 64) {
    const int h = e / rows, rr = e - h * rows, r = r0 + rr;
    float an, sn;
    if (mode == 1) {  // reduced-set row m of the mother set: controls repeat(acc, n) x tile(steer, n)
      const int m = p.bestsel[size_t(b) * n + r];
      an = ctrl[(m / n) * H + h];
      sn = ctrl[n * H + (m % n) * H + h];
    } else {
      noisy_control<true>(p, cf, t, r, h, p.acc[size_t(b) * kN + h], p.steer[size_t(b) * kN + h], an, sn, bpl);
    }
    an_l[h * 64 + rr] = an;
    tn_l[h * 64 + rr] = float(tan(double(sn)));
  }
  __syncthreads();
  if (lane >= rows) return;
  const int r = r0 + lane;
  const int m = mode == 1 ? p.bestsel[size_t(b) * n + r] : r;  // the row's noisy initial state
  const float* st = p.st0r + (size_t(cf.g) * p.R0 + m) * 8;
  float x = st[0], y = st[1], vx = st[2], vy = st[3], psi = st[4];
  float* out = p.rxy + (size_t(b) * S + r) * 2 * H;
  for (int h = 0; h < H; ++h) {
    out[h] = x;  // x_roll[:, h] = state before step h (cem_helper.py:794-797)
    out[H + h] = y;
    if (h == H - 1) break;
    bicycle_step_cr_t(x, y, vx, vy, psi, an_l[h * 64 + lane], tn_l[h * 64 + lane], p.wheel_base);
  }
}

// four lanes per point (frenet_point_quad): B x rows x H x 4 threads, so the
// path scan's LDS latency is hidden by ~4 waves per SIMD
__global__ __launch_bounds__(256) void k_frenet(Params p, int total) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int P = p.P, H = p.H, S = p.S, g = blockIdx.y, Pq = frenet_quarter(P);
  float2* pxy = reinterpret_cast<float2*>(smem);
  float* arc = reinterpret_cast<float*>(pxy + 4 * Pq);
  float* Fxd = arc + P;
  float* Fyd = Fxd + P;
  const float* pa = p.path + size_t(g) * 6 * kMaxPath;
  const float inf = __int_as_float(0x7f800000);
  for (int j = threadIdx.x; j < 4 * Pq; j += blockDim.x) {
    pxy[j] = j < P ? make_float2(pa[j], pa[kMaxPath + j]) : make_float2(inf, inf);
    if (j < P) {
      arc[j] = pa[2 * kMaxPath + j];
      Fxd[j] = pa[3 * kMaxPath + j];
      Fyd[j] = pa[4 * kMaxPath + j];
    }
  }
  __syncthreads();
  const int e = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;  // point of configuration g (quad-uniform)
  if (e >= total) return;
  const int bl = e / (S * H), rh = e - bl * S * H, r = rh / H, h = rh - r * H;
  float* q = p.rxy + ((size_t(g) * p.B + bl) * S + r) * 2 * H + h;
  float s, d;
  frenet_point_quad(q[0], q[H], pxy, arc, Fxd, Fyd, P, Pq, s, d);
  if ((threadIdx.x & 3) == 0) {
    q[0] = s;
    q[H] = d;
  }
}

size_t risk_carla_lds(int O, int H, int S) {
  size_t f = size_t(2 * O * H + 4 * S) * 4;
  f = (f + 15) & ~size_t(15);
  f += size_t(S) * 8;
  f = (f + 15) & ~size_t(15);
  f += sizeof(ReduceScratch);
  f = (f + 15) & ~size_t(15);
  return f + size_t(std::max(256, S)) * 4 * 4;  // the (row, step chunk) partial maxima
}

// Workgroup per candidate (256 threads).  The per-row maxima over the H steps
// (collision residual over the obstacles, lane bars) are split over (row,
// chunk of steps) threads, then each row's chunks are combined -- max is
// exact in any order, so the bars are those of a sequential scan; the
// desired-lane sums stay one sequential fp64 sum per row.
__global__ __launch_bounds__(256) void k_risk_carla(Params p, int t, int mode) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int O = p.O, H = p.H, S = p.S, b = blockIdx.x, tid = threadIdx.x;
  const Cfg cf = cfg_of(p, b / p.B);
  float* xo = reinterpret_cast<float*>(smem);
  float* yo = xo + O * H;
  float* cbar = yo + O * H;
  float* lb = cbar + S;
  float* ub = lb + S;
  float* des = ub + S;
  size_t off = size_t(2 * O * H + 4 * S) * 4;
  off = (off + 15) & ~size_t(15);
  unsigned long long* list = reinterpret_cast<unsigned long long*>(smem + off);
  off += size_t(S) * 8;
  off = (off + 15) & ~size_t(15);
  ReduceScratch& rs = *reinterpret_cast<ReduceScratch*>(smem + off);
  off += sizeof(ReduceScratch);
  off = (off + 15) & ~size_t(15);
  // [S K] (<= max(256, S)): chunk maxima c, l, u and the NaN flag
  const int K = max(1, int(blockDim.x) / S), L = (H + K - 1) / K;  // chunks per row, steps per chunk
  const int NP = max(256, S);
  float* pc = reinterpret_cast<float*>(smem + off);
  float* pl = pc + NP;
  float* pu = pl + NP;
  int* pn = reinterpret_cast<int*>(pu + NP);
  for (int i = tid; i < O * H; i += blockDim.x) {
    xo[i] = cf.obs[i];  // Frenet obstacle tracks x_obs_traj[:, :H], y_obs_traj[:, :H]
    yo[i] = cf.obs[O * H + i];
  }
  __syncthreads();
  for (int e = tid; e < S * K; e += blockDim.x) {  // S > 256: K = 1, rows strided over the threads
    const int r = e / K, c = e - r * K;
    const float* q = p.rxy + (size_t(b) * S + r) * 2 * H;
    float cm = 0.0f, l = 0.0f, u = 0.0f;
    bool nan = false;
    for (int h = c * L; h < min(H, (c + 1) * L); ++h) {
      const float s = q[h], d = q[H + h];
      for (int o = 0; o < O; ++o) {
        const float f = f_bar_ab(s, d, xo[o * H + h], yo[o * H + h], p.obs_a2, p.obs_b2);
        nan |= (f != f);
        cm = fmaxf(cm, f);
      }
      nan |= (d != d);
      l = fmaxf(l, -d + p.y_lb);
      u = fmaxf(u, d - p.y_ub);
    }
    pc[e] = cm;
    pl[e] = l;
    pu[e] = u;
    pn[e] = nan ? 1 : 0;
  }
  double s1 = 0.0, s2 = 0.0;  // ||y - y_des_1||_F^2, ||y - y_des_2||_F^2 over rows x steps
  for (int r = tid; r < S; r += blockDim.x) {
    const float* q = p.rxy + (size_t(b) * S + r) * 2 * H;
    for (int h = 0; h < H; ++h) {
      const double e1 = double(q[H + h]) - double(p.y_des1), e2 = double(q[H + h]) - double(p.y_des2);
      s1 += e1 * e1;
      s2 += e2 * e2;
    }
  }
  __syncthreads();
  for (int r = tid; r < S; r += blockDim.x) {
    float cm = 0.0f, l = 0.0f, u = 0.0f;
    int nan = 0;
    for (int c = 0; c < K; ++c) {
      cm = fmaxf(cm, pc[r * K + c]);
      l = fmaxf(l, pl[r * K + c]);
      u = fmaxf(u, pu[r * K + c]);
      nan |= pn[r * K + c];
    }
    const float qnan = __int_as_float(0x7fc00000);
    cbar[r] = nan ? qnan : cm;
    lb[r] = nan ? qnan : l;
    ub[r] = nan ? qnan : u;
  }
  s1 = block_sum(s1, rs.d);
  s2 = block_sum(s2, rs.d);
  // compute_lane_des_*: max(0, ||y - y1|| ||y - y2|| - gamma), one value for every row.
  // The two squared norms are fp64 sums rounded once (the reference: fp32
  // jnp.linalg.norm; oracle/carla.py lane_des_bar does the same as here), and
  // a NaN rollout gives NaN as jnp.maximum does (fmaxf would drop it)
  const float cdv = float(sqrt(s1)) * float(sqrt(s2)) - p.gamma_des;
  const float cd = cdv != cdv ? cdv : fmaxf(0.0f, cdv);
  for (int r = tid; r < S; r += blockDim.x) des[r] = cd;
  __syncthreads();
  float obs, lane, dl;
  if (mode == 0) {
    obs = block_cvar(cbar, S, list, rs);
    const float cl = block_cvar(lb, S, list, rs);
    const float cu = block_cvar(ub, S, list, rs);
    lane = cl + cu;
    dl = block_cvar(des, S, list, rs);
  } else {
    const float* bt = p.beta + size_t(b) * p.n;
    const float sigma = p.sigma[b];
    obs = block_mmd(cbar, bt, S, sigma, 1000.0f, rs);
    const float ml = block_mmd(lb, bt, S, sigma, 1000.0f, rs);
    const float mu = block_mmd(ub, bt, S, sigma, 1000.0f, rs);
    lane = ml + mu;
    dl = block_mmd(des, bt, S, sigma, 1000.0f, rs);
  }
  if (tid == 0) {
    p.obs_cost[b] = obs;
    p.lane_cost[b] = lane;
    p.lane_des[b] = dl;
  }
}

}  // namespace

void launch_roll_carla(const Params& p, int t, int mode, hipStream_t s) {
  hipLaunchKernelGGL(k_roll_carla, dim3(p.Bt, (p.S + 63) / 64), dim3(64), 0, s, p, t, mode);
}

void launch_frenet(const Params& p, hipStream_t s) {
  const int total = p.B * p.S * p.H;
  const size_t lds = size_t(4) * frenet_quarter(p.P) * 8 + size_t(p.P) * 12;
  hipLaunchKernelGGL(k_frenet, dim3((total * 4 + 255) / 256, p.G), dim3(256), lds, s, p, total);
}

void launch_risk_carla(const Params& p, int t, int mode, hipStream_t s) {
  hipLaunchKernelGGL(k_risk_carla, dim3(p.Bt), dim3(256), risk_carla_lds(p.O, p.H, p.S), s, p, t, mode);
}

}  // namespace mpcmmd
