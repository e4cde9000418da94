// Stage "risk" for the baseline cost variants (cvar, saa, mmd_random): one
// workgroup per candidate, one thread per noisy rollout sample.
//
//   noise injection          optimizer/cem_helper.py:405-443 (gaussian / beta)
//   compute_rollout_one_step optimizer/cem_helper.py:380-400
//   H-step scan              optimizer/cem_helper.py:445-461
//   compute_f_bar + max      optimizer/costs.py:50-60, 210-213
//   compute_lane_bar + max   optimizer/costs.py:62-71
//   reducers                 costs.py:206-234 (obs), 137-171 (lane),
//                            kernel_computation.py:67-87 (mmd_random)
//
// The B x S x H rollout planes of the reference are never materialised: each
// thread keeps its state in registers and folds the collision residual
// (O obstacles, staged in LDS) and the lane bars into running maxima, so
// the stage reads only the candidate's H controls and the shared noise rows
// (L2-resident, [H][S] for coalescing) and writes two floats per candidate.
#include "block.hpp"
#include "kernels.hpp"
#include "rng.hpp"
#include "rollout.hpp"

namespace mpcmmd {

namespace {

struct RiskLds {
  float* xo;
  float* yo;
  float* a;
  float* st;
  float* cbar;
  float* lb;
  float* ub;
  unsigned long long* list;
  ReduceScratch* rs;
};

DEVI RiskLds carve(char* base, int O, int H, int S) {
  RiskLds L;
  float* f = reinterpret_cast<float*>(base);
  L.xo = f;
  f += O * H;
  L.yo = f;
  f += O * H;
  L.a = f;
  f += H;
  L.st = f;
  f += H;
  L.cbar = f;
  f += S;
  L.lb = f;
  f += S;
  L.ub = f;
  f += S;
  size_t off = size_t(reinterpret_cast<char*>(f) - base);
  off = (off + 15) & ~size_t(15);
  L.list = reinterpret_cast<unsigned long long*>(base + off);
  off += size_t(S) * 8;
  off = (off + 15) & ~size_t(15);
  L.rs = reinterpret_cast<ReduceScratch*>(base + off);
  return L;
}

}  // namespace

size_t risk_lds_bytes(int O, int H, int S) {
  size_t f = size_t(2 * O * H + 2 * H + 3 * S) * 4;
  f = (f + 15) & ~size_t(15);
  f += size_t(S) * 8;  // (key, index) pairs of block_cvar
  f = (f + 15) & ~size_t(15);
  return f + sizeof(ReduceScratch);
}

namespace {

__global__ __launch_bounds__(512) void k_risk_baseline(Params p, int t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int O = p.O, H = p.H, S = p.S;
  RiskLds L = carve(smem, O, H, S);
  const int b = blockIdx.x;
  const Cfg cf = cfg_of(p, b / p.B);
  for (int i = threadIdx.x; i < O * H; i += blockDim.x) {
    L.xo[i] = cf.obs[i];
    L.yo[i] = cf.obs[O * H + i];
  }
  for (int h = threadIdx.x; h < H; h += blockDim.x) {
    L.a[h] = p.acc[size_t(b) * 100 + h];
    L.st[h] = p.steer[size_t(b) * 100 + h];
  }
  __syncthreads();
  const float* bpl = p.noise == 1 ? p.bplane + size_t(b) * 2 * H * S : nullptr;
  for (int r = threadIdx.x; r < S; r += blockDim.x) {
    float x = cf.st0[0], y = cf.st0[1], vx = cf.st0[2], vy = cf.st0[3], psi = cf.st0[4];
    float cb = 0.0f, lb = 0.0f, ub = 0.0f;
    bool nan = false;
    for (int h = 0; h < H; ++h) {
      // residual of the recorded state (x_roll[:, h] = state before step h)
      for (int o = 0; o < O; ++o) {
        const float c = f_bar(x, y, L.xo[o * H + h], L.yo[o * H + h]);
        nan |= (c != c);
        cb = fmaxf(cb, c);
      }
      const float l1 = -y + p.y_lb, u1 = y - p.y_ub;
      nan |= (y != y);
      lb = fmaxf(lb, l1);
      ub = fmaxf(ub, u1);
      if (h == H - 1) break;  // the last step's state is never recorded
      float an, sn;
      noisy_control<true>(p, cf, t, r, h, L.a[h], L.st[h], an, sn, bpl);
      bicycle_step(x, y, vx, vy, psi, an, sn);
    }
    const float qnan = __int_as_float(0x7fc00000);
    L.cbar[r] = nan ? qnan : cb;
    L.lb[r] = nan ? qnan : lb;
    L.ub[r] = nan ? qnan : ub;
  }
  __syncthreads();
  ReduceScratch& rs = *L.rs;
  float obs = 0.0f, lane = 0.0f;
  if (p.cost == 2) {  // cvar
    obs = block_cvar(L.cbar, S, L.list, rs);
    const float cl = block_cvar(L.lb, S, L.list, rs);
    const float cu = block_cvar(L.ub, S, L.list, rs);
    lane = cl + cu;
  } else if (p.cost == 3) {  // saa
    obs = float(block_count_pos(L.cbar, S, rs)) / float(S);
    const int cl = block_count_pos(L.lb, S, rs);
    const int cu = block_count_pos(L.ub, S, rs);
    lane = float(cl + cu) / float(S);
  } else {  // mmd_random: beta = 1/n, sigma = 0.01 (cem.py:355-356); lane cost zeros (cem.py:427)
    obs = block_mmd(L.cbar, nullptr, S, 0.01f, 1000.0f, rs);
    lane = 0.0f;
  }
  if (threadIdx.x == 0) {
    p.obs_cost[b] = obs;
    p.lane_cost[b] = lane;
  }
}

// Beta-noise attempt table of outer iteration t (rng.hpp): one thread per
// (stream, attempt, r, h)
__global__ __launch_bounds__(256) void k_gamma_tab(Params p, int t) {
  const int S = p.S, H = p.H;
  const int plane = S * H;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const Cfg cf = cfg_of(p, blockIdx.y);
  if (idx == 0 && blockIdx.y == 0) *p.bfix_n = 0u;  // k_beta_planes' deferred list of this iteration
  if (idx >= kGammaTabStreams * kGammaTabAttempts * plane) return;
  const int e = idx % plane, sk = idx / plane;
  const int k = sk % kGammaTabAttempts, st = sk / kGammaTabAttempts;
  const int h = e / S, r = e - h * S;
  const uint32_t k0 = iteration_key0(cf.idx_mpc, t), k1 = p.seed;
  const GammaAttempt g = gamma_attempt(k0, k1, kStreamGammaAccA + uint32_t(st), uint32_t(r) * uint32_t(H) + h, k);
  double* o = cf.gtab + (size_t(sk) * 4) * plane + e;
  o[0] = g.x;
  o[plane] = g.u;
  o[2 * size_t(plane)] = g.lu;
  const bool squeeze = g.u < 1.0 - 0.0331 * (g.x * g.x) * (g.x * g.x);  // alpha-independent (rng.hpp)
  o[3 * size_t(plane)] = squeeze ? g.lw : -g.lw;
}

// Beta draws of every (candidate, row, step) of the baseline rollouts:
// thread (r) of block (h, b); written [B][2][H][S] for k_risk_baseline, so
// the rollout kernel stays fp32 and its occupancy is not set by the fp64
// gamma sampler
__global__ __launch_bounds__(256) void k_beta_planes(Params p, int t) {
  const int S = p.S, H = p.H;
  const int r = blockIdx.x * blockDim.x + threadIdx.x, h = blockIdx.y, b = blockIdx.z;
  const double* gtab = p.gtab + size_t(b / p.B) * gtab_stride(S, H);  // this candidate's configuration
  __shared__ MtConst mc[4];
  const float a = p.acc[size_t(b) * 100 + h], st = p.steer[size_t(b) * 100 + h];
  if (threadIdx.x < 4) {  // alphas 2|a|, 5|a|, 2|s|, 5|s| of this (candidate, step)
    const float f = threadIdx.x < 2 ? fabsf(a) : fabsf(st);
    mc[threadIdx.x] = mt_const(double((threadIdx.x & 1 ? 5.0f : 2.0f) * f));
  }
  __syncthreads();
  if (r >= S) return;
  // table-only fast path; the rare rest (more than the tabulated attempts)
  // is deferred to k_beta_fix so this kernel does not carry that code's registers
  const size_t sl = size_t(kGammaTabAttempts) * 4 * S * H;
  const float fa = fabsf(a), fs = fabsf(st);
  float nba, nbs;
  const bool ok = beta_draw_fast(double(2.0f * fa), double(5.0f * fa), 2.0, 5.0, mc[0], mc[1], gtab, gtab + sl,
                                 S, H, r, h, nba) &&
                  beta_draw_fast(double(2.0f * fs), double(5.0f * fs), 2.0, 5.0, mc[2], mc[3], gtab + 2 * sl,
                                 gtab + 3 * sl, S, H, r, h, nbs);
  if (!ok) {
    const unsigned slot = atomicAdd(p.bfix_n, 1u);
    p.bfix[slot] = (uint32_t(b) * uint32_t(H) + uint32_t(h)) * uint32_t(S) + uint32_t(r);
    return;
  }
  float* o = p.bplane + size_t(b) * 2 * H * S;
  o[size_t(h) * S + r] = nba;
  o[(size_t(H) + h) * S + r] = nbs;
}

// the deferred elements of k_beta_planes, through the full sampler
__global__ __launch_bounds__(256) void k_beta_fix(Params p, int t) {
  const int S = p.S, H = p.H;
  const unsigned cnt = *p.bfix_n;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    const uint32_t e = p.bfix[i];
    const int r = int(e % uint32_t(S)), bh = int(e / uint32_t(S));
    const int h = bh % H, b = bh / H;
    float nba, nbs;
    beta_pair(p, cfg_of(p, b / p.B), t, r, h, p.acc[size_t(b) * 100 + h], p.steer[size_t(b) * 100 + h], nba, nbs);
    float* o = p.bplane + size_t(b) * 2 * H * S;
    o[size_t(h) * S + r] = nba;
    o[(size_t(H) + h) * S + r] = nbs;
  }
}

}  // namespace

void launch_beta_planes(const Params& p, int t, hipStream_t s) {
  hipLaunchKernelGGL(k_beta_planes, dim3((p.S + 255) / 256, p.H, p.Bt), dim3(256), 0, s, p, t);
  hipLaunchKernelGGL(k_beta_fix, dim3(256), dim3(256), 0, s, p, t);
}

void launch_gamma_tab(const Params& p, int t, hipStream_t s) {
  const int total = kGammaTabStreams * kGammaTabAttempts * p.S * p.H;
  hipLaunchKernelGGL(k_gamma_tab, dim3((total + 255) / 256, p.G), dim3(256), 0, s, p, t);
}

void launch_risk_baseline(const Params& p, int t, hipStream_t s) {
  const size_t lds = risk_lds_bytes(p.O, p.H, p.S);
  const int threads = p.S >= 512 ? 512 : ((p.S + 63) / 64) * 64;
  hipLaunchKernelGGL(k_risk_baseline, dim3(p.Bt), dim3(threads), lds, s, p, t);
}

}  // namespace mpcmmd
