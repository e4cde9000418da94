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
#include <algorithm>
#include <cstdlib>

#include "block.hpp"
#include "cost.hpp"
#include "draws.hpp"
#include "kernels.hpp"
#include "rng.hpp"
#include "rollout.hpp"

namespace mpcmmd {

namespace {

struct RiskLds {
  float* xo;
  float* yo;
  float* xs;  // [H][O] obstacles of each step sorted by x (k_risk_baseline's window)
  float* ys;
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
  L.xs = f;
  f += O * H;
  L.ys = f;
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
  size_t f = size_t(4 * O * H + 2 * H + 3 * S) * 4;
  f = (f + 15) & ~size_t(15);
  f += size_t(S) * 8;  // (key, index) pairs of block_cvar
  f = (f + 15) & ~size_t(15);
  return f + sizeof(ReduceScratch);
}

namespace {

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8))) void k_risk_baseline(Params p, int t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int O = p.O, H = p.H, S = p.S;
  RiskLds L = carve(smem, O, H, S);
  const int prep = select_prep_groups(p, blockDim.x);
  if (int(blockIdx.x) < prep) {  // k_select's residual sort / cost norms, beside the rollouts
    select_prep(p, t, blockIdx.x, reinterpret_cast<unsigned long long*>(smem));
    return;
  }
  const int b = blockIdx.x - prep;
  MPCMMD_STAMPW(p, 0);
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
  // each step's obstacles sorted by x (insertion sort, a thread per step);
  // a NaN obstacle coordinate keeps the full scan for the whole candidate
  constexpr int kWindowMaxObs = 64;  // above: the full scan (the sort is O^2 per step)
  bool any_nan = O > kWindowMaxObs;
  for (int h = threadIdx.x; h < H && O <= kWindowMaxObs; h += blockDim.x) {
    float* xs = L.xs + h * O;
    float* ys = L.ys + h * O;
    for (int o = 0; o < O; ++o) {
      const float xv = L.xo[o * H + h], yv = L.yo[o * H + h];
      any_nan |= (xv != xv) | (yv != yv);
      int k = o;
      while (k > 0 && xs[k - 1] > xv) {
        xs[k] = xs[k - 1];
        ys[k] = ys[k - 1];
        --k;
      }
      xs[k] = xv;
      ys[k] = yv;
    }
  }
  const bool window = !__syncthreads_or(any_nan);
  MPCMMD_STAMPW(p, 1);
  const float* bpl = p.noise == 1 ? p.bplane + size_t(b) * 2 * H * S : nullptr;
  const size_t HS = size_t(H) * S;
  for (int r = threadIdx.x; r < S; r += blockDim.x) {
    float x = cf.st0[0], y = cf.st0[1], vx = cf.st0[2], vy = cf.st0[3], psi = cf.st0[4];
    float cb = 0.0f, lb = 0.0f, ub = 0.0f;
    bool nan = false;
    // the step's three noise values (gaussian: acc / steer / const normals,
    // beta: the two Beta draws and the const normal), the next step's loads
    // issued one step ahead so the scan does not wait on L2 every step
    const float* rl = cf.roll + size_t(t) * 3 * HS + r;
    const float* n01 = p.noise == 1 ? bpl + r : rl;  // [2][H][S] planes or roll rows 0, 1
    float c0 = n01[0], c1 = n01[HS], c2 = rl[2 * HS];
    int lo_prev = 0;  // the obstacle window's start at the previous step
    for (int h = 0; h < H; ++h) {
      // residual of the recorded state (x_roll[:, h] = state before step h)
      // |x - x_o| >= a gives (x - x_o)^2 / a^2 >= 1 (monotone roundings), so
      // f_bar <= 0 cannot raise the maximum: skipped.  With the step's
      // obstacles sorted by x, fl(x - x_o) falls as x_o grows, so the ones
      // left are a contiguous run: its start by binary search, then the run
      if (window) {
        const float* xs = L.xs + h * O;
        const float* ys = L.ys + h * O;
        // lo = the first o with x - xs[o] < a (a monotone predicate), found
        // by walking from the previous step's lo: the rollout and the
        // obstacles move little per step, so usually no step is taken
        int lo = lo_prev;
        while (lo < O && !(x - xs[lo] < kObsA)) ++lo;
        while (lo > 0 && x - xs[lo - 1] < kObsA) --lo;
        lo_prev = lo;
        for (int o = lo; o < O; ++o) {
          const float xo = xs[o];
          if (fabsf(x - xo) >= kObsA) break;
          const float c = f_bar(x, y, xo, ys[o]);
          nan |= (c != c);
          cb = fmaxf(cb, c);
        }
      } else {
        for (int o = 0; o < O; ++o) {
          const float xo = L.xo[o * H + h];
          if (!(fabsf(x - xo) >= kObsA)) {
            const float c = f_bar(x, y, xo, L.yo[o * H + h]);
            nan |= (c != c);
            cb = fmaxf(cb, c);
          }
        }
      }
      const float l1 = -y + p.y_lb, u1 = y - p.y_ub;
      nan |= (y != y) | (x != x);
      lb = fmaxf(lb, l1);
      ub = fmaxf(ub, u1);
      if (h == H - 1) break;  // the last step's state is never recorded
      const size_t hn = size_t(h + 1) * S;
      const float f0 = n01[hn], f1 = n01[HS + hn], f2 = rl[2 * HS + hn];
      float an, sn;
      noisy_from(p, L.a[h], L.st[h], c0, c1, c2, an, sn);
      bicycle_step(x, y, vx, vy, psi, an, sn);
      c0 = f0, c1 = f1, c2 = f2;
    }
    const float qnan = __int_as_float(0x7fc00000);
    L.cbar[r] = nan ? qnan : cb;
    L.lb[r] = nan ? qnan : lb;
    L.ub[r] = nan ? qnan : ub;
  }
  __syncthreads();
  MPCMMD_STAMPW(p, 2);
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
  MPCMMD_STAMPW(p, 3);
}

// Beta-noise attempt table of outer iteration t (rng.hpp): one thread per
// (stream, attempt, r, h) of configuration blockIdx.y (draws.hpp)
__global__ __launch_bounds__(256) void k_gamma_tab(Params p, int t) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < gamma_items(p)) gamma_item(p, t, cfg_of(p, blockIdx.y), idx);
}

// Beta draws of every (candidate, row, step) of the baseline rollouts,
// written [B][2][H][S] for k_risk_baseline (the rollout kernel stays fp32 and
// its occupancy is not set by the fp64 gamma sampler).  The attempt table
// depends only on (row r, step h) (Q2): a workgroup stages attempt 0 of the
// four gammas for 64 rows of one step in LDS once and applies it to
// kBetaCands candidates of one configuration (wave w takes candidates w, w +
// 4, ...; lane = row), so the table is read from L2 once per 16 candidates
// instead of once per candidate.  The rarely needed attempts 1-3 come from
// the table in global memory; more than that goes to k_beta_fix.
constexpr int kBetaCands = 16;
constexpr int kBetaRows = 64;

__global__ __launch_bounds__(256) void k_beta_planes(Params p, int t) {
  const int S = p.S, H = p.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * kBetaRows + lane, h = blockIdx.y;
  const int groups = (p.B + kBetaCands - 1) / kBetaCands;
  const int g = blockIdx.z / groups, j0 = (blockIdx.z - g * groups) * kBetaCands;  // configuration, first candidate
  const int nc = min(kBetaCands, p.B - j0);
  const double* gtab_ = p.gtab + size_t(g) * gtab_stride(S, H);
  const size_t plane = size_t(S) * H, at = size_t(h) * S + r, sl = size_t(kGammaTabAttempts) * 4 * plane;
  __shared__ double tx[4][kBetaRows], tlu[4][kBetaRows], tlw[4][kBetaRows];
  __shared__ MtConst mc[kBetaCands][4];
  __shared__ float fab[kBetaCands][2];
  {  // wave w stages gamma stream w (acc A, acc B, steer A, steer B)
    const double* tw = gtab_ + w * sl + size_t(h) * S + min(r, S - 1);
    tx[w][lane] = tw[0];
    tlu[w][lane] = tw[2 * plane];
    tlw[w][lane] = tw[3 * plane];
  }
  if (threadIdx.x < 4 * kBetaCands) {  // alphas 2|a|, 5|a|, 2|s|, 5|s| of each candidate at this step
    const int c = threadIdx.x >> 2, i = threadIdx.x & 3;
    const size_t b = size_t(g) * p.B + j0 + min(c, nc - 1);
    const float f = fabsf(i < 2 ? p.acc[b * 100 + h] : p.steer[b * 100 + h]);
    mc[c][i] = mt_const(double((i & 1 ? 5.0f : 2.0f) * f));
    if ((i & 1) == 0) fab[c][i >> 1] = f;
  }
  __syncthreads();
  if (r >= S) return;
  // one gamma pair (streams k, k + 1: acc or steer) of candidate c -> its Beta draw
  auto draw = [&](int c, int k, float f, float& out) {
    double ga, ua, gb, ub;
    // the fallback's table pointer laundered per call: its (loop-invariant)
    // loads must not be hoisted out of the candidate loop (72 registers)
    const double* gtab = gtab_;
    __asm__ volatile("" : "+s"(gtab));
    const bool ok = (tab_try(mc[c][k], TabAtt{tx[k][lane], tlu[k][lane], tlw[k][lane]}, ga, ua) ||
                     gamma_tab_from(mc[c][k], gtab + k * sl, plane, at, 1, ga, ua)) &&
                    (tab_try(mc[c][k + 1], TabAtt{tx[k + 1][lane], tlu[k + 1][lane], tlw[k + 1][lane]}, gb, ub) ||
                     gamma_tab_from(mc[c][k + 1], gtab + (k + 1) * sl, plane, at, 1, gb, ub));
    if (ok) out = beta_combine(double(2.0f * f), double(5.0f * f), 2.0, 5.0, ga, ua, gb, ub);
    return ok;
  };
#pragma unroll 1
  for (int c = w; c < nc; c += 4) {
    const uint32_t b = uint32_t(g) * p.B + j0 + c;
    float* o = p.bplane + size_t(b) * 2 * H * S;
    float nba, nbs;
    if (draw(c, 0, fab[c][0], nba) && draw(c, 2, fab[c][1], nbs)) {
      o[size_t(h) * S + r] = nba;
      o[(size_t(H) + h) * S + r] = nbs;
    } else {  // more attempts than tabulated (rare): the full sampler in k_beta_fix
      const unsigned slot = atomicAdd(p.bfix_n, 1u);
      p.bfix[slot] = (b * uint32_t(H) + uint32_t(h)) * uint32_t(S) + uint32_t(r);
    }
  }
}

// mt_log_test's fp32 test on v = vp, the common path's fp32 v to within two
// ulp (v_precise): an error e <= 2.4e-7 relative in v moves rhs = q + d - d v^3
// + d ln v^3 by at most 3 e (d v^3 + d) + fp32 rounding of the terms, far inside
// the test's band 1e-5 (1 + |lu| + q + d + d v^3 + |d ln v^3|), so a decided
// result is the exact fp64 decision.  +1 accept, 0 reject, -1 undecided (the
// caller takes the exact path).
DEVI int mt_log_test_vf(float xf, float luf, float df, float vp) {
  const float v3f = vp * vp * vp;
  const float q = 0.5f * xf * xf, dv = df * v3f, dl = df * (3.0f * __builtin_amdgcn_logf(vp) * 0.693147180559945309f);
  const float rhs = ((q + df) - dv) + dl;
  const float tol = 1e-5f * (1.0f + fabsf(luf) + q + fabsf(df) + fabsf(dv) + fabsf(dl));
  if (luf < rhs - tol) return 1;
  if (luf > rhs + tol) return 0;
  return -1;
}

// v = 1 + c x to within two fp32 ulp for any v >> 1e-13, from the fp32 pairs
// c = c + clo, x = xf + xlo (the fp64 values split): c xf = ph + pl exactly
// (fma), 1 + ph = s + e1 exactly (two-sum); the small terms added once.
DEVI float v_precise(float c, float clo, float xf, float xlo) {
  const float ph = c * xf;
  const float pl = fmaf(c, xf, -ph);
  const float s = 1.0f + ph;
  const float bb = s - 1.0f;
  const float e1 = (1.0f - (s - bb)) + (ph - bb);
  return s + (e1 + (pl + (c * xlo + clo * xf)));
}

// attempt 0 of one gamma stream at (row, step), staged in LDS: x as an fp32
// pair and log u in fp32 (the common path's operands), +-log w in fp64 (the
// boost log-uniform)
struct Tab0 {
  float xf, xlo, luf;
  double lw;
};
DEVI Tab0 tab0_of(const double* e, size_t plane) {
  const double x = e[0];
  const float xf = float(x);
  return Tab0{xf, float(x - double(xf)), float(e[2 * plane]), e[3 * plane]};
}

// One gamma by the fp32 common path: attempt 0 from LDS, attempts 1.. from
// the table in global memory (wave-uniform entries); c, clo: the fp32 pair of
// the gamma's c.  v = 1 + c x is formed in plain fp32 first; where the squeeze
// rejected (the log test follows) or v < 0.5 (log2 v carries into the draw),
// v_precise replaces it.  |v| <= 1e-5 (its sign in doubt), a log test inside
// its band, or more attempts than tabulated: false -- the caller takes the
// exact path.
DEVI bool gamma_fast(float c, float clo, float l2d, float df, const Tab0& e0, const double* tab, size_t plane,
                     float& lg, double& lub) {
  Tab0 e = e0;
  for (int a = 0;;) {
    const float vf = 1.0f + c * e.xf;
    int dec;  // 1 accept, 0 reject, -1 undecided
    float v = vf;
    if (!(fabsf(vf) > 1e-5f)) {
      dec = -1;
    } else if (!(vf > 0.0f)) {
      dec = 0;
    } else {
      if (!(e.lw < 0.0) || vf < 0.5f) v = v_precise(c, clo, e.xf, e.xlo);
      dec = e.lw < 0.0 ? 1 : mt_log_test_vf(e.xf, e.luf, df, v);  // lw < 0: the squeeze accepted
    }
    if (dec == 1) {
      lg = l2d + 3.0f * __builtin_amdgcn_logf(v);
      lub = -fabs(e.lw);
      return true;
    }
    if (dec < 0 || ++a == kGammaTabAttempts) return false;
    e = tab0_of(tab + size_t(a) * 4 * plane, plane);
  }
}

constexpr int kBpRows = 32;   // rows per k_beta_planes_c chunk (8 per wave)
constexpr int kBpChunks = 1;  // chunks per workgroup (more measured slower: 2 -> +10%, 4 -> +25%)

// Beta(a, b) = 1 / (1 + 2^(log2 Gb - log2 Ga)) from the gammas' log2 G' and
// boost log-uniforms (beta_combine's formula, the log2 G' given).
DEVI float beta_from_logs(double a, double b, double ra, double rb, float lga, double ua, float lgb, double ub) {
  if (a == 0.0 && b == 0.0) return (ua * rb > ub * ra) ? 1.0f : 0.0f;
  const bool ka = a < 1.0, kb = b < 1.0;
  float e = 0.0f;
  if (ka || kb) {
    const double fa = ka ? a : 1.0, fb = kb ? b : 1.0;
    e = float(((kb ? ub : 0.0) * fa - (ka ? ua : 0.0) * fb) * __builtin_amdgcn_rcp(fa * fb));
  }
  const float d = (lgb - lga) + 1.44269504088896340736f * e;
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(d));
}

// The same draws with one lane per CANDIDATE (64 candidates of one
// configuration) and a wave walking 8 rows of one step: the attempt-table
// entry of a (row, step) is one value for the whole wave, so the
// alpha-independent squeeze decision -- which decides whether the log test
// runs at all -- is wave-uniform (row lanes would take the rare paths whenever
// any of their 64 rows does).  Attempt 0 of the workgroup's rows is staged in
// LDS (one coalesced pass); every gamma runs the fp32 common path (gamma_fast,
// later attempts from global memory); an element it cannot decide (about 4
// in 10^4) goes to k_beta_fix, the full fp64 sampler.  The [32 rows][64
// candidates] result tile goes through LDS so the planes are stored as
// 128-byte row runs per candidate.
__global__ __launch_bounds__(256) void k_beta_planes_c(Params p, int t) {
  const int S = p.S, H = p.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = blockIdx.y;
  const int groups = (p.B + 63) / 64;
  const int g = blockIdx.z / groups, j0 = (blockIdx.z - g * groups) * 64;
  const int nc = min(64, p.B - j0);
  const double* gt = p.gtab + size_t(g) * gtab_stride(S, H);
  const size_t plane = size_t(S) * H, sl = size_t(kGammaTabAttempts) * 4 * plane;
  __shared__ Tab0 t0[4][kBpRows];
  __shared__ float tile[2][kBpRows][65];
  const int c = min(lane, nc - 1);
  const uint32_t b = uint32_t(g) * p.B + j0 + c;
  const float fa = fabsf(p.acc[size_t(b) * 100 + h]), fs = fabsf(p.steer[size_t(b) * 100 + h]);
  const double aa = double(2.0f * fa), ab = double(5.0f * fa), sa = double(2.0f * fs), sb = double(5.0f * fs);
  const double al[4] = {aa, ab, sa, sb};
  float cv[4], cl[4], lv[4], dv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // the gammas' constants (k_mt_tab's), once for the workgroup's chunks
    const MtConst m = mt_const(al[k]);
    cv[k] = float(m.c);
    cl[k] = float(m.c - double(cv[k]));
    lv[k] = __builtin_amdgcn_logf(float(m.d));
    dv[k] = float(m.d);
  }
  // kBpChunks chunks of kBpRows rows, one after another through the same LDS
  for (int ch = 0; ch < kBpChunks; ++ch) {
    const int r0 = (blockIdx.x * kBpChunks + ch) * kBpRows;
    if (r0 >= S) break;  // workgroup-uniform
    const int nr = min(kBpRows, S - r0);
    if (ch > 0) __syncthreads();  // the previous chunk's tile and table reads are done
    for (int q = threadIdx.x; q < 4 * kBpRows; q += blockDim.x) {  // attempt 0, streams acc A/B, steer A/B
      const int k = q / kBpRows, rl = q - k * kBpRows;
      const double* e = gt + k * sl + size_t(h) * S + r0 + min(rl, nr - 1);
      t0[k][rl] = tab0_of(e, plane);
    }
    __syncthreads();
    for (int i = 0; i < kBpRows / 4; ++i) {
      const int rl = w * (kBpRows / 4) + i, r = r0 + rl;
      if (rl >= nr) break;
      const double* e = gt + size_t(h) * S + r;
      float lg[4];
      double ug[4];
      int ok = 1;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        ok &= int(gamma_fast(cv[k], cl[k], lv[k], dv[k], t0[k][rl], e + k * sl, plane, lg[k], ug[k]));
      if (ok) {
        tile[0][rl][lane] = beta_from_logs(aa, ab, 2.0, 5.0, lg[0], ug[0], lg[1], ug[1]);
        tile[1][rl][lane] = beta_from_logs(sa, sb, 2.0, 5.0, lg[2], ug[2], lg[3], ug[3]);
      } else if (lane < nc) {  // undecided in fp32 or more attempts than tabulated: k_beta_fix writes it
        const unsigned slot = atomicAdd(p.bfix_n, 1u);
        p.bfix[slot] = (b * uint32_t(H) + uint32_t(h)) * uint32_t(S) + uint32_t(r);
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nc * 2 * kBpRows; q += blockDim.x) {
      const int rl = q & (kBpRows - 1), kc = q / kBpRows, k = kc & 1, cl2 = kc >> 1;
      if (rl >= nr) continue;
      p.bplane[(size_t(g) * p.B + j0 + cl2) * 2 * H * S + (size_t(k) * H + h) * S + r0 + rl] = tile[k][rl][cl2];
    }
  }
}

// ---------------------------------------------------------------------------
// Fused baseline risk with one lane per CANDIDATE (cvar / saa / mmd_random;
// both noise models).  A wave runs one noise row r for 64 candidates of one
// configuration, so everything indexed by (row, step) -- the Gaussian normals
// and, for Beta noise, the attempt-table entries of the four gamma streams
// (cem_helper.py:405-443: one realisation shared by every candidate, Q2) --
// is one value per wave, and the Beta draws are made inside the rollout: no
// [B][2][H][S] planes are written or read.  The alpha-independent squeeze
// decision being wave-uniform, the log test and the later attempts run only
// where their (row, step) needs them.  The per-(candidate, step) gamma
// constants come from k_mt_tab.  Rollout, collision residual and lane bars
// are k_risk_baseline's arithmetic; the per-row maxima go to Params::rbar and
// k_risk_reduce applies the reducer (one workgroup per candidate).
struct MtTab {
  float4 c;      // c = 1 / sqrt(9 d) of the four gammas (acc a, acc b, steer a, steer b)
  float4 l2d;    // log2 d
  float4 d;      // d = alpha' - 1/3 (fp32 of the fp64 value)
  float4 ctl;    // the controls: acc, steer (and two spare)
  float4 clo;    // c - float(c) (the fp32 pair of c, v_precise)
  double4 rinv;  // 1 / alpha where alpha < 1 (the boost), else 0: acc a, acc b, steer a, steer b
};
static_assert(sizeof(MtTab) == 128, "MtTab: 5 float4 + double4 (32-byte aligned)");
// followed in Params::mttab by [H][Bt] double4: the fp64 c of the four gammas
// (the exact v = 1 + c x of the rare paths)

__global__ __launch_bounds__(256) void k_mt_tab(Params p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (h, b): b fastest
  if (i >= p.Bt * p.H) return;
  const int h = i / p.Bt, b = i - h * p.Bt;
  const float ac = p.acc[size_t(b) * 100 + h], sc = p.steer[size_t(b) * 100 + h];
  const float fa = fabsf(ac), fs = fabsf(sc);
  const double al[4] = {double(2.0f * fa), double(5.0f * fa), double(2.0f * fs), double(5.0f * fs)};
  float c[4], l[4], d[4], cl[4];
  double r[4], c64[4];
  for (int k = 0; k < 4; ++k) {
    const MtConst m = mt_const(al[k]);
    c[k] = float(m.c);
    cl[k] = float(m.c - double(c[k]));
    l[k] = __builtin_amdgcn_logf(float(m.d));
    d[k] = float(m.d);
    r[k] = al[k] < 1.0 ? 1.0 / al[k] : 0.0;
    c64[k] = m.c;
  }
  MtTab* o = reinterpret_cast<MtTab*>(p.mttab) + i;
  o->c = make_float4(c[0], c[1], c[2], c[3]);
  o->l2d = make_float4(l[0], l[1], l[2], l[3]);
  o->d = make_float4(d[0], d[1], d[2], d[3]);
  o->ctl = make_float4(ac, sc, 0.0f, 0.0f);
  o->clo = make_float4(cl[0], cl[1], cl[2], cl[3]);
  o->rinv = double4{r[0], r[1], r[2], r[3]};
  reinterpret_cast<double4*>(reinterpret_cast<MtTab*>(p.mttab) + size_t(p.Bt) * p.H)[i] =
      double4{c64[0], c64[1], c64[2], c64[3]};
}

// One Marsaglia-Tsang attempt from a (wave-uniform) table entry (x, log u,
// +-log w): v = 1 + c x in fp32 decides v > 0 unless it is within 1e-5 of 0
// (then the fp64 v); the squeeze decision is the stored sign of log w; the log
// test is mt_log_test on the fp64 v^3 (fp32 test, fp64 re-check).  The same
// decisions as gamma_parts_tab's fp64 tab_try.  c64: the lane's fp64 c, loaded
// only on those rare paths.  Returns log2 G' = log2 d + 3 log2 v and the boost
// log-uniform when accepted.
DEVI bool mt_try(float c, float l2d, double d, const double* c64, double x, double lu, double lw, float& lg,
                 double& lub) {
  const float vf = 1.0f + c * float(x);
  float v = vf;
  if (!(fabsf(vf) > 1e-5f)) {
    const double vd = 1.0 + *c64 * x;
    if (!(vd > 0.0)) return false;
    v = float(vd);
    if (!(lw < 0.0) && !mt_log_test(x, lu, d, vd * vd * vd)) return false;
  } else {
    if (!(vf > 0.0f)) return false;
    if (!(lw < 0.0)) {  // the squeeze rejected (wave-uniform): the exact log test
      const double vd = 1.0 + *c64 * x;
      if (!mt_log_test(x, lu, d, vd * vd * vd)) return false;
    }
  }
  lg = l2d + 3.0f * __builtin_amdgcn_logf(v);
  lub = -fabs(lw);
  return true;
}

// One gamma by the exact path: the table's attempts from 0 (mt_try, the
// exact decisions), then the full fp64 sampler for longer chains (about one
// gamma in 10^6).  tab: this stream's table at (attempt 0, h, r).
DEVI void gamma_exact(float c, float l2d, double alpha, const double* c64, const double* tab, size_t plane, int S,
                      int H, int r, int h, uint32_t k0, uint32_t k1, uint32_t stream, float& lg, double& lub) {
  const double d = (alpha < 1.0 ? alpha + 1.0 : alpha) - 1.0 / 3.0;  // mt_const's d
#pragma unroll 1
  for (int a = 0; a < kGammaTabAttempts; ++a) {
    const double* e = tab + size_t(a) * 4 * plane;
    if (mt_try(c, l2d, d, c64, e[0], e[2 * plane], e[3 * plane], lg, lub)) return;
  }
  const size_t at = size_t(h) * S + r;
  double gg;
  gamma_parts_tab(mt_const(alpha), tab - at, S, H, r, h, k0, k1, stream, uint32_t(r) * uint32_t(H) + uint32_t(h), gg,
                  lub);
  lg = __builtin_amdgcn_logf(float(gg));
}

DEVI float beta_fused(float fabs_ctl, double ra, double rb, float lga, double ua, float lgb, double ub) {
  if (fabs_ctl == 0.0f) return (ua * 5.0 > ub * 2.0) ? 1.0f : 0.0f;  // Beta(0, 0): the alpha -> 0+ limit
  const float e = (ra != 0.0 || rb != 0.0) ? float(ub * rb - ua * ra) : 0.0f;
  const float d = (lgb - lga) + 1.44269504088896340736f * e;
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(d));
}

typedef float f2v __attribute__((ext_vector_type(2)));

// f_bar (compute_f_bar, costs.py:50-60) of two obstacles at once in packed
// fp32 (v_pk_*: the same IEEE roundings as f_bar, two lanes per instruction)
DEVI f2v f_bar2(float x, float y, f2v xo, f2v yo) {
  constexpr float kA2 = 18.0625f, kB2 = 7.5625f;
  const f2v wc = f2v{x, x} - xo, ws = f2v{y, y} - yo;
  const f2v a = wc * wc, b = ws * ws;
  const f2v ra = f2v{1.0f / kA2, 1.0f / kA2}, rb = f2v{1.0f / kB2, 1.0f / kB2};
  const f2v qa = a * ra, qb = b * rb;  // div_rc(x, d, r): q + (x - q d) r
  const f2v ea = __builtin_elementwise_fma(-qa, f2v{kA2, kA2}, a), eb = __builtin_elementwise_fma(-qb, f2v{kB2, kB2}, b);
  const f2v da = __builtin_elementwise_fma(ea, ra, qa), db = __builtin_elementwise_fma(eb, rb, qb);
  return (-da - db) + f2v{1.0f, 1.0f};
}

constexpr int kRcWaves = 4;

// Fused baseline rollouts (see above): per step the four gammas by the fp32
// common path (gamma_fast; attempt 0 staged in LDS), a gamma it cannot
// decide by the exact path (gamma_exact), the Beta draws, then the rollout
// step; nothing but the per-row maxima leaves the kernel.
__global__ __launch_bounds__(64 * kRcWaves) void k_roll_cand(Params p, int t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int S = p.S, H = p.H, O = p.O, Op = (O + 1) & ~1;  // obstacles padded to pairs
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int groups = (p.B + 63) / 64;
  const int g = blockIdx.y / groups, j0 = (blockIdx.y - g * groups) * 64;
  const int nc = min(64, p.B - j0);
  const int r0 = blockIdx.x * kRcWaves, nr = min(kRcWaves, S - r0);
  const Cfg cf = cfg_of(p, g);
  const bool beta = p.noise == 1;
  const size_t HS = size_t(H) * S;
  const size_t plane = HS, sl = size_t(kGammaTabAttempts) * 4 * plane;
  f2v* ob = reinterpret_cast<f2v*>(smem);                  // [H][Op/2] x pairs, then y pairs
  Tab0* t0 = reinterpret_cast<Tab0*>(ob + H * Op);         // [kRcWaves][H][4 streams]
  for (int i = threadIdx.x; i < Op * H; i += blockDim.x) {  // transpose [O][H] -> [H][O]; a pad repeats obstacle 0
    const int h = i / Op, o = i - h * Op, os = o < O ? o : 0;
    reinterpret_cast<float*>(ob)[i] = cf.obs[os * H + h];
    reinterpret_cast<float*>(ob + (H * Op) / 2)[i] = cf.obs[O * H + os * H + h];
  }
  if (beta) {
    for (int i = threadIdx.x; i < kRcWaves * H * 4; i += blockDim.x) {  // (row, step, stream), stream fastest
      const int k = i & 3, wh = i >> 2, rw = wh / H, h = wh - rw * H;
      const double* e = cf.gtab + k * sl + size_t(h) * S + r0 + min(rw, nr - 1);
      t0[i] = tab0_of(e, plane);
    }
  }
  __syncthreads();
  const int r = r0 + w;
  if (w >= nr) return;
  const int c = min(lane, nc - 1);
  const size_t b = size_t(g) * p.B + j0 + c;
  const float* rl = cf.roll + size_t(t) * 3 * HS + r;  // [3][H][S]: uniform per wave
  const double* gt = beta ? cf.gtab + size_t(r) : nullptr;  // + h S + k sl + a 4 plane + field plane
  const uint32_t k0 = iteration_key0(cf.idx_mpc, t), k1 = p.seed;
  const MtTab* mt = reinterpret_cast<const MtTab*>(p.mttab);
  const double* mc64 = reinterpret_cast<const double*>(mt + size_t(p.Bt) * H);
  const Tab0* tw = t0 + w * H * 4;
  const f2v* obx = ob;
  const f2v* oby = ob + (H * Op) / 2;
  const int Op2 = Op / 2;
  float x = cf.st0[0], y = cf.st0[1], vx = cf.st0[2], vy = cf.st0[3], psi = cf.st0[4];
  float cb = 0.0f, lb = 0.0f, ub = 0.0f;
  f2v nsum = f2v{0.0f, 0.0f};  // sum of every f_bar: NaN iff one is (f_bar <= 1, never +inf)
  bool nan = false;
  for (int h = 0; h < H; ++h) {
    for (int o = 0; o < Op2; ++o) {  // k_risk_baseline's residual max over the obstacles, two at a time
      const f2v cc = f_bar2(x, y, obx[h * Op2 + o], oby[h * Op2 + o]);
      nsum += cc;
      cb = fmaxf(cb, fmaxf(cc.x, cc.y));
    }
    const float l1 = -y + p.y_lb, u1 = y - p.y_ub;
    nan |= (y != y) | (x != x);
    lb = fmaxf(lb, l1);
    ub = fmaxf(ub, u1);
    if (h == H - 1 && !p.beta_dump) break;  // the last step's draw moves nothing (dumped for the tests only)
    const float nc2 = rl[2 * HS + size_t(h) * S];
    float a, st, n0, n1;
    if (!beta) {
      a = p.acc[b * 100 + h];
      st = p.steer[b * 100 + h];
      n0 = rl[size_t(h) * S];
      n1 = rl[HS + size_t(h) * S];
    } else {
      const size_t hb = size_t(h) * p.Bt + b;
      const MtTab m = mt[hb];
      a = m.ctl.x;
      st = m.ctl.y;
      const double* e = gt + size_t(h) * S;
      const float cv[4] = {m.c.x, m.c.y, m.c.z, m.c.w}, lv[4] = {m.l2d.x, m.l2d.y, m.l2d.z, m.l2d.w};
      const float dv[4] = {m.d.x, m.d.y, m.d.z, m.d.w}, clv[4] = {m.clo.x, m.clo.y, m.clo.z, m.clo.w};
      float lg[4];
      double ug[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // the fp32 common path, else the exact path
        if (!gamma_fast(cv[k], clv[k], lv[k], dv[k], tw[h * 4 + k], e + k * sl, plane, lg[k], ug[k])) {
          const double alpha = double(((k & 1) ? 5.0f : 2.0f) * fabsf(k < 2 ? a : st));
          const uint32_t stream = k == 0 ? kStreamGammaAccA : k == 1 ? kStreamGammaAccB : k == 2 ? kStreamGammaSteerA
                                                                                                 : kStreamGammaSteerB;
          gamma_exact(cv[k], lv[k], alpha, mc64 + 4 * hb + k, e + k * sl, plane, S, H, r, h, k0, k1, stream, lg[k],
                      ug[k]);
        }
      }
      n0 = beta_fused(fabsf(a), m.rinv.x, m.rinv.y, lg[0], ug[0], lg[1], ug[1]);
      n1 = beta_fused(fabsf(st), m.rinv.z, m.rinv.w, lg[2], ug[2], lg[3], ug[3]);
      if (p.beta_dump && lane < nc) {  // parity tests: the draws as the [B][2][H][S] planes
        p.bplane[b * 2 * HS + size_t(h) * S + r] = n0;
        p.bplane[b * 2 * HS + HS + size_t(h) * S + r] = n1;
      }
    }
    if (h == H - 1) break;
    float an, sn;
    noisy_from(p, a, st, n0, n1, nc2, an, sn);
    bicycle_step(x, y, vx, vy, psi, an, sn);
  }
  nan |= (nsum.x != nsum.x) | (nsum.y != nsum.y);
  if (lane < nc) {
    const float qnan = __int_as_float(0x7fc00000);
    const size_t bs = size_t(p.Bt) * S;
    p.rbar[b * S + r] = nan ? qnan : cb;
    p.rbar[bs + b * S + r] = nan ? qnan : lb;
    p.rbar[2 * bs + b * S + r] = nan ? qnan : ub;
  }
}

// the reducers of k_risk_baseline over the per-row maxima of k_roll_cand
__global__ __launch_bounds__(512) void k_risk_reduce(Params p, int t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int S = p.S, b = blockIdx.x;
  RiskLds L = carve(smem, p.O, p.H, S);
  const size_t bs = size_t(p.Bt) * S;
  for (int r = threadIdx.x; r < S; r += blockDim.x) {
    L.cbar[r] = p.rbar[size_t(b) * S + r];
    L.lb[r] = p.rbar[bs + size_t(b) * S + r];
    L.ub[r] = p.rbar[2 * bs + size_t(b) * S + r];
  }
  __syncthreads();
  ReduceScratch& rs = *L.rs;
  float obs = 0.0f, lane = 0.0f;
  if (p.cost == 2) {
    obs = block_cvar(L.cbar, S, L.list, rs);
    const float cl = block_cvar(L.lb, S, L.list, rs);
    const float cu = block_cvar(L.ub, S, L.list, rs);
    lane = cl + cu;
  } else if (p.cost == 3) {
    obs = float(block_count_pos(L.cbar, S, rs)) / float(S);
    const int cl = block_count_pos(L.lb, S, rs);
    const int cu = block_count_pos(L.ub, S, rs);
    lane = float(cl + cu) / float(S);
  } else {
    obs = block_mmd(L.cbar, nullptr, S, 0.01f, 1000.0f, rs);
    lane = 0.0f;
  }
  if (threadIdx.x == 0) {
    p.obs_cost[b] = obs;
    p.lane_cost[b] = lane;
  }
}

// the deferred elements of k_beta_planes, through the full sampler
// a quad per element: lane k of the quad runs gamma k (acc a, acc b, steer a,
// steer b) through the full sampler (gamma_parts_tab, as beta_pair), lanes 0
// and 2 combine their pair (beta_combine): beta_pair's bits, a quarter of
// its serial chain (the launch's time is one element's latency)
__global__ __launch_bounds__(256) void k_beta_fix(Params p, int t) {
  const int S = p.S, H = p.H;
  const unsigned cnt = *p.bfix_n;
  const int lane = threadIdx.x & 63, k = lane & 3, q0 = lane & ~3;
  const size_t sl = size_t(kGammaTabAttempts) * 4 * S * H;  // one stream's table
  const uint32_t streams[4] = {kStreamGammaAccA, kStreamGammaAccB, kStreamGammaSteerA, kStreamGammaSteerB};
  for (unsigned gi = blockIdx.x * blockDim.x + threadIdx.x; gi < 4 * cnt; gi += gridDim.x * blockDim.x) {
    const uint32_t e = p.bfix[gi >> 2];
    const int r = int(e % uint32_t(S)), bh = int(e / uint32_t(S));
    const int h = bh % H, b = bh / H;
    const Cfg cf = cfg_of(p, b / p.B);
    const float fa = fabsf(p.acc[size_t(b) * 100 + h]), fs = fabsf(p.steer[size_t(b) * 100 + h]);
    const double al[4] = {double(2.0f * fa), double(5.0f * fa), double(2.0f * fs), double(5.0f * fs)};
    const double alpha = k == 0 ? al[0] : k == 1 ? al[1] : k == 2 ? al[2] : al[3];
    const uint32_t stream = k == 0 ? streams[0] : k == 1 ? streams[1] : k == 2 ? streams[2] : streams[3];
    double g, u;
    gamma_parts_tab(mt_const(alpha), cf.gtab + size_t(k) * sl, S, H, r, h, iteration_key0(cf.idx_mpc, t), p.seed,
                    stream, uint32_t(r) * uint32_t(H) + uint32_t(h), g, u);
    const double g1 = __shfl(g, q0 + (k | 1), 64), u1 = __shfl(u, q0 + (k | 1), 64);  // the pair's b gamma
    if ((k & 1) == 0) {
      const double a = k == 0 ? al[0] : al[2], bb = k == 0 ? al[1] : al[3];
      const float v = beta_combine(a, bb, 2.0, 5.0, g, u, g1, u1);
      p.bplane[size_t(b) * 2 * H * S + (size_t(k == 0 ? 0 : H) + h) * S + r] = v;
    }
  }
}

// The CARLA variant's planes: every element through the full sampler (as
// k_beta_fix, a quad per element) and the fp64 combine (beta_combine_cr)
__global__ __launch_bounds__(256) void k_beta_planes_cr(Params p, int t, unsigned total) {
  const int S = p.S, H = p.H;
  const int lane = threadIdx.x & 63, k = lane & 3, q0 = lane & ~3;
  const size_t sl = size_t(kGammaTabAttempts) * 4 * S * H;
  const uint32_t streams[4] = {kStreamGammaAccA, kStreamGammaAccB, kStreamGammaSteerA, kStreamGammaSteerB};
  const unsigned gi = blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= 4 * total) return;  // whole quads
  const unsigned e = gi >> 2;
  const int r = int(e % unsigned(S)), bh = int(e / unsigned(S));
  const int h = bh % H, b = bh / H;
  const Cfg cf = cfg_of(p, b / p.B);
  const float fa = fabsf(p.acc[size_t(b) * 100 + h]), fs = fabsf(p.steer[size_t(b) * 100 + h]);
  const double al[4] = {double(2.0f * fa), double(5.0f * fa), double(2.0f * fs), double(5.0f * fs)};
  const double alpha = k == 0 ? al[0] : k == 1 ? al[1] : k == 2 ? al[2] : al[3];
  const uint32_t stream = k == 0 ? streams[0] : k == 1 ? streams[1] : k == 2 ? streams[2] : streams[3];
  double g, u;
  gamma_parts_tab(mt_const(alpha), cf.gtab + size_t(k) * sl, S, H, r, h, iteration_key0(cf.idx_mpc, t), p.seed, stream,
                  uint32_t(r) * uint32_t(H) + uint32_t(h), g, u);
  const double g1 = __shfl(g, q0 + (k | 1), 64), u1 = __shfl(u, q0 + (k | 1), 64);  // the pair's b gamma
  if ((k & 1) == 0) {
    const double a = k == 0 ? al[0] : al[2], bb = k == 0 ? al[1] : al[3];
    p.bplane[size_t(b) * 2 * H * S + (size_t(k == 0 ? 0 : H) + h) * S + r] = beta_combine_cr(a, bb, 2.0, 5.0, g, u, g1, u1);
  }
}

}  // namespace

void launch_beta_planes(const Params& p, int t, hipStream_t s) {
  if (p.carla) {
    const unsigned total = unsigned(p.Bt) * p.H * p.S;
    hipLaunchKernelGGL(k_beta_planes_cr, dim3((4 * total + 255) / 256), dim3(256), 0, s, p, t, total);
    return;
  }
  static const bool rows = [] {  // MPCMMD_BETA_ROWS=1: the row-lane kernel (A/B)
    const char* e = std::getenv("MPCMMD_BETA_ROWS");
    return e && std::atoi(e) != 0;
  }();
  if (rows) {
    const int groups = (p.B + kBetaCands - 1) / kBetaCands;
    hipLaunchKernelGGL(k_beta_planes, dim3((p.S + kBetaRows - 1) / kBetaRows, p.H, p.G * groups), dim3(256), 0, s, p,
                       t);
  } else {
    const int groups = (p.B + 63) / 64;
    // the last step's draws move nothing (k_risk_baseline never applies them):
    // not drawn, except for the parity tests' plane dump
    hipLaunchKernelGGL(k_beta_planes_c,
                       dim3((p.S + kBpRows * kBpChunks - 1) / (kBpRows * kBpChunks), p.beta_dump ? p.H : p.H - 1,
                            p.G * groups),
                       dim3(256), 0, s, p, t);
  }
  hipLaunchKernelGGL(k_beta_fix, dim3(1024), dim3(256), 0, s, p, t);
}

void launch_gamma_tab(const Params& p, int t, hipStream_t s) {
  const int total = gamma_items(p);
  hipLaunchKernelGGL(k_gamma_tab, dim3((total + 255) / 256, p.G), dim3(256), 0, s, p, t);
}

size_t mt_tab_entry_bytes() { return sizeof(MtTab) + sizeof(double4); }

void launch_risk_fused(const Params& p, int t, hipStream_t s) {
  if (p.noise == 1)
    hipLaunchKernelGGL(k_mt_tab, dim3((p.Bt * p.H + 255) / 256), dim3(256), 0, s, p);
  const int groups = (p.B + 63) / 64;
  const size_t lds = size_t(2 * ((p.O + 1) & ~1) * p.H) * 4 + (p.noise == 1 ? sizeof(Tab0) * kRcWaves * p.H * 4 : 0);
  hipLaunchKernelGGL(k_roll_cand, dim3((p.S + kRcWaves - 1) / kRcWaves, p.G * groups), dim3(64 * kRcWaves), lds, s,
                     p, t);
  const int threads = p.S >= 512 ? 512 : ((p.S + 63) / 64) * 64;
  hipLaunchKernelGGL(k_risk_reduce, dim3(p.Bt), dim3(threads), risk_lds_bytes(p.O, p.H, p.S), s, p, t);
}

void launch_risk_baseline(const Params& p, int t, hipStream_t s) {
  const int threads = p.S >= 512 ? 512 : ((p.S + 63) / 64) * 64;
  const int prep = select_prep_groups(p, threads);
  size_t n2 = 1;
  while (n2 < size_t(p.B)) n2 <<= 1;
  const size_t lds = std::max(risk_lds_bytes(p.O, p.H, p.S), prep ? n2 * 8 : size_t(0));
  hipLaunchKernelGGL(k_risk_baseline, dim3(p.Bt + prep), dim3(threads), lds, s, p, t);
}

}  // namespace mpcmmd
