// Stage "front": initial guess QP + one ADMM projection iteration + controls,
// one wave64 per candidate, 4 candidates per 256-thread workgroup.
//
//   compute_x_guess      optimizer/cem_helper.py:169-230
//   compute_projection   optimizer/projection.py:276-323
//     initial_alpha_d_obs  :52-121   (obstacle terms dead)
//     compute_x            :123-185
//     compute_alph_d       :193-274
//   compute_controls     optimizer/cem_helper.py:540-551
//
// k_front<true> is compute_cem_det's projection (carla/optimizer/
// projection_det.py:56-336): the same, plus the obstacle terms the other
// projections leave dead -- per (obstacle, point) polar forms alpha_obs /
// d_obs on the guess and on the projected trajectory, rho_obs A_obs^T b_obs in
// the linear cost, its own KKT inverse (A_obs^T A_obs in the cost), the
// obstacle residual in res_norm and A_obs^T r_obs in the multipliers.
//
// Lane l owns planning points t = l and t = l + 64 (< 100).  The 100x11
// Bernstein bases are staged once per workgroup in LDS (13.2 KB).  Every
// basis product P c / P^T r accumulates in fp64 and is rounded to fp32 where
// the reference holds an fp32 array; the batch-invariant KKT solves are fp64
// GEMVs with inverses built on the host (host_constants.cpp).  Elementwise
// work is fp32 in the reference's operation order (-ffp-contract=off).
#include "common.hpp"
#include "cost.hpp"
#include "frenet.hpp"
#include "kernels.hpp"

namespace mpcmmd {

namespace {

constexpr int kN = 100;
constexpr int kNv = 11;
constexpr float kPiF = 3.14159274101257324f;     // float32(pi)
constexpr float kTwoPiF = 6.28318548202514648f;  // float32(2 pi)

struct Rows {
  float P[2][kNv], D[2][kNv], DD[2][kNv];
};

DEVI float eval_row(const float (&r)[kNv], const double (&c)[kNv]) {
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < kNv; ++k) s += double(r[k]) * c[k];
  return float(s);
}

// the 11 wave totals of s (fp64), rounded to fp32, in every lane
DEVI void totals11(const double (&s)[kNv], float (&out)[kNv]) {
  const double z = wave_totals16_d(s);
#pragma unroll
  for (int k = 0; k < kNv; ++k) out[k] = float(readlane_d(z, 4 * k));
}

// out[k] = fp32( sum_t M[t][k] r[t] ) over the wave's 100 points
DEVI void adj(const float (&M0)[kNv], float r0, const float (&M1)[kNv], float r1, bool v1, float (&out)[kNv]) {
  double s[kNv];
#pragma unroll
  for (int k = 0; k < kNv; ++k) {
    s[k] = double(M0[k]) * double(r0);
    if (v1) s[k] += double(M1[k]) * double(r1);
  }
  totals11(s, out);
}

// jnp.remainder(x, 2pi) for the unwrap (fmod, then shift into [0, 2pi))
DEVI float rem_2pi(float x) {
  float r = fmodf(x, kTwoPiF);
  if (r != 0.0f && r < 0.0f) r = r + kTwoPiF;
  return r;
}

// per-step phase correction of jnp.unwrap (period 2 pi, discont pi)
DEVI float unwrap_corr(float dd) {
  float ddmod = rem_2pi(dd + kPiF) - kPiF;
  if (ddmod == -kPiF && dd > 0.0f) ddmod = kPiF;
  return fabsf(dd) < kPiF ? 0.0f : ddmod - dd;
}

// alpha = unwrap(atan2) along the 100 points; lane owns t0 = lane, t1 = lane + 64
DEVI void unwrap2(float& a0, float& a1, int lane, bool v1) {
  const float prev0 = __shfl_up(a0, 1, kWave);
  const float last0 = readlane_f(a0, 63);
  const float up1 = __shfl_up(a1, 1, kWave);  // shuffles outside any divergent branch
  const float prev1 = lane == 0 ? last0 : up1;
  const float ph0 = lane == 0 ? 0.0f : unwrap_corr(a0 - prev0);
  const float ph1 = v1 ? unwrap_corr(a1 - prev1) : 0.0f;
  // sequential cumsum (numpy / oracle order) over the nonzero corrections only:
  // adding a +0 leaves the fp32 running sum unchanged, so the sums are those of
  // the full sequential scan; usually no correction is nonzero and nothing runs
  float acc = 0.0f, cs0 = 0.0f, cs1 = 0.0f;
  unsigned long long m0 = __ballot(ph0 != 0.0f), m1 = __ballot(ph1 != 0.0f);
  while (m0) {
    const int i = __builtin_ctzll(m0);
    m0 &= m0 - 1;
    acc = acc + readlane_f(ph0, i);
    cs0 = lane >= i ? acc : cs0;
  }
  cs1 = acc;
  while (m1) {
    const int i = __builtin_ctzll(m1);
    m1 &= m1 - 1;
    acc = acc + readlane_f(ph1, i);
    cs1 = lane >= i ? acc : cs1;
  }
  if (lane > 0) a0 = a0 + cs0;
  if (v1) a1 = a1 + cs1;
}

// Correctly rounded fp32 transcendentals (fp64 evaluation, one rounding).
// The oracle does the same (oracle/helper.py: cr): feasible candidates'
// res_norm is rounding noise, so reproducible transcendentals are what makes
// the projection-elite order reproducible (DESIGN.md Numerics).
DEVI float cr_atan2(float y, float x) { return float(atan2(double(y), double(x))); }
DEVI float cr_sin(float a) { return float(sin(double(a))); }
// cos and sin from one fp64 sincos (OCML: one argument reduction, the values
// of cos and sin), each rounded once
DEVI void cr_sincos(float a, float& s, float& c) {
  double sd, cd;
  sincos(double(a), &sd, &cd);
  s = float(sd);
  c = float(cd);
}

struct Polar {
  float ca, sa, d;
};

// the det projection's obstacle polar form (projection_det.py:69-73,
// 210-214) of the offset (wc, ws) = (x - x_obs, y - y_obs):
// alpha = atan2(ws a, wc b), d = (a wc cos + b ws sin) / (a^2 cos^2 + b^2 sin^2)
DEVI Polar obs_polar(float wc, float ws, const Params& p) {
  const float al = cr_atan2(ws * p.obs_a, wc * p.obs_b);
  float ca, sa;
  cr_sincos(al, sa, ca);
  const float c1 = p.obs_a2 * (ca * ca) + p.obs_b2 * (sa * sa);
  const float c2 = (p.obs_a * wc) * ca + (p.obs_b * ws) * sa;
  return Polar{ca, sa, c2 / c1};
}

// jnp.maximum(lo, v), NaN propagating
DEVI float max_nan(float lo, float v) { return v != v ? v : fmaxf(lo, v); }

DEVI unsigned long long readlane_u64(unsigned long long v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane(int(unsigned(v)), l), hi = __builtin_amdgcn_readlane(int(unsigned(v >> 32)), l);
  return (unsigned long long)hi << 32 | lo;
}

DEVI unsigned long long shfl_up_u64(unsigned long long v, int d) {
  const int lo = __shfl_up(int(unsigned(v)), d, kWave), hi = __shfl_up(int(unsigned(v >> 32)), d, kWave);
  return (unsigned long long)unsigned(hi) << 32 | unsigned(lo);
}

// alpha = atan2(wy, wx); d = clip((wx cos + wy sin) / (cos^2 + sin^2), lo, hi)
DEVI Polar polar_of(float alpha, float wx, float wy, float lo, float hi) {
  float ca, sa;
  cr_sincos(alpha, sa, ca);
  const float c1 = ca * ca + sa * sa;
  const float c2 = wx * ca + wy * sa;
  float d = c2 / c1;
  d = fminf(fmaxf(d, lo), hi);
  return Polar{ca, sa, d};
}

// Two wave-uniform GEMVs out_x[k] = float(cx0[k] + sum_j Ax[k][j] x[j]) and
// out_y likewise (fp64, j in order): a row per lane (lanes k and 16 + k; the
// rest repeat row 10) and the 22 results broadcast by readlane -- the same
// operations in the same order as every lane forming all 22 sums, with a
// tenth of the VALU instructions (k_front runs one wave per SIMD, where each
// instruction is exposed).
template <int NJ>
DEVI void gemv2_rows(const double* cx0, const double* cy0, const double* Ax, const double* Ay, const double (&x)[NJ],
                     const double (&y)[NJ], float (&ox)[kNv], float (&oy)[kNv]) {
  const int lane = threadIdx.x & 63, sel = (lane >> 4) & 1, k = min(lane & 15, kNv - 1);
  const double* A = (sel ? Ay : Ax) + k * NJ;
  double s = (sel ? cy0 : cx0)[k];
#pragma unroll
  for (int j = 0; j < NJ; ++j) s += A[j] * (sel ? y[j] : x[j]);
  const int f = __float_as_int(float(s));
#pragma unroll
  for (int q = 0; q < kNv; ++q) {
    ox[q] = __int_as_float(__builtin_amdgcn_readlane(f, q));
    oy[q] = __int_as_float(__builtin_amdgcn_readlane(f, 16 + q));
  }
}

template <bool kDet>
__global__ __launch_bounds__(256) void k_front(Params p, int t) {
  __shared__ __attribute__((aligned(16))) float sB[3 * kN * kNv];
  // CARLA: arc_vec [P], kappa [P] of the candidate block's configuration;
  // det: then its obstacle tracks x_obs [O][100], y_obs [O][100]
  extern __shared__ float sPath[];
  MPCMMD_STAMPW(p, 0);
  {  // the basis (3 x 100 x 11 floats) as float4s, every load of a thread in
     // flight before its first LDS store (one memory latency, not thirteen)
    static_assert((3 * kN * kNv) % 4 == 0, "float4 staging");
    constexpr int kQ = 3 * kN * kNv / 4, kPer = (kQ + 255) / 256;
    const float4* b4 = reinterpret_cast<const float4*>(p.basis);
    float4* s4 = reinterpret_cast<float4*>(sB);
    float4 v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) v[j] = b4[min(int(threadIdx.x) + 256 * j, kQ - 1)];
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (int(threadIdx.x) + 256 * j < kQ) s4[threadIdx.x + 256 * j] = v[j];
  }
  if (p.carla) {
    // every candidate of a block belongs to one configuration when B % 4 == 0
    // (the host checks); the block's first candidate names it
    const int g = min(blockIdx.x * 4, p.Bt - 1) / p.B;
    const float* pa = p.path + size_t(g) * 6 * kMaxPath;
    for (int i = threadIdx.x; i < p.P; i += blockDim.x) {
      sPath[i] = pa[2 * kMaxPath + i];
      sPath[p.P + i] = pa[5 * kMaxPath + i];
    }
    if (kDet) {
      const float* of = p.obs_full + size_t(g) * 2 * p.O * kN;
      for (int i = threadIdx.x; i < 2 * p.O * kN; i += blockDim.x) sPath[2 * p.P + i] = of[i];
    }
  }
  __syncthreads();
  MPCMMD_STAMP(p, 40);
  MPCMMD_STAMPW(p, 1);
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= p.Bt) return;
  const double* solve_c = p.solve_c + size_t(b / p.B) * 4 * kNv;  // this candidate's configuration
  const int t0 = lane, t1 = lane + 64;
  const bool v1 = t1 < kN;
  const int t1c = v1 ? t1 : kN - 1;
  Rows R;
#pragma unroll
  for (int k = 0; k < kNv; ++k) {
    R.P[0][k] = sB[0 * kN * kNv + t0 * kNv + k];
    R.P[1][k] = sB[0 * kN * kNv + t1c * kNv + k];
    R.D[0][k] = sB[1 * kN * kNv + t0 * kNv + k];
    R.D[1][k] = sB[1 * kN * kNv + t1c * kNv + k];
    R.DD[0][k] = sB[2 * kN * kNv + t0 * kNv + k];
    R.DD[1][k] = sB[2 * kN * kNv + t1c * kNv + k];
  }

  // ---- compute_x_guess: c_bar = G v + h (fp64) -------------------------------
  const float* pop = p.pop + (size_t(t & 1) * p.Bt + b) * 8;
  double cxb[kNv], cyb[kNv];
  float fcxb[kNv], fcyb[kNv];
  {
    double vx[4], vy[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vx[j] = double(pop[j]);
      vy[j] = double(pop[4 + j]);
    }
    gemv2_rows<4>(solve_c, solve_c + kNv, p.guess_g, p.guess_g + kNv * 4, vx, vy, fcxb, fcyb);
#pragma unroll
    for (int k = 0; k < kNv; ++k) {
      cxb[k] = double(fcxb[k]);
      cyb[k] = double(fcyb[k]);
    }
  }

  // ---- initial_alpha_d_obs (projection.py:52-121) ----------------------------
  float xd[2], yd[2], xdd[2], ydd[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    xd[q] = eval_row(R.D[q], cxb);
    yd[q] = eval_row(R.D[q], cyb);
    xdd[q] = eval_row(R.DD[q], cxb);
    ydd[q] = eval_row(R.DD[q], cyb);
  }
  float av0 = cr_atan2(yd[0], xd[0]), av1 = cr_atan2(yd[1], xd[1]);
  float aa0 = cr_atan2(ydd[0], xdd[0]), aa1 = cr_atan2(ydd[1], xdd[1]);
  MPCMMD_STAMP(p, 41);
  unwrap2(av0, av1, lane, v1);
  unwrap2(aa0, aa1, lane, v1);
  MPCMMD_STAMP(p, 42);
  Polar pv[2] = {polar_of(av0, xd[0], yd[0], 0.1f, 30.0f), polar_of(av1, xd[1], yd[1], 0.1f, 30.0f)};
  Polar pa[2] = {polar_of(aa0, xdd[0], ydd[0], 0.0f, 18.0f), polar_of(aa1, xdd[1], ydd[1], 0.0f, 18.0f)};

  float lx[kNv], ly[kNv], tmp[kNv], tmp2[kNv];
#pragma unroll
  for (int k = 0; k < kNv; ++k) {
    lx[k] = p.lam_x[size_t(b) * kNv + k];
    ly[k] = p.lam_y[size_t(b) * kNv + k];
  }
  {
    float rax[2], ray[2], rvx[2], rvy[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      rax[q] = xdd[q] - pa[q].d * pa[q].ca;
      ray[q] = ydd[q] - pa[q].d * pa[q].sa;
      rvx[q] = xd[q] - pv[q].d * pv[q].ca;
      rvy[q] = yd[q] - pv[q].d * pv[q].sa;
    }
    adj(R.DD[0], rax[0], R.DD[1], rax[1], v1, tmp);
    adj(R.D[0], rvx[0], R.D[1], rvx[1], v1, tmp2);
#pragma unroll
    for (int k = 0; k < kNv; ++k) lx[k] = (lx[k] - tmp[k]) - tmp2[k];
    adj(R.DD[0], ray[0], R.DD[1], ray[1], v1, tmp);
    adj(R.D[0], rvy[0], R.D[1], rvy[1], v1, tmp2);
#pragma unroll
    for (int k = 0; k < kNv; ++k) ly[k] = (ly[k] - tmp[k]) - tmp2[k];
  }

  // ---- det: obstacle polar forms on the guess (projection_det.py:60-74) and
  // rho_obs A_obs^T b_obs of compute_x (:143-147, 164, 169); the multipliers
  // get no obstacle term here (:119-123).  sobs_* = A_obs^T b_obs_* (fp64)
  const float* xob = sPath + 2 * p.P;
  const float* yob = xob + p.O * kN;
  float obsx[kNv], obsy[kNv];
  unsigned long long nonfin = 0;  // bit 2 o + q: d_obs of the guess at (o, point q) is not finite
  if (kDet) {
    double sox[kNv], soy[kNv];
#pragma unroll
    for (int k = 0; k < kNv; ++k) sox[k] = soy[k] = 0.0;
    float xg[2], yg[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      xg[q] = eval_row(R.P[q], cxb);
      yg[q] = eval_row(R.P[q], cyb);
    }
    for (int o = 0; o < p.O; ++o) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (q == 1 && !v1) continue;
        const int tt = q == 0 ? t0 : t1;
        const float xo = xob[o * kN + tt], yo = yob[o * kN + tt];
        const Polar op = obs_polar(xg[q] - xo, yg[q] - yo, p);
        const float d0 = max_nan(1.0f, op.d);
        if (!isfinite(d0)) nonfin |= 1ull << (2 * o + q);
        const float bx = xo + (d0 * op.ca) * p.obs_a;  // x_obs + d cos(alpha) a
        const float by = yo + (d0 * op.sa) * p.obs_b;
#pragma unroll
        for (int k = 0; k < kNv; ++k) {
          sox[k] += double(R.P[q][k]) * double(bx);
          soy[k] += double(R.P[q][k]) * double(by);
        }
      }
    }
    totals11(sox, obsx);
    totals11(soy, obsy);
  }

  MPCMMD_STAMP(p, 43);
  // ---- compute_x (projection.py:123-185) --------------------------------------
  // lane-bound rows j = t-1 (t = 1..99): ub row j, lb row 99 + j; A_lane = [P[1:]; -P[1:]]
  const float y_ub = p.y_ub, mlb = -p.y_lb;  // b_lane: ub rows y_ub, lb rows -y_lb (gamma = 1)
  float* sl = p.s_lane + size_t(b) * (2 * (kN - 1));
  const bool h0 = t0 >= 1;  // t0 = 0 has no lane row
  float baug_ub[2] = {0.f, 0.f}, baug_lb[2] = {0.f, 0.f};
  if (h0) {
    baug_ub[0] = y_ub - sl[t0 - 1];
    baug_lb[0] = mlb - sl[kN - 1 + t0 - 1];
  }
  if (v1) {
    baug_ub[1] = y_ub - sl[t1 - 1];
    baug_lb[1] = mlb - sl[kN - 1 + t1 - 1];
  }
  float cx[kNv], cy[kNv];
  {
    float bx[2], by[2], vxb[2], vyb[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      bx[q] = pa[q].d * pa[q].ca;
      by[q] = pa[q].d * pa[q].sa;
      vxb[q] = pv[q].d * pv[q].ca;
      vyb[q] = pv[q].d * pv[q].sa;
    }
    float linx[kNv], liny[kNv];
    adj(R.DD[0], bx[0], R.DD[1], bx[1], v1, tmp);
    adj(R.D[0], vxb[0], R.D[1], vxb[1], v1, tmp2);
#pragma unroll
    for (int k = 0; k < kNv; ++k) linx[k] = ((-lx[k] - fcxb[k]) - tmp[k]) - tmp2[k];
    if (kDet)
#pragma unroll
      for (int k = 0; k < kNv; ++k) linx[k] = linx[k] - obsx[k];
    adj(R.DD[0], by[0], R.DD[1], by[1], v1, tmp);
    adj(R.D[0], vyb[0], R.D[1], vyb[1], v1, tmp2);
#pragma unroll
    for (int k = 0; k < kNv; ++k) liny[k] = ((-ly[k] - fcyb[k]) - tmp[k]) - tmp2[k];
    // A_lane^T b_aug: sum_j P[j+1][k] (baug_ub[j] - baug_lb[j]) in fp64
    double sa[kNv];
#pragma unroll
    for (int k = 0; k < kNv; ++k) {
      double s = 0.0;
      if (h0) s += double(R.P[0][k]) * double(baug_ub[0]) - double(R.P[0][k]) * double(baug_lb[0]);
      if (v1) s += double(R.P[1][k]) * double(baug_ub[1]) - double(R.P[1][k]) * double(baug_lb[1]);
      sa[k] = s;
    }
    totals11(sa, tmp);
#pragma unroll
    for (int k = 0; k < kNv; ++k) liny[k] = liny[k] - tmp[k];
    if (kDet)
#pragma unroll
      for (int k = 0; k < kNv; ++k) liny[k] = liny[k] - obsy[k];
    // KKT solve: c = Kinv[:11,:11] (-lincost) + Kinv[:11,11:] b_eq
    double nx[kNv], ny[kNv];
#pragma unroll
    for (int j = 0; j < kNv; ++j) {
      nx[j] = -double(linx[j]);
      ny[j] = -double(liny[j]);
    }
    const double* pm = kDet ? p.proj_m_det : p.proj_m;
    gemv2_rows<kNv>(solve_c + 2 * kNv, solve_c + 3 * kNv, pm, pm + kNv * kNv, nx, ny, cx, cy);
  }
  double dcx[kNv], dcy[kNv];
#pragma unroll
  for (int k = 0; k < kNv; ++k) {
    dcx[k] = double(cx[k]);
    dcy[k] = double(cy[k]);
  }
  float x[2], y[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    x[q] = eval_row(R.P[q], dcx);
    y[q] = eval_row(R.P[q], dcy);
    xd[q] = eval_row(R.D[q], dcx);
    yd[q] = eval_row(R.D[q], dcy);
    xdd[q] = eval_row(R.DD[q], dcx);
    ydd[q] = eval_row(R.DD[q], dcy);
  }
  // s_lane / res_lane (A_lane c_y = [y[1:]; -y[1:]])
  float rl_ub[2] = {0.f, 0.f}, rl_lb[2] = {0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const bool ok = q == 0 ? h0 : v1;
    if (!ok) continue;
    const int j = (q == 0 ? t0 : t1) - 1;
    const float ac_ub = y[q], ac_lb = -y[q];
    const float s_ub = fmaxf(0.0f, -ac_ub + y_ub);
    const float s_lb = fmaxf(0.0f, -ac_lb + mlb);
    rl_ub[q] = (ac_ub - y_ub) + s_ub;
    rl_lb[q] = (ac_lb - mlb) + s_lb;
    sl[j] = s_ub;
    sl[kN - 1 + j] = s_lb;
  }

  MPCMMD_STAMP(p, 44);
  // ---- compute_alph_d (projection.py:193-274), no unwrap (Q13) ---------------
  Polar qv[2], qa[2];
  float alv[2], ala[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    alv[q] = cr_atan2(yd[q], xd[q]);
    ala[q] = cr_atan2(ydd[q], xdd[q]);
    qv[q] = polar_of(alv[q], xd[q], yd[q], 0.1f, 30.0f);
    qa[q] = polar_of(ala[q], xdd[q], ydd[q], 0.0f, 18.0f);
  }
  float rax[2], ray[2], rvx[2], rvy[2];
  double n_acc = 0.0, n_vel = 0.0, n_lane = 0.0;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    rax[q] = xdd[q] - qa[q].d * qa[q].ca;
    ray[q] = ydd[q] - qa[q].d * qa[q].sa;
    rvx[q] = xd[q] - qv[q].d * qv[q].ca;
    rvy[q] = yd[q] - qv[q].d * qv[q].sa;
    const bool ok = q == 0 ? true : v1;
    if (ok) {
      n_acc += double(rax[q]) * double(rax[q]) + double(ray[q]) * double(ray[q]);
      n_vel += double(rvx[q]) * double(rvx[q]) + double(rvy[q]) * double(rvy[q]);
      n_lane += double(rl_ub[q]) * double(rl_ub[q]) + double(rl_lb[q]) * double(rl_lb[q]);
    }
  }
  // ---- det: obstacle residuals on the projected trajectory (projection_det.py:
  // 201-217, 257-274): d_obs >= 1 + (1 - gamma_obs) (d_obs_prev - 1), the
  // previous d_obs shifted one point (comp_d_obs_prev, :192-195; gamma_obs = 1,
  // so the bound is 1, or NaN where the shifted guess value is not finite)
  double n_obs = 0.0;
  float rox[kNv], roy[kNv];
  if (kDet) {
    constexpr unsigned long long kEven = 0x5555555555555555ull;
    const unsigned long long up = shfl_up_u64(nonfin, 1), m63 = readlane_u64(nonfin, 63);
    const unsigned long long prev0 = lane == 0 ? 0ull : (up & kEven);           // point t0 - 1 (t0 = 0: the 1)
    const unsigned long long prev1 = lane == 0 ? (m63 & kEven) : ((up >> 1) & kEven);  // point t1 - 1
    double sx[kNv], sy[kNv];
#pragma unroll
    for (int k = 0; k < kNv; ++k) sx[k] = sy[k] = 0.0;
    const float qnan = __int_as_float(0x7fc00000);
    for (int o = 0; o < p.O; ++o) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (q == 1 && !v1) continue;
        const int tt = q == 0 ? t0 : t1;
        const float wc = x[q] - xob[o * kN + tt], ws = y[q] - yob[o * kN + tt];
        const Polar op = obs_polar(wc, ws, p);
        const bool pnf = (((q == 0 ? prev0 : prev1) >> (2 * o)) & 1ull) != 0;
        const float d = pnf ? qnan : max_nan(1.0f, op.d);
        const float rx = wc - (p.obs_a * d) * op.ca, ry = ws - (p.obs_b * d) * op.sa;
        n_obs += double(rx) * double(rx) + double(ry) * double(ry);
#pragma unroll
        for (int k = 0; k < kNv; ++k) {
          sx[k] += double(R.P[q][k]) * double(rx);
          sy[k] += double(R.P[q][k]) * double(ry);
        }
      }
    }
    totals11(sx, rox);
    totals11(sy, roy);
  }
  {
    const double nv[4] = {n_acc, n_vel, n_lane, n_obs};
    const double z = wave_totals16_d(nv);
    n_acc = readlane_d(z, 0);
    n_vel = readlane_d(z, 4);
    n_lane = readlane_d(z, 8);
    n_obs = readlane_d(z, 12);
  }
  float rn = (float(sqrt(n_acc)) + float(sqrt(n_vel))) + float(sqrt(n_lane));
  if (kDet) rn = rn + float(sqrt(n_obs));
  adj(R.DD[0], rax[0], R.DD[1], rax[1], v1, tmp);
  adj(R.D[0], rvx[0], R.D[1], rvx[1], v1, tmp2);
#pragma unroll
  for (int k = 0; k < kNv; ++k) lx[k] = (lx[k] - tmp[k]) - tmp2[k];
  if (kDet)
#pragma unroll
    for (int k = 0; k < kNv; ++k) lx[k] = lx[k] - rox[k];
  adj(R.DD[0], ray[0], R.DD[1], ray[1], v1, tmp);
  adj(R.D[0], rvy[0], R.D[1], rvy[1], v1, tmp2);
  {
    double sa[kNv];
    float t3[kNv];
#pragma unroll
    for (int k = 0; k < kNv; ++k) {
      double s = 0.0;
      if (h0) s += double(R.P[0][k]) * double(rl_ub[0]) - double(R.P[0][k]) * double(rl_lb[0]);
      if (v1) s += double(R.P[1][k]) * double(rl_ub[1]) - double(R.P[1][k]) * double(rl_lb[1]);
      sa[k] = s;
    }
    totals11(sa, t3);
#pragma unroll
    for (int k = 0; k < kNv; ++k) ly[k] = ((ly[k] - tmp[k]) - tmp2[k]) - t3[k];
    if (kDet)
#pragma unroll
      for (int k = 0; k < kNv; ++k) ly[k] = ly[k] - roy[k];
  }

  MPCMMD_STAMP(p, 45);
  // ---- compute_controls (cem_helper.py:540-551) ------------------------------
  float v[2], accv[2], steer[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) v[q] = sqrtf(xd[q] * xd[q] + yd[q] * yd[q]);
  {
    const float d0 = __shfl_down(v[0], 1, kWave);
    const float first1 = readlane_f(v[1], 0);
    const float n1 = __shfl_down(v[1], 1, kWave);
    const float nxt0 = lane < 63 ? d0 : first1;
    const float nxt1 = (t1 == kN - 1) ? v[1] : n1;
    accv[0] = (nxt0 - v[0]) / 0.15f;
    accv[1] = (nxt1 - v[1]) / 0.15f;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const float s2 = xd[q] * xd[q] + yd[q] * yd[q];
    const float curv = (ydd[q] * xd[q] - yd[q] * xdd[q]) / float(pow(double(s2), 1.5));
    steer[q] = float(atan(double(curv * 2.5f)));
  }

  // ---- CARLA (carla/optimizer/projection.py:307-315): curvature at the
  // clipped station, steering from the projected polar forms (replaces
  // compute_controls' steering, carla/optimizer/cem.py:307-317)
  float kapv[2] = {0.f, 0.f};
  if (p.carla) {
    const int P = p.P;
    const float* arc = sPath;
    const float* kap = sPath + P;
    const float hi = arc[P - 1];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float xs = x[q] != x[q] ? x[q] : fminf(fmaxf(x[q], 0.0f), hi);  // jnp.clip (NaN kept)
      const float k = interp_jnp(xs, arc, kap, P);
      const float curv = (qa[q].d * cr_sin(ala[q] - alv[q])) / (qv[q].d * qv[q].d);
      steer[q] = float(atan(double((curv + (k * qv[q].ca) / (1.0f - y[q] * k)) * p.wheel_base)));
      kapv[q] = k;
    }
  }

  // ---- stores -----------------------------------------------------------------
  float* tr = p.traj;
  const size_t plane = size_t(p.Bt) * kN;
  const size_t row = size_t(b) * kN;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (q == 1 && !v1) break;
    const int tt = q == 0 ? t0 : t1;
    tr[0 * plane + row + tt] = x[q];
    tr[1 * plane + row + tt] = y[q];
    tr[2 * plane + row + tt] = xd[q];
    tr[3 * plane + row + tt] = yd[q];
    tr[4 * plane + row + tt] = xdd[q];
    tr[5 * plane + row + tt] = ydd[q];
    p.acc[row + tt] = accv[q];
    p.steer[row + tt] = steer[q];
    if (p.carla) p.kappa_i[row + tt] = kapv[q];
  }
  if (lane < kNv) {
    // lane k stores component k (every lane holds all 11 in registers)
    float vcx = 0.f, vcy = 0.f, vlx = 0.f, vly = 0.f;
#pragma unroll
    for (int k = 0; k < kNv; ++k)
      if (lane == k) {
        vcx = cx[k];
        vcy = cy[k];
        vlx = lx[k];
        vly = ly[k];
      }
    p.cx[size_t(b) * kNv + lane] = vcx;
    p.cy[size_t(b) * kNv + lane] = vcy;
    p.lam_x[size_t(b) * kNv + lane] = vlx;
    p.lam_y[size_t(b) * kNv + lane] = vly;
  }
  if (lane == 0) p.res_norm[b] = rn;
  if (!p.select_prep) {  // compute_cost's norms for k_select (cost.hpp), from the values just stored
    double nk[11];
    cost_norms(p, p.v_des[b / p.B], lane, y, xd, yd, xdd, ydd, steer, kapv, nk);
    store_norms(p, b, lane, nk);
  }
  MPCMMD_STAMP(p, 46);
  MPCMMD_STAMPW(p, 2);
}

}  // namespace

void launch_front(const Params& p, int t, hipStream_t s) {
  if (p.cost == 4) {  // MPCMMD_COST_DET (CARLA handles only)
    const size_t lds = (size_t(2) * p.P + size_t(2) * p.O * kN) * 4;
    hipLaunchKernelGGL(k_front<true>, dim3((p.Bt + 3) / 4), dim3(256), lds, s, p, t);
    return;
  }
  hipLaunchKernelGGL(k_front<false>, dim3((p.Bt + 3) / 4), dim3(256), p.carla ? size_t(2) * p.P * 4 : 0, s, p, t);
}

}  // namespace mpcmmd
