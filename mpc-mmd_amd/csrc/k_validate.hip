// Monte-Carlo validation of saved optima: S/validation.py
// compute_stats (:134-171) for a batch of configurations on the GPU.
//
// One workgroup per configuration.  Threads 0..99 first evaluate the saved
// trajectory's derivatives (xdot = Pdot cx, ... with the fp32 basis, fp64
// sums: validation.py:140-141) and its controls (compute_controls,
// :122-132); then every thread runs noisy rollouts (compute_rollout_complete,
// :42-101) in fp64, the arithmetic NumPy does there, and counts per
// (obstacle, step) and per step the rollouts inside an obstacle ellipse
// (compute_f_bar_temp :103-110, count_nonzero) or across a lane bound
// (compute_lane_bar :112-120).  The counts are integer LDS atomics, so the
// result does not depend on the thread order.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"
#include "rng.hpp"

namespace mpcmmd {
namespace {

constexpr int kValThreads = 1024;
constexpr int kValMaxObs = 32;
constexpr int kValMaxH = 100;

// uniform-free Beta(a, b) straight from the Philox attempt streams
// (rng.hpp: gamma_attempt), log-space ratio as beta_draw_tab
DEVI void log_gamma_direct(double alpha, uint32_t k0, uint32_t k1, uint32_t stream, uint32_t elem, double& lg,
                           double& lub) {
  const MtConst mc = mt_const(alpha);
  lg = log(mc.d);
  lub = 0.0;
  for (int k = 0; k < kGammaMaxAttempts; ++k) {
    const GammaAttempt g = gamma_attempt(k0, k1, stream, elem, k);
    const double v = 1.0 + mc.c * g.x;
    if (v > 0.0) {
      const double v3 = v * v * v;
      if (mt_accept(g.x, g.u, g.lu, mc.d, v3)) {
        lg = log(mc.d * v3);
        lub = g.lw;
        return;
      }
    }
  }
}

DEVI double beta_direct(double a, double b, uint32_t k0, uint32_t k1, uint32_t sa, uint32_t sb, uint32_t elem) {
  double ga, ua, gb, ub;
  log_gamma_direct(a, k0, k1, sa, elem, ga, ua);
  log_gamma_direct(b, k0, k1, sb, elem, gb, ub);
  if (a == 0.0 && b == 0.0) return (ua * 5.0 > ub * 2.0) ? 1.0 : 0.0;
  const double la = a < 1.0 ? ga + ua / a : ga;
  const double lb = b < 1.0 ? gb + ub / b : gb;
  if (la > lb) return 1.0 / (1.0 + exp(lb - la));
  const double ea = exp(la - lb);
  return ea / (ea + 1.0);
}

// standard normal e of stream (k0, k1, stream): block e/4 of philox_normals4
DEVI double philox_normal(uint32_t k0, uint32_t k1, uint32_t stream, uint32_t e) {
  double z[4];
  philox_normals4(k0, k1, stream, 0u, e >> 2, z);
  return z[e & 3];
}

__global__ __launch_bounds__(kValThreads) void k_validate(ValidateParams v) {
  __shared__ double sacc[kValMaxH], ssteer[kValMaxH], sv[kValMaxH];
  __shared__ float sxo[kValMaxObs * kValMaxH], syo[kValMaxObs * kValMaxH];
  __shared__ int cnt[kValMaxObs * kValMaxH], clb[kValMaxH], cub[kValMaxH];
  const int k = blockIdx.x, tid = threadIdx.x;
  const int H = v.H, O = v.O, R = v.R;
  const double dt = 0.15, wb = 2.5;  // prob.t, prob.wheel_base (cem.py:26,40)
  const double* cx = v.cx + size_t(k) * 11;
  const double* cy = v.cy + size_t(k) * 11;
  for (int i = tid; i < O * H; i += kValThreads) {
    const int o = i / H, h = i - o * H;
    sxo[i] = v.x_obs[(size_t(k) * O + o) * 100 + h];
    syo[i] = v.y_obs[(size_t(k) * O + o) * 100 + h];
    cnt[i] = 0;
  }
  double xd = 0.0, yd = 0.0, xdd = 0.0, ydd = 0.0;
  if (tid < 100) {  // np.dot(prob.Pdot_jax, cx) etc. (validation.py:140-141)
    for (int j = 0; j < 11; ++j) {
      xd += double(v.Pdot[tid * 11 + j]) * cx[j];
      yd += double(v.Pdot[tid * 11 + j]) * cy[j];
      xdd += double(v.Pddot[tid * 11 + j]) * cx[j];
      ydd += double(v.Pddot[tid * 11 + j]) * cy[j];
    }
    sv[tid] = sqrt(xd * xd + yd * yd);
  }
  if (tid < H) clb[tid] = cub[tid] = 0;
  __syncthreads();
  if (tid < H) {  // compute_controls (:122-132): acc = diff([v, v_end]) / t, steer = atan(2.5 kappa)
    const double vn = tid < 99 ? sv[tid + 1] : sv[99];
    sacc[tid] = (vn - sv[tid]) / dt;
    const double curv = (ydd * xd - yd * xdd) / pow(xd * xd + yd * yd, 1.5);
    ssteer[tid] = atan(curv * wb);
  }
  __syncthreads();
  const double* st = v.init_state + size_t(k) * 6;
  const uint32_t k0 = v.keys[k], k1 = v.seed;
  const double* dr = v.draws ? v.draws + size_t(k) * 3 * R * H : nullptr;
  for (int r = tid; r < R; r += kValThreads) {
    double x = st[0], y = st[1], vx = st[2], vy = st[3], psi = atan2(st[3], st[2]);  // :147
    for (int h = 0; h < H; ++h) {
      // x_roll[:, h] = state before step h (:94-99)
      for (int o = 0; o < O; ++o) {
        const double wc = x - double(sxo[o * H + h]), ws = y - double(syo[o * H + h]);
        const double c = -(wc * wc) / 18.0625 - (ws * ws) / 7.5625 + 1.0;  // :106-109
        if (!(c <= 0.0)) atomicAdd(&cnt[o * H + h], 1);                     // count_nonzero(max(0, c))
      }
      if (!(-y + v.y_lb <= 0.0)) atomicAdd(&clb[h], 1);  // :116-119
      if (!(y - v.y_ub <= 0.0)) atomicAdd(&cub[h], 1);
      if (h == H - 1) break;
      // noisy controls (:73-92)
      const uint32_t e = uint32_t(r) * uint32_t(H) + uint32_t(h);
      double na, ns, nc;
      if (dr) {
        na = dr[(0 * size_t(R) + r) * H + h];
        ns = dr[(1 * size_t(R) + r) * H + h];
        nc = dr[(2 * size_t(R) + r) * H + h];
      } else if (v.noise == 0) {
        na = philox_normal(k0, k1, kStreamValAcc, e);
        ns = philox_normal(k0, k1, kStreamValSteer, e);
        nc = philox_normal(k0, k1, kStreamValConst, e);
      } else {
        const double fa = fabs(sacc[h]), fs = fabs(ssteer[h]);
        na = beta_direct(2.0 * fa, 5.0 * fa, k0, k1, kStreamValGammaAccA, kStreamValGammaAccB, e);
        ns = beta_direct(2.0 * fs + 1e-5, 5.0 * fs + 1e-5, k0, k1, kStreamValGammaSteerA, kStreamValGammaSteerB, e);
        nc = philox_normal(k0, k1, kStreamValConst, e);
      }
      double ap, sp;
      if (v.noise == 0) {
        ap = v.noise_level * fabs(sacc[h]) * na;
        sp = v.noise_level * fabs(ssteer[h]) * ns;
      } else {  // na, ns are the Beta draws
        ap = v.noise_level * (2.0 * na - 1.0);
        sp = v.K_steer * v.noise_level * (2.0 * ns - 1.0);
      }
      const double an = sacc[h] + ap + v.acc_const * nc;
      const double sn = ssteer[h] + sp + v.steer_const * nc;
      // compute_rollout_one_step (:21-40)
      double sp_ = sqrt(vx * vx + vy * vy);
      sp_ = sp_ + an * dt;
      const double psidot = sp_ * tan(sn) / wb;
      psi = psi + psidot * dt;
      vx = sp_ * cos(psi);
      vy = sp_ * sin(psi);
      x = x + vx * dt;
      y = y + vy * dt;
    }
  }
  __syncthreads();
  // count = max_o max_t #(rollouts in collision); lane = max_t #lb + max_t #ub (:153-169)
  if (tid < 64) {
    int m = 0, mlb = 0, mub = 0;
    for (int i = tid; i < O * H; i += 64) m = max(m, cnt[i]);
    for (int i = tid; i < H; i += 64) {
      mlb = max(mlb, clb[i]);
      mub = max(mub, cub[i]);
    }
    for (int o = 32; o > 0; o >>= 1) {
      m = max(m, __shfl_xor(m, o, 64));
      mlb = max(mlb, __shfl_xor(mlb, o, 64));
      mub = max(mub, __shfl_xor(mub, o, 64));
    }
    if (tid == 0) {
      v.count[k] = m;
      v.count_lane[k] = mlb + mub;
    }
  }
}

}  // namespace

bool validate_shape_ok(int O, int H) { return O >= 1 && O <= kValMaxObs && H >= 2 && H <= kValMaxH; }

void launch_validate(const ValidateParams& v, hipStream_t s) {
  hipLaunchKernelGGL(k_validate, dim3(v.K), dim3(kValThreads), 0, s, v);
}

}  // namespace mpcmmd
