// compute_cost (cem_helper.py:232-262; CARLA carla/optimizer/cem_helper.py:
// 529-554): the eleven norms of a candidate's trajectory and controls, formed
// by k_front for every candidate (its values are in registers there) into
// Params::cnorm, and the total k_select forms for the 20 obstacle elites.
#pragma once
#include "block.hpp"
#include "kernels.hpp"

namespace mpcmmd {

// One wave per candidate, steps t0 = lane and t1 = lane + 64 (values of
// lanes with t1 >= 100 are never summed, nor shuffled into a summed step).
// Returns the norms (des, st, sv, sa, v, sp, svp, ydd, xdd, des2, cen),
// wave-uniform.
DEVI void cost_norms(const Params& p, float v_des, int lane, const float (&y)[2], const float (&xd)[2],
                     const float (&yd)[2], const float (&xdd)[2], const float (&ydd)[2], const float (&st)[2],
                     const float (&kap)[2], double (&nk)[11]) {
  constexpr int kSteps = 100;
  const int t0 = lane, t1 = lane + 64;
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
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int tt = q == 0 ? t0 : t1;
    if (tt >= kSteps) continue;
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
    const double dv = double(v - v_des);
    n_v += dv * dv;
    const double sp = double(fmaxf(0.0f, fabsf(st[q]) - 0.6f));
    n_sp += sp * sp;
    n_ydd += double(ydd[q]) * double(ydd[q]);
    n_xdd += double(xdd[q]) * double(xdd[q]);
    if (tt < kSteps - 1) {
      n_sv += double(sv[q]) * double(sv[q]);
      const double svp = double(fmaxf(0.0f, fabsf(sv[q]) - 0.05f));
      n_svp += svp * svp;
    }
    if (tt < kSteps - 2) n_sa += double(sa[q]) * double(sa[q]);
  }
  // the eleven wave totals at once (lanes 4 k .. 4 k + 3 hold total k)
  const double nv[11] = {n_des, n_st, n_sv, n_sa, n_v, n_sp, n_svp, n_ydd, n_xdd, n_des2, n_cen};
  const double z = wave_totals16_d(nv);
#pragma unroll
  for (int k = 0; k < 11; ++k) nk[k] = sqrt(readlane_d(z, 4 * k));
}

// compute_cost's total of candidate e from its norms (cem_helper.py:254-262)
DEVI float cost_total(const Params& p, int e, const double (&nk)[11]) {
  const double n_des = nk[0], n_st = nk[1], n_sv = nk[2], n_sa = nk[3], n_v = nk[4], n_sp = nk[5], n_svp = nk[6];
  const double n_ydd = nk[7], n_xdd = nk[8], n_des2 = nk[9], n_cen = nk[10];
  const double cobs = double(p.w_obs * p.obs_cost[e]);
  const double clane = double(p.w_lane * p.lane_cost[e]);
  double tot;
  if (p.carla) {  // carla/optimizer/cem_helper.py:546-554; risk terms weighted in fp32 (cem.py:373-375)
    const double cdes = double(p.w_des * p.lane_des[e]);
    tot = (double(p.res_norm[e]) + 0.1 * n_v + 0.1 * (n_st + n_sv + n_sa) + 0.1 * (n_sp + n_svp) + 0.02 * n_ydd +
           0.02 * n_xdd + 0.01 * (n_des * n_des2) + 0.1 * n_cen) +
          cobs + clane + cdes;
  } else {
    tot = double(p.res_norm[e]) + 0.1 * n_v + 0.1 * (n_st + n_sv + n_sa) + 0.1 * (n_sp + n_svp) + 0.02 * n_ydd +
          0.02 * n_xdd + 0.0 * n_des + cobs + 0.0 * clane;
  }
  return float(tot);
}

// cost_norms of candidate e from k_front's stores (traj, steer, kappa_i)
DEVI void cost_norms_at(const Params& p, int e, int lane, double (&nk)[11]) {
  constexpr int kSteps = 100;
  const size_t plane = size_t(p.Bt) * kSteps, row = size_t(e) * kSteps;
  const int t0 = lane, t1c = min(lane + 64, kSteps - 1);
  auto ld = [&](int k, int tt) { return p.traj[size_t(k) * plane + row + tt]; };
  const float y[2] = {ld(1, t0), ld(1, t1c)}, xd[2] = {ld(2, t0), ld(2, t1c)}, yd[2] = {ld(3, t0), ld(3, t1c)};
  const float xdd[2] = {ld(4, t0), ld(4, t1c)}, ydd[2] = {ld(5, t0), ld(5, t1c)};
  const float st[2] = {p.steer[row + t0], p.steer[row + t1c]};
  const float kap[2] = {p.carla ? p.kappa_i[row + t0] : 0.0f, p.carla ? p.kappa_i[row + t1c] : 0.0f};
  cost_norms(p, p.v_des[e / p.B], lane, y, xd, yd, xdd, ydd, st, kap, nk);
}

// the norms of lane k (k < 11) into cnorm
DEVI void store_norms(const Params& p, int e, int lane, const double (&nk)[11]) {
  if (lane < 11) {
    double v = nk[0];
#pragma unroll
    for (int k = 1; k < 11; ++k) v = lane == k ? nk[k] : v;
    p.cnorm[size_t(e) * kCnormStride + lane] = v;
  }
}

// k_select's preparation in leading workgroups of the risk launch
// (Params::select_prep; they run beside the rollouts): workgroup w < G sorts
// configuration w's projection residuals (cem.py:233-248; the LDS bitonic
// network over the workgroup, keys: next_pow2(B) words) into tr_proj[t], the
// others compute the cost norms of threads / 64 candidates each.
HDI int select_prep_groups(const Params& p, int threads) {
  const int nw = threads / 64;
  return p.select_prep ? p.G + (p.Bt + nw - 1) / nw : 0;
}
DEVI void select_prep(const Params& p, int t, int w, unsigned long long* keys) {
  if (w < p.G) {
    const int B = p.B, g0 = w * B;
    int N = 1;
    while (N < B) N <<= 1;
    for (int i = threadIdx.x; i < N; i += blockDim.x)
      keys[i] = i < B ? ((unsigned long long)sort_key(p.res_norm[g0 + i]) << 32) | unsigned(i) : ~0ull;
    bitonic_sort(keys, N);
    int32_t* tr = p.tr_proj + (size_t(w) * p.T + t) * B;
    for (int i = threadIdx.x; i < B; i += blockDim.x) tr[i] = int(keys[i] & 0xFFFFFFFFu);
    return;
  }
  const int e = (w - p.G) * int(blockDim.x >> 6) + int(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (e >= p.Bt) return;  // whole waves; no barrier follows
  double nk[11];
  cost_norms_at(p, e, lane, nk);
  store_norms(p, e, lane, nk);
}

}  // namespace mpcmmd
