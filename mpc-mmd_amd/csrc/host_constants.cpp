// See host_constants.hpp.
#include "host_constants.hpp"

#include <cmath>
#include <stdexcept>

namespace mpcmmd {

std::vector<double> linspace(double start, double stop, int num) {
  std::vector<double> y(num);
  if (num == 1) {
    y[0] = start;
    return y;
  }
  const double step = (stop - start) / double(num - 1);
  for (int i = 0; i < num; ++i) y[i] = double(i) * step + start;
  y[num - 1] = stop;  // numpy sets the endpoint exactly
  return y;
}

static double binom(int n, int k) {
  if (k < 0 || k > n) return 0.0;
  long long r = 1;
  for (int i = 1; i <= k; ++i) r = r * (n - k + i) / i;
  return double(r);
}

// C(n,i) (1-s)^(n-i) s^i, powers by repeated multiplication
static double bern(int n, int i, double s, double oms) {
  if (i < 0 || i > n) return 0.0;
  double a = 1.0, b = 1.0;
  for (int k = 0; k < n - i; ++k) a = a * oms;
  for (int k = 0; k < i; ++k) b = b * s;
  return (binom(n, i) * a) * b;
}

void bernstein10(const std::vector<double>& t, double tmin, double tmax, std::vector<double>& P,
                 std::vector<double>& Pd, std::vector<double>& Pdd) {
  const int n = 10;
  const int L = int(t.size());
  const double l = tmax - tmin;
  P.assign(size_t(L) * kNvar, 0.0);
  Pd = P;
  Pdd = P;
  for (int r = 0; r < L; ++r) {
    const double s = (t[r] - tmin) / l;
    const double oms = 1.0 - s;
    for (int i = 0; i <= n; ++i) {
      P[r * kNvar + i] = bern(n, i, s, oms);
      Pd[r * kNvar + i] = (double(n) * (bern(n - 1, i - 1, s, oms) - bern(n - 1, i, s, oms))) / l;
      Pdd[r * kNvar + i] =
          (double(n * (n - 1)) *
           ((bern(n - 2, i - 2, s, oms) - 2.0 * bern(n - 2, i - 1, s, oms)) + bern(n - 2, i, s, oms))) /
          (l * l);
    }
  }
}

bool invert(std::vector<double>& a, int n) {
  std::vector<double> inv(size_t(n) * n, 0.0);
  for (int i = 0; i < n; ++i) inv[i * n + i] = 1.0;
  for (int c = 0; c < n; ++c) {
    int piv = c;
    for (int r = c + 1; r < n; ++r)
      if (std::fabs(a[r * n + c]) > std::fabs(a[piv * n + c])) piv = r;
    if (a[piv * n + c] == 0.0) return false;
    if (piv != c)
      for (int k = 0; k < n; ++k) {
        std::swap(a[c * n + k], a[piv * n + k]);
        std::swap(inv[c * n + k], inv[piv * n + k]);
      }
    const double d = a[c * n + c];
    for (int k = 0; k < n; ++k) {
      a[c * n + k] /= d;
      inv[c * n + k] /= d;
    }
    for (int r = 0; r < n; ++r) {
      if (r == c) continue;
      const double f = a[r * n + c];
      if (f == 0.0) continue;
      for (int k = 0; k < n; ++k) {
        a[r * n + k] -= f * a[c * n + k];
        inv[r * n + k] -= f * inv[c * n + k];
      }
    }
  }
  a.swap(inv);
  return true;
}

static inline double round32(double v) { return double(float(v)); }

// C = A^T B for A [m][p], B [m][q] (row-major) -> [p][q]
static std::vector<double> atb(const double* A, const double* B, int m, int p, int q) {
  std::vector<double> C(size_t(p) * q, 0.0);
  for (int r = 0; r < m; ++r)
    for (int i = 0; i < p; ++i)
      for (int j = 0; j < q; ++j) C[i * q + j] += A[r * p + i] * B[r * q + j];
  return C;
}

static std::vector<double> kkt(const std::vector<double>& cost, const std::vector<double>& Aeq, int ne) {
  const int n = kNvar + ne;
  std::vector<double> K(size_t(n) * n, 0.0);
  for (int i = 0; i < kNvar; ++i)
    for (int j = 0; j < kNvar; ++j) K[i * n + j] = cost[i * kNvar + j];
  for (int e = 0; e < ne; ++e)
    for (int j = 0; j < kNvar; ++j) {
      K[j * n + kNvar + e] = Aeq[e * kNvar + j];
      K[(kNvar + e) * n + j] = Aeq[e * kNvar + j];
    }
  return K;
}

ProblemConsts build_constants(int num_prime, int variant) {
  ProblemConsts c;
  if (num_prime < 2 || num_prime > kNum) throw std::runtime_error("num_prime must be in [2, 100]");
  if (variant < 0 || variant > 3) throw std::runtime_error("variant must be 0..3");
  if (variant == 1) {  // synthetic_dynamic_obs/optimizer/cem.py:155, cem_helper.py:24
    c.y_lb = -2.25;
    c.y_ub = -1.25;
    c.K_steer = 0.05;
  }
  if (variant >= 2) {  // carla/optimizer/cem.py:25-36, 161-166; beta steer noise sigma (2b - 1) (cem_helper.py:777)
    c.a_obs = 4.5;
    c.b_obs = 3.0;
    c.wheel_base = 2.875;
    c.K_steer = 1.0;
    c.carla = true;
    if (variant == 3) {  // Town10HD
      c.y_lb = -0.3, c.y_ub = 3.8, c.y_des_1 = 0.0, c.y_des_2 = 3.5;
    } else {  // Town05
      c.y_lb = -3.8, c.y_ub = 0.3, c.y_des_1 = 0.0, c.y_des_2 = -3.5;
    }
  }
  c.H = num_prime;
  // planning basis on linspace(0, 15, 100) (cem.py:42-48), cast to fp32
  std::vector<double> P, Pd, Pdd;
  const auto t = linspace(0.0, c.t_fin, kNum);
  bernstein10(t, t.front(), t.back(), P, Pd, Pdd);
  c.P64 = P;
  c.Pd64 = Pd;
  c.Pdd64 = Pdd;
  for (auto* v : {&P, &Pd, &Pdd})
    for (auto& x : *v) x = round32(x);
  c.P = P;
  c.Pd = Pd;
  c.Pdd = Pdd;
  // horizon basis (cem_helper.py:112-118)
  std::vector<double> Pp, Ppd, Ppdd;
  const auto tp = linspace(0.0, double(num_prime) * c.dt, num_prime);
  bernstein10(tp, tp.front(), tp.back(), Pp, Ppd, Ppdd);
  for (auto& x : Pp) x = round32(x);
  c.P_prime = Pp;

  // equality rows (cem.py:55-56)
  std::vector<double> Aeq_x(3 * kNvar), Aeq_y(4 * kNvar);
  for (int j = 0; j < kNvar; ++j) {
    Aeq_x[0 * kNvar + j] = Aeq_y[0 * kNvar + j] = P[j];
    Aeq_x[1 * kNvar + j] = Aeq_y[1 * kNvar + j] = Pd[j];
    Aeq_x[2 * kNvar + j] = Aeq_y[2 * kNvar + j] = Pdd[j];
    Aeq_y[3 * kNvar + j] = Pd[(kNum - 1) * kNvar + j];
  }
  // guess QP (cem_helper.py:183-217)
  {
    auto sm = atb(Pdd.data(), Pdd.data(), kNum, kNvar, kNvar);
    std::vector<double> cx(kNvar * kNvar), cy(kNvar * kNvar);
    for (int i = 0; i < kNvar * kNvar; ++i) cx[i] = cy[i] = 100.0 * sm[i];
    c.guess_colsum_x.assign(4 * kNvar, 0.0);
    c.guess_colsum_y.assign(4 * kNvar, 0.0);
    std::vector<double> Avd(25 * kNvar), Apd(25 * kNvar);
    for (int k = 0; k < 4; ++k) {
      for (int r = 0; r < 25; ++r)
        for (int j = 0; j < kNvar; ++j) {
          const int row = (25 * k + r) * kNvar + j;
          Avd[r * kNvar + j] = Pdd[row] - c.k_p_v * Pd[row];
          Apd[r * kNvar + j] = Pdd[row] - c.k_p * P[row];
          c.guess_colsum_x[k * kNvar + j] += Avd[r * kNvar + j];
          c.guess_colsum_y[k * kNvar + j] += Apd[r * kNvar + j];
        }
      auto ax = atb(Avd.data(), Avd.data(), 25, kNvar, kNvar);
      auto ay = atb(Apd.data(), Apd.data(), 25, kNvar, kNvar);
      for (int i = 0; i < kNvar * kNvar; ++i) {
        cx[i] += ax[i];
        cy[i] += ay[i];
      }
    }
    c.guess_kinv_x = kkt(cx, Aeq_x, 3);
    c.guess_kinv_y = kkt(cy, Aeq_y, 4);
    if (!invert(c.guess_kinv_x, 14) || !invert(c.guess_kinv_y, 15))
      throw std::runtime_error("singular guess KKT");
  }
  // projection KKT (projection.py:145-156): I + Pdd^T Pdd + Pd^T Pd (+ A_lane^T A_lane)
  {
    auto a = atb(Pdd.data(), Pdd.data(), kNum, kNvar, kNvar);
    auto b = atb(Pd.data(), Pd.data(), kNum, kNvar, kNvar);
    std::vector<double> base(kNvar * kNvar);
    for (int i = 0; i < kNvar; ++i)
      for (int j = 0; j < kNvar; ++j) base[i * kNvar + j] = (i == j ? 1.0 : 0.0) + a[i * kNvar + j] + b[i * kNvar + j];
    // A_lane = [P[1:]; -P[1:]] (gamma = 1, cem.py:126-134)
    std::vector<double> Al(size_t(kLane) * kNvar);
    for (int r = 0; r < kNum - 1; ++r)
      for (int j = 0; j < kNvar; ++j) {
        Al[r * kNvar + j] = P[(r + 1) * kNvar + j];
        Al[(r + kNum - 1) * kNvar + j] = -P[(r + 1) * kNvar + j];
      }
    auto ll = atb(Al.data(), Al.data(), kLane, kNvar, kNvar);
    std::vector<double> by(base);
    for (int i = 0; i < kNvar * kNvar; ++i) by[i] += ll[i];
    c.proj_kinv_x = kkt(base, Aeq_x, 3);
    c.proj_kinv_y = kkt(by, Aeq_y, 4);
    if (!invert(c.proj_kinv_x, 14) || !invert(c.proj_kinv_y, 15))
      throw std::runtime_error("singular projection KKT");
  }
  // Bernstein fit (cem_helper.py:553-564): (P'^T P' + 0.05 I)^-1 P'^T
  {
    const int H = num_prime;
    auto g = atb(Pp.data(), Pp.data(), H, kNvar, kNvar);
    for (int i = 0; i < kNvar; ++i) g[i * kNvar + i] += 0.05;
    if (!invert(g, kNvar)) throw std::runtime_error("singular fit matrix");
    c.fit.assign(size_t(kNvar) * H, 0.0);
    for (int i = 0; i < kNvar; ++i)
      for (int h = 0; h < H; ++h) {
        double s = 0.0;
        for (int k = 0; k < kNvar; ++k) s += g[i * kNvar + k] * Pp[h * kNvar + k];
        c.fit[i * H + h] = s;
      }
  }
  return c;
}

void det_projection_kinv(const ProblemConsts& c, int num_obs, std::vector<double>& kx, std::vector<double>& ky) {
  if (num_obs < 1) throw std::runtime_error("det projection: num_obs >= 1");
  const std::vector<double>& P = c.P;
  auto a = atb(c.Pdd.data(), c.Pdd.data(), kNum, kNvar, kNvar);
  auto b = atb(c.Pd.data(), c.Pd.data(), kNum, kNvar, kNvar);
  std::vector<double> base(kNvar * kNvar);
  for (int i = 0; i < kNvar; ++i)
    for (int j = 0; j < kNvar; ++j) base[i * kNvar + j] = (i == j ? 1.0 : 0.0) + a[i * kNvar + j] + b[i * kNvar + j];
  std::vector<double> Al(size_t(kLane) * kNvar);
  for (int r = 0; r < kNum - 1; ++r)
    for (int j = 0; j < kNvar; ++j) {
      Al[r * kNvar + j] = P[(r + 1) * kNvar + j];
      Al[(r + kNum - 1) * kNvar + j] = -P[(r + 1) * kNvar + j];
    }
  auto ll = atb(Al.data(), Al.data(), kLane, kNvar, kNvar);
  // A_obs = tile(P, (num_obs, 1)) (carla/optimizer/cem.py:66), accumulated row by row
  std::vector<double> Ao(size_t(num_obs) * kNum * kNvar);
  for (int o = 0; o < num_obs; ++o)
    for (int i = 0; i < kNum * kNvar; ++i) Ao[size_t(o) * kNum * kNvar + i] = P[i];
  auto oo = atb(Ao.data(), Ao.data(), num_obs * kNum, kNvar, kNvar);
  std::vector<double> cx(base), cy(base);
  for (int i = 0; i < kNvar * kNvar; ++i) {
    cx[i] += oo[i];
    cy[i] += ll[i];
    cy[i] += oo[i];
  }
  std::vector<double> Aeq_x(3 * kNvar), Aeq_y(4 * kNvar);
  for (int j = 0; j < kNvar; ++j) {
    Aeq_x[0 * kNvar + j] = Aeq_y[0 * kNvar + j] = P[j];
    Aeq_x[1 * kNvar + j] = Aeq_y[1 * kNvar + j] = c.Pd[j];
    Aeq_x[2 * kNvar + j] = Aeq_y[2 * kNvar + j] = c.Pdd[j];
    Aeq_y[3 * kNvar + j] = c.Pd[(kNum - 1) * kNvar + j];
  }
  kx = kkt(cx, Aeq_x, 3);
  ky = kkt(cy, Aeq_y, 4);
  if (!invert(kx, 14) || !invert(ky, 15)) throw std::runtime_error("singular det projection KKT");
}

DynObsConsts build_dyn_obs_consts() {
  // obs_data.__init__ (obs_data_generate_dynamic.py:10-36): the same
  // linspace(0, 15, 100) basis, cast to fp32 by jnp.asarray
  DynObsConsts c;
  std::vector<double> P, Pd, Pdd;
  const auto t = linspace(0.0, 15.0, kNum);
  bernstein10(t, t.front(), t.back(), P, Pd, Pdd);
  for (auto* v : {&P, &Pd, &Pdd})
    for (auto& x : *v) x = round32(x);
  const double k_p_v = 2.0, k_p = 2.0;
  std::vector<double> Avd(size_t(kNum) * kNvar), Apd(size_t(kNum) * kNvar);
  c.colsum_x.assign(kNvar, 0.0);
  c.colsum_y.assign(kNvar, 0.0);
  for (int r = 0; r < kNum; ++r)
    for (int j = 0; j < kNvar; ++j) {
      const int i = r * kNvar + j;
      Avd[i] = Pdd[i] - k_p_v * Pd[i];
      Apd[i] = Pdd[i] - k_p * P[i];
      c.colsum_x[j] += Avd[i];
      c.colsum_y[j] += Apd[i];
    }
  // cost = 100 Pdd^T Pdd + rho A^T A (:86-90, rho_v = rho_offset = 1)
  auto sm = atb(Pdd.data(), Pdd.data(), kNum, kNvar, kNvar);
  auto ax = atb(Avd.data(), Avd.data(), kNum, kNvar, kNvar);
  auto ay = atb(Apd.data(), Apd.data(), kNum, kNvar, kNvar);
  std::vector<double> cx(kNvar * kNvar), cy(kNvar * kNvar);
  for (int i = 0; i < kNvar * kNvar; ++i) {
    cx[i] = 100.0 * sm[i] + ax[i];
    cy[i] = 100.0 * sm[i] + ay[i];
  }
  // A_eq_x = [P0; Pd0; Pdd0], A_eq_y = [P0; Pd0; Pdd0; Pd_end] (:33-34)
  std::vector<double> Aeq_x(3 * kNvar), Aeq_y(4 * kNvar);
  for (int j = 0; j < kNvar; ++j) {
    Aeq_x[0 * kNvar + j] = Aeq_y[0 * kNvar + j] = P[j];
    Aeq_x[1 * kNvar + j] = Aeq_y[1 * kNvar + j] = Pd[j];
    Aeq_x[2 * kNvar + j] = Aeq_y[2 * kNvar + j] = Pdd[j];
    Aeq_y[3 * kNvar + j] = Pd[(kNum - 1) * kNvar + j];
  }
  c.kinv_x = kkt(cx, Aeq_x, 3);
  c.kinv_y = kkt(cy, Aeq_y, 4);
  if (!invert(c.kinv_x, 14) || !invert(c.kinv_y, 15)) throw std::runtime_error("singular obstacle KKT");
  c.P = P;
  return c;
}

void dyn_obs_traj(const DynObsConsts& c, int num_obs, const float* x0, const float* y0, const float* vx0,
                  const float* vy0, const float* v_des, float y_des, float* x_traj, float* y_traj) {
  // rhs = [-lincost; b_eq] with -lincost = A^T b = -k_p * target * colsum(A)
  // (:81-96); b_eq_x = [x0, vx0, 0], b_eq_y = [y0, vy0, 0, 0] (:56-71)
  for (int o = 0; o < num_obs; ++o) {
    double rx[14], ry[15];
    const double tv = -2.0 * double(v_des[o]), ty = -2.0 * double(y_des);
    for (int j = 0; j < kNvar; ++j) {
      rx[j] = tv * c.colsum_x[j];
      ry[j] = ty * c.colsum_y[j];
    }
    rx[11] = x0[o], rx[12] = vx0[o], rx[13] = 0.0;
    ry[11] = y0[o], ry[12] = vy0[o], ry[13] = 0.0, ry[14] = 0.0;
    float cxf[kNvar], cyf[kNvar];
    for (int j = 0; j < kNvar; ++j) {
      double sx = 0.0, sy = 0.0;
      for (int i = 0; i < 14; ++i) sx += c.kinv_x[j * 14 + i] * rx[i];
      for (int i = 0; i < 15; ++i) sy += c.kinv_y[j * 15 + i] * ry[i];
      cxf[j] = float(sx);
      cyf[j] = float(sy);
    }
    // x = P c (:104-105), fp32 coefficients, fp64 accumulation
    for (int r = 0; r < kNum; ++r) {
      double sx = 0.0, sy = 0.0;
      for (int j = 0; j < kNvar; ++j) {
        sx += c.P[r * kNvar + j] * double(cxf[j]);
        sy += c.P[r * kNvar + j] * double(cyf[j]);
      }
      x_traj[size_t(o) * kNum + r] = float(sx);
      y_traj[size_t(o) * kNum + r] = float(sy);
    }
  }
}

}  // namespace mpcmmd
