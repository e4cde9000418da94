// Host pieces of the CARLA optimizer variant (see carla_host.hpp).  Built
// with g++ -ffp-contract=off: every fp32 expression below rounds exactly as
// its NumPy restatement in oracle/carla.py.
#include "carla_host.hpp"

#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>

#include "host_constants.hpp"

namespace mpcmmd {

namespace {

float crf(double v) { return float(v); }

}  // namespace

float interp_jnp(float x, const float* xp, const float* fp, int P) {
  int lo = 0, hi = P;  // searchsorted(xp, x, side='right'): first index with xp > x
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (xp[m] <= x) lo = m + 1;
    else hi = m;
  }
  const int i = lo < 1 ? 1 : (lo > P - 1 ? P - 1 : lo);
  const float dx = xp[i] - xp[i - 1];
  const float df = fp[i] - fp[i - 1];
  const float delta = x - xp[i - 1];
  const float eps = 1.4210855e-14f;  // np.spacing(np.finfo(float32).eps)
  float f = std::fabs(dx) <= eps ? fp[i - 1] : fp[i - 1] + (delta / dx) * df;
  if (x < xp[0]) f = fp[0];
  if (x > xp[P - 1]) f = fp[P - 1];
  return f;
}

int closest_index(float x, float y, const float* xp, const float* yp, int P) {
  int best = 0;
  float bd = 0.0f;
  for (int j = 0; j < P; ++j) {
    const float dx = xp[j] - x, dy = yp[j] - y;
    const float d = std::sqrt(dx * dx + dy * dy);
    if (d != d) return j;  // jnp.argmin: the first NaN
    if (j == 0 || d < bd) {
      bd = d;
      best = j;
    }
  }
  return best;
}

FrenetState global_to_frenet(const PathView& p, float x, float y, float v, float vdot, float psi, float psidot) {
  const int idx = closest_index(x, y, p.x, p.y, p.P);
  const float s = p.arc[idx];
  const float ki = interp_jnp(s, p.arc, p.kappa, p.P);
  const float kp = interp_jnp(s + 0.001f, p.arc, p.kappa, p.P);
  const float kprime = (kp - ki) / 0.001f;
  const float Fx = interp_jnp(s, p.arc, p.Fxd, p.P);
  const float Fy = interp_jnp(s, p.arc, p.Fyd, p.P);
  const float nx = -Fy, ny = Fx;
  const float nrm = std::sqrt(nx * nx + ny * ny);
  const float d = (1.0f / nrm) * (nx * (x - p.x[idx]) + ny * (y - p.y[idx]));
  float pf = psi - crf(std::atan2(double(Fy), double(Fx)));
  pf = crf(std::atan2(double(crf(std::sin(double(pf)))), double(crf(std::cos(double(pf))))));
  const float cp = crf(std::cos(double(pf))), sp = crf(std::sin(double(pf)));
  const float om = 1.0f - d * ki;
  FrenetState o;
  o.x = s;
  o.y = d;
  o.vx = v * cp / om;
  o.vy = v * sp;
  const float pd = psidot - ki * o.vx;
  o.ay = vdot * sp + v * cp * pd;
  const float ax1 = vdot * cp - v * sp * pd;
  const float ax2 = -o.vy * ki - d * kprime * o.vx;
  o.ax = (ax1 * om - (v * cp) * ax2) / (om * om);
  o.psi = pf;
  return o;
}

// The (P+1)^2 inverse, column-major.  Built outside the lock (O(P^3): a few
// seconds at the 2048-point maximum), so other threads keep smoothing paths of
// lengths already cached meanwhile; at most kCacheMax lengths are kept (the
// reference uses one, num_path = 600), the oldest evicted first.  Callers hold
// a shared_ptr, so an eviction never frees a matrix in use.
std::shared_ptr<const std::vector<double>> smoothing_inverse_cm(int P) {
  constexpr size_t kCacheMax = 4;
  static std::mutex mu;
  static std::vector<std::pair<int, std::shared_ptr<const std::vector<double>>>> cache;
  {
    std::lock_guard<std::mutex> lock(mu);
    for (auto& e : cache)
      if (e.first == P) return e.second;
  }
  if (P < 4) throw std::invalid_argument("path smoothing needs >= 4 points");
  const int n = P + 1;
  // cost = 20 D3^T D3 + I (D3: third differences, (P-3) x P), KKT with e0
  std::vector<double> a(size_t(n) * n, 0.0);
  const double c3[4] = {-1.0, 3.0, -3.0, 1.0};  // row r of D3: columns r..r+3
  for (int r = 0; r + 3 < P; ++r)
    for (int u = 0; u < 4; ++u)
      for (int w = 0; w < 4; ++w) a[size_t(r + u) * n + (r + w)] += 20.0 * (c3[u] * c3[w]);
  for (int i = 0; i < P; ++i) a[size_t(i) * n + i] += 1.0;
  a[size_t(P) * n + 0] = 1.0;
  a[size_t(0) * n + P] = 1.0;
  if (!invert(a, n)) throw std::runtime_error("singular path-smoothing KKT");
  auto cm = std::make_shared<std::vector<double>>(size_t(n) * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) (*cm)[size_t(j) * n + i] = a[size_t(i) * n + j];
  std::lock_guard<std::mutex> lock(mu);
  for (auto& e : cache)
    if (e.first == P) return e.second;  // another thread built it meanwhile (the same bits)
  if (cache.size() >= kCacheMax) cache.erase(cache.begin());
  cache.emplace_back(P, cm);
  return cm;
}

void path_smoothing(int P, const float* xw, const float* yw, float thr, float* xo, float* yo) {
  const auto inv_p = smoothing_inverse_cm(P);
  const std::vector<double>& inv = *inv_p;
  const int n = P + 1;
  std::vector<float> alpha(P, 0.0f), d(P, thr), lx(P, 0.0f), ly(P, 0.0f), xs(xw, xw + P), ys(yw, yw + P);
  std::vector<double> rx(n), ry(n), sx(P), sy(P);
  for (int it = 0; it < 10; ++it) {
    for (int i = 0; i < P; ++i) {
      const float bx = xw[i] + d[i] * crf(std::cos(double(alpha[i])));
      const float by = yw[i] + d[i] * crf(std::sin(double(alpha[i])));
      const float linx = -lx[i] - bx, liny = -ly[i] - by;
      rx[i] = -double(linx);
      ry[i] = -double(liny);
    }
    rx[P] = double(xw[0]);
    ry[P] = double(yw[0]);
    // sol = inv [rhs], sequential over the columns (the oracle's order)
    for (int i = 0; i < P; ++i) sx[i] = sy[i] = 0.0;
    for (int j = 0; j < n; ++j) {
      const double* col = inv.data() + size_t(j) * n;
      const double vx = rx[j], vy = ry[j];
      for (int i = 0; i < P; ++i) {
        sx[i] = sx[i] + col[i] * vx;
        sy[i] = sy[i] + col[i] * vy;
      }
    }
    for (int i = 0; i < P; ++i) {
      xs[i] = float(sx[i]);
      ys[i] = float(sy[i]);
      const float wc = xs[i] - xw[i], ws = ys[i] - yw[i];
      alpha[i] = crf(std::atan2(double(ws), double(wc)));
      const float ca = crf(std::cos(double(alpha[i]))), sa = crf(std::sin(double(alpha[i])));
      const float c1 = ca * ca + sa * sa;
      const float c2 = wc * ca + ws * sa;
      const float dd = c2 / c1;
      d[i] = dd < thr ? dd : thr;  // jnp.minimum (no NaN here for finite waypoints)
      lx[i] = lx[i] - (wc - d[i] * ca);
      ly[i] = ly[i] - (ws - d[i] * sa);
    }
  }
  for (int i = 0; i < P; ++i) {
    xo[i] = xs[i];
    yo[i] = ys[i];
  }
}

void path_parameters(int P, const float* x, const float* y, float* Fxd, float* Fyd, float* Fxdd, float* Fydd,
                     float* arc, float* kappa, float* arc_length) {
  if (P < 3) throw std::invalid_argument("path needs >= 3 points");
  for (int i = 1; i < P; ++i) {
    Fxd[i] = x[i] - x[i - 1];
    Fyd[i] = y[i] - y[i - 1];
  }
  Fxd[0] = Fxd[1];
  Fyd[0] = Fyd[1];
  for (int i = 1; i < P; ++i) {
    Fxdd[i] = Fxd[i] - Fxd[i - 1];
    Fydd[i] = Fyd[i] - Fyd[i - 1];
  }
  Fxdd[0] = Fxdd[1];
  Fydd[0] = Fydd[1];
  double acc = 0.0;
  arc[0] = 0.0f;
  for (int i = 0; i + 1 < P; ++i) {
    acc += double(std::sqrt(Fxd[i] * Fxd[i] + Fyd[i] * Fyd[i]));
    arc[i + 1] = float(acc);
  }
  for (int i = 0; i < P; ++i) {
    const float s2 = Fxd[i] * Fxd[i] + Fyd[i] * Fyd[i];
    kappa[i] = (Fydd[i] * Fxd[i] - Fxdd[i] * Fyd[i]) / crf(std::pow(double(s2), 1.5));
  }
  if (arc_length) *arc_length = arc[P - 1];
}

}  // namespace mpcmmd
