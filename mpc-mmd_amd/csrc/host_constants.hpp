// Batch-invariant constants of the optimizer, computed on the host in fp64.
// Restates CEM.__init__ / Helper.__init__ (synthetic_static_obs/optimizer/
// cem.py:17-199, cem_helper.py:10-120) and the matrices the reference rebuilds
// inside every jitted call (guess QP cem_helper.py:207-217, projection KKT
// projection.py:145-156, Bernstein fit cem_helper.py:556).  The reference
// solves each of these batch-invariant systems with an fp32 LU per call; here
// they are inverted once in fp64 and applied as fp64 GEMVs on the device.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mpcmmd {

constexpr int kNum = 100;   // planning points (cem.py:38)
constexpr int kNvar = 11;   // Bernstein degree 10 (cem.py:50)
constexpr int kLane = 2 * (kNum - 1);

struct ProblemConsts {
  // scalars (Appendix B of SURVEY.md)
  double a_obs = 4.25, b_obs = 2.75, wheel_base = 2.5;
  double v_min = 0.1, v_max = 30.0, a_max = 18.0, steer_max = 0.6;
  double t_fin = 15.0, dt = 0.15;
  double k_p_v = 2.0, k_p = 2.0;
  double y_lb = -2.25, y_ub = 2.25, K_steer = 0.01;
  double alpha_mean = 0.6, alpha_cov = 0.6, lamda = 0.9;
  double ker_wt = 1000.0, alpha_quant = 0.98;
  double y_des_1 = -1.75, y_des_2 = 1.75;
  // CARLA variant (carla/optimizer/cem.py:29, 152-153, 182)
  bool carla = false;
  double a_centr = 1.5, init_mu_x = 0.3, init_mu_y = 0.0, init_sigma_x = 0.05, init_sigma_y = 0.1;
  double gamma_lane_des = 0.3;
  int H = 0;
  // fp32-rounded basis, stored as double [100][11]
  std::vector<double> P, Pd, Pdd;
  std::vector<double> P64, Pd64, Pdd64;   // unrounded (the reference's self.P etc.)
  std::vector<double> P_prime;            // [H][11], fp32-rounded
  std::vector<double> guess_kinv_x;       // [14][14]
  std::vector<double> guess_kinv_y;       // [15][15]
  std::vector<double> guess_colsum_x;     // [4][11]
  std::vector<double> guess_colsum_y;     // [4][11]
  std::vector<double> proj_kinv_x;        // [14][14]
  std::vector<double> proj_kinv_y;        // [15][15]
  std::vector<double> fit;                // [11][H] = (P'^T P' + 0.05 I)^-1 P'^T
};

// Constant-speed / lane-keeping QP that generates the dynamic obstacles'
// trajectories: obs_data.compute_obs_guess
// (synthetic_dynamic_obs/obs_data_generate_dynamic.py:73-109).  One segment
// over the whole 100-point plan (unlike the 4-segment guess QP of the
// optimizer), smoothness weight 100, k_p_v = k_p = 2.
struct DynObsConsts {
  std::vector<double> P;         // [100][11] fp32-rounded basis
  std::vector<double> kinv_x;    // [14][14]
  std::vector<double> kinv_y;    // [15][15]
  std::vector<double> colsum_x;  // [11] column sums of A_vd = Pdd - k_p_v Pd
  std::vector<double> colsum_y;  // [11] column sums of A_pd = Pdd - k_p P
};
DynObsConsts build_dyn_obs_consts();

// x_traj/y_traj [num_obs][100] fp32 for obstacles starting at (x0, y0) with
// speeds (vx0, vy0), zero acceleration, tracking speed v_des[i] and lane
// y_des (dynamic main_mpc.py:116-126 uses y_des = -1.75).
void dyn_obs_traj(const DynObsConsts& c, int num_obs, const float* x0, const float* y0, const float* vx0,
                  const float* vy0, const float* v_des, float y_des, float* x_traj, float* y_traj);

// variant: 0 static, 1 dynamic, 2 CARLA Town05, 3 CARLA Town10HD.  Throws std::runtime_error on a singular
// matrix (never for valid H >= 2).
ProblemConsts build_constants(int num_prime, int variant);

// KKT inverses of the CARLA det projection (carla/optimizer/projection_det.py:
// 149-160): the projection KKT cost matrices plus rho_obs A_obs^T A_obs, A_obs
// = tile(P, (num_obs, 1)) accumulated row by row (oracle/problem.py: det_kinv
// in the same order).  kx [14][14], ky [15][15].
void det_projection_kinv(const ProblemConsts& c, int num_obs, std::vector<double>& kx, std::vector<double>& ky);

// numpy.linspace(start, stop, num) (fp64, endpoint included).
std::vector<double> linspace(double start, double stop, int num);

// Bernstein degree-10 basis on grid t, same operation order as
// oracle/problem.py:bernstein_order10 (so the two agree bit for bit).
void bernstein10(const std::vector<double>& t, double tmin, double tmax, std::vector<double>& P,
                 std::vector<double>& Pd, std::vector<double>& Pdd);

// In-place Gauss-Jordan inverse with partial pivoting (n x n, row-major).
bool invert(std::vector<double>& a, int n);

}  // namespace mpcmmd
