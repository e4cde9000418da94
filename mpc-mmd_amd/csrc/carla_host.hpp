// Host pieces of the CARLA optimizer variant (carla/optimizer/*.py of the
// reference, "C/opt/" below): the path preprocessing main_carla.py runs every
// tick (custom_path_smoothing, compute_path_parameters, global_to_frenet_obs)
// and the per-solve setup of compute_cem_mmd / compute_cem_cvar (noisy
// initial states and their Frenet boundary vectors).  fp32 state in the
// reference's operation order; transcendentals evaluated in fp64 and rounded
// once; small dense products in fp64 (oracle/carla.py restates the same).
#pragma once
#include <cstdint>
#include <memory>
#include <vector>

namespace mpcmmd {

// One path as the solve takes it (C/main_carla.py:366-382).
struct PathView {
  int P = 0;
  const float *x = nullptr, *y = nullptr, *arc = nullptr, *Fxd = nullptr, *Fyd = nullptr, *kappa = nullptr;
};

// jnp.interp (jax 0.3.23): fp[i-1] + ((x - xp[i-1]) / dx) * df with
// i = clip(searchsorted(xp, x, 'right'), 1, P-1); fp[0] / fp[P-1] outside.
float interp_jnp(float x, const float* xp, const float* fp, int P);

// argmin_j sqrt((xp_j - x)^2 + (yp_j - y)^2), first minimum (first NaN).
int closest_index(float x, float y, const float* xp, const float* yp, int P);

// Helper.global_to_frenet (C/opt/cem_helper.py:348-388) of one state.
struct FrenetState {
  float x, y, vx, vy, ax, ay, psi;
};
FrenetState global_to_frenet(const PathView& path, float x, float y, float v, float vdot, float psi, float psidot);

// inv([[20 D3^T D3 + I, e0^T], [e0, 0]]) for P path points
// (C/opt/cem_helper.py:115-129), fp64 Gauss-Jordan, stored column-major
// ((P+1) x (P+1)); the last few P cached (built outside the cache lock).
std::shared_ptr<const std::vector<double>> smoothing_inverse_cm(int P);

// Helper.custom_path_smoothing (C/opt/cem_helper.py:279-318, 391-410).
void path_smoothing(int P, const float* x_wp, const float* y_wp, float threshold, float* x_out, float* y_out);

// Helper.compute_path_parameters (C/opt/cem_helper.py:321-345); arc-length
// cumsum in fp64.
void path_parameters(int P, const float* x, const float* y, float* Fxd, float* Fyd, float* Fxdd, float* Fydd,
                     float* arc, float* kappa, float* arc_length);

}  // namespace mpcmmd
