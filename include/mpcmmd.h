/*
 * mpcmmd.h -- C ABI of libmpcmmd.so, the MI355X (gfx950) implementation of the
 * MMD / CVaR / SAA CEM-projection optimizer of Basant1861/MPC-MMD.
 *
 * The reference has no native code and no FFI: its optimizer is the Python
 * class `CEM` in synthetic_static_obs/optimizer/cem.py (pure JAX).  This ABI is
 * what that class's drop-in replacement (mpc-mmd_amd/optimizer/cem.py) binds
 * through ctypes; each entry point names the reference interface it replaces.
 * Plain C types only: no torch / HIP types in any signature (a stream is a
 * `void*` holding a hipStream_t).
 *
 * Threading: a handle is bound to one HIP device and one stream and is not
 * thread-safe; use one handle per thread / GPU.  Every call returns an int
 * status (0 = ok, < 0 = error; mpcmmd_last_error() has the message, thread
 * local).
 */
#ifndef MPCMMD_H
#define MPCMMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 4: MPCMMD_COST_DET (CARLA compute_cem_det), mpcmmd_handle_info */
#define MPCMMD_ABI_VERSION 4

/* status codes */
#define MPCMMD_OK 0
#define MPCMMD_E_INVALID (-1)     /* bad argument / shape */
#define MPCMMD_E_HIP (-2)         /* HIP runtime error (message has details) */
#define MPCMMD_E_UNSUPPORTED (-3) /* configuration outside what is built */
#define MPCMMD_E_STATE (-4)       /* call order (e.g. iterate before begin) */

/* cost variants: CEM.compute_cem_{mmd_opt,mmd_random,cvar,saa}
 * (synthetic_static_obs/optimizer/cem.py:201,335,464,590) */
#define MPCMMD_COST_MMD_OPT 0
#define MPCMMD_COST_MMD_RANDOM 1
#define MPCMMD_COST_CVAR 2
#define MPCMMD_COST_SAA 3
/* CARLA handles only: CEM.compute_cem_det of carla/optimizer/cem.py:633-790,
 * the deterministic baseline -- one noisy initial state, the projection with
 * its obstacle terms live (projection_det.py), no rollouts and no risk terms */
#define MPCMMD_COST_DET 4

/* noise models: Helper noise=="gaussian" / else beta (optimizer/cem_helper.py:405) */
#define MPCMMD_NOISE_GAUSSIAN 0
#define MPCMMD_NOISE_BETA 1

/* scenario constants: synthetic_static_obs vs synthetic_dynamic_obs
 * (y_lb,y_ub at optimizer/cem.py:155; K_steer at optimizer/cem_helper.py:24) */
#define MPCMMD_VARIANT_STATIC 0
#define MPCMMD_VARIANT_DYNAMIC 1
/* The CARLA optimizer (carla/optimizer/cem.py, CEM(num_reduced_sqrt,
 * num_mother, num_obs, noise_level, num_prime, noise, town, ...)): town
 * "Town05" / "Town10HD" select y_lb, y_ub, y_des (cem.py:161-166).  A CARLA
 * handle solves through mpcmmd_carla_begin / mpcmmd_carla_solve only. */
#define MPCMMD_VARIANT_CARLA_TOWN05 2
#define MPCMMD_VARIANT_CARLA_TOWN10HD 3

/* Replaces CEM.__init__(num_reduced, num_obs, noise_level, num_prime, noise,
 * acc_const_noise, steer_const_noise) (optimizer/cem.py:17-18).  num_batch is
 * the reference's hard-coded 100 (cem.py:137) made configurable. */
typedef struct mpcmmd_config {
  int32_t num_reduced;     /* n: samples per candidate (baseline) / reduced set (mmd_opt) */
  int32_t num_obs;         /* O */
  float noise_level;       /* sigma_acc = sigma_steer (cem.py:168-169) */
  int32_t num_prime;       /* H: rollout horizon */
  int32_t noise;           /* MPCMMD_NOISE_* */
  float acc_const_noise;
  float steer_const_noise;
  int32_t num_batch;       /* B (reference: 100) */
  int32_t variant;         /* MPCMMD_VARIANT_* */
  int32_t maxiter_cem;     /* outer CEM iterations (reference: 20, cem.py:89) */
  int32_t device;          /* HIP device ordinal */
  uint32_t seed;           /* key word 1 of the internal Philox streams */
} mpcmmd_config;

/* External draws (the parity contract): every standard normal the solve
 * consumes, host fp32 row-major.  A NULL field selects the internal Philox
 * stream for that tensor.  Shapes (T = maxiter_cem, S = num_reduced,
 * M = num_reduced^2):
 *   pop0     [B][8]             sampling_param, fixed key      (cem_helper.py:122-150)
 *   roll     [T][3][S][H]       acc / steer / const noise rows (cem_helper.py:405-441)
 *   resample [T][B-5][8]        compute_shifted_samples        (cem_helper.py:292)
 *   beta_z0  [100][M+1]         beta-CEM initial samples       (compute_beta.py:41-49)
 *   beta_z   [20][89][M+1]      beta-CEM resamples             (compute_beta.py:63)
 * Beta noise depends on the controls and is always internal. */
typedef struct mpcmmd_draws {
  const float* pop0;
  const float* roll;
  const float* resample;
  const float* beta_z0;
  const float* beta_z;
  /* CARLA: [R][4] normals of the noisy initial states, R = n^2 (mmd_opt) or
   * n (cvar) (compute_noisy_init_state(_baseline), carla/optimizer/
   * cem_helper.py:660-715) */
  const float* init_eps;
} mpcmmd_draws;

/* Return of compute_cem_* (cem.py:324-333 / 456-462): the obstacle-cost
 * elite 0 of the LAST outer iteration.  beta must point to >= n floats for
 * mmd_opt (may be NULL otherwise).  The trace pointers are optional (NULL =
 * not copied) and receive per-iteration elite index sets for parity tests:
 * elite_proj [T][B] (argsort of res_norm), elite_obs [T][20] (candidate
 * indices), elite_cem [T][5] (indices into the 20). */
typedef struct mpcmmd_result {
  float cx[11];
  float cy[11];
  float cost_lane;
  float cost_obs;
  float sigma;          /* mmd_opt */
  float res_beta[20];   /* mmd_opt */
  float* beta;          /* [n], mmd_opt */
  int32_t* elite_proj;
  int32_t* elite_obs;
  int32_t* elite_cem;
  /* CARLA return (carla/optimizer/cem.py:413-441): steering_best [100],
   * v_best [100] (optional, NULL = not written), mean_param after the last
   * iteration */
  float* steering;
  float* v_best;
  float mean_param[8];
} mpcmmd_result;

typedef struct mpcmmd_handle mpcmmd_handle;

int32_t mpcmmd_abi_version(void);
const char* mpcmmd_last_error(void);

/* Number of visible HIP devices (0 when none; never fails). */
int32_t mpcmmd_device_count(void);

/* CEM.__init__: allocates every device buffer and uploads the
 * batch-invariant matrices.  No allocation happens after this. */
int mpcmmd_create(const mpcmmd_config* cfg, mpcmmd_handle** out);
void mpcmmd_destroy(mpcmmd_handle* h);

/* A handle that solves up to max_configs configurations of the same
 * CEM(...) shape in one go (mpcmmd_solve_batch): every stage is ONE launch
 * over (configuration x candidate), so the reference's num_batch = 100 sweep
 * (S/main_mpc.py:106-128, 200 independent configurations) fills the GPU.
 * Buffers are sized for max_configs * num_batch candidates (<= 65535).
 * mpcmmd_create(cfg, out) == mpcmmd_create_batch(cfg, 1, out). */
int mpcmmd_create_batch(const mpcmmd_config* cfg, int32_t max_configs, mpcmmd_handle** out);
int32_t mpcmmd_max_configs(mpcmmd_handle* h);

/* Implementation choices of a handle, fixed at create (no reference
 * counterpart: the reference has one JAX program).  name:
 *   "gen_wave"     1: the beta-CEM generators by one wave per 16-position block
 *                  (k_bgen_wave, fp64 MFMA), 0: a quad per block (k_bgen).  The
 *                  two sum in different orders, so their bits differ (both
 *                  within the parity tolerances).  Default: 1 when the handle's
 *                  capacity max_configs * num_batch <= 512 and num_reduced <= 24
 *                  -- the SAME problem can therefore give different bits on a
 *                  handle of 512 and one of 1024 candidates, or with another
 *                  max_configs.  Pin it with the environment variable
 *                  MPCMMD_GENWAVE=0/1 (read at create) to compare batch sizes.
 *   "select_prep"  1: for cvar / saa / mmd_random the risk launch (stage 2) also
 *                  sorts the residuals and forms compute_cost's norms, so stage 3
 *                  needs stage 2 of the same iteration (MPCMMD_SELECT_PREP=0: in
 *                  stages 1 and 3; same bits either way)
 *   "fused_small"  1: small batches run the 20 beta-iterations as one launch
 *                  (k_bcem_small; same bits as the per-iteration kernels)
 *   "groups"       beta-CEM candidate groups on their own streams (same bits)
 *   "capacity"     max_configs * num_batch
 * Writes *value; MPCMMD_E_INVALID for an unknown name. */
int mpcmmd_handle_info(mpcmmd_handle* h, const char* name, int64_t* value);

/* Run on a caller-owned hipStream_t instead of the handle's own stream. */
int mpcmmd_set_stream(mpcmmd_handle* h, void* hip_stream);
void* mpcmmd_get_stream(mpcmmd_handle* h);

/* CEM.compute_cem_{mmd_opt,mmd_random,cvar,saa}(idx_mpc, init_state,
 * mean_param_init, cov_param_init, x_obs_traj, y_obs_traj, v_des)
 * (cem.py:201-204 etc.).  x_obs / y_obs are [O][100] row-major.  draws may
 * be NULL (internal RNG).  Synchronous. */
int mpcmmd_solve(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                 const float mean[8], const float cov[64], const float* x_obs, const float* y_obs,
                 float v_des, const mpcmmd_draws* draws, mpcmmd_result* out);

/* The same solve in three steps (what mpcmmd_solve does), for callers that
 * time or interleave work: begin uploads inputs and builds the initial carry
 * (sampling_param, compute_boundary_vec; cem.py:206-219); iterate enqueues
 * outer iterations [t_begin, t_begin+count) (the lax_cem body, cem.py:221-315)
 * asynchronously on the handle's stream; finish synchronises and downloads
 * the result of the last enqueued iteration. */
int mpcmmd_begin(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                 const float mean[8], const float cov[64], const float* x_obs, const float* y_obs,
                 float v_des, const mpcmmd_draws* draws);
int mpcmmd_iterate(mpcmmd_handle* h, int32_t t_begin, int32_t count);
int mpcmmd_finish(mpcmmd_handle* h, mpcmmd_result* out);
int mpcmmd_sync(mpcmmd_handle* h);

/* n_cfg <= max_configs independent solves of the loop of S/main_mpc.py:106-128
 * (compute_cem_* per configuration) in one batch.  Arrays carry a leading
 * configuration axis: idx_mpc [n], init_state [n][6], mean [n][8], cov
 * [n][64], x_obs / y_obs [n][O][100], v_des [n]; out [n].  Configuration g
 * uses the internal RNG streams keyed by idx_mpc[g], so its result is
 * bit-identical to mpcmmd_solve of that configuration alone (external draws
 * are a single-configuration feature).  Synchronous. */
int mpcmmd_solve_batch(mpcmmd_handle* h, int32_t n_cfg, int32_t cost_kind, const int32_t* idx_mpc,
                       const float* init_state, const float* mean, const float* cov, const float* x_obs,
                       const float* y_obs, const float* v_des, mpcmmd_result* out);
/* The batch split like begin / iterate / finish (iterate is shared). */
int mpcmmd_begin_batch(mpcmmd_handle* h, int32_t n_cfg, int32_t cost_kind, const int32_t* idx_mpc,
                       const float* init_state, const float* mean, const float* cov, const float* x_obs,
                       const float* y_obs, const float* v_des);
int mpcmmd_finish_batch(mpcmmd_handle* h, int32_t n_cfg, mpcmmd_result* out);

/* ---- CARLA variant ---------------------------------------------------------
 * The path arguments of compute_cem_mmd / compute_cem_cvar
 * (carla/optimizer/cem.py:217-220, 444-448; main_carla.py:366-382), num_path
 * points each (reference: 600), fp32. */
typedef struct mpcmmd_path {
  int32_t num_path;
  const float* x_path;
  const float* y_path;
  const float* arc_vec;
  const float* Fx_dot;
  const float* Fy_dot;
  const float* kappa;
} mpcmmd_path;

/* CEM.compute_cem_mmd (cost_kind MPCMMD_COST_MMD_OPT) / compute_cem_cvar
 * (MPCMMD_COST_CVAR) / compute_cem_det (MPCMMD_COST_DET, num_obs <= 32) of
 * the CARLA optimizer (carla/optimizer/cem.py:217-790):
 * init_state = init_state_global (x, y, v, vdot, psi, psidot), x_obs / y_obs
 * the Frenet obstacle tracks [O][100], path as above.  begin then
 * mpcmmd_iterate / mpcmmd_finish, or solve in one call.  out->steering,
 * out->v_best, out->mean_param carry the reference's return
 * (cx, cy, v_best, steering_best, mean_param). */
int mpcmmd_carla_begin(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                       const float mean[8], const float cov[64], const float* x_obs, const float* y_obs, float v_des,
                       const mpcmmd_path* path, const mpcmmd_draws* draws);
int mpcmmd_carla_solve(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                       const float mean[8], const float cov[64], const float* x_obs, const float* y_obs, float v_des,
                       const mpcmmd_path* path, const mpcmmd_draws* draws, mpcmmd_result* out);

/* Helper.custom_path_smoothing(x_waypoints, y_waypoints, threshold)
 * (carla/optimizer/cem_helper.py:279-318, 391-410): 10 ADMM iterations of the
 * jerk-smoothing QP; the (num_path+1)^2 KKT inverse is built once per
 * num_path (fp64).  Host; no GPU needed. */
int mpcmmd_path_smoothing(int32_t num_path, const float* x_wp, const float* y_wp, float threshold, float* x_path,
                          float* y_path);
/* Helper.compute_path_parameters(x_path, y_path) (cem_helper.py:321-345).
 * Host; arc_length may be NULL. */
int mpcmmd_path_parameters(int32_t num_path, const float* x_path, const float* y_path, float* Fx_dot, float* Fy_dot,
                           float* Fx_ddot, float* Fy_ddot, float* arc_vec, float* kappa, float* arc_length);
/* Helper.global_to_frenet (cem_helper.py:348-388) of count states; out
 * [count][7] = (x, y, vx, vy, ax, ay, psi) in the Frenet frame
 * (global_to_frenet_obs, :171-200, is this with vdot = psidot = 0 and
 * v = |(vx, vy)|).  Host. */
int mpcmmd_global_to_frenet(const mpcmmd_path* path, int32_t count, const float* x, const float* y, const float* v,
                            const float* vdot, const float* psi, const float* psidot, float* out);

/* Whole-solve HIP graphs: with enable != 0, mpcmmd_iterate(h, 0, T) captures
 * the solve's launch sequence once per (cost, path length, external draws,
 * configurations) and replays it with one hipGraphLaunch (handles whose
 * launches use one stream, i.e. fewer than 1024 candidates).  Results are
 * identical to the launched sequence.  Default off (environment MPCMMD_GRAPH=1
 * turns it on at create). */
int mpcmmd_set_graphs(mpcmmd_handle* h, int32_t enable);

/* Per-kernel HIP-event timing (on the handle's stream).  When enabled, every
 * launch of every kernel is bracketed by events; mpcmmd_kernel_times returns,
 * per kernel id, the number of launches and the total milliseconds since the
 * last reset.  Kernel ids: see mpcmmd_kernel_name. */
int mpcmmd_profile(mpcmmd_handle* h, int32_t enable);
int mpcmmd_kernel_times(mpcmmd_handle* h, int32_t* launches, double* total_ms, int32_t max_kernels);
const char* mpcmmd_kernel_name(int32_t id);

/* Named device buffers, for stage-level parity tests (read / overwrite the
 * scan carry and intermediates between stages).  Names and sizes: see
 * mpcmmd_buffer_info; the name "*" gives the total bytes of every buffer of
 * the handle.  Tests can cap a handle's device memory with the environment
 * variable MPCMMD_MAX_HANDLE_BYTES (read at create): buffers past the cap fail
 * with the runtime's own out-of-memory error. */
int mpcmmd_buffer_info(mpcmmd_handle* h, const char* name, size_t* bytes);
int mpcmmd_read(mpcmmd_handle* h, const char* name, void* dst, size_t bytes);
int mpcmmd_write(mpcmmd_handle* h, const char* name, const void* src, size_t bytes);

/* Stage entry points: run one kernel of iteration t on the current device
 * state (the stages mpcmmd_iterate chains):
 *   0 noise      (internal RNG draws of iteration t)
 *   1 front      compute_x_guess + compute_projection + compute_controls
 *                (cem_helper.py:169-230, projection.py:276-323, cem_helper.py:540-551)
 *   2 risk       noisy rollouts + collision residual + risk reducer per candidate
 *                (cem_helper.py:402-538, costs.py:50-234, compute_beta.py:93-157)
 *   3 select     argsorts, compute_cost, elites, compute_shifted_samples
 *                (cem.py:233-315, cem_helper.py:232-314).  With the select
 *                preparation on (mpcmmd_handle_info "select_prep": cvar / saa /
 *                mmd_random) stage 2 sorts the residuals and forms the cost
 *                norms, so stage 3 needs stage 2 of the same iteration after
 *                stage 1 (else MPCMMD_E_INVALID)
 * cost = mmd_opt splits stage 2 into sub-stages (t = outer iteration for 4, 8;
 * t = beta-CEM iteration 0..19 for 5-7):
 *   4 mother     noisy rows, n^2 mother rollouts, Bernstein fit (cem_helper.py:469-564)
 *   5 bsample    beta-CEM samples + top-n |beta| rows     (compute_beta.py:41-68, 117-118)
 *   6 bkernel    kernel row sums, reduced QP, QP cost     (compute_beta.py:70-91, 120-129)
 *   7 belite     elites, mean, next generators             (compute_beta.py:51-68, 133-157)
 *   8 mmdfinal   reduced rollouts, MMD obs / lane          (costs.py:121-135, 173-186)
 * Buffer "beta_z" holds the device layout [20][P][96], P = M+1 rounded up to
 * 16, zero padded (transposed on upload in mpcmmd_begin; mpcmmd_write writes
 * it raw). */
int mpcmmd_run_stage(mpcmmd_handle* h, int32_t stage, int32_t t);

/* Host-side batch-invariant constants (no GPU needed): fills dst with the
 * fp64 values of `name` ("P","Pdot","Pddot" [100][11] (fp32-rounded),
 * "P_prime" [H][11], "guess_kinv_x" [14][14], "guess_kinv_y" [15][15],
 * "proj_kinv_x", "proj_kinv_y", "fit" [11][H], "det_kinv_x", "det_kinv_y"
 * (the CARLA det projection's, for cfg->num_obs obstacles)).  Returns element count, or
 * < 0 on error / when count is too small. */
int mpcmmd_host_constant(const mpcmmd_config* cfg, const char* name, double* dst, size_t count);

/* Dynamic-obstacle trajectories of the synthetic_dynamic_obs driver:
 * obs_data.compute_boundary_vec + obs_data.compute_obs_guess
 * (synthetic_dynamic_obs/obs_data_generate_dynamic.py:56-109, called per
 * obstacle at synthetic_dynamic_obs/main_mpc.py:116-126).  Obstacle i starts
 * at (x0[i], y0[i]) with speed (vx0[i], vy0[i]) and zero acceleration and
 * tracks speed v_des[i] (obs_data.sampling_param, :111-133) and lane y_des
 * (the driver passes -1.75).  Writes x_traj, y_traj [num_obs][100].  Host
 * fp64 KKT (inverted once), fp32 output; no GPU needed. */
int mpcmmd_obs_dynamic_traj(int32_t num_obs, const float* x0, const float* y0, const float* vx0, const float* vy0,
                            const float* v_des, float y_des, float* x_traj, float* y_traj);

/* Monte-Carlo validation of saved optima on the GPU: synthetic_static_obs/
 * validation.py compute_stats (:134-171) for num_cfg configurations at
 * once.  Per configuration k: controls of the saved trajectory (cx, cy)
 * (compute_controls :122-132), num_rollouts noisy fp64 rollouts from
 * init_state (compute_rollout_complete :42-101), then
 *   count[k]      = max over (obstacle, step) of #rollouts inside the ellipse
 *   count_lane[k] = max_step #(y < y_lb) + max_step #(y > y_ub)
 * (:153-169).  x_obs / y_obs: [num_cfg][num_obs][100] obstacle tracks
 * (compute_obs_trajectories).  draws: [num_cfg][3][num_rollouts][num_prime]
 * fp64 -- gaussian: the standard normals of acc, steer, const noise; beta:
 * the Beta(2|acc|, 5|acc|) and Beta(2|steer|+1e-5, 5|steer|+1e-5) draws and
 * the const normals -- or NULL for the library's Philox streams keyed by
 * (keys[k], seed).  Synchronous; allocates its own device buffers. */
typedef struct mpcmmd_validate_args {
  int32_t num_cfg, num_obs, num_prime, num_rollouts;
  int32_t noise;          /* MPCMMD_NOISE_* */
  int32_t variant;        /* MPCMMD_VARIANT_* (y_lb, y_ub, K_steer) */
  double noise_level, acc_const_noise, steer_const_noise;
  uint32_t seed;
  int32_t device;
  const double* cx;       /* [num_cfg][11] */
  const double* cy;
  const double* init_state; /* [num_cfg][6] */
  const float* x_obs;
  const float* y_obs;
  const double* draws;
  const uint32_t* keys;   /* [num_cfg] (validation.py seeds np.random with the config key) */
  int32_t* count;         /* [num_cfg] out */
  int32_t* count_lane;    /* [num_cfg] out */
} mpcmmd_validate_args;
int mpcmmd_validate(const mpcmmd_validate_args* args);

#ifdef __cplusplus
}
#endif
#endif /* MPCMMD_H */
