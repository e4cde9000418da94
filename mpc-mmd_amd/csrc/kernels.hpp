// Kernel argument block and launch declarations.  One struct for every
// kernel keeps the host side simple: it is passed by value (kernarg segment).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#define HDI_CONST __host__ __device__ __forceinline__ constexpr

namespace mpcmmd {

constexpr int kMaxH = 100;
constexpr int kMaxReduced = 64;        // n for mmd_opt (M = n^2 <= 4096) -- see DESIGN.md
constexpr int kBetaSamples = 100;      // compute_beta.py:14
constexpr int kBetaIters = 20;         // compute_beta.py:15
constexpr int kBetaElite = 11;         // compute_beta.py:26
constexpr int kEliteCost = 20;         // cem.py:140
constexpr int kCnormStride = 12;       // doubles per candidate of Params::cnorm (11 norms)
constexpr int kElite = 5;              // cem.py:138
constexpr int kResultStride = 11 + 11 + 2 + 1 + 20 + kMaxReduced;  // cx, cy, lane, obs, sigma, res_beta, beta
// generators per candidate: two planes of pos_pad(M) rows x kGenRow doubles,
// W (features 0..10, slot 11 zero) then U (features 0..10, the position's
// fp32-rounded elite mean in slot 11), and L_jj in Params::genm.  The sampler
// feeds slot 11 through the 16x16x4 MFMA operands unmasked: W's zero slot
// keeps the mean out of W U^T, and row 11 of its S_pre is 1, so U S adds the
// mean.  192 B per position; planes, not interleaved rows, so k_bgen's U
// reads and W writes never share a line.
constexpr int kGenRow = 12;
constexpr int kGenStride = 2 * kGenRow;  // doubles per position and candidate
constexpr int kGenW = 0, kGenMean = 11;
HDI_CONST size_t gen_uplane(int Pp) { return size_t(Pp) * kGenRow; }  // U plane offset
HDI_CONST int ygen_stride(int M) { return ((M + 1) + 31) & ~31; }
// beta-CEM sample generation works on pairs of blocks of 16 positions and
// tiles of 16 samples: generators (gen, genm) and the device normals (beta_z)
// are padded with zeros to pos_pad(M) positions, beta_z rows and ygen to
// kBzCols samples
constexpr int kBzCols = 96;
// beta_z device layout per iteration: blocks of 16 positions x kBzCols
// samples, each block the sampler's lane image [6 chunks][64 lanes][4 floats]:
// lane r + 16 h holds positions p0 + 4 k + h (k < 4) of samples 32 u + 2 r + e
// (u < 3, e < 2) at index 6 k + 2 u + e, so a wave reads a block's normals in
// six fully coalesced float4 loads
HDI_CONST size_t bz_index(int j, int s) {
  const int jj = j & 15, lane = ((s & 31) >> 1) + 16 * (jj & 3), idx = 6 * (jj >> 2) + 2 * (s >> 5) + (s & 1);
  return size_t(j >> 4) * (16 * kBzCols) + (idx >> 2) * 256 + lane * 4 + (idx & 3);
}HDI_CONST int pos_pad(int M) { return ((M + 1) + 31) & ~31; }  // whole pairs of 16-blocks
// row stride (floats) of the mother distance matrix: whole 256-column blocks
// (k_bkernel: a wave holds a row as one float4 per lane and block); pad
// columns hold +inf
HDI_CONST int dist_stride(int M) { return (M + 255) & ~255; }
// floats per sample of Params::bkred: the n (n - 1) / 2 strict lower triangle
// rounded to whole 16-byte groups (the QP kernel stages rows as float4)
HDI_CONST int tri_stride(int n) { return ((n * (n - 1) / 2) + 3) & ~3; }
// floats per mother row of Params::featr (22 features, 2 zero pads: six float4)
constexpr int kFeatStride = 24;
// series record of a distance row (Params::bmom, k_bmoment): P_0..P_11, R, pad
constexpr int kMom = 12;
constexpr int kMomStride = 16;
constexpr int kMomR = 12;
constexpr int kMaxSplit = 8;  // workgroups per candidate of the row-sum kernels
constexpr int kMaxPath = 2048;  // CARLA path points (the reference's num_path = 600)
constexpr int kMaxDetObs = 32;  // obstacles of compute_cem_det (k_front's per-lane non-finite mask: 2 bits each)

struct Params {
  // shapes / configuration.  A launch covers G configurations of B
  // candidates each (mpcmmd_solve_batch; G = 1 for mpcmmd_solve): candidate
  // arrays are indexed by the global candidate b in [0, Bt), Bt = G B, and
  // the per-configuration arrays below are [G][...] (cfg_of)
  int32_t B, S, H, O, n, M, T;
  int32_t G, Bt;
  int32_t cost;      // MPCMMD_COST_*
  int32_t noise;     // MPCMMD_NOISE_*
  uint32_t seed;
  // candidate range of one beta-CEM launch: [b0, b0 + nb) (the beta-iteration
  // kernels run per candidate group, each group on its own stream)
  int32_t b0, nb;
  float sigma_acc, sigma_steer, acc_const, steer_const, K_steer;
  float y_lb, y_ub;
  float w_obs, w_lane;
  // constants (device)
  const float* basis;      // [3][100][11] fp32: P, Pd, Pdd
  const double* guess_g;   // [2][11][4]  (x: v-columns, y: y-columns)
  const double* proj_m;    // [2][11][11] (Kinv[:11,:11] for x, y)
  const double* fit;       // [11][H]
  // per configuration
  const int32_t* idx_mpc;  // [G]
  const float* v_des;      // [G]
  const double* solve_c;   // [G][4][11] per solve: guess h_x, h_y, proj e_x, e_y
  const float* obs;        // [G][2][O][H] x_obs, y_obs (first H columns)
  const float* st0;        // [G][8] initial rollout state
  // noise tables, device layout (iteration-major, sample-minor for coalescing)
  const float* roll;       // [G][T][3][H][S]
  const float* resample;   // [G][T][B-5][8]
  float* bplane;           // [Bt][2][H][S] Beta draws (acc, steer) of the baseline rollouts (beta noise)
  uint32_t* bfix;          // [Bt*H*S] elements k_beta_planes deferred to k_beta_fix
  uint32_t* bfix_n;        // their count (zeroed by k_gamma_tab)
  double* gtab;            // [G][gamma_tab_size] Beta-noise attempt tables of the current iteration
  void* mttab;             // [H][Bt] gamma constants per (step, candidate) of the fused rollouts (k_mt_tab)
  float* rbar;             // [3][Bt][S] per-row maxima (collision, lane lb, ub) of the fused rollouts
  int32_t select_prep;     // the risk launch also sorts the residuals and forms the cost norms (cost.hpp)
  int32_t beta_dump;       // fused rollouts also store their Beta draws in bplane (MPCMMD_BETA_DUMP, tests)
  int32_t risk_rows;       // 1 (default): the row-lane rollouts over Beta planes; 0: fused (MPCMMD_RISK_FUSED=1)
  int32_t* bdlist;         // [Bt][100 n] the flagged (direct) pairs of a beta-iteration, appended by k_bkernel
  int32_t* bdlcount;       // [Bt][20] their count per beta-iteration (zeroed by k_bselect of that iteration)
  int32_t dir_pairs;       // 1: k_bdirect_pairs (a wave per 8 listed pairs); 0: k_bdirect (rows sorted in LDS)
  int32_t qp_small;        // k_bqp at 64 threads (16 QPs) per workgroup for launches of < 2 workgroups per CU
  int32_t sel_cap;         // k_bselect: at most this many single-wave workgroups per candidate (default 16)
  int32_t dir_waves;       // waves per k_bdirect workgroup (4, 8 or 16)
  int32_t ker_target;      // k_bkernel parts: enough for this many workgroups per launch (default 512)
  int32_t dir_target;      // k_bdirect parts: enough for this many workgroups per launch (default 2048)
  int32_t mom_rows;        // 1 (default): k_bmoment_rows (16 lanes per distance row, 4 rows per wave); 0: a wave
                           // per row (MPCMMD_MOM_ROWS=0)
  double mom_amax;         // k_bmoment's first-iteration direct test a > mom_amax: kSeriesAMax (1.0), k_bkernel's;
                           // MPCMMD_MOM_AMAX (tests only: 0 sends every first-iteration pair to the direct sums)
  int32_t gen_wave;        // 1: beta-CEM generators by k_bgen_wave (a wave per block: the latency-bound small
                           // batches, Bt <= 512); 0: k_bgen (a quad per block: throughput). Fixed per handle.
  const float* beta_z0;    // [100][M+1]
  const float* beta_z;     // [20][pos_pad(M) * kBzCols] fp32 normals (bz_index layout, zero padded)
  // carry / state
  float* pop;              // [2][Bt][8] double-buffered population
  float* mean;             // [G][8]
  float* cov;              // [G][64]
  float* lam_x;            // [Bt][11]
  float* lam_y;            // [Bt][11]
  float* s_lane;           // [Bt][198]
  // per-iteration intermediates
  float* cx;               // [B][11]
  float* cy;               // [B][11]
  float* traj;             // [6][B][100]: x, y, xd, yd, xdd, ydd
  float* res_norm;         // [B]
  double* cnorm;           // [B][kCnormStride] compute_cost's eleven norms (k_front, cost.hpp)
  float* acc;              // [B][100]
  float* steer;            // [B][100]
  float* obs_cost;         // [B]
  float* lane_cost;        // [B]
  float* beta;             // [B][n]
  float* sigma;            // [B]
  float* res_beta;         // [B][20]
  float* btrace;           // [B][20] sum of the 11 elite QP costs per beta-iteration (parity trace: where two
                           //         runs of the beta-CEM part, compute_beta.py:133)
  // mmd_opt scratch (beta-CEM, compute_beta.py:93-157)
  float* feat;             // [B][22][M]   mother Bernstein coefficients (cx | cy)
  float* featr;            // [B][M][kFeatStride] the same, row-major (K_red distances)
  float* bmom;             // [B][M][kMomStride] series record of each distance row (k_bmoment)
  unsigned char* bdflag;   // [B][100][n]  pairs k_bkernel left to k_bdirect (a > 1)
  // the first beta-iteration's selection: its samples are the fixed-key
  // normals beta_z0 (shared by every candidate, Q3), so the top-n rows and
  // sigma are one table per handle, and the pairs are indexed by mother row
  const int32_t* sel0;     // [100][n]     top-n rows of sample s (argsort order)
  const float* sig0;       // [100]        its sigma
  const int32_t* rp0;      // [M+1]        pairs of mother row r: rpair0[rp0[r] .. rp0[r+1])
  const int2* rpair0;      // [100 n]      pair (i = s n + k, sigma_s bits), grouped by row
  const int32_t* rperm;    // [M]          mother rows by descending pair count (k_bmoment_rows: four rows of
                           //              nearly equal count per wave, so its direct-sum loop idles little)
  int32_t* bdcount;        // [B][kMaxSplit] their count per k_bkernel part
  float* bdist;            // [B][M][dist_stride(M)] L1 distances of the mother features
                           //              (kernel_computation.py:33-39), once per outer iteration
  float* ctrl_n;           // [B][2][n][H] noisy control rows (acc, steer)
  int32_t* bsel;           // [B][100][n]  top-n |beta| indices (argsort order)
  float* bsig;             // [B][100]     sample sigma (last coordinate, clipped)
  float* btop;             // [B][100][n]  QP solutions
  float* bcost;            // [B][100]     QP costs
  float* belite;           // [2][B][11][M+1] elite sample vectors (ping-pong)
  double* gen;             // [B][W, U plane][pos_pad(M)][kGenRow] (pad rows 0)
  double* phib;            // [B][ceil((M+1)/16)][66] Phi at the start of each 16-position block
  int32_t* bimin;          // [B] argmin sample of the last beta-iteration
  double* genm;            // [B][pos_pad(M)]  L_jj of the generators (pad 0)
  int32_t* bestsel;        // [B][n]       reduced set of the best sample
  float* brow;             // [B][100][n]  K_mixed row sums (fp32 partial sums, the reference's precision)
  float* bkred;            // [B][100][tri_stride(n)] K_red strict lower triangle (entry (k, kk < k) at k (k-1)/2 + kk)
  float* ygen;             // [B][kBzCols][ygs] new samples of the current beta-iteration (ygs = M+1 rounded to 32)
  // phase timestamps (s_memrealtime, 100 MHz) of workgroup 0, for profiling
  unsigned long long* dbg;  // [64]
  unsigned long long* dbgw;  // [65536][8] per-workgroup phase stamps of one kernel (MPCMMD_STAMPW)
  // work counters for the roofline, summed over k_bkernel workgroups:
  // [0] distinct distance rows summed directly, [1] (sample, reduced row) pairs
  // summed directly (M exponentials each), [2] pairs summed by the series,
  // [3] K_red entries
  unsigned long long* stats;  // [8]
  // CARLA variant (carla/optimizer/*.py of the reference): Frenet path,
  // one noisy initial state per rollout row, extra cost terms
  int32_t carla;           // 0: static / dynamic constants, 1: CARLA
  int32_t P;               // path points of the current solve
  int32_t R0;              // noisy initial rows per configuration (n^2 mmd_opt, n cvar)
  float wheel_base;        // carla/optimizer/cem.py:27
  float obs_a2, obs_b2;    // a_obs^2, b_obs^2 (cem.py:26)
  float obs_a, obs_b;      // a_obs, b_obs (the det projection's obstacle polar forms)
  float a_centr;           // cem.py:29
  float y_des1, y_des2;    // cem.py:161-166
  float w_des;             // weight of the desired-lane risk (cem.py:171-173)
  float gamma_des;         // gamma_lane_des (cem.py:182)
  const float* path;       // [G][6][kMaxPath]: x, y, arc_vec, Fx_dot, Fy_dot, kappa
  const float* st0r;       // [G][R0][8] noisy initial rollout states (x, y, vx, vy, psi)
  float* kappa_i;          // [Bt][100] curvature at the projected stations (projection.py:307)
  float* lane_des;         // [Bt] desired-lane risk (costs.py:70-100), unweighted
  float* rxy;              // [Bt][S][2][H] rollout points: global (x, y), then Frenet (s, d) in place
  float* res_steer;        // [G][T][100] steering of each iteration's chosen elite
  // compute_cem_det (cost MPCMMD_COST_DET): the projection with its obstacle
  // terms live (carla/optimizer/projection_det.py)
  const double* proj_m_det;  // [2][11][11] Kinv[:11,:11] of the det KKT (x, y)
  const float* obs_full;     // [G][2][O][100] Frenet obstacle tracks, all 100 plan points
  // outputs
  float* results;          // [G][T][kResultStride]
  int32_t* tr_proj;        // [G][T][B]
  int32_t* tr_obs;         // [G][T][20]
  int32_t* tr_cem;         // [G][T][5]
};

// The slices of configuration g (candidates [g B, (g + 1) B)).
struct Cfg {
  int g;
  int32_t idx_mpc;
  float v_des;
  const double* solve_c;
  const float* obs;
  const float* st0;
  const float* roll;
  const float* resample;
  double* gtab;
  float* mean;
  float* cov;
  float* results;
  int32_t* tr_proj;
  int32_t* tr_obs;
  int32_t* tr_cem;
};
HDI_CONST size_t gtab_stride(int S, int H) { return size_t(4) * 4 * 4 * S * H; }  // == gamma_tab_size (rng.hpp)
__device__ inline Cfg cfg_of(const Params& p, int g) {
  Cfg c;
  const size_t T = size_t(p.T), H = size_t(p.H), S = size_t(p.S), O = size_t(p.O);
  c.g = g;
  c.idx_mpc = p.idx_mpc[g];
  c.v_des = p.v_des[g];
  c.solve_c = p.solve_c + size_t(g) * 4 * 11;
  c.obs = p.obs + size_t(g) * 2 * O * H;
  c.st0 = p.st0 + size_t(g) * 8;
  c.roll = p.roll + size_t(g) * T * 3 * H * S;
  c.resample = p.resample + size_t(g) * T * (p.B - 5) * 8;
  c.gtab = p.gtab ? p.gtab + size_t(g) * gtab_stride(p.S, p.H) : nullptr;
  c.mean = p.mean + size_t(g) * 8;
  c.cov = p.cov + size_t(g) * 64;
  c.results = p.results + size_t(g) * T * kResultStride;
  c.tr_proj = p.tr_proj + size_t(g) * T * p.B;
  c.tr_obs = p.tr_obs + size_t(g) * T * kEliteCost;
  c.tr_cem = p.tr_cem + size_t(g) * T * kElite;
  return c;
}

void launch_noise(const Params& p, int t, hipStream_t s);
void launch_front(const Params& p, int t, hipStream_t s);
// ahead_t >= 0: the launch also draws iteration ahead_t's items of `kind`
// (draws.hpp: kAheadNoise | kAheadGamma) in spare workgroups
void launch_select(const Params& p, int t, hipStream_t s, int ahead_t = -1, int kind = 0);
void launch_risk_baseline(const Params& p, int t, hipStream_t s);
// the same risk with candidate lanes and the Beta draws inside the rollouts
// (k_mt_tab, k_roll_cand, k_risk_reduce): Params::risk_rows = 0 (MPCMMD_RISK_FUSED=1)
void launch_risk_fused(const Params& p, int t, hipStream_t s);
size_t mt_tab_entry_bytes();  // Params::mttab bytes per (step, candidate)

// Monte-Carlo validation (k_validate.hip; S/validation.py:134-171)
struct ValidateParams {
  int32_t K, O, H, R, noise;
  double noise_level, acc_const, steer_const, K_steer, y_lb, y_ub;
  uint32_t seed;
  const float* Pdot;    // [100][11] fp32 basis
  const float* Pddot;
  const double* cx;     // [K][11]
  const double* cy;
  const double* init_state;  // [K][6]
  const float* x_obs;   // [K][O][100]
  const float* y_obs;
  const double* draws;  // [K][3][R][H] or null (internal Philox)
  const uint32_t* keys; // [K]
  int32_t* count;       // [K]
  int32_t* count_lane;  // [K]
};
bool validate_shape_ok(int O, int H);
void launch_validate(const ValidateParams& v, hipStream_t s);
void launch_gamma_tab(const Params& p, int t, hipStream_t s);
void launch_beta_planes(const Params& p, int t, hipStream_t s);
// mmd_opt risk, one launch each (mpcmmd.hip chains them)
void launch_mother(const Params& p, int t, hipStream_t s);
void launch_dist_pad(const Params& p, int cap, hipStream_t s);  // once per handle (cap candidates), before the first launch_bdist
void launch_bdist(const Params& p, hipStream_t s);
void launch_bmoment(const Params& p, hipStream_t s);  // after launch_bdist: series records of the distance rows
void launch_bsample(const Params& p, int tb, hipStream_t s);
void launch_bselect(const Params& p, int tb, hipStream_t s);
void launch_bsel0(const Params& p, hipStream_t s);  // first beta-iteration: the handle's table into bsel / bsig
void launch_bkernel(const Params& p, int tb, hipStream_t s);  // K_mixed row sums by the series, K_red
void launch_bdirect(const Params& p, int tb, hipStream_t s);  // the other row sums, directly
void launch_bqp(const Params& p, int tb, hipStream_t s);
void launch_belite(const Params& p, int tb, hipStream_t s);
void launch_bgen(const Params& p, int tb, hipStream_t s);  // + k_bsigma on the last beta-iteration
void launch_mmdfinal(const Params& p, int t, hipStream_t s);
// the 20 beta-iterations of every candidate of [b0, b0 + nb) in one launch, a
// workgroup per candidate (small batches, n <= 24; bit-identical to the
// per-iteration kernels above)
bool bcem_small_ok(const Params& p);
void launch_bcem_small(const Params& p, hipStream_t s);
bool mmdopt_supported(int n, int H, int O, std::string* why);
// CARLA variant (k_carla.hip): rollouts of rows from their noisy initial
// states (mode 0: the baseline rows of cvar; mode 1: the reduced set of
// mmd_opt), their Frenet transforms, then the risk reducers
void launch_roll_carla(const Params& p, int t, int mode, hipStream_t s);
void launch_frenet(const Params& p, hipStream_t s);
void launch_risk_carla(const Params& p, int t, int mode, hipStream_t s);
}  // namespace mpcmmd
