// libmpcmmd: the C ABI (include/mpcmmd.h), handle / buffer management and
// the per-iteration launch sequence.  Host code is plain HIP runtime; no
// torch, no allocation after mpcmmd_create.
#include "../../include/mpcmmd.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "carla_host.hpp"
#include "draws.hpp"
#include "host_constants.hpp"
#include "kernels.hpp"
#include "rng.hpp"

using namespace mpcmmd;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPC(x)                                                                                     \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess)                                                                           \
      throw HipError(std::string(#x) + ": " + hipGetErrorString(e_) + " (" + __FILE__ + ":" +     \
                     std::to_string(__LINE__) + ")");                                              \
  } while (0)

enum KernelId {
  kKNoise = 0,
  kKFront,
  kKRiskBaseline,
  kKMother,
  kKBDist,
  kKBSample,
  kKBSelect,
  kKBKernel,
  kKBQp,
  kKBElite,
  kKMmdFinal,
  kKSelect,
  kKGammaTab,
  kKBetaPlanes,
  kKBGen,
  kKBMoment,
  kKBDirect,
  kKRollCarla,
  kKFrenet,
  kKRiskCarla,
  kKBcemSmall,
  kNumKernels
};
const char* kKernelNames[kNumKernels] = {"noise",   "front", "risk_baseline", "mother",   "bdist", "bsample",
                                         "bselect", "bkernel", "bqp",         "belite", "mmdfinal", "select",
                                         "gamma_tab", "beta_planes", "bgen",    "bmoment",     "bdirect",
                                         "roll_carla", "frenet", "risk_carla", "bcem_small"};

}  // namespace

struct mpcmmd_handle {
  mpcmmd_config cfg{};
  ProblemConsts pc;
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  Params p{};
  int B = 0, S = 0, H = 0, O = 0, n = 0, M = 0, T = 0;
  int Gmax = 1;  // configurations the buffers hold (mpcmmd_create_batch)
  int G = 1;     // configurations of the current solve
  std::map<std::string, std::pair<void*, size_t>> bufs;
  // solve state
  int cost = -1;
  bool begun = false;
  int last_t = -1;
  bool ext_roll = false, ext_res = false;
  bool beta_tables_internal = false;  // device beta tables hold the internal streams
  bool dist_pad = false;              // the distance matrix's +inf pad columns written (k_dist_pad)
  bool sel0_valid = false;            // sel0 / sig0 / rp0 / rpair0 match the device beta_z0
  // generation of the sel0 table (bumped by every rebuild) and the one
  // k_bmoment last used for the first beta-iteration's direct row sums: the
  // stage API may rewrite beta_z0 between stage 4 and stage 5/6 at t = 0
  unsigned sel0_gen = 0, bmoment_gen = ~0u;
  bool mmd_ok = false;                // mmd_opt buffers allocated (mmdopt_supported)
  bool carla = false;                 // CARLA variant handle (mpcmmd_carla_begin)
  int R0 = 0;                         // noisy initial rows per configuration (CARLA)
  std::vector<double> det_kx, det_ky;  // KKT inverses of the CARLA det projection (14^2, 15^2)
  std::string mmd_why;
  // pinned staging for the per-solve uploads of mpcmmd_begin: the copies are
  // asynchronous, so their source must outlive the call; the next begin waits
  // for stage_ev before refilling it
  char* stage = nullptr;
  size_t stage_bytes = 0, stage_used = 0;
  hipEvent_t stage_ev = nullptr;
  bool stage_pending = false;
  // candidate groups of the beta-CEM, each on its own stream (kernels of
  // different groups overlap); 1 = everything on the handle's stream
  static constexpr int kMaxGroups = 4;
  int groups = 1;
  bool groups_forced = false;
  int small_groups = 2;  // groups for launches of 64..256 candidates (MPCMMD_SMALL_GROUPS)
  hipStream_t gstream[kMaxGroups] = {};
  hipEvent_t gev_start = nullptr, gev_done[kMaxGroups] = {};
  // whole-solve graphs: mpcmmd_iterate(0, T) captured once per (cost, path
  // length, external draws, configurations) and replayed (one hipGraphLaunch
  // instead of ~150 launches per outer iteration)
  bool graphs = false;
  using GraphKey = std::tuple<int, int, int, int, int, int, int>;
  std::map<GraphKey, std::pair<hipGraph_t, hipGraphExec_t>> gexec;
  std::map<GraphKey, int> gahead;  // ahead_t after the captured iterations ran
  // draws ahead: k_select of iteration t also draws iteration t + 1's noise
  // and Beta attempt table (draws.hpp); ahead_t = the iteration whose draws
  // are already on the device that way (-1: none).  Deterministic draws, so
  // producing them early changes no value; invalidated by begin and by any
  // gamma table drawn for another iteration (the table has one slot)
  bool ahead_on = true;
  int ahead_t = -1;
  // k_select's residual sort and cost norms run in the risk launch where it
  // is k_risk_baseline (Params::select_prep); MPCMMD_SELECT_PREP=0: in
  // k_select / k_front
  bool prep_on = true;
  // sampling_param's internal standard normals [B][8] (fixed key: every solve's)
  std::vector<float> pop0_normals;
  // the iteration whose residual sort and cost norms the risk launch made
  // (-1: none since begin / the last front stage); stage 3 with select_prep
  // needs them for its own t
  int prep_t = -1;
  // small batches: the 20 beta-iterations as one launch (k_bcem_small);
  // MPCMMD_FUSED=0 keeps the per-iteration kernels
  bool fused_small = true;
  // profiling
  bool prof = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> free_events;
  int launches[kNumKernels] = {0};
  double total_ms[kNumKernels] = {0};

  size_t alloc_total = 0;
  size_t alloc_cap = 0;  // MPCMMD_MAX_HANDLE_BYTES (tests): refuse buffers past it with a real HIP OOM
  void* alloc(const std::string& name, size_t bytes) {
    void* d = nullptr;
    if (bytes == 0) bytes = 16;
    alloc_total += bytes;
    // over the cap: ask for an impossible size, so the failure is the
    // runtime's own out-of-memory error (and its sticky last-error state)
    HIPC(hipMalloc(&d, alloc_cap && alloc_total > alloc_cap ? (size_t(1) << 52) : bytes));
    // zeroed on the handle's own (non-blocking) stream: a null-stream memset
    // is not ordered before the constant uploads that follow on this stream
    // and could land after them
    HIPC(hipMemsetAsync(d, 0, bytes, stream));
    bufs[name] = {d, bytes};
    return d;
  }
  hipEvent_t ev() {
    if (!free_events.empty()) {
      hipEvent_t e = free_events.back();
      free_events.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPC(hipEventCreate(&e));
    return e;
  }
  template <class F>
  void launch(int kid, F&& f) {
    if (!prof) {
      f();
      HIPC(hipGetLastError());
      return;
    }
    hipEvent_t a = ev(), b = ev();
    HIPC(hipEventRecord(a, stream));
    f();
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(b, stream));
    pending.push_back({kid, {a, b}});
  }
  void collect() {
    for (auto& pe : pending) {
      float ms = 0.f;
      HIPC(hipEventSynchronize(pe.second.second));
      HIPC(hipEventElapsedTime(&ms, pe.second.first, pe.second.second));
      launches[pe.first] += 1;
      total_ms[pe.first] += ms;
      free_events.push_back(pe.second.first);
      free_events.push_back(pe.second.second);
    }
    pending.clear();
  }
};

namespace {

void check_device(mpcmmd_handle* h) { HIPC(hipSetDevice(h->device)); }

// host Philox normals of stream (stream, word1) with key (k0, k1): `count` values
std::vector<float> host_normals(uint32_t k0, uint32_t k1, uint32_t stream, uint32_t word1, size_t count) {
  std::vector<float> out(count);
  double z[4];
  for (size_t j = 0; j * 4 < count; ++j) {
    philox_normals4(k0, k1, stream, word1, uint32_t(j), z);
    for (int q = 0; q < 4 && j * 4 + q < count; ++q) out[j * 4 + q] = float(z[q]);
  }
  return out;
}

bool chol8(const double* a, double* L) {
  for (int i = 0; i < 64; ++i) L[i] = 0.0;
  for (int j = 0; j < 8; ++j) {
    double d = a[j * 8 + j];
    for (int k = 0; k < j; ++k) d -= L[j * 8 + k] * L[j * 8 + k];
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    L[j * 8 + j] = d;
    for (int i = j + 1; i < 8; ++i) {
      double s = a[i * 8 + j];
      for (int k = 0; k < j; ++k) s -= L[i * 8 + k] * L[j * 8 + k];
      L[i * 8 + j] = s / d;
    }
  }
  return true;
}

void upload(mpcmmd_handle* h, const char* name, const void* src, size_t bytes, size_t offset = 0) {
  auto it = h->bufs.find(name);
  if (it == h->bufs.end() || offset + bytes > it->second.second) throw std::runtime_error(std::string("buffer ") + name);
  HIPC(hipMemcpyAsync(static_cast<char*>(it->second.first) + offset, src, bytes, hipMemcpyHostToDevice, h->stream));
}

// upload through the handle's pinned staging area (mpcmmd_begin): src may be
// a host temporary, the copy still runs after the call returns
void upload_staged(mpcmmd_handle* h, const char* name, const void* src, size_t bytes, size_t offset = 0) {
  const size_t at = (h->stage_used + 63) & ~size_t(63);
  if (at + bytes > h->stage_bytes) throw std::runtime_error(std::string("staging area too small for ") + name);
  std::memcpy(h->stage + at, src, bytes);
  h->stage_used = at + bytes;
  upload(h, name, h->stage + at, bytes, offset);
}

// bytes of staging mpcmmd_begin needs at most (each piece 64-byte aligned)
size_t stage_size(int B, int S, int H, int O, int T, int G) {
  const size_t pieces[] = {size_t(4) * 11 * 8, 8 * 4, size_t(2) * O * H * 4, size_t(B) * 8 * 4, 8 * 4, 64 * 4,
                           size_t(T) * 3 * H * S * 4, size_t(T) * (B - kElite) * 8 * 4, 4, 4};
  size_t s = 0;
  for (size_t b : pieces) s += size_t(G) * b;
  return s + 16 * 64;
}

// beta_z iteration t: [89][M+1] (draw order) -> device bz_index layout (the
// sampler's lane image per 16-position block, zero padded), so the generation
// kernel reads whole blocks without bounds in coalesced float4 loads
void upload_beta_z(mpcmmd_handle* h, int t, const float* z) {
  const int M1 = h->M + 1, R = kBetaSamples - kBetaElite;
  std::vector<float> tr(size_t(pos_pad(h->M)) * kBzCols, 0.0f);
  for (int r = 0; r < R; ++r)
    for (int j = 0; j < M1; ++j) tr[bz_index(j, r)] = z[size_t(r) * M1 + j];
  upload(h, "beta_z", tr.data(), tr.size() * 4, size_t(t) * tr.size() * 4);
  HIPC(hipStreamSynchronize(h->stream));  // tr is a host temporary
}

void gen_beta_tables(mpcmmd_handle* h) {
  const int M1 = h->M + 1;
  const uint32_t k0 = kFixedKey0, k1 = h->cfg.seed;
  auto z0 = host_normals(k0, k1, kStreamBetaZ0, 0, size_t(kBetaSamples) * M1);
  upload(h, "beta_z0", z0.data(), z0.size() * 4);
  for (int t = 0; t < kBetaIters; ++t) {
    auto z = host_normals(k0, k1, kStreamBetaZ, uint32_t(t), size_t(kBetaSamples - kBetaElite) * M1);
    upload_beta_z(h, t, z.data());
  }
  HIPC(hipStreamSynchronize(h->stream));
  h->beta_tables_internal = true;
  h->sel0_valid = false;
}

// The first beta-iteration's selection (samples sqrt(20) beta_z0, shared by
// every candidate): k_bselect on one candidate, read back, and its pairs
// indexed by mother row for k_bmoment.  Once per beta_z0 table.
void ensure_sel0(mpcmmd_handle* h) {
  if (h->sel0_valid) return;
  const int n = h->n, M = h->M, np = kBetaSamples * n;
  Params q = h->p;
  q.b0 = 0;
  q.nb = 1;
  launch_bselect(q, 0, h->stream);
  HIPC(hipGetLastError());
  std::vector<int32_t> sel(np);
  std::vector<float> sig(kBetaSamples);
  HIPC(hipMemcpyAsync(sel.data(), h->p.bsel, np * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(hipMemcpyAsync(sig.data(), h->p.bsig, kBetaSamples * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(hipStreamSynchronize(h->stream));
  std::vector<int32_t> rp(M + 1, 0), pairs(2 * size_t(np));  // (i, sigma bits): one 8-byte load per pair
  for (int i = 0; i < np; ++i) {
    if (sel[i] < 0 || sel[i] >= M) throw std::runtime_error("first beta-iteration selection out of range");
    ++rp[sel[i] + 1];
  }
  for (int r = 0; r < M; ++r) rp[r + 1] += rp[r];
  std::vector<int32_t> fill(rp.begin(), rp.end() - 1);
  for (int i = 0; i < np; ++i) {
    const int at = fill[sel[i]]++;
    pairs[2 * at] = i;
    std::memcpy(&pairs[2 * at + 1], &sig[i / n], 4);
  }
  upload(h, "sel0", sel.data(), np * 4);
  upload(h, "sig0", sig.data(), kBetaSamples * 4);
  upload(h, "rp0", rp.data(), (M + 1) * 4);
  upload(h, "rpair0", pairs.data(), size_t(np) * 8);
  // k_bmoment_rows' row order: descending number of distinct sigmas among a
  // row's pairs (its direct-sum rounds), so a wave's four rows need about the
  // same number
  std::vector<int32_t> perm(M), nsig(M, 0);
  for (int r = 0; r < M; ++r) {
    perm[r] = r;
    std::vector<int32_t> sg;
    for (int q = rp[r]; q < rp[r + 1]; ++q) sg.push_back(pairs[2 * q + 1]);
    std::sort(sg.begin(), sg.end());
    nsig[r] = int(std::unique(sg.begin(), sg.end()) - sg.begin());
  }
  std::stable_sort(perm.begin(), perm.end(), [&](int a, int c) { return nsig[a] > nsig[c]; });
  upload(h, "rperm", perm.data(), size_t(M) * 4);
  HIPC(hipStreamSynchronize(h->stream));  // host temporaries
  h->sel0_valid = true;
  ++h->sel0_gen;
}

// k_bmoment wrote the first beta-iteration's direct row sums for the sel0
// table current at its launch; stages 5/6 at t = 0 rely on them
void check_bmoment_gen(mpcmmd_handle* h) {
  if (h->bmoment_gen != h->sel0_gen)
    throw std::invalid_argument(
        "beta_z0 changed (or stage 4 not run) since k_bmoment: rerun stage 4 before beta-iteration 0");
}

// one beta-CEM iteration (compute_beta.py:112-147) of candidates [p.b0, p.b0 + p.nb)
void run_beta_iteration(mpcmmd_handle* h, const Params& p, int tb, hipStream_t st) {
  if (tb > 0) h->launch(kKBSample, [&] { launch_bsample(p, tb, st); });
  h->launch(kKBSelect, [&] { tb == 0 ? launch_bsel0(p, st) : launch_bselect(p, tb, st); });
  h->launch(kKBKernel, [&] { launch_bkernel(p, tb, st); });
  if (tb > 0) h->launch(kKBDirect, [&] { launch_bdirect(p, tb, st); });  // first iteration: in k_bmoment
  h->launch(kKBQp, [&] { launch_bqp(p, tb, st); });
  h->launch(kKBElite, [&] { launch_belite(p, tb, st); });
  h->launch(kKBGen, [&] { launch_bgen(p, tb, st); });
}

// the 20 beta-CEM iterations of every candidate: one chain per candidate
// group, each group on its own stream between two events of the handle's
// stream (profiling runs them on the handle's stream, one after another,
// so the HIP-event timings are per kernel)
void run_beta_cem(mpcmmd_handle* h) {
  const int B = h->p.Bt;  // every candidate of every configuration
  if (h->fused_small && bcem_small_ok(h->p)) {
    h->launch(kKBcemSmall, [&] { launch_bcem_small(h->p, h->stream); });
    return;
  }
  // the default split applies to launches of >= 1024 candidates (a batch
  // handle may run fewer configurations than it holds); MPCMMD_GROUPS forces it
  const bool small = B >= 64 && B <= 256;
  const int G = h->prof ? 1 : (B >= 1024 || h->groups_forced ? h->groups : (small ? std::min(h->groups, h->small_groups) : 1));
  if (G <= 1) {
    for (int tb = 0; tb < kBetaIters; ++tb) run_beta_iteration(h, h->p, tb, h->stream);
    return;
  }
  std::vector<Params> pg(G, h->p);
  const int per = (B + G - 1) / G;
  for (int g = 0; g < G; ++g) {
    pg[g].b0 = g * per;
    pg[g].nb = std::max(0, std::min(per, B - g * per));
  }
  HIPC(hipEventRecord(h->gev_start, h->stream));
  for (int g = 0; g < G; ++g) HIPC(hipStreamWaitEvent(h->gstream[g], h->gev_start, 0));
  for (int tb = 0; tb < kBetaIters; ++tb)
    for (int g = 0; g < G; ++g)
      if (pg[g].nb > 0) run_beta_iteration(h, pg[g], tb, h->gstream[g]);
  for (int g = 0; g < G; ++g) {
    HIPC(hipEventRecord(h->gev_done[g], h->gstream[g]));
    HIPC(hipStreamWaitEvent(h->stream, h->gev_done[g], 0));
  }
}

// CARLA risk (k_carla.hip): rollouts of the rows from their noisy initial
// states (mode 0: cvar's n baseline rows; mode 1: mmd_opt's reduced set),
// their Frenet transforms, the reducers
void run_carla_risk(mpcmmd_handle* h, int t, int mode) {
  const Params& p = h->p;
  h->launch(kKRollCarla, [&] { launch_roll_carla(p, t, mode, h->stream); });
  h->launch(kKFrenet, [&] { launch_frenet(p, h->stream); });
  h->launch(kKRiskCarla, [&] { launch_risk_carla(p, t, mode, h->stream); });
}

// the draws k_select produces ahead for this solve (mpcmmd_handle::ahead_t)
int ahead_kind(const mpcmmd_handle* h) {
  if (!h->ahead_on) return 0;
  const bool beta = h->p.noise == MPCMMD_NOISE_BETA && h->p.cost != MPCMMD_COST_DET;  // det: no rollouts
  return (h->ext_roll && h->ext_res ? 0 : kAheadNoise) | (beta ? kAheadGamma : 0);
}

// the Beta attempt table of iteration t, unless k_select of t - 1 drew it
// (k_gamma_tab also zeroes the Beta fix-up count).  A table drawn ahead is
// used once: ahead_t is cleared here, so a rerun of stage 2 / 4 for the same t
// (stage API) draws the table again and restarts the fix-up list instead of
// appending to it.
void ensure_gamma_tab(mpcmmd_handle* h, int t) {
  if (h->p.noise != MPCMMD_NOISE_BETA) return;
  if (h->ahead_t == t) {
    h->ahead_t = -1;  // consumed (this iteration's noise was drawn ahead too: stage 0 ran before)
    return;
  }
  h->launch(kKGammaTab, [&] { launch_gamma_tab(h->p, t, h->stream); });
  h->ahead_t = -1;  // the table's one slot now holds t
}

void run_stage(mpcmmd_handle* h, int stage, int t) {
  const Params& p = h->p;
  switch (stage) {
    case 0:
      if (!(h->ahead_t == t && (ahead_kind(h) & kAheadNoise))) h->launch(kKNoise, [&] { launch_noise(p, t, h->stream); });
      break;
    case 1:
      h->launch(kKFront, [&] { launch_front(p, t, h->stream); });
      h->prep_t = -1;  // new residuals; with select_prep no cost norms until stage 2
      break;
    case 2:
      if (p.cost == MPCMMD_COST_DET) break;  // compute_cem_det: no rollouts, zero risks (carla/optimizer/cem.py:717-722)
      ensure_gamma_tab(h, t);
      if (p.cost == MPCMMD_COST_MMD_OPT) {
        if (!h->mmd_ok) throw std::invalid_argument("mmd_opt unsupported for this configuration: " + h->mmd_why);
        ensure_sel0(h);
        h->launch(kKMother, [&] { launch_mother(p, t, h->stream); });
        if (!h->dist_pad) {
          launch_dist_pad(p, h->Gmax * h->B, h->stream);  // the whole capacity: later solves may hold more candidates
          h->dist_pad = true;
        }
        h->launch(kKBDist, [&] { launch_bdist(p, h->stream); });
        h->launch(kKBMoment, [&] { launch_bmoment(p, h->stream); });
        h->bmoment_gen = h->sel0_gen;
        run_beta_cem(h);
        if (h->carla) run_carla_risk(h, t, 1);
        else h->launch(kKMmdFinal, [&] { launch_mmdfinal(p, t, h->stream); });
      } else if (h->carla) {
        if (p.noise == MPCMMD_NOISE_BETA) h->launch(kKBetaPlanes, [&] { launch_beta_planes(p, t, h->stream); });
        run_carla_risk(h, t, 0);
      } else if (!p.risk_rows) {
        h->launch(kKRiskBaseline, [&] { launch_risk_fused(p, t, h->stream); });
      } else {
        if (p.noise == MPCMMD_NOISE_BETA) h->launch(kKBetaPlanes, [&] { launch_beta_planes(p, t, h->stream); });
        h->launch(kKRiskBaseline, [&] { launch_risk_baseline(p, t, h->stream); });
        if (p.select_prep) h->prep_t = t;
      }
      break;
    case 3: {
      if (p.select_prep && h->prep_t != t)
        throw std::invalid_argument(
            "stage 3 needs stage 2 of the same iteration after stage 1 (the risk launch sorts the residuals and "
            "forms the cost norms: select_prep; MPCMMD_SELECT_PREP=0 moves them back to stages 1 and 3)");
      const int kind = ahead_kind(h), nxt = kind && t + 1 < h->T ? t + 1 : -1;
      h->launch(kKSelect, [&] { launch_select(p, t, h->stream, nxt, kind); });
      h->ahead_t = nxt;
      break;
    }
    case 4:
    case 5:
    case 6:
    case 7:
    case 8:
      if (p.cost != MPCMMD_COST_MMD_OPT || !h->mmd_ok) throw std::invalid_argument("stages 4-8 need cost mmd_opt");
      if (stage >= 5 && stage <= 7 && t >= kBetaIters) throw std::invalid_argument("beta-CEM iteration out of range");
      if (stage == 4) {  // mother rollouts, features and their distance matrix
        ensure_gamma_tab(h, t);
        ensure_sel0(h);
        h->launch(kKMother, [&] { launch_mother(p, t, h->stream); });
        if (!h->dist_pad) {
          launch_dist_pad(p, h->Gmax * h->B, h->stream);  // the whole capacity: later solves may hold more candidates
          h->dist_pad = true;
        }
        h->launch(kKBDist, [&] { launch_bdist(p, h->stream); });
        h->launch(kKBMoment, [&] { launch_bmoment(p, h->stream); });
        h->bmoment_gen = h->sel0_gen;
      }
      if (stage == 5) {  // samples + their top-n rows
        if (t > 0) h->launch(kKBSample, [&] { launch_bsample(p, t, h->stream); });
        if (t == 0) {
          ensure_sel0(h);
          check_bmoment_gen(h);
        }
        h->launch(kKBSelect, [&] { t == 0 ? launch_bsel0(p, h->stream) : launch_bselect(p, t, h->stream); });
      }
      if (stage == 6) {  // kernel sums + QP
        if (t == 0) check_bmoment_gen(h);
        h->launch(kKBKernel, [&] { launch_bkernel(p, t, h->stream); });
        if (t > 0) h->launch(kKBDirect, [&] { launch_bdirect(p, t, h->stream); });
        h->launch(kKBQp, [&] { launch_bqp(p, t, h->stream); });
      }
      if (stage == 7) {
        h->launch(kKBElite, [&] { launch_belite(p, t, h->stream); });
        h->launch(kKBGen, [&] { launch_bgen(p, t, h->stream); });
      }
      if (stage == 8) {
        if (h->carla) run_carla_risk(h, t, 1);
        else h->launch(kKMmdFinal, [&] { launch_mmdfinal(p, t, h->stream); });
      }
      break;
    default:
      throw std::invalid_argument("stage must be 0..8");
  }
}

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const HipError& e) {
    return fail(MPCMMD_E_HIP, e.what());
  } catch (const std::invalid_argument& e) {
    return fail(MPCMMD_E_INVALID, e.what());
  } catch (const std::exception& e) {
    return fail(MPCMMD_E_INVALID, e.what());
  }
}

}  // namespace

extern "C" {

int32_t mpcmmd_abi_version(void) { return MPCMMD_ABI_VERSION; }
const char* mpcmmd_last_error(void) { return g_err.c_str(); }

int32_t mpcmmd_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mpcmmd_create(const mpcmmd_config* cfg, mpcmmd_handle** out) { return mpcmmd_create_batch(cfg, 1, out); }

int mpcmmd_create_batch(const mpcmmd_config* cfg, int32_t max_configs, mpcmmd_handle** out) {
  if (!cfg || !out) return fail(MPCMMD_E_INVALID, "null argument");
  *out = nullptr;
  const mpcmmd_config& c = *cfg;
  if (c.num_reduced < 2 || c.num_obs < 1 || c.num_prime < 2 || c.num_prime > 100 || c.num_batch < 20 ||
      c.num_batch > 4096 || c.maxiter_cem < 1 || (c.noise != 0 && c.noise != 1) || c.variant < 0 || c.variant > 3)
    return fail(MPCMMD_E_INVALID,
                "config out of range (num_reduced>=2, num_obs>=1, 2<=num_prime<=100, 20<=num_batch<=4096)");
  if (c.num_reduced > 1024) return fail(MPCMMD_E_UNSUPPORTED, "num_reduced > 1024");
  if (size_t(c.num_obs) * c.num_prime > 8192) return fail(MPCMMD_E_UNSUPPORTED, "num_obs * num_prime > 8192");
  if (max_configs < 1) return fail(MPCMMD_E_INVALID, "max_configs must be >= 1");
  // grid limits: candidates on grid y / z (<= 65535), Beta fix-up list entries (32-bit)
  const size_t Bt = size_t(max_configs) * c.num_batch;
  if (Bt > 65535 || Bt * c.num_prime * c.num_reduced >= (size_t(1) << 32))
    return fail(MPCMMD_E_UNSUPPORTED, "max_configs * num_batch too large (<= 65535 candidates per handle)");
  auto* h = new mpcmmd_handle();
  int rc = guarded([&] {
    h->cfg = c;
    h->device = c.device;
    if (const char* cap = std::getenv("MPCMMD_MAX_HANDLE_BYTES")) h->alloc_cap = size_t(std::strtoull(cap, nullptr, 10));
    int ndev = 0;
    HIPC(hipGetDeviceCount(&ndev));
    if (c.device < 0 || c.device >= ndev) throw std::invalid_argument("device ordinal out of range");
    HIPC(hipSetDevice(c.device));
    HIPC(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->own_stream = true;
    h->pc = build_constants(c.num_prime, c.variant);
    h->B = c.num_batch;
    h->S = c.num_reduced;
    h->H = c.num_prime;
    h->O = c.num_obs;
    h->n = c.num_reduced;
    h->M = c.num_reduced * c.num_reduced;
    h->T = c.maxiter_cem;
    h->Gmax = max_configs;
    h->G = 1;
    const int B = h->B, S = h->S, H = h->H, O = h->O, T = h->T;
    const int GM = h->Gmax;
    const size_t BT = size_t(GM) * B;  // candidate capacity
    if (gtab_stride(S, H) != gamma_tab_size(S, H)) throw std::logic_error("Beta attempt table stride");
    const bool mmd_ok = mmdopt_supported(h->n, h->H, h->O, &h->mmd_why);
    h->mmd_ok = mmd_ok;
    Params& p = h->p;
    p.B = B;
    p.S = S;
    p.H = H;
    p.O = O;
    p.n = h->n;
    p.M = h->M;
    p.T = T;
    p.noise = c.noise;
    p.seed = c.seed;
    p.G = 1;
    p.Bt = B;
    p.b0 = 0;
    p.nb = B;
    p.sigma_acc = c.noise_level;
    p.sigma_steer = c.noise_level;
    p.acc_const = c.acc_const_noise;
    p.steer_const = c.steer_const_noise;
    // beta noise: steer_pert = float32(K_steer * sigma_steer) * (2 b - 1) (cem_helper.py:436)
    p.K_steer = float(h->pc.K_steer * double(c.noise_level));
    p.y_lb = float(h->pc.y_lb);
    p.y_ub = float(h->pc.y_ub);
    h->carla = h->pc.carla;
    p.carla = h->carla ? 1 : 0;
    p.wheel_base = float(h->pc.wheel_base);
    p.obs_a2 = float(h->pc.a_obs * h->pc.a_obs);
    p.obs_b2 = float(h->pc.b_obs * h->pc.b_obs);
    p.obs_a = float(h->pc.a_obs);
    p.obs_b = float(h->pc.b_obs);
    p.a_centr = float(h->pc.a_centr);
    p.y_des1 = float(h->pc.y_des_1);
    p.y_des2 = float(h->pc.y_des_2);
    p.gamma_des = float(h->pc.gamma_lane_des);
    if (h->carla && max_configs != 1)
      throw std::invalid_argument("CARLA handles solve one configuration (max_configs = 1)");
    // constants
    std::vector<float> basis(3 * kNum * kNvar);
    for (int i = 0; i < kNum * kNvar; ++i) {
      basis[i] = float(h->pc.P[i]);
      basis[kNum * kNvar + i] = float(h->pc.Pd[i]);
      basis[2 * kNum * kNvar + i] = float(h->pc.Pdd[i]);
    }
    p.basis = (const float*)h->alloc("basis", basis.size() * 4);
    // guess: c_bar = G v + h with G[k][j] = sum_i Kinv[k][i] (-k_p colsum_j[i])
    std::vector<double> gg(2 * kNvar * 4);
    for (int xy = 0; xy < 2; ++xy) {
      const auto& Ki = xy == 0 ? h->pc.guess_kinv_x : h->pc.guess_kinv_y;
      const auto& cs = xy == 0 ? h->pc.guess_colsum_x : h->pc.guess_colsum_y;
      const int n = xy == 0 ? 14 : 15;
      const double kp = xy == 0 ? h->pc.k_p_v : h->pc.k_p;
      for (int k = 0; k < kNvar; ++k)
        for (int j = 0; j < 4; ++j) {
          double s = 0.0;
          for (int i = 0; i < kNvar; ++i) s += Ki[k * n + i] * (-kp * cs[j * kNvar + i]);
          gg[(xy * kNvar + k) * 4 + j] = s;
        }
    }
    p.guess_g = (const double*)h->alloc("guess_g", gg.size() * 8);
    std::vector<double> pm(2 * kNvar * kNvar);
    for (int xy = 0; xy < 2; ++xy) {
      const auto& Ki = xy == 0 ? h->pc.proj_kinv_x : h->pc.proj_kinv_y;
      const int n = xy == 0 ? 14 : 15;
      for (int k = 0; k < kNvar; ++k)
        for (int j = 0; j < kNvar; ++j) pm[(xy * kNvar + k) * kNvar + j] = Ki[k * n + j];
    }
    p.proj_m = (const double*)h->alloc("proj_m", pm.size() * 8);
    p.fit = (const double*)h->alloc("fit", h->pc.fit.size() * 8);
    p.solve_c = (const double*)h->alloc("solve_c", size_t(GM) * 4 * kNvar * 8);
    p.obs = (const float*)h->alloc("obs", size_t(GM) * 2 * O * H * 4);
    p.st0 = (const float*)h->alloc("st0", size_t(GM) * 8 * 4);
    p.idx_mpc = (const int32_t*)h->alloc("idx_mpc", size_t(GM) * 4);
    p.v_des = (const float*)h->alloc("v_des", size_t(GM) * 4);
    p.roll = (const float*)h->alloc("roll", size_t(GM) * T * 3 * H * S * 4);
    p.resample = (const float*)h->alloc("resample", size_t(GM) * T * (B - kElite) * 8 * 4);
    p.bplane = (float*)h->alloc("bplane", c.noise == MPCMMD_NOISE_BETA ? BT * 2 * H * S * 4 : 16);
    p.bfix = (uint32_t*)h->alloc("bfix", c.noise == MPCMMD_NOISE_BETA ? BT * H * S * 4 : 16);
    p.bfix_n = (uint32_t*)h->alloc("bfix_n", 16);
    p.gtab = c.noise == MPCMMD_NOISE_BETA ? (double*)h->alloc("gtab", size_t(GM) * gamma_tab_size(S, H) * 8) : nullptr;
    p.mttab = c.noise == MPCMMD_NOISE_BETA ? h->alloc("mttab", BT * H * mt_tab_entry_bytes()) : nullptr;
    p.rbar = (float*)h->alloc("rbar", size_t(3) * BT * S * 4);
    if (mmd_ok) {
      p.beta_z0 = (const float*)h->alloc("beta_z0", size_t(kBetaSamples) * (h->M + 1) * 4);
      p.beta_z = (const float*)h->alloc("beta_z", size_t(kBetaIters) * pos_pad(h->M) * kBzCols * 4);
      const size_t M = h->M, M1 = M + 1, n = h->n;
      p.feat = (float*)h->alloc("feat", BT * 22 * M * 4);
      p.featr = (float*)h->alloc("featr", BT * M * kFeatStride * 4);
      p.bmom = (float*)h->alloc("bmom", BT * M * kMomStride * 4);
      p.bdflag = (unsigned char*)h->alloc("bdflag", BT * kBetaSamples * n);
      p.bdcount = (int32_t*)h->alloc("bdcount", BT * kMaxSplit * 4);
      p.bdlist = (int32_t*)h->alloc("bdlist", BT * kBetaSamples * h->n * 4);
      p.bdlcount = (int32_t*)h->alloc("bdlcount", BT * kBetaIters * 4);
      p.sel0 = (const int32_t*)h->alloc("sel0", size_t(kBetaSamples) * n * 4);
      p.sig0 = (const float*)h->alloc("sig0", size_t(kBetaSamples) * 4);
      p.rp0 = (const int32_t*)h->alloc("rp0", (M + 1) * 4);
      p.rpair0 = (const int2*)h->alloc("rpair0", size_t(kBetaSamples) * n * 8);
      p.rperm = (const int32_t*)h->alloc("rperm", size_t(M) * 4);
      p.bdist = (float*)h->alloc("bdist", BT * M * dist_stride(int(M)) * 4);
      p.ctrl_n = (float*)h->alloc("ctrl_n", BT * 2 * n * H * 4);
      p.bsel = (int32_t*)h->alloc("bsel", BT * kBetaSamples * n * 4);
      p.bsig = (float*)h->alloc("bsig", BT * kBetaSamples * 4);
      p.btop = (float*)h->alloc("btop", BT * kBetaSamples * n * 4);
      p.bcost = (float*)h->alloc("bcost", BT * kBetaSamples * 4);
      p.belite = (float*)h->alloc("belite", size_t(2) * BT * kBetaElite * M1 * 4);
      const size_t Pp = pos_pad(h->M);
      p.gen = (double*)h->alloc("gen", BT * Pp * kGenStride * 8);
      p.genm = (double*)h->alloc("genm", BT * Pp * 8);
      p.phib = (double*)h->alloc("phib", BT * ((h->M + 1 + 15) / 16) * 66 * 8);
      p.bimin = (int32_t*)h->alloc("bimin", BT * 4);
      p.bestsel = (int32_t*)h->alloc("bestsel", BT * n * 4);
      p.brow = (float*)h->alloc("brow", BT * kBetaSamples * n * 4);
      p.bkred = (float*)h->alloc("bkred", BT * kBetaSamples * tri_stride(int(n)) * 4);
      p.ygen = (float*)h->alloc("ygen", BT * kBzCols * ygen_stride(h->M) * 4);
    }
    std::vector<double> pm_det;
    if (h->carla) {  // path, noisy initial rows, curvature, rollout points, steering results
      h->R0 = mmd_ok ? std::max(h->M, S) : S;
      // compute_cem_det's projection (projection_det.py:149-160): its own KKT
      det_projection_kinv(h->pc, O, h->det_kx, h->det_ky);
      pm_det.assign(2 * kNvar * kNvar, 0.0);
      for (int xy = 0; xy < 2; ++xy) {
        const auto& Ki = xy == 0 ? h->det_kx : h->det_ky;
        const int n = xy == 0 ? 14 : 15;
        for (int k = 0; k < kNvar; ++k)
          for (int j = 0; j < kNvar; ++j) pm_det[(xy * kNvar + k) * kNvar + j] = Ki[k * n + j];
      }
      p.proj_m_det = (const double*)h->alloc("proj_m_det", pm_det.size() * 8);
      p.obs_full = (const float*)h->alloc("obs_full", size_t(GM) * 2 * O * kNum * 4);
      p.R0 = h->R0;
      p.path = (const float*)h->alloc("path", size_t(GM) * 6 * kMaxPath * 4);
      p.st0r = (const float*)h->alloc("st0r", size_t(GM) * h->R0 * 8 * 4);
      p.kappa_i = (float*)h->alloc("kappa_i", BT * kNum * 4);
      p.lane_des = (float*)h->alloc("lane_des", BT * 4);
      p.rxy = (float*)h->alloc("rxy", BT * S * 2 * H * 4);
      p.res_steer = (float*)h->alloc("res_steer", size_t(GM) * T * kNum * 4);
    }
    p.pop = (float*)h->alloc("pop", size_t(2) * BT * 8 * 4);
    p.mean = (float*)h->alloc("mean", size_t(GM) * 8 * 4);
    p.cov = (float*)h->alloc("cov", size_t(GM) * 64 * 4);
    p.lam_x = (float*)h->alloc("lam_x", BT * kNvar * 4);
    p.lam_y = (float*)h->alloc("lam_y", BT * kNvar * 4);
    p.s_lane = (float*)h->alloc("s_lane", BT * kLane * 4);
    p.cx = (float*)h->alloc("cx", BT * kNvar * 4);
    p.cy = (float*)h->alloc("cy", BT * kNvar * 4);
    p.traj = (float*)h->alloc("traj", size_t(6) * BT * kNum * 4);
    p.cnorm = (double*)h->alloc("cnorm", BT * kCnormStride * 8);
    p.res_norm = (float*)h->alloc("res_norm", BT * 4);
    p.acc = (float*)h->alloc("acc", BT * kNum * 4);
    p.steer = (float*)h->alloc("steer", BT * kNum * 4);
    p.obs_cost = (float*)h->alloc("obs_cost", BT * 4);
    p.lane_cost = (float*)h->alloc("lane_cost", BT * 4);
    p.beta = (float*)h->alloc("beta", BT * h->n * 4);
    p.sigma = (float*)h->alloc("sigma", BT * 4);
    p.res_beta = (float*)h->alloc("res_beta", BT * kBetaIters * 4);
    p.btrace = (float*)h->alloc("btrace", BT * kBetaIters * 4);
    p.dbg = (unsigned long long*)h->alloc("dbg", 64 * 8);
    // per-workgroup phase stamps (tools/stampsw.py) only when asked for:
    // with dbgw null MPCMMD_STAMPW writes nothing
    p.dbgw = std::getenv("MPCMMD_STAMPW") ? (unsigned long long*)h->alloc("dbgw", size_t(65536) * 8 * 8) : nullptr;
    p.stats = (unsigned long long*)h->alloc("stats", 8 * 8);
    p.results = (float*)h->alloc("results", size_t(GM) * T * kResultStride * 4);
    p.tr_proj = (int32_t*)h->alloc("tr_proj", size_t(GM) * T * B * 4);
    p.tr_obs = (int32_t*)h->alloc("tr_obs", size_t(GM) * T * kEliteCost * 4);
    p.tr_cem = (int32_t*)h->alloc("tr_cem", size_t(GM) * T * kElite * 4);
    // two candidate groups on two streams once each group still fills the
    // chip: one group's MFMA-bound sampler overlaps the other's VALU-bound
    // kernel sums (B = 1024: 82.2 -> 92.8 steps/s; four groups: 72.6)
    if (BT >= 1024) h->groups = 2;
    // small batches on the per-iteration kernels (num_reduced > 16; CARLA n = 22 at
    // B = 100): two groups as well, for launches of 64..256 candidates
    if (const char* g = std::getenv("MPCMMD_SMALL_GROUPS")) h->small_groups = std::max(1, std::atoi(g));
    if (BT >= 64 && BT <= 256) h->groups = std::max(h->groups, h->small_groups);
    h->groups_forced = std::getenv("MPCMMD_GROUPS") != nullptr;
    if (const char* g = std::getenv("MPCMMD_GRAPH")) h->graphs = std::atoi(g) != 0;
    if (const char* g = std::getenv("MPCMMD_AHEAD")) h->ahead_on = std::atoi(g) != 0;
    if (const char* g = std::getenv("MPCMMD_FUSED")) h->fused_small = std::atoi(g) != 0;
    if (const char* g = std::getenv("MPCMMD_SELECT_PREP")) h->prep_on = std::atoi(g) != 0;
    // the generators' variant is a property of the handle (its capacity), not
    // of a launch's candidate group: a candidate's bits do not depend on how
    // the batch is split into groups or whether k_bcem_small runs it
    p.gen_wave = BT <= 512 && h->n <= 24;
    if (const char* g = std::getenv("MPCMMD_GENWAVE")) p.gen_wave = std::atoi(g) != 0;
    p.mom_rows = 1;
    if (const char* g = std::getenv("MPCMMD_MOM_ROWS")) p.mom_rows = std::atoi(g) != 0;
    p.mom_amax = 1.0;  // == kSeriesAMax
    if (const char* g = std::getenv("MPCMMD_MOM_AMAX")) p.mom_amax = std::atof(g);
    p.dir_pairs = 1;
    if (const char* g = std::getenv("MPCMMD_DIR_PAIRS")) p.dir_pairs = std::atoi(g) != 0;
    p.qp_small = 1;
    if (const char* g = std::getenv("MPCMMD_QP_SMALL")) p.qp_small = std::atoi(g) != 0;
    p.sel_cap = 64;
    if (const char* g = std::getenv("MPCMMD_SEL_CAP")) p.sel_cap = std::max(1, std::atoi(g));
    p.dir_waves = 4;
    if (const char* g = std::getenv("MPCMMD_DIR_WAVES")) p.dir_waves = std::atoi(g);
    p.ker_target = 128;  // parts per candidate only below 128 candidates per launch (B = 100: 8 -> 2 parts)
    p.dir_target = 2048;
    if (const char* g = std::getenv("MPCMMD_KER_TARGET")) p.ker_target = std::max(1, std::atoi(g));
    if (const char* g = std::getenv("MPCMMD_DIR_TARGET")) p.dir_target = std::max(1, std::atoi(g));
    if (const char* g = std::getenv("MPCMMD_BETA_DUMP")) p.beta_dump = std::atoi(g) != 0;
    p.risk_rows = 1;  // the row-lane path is the faster one at configs[2]; MPCMMD_RISK_FUSED=1: fused
    if (const char* g = std::getenv("MPCMMD_RISK_FUSED")) p.risk_rows = std::atoi(g) == 0;
    if (const char* g = std::getenv("MPCMMD_GROUPS")) h->groups = std::max(1, std::min(mpcmmd_handle::kMaxGroups, std::atoi(g)));
    if (h->groups > 1) {
      HIPC(hipEventCreateWithFlags(&h->gev_start, hipEventDisableTiming));
      for (int g = 0; g < h->groups; ++g) {
        HIPC(hipStreamCreateWithFlags(&h->gstream[g], hipStreamNonBlocking));
        HIPC(hipEventCreateWithFlags(&h->gev_done[g], hipEventDisableTiming));
      }
    }
    h->stage_bytes = stage_size(B, S, H, O, T, GM) +
                     (h->carla ? size_t(6) * kMaxPath * 4 + size_t(h->R0) * 8 * 4 + size_t(2) * O * kNum * 4 + 512 : 0);
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&h->stage), h->stage_bytes, hipHostMallocDefault));
    HIPC(hipEventCreateWithFlags(&h->stage_ev, hipEventDisableTiming));
    upload(h, "basis", basis.data(), basis.size() * 4);
    upload(h, "guess_g", gg.data(), gg.size() * 8);
    upload(h, "proj_m", pm.data(), pm.size() * 8);
    upload(h, "fit", h->pc.fit.data(), h->pc.fit.size() * 8);
    if (h->carla) upload(h, "proj_m_det", pm_det.data(), pm_det.size() * 8);
    HIPC(hipStreamSynchronize(h->stream));
    return MPCMMD_OK;
  });
  if (rc != MPCMMD_OK) {
    mpcmmd_destroy(h);
    // a failed hipMalloc leaves its error as the runtime's last error; clear
    // it so a retry in this process (optimizer/sweep.py: batch_handle halves
    // max_configs) does not see the stale code at its first launch check
    (void)hipGetLastError();
    return rc;
  }
  *out = h;
  return MPCMMD_OK;
}

void mpcmmd_destroy(mpcmmd_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (auto& kv : h->gexec) {
    (void)hipGraphExecDestroy(kv.second.second);
    (void)hipGraphDestroy(kv.second.first);
  }
  for (int g = 0; g < mpcmmd_handle::kMaxGroups; ++g)  // group streams drained before their buffers go
    if (h->gstream[g]) (void)hipStreamSynchronize(h->gstream[g]);
  for (auto& kv : h->bufs) (void)hipFree(kv.second.first);
  for (auto& pe : h->pending) {
    (void)hipEventDestroy(pe.second.first);
    (void)hipEventDestroy(pe.second.second);
  }
  for (auto e : h->free_events) (void)hipEventDestroy(e);
  if (h->stage_ev) (void)hipEventDestroy(h->stage_ev);
  for (int g = 0; g < mpcmmd_handle::kMaxGroups; ++g) {
    if (h->gstream[g]) (void)hipStreamSynchronize(h->gstream[g]);
    if (h->gstream[g]) (void)hipStreamDestroy(h->gstream[g]);
    if (h->gev_done[g]) (void)hipEventDestroy(h->gev_done[g]);
  }
  if (h->gev_start) (void)hipEventDestroy(h->gev_start);
  if (h->stage) (void)hipHostFree(h->stage);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int mpcmmd_set_stream(mpcmmd_handle* h, void* s) {
  if (!h) return fail(MPCMMD_E_INVALID, "null handle");
  return guarded([&] {
    check_device(h);
    HIPC(hipStreamSynchronize(h->stream));
    if (h->own_stream) HIPC(hipStreamDestroy(h->stream));
    h->own_stream = false;
    h->stream = static_cast<hipStream_t>(s);
    return MPCMMD_OK;
  });
}

void* mpcmmd_get_stream(mpcmmd_handle* h) { return h ? (void*)h->stream : nullptr; }

namespace {

// CARLA per-solve setup (carla/optimizer/cem.py:248-264 mmd, 476-492 cvar):
// R noisy initial states (compute_noisy_init_state(_baseline),
// cem_helper.py:660-715; R = n^2 for mmd_opt, n for cvar) as rollout rows, and
// the boundary vectors from the mean of their Frenet states
// (global_to_frenet_vmap_1, cem_helper.py:348-388).  init_state is
// init_state_global = (x, y, v, vdot, psi, psidot) (C/main_carla.py:352).
void carla_rows(mpcmmd_handle* h, int cost_kind, int32_t idx_mpc, const float* is, const mpcmmd_path& path,
                const mpcmmd_draws* draws, std::vector<float>& rows, double* bx, double* by) {
  // compute_noisy_init_state / _baseline / _det (cem_helper.py:661-715): n^2, n or 1 rows
  const int R = cost_kind == MPCMMD_COST_MMD_OPT ? h->M : cost_kind == MPCMMD_COST_DET ? 1 : h->S;
  std::vector<float> eps;
  if (draws && draws->init_eps) eps.assign(draws->init_eps, draws->init_eps + size_t(R) * 4);
  else eps = host_normals(uint32_t(idx_mpc), h->cfg.seed, kStreamInitEps, 0, size_t(R) * 4);
  const float x0 = is[0], y0 = is[1], v0 = is[2], vdot = is[3], psi0 = is[4], psidot = is[5];
  const float vx = v0 * float(std::cos(double(psi0))), vy = v0 * float(std::sin(double(psi0)));
  const float psi = float(std::atan2(double(vy), double(vx)));
  const float mux = float(h->pc.init_mu_x), muy = float(h->pc.init_mu_y);
  const float sgx = float(h->pc.init_sigma_x), sgy = float(h->pc.init_sigma_y);
  rows.assign(size_t(h->R0) * 8, 0.0f);
  PathView pv;
  pv.P = path.num_path, pv.x = path.x_path, pv.y = path.y_path, pv.arc = path.arc_vec;
  pv.Fxd = path.Fx_dot, pv.Fyd = path.Fy_dot, pv.kappa = path.kappa;
  double sum[6] = {0, 0, 0, 0, 0, 0};
  for (int r = 0; r < R; ++r) {
    float* o = rows.data() + size_t(r) * 8;
    o[0] = x0 + (eps[size_t(r) * 4] * sgx + mux);
    o[1] = y0 + (eps[size_t(r) * 4 + 1] * sgy + muy);
    o[2] = vx;
    o[3] = vy;
    o[4] = psi;
    const float v = std::sqrt(vx * vx + vy * vy);
    const FrenetState f = global_to_frenet(pv, o[0], o[1], v, vdot, psi, psidot);
    const float vals[6] = {f.x, f.y, f.vx, f.vy, f.ax, f.ay};
    for (int k = 0; k < 6; ++k) sum[k] += double(vals[k]);  // sequential (the oracle's cumsum order)
  }
  float m[6];
  for (int k = 0; k < 6; ++k) m[k] = float(sum[k] / double(R));
  bx[0] = m[0], bx[1] = m[2], bx[2] = m[4];
  by[0] = m[1], by[1] = m[3], by[2] = m[5], by[3] = 0.0;
}

// mpcmmd_begin for n configurations (arrays with a leading configuration
// axis); external draws only for n == 1 (the parity contract)
int begin_impl(mpcmmd_handle* h, int32_t n_cfg, int32_t cost_kind, const int32_t* idx_mpc, const float* init_state,
               const float* mean, const float* cov, const float* x_obs, const float* y_obs, const float* v_des,
               const mpcmmd_draws* draws, const mpcmmd_path* path = nullptr) {
  if (!h || !idx_mpc || !init_state || !mean || !cov || !x_obs || !y_obs || !v_des)
    return fail(MPCMMD_E_INVALID, "null argument");
  if (h->carla != (path != nullptr))
    return fail(MPCMMD_E_INVALID, h->carla ? "CARLA handle: use mpcmmd_carla_begin / mpcmmd_carla_solve (a path is needed)"
                                           : "mpcmmd_carla_begin needs a handle of a CARLA variant");
  if (h->carla && cost_kind != MPCMMD_COST_MMD_OPT && cost_kind != MPCMMD_COST_CVAR && cost_kind != MPCMMD_COST_DET)
    return fail(MPCMMD_E_UNSUPPORTED,
                "the CARLA optimizer has compute_cem_mmd (mmd_opt), compute_cem_cvar and compute_cem_det only");
  if (!h->carla && cost_kind == MPCMMD_COST_DET)
    return fail(MPCMMD_E_INVALID, "compute_cem_det exists for the CARLA optimizer only");
  if (cost_kind == MPCMMD_COST_DET && h->O > kMaxDetObs)
    return fail(MPCMMD_E_UNSUPPORTED, "compute_cem_det: num_obs <= 32");
  if (path && (path->num_path < 4 || path->num_path > kMaxPath || !path->x_path || !path->y_path || !path->arc_vec ||
               !path->Fx_dot || !path->Fy_dot || !path->kappa))
    return fail(MPCMMD_E_INVALID, "path: 4 <= num_path <= 2048 and six arrays");
  if (cost_kind < 0 || cost_kind > 4) return fail(MPCMMD_E_INVALID, "cost_kind must be 0..4");
  if (n_cfg < 1 || n_cfg > h->Gmax) return fail(MPCMMD_E_INVALID, "n_cfg must be 1..max_configs of the handle");
  if (draws && n_cfg > 1) return fail(MPCMMD_E_INVALID, "external draws need n_cfg == 1");
  if (cost_kind == MPCMMD_COST_MMD_OPT && !h->mmd_ok) return fail(MPCMMD_E_UNSUPPORTED, h->mmd_why);
  return guarded([&] {
    check_device(h);
    Params& p = h->p;
    const int B = h->B, S = h->S, H = h->H, O = h->O, T = h->T, G = n_cfg;
    if (h->stage_pending) HIPC(hipEventSynchronize(h->stage_ev));  // previous begin's copies done
    h->stage_pending = false;
    h->stage_used = 0;
    // a failure after the first staged copy: drain them before the staging area is reused
    struct DrainOnThrow {
      mpcmmd_handle* h;
      bool armed = true;
      ~DrainOnThrow() {
        if (armed) (void)hipStreamSynchronize(h->stream);
      }
    } drain{h};
    h->cost = cost_kind;
    h->G = G;
    p.cost = cost_kind;
    // k_select's residual sort and cost norms in the risk launch (cost.hpp):
    // the baseline rollouts on Beta / Gaussian planes (k_risk_baseline)
    p.select_prep = h->prep_on && !h->carla && p.risk_rows &&
                    (cost_kind == MPCMMD_COST_CVAR || cost_kind == MPCMMD_COST_SAA || cost_kind == MPCMMD_COST_MMD_RANDOM);
    p.G = G;
    p.Bt = G * B;
    p.b0 = 0;
    p.nb = p.Bt;
    // cem.py:161-163 weights (obs, lane); CARLA: carla/optimizer/cem.py:171-173 (+ desired lane)
    const float w_obs[5] = {1e3f, 1e3f, 1e3f, 1e6f, 0.f}, w_lane[5] = {0.f, 0.f, 0.f, 1e6f, 0.f};
    p.w_obs = w_obs[cost_kind];
    p.w_lane = w_lane[cost_kind];
    p.w_des = 0.0f;
    if (h->carla) {  // det: 0 * the zero risks (cem.py:750)
      p.w_obs = cost_kind == MPCMMD_COST_MMD_OPT ? 0.1f : cost_kind == MPCMMD_COST_DET ? 0.0f : 100.0f;
      p.w_lane = cost_kind == MPCMMD_COST_MMD_OPT ? 0.01f : cost_kind == MPCMMD_COST_DET ? 0.0f : 25.0f;
      p.w_des = 0.0f;
    }
    upload_staged(h, "idx_mpc", idx_mpc, size_t(G) * 4);
    upload_staged(h, "v_des", v_des, size_t(G) * 4);
    // sampling_param (cem_helper.py:122-150): fixed key, the same draws for every configuration
    // (the internal draws depend on the seed and B only: made once per handle)
    std::vector<float> z0x;
    if (draws && draws->pop0) z0x.assign(draws->pop0, draws->pop0 + size_t(B) * 8);
    else if (h->pop0_normals.empty()) h->pop0_normals = host_normals(kFixedKey0, h->cfg.seed, kStreamPop0, 0, size_t(B) * 8);
    const std::vector<float>& z0 = draws && draws->pop0 ? z0x : h->pop0_normals;
    std::vector<double> sc(size_t(G) * 4 * kNvar, 0.0);
    std::vector<float> st0(size_t(G) * 8, 0.f), ob(size_t(G) * 2 * O * H), pop(size_t(G) * B * 8);
    std::vector<float> rows0;  // CARLA noisy initial rows [R0][8]
    for (int g = 0; g < G; ++g) {
      const float* is = init_state + size_t(g) * 6;
      // boundary vectors (cem_helper.py:152-167) and the per-solve KKT columns
      double bx[3] = {is[0], is[2], is[4]};
      double by[4] = {is[1], is[3], is[5], 0.0};
      if (h->carla) carla_rows(h, cost_kind, idx_mpc[g], is, *path, draws, rows0, bx, by);
      double* scg = sc.data() + size_t(g) * 4 * kNvar;
      for (int k = 0; k < kNvar; ++k) {
        for (int e = 0; e < 3; ++e) scg[0 * kNvar + k] += h->pc.guess_kinv_x[k * 14 + kNvar + e] * bx[e];
        for (int e = 0; e < 4; ++e) scg[1 * kNvar + k] += h->pc.guess_kinv_y[k * 15 + kNvar + e] * by[e];
        const bool det = cost_kind == MPCMMD_COST_DET;  // the det projection's own KKT
        const double* pkx = det ? h->det_kx.data() : h->pc.proj_kinv_x.data();
        const double* pky = det ? h->det_ky.data() : h->pc.proj_kinv_y.data();
        for (int e = 0; e < 3; ++e) scg[2 * kNvar + k] += pkx[k * 14 + kNvar + e] * bx[e];
        for (int e = 0; e < 4; ++e) scg[3 * kNvar + k] += pky[k * 15 + kNvar + e] * by[e];
      }
      float* s0 = st0.data() + size_t(g) * 8;
      s0[0] = is[0], s0[1] = is[1], s0[2] = is[2], s0[3] = is[3], s0[4] = atan2f(is[3], is[2]);
      const float* xo = x_obs + size_t(g) * O * kNum;
      const float* yo = y_obs + size_t(g) * O * kNum;
      float* obg = ob.data() + size_t(g) * 2 * O * H;
      for (int o = 0; o < O; ++o)
        for (int t = 0; t < H; ++t) {
          obg[size_t(o) * H + t] = xo[o * kNum + t];
          obg[size_t(O) * H + o * H + t] = yo[o * kNum + t];
        }
      const float* mg = mean + size_t(g) * 8;
      double cv[64], L[64];
      for (int i = 0; i < 64; ++i) cv[i] = double(cov[size_t(g) * 64 + i]);
      if (!chol8(cv, L)) throw std::invalid_argument("cov_param_init is not positive definite");
      float* pg = pop.data() + size_t(g) * B * 8;
      for (int b = 0; b < B; ++b)
        for (int a = 0; a < 8; ++a) {
          double s = double(mg[a]);
          for (int c = 0; c <= a; ++c) s += L[a * 8 + c] * double(z0[size_t(b) * 8 + c]);
          float v = float(s);
          if (a < 4) v = fminf(fmaxf(v, 0.1f), 30.0f);
          pg[size_t(b) * 8 + a] = v;
        }
    }
    upload_staged(h, "solve_c", sc.data(), sc.size() * 8);
    if (h->carla) {
      upload_staged(h, "st0r", rows0.data(), rows0.size() * 4);
      const float* arrs[6] = {path->x_path, path->y_path, path->arc_vec, path->Fx_dot, path->Fy_dot, path->kappa};
      for (int k = 0; k < 6; ++k)
        upload_staged(h, "path", arrs[k], size_t(path->num_path) * 4, size_t(k) * kMaxPath * 4);
      p.P = path->num_path;
      if (cost_kind == MPCMMD_COST_DET) {  // all 100 plan points of the tracks; risks stay 0 (no risk stage)
        upload_staged(h, "obs_full", x_obs, size_t(O) * kNum * 4);
        upload_staged(h, "obs_full", y_obs, size_t(O) * kNum * 4, size_t(O) * kNum * 4);
        HIPC(hipMemsetAsync(p.obs_cost, 0, size_t(B) * 4, h->stream));
        HIPC(hipMemsetAsync(p.lane_cost, 0, size_t(B) * 4, h->stream));
        HIPC(hipMemsetAsync(p.lane_des, 0, size_t(B) * 4, h->stream));
      }
    }
    upload_staged(h, "st0", st0.data(), st0.size() * 4);
    upload_staged(h, "obs", ob.data(), ob.size() * 4);
    upload_staged(h, "pop", pop.data(), pop.size() * 4);  // iteration 0's half: [0][G B][8]
    upload_staged(h, "mean", mean, size_t(G) * 8 * 4);
    upload_staged(h, "cov", cov, size_t(G) * 64 * 4);
    HIPC(hipMemsetAsync(p.lam_x, 0, size_t(G) * B * kNvar * 4, h->stream));
    HIPC(hipMemsetAsync(p.lam_y, 0, size_t(G) * B * kNvar * 4, h->stream));
    HIPC(hipMemsetAsync(p.s_lane, 0, size_t(G) * B * kLane * 4, h->stream));
    // external noise rows: [T][3][S][H] -> device [T][3][H][S]
    h->ext_roll = draws && draws->roll;
    h->ext_res = draws && draws->resample;
    if (h->ext_roll) {
      std::vector<float> r(size_t(T) * 3 * H * S);
      for (int t = 0; t < T; ++t)
        for (int k = 0; k < 3; ++k)
          for (int s = 0; s < S; ++s)
            for (int q = 0; q < H; ++q)
              r[((size_t(t) * 3 + k) * H + q) * S + s] = draws->roll[((size_t(t) * 3 + k) * S + s) * H + q];
      upload_staged(h, "roll", r.data(), r.size() * 4);
    }
    if (h->ext_res) upload_staged(h, "resample", draws->resample, size_t(T) * (B - kElite) * 8 * 4);
    if (cost_kind == MPCMMD_COST_MMD_OPT) {
      const size_t M1 = size_t(h->M) + 1;
      const bool ext_b = draws && (draws->beta_z0 || draws->beta_z);
      if (ext_b) {
        if (!draws->beta_z0 || !draws->beta_z) throw std::invalid_argument("beta_z0 and beta_z go together");
        upload(h, "beta_z0", draws->beta_z0, size_t(kBetaSamples) * M1 * 4);
        for (int t = 0; t < kBetaIters; ++t)
          upload_beta_z(h, t, draws->beta_z + size_t(t) * (kBetaSamples - kBetaElite) * M1);
        h->beta_tables_internal = false;
        h->sel0_valid = false;
      } else if (!h->beta_tables_internal) {
        gen_beta_tables(h);
      }
    }
    HIPC(hipEventRecord(h->stage_ev, h->stream));
    h->stage_pending = true;
    drain.armed = false;
    h->begun = true;
    h->last_t = -1;
    h->ahead_t = -1;
    h->prep_t = -1;
    return MPCMMD_OK;
  });
}

// the result of configuration g (cem.py:324-333): the last enqueued iteration
void read_result(mpcmmd_handle* h, int g, mpcmmd_result* out) {
  const int T = h->T;
  std::vector<float> r(kResultStride);
  HIPC(hipMemcpy(r.data(), h->p.results + (size_t(g) * T + h->last_t) * kResultStride, kResultStride * 4,
                 hipMemcpyDeviceToHost));
  std::memcpy(out->cx, &r[0], 11 * 4);
  std::memcpy(out->cy, &r[11], 11 * 4);
  out->cost_lane = r[22];
  out->cost_obs = r[23];
  out->sigma = r[24];
  std::memcpy(out->res_beta, &r[25], 20 * 4);
  if (out->beta && h->cost == MPCMMD_COST_MMD_OPT) std::memcpy(out->beta, &r[45], size_t(h->n) * 4);
  if (h->carla) {  // carla/optimizer/cem.py:413-441: cx, cy, v_best, steering_best, mean_param
    std::vector<float> st(kNum);
    HIPC(hipMemcpy(st.data(), h->p.res_steer + (size_t(g) * T + h->last_t) * kNum, kNum * 4, hipMemcpyDeviceToHost));
    if (out->steering) std::memcpy(out->steering, st.data(), kNum * 4);
    HIPC(hipMemcpy(out->mean_param, h->p.mean + size_t(g) * 8, 8 * 4, hipMemcpyDeviceToHost));
    if (out->v_best)
      for (int i = 0; i < kNum; ++i) {  // v = sqrt((Pdot cx)^2 + (Pdot cy)^2), fp64 sums rounded once
        double sx = 0.0, sy = 0.0;
        for (int k = 0; k < kNvar; ++k) {
          sx += h->pc.Pd[i * kNvar + k] * double(out->cx[k]);
          sy += h->pc.Pd[i * kNvar + k] * double(out->cy[k]);
        }
        const float xd = float(sx), yd = float(sy);
        out->v_best[i] = std::sqrt(xd * xd + yd * yd);
      }
  }
  const int Tr = h->last_t + 1;
  if (out->elite_proj)
    HIPC(hipMemcpy(out->elite_proj, h->p.tr_proj + size_t(g) * T * h->B, size_t(Tr) * h->B * 4,
                   hipMemcpyDeviceToHost));
  if (out->elite_obs)
    HIPC(hipMemcpy(out->elite_obs, h->p.tr_obs + size_t(g) * T * kEliteCost, size_t(Tr) * kEliteCost * 4,
                   hipMemcpyDeviceToHost));
  if (out->elite_cem)
    HIPC(hipMemcpy(out->elite_cem, h->p.tr_cem + size_t(g) * T * kElite, size_t(Tr) * kElite * 4,
                   hipMemcpyDeviceToHost));
}

}  // namespace

int mpcmmd_begin(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                 const float mean[8], const float cov[64], const float* x_obs, const float* y_obs, float v_des,
                 const mpcmmd_draws* draws) {
  return begin_impl(h, 1, cost_kind, &idx_mpc, init_state, mean, cov, x_obs, y_obs, &v_des, draws);
}

int mpcmmd_begin_batch(mpcmmd_handle* h, int32_t n_cfg, int32_t cost_kind, const int32_t* idx_mpc,
                       const float* init_state, const float* mean, const float* cov, const float* x_obs,
                       const float* y_obs, const float* v_des) {
  return begin_impl(h, n_cfg, cost_kind, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, nullptr);
}

int mpcmmd_iterate(mpcmmd_handle* h, int32_t t_begin, int32_t count) {
  if (!h) return fail(MPCMMD_E_INVALID, "null handle");
  if (!h->begun) return fail(MPCMMD_E_STATE, "mpcmmd_iterate before mpcmmd_begin");
  if (t_begin < 0 || count < 0 || t_begin + count > h->T) return fail(MPCMMD_E_INVALID, "iteration range");
  return guarded([&] {
    check_device(h);
    auto body = [&](int t_lo, int cnt) {
      for (int t = t_lo; t < t_lo + cnt; ++t) {
        if (!h->ext_roll || !h->ext_res) {
          if (h->ext_roll != h->ext_res) throw std::invalid_argument("roll and resample draws go together");
          run_stage(h, 0, t);
        }
        run_stage(h, 1, t);
        run_stage(h, 2, t);
        run_stage(h, 3, t);
      }
    };
    // graphs of a whole solve (count == T) or of single iterations (count ==
    // 1: all T captured at the first use, so no capture lands in a timed
    // loop) on one stream -- the beta-CEM candidate groups of large mmd_opt
    // batches fork onto other streams and are launched directly
    const bool one_stream = h->cost != MPCMMD_COST_MMD_OPT || (h->p.Bt < 1024 && !h->groups_forced);
    const bool whole = t_begin == 0 && count == h->T;
    if (h->graphs && !h->prof && one_stream && (whole || count == 1)) {
      if (h->cost == MPCMMD_COST_MMD_OPT) ensure_sel0(h);  // host read-back: never inside a capture
      // key: ... and whether the first iteration's draws were drawn ahead (ai)
      auto key_of = [&](int tb, int cnt, int ai) {
        return std::make_tuple(h->cost, h->p.P, int(h->ext_roll), h->G, whole ? 0 : tb, cnt, ai);
      };
      auto capture = [&](int tb, int cnt, int ai) {
        const int saved = h->ahead_t;
        h->ahead_t = ai ? tb : -1;
        hipGraph_t g = nullptr;
        HIPC(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
        try {
          body(tb, cnt);
        } catch (...) {
          (void)hipStreamEndCapture(h->stream, &g);
          if (g) (void)hipGraphDestroy(g);
          h->ahead_t = saved;
          throw;
        }
        HIPC(hipStreamEndCapture(h->stream, &g));
        hipGraphExec_t e = nullptr;
        HIPC(hipGraphInstantiate(&e, g, nullptr, nullptr, 0));
        h->gexec.emplace(key_of(tb, cnt, ai), std::make_pair(g, e));
        h->gahead[key_of(tb, cnt, ai)] = h->ahead_t;
        h->ahead_t = saved;
      };
      const int ai_now = h->ahead_t == t_begin && ahead_kind(h) ? 1 : 0;
      if (h->gexec.find(key_of(t_begin, count, ai_now)) == h->gexec.end()) {
        if (whole) {
          capture(0, h->T, ai_now);
        } else {  // the in-order pattern (iteration tb's draws drawn by tb - 1), then the one asked for
          for (int tb = 0; tb < h->T; ++tb) {
            const int ai = tb > 0 && ahead_kind(h) ? 1 : 0;
            if (h->gexec.find(key_of(tb, 1, ai)) == h->gexec.end()) capture(tb, 1, ai);
          }
          if (h->gexec.find(key_of(t_begin, 1, ai_now)) == h->gexec.end()) capture(t_begin, 1, ai_now);
        }
      }
      HIPC(hipGraphLaunch(h->gexec.find(key_of(t_begin, count, ai_now))->second.second, h->stream));
      h->ahead_t = h->gahead[key_of(t_begin, count, ai_now)];
    } else {
      body(t_begin, count);
    }
    if (count > 0) h->last_t = t_begin + count - 1;  // a zero-count call runs nothing
    return MPCMMD_OK;
  });
}

int mpcmmd_set_graphs(mpcmmd_handle* h, int32_t enable) {
  if (!h) return fail(MPCMMD_E_INVALID, "null handle");
  return guarded([&] {
    check_device(h);
    h->graphs = enable != 0;
    return MPCMMD_OK;
  });
}

int mpcmmd_sync(mpcmmd_handle* h) {
  if (!h) return fail(MPCMMD_E_INVALID, "null handle");
  return guarded([&] {
    check_device(h);
    HIPC(hipStreamSynchronize(h->stream));
    if (h->prof) h->collect();
    return MPCMMD_OK;
  });
}

int mpcmmd_finish(mpcmmd_handle* h, mpcmmd_result* out) { return mpcmmd_finish_batch(h, 1, out); }

int mpcmmd_finish_batch(mpcmmd_handle* h, int32_t n_cfg, mpcmmd_result* out) {
  if (!h || !out) return fail(MPCMMD_E_INVALID, "null argument");
  if (!h->begun || h->last_t < 0) return fail(MPCMMD_E_STATE, "no iteration has run");
  if (n_cfg < 1 || n_cfg > h->G) return fail(MPCMMD_E_INVALID, "n_cfg exceeds the configurations of the solve");
  return guarded([&] {
    check_device(h);
    HIPC(hipStreamSynchronize(h->stream));
    if (h->prof) h->collect();
    for (int g = 0; g < n_cfg; ++g) read_result(h, g, out + g);
    return MPCMMD_OK;
  });
}

int mpcmmd_solve(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                 const float mean[8], const float cov[64], const float* x_obs, const float* y_obs, float v_des,
                 const mpcmmd_draws* draws, mpcmmd_result* out) {
  int rc = mpcmmd_begin(h, cost_kind, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, draws);
  if (rc) return rc;
  rc = mpcmmd_iterate(h, 0, h->T);
  if (rc) return rc;
  return mpcmmd_finish(h, out);
}

int mpcmmd_solve_batch(mpcmmd_handle* h, int32_t n_cfg, int32_t cost_kind, const int32_t* idx_mpc,
                       const float* init_state, const float* mean, const float* cov, const float* x_obs,
                       const float* y_obs, const float* v_des, mpcmmd_result* out) {
  int rc = mpcmmd_begin_batch(h, n_cfg, cost_kind, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des);
  if (rc) return rc;
  rc = mpcmmd_iterate(h, 0, h->T);
  if (rc) return rc;
  return mpcmmd_finish_batch(h, n_cfg, out);
}

int32_t mpcmmd_max_configs(mpcmmd_handle* h) { return h ? h->Gmax : 0; }

int mpcmmd_handle_info(mpcmmd_handle* h, const char* name, int64_t* value) {
  if (!h || !name || !value) return fail(MPCMMD_E_INVALID, "null argument");
  const std::string k(name);
  if (k == "gen_wave") *value = h->p.gen_wave ? 1 : 0;
  else if (k == "select_prep") *value = h->prep_on && !h->carla && h->p.risk_rows ? 1 : 0;
  else if (k == "fused_small") *value = h->fused_small ? 1 : 0;
  else if (k == "groups") *value = h->groups;
  else if (k == "capacity") *value = int64_t(h->Gmax) * h->B;
  else return fail(MPCMMD_E_INVALID, "unknown handle_info name " + k);
  return MPCMMD_OK;
}

int mpcmmd_carla_begin(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                       const float mean[8], const float cov[64], const float* x_obs, const float* y_obs, float v_des,
                       const mpcmmd_path* path, const mpcmmd_draws* draws) {
  if (!path) return fail(MPCMMD_E_INVALID, "null path");
  return begin_impl(h, 1, cost_kind, &idx_mpc, init_state, mean, cov, x_obs, y_obs, &v_des, draws, path);
}

int mpcmmd_carla_solve(mpcmmd_handle* h, int32_t cost_kind, int32_t idx_mpc, const float init_state[6],
                       const float mean[8], const float cov[64], const float* x_obs, const float* y_obs, float v_des,
                       const mpcmmd_path* path, const mpcmmd_draws* draws, mpcmmd_result* out) {
  int rc = mpcmmd_carla_begin(h, cost_kind, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, path, draws);
  if (rc) return rc;
  rc = mpcmmd_iterate(h, 0, h->T);
  if (rc) return rc;
  return mpcmmd_finish(h, out);
}

int mpcmmd_path_smoothing(int32_t num_path, const float* x_wp, const float* y_wp, float threshold, float* x_path,
                          float* y_path) {
  if (num_path < 4 || num_path > kMaxPath || !x_wp || !y_wp || !x_path || !y_path)
    return fail(MPCMMD_E_INVALID, "path smoothing: 4 <= num_path <= 2048, non-null arrays");
  try {
    path_smoothing(num_path, x_wp, y_wp, threshold, x_path, y_path);
    return MPCMMD_OK;
  } catch (const std::exception& e) {
    return fail(MPCMMD_E_INVALID, e.what());
  }
}

int mpcmmd_path_parameters(int32_t num_path, const float* x_path, const float* y_path, float* Fx_dot, float* Fy_dot,
                           float* Fx_ddot, float* Fy_ddot, float* arc_vec, float* kappa, float* arc_length) {
  if (num_path < 3 || !x_path || !y_path || !Fx_dot || !Fy_dot || !Fx_ddot || !Fy_ddot || !arc_vec || !kappa)
    return fail(MPCMMD_E_INVALID, "path parameters: num_path >= 3, non-null arrays");
  try {
    path_parameters(num_path, x_path, y_path, Fx_dot, Fy_dot, Fx_ddot, Fy_ddot, arc_vec, kappa, arc_length);
    return MPCMMD_OK;
  } catch (const std::exception& e) {
    return fail(MPCMMD_E_INVALID, e.what());
  }
}

int mpcmmd_global_to_frenet(const mpcmmd_path* path, int32_t count, const float* x, const float* y, const float* v,
                            const float* vdot, const float* psi, const float* psidot, float* out) {
  if (!path || count < 0 || (count > 0 && (!x || !y || !v || !vdot || !psi || !psidot || !out)))
    return fail(MPCMMD_E_INVALID, "null argument");
  if (path->num_path < 2 || !path->x_path || !path->y_path || !path->arc_vec || !path->Fx_dot || !path->Fy_dot ||
      !path->kappa)
    return fail(MPCMMD_E_INVALID, "path: num_path >= 2 and six arrays");
  PathView pv;
  pv.P = path->num_path, pv.x = path->x_path, pv.y = path->y_path, pv.arc = path->arc_vec;
  pv.Fxd = path->Fx_dot, pv.Fyd = path->Fy_dot, pv.kappa = path->kappa;
  for (int i = 0; i < count; ++i) {
    const FrenetState f = global_to_frenet(pv, x[i], y[i], v[i], vdot[i], psi[i], psidot[i]);
    float* o = out + size_t(i) * 7;
    o[0] = f.x, o[1] = f.y, o[2] = f.vx, o[3] = f.vy, o[4] = f.ax, o[5] = f.ay, o[6] = f.psi;
  }
  return MPCMMD_OK;
}

int mpcmmd_profile(mpcmmd_handle* h, int32_t enable) {
  if (!h) return fail(MPCMMD_E_INVALID, "null handle");
  return guarded([&] {
    check_device(h);
    HIPC(hipStreamSynchronize(h->stream));
    h->collect();
    h->prof = enable != 0;
    for (int k = 0; k < kNumKernels; ++k) {
      h->launches[k] = 0;
      h->total_ms[k] = 0.0;
    }
    return MPCMMD_OK;
  });
}

int mpcmmd_kernel_times(mpcmmd_handle* h, int32_t* launches, double* total_ms, int32_t max_kernels) {
  if (!h) return fail(MPCMMD_E_INVALID, "null handle");
  return guarded([&] {
    check_device(h);
    h->collect();
    for (int k = 0; k < kNumKernels && k < max_kernels; ++k) {
      if (launches) launches[k] = h->launches[k];
      if (total_ms) total_ms[k] = h->total_ms[k];
    }
    return int(kNumKernels);
  });
}

const char* mpcmmd_kernel_name(int32_t id) {
  return (id >= 0 && id < kNumKernels) ? kKernelNames[id] : nullptr;
}

int mpcmmd_buffer_info(mpcmmd_handle* h, const char* name, size_t* bytes) {
  if (!h || !name) return fail(MPCMMD_E_INVALID, "null argument");
  if (std::string(name) == "*") {  // every device buffer of the handle
    size_t tot = 0;
    for (auto& kv : h->bufs) tot += kv.second.second;
    if (bytes) *bytes = tot;
    return MPCMMD_OK;
  }
  auto it = h->bufs.find(name);
  if (it == h->bufs.end()) return fail(MPCMMD_E_INVALID, std::string("no buffer ") + name);
  if (bytes) *bytes = it->second.second;
  return MPCMMD_OK;
}

int mpcmmd_read(mpcmmd_handle* h, const char* name, void* dst, size_t bytes) {
  if (!h || !name || !dst) return fail(MPCMMD_E_INVALID, "null argument");
  auto it = h->bufs.find(name);
  if (it == h->bufs.end()) return fail(MPCMMD_E_INVALID, std::string("no buffer ") + name);
  if (bytes > it->second.second) return fail(MPCMMD_E_INVALID, "read larger than buffer");
  return guarded([&] {
    check_device(h);
    HIPC(hipStreamSynchronize(h->stream));
    HIPC(hipMemcpy(dst, it->second.first, bytes, hipMemcpyDeviceToHost));
    return MPCMMD_OK;
  });
}

int mpcmmd_write(mpcmmd_handle* h, const char* name, const void* src, size_t bytes) {
  if (!h || !name || !src) return fail(MPCMMD_E_INVALID, "null argument");
  auto it = h->bufs.find(name);
  if (it == h->bufs.end()) return fail(MPCMMD_E_INVALID, std::string("no buffer ") + name);
  if (bytes > it->second.second) return fail(MPCMMD_E_INVALID, "write larger than buffer");
  return guarded([&] {
    check_device(h);
    HIPC(hipStreamSynchronize(h->stream));
    HIPC(hipMemcpy(it->second.first, src, bytes, hipMemcpyHostToDevice));
    if (std::string(name) == "beta_z0" || std::string(name) == "beta_z") h->beta_tables_internal = false;
    if (std::string(name) == "beta_z0") h->sel0_valid = false;
    return MPCMMD_OK;
  });
}

int mpcmmd_run_stage(mpcmmd_handle* h, int32_t stage, int32_t t) {
  if (!h) return fail(MPCMMD_E_INVALID, "null handle");
  if (!h->begun) return fail(MPCMMD_E_STATE, "run_stage before mpcmmd_begin");
  const bool beta_stage = stage >= 5 && stage <= 7;
  if (t < 0 || (!beta_stage && t >= h->T)) return fail(MPCMMD_E_INVALID, "iteration out of range");
  return guarded([&] {
    check_device(h);
    run_stage(h, stage, t);
    if (stage == 3) h->last_t = t;
    HIPC(hipStreamSynchronize(h->stream));
    return MPCMMD_OK;
  });
}

int mpcmmd_host_constant(const mpcmmd_config* cfg, const char* name, double* dst, size_t count) {
  if (!cfg || !name) return fail(MPCMMD_E_INVALID, "null argument");
  try {
    ProblemConsts c = build_constants(cfg->num_prime, cfg->variant);
    const std::vector<double>* v = nullptr;
    std::string n(name);
    if (n == "P") v = &c.P;
    else if (n == "Pdot") v = &c.Pd;
    else if (n == "Pddot") v = &c.Pdd;
    else if (n == "P_prime") v = &c.P_prime;
    else if (n == "P64") v = &c.P64;
    else if (n == "Pdot64") v = &c.Pd64;
    else if (n == "Pddot64") v = &c.Pdd64;
    else if (n == "guess_kinv_x") v = &c.guess_kinv_x;
    else if (n == "guess_kinv_y") v = &c.guess_kinv_y;
    else if (n == "proj_kinv_x") v = &c.proj_kinv_x;
    else if (n == "proj_kinv_y") v = &c.proj_kinv_y;
    else if (n == "fit") v = &c.fit;
    std::vector<double> dk[2];
    if (n == "det_kinv_x" || n == "det_kinv_y") {
      det_projection_kinv(c, cfg->num_obs, dk[0], dk[1]);
      v = &dk[n == "det_kinv_y" ? 1 : 0];
    }
    if (!v) return fail(MPCMMD_E_INVALID, "unknown constant " + n);
    if (dst) {
      if (count < v->size()) return fail(MPCMMD_E_INVALID, "dst too small");
      std::memcpy(dst, v->data(), v->size() * 8);
    }
    return int(v->size());
  } catch (const std::exception& e) {
    return fail(MPCMMD_E_INVALID, e.what());
  }
}

int mpcmmd_validate(const mpcmmd_validate_args* a) {
  if (!a) return fail(MPCMMD_E_INVALID, "null argument");
  const int K = a->num_cfg, O = a->num_obs, H = a->num_prime, R = a->num_rollouts;
  if (K < 0 || R < 1 || !validate_shape_ok(O, H)) return fail(MPCMMD_E_INVALID, "validate: shape out of range");
  if (a->noise != MPCMMD_NOISE_GAUSSIAN && a->noise != MPCMMD_NOISE_BETA) return fail(MPCMMD_E_INVALID, "noise");
  if (a->variant != MPCMMD_VARIANT_STATIC && a->variant != MPCMMD_VARIANT_DYNAMIC)
    return fail(MPCMMD_E_UNSUPPORTED, "validate: static / dynamic variants (S/validation.py, D/validation.py)");
  if (K == 0) return MPCMMD_OK;
  if (!a->cx || !a->cy || !a->init_state || !a->x_obs || !a->y_obs || !a->keys || !a->count || !a->count_lane)
    return fail(MPCMMD_E_INVALID, "null argument");
  return guarded([&] {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) throw HipError("no HIP device visible");
    if (a->device < 0 || a->device >= ndev) throw std::invalid_argument("device out of range");
    HIPC(hipSetDevice(a->device));
    const ProblemConsts pc = build_constants(H, a->variant);
    std::vector<float> basis(2 * kNum * kNvar);
    for (int i = 0; i < kNum * kNvar; ++i) {
      basis[i] = float(pc.Pd[i]);
      basis[kNum * kNvar + i] = float(pc.Pdd[i]);
    }
    std::vector<std::pair<void*, size_t>> bufs;
    auto up = [&](const void* src, size_t bytes) -> void* {
      void* d = nullptr;
      HIPC(hipMalloc(&d, bytes));
      bufs.push_back({d, bytes});
      if (src) HIPC(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice));
      return d;
    };
    struct Free {
      std::vector<std::pair<void*, size_t>>& b;
      ~Free() {
        for (auto& x : b) (void)hipFree(x.first);
      }
    } guard{bufs};
    ValidateParams v{};
    v.K = K, v.O = O, v.H = H, v.R = R, v.noise = a->noise;
    v.noise_level = a->noise_level, v.acc_const = a->acc_const_noise, v.steer_const = a->steer_const_noise;
    v.K_steer = pc.K_steer, v.y_lb = pc.y_lb, v.y_ub = pc.y_ub, v.seed = a->seed;
    v.Pdot = (const float*)up(basis.data(), kNum * kNvar * 4);
    v.Pddot = (const float*)up(basis.data() + kNum * kNvar, kNum * kNvar * 4);
    v.cx = (const double*)up(a->cx, size_t(K) * 11 * 8);
    v.cy = (const double*)up(a->cy, size_t(K) * 11 * 8);
    v.init_state = (const double*)up(a->init_state, size_t(K) * 6 * 8);
    v.x_obs = (const float*)up(a->x_obs, size_t(K) * O * 100 * 4);
    v.y_obs = (const float*)up(a->y_obs, size_t(K) * O * 100 * 4);
    v.draws = a->draws ? (const double*)up(a->draws, size_t(K) * 3 * R * H * 8) : nullptr;
    v.keys = (const uint32_t*)up(a->keys, size_t(K) * 4);
    v.count = (int32_t*)up(nullptr, size_t(K) * 4);
    v.count_lane = (int32_t*)up(nullptr, size_t(K) * 4);
    launch_validate(v, nullptr);
    HIPC(hipGetLastError());
    HIPC(hipDeviceSynchronize());
    HIPC(hipMemcpy(a->count, v.count, size_t(K) * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(a->count_lane, v.count_lane, size_t(K) * 4, hipMemcpyDeviceToHost));
    return MPCMMD_OK;
  });
}

int mpcmmd_obs_dynamic_traj(int32_t num_obs, const float* x0, const float* y0, const float* vx0, const float* vy0,
                            const float* v_des, float y_des, float* x_traj, float* y_traj) {
  if (num_obs < 0) return fail(MPCMMD_E_INVALID, "num_obs < 0");
  if (num_obs > 0 && (!x0 || !y0 || !vx0 || !vy0 || !v_des || !x_traj || !y_traj))
    return fail(MPCMMD_E_INVALID, "null argument");
  try {
    static const DynObsConsts c = build_dyn_obs_consts();
    dyn_obs_traj(c, num_obs, x0, y0, vx0, vy0, v_des, y_des, x_traj, y_traj);
    return MPCMMD_OK;
  } catch (const std::exception& e) {
    return fail(MPCMMD_E_INVALID, e.what());
  }
}

}  // extern "C"
