// Latency / throughput calibration of the instruction patterns the beta-CEM
// kernels lean on (profiling aid, not product code):
//   clock rate (s_memtime vs s_memrealtime), dependent fp64 FMA, dependent
//   LDS load, ballot + popcount chain, readlane broadcast.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_probe(unsigned long long* out, double* sink, int iters) {
  __shared__ double lds[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += blockDim.x) lds[i] = double(i % 7);
  __syncthreads();
  unsigned long long t0, t1, r0, r1;
  // clock
  r0 = __builtin_amdgcn_s_memrealtime();
  t0 = __builtin_amdgcn_s_memtime();
  double x = lane * 1e-3;
  for (int i = 0; i < iters; ++i) x = fma(x, 1.0000001, 1e-9);
  t1 = __builtin_amdgcn_s_memtime();
  r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
  }
  // dependent LDS loads
  int idx = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) idx = int(lds[idx & 1023]) + lane;
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = t1 - t0;
  // ballot + popcount chain
  unsigned key = lane * 2654435761u;
  unsigned T = 0;
  int acc = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const unsigned cand = T | (1u << (i & 31));
    int c = __popcll(__ballot(key >= cand)) + __popcll(__ballot((key ^ 1) >= cand)) +
            __popcll(__ballot((key ^ 2) >= cand)) + __popcll(__ballot((key ^ 3) >= cand));
    if (c >= 100) T = cand;
    acc += c;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = t1 - t0;
  // readlane broadcast chain (fp64 via two 32-bit halves)
  double v = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(int(b), i & 31), hi = __builtin_amdgcn_readlane(int(b >> 32), i & 31);
    v = v * 0.5 + __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[4] = t1 - t0;
  // independent fp64 FMAs (throughput, 8 chains)
  double a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    a0 = fma(a0, 1.0000001, 1e-9); a1 = fma(a1, 1.0000001, 1e-9); a2 = fma(a2, 1.0000001, 1e-9);
    a3 = fma(a3, 1.0000001, 1e-9); a4 = fma(a4, 1.0000001, 1e-9); a5 = fma(a5, 1.0000001, 1e-9);
    a6 = fma(a6, 1.0000001, 1e-9); a7 = fma(a7, 1.0000001, 1e-9);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[5] = t1 - t0;
  // independent f64 MFMA 16x16x4 (throughput, 4 accumulators)
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  const double fa = 1e-3 * lane, fb = 2e-3 * lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(fb, fa, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fa, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(fb, fb, c3, 0, 0, 0);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[6] = t1 - t0;
  // dependent f64 MFMA chain (one accumulator)
  d4 e0 = {0, 0, 0, 0};
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, e0, 0, 0, 0);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[7] = t1 - t0;
  // independent v_exp_f32 (8 chains)
  float q0 = lane * -1e-3f, q1 = q0 - 1, q2 = q0 - 2, q3 = q0 - 3, q4 = q0 - 4, q5 = q0 - 5, q6 = q0 - 6, q7 = q0 - 7;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    q0 = __builtin_amdgcn_exp2f(q0); q1 = __builtin_amdgcn_exp2f(q1); q2 = __builtin_amdgcn_exp2f(q2);
    q3 = __builtin_amdgcn_exp2f(q3); q4 = __builtin_amdgcn_exp2f(q4); q5 = __builtin_amdgcn_exp2f(q5);
    q6 = __builtin_amdgcn_exp2f(q6); q7 = __builtin_amdgcn_exp2f(q7);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[8] = t1 - t0;
  sink[lane] = x + idx + acc + v + a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + c0[0] + c1[1] + c2[2] + c3[3] + e0[0] +
               q0 + q1 + q2 + q3 + q4 + q5 + q6 + q7;
}

int main() {
  unsigned long long* d;
  double* s;
  const int iters = 4096;
  (void)hipMalloc(&d, 64 * 8);
  (void)hipMalloc(&s, 1024 * 8);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d, s, iters);
    (void)hipDeviceSynchronize();
  }
  unsigned long long h[16];
  (void)hipMemcpy(h, d, 9 * 8, hipMemcpyDeviceToHost);
  std::printf("clock: %llu cycles in %llu ticks of 100 MHz -> %.2f GHz\n", h[0], h[1], h[0] / (h[1] * 10.0));
  std::printf("dependent fp64 fma: %.1f cycles\n", double(h[0]) / iters);
  std::printf("dependent LDS load (+cvt): %.1f cycles\n", double(h[2]) / iters);
  std::printf("4x ballot+popc step: %.1f cycles\n", double(h[3]) / iters);
  std::printf("readlane fp64 bcast step: %.1f cycles\n", double(h[4]) / iters);
  std::printf("8 independent fp64 fma: %.1f cycles\n", double(h[5]) / iters);
  std::printf("4 independent f64 mfma 16x16x4: %.1f cycles\n", double(h[6]) / iters);
  std::printf("dependent f64 mfma 16x16x4: %.1f cycles\n", double(h[7]) / iters);
  std::printf("8 independent v_exp_f32: %.1f cycles\n", double(h[8]) / iters);
  return 0;
}
