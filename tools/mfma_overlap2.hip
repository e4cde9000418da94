// Two waves on one SIMD: does another wave's VALU work run while a wave's
// fp64 MFMAs execute?  (profiling aid for k_bsample, not product code)
// Workgroup of 4 or 8 waves: waves 0-3 (one per SIMD) issue rounds of 6
// independent v_mfma_f64_16x16x4; waves 4-7 (the second wave of each SIMD)
// issue independent VALU instructions (KIND 0: v_add_f32, 1: v_add_f64).
// Prints the clocks of an MFMA wave and of a VALU wave.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
#define MF(acc) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))

template <int KIND>
__global__ void k_pair(unsigned long long* out, float* sink, int rounds, int vrounds) {
  const int w = threadIdx.x >> 6;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (w < 4) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0;
    const double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    for (int r = 0; r < rounds; ++r) {
      MF(c0); MF(c1); MF(c2); MF(c3); MF(c4); MF(c5);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::);
    const d4 s = c0 + c1 + c2 + c3 + c4 + c5;
    sink[threadIdx.x] = float(s.x + s.y + s.z + s.w);
  } else {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 1.5f;
    double d0 = x0, d1 = x1, d2 = x2, d3 = x3, e = 1.5;
    for (int r = 0; r < vrounds; ++r) {
      if constexpr (KIND == 0) {
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x0) : "v"(y));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x1) : "v"(y));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x2) : "v"(y));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x3) : "v"(y));
      } else {
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(d0) : "v"(e));
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(d1) : "v"(e));
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(d2) : "v"(e));
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(d3) : "v"(e));
      }
    }
    sink[threadIdx.x] = x0 + x1 + x2 + x3 + float(d0 + d1 + d2 + d3);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[w] = t1 - t0;
}

int main() {
  unsigned long long* d_out;
  float* sink;
  unsigned long long h[8] = {};
  (void)hipMalloc(&d_out, 64);
  (void)hipMalloc(&sink, 4096);
  const int rounds = 2000, vrounds = 12000;  // 12000 x 4 VALU ~ the MFMA waves' span at 4 clocks each
  struct Case { const char* name; int threads; int kind; };
  const Case cases[] = {{"mfma alone", 256, 0}, {"mfma + add_f32 wave", 512, 0}, {"mfma + add_f64 wave", 512, 1}};
  for (const Case& c : cases) {
    for (int rep = 0; rep < 2; ++rep) {
      if (c.kind == 0)
        hipLaunchKernelGGL(k_pair<0>, dim3(1), dim3(c.threads), 0, 0, d_out, sink, rounds, vrounds);
      else
        hipLaunchKernelGGL(k_pair<1>, dim3(1), dim3(c.threads), 0, 0, d_out, sink, rounds, vrounds);
    }
    (void)hipMemcpy(h, d_out, 64, hipMemcpyDeviceToHost);
    printf("%-22s MFMA wave: %.1f clocks per MFMA", c.name, double(h[0]) / (6.0 * rounds));
    if (c.threads > 256) printf("   VALU wave: %.1f clocks per VALU instruction", double(h[4]) / (4.0 * vrounds));
    printf("\n");
  }
  // the VALU waves alone (no MFMA wave running): launch 512 with rounds = 0
  hipLaunchKernelGGL(k_pair<0>, dim3(1), dim3(512), 0, 0, d_out, sink, 0, vrounds);
  hipLaunchKernelGGL(k_pair<0>, dim3(1), dim3(512), 0, 0, d_out, sink, 0, vrounds);
  (void)hipMemcpy(h, d_out, 64, hipMemcpyDeviceToHost);
  printf("%-22s VALU wave: %.1f clocks per VALU instruction\n", "add_f32 alone", double(h[4]) / (4.0 * vrounds));
  hipLaunchKernelGGL(k_pair<1>, dim3(1), dim3(512), 0, 0, d_out, sink, 0, vrounds);
  hipLaunchKernelGGL(k_pair<1>, dim3(1), dim3(512), 0, 0, d_out, sink, 0, vrounds);
  (void)hipMemcpy(h, d_out, 64, hipMemcpyDeviceToHost);
  printf("%-22s VALU wave: %.1f clocks per VALU instruction\n", "add_f64 alone", double(h[4]) / (4.0 * vrounds));
  (void)hipDeviceSynchronize();
  return 0;
}
