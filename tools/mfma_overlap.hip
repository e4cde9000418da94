// Does VALU / memory work issued between fp64 MFMAs of the same wave run in
// their shadow on gfx950?  (profiling aid for k_bsample, not product code)
// One wave alone on its SIMD issues N rounds of 6 independent
// v_mfma_f64_16x16x4 (6 accumulators, so no MFMA waits on another), with F
// filler instructions after each MFMA; inline asm keeps the order exact.
// Prints clocks per round for each filler kind and count.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

#define MF(acc) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))

template <int KIND, int F>
__global__ void k_overlap(unsigned long long* out, float* sink, int rounds) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0;
  const double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  double y0 = x0, y1 = x1;
  float* dst = sink + threadIdx.x;
  auto fill = [&]() {
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if constexpr (KIND == 0)
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(f & 1 ? x1 : x0) : "v"(x2));
      else if constexpr (KIND == 1)
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(f & 1 ? y1 : y0) : "v"(y0));
      else if constexpr (KIND == 2)
        asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f & 1 ? x3 : x2) : "v"(y1));
      else
        asm volatile("global_store_dword %0, %1, off" : : "v"(dst), "v"(x0) : "memory");
    }
  };
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < rounds; ++r) {
    MF(c0); fill();
    MF(c1); fill();
    MF(c2); fill();
    MF(c3); fill();
    MF(c4); fill();
    MF(c5); fill();
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::);
  const d4 s = c0 + c1 + c2 + c3 + c4 + c5;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[64 + threadIdx.x] = float(s.x + s.y + s.z + s.w) + x0 + x1 + x2 + x3 + float(y0 + y1);
}

template <int KIND, int F>
void run(const char* name, unsigned long long* d_out, float* sink, int rounds) {
  unsigned long long h = 0;
  hipLaunchKernelGGL((k_overlap<KIND, F>), dim3(1), dim3(64), 0, 0, d_out, sink, rounds);  // warm
  hipLaunchKernelGGL((k_overlap<KIND, F>), dim3(1), dim3(64), 0, 0, d_out, sink, rounds);
  hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);
  printf("%-10s F=%d  clocks per MFMA %.1f\n", name, F, double(h) / (6.0 * rounds));
}

int main() {
  unsigned long long* d_out;
  float* sink;
  hipMalloc(&d_out, 64);
  hipMalloc(&sink, 4096);
  const int rounds = 2000;
  run<0, 0>("none", d_out, sink, rounds);
  run<0, 4>("add_f32", d_out, sink, rounds);
  run<0, 8>("add_f32", d_out, sink, rounds);
  run<0, 16>("add_f32", d_out, sink, rounds);
  run<1, 4>("add_f64", d_out, sink, rounds);
  run<1, 8>("add_f64", d_out, sink, rounds);
  run<2, 4>("cvt_f32_f64", d_out, sink, rounds);
  run<2, 8>("cvt_f32_f64", d_out, sink, rounds);
  run<3, 1>("store", d_out, sink, rounds);
  run<3, 2>("store", d_out, sink, rounds);
  hipDeviceSynchronize();
  return 0;
}
