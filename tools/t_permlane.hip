// checks the lane semantics of the permlane swaps / DPP used by k_bkernel's transpose_sum8
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__device__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
__global__ void k(const float* in, float* out, float* sw) {
  const int lane = threadIdx.x;
  float v[8];
  for (int j = 0; j < 8; ++j) v[j] = in[j * 64 + lane];
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[0]), __float_as_uint(v[4]), false, false);
  sw[lane] = __uint_as_float(r[0]);
  sw[64 + lane] = __uint_as_float(r[1]);
  auto r2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[0]), __float_as_uint(v[4]), false, false);
  sw[128 + lane] = __uint_as_float(r2[0]);
  sw[192 + lane] = __uint_as_float(r2[1]);
  float a[4], c2[2];
  for (int i = 0; i < 4; ++i) {
    float x = v[i], y = v[4 + i];
    __asm__ volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
    a[i] = x + y;
  }
  for (int i = 0; i < 2; ++i) {
    float x = a[i], y = a[2 + i];
    __asm__ volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
    c2[i] = x + y;
  }
  const bool b3 = lane & 8;
  const float y0 = __int_as_float(dpp_i<0x128>(__float_as_int(c2[0]))), y1 = __int_as_float(dpp_i<0x128>(__float_as_int(c2[1])));
  float x = b3 ? c2[1] + y1 : c2[0] + y0;
  x += __int_as_float(dpp_i<0xB1>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x4E>(__float_as_int(x)));
  x += __int_as_float(dpp_i<0x124>(__float_as_int(x)));
  out[lane] = x;
}
int main() {
  float h[512], o[64], s[256];
  for (int j = 0; j < 8; ++j)
    for (int l = 0; l < 64; ++l) h[j * 64 + l] = float((j + 1) * 1000 + l);
  float *di, *dout, *ds;
  hipMalloc(&di, sizeof h); hipMalloc(&dout, sizeof o); hipMalloc(&ds, sizeof s);
  hipMemcpy(di, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout, ds);
  hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
  hipMemcpy(s, ds, sizeof s, hipMemcpyDeviceToHost);
  printf("swap32 r0:"); for (int l = 0; l < 64; l += 8) printf(" %g", s[l]); printf(" | lane 40: %g\n", s[40]);
  printf("swap32 r1:"); for (int l = 0; l < 64; l += 8) printf(" %g", s[64 + l]); printf("\n");
  printf("swap16 r0:"); for (int l = 0; l < 64; l += 8) printf(" %g", s[128 + l]); printf("\n");
  printf("swap16 r1:"); for (int l = 0; l < 64; l += 8) printf(" %g", s[192 + l]); printf("\n");
  int bad = 0;
  for (int j = 0; j < 8; ++j) {
    double want = 0;
    for (int l = 0; l < 64; ++l) want += h[j * 64 + l];
    printf("slot %d: lane %d = %g want %g\n", j, 8 * j + 4, o[8 * j + 4], want);
    bad += o[8 * j + 4] != float(want);
  }
  printf(bad ? "FAIL\n" : "OK\n");
  return bad;
}
