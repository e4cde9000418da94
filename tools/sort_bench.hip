// Microbenchmark of one-workgroup sorts of N <= 1024 distinct 64-bit keys
// (k_select's stable argsort of the projection residuals), one key per
// thread.  Build and run (GPU box):
//   hipcc -O3 --offload-arch=gfx950 -I mpc-mmd_amd/csrc tools/sort_bench.hip -o /tmp/sort_bench && /tmp/sort_bench
// Variants: 0 = bitonic_sort_reg (lane shuffles through ds_bpermute, LDS for
// strides >= 64), 1 = the same network with DPP / permlane exchanges in the
// wave, 2 = the wave bitonic to sorted 64-runs, then pairwise merges by a
// binary search of each key in the partner run (one barrier per level).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "block.hpp"
#include "sort.hpp"

using namespace mpcmmd;
using u64 = unsigned long long;

template <int V>
__global__ __launch_bounds__(1024) void k_sort(const u64* in, u64* out, int N, int reps, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) u64 k[2 * 1024];
  const int i = threadIdx.x;
  unsigned long long t0 = 0;
  for (int r = 0; r < reps; ++r) {
    if (r == 1) t0 = __builtin_amdgcn_s_memrealtime();  // rep 0 warms up
    u64 a = i < N ? in[i] : ~0ull;
    if constexpr (V == 0) {
      k[i] = a;
      bitonic_sort_reg(k, N);
      if (i < N) out[i] = k[i];
    } else if constexpr (V == 1) {
      a = bitonic_reg_dpp(a, N, k);
      if (i < N) out[i] = a;
    } else {
      int idx = i;
      a = merge_sort_reg(a, idx, N, k);
      if (i < N) out[idx] = a;
    }
    __syncthreads();
  }
  if (i == 0) clk[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main() {
  const int N = 1024, reps = 21;
  std::vector<u64> h(N);
  srand(5);
  for (int i = 0; i < N; ++i) h[i] = (u64(unsigned(rand()) & 0x7FFFFFFFu) << 32) | unsigned(i);
  std::vector<u64> ref = h;
  std::sort(ref.begin(), ref.end());
  u64 *din, *dout, *dclk;
  hipMalloc(&din, N * 8);
  hipMalloc(&dout, N * 8);
  hipMalloc(&dclk, 8);
  hipMemcpy(din, h.data(), N * 8, hipMemcpyHostToDevice);
  for (int v = 0; v < 3; ++v) {
    for (int n : {64, 128, 1024}) {
      std::vector<u64> hn(h.begin(), h.begin() + n), rn = hn;
      std::sort(rn.begin(), rn.end());
      hipMemcpy(din, hn.data(), n * 8, hipMemcpyHostToDevice);
      hipMemset(dout, 0, N * 8);
      if (v == 0) hipLaunchKernelGGL(k_sort<0>, dim3(1), dim3(1024), 0, 0, din, dout, n, reps, dclk);
      if (v == 1) hipLaunchKernelGGL(k_sort<1>, dim3(1), dim3(1024), 0, 0, din, dout, n, reps, dclk);
      if (v == 2) hipLaunchKernelGGL(k_sort<2>, dim3(1), dim3(1024), 0, 0, din, dout, n, reps, dclk);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("variant %d n %d: launch failed\n", v, n);
        return 1;
      }
      std::vector<u64> got(n);
      unsigned long long clk = 0;
      hipMemcpy(got.data(), dout, n * 8, hipMemcpyDeviceToHost);
      hipMemcpy(&clk, dclk, 8, hipMemcpyDeviceToHost);
      const bool ok = got == rn;
      printf("variant %d n %4d: %s  %.2f us per sort (load + sort + store)\n", v, n, ok ? "ok " : "BAD",
             clk / 100.0 / (reps - 1));
    }
  }
  return 0;
}
