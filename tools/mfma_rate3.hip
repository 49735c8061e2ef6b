// Per-block start/end (s_memrealtime, 100 MHz) of the conv-pattern MFMA loop:
// tells whether a grid runs in one wave of workgroups and the per-SIMD MFMA rate.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(512, 1) k(float* out, unsigned long long* ts, int iters) {
  h8 a[4], b[3];
  for(int t = 0; t < 4; t++) a[t] = (h8)(_Float16)(threadIdx.x * 0.001f + t);
  for(int c = 0; c < 3; c++) b[c] = (h8)(_Float16)(c * 0.5f);
  f4 acc[4][3];
  for(int t = 0; t < 4; t++) for(int c = 0; c < 3; c++) acc[t][c] = (f4){0, 0, 0, 0};
  __syncthreads();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long c0 = clock64();
  for(int it = 0; it < iters; it++) {
#pragma unroll
    for(int t = 0; t < 4; t++)
#pragma unroll
      for(int c = 0; c < 3; c++)
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], b[c], acc[t][c], 0, 0, 0);
  }
  unsigned long long c1 = clock64();
  __syncthreads();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for(int t = 0; t < 4; t++) for(int c = 0; c < 3; c++) s += acc[t][c][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if(threadIdx.x == 0) {
    ts[3 * blockIdx.x] = r0;
    ts[3 * blockIdx.x + 1] = r1;
    ts[3 * blockIdx.x + 2] = c1 - c0;
  }
}
int main() {
  float* out; unsigned long long* ts;
  hipMalloc(&out, 64 << 20); hipMalloc(&ts, 1 << 20);
  const int iters = 2048;
  for(int grid : {128, 256, 512}) {
    for(int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, 0, out, ts, iters);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(3 * grid);
    hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long s0 = ~0ull, e1 = 0;
    double dmin = 1e30, dmax = 0, cyc = 0;
    for(int b = 0; b < grid; b++) {
      s0 = std::min(s0, h[3 * b]); e1 = std::max(e1, h[3 * b + 1]);
      double d = (h[3 * b + 1] - h[3 * b]) / 100.0;
      dmin = std::min(dmin, d); dmax = std::max(dmax, d);
      cyc += h[3 * b + 2];
    }
    int late = 0;
    for(int b = 0; b < grid; b++) late += (h[3 * b] - s0) > 200;  // started > 2 us after the first
    cyc /= grid;
    double span = (e1 - s0) / 100.0;
    printf("grid %3d: span %.1f us, block dur %.1f..%.1f us, %d blocks started >2us late, %.0f cyc/block -> "
           "%.2f cyc per MFMA per SIMD (2 waves), clock %.2f GHz, %.0f TFLOP/s over span\n",
           grid, span, dmin, dmax, late, cyc, cyc / (iters * 12.0 * 2), cyc / (dmax * 1e3),
           grid * 8.0 * iters * 12 * 16384 / (span * 1e-6) / 1e12);
  }
  return 0;
}
