// MFMA issue rate with the conv kernel's register pattern: 4 A x 3 B fragments,
// 12 accumulators per wave, 512-thread workgroups (2 waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(512, 2) k(float* out, unsigned long long* cyc, int iters) {
  h8 a[4], b[3];
  for(int t = 0; t < 4; t++) a[t] = (h8)(_Float16)(threadIdx.x * 0.001f + t);
  for(int c = 0; c < 3; c++) b[c] = (h8)(_Float16)(c * 0.5f);
  f4 acc[4][3];
  for(int t = 0; t < 4; t++) for(int c = 0; c < 3; c++) acc[t][c] = (f4){0, 0, 0, 0};
  __syncthreads();
  unsigned long long t0 = clock64();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for(int it = 0; it < iters; it++) {
#pragma unroll
    for(int t = 0; t < 4; t++)
#pragma unroll
      for(int c = 0; c < 3; c++)
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], b[c], acc[t][c], 0, 0, 0);
  }
  unsigned long long t1 = clock64();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for(int t = 0; t < 4; t++) for(int c = 0; c < 3; c++) s += acc[t][c][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if(threadIdx.x == 0) {
    cyc[2 * blockIdx.x] = t1 - t0;
    cyc[2 * blockIdx.x + 1] = r1 - r0;  // 100 MHz constant clock
  }
}
int main() {
  float* out; unsigned long long* cyc;
  hipMalloc(&out, 64 << 20); hipMalloc(&cyc, 1 << 16);
  const int iters = 1024;
  for(int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, out, cyc, iters);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, out, cyc, iters);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long cc[2]; hipMemcpy(cc, cyc, 16, hipMemcpyDeviceToHost);
  unsigned long long c = cc[0];
  printf("wave0: %llu ticks in %.1f us (memrealtime) -> tick %.3f GHz\n", c, cc[1] / 100.0, c / (cc[1] * 10.0));
  double mf = iters * 12.0 * 2;  // per SIMD: 2 waves
  printf("256 WGs x 512 thr: wall %.3f ms -> %.1f ns/MFMA/SIMD; wave0 %.1f cycles per own MFMA, TFLOP/s %.0f\n", ms,
         ms * 1e6 / mf, (double)c / (iters * 12.0), 256 * 8 * iters * 12.0 * 16384 / (ms * 1e-3) / 1e12);
  return 0;
}
