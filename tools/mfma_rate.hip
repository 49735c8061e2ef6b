// Microbenchmark: issue rate of v_mfma_f32_16x16x32_f16 / _bf16 on one SIMD
// (cycles per instruction, shader clock), one and two waves per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool BF>
__global__ void k(float* out, unsigned long long* cyc, int iters) {
  h8 a, b;
  b8 ab, bb;
  for(int i = 0; i < 8; i++) {
    a[i] = (_Float16)(threadIdx.x * 0.001f + i);
    b[i] = (_Float16)(i * 0.5f);
    ab[i] = (__bf16)(threadIdx.x * 0.001f + i);
    bb[i] = (__bf16)(i * 0.5f);
  }
  f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  __syncthreads();
  unsigned long long t0 = clock64();
  for(int it = 0; it < iters; it++) {
    if(BF) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c3, 0, 0, 0);
    }
  }
  unsigned long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
  if(threadIdx.x == 0)
    cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 1 << 12);
  const int iters = 4096;
  for(int bf = 0; bf < 2; bf++)
    for(int waves : {4, 8, 16}) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for(int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0, 0);
        if(bf)
          hipLaunchKernelGGL(k<true>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, iters);
        else
          hipLaunchKernelGGL(k<false>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, iters);
        hipEventRecord(e1, 0);
      }
      hipDeviceSynchronize();
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("   wall %.3f ms -> %.2f ns per MFMA per SIMD; ", ms, ms * 1e6 / (iters * 4.0 * waves / 4.0));
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("%s waves/CU=%2d (%.0f/SIMD): %.2f cycles per MFMA per SIMD\n", bf ? "bf16" : "f16 ", waves,
             waves / 4.0, (double)c / (iters * 4.0 * (waves / 4.0)));
    }
  return 0;
}
