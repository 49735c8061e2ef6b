// Issue cost of the e4m3 conversions the corrected network could run per K-step, alone and
// beside the conv's MFMA stream (8 waves per CU, 2 per SIMD, like kNNForward):
//   OP 0: v_cvt_scalef32_pk_fp8_f16 (two fp16 -> two e4m3, the word half kept)
//   OP 1: v_cvt_pk_fp8_f32          (two f32 -> two e4m3)
//   OP 2: v_add_f32                 (reference VALU op)
// MODE 0: conversions only (16 independent chains); MODE 1: per iteration 6 16x16x32 f16
// MFMAs + 3 scaled 16x16x128 f8 MFMAs (one corrected K-step pair's worth / 2) and NCVT
// conversions.  Prints cycles per wave and iteration.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/cvt_rate tools/cvt_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2x __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i8v __attribute__((ext_vector_type(8)));

template <int OP, int MODE, int NCVT>
__global__ void __launch_bounds__(512, 2) k(float* out, unsigned long long* cyc, int iters) {
  const float x = threadIdx.x * 0.001f;
  int r[16];
  float fr[16];
  for(int i = 0; i < 16; i++) {
    r[i] = threadIdx.x + i;
    fr[i] = x + i;
  }
  h8 a[2], b[3];
  for(int t = 0; t < 2; t++) a[t] = (h8)(_Float16)(x + t);
  for(int c = 0; c < 3; c++) b[c] = (h8)(_Float16)(c * 0.5f);
  i8v qa[2], qb[3];
  for(int t = 0; t < 2; t++) qa[t] = (i8v)(0x38383838 + t);
  for(int c = 0; c < 3; c++) qb[c] = (i8v)(0x30303030 + c);
  f4 acc[2][3];
  for(int t = 0; t < 2; t++)
    for(int c = 0; c < 3; c++) acc[t][c] = (f4){0, 0, 0, 0};
  __syncthreads();
  const unsigned long long c0 = clock64();
  for(int it = 0; it < iters; it++) {
    if(MODE == 1) {
#pragma unroll
      for(int t = 0; t < 2; t++)
#pragma unroll
        for(int c = 0; c < 3; c++)
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[c], a[t], acc[t][c], 0, 0, 0);
      if(it & 1) {
#pragma unroll
        for(int t = 0; t < 2; t++)
#pragma unroll
          for(int c = 0; c < 3; c++)
            acc[t][c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(qb[c], qa[t], acc[t][c], 0, 0, 0, 120, 0, 127);
      }
    }
#pragma unroll
    for(int i = 0; i < (MODE == 0 ? 16 : NCVT); i++) {
      const int j = i & 15;
      if(OP == 0) {
        s16x2 v = __builtin_bit_cast(s16x2, r[j]);
        v = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(v, h2x{(_Float16)fr[j], (_Float16)x}, 2.0f, false);
        r[j] = __builtin_bit_cast(int, v);
      } else if(OP == 1) {
        r[j] = __builtin_amdgcn_cvt_pk_fp8_f32(fr[j], x, r[j], false);
      } else {
        fr[j] = fr[j] + x;
      }
      if(MODE == 1 && j == 15) {
        // feed the converted bytes back into the MFMA operands (a real dependency)
        qa[0][i & 7] ^= r[j];
      }
    }
  }
  const unsigned long long c1 = clock64();
  float s = 0;
  for(int i = 0; i < 16; i++) s += (float)r[i] + fr[i];
  for(int t = 0; t < 2; t++)
    for(int c = 0; c < 3; c++) s += acc[t][c][0];
  s += (float)qa[0][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if((threadIdx.x & 63) == 0)
    cyc[blockIdx.x * 8 + threadIdx.x / 64] = c1 - c0;
}

template <int OP, int MODE, int NCVT>
static void run(const char* name, float* out, unsigned long long* cyc) {
  const int iters = 1024, grid = 256;
  for(int rep = 0; rep < 2; rep++)
    hipLaunchKernelGGL((k<OP, MODE, NCVT>), dim3(grid), dim3(512), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(grid * 8);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for(auto v : h) s += (double)v;
  s /= h.size();
  const double per = s / iters;
  if(MODE == 0)
    printf("%-44s %7.1f cycles per iteration (16 ops/wave) = %.2f cycles per op per wave\n", name, per, per / 16);
  else
    printf("%-44s %7.1f cycles per iteration (6 f16 + 3 f8 MFMA per 2 its, %d conversions)\n", name, per, NCVT);
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 256 * 8 * 8);
  run<0, 0, 0>("cvt_scalef32_pk_fp8_f16 alone", out, cyc);
  run<1, 0, 0>("cvt_pk_fp8_f32 alone", out, cyc);
  run<2, 0, 0>("v_add_f32 alone", out, cyc);
  run<2, 1, 0>("MFMA stream, no conversion", out, cyc);
  run<0, 1, 8>("MFMA stream + 8 cvt_scalef32_pk_fp8_f16", out, cyc);
  run<0, 1, 12>("MFMA stream + 12 cvt_scalef32_pk_fp8_f16", out, cyc);
  run<0, 1, 20>("MFMA stream + 20 cvt_scalef32_pk_fp8_f16", out, cyc);
  run<1, 1, 20>("MFMA stream + 20 cvt_pk_fp8_f32", out, cyc);
  run<2, 1, 20>("MFMA stream + 20 v_add_f32", out, cyc);
  return 0;
}
