// Steady-state cycles of the corrected network's 96->96 3x3 convolution (convTilesB, the
// borderless 5-board NN_MODE_F8C instance, capped at KC_F8C_VGPR like kNNForwardCap) and
// of ablations of it (convTilesB's DBG flags), one workgroup per CU on every CU:
//   real        as shipped: weight ring (LDS-DMA + per-chunk vmcnt wait + barrier),
//               fp16 and e4m3 fragment reads, f16 + scaled f8 MFMAs
//   nodma       no weight requests (the ring's slots keep their contents)
//   nobar       requests without their waits and barriers
//   nowait      barriers without the DMA waits before them
//   nodma-nobar neither
//   nof8        no scaled e4m3 MFMAs (the fast instance's MFMA work)
//   noplane2    no second-plane (e4m3) fragment reads
//   noloads     fragments read at the first K-step only (MFMAs on registers)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Ikatacoffee_amd/csrc
//        -o tools/_build/convb_bench tools/convb_bench.hip
#include "../katacoffee_amd/csrc/nn.hip"

#include <cstdio>
#include <vector>

using namespace kc;
constexpr int REPS = 16;
using GC = NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_F8C, true>;

template <int DBG>
__global__ void __launch_bounds__(512, 2) __attribute__((amdgpu_num_vgpr(KC_F8C_VGPR ? KC_F8C_VGPR : 128)))
    kConvB(const h16x8* __restrict__ w, float* out, unsigned long long* cyc) {
  using G = GC;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rg = wave >> 1, cg = wave & 1;
  const int tstart = rg * G::MAXT;
  uint16_t* act = reinterpret_cast<uint16_t*>(smem);
  h16x8* wl = reinterpret_cast<h16x8*>(smem + G::OFF_W);
  // fp16 activations in (0.25, 1); e4m3 plane bytes 0x30-0x3f (finite, ~0.5-1)
  for(int i = tid; i < G::PLANE_BYTES / 2; i += G::NT)
    act[i] = (uint16_t)(0x3400 + (i * 7 & 0x3ff));
  for(int i = tid; i < G::PLANE2_BYTES; i += G::NT)
    reinterpret_cast<uint8_t*>(smem)[G::PLANE_BYTES + i] = (uint8_t)(0x30 + (i & 15));
  constexpr int CH = G::tapPieces(3);
  stageChunk<G::NW>(w, ldsAddr(wl) + G::WSLOT * 16, CH, wave, lane);  // conv 1's chunk 0: slot 1
  waitVm<0>();
  __syncthreads();
  int rb[G::MAXT];
  uint32_t vm[G::MAXT];
  aRowsBL<G>(rb, vm, tstart, lane);
  f32x4 acc[G::MAXT][G::NCT];
  zeroAcc<G>(acc);
  const int sA = 127 - F8C_SHIFT - 8;
  const unsigned long long t0 = clock64();
  for(int r = 0; r < REPS; r += 2) {
    // two convs per iteration: chunk parities 1 and 0 alternate as in the network
    convTilesB<G, 9, 3, 1, DBG>(act, w, wl, acc, rb, vm, cg, lane, tid, w, CH, 9, sA);
    if(!(DBG & 1))
      waitVm<0>();
    __syncthreads();
    convTilesB<G, 9, 3, 0, DBG>(act, w, wl, acc, rb, vm, cg, lane, tid, w, CH, 9, sA);
    if(!(DBG & 1))
      waitVm<0>();
    __syncthreads();
  }
  const unsigned long long t1 = clock64();
  float s = 0;
  for(int t = 0; t < G::MAXT; t++)
    for(int ct = 0; ct < G::NCT; ct++)
      s += acc[t][ct][0] + acc[t][ct][3];
  out[blockIdx.x * G::NT + tid] = s;
  if(tid == 0)
    cyc[blockIdx.x] = t1 - t0;
}

template <int DBG>
void run(const char* name, const h16x8* w, float* out, unsigned long long* cyc) {
  using G = GC;
  const int grid = 256;
  KC_HIP(hipFuncSetAttribute((const void*)kConvB<DBG>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
  for(int it = 0; it < 3; it++)
    hipLaunchKernelGGL((kConvB<DBG>), dim3(grid), dim3(G::NT), G::LDS, 0, w, out, cyc);
  KC_HIP(hipDeviceSynchronize());
  std::vector<unsigned long long> c(grid);
  KC_HIP(hipMemcpy(c.data(), cyc, grid * 8, hipMemcpyDeviceToHost));
  double avg = 0;
  for(auto v : c)
    avg += v;
  avg /= grid;
  // MFMA issue floor per SIMD per conv: 27 K-steps x 6 f16 MFMAs x 16 cycles + 13.5 x 6
  // scaled f8 MFMAs x 32 cycles, two waves per SIMD
  const double floor = (27.0 * 6 * 16 + 13.5 * 6 * 32) * 2;
  printf("corrected BL %-12s %8.0f cycles per conv (%.1f per K-step; MFMA floor %.0f)\n", name, avg / REPS,
         avg / REPS / 27, floor);
}

int main() {
  using G = GC;
  std::vector<uint16_t> hw((size_t)9 * G::tapPieces(3) * 512);
  for(size_t i = 0; i < hw.size(); i++)
    hw[i] = (uint16_t)(0x2000 + (i * 13 & 0x7ff)) & 0x3f3f;  // fp16 and e4m3 bytes finite
  h16x8* w;
  KC_HIP(hipMalloc(&w, hw.size() * 2));
  KC_HIP(hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  float* out;
  unsigned long long* cyc;
  KC_HIP(hipMalloc(&out, (size_t)256 * G::NT * 4));
  KC_HIP(hipMalloc(&cyc, 256 * 8));
  run<0>("real", w, out, cyc);
  run<1>("nodma", w, out, cyc);
  run<2>("nobar", w, out, cyc);
  run<3>("nodma-nobar", w, out, cyc);
  run<4>("nof8", w, out, cyc);
  run<8>("noplane2", w, out, cyc);
  run<12>("nof8-noplane2", w, out, cyc);
  run<32>("nowait", w, out, cyc);
  run<16>("noloads", w, out, cyc);
  run<19>("noloads-nodma-nobar", w, out, cyc);
  return 0;
}
