// Steady-state cycles of the network's 96->96 3x3 convolution (convTiles) and of
// stripped variants for each fused-kernel instance (8 / 5 boards on 8 waves, one
// workgroup per CU).
//   real      : convTiles as shipped (LDS weight ring + barriers + fragment loads)
//   nobar     : same loads, weights read from a fixed LDS slot, no ring stores/barriers
//   noload    : MFMAs on register-resident fragments only (no LDS reads)
//   nodma / dma-nowait-nobar / dma-neverwait: convTiles with parts of the weight
//               stream removed (convTiles' DBG ablation flags)
// Build: make -C tools conv_bench ; run: tools/_build/conv_bench
#include "../katacoffee_amd/csrc/nn.hip"

#include <cstdio>
#include <vector>

using namespace kc;
constexpr int REPS = 16;

// convTiles DBG flags per mode (modes 1 and 2 are hand-written loops)
constexpr int kDbg[6] = {0, 0, 0, 1, 10, 256 + 10};

template <class G, int MODE>
__global__ void __launch_bounds__(G::NT, 2) kConv(const h16x8* __restrict__ w, const uint16_t* __restrict__ tabs,
                                                  float* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rg = wave >> 1, cg = wave & 1;
  const int tstart = rg * G::MAXT;
  uint16_t* act = reinterpret_cast<uint16_t*>(smem);
  uint16_t* rowPa = reinterpret_cast<uint16_t*>(smem + G::OFF_TAB);
  h16x8* wl = reinterpret_cast<h16x8*>(smem + G::OFF_W);
  for(int i = tid; i < G::NTAB; i += G::NT)
    rowPa[i] = tabs[i];
  for(int i = tid; i < G::ACT_BYTES / 2; i += G::NT)
    act[i] = (uint16_t)(0x3000 + (i * 7 & 0x3ff));
  for(int i = tid; i < G::RING * G::WBUF; i += G::NT)
    wl[i] = w[i % (9 * G::WBUF)];
  __syncthreads();
  int ab[G::MAXT];
  aBases<G>(ab, rowPa, tstart, lane);
  f32x4 acc[G::MAXT][G::NCT];
  zeroAcc<G>(acc);
  unsigned long long t0 = clock64();
  for(int r = 0; r < REPS; r += 2) {
    if(MODE == 0 || MODE >= 3) {
      // the stream's last taps re-request this conv's first taps for the next rep; two
      // reps per iteration so the small-batch instance's tap pairs alternate as in the
      // network (conv1 starts at an odd stream tap, conv2 at an even one)
      constexpr int DBG = kDbg[MODE];
      convTiles<G, 9, 3, 1, DBG>(act, w, wl, acc, ab, cg, lane, tid, w, 3 * G::NCT_ALL, 9, 9 + 9 * r);
      if(!(DBG & 256))
        __syncthreads();
      convTiles<G, 9, 3, 0, DBG>(act, w, wl, acc, ab, cg, lane, tid, w, 3 * G::NCT_ALL, 9, 18 + 9 * r);
      if(!(DBG & 256))
        __syncthreads();
    } else if(MODE == 1) {
      const char* actB = reinterpret_cast<const char*>(act);
      const h16x8* wlane = wl + (cg * G::NCT) * 64 + lane;
      h16x8 af[2][G::MAXT], bf[2][G::NCT];
      auto loadStep = [&](int st, int buf) {
        const int tap = st / 3, cb = st - tap * 3;
        const int aoff = ((tap / 3) * G::PX + tap % 3) * G::ROWB + cb * 64;
        const h16x8* wb = wlane + (tap % G::RING) * G::WBUF + cb * G::NCT_ALL * 64;
#pragma unroll
        for(int ct = 0; ct < G::NCT; ct++)
          bf[buf][ct] = wb[ct * 64];
#pragma unroll
        for(int t = 0; t < G::MAXT; t++)
          af[buf][t] = *reinterpret_cast<const h16x8*>(actB + ab[t] + aoff);
      };
      loadStep(0, 0);
#pragma unroll
      for(int st = 0; st < 54; st++) {  // two convs per iteration
        if(st + 1 < 54)
          loadStep((st + 1) % 27, (st + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for(int t = 0; t < G::MAXT; t++)
#pragma unroll
          for(int ct = 0; ct < G::NCT; ct++)
            acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[st & 1][ct], af[st & 1][t], acc[t][ct], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      h16x8 af[G::MAXT], bf[G::NCT];
#pragma unroll
      for(int t = 0; t < G::MAXT; t++)
        af[t] = *reinterpret_cast<const h16x8*>(reinterpret_cast<const char*>(act) + ab[t]);
#pragma unroll
      for(int ct = 0; ct < G::NCT; ct++)
        bf[ct] = wl[(cg * G::NCT + ct) * 64 + lane];
#pragma unroll
      for(int st = 0; st < 54; st++) {  // two convs per iteration
#pragma unroll
        for(int t = 0; t < G::MAXT; t++)
#pragma unroll
          for(int ct = 0; ct < G::NCT; ct++)
            acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[ct], af[t], acc[t][ct], 0, 0, 0);
      }
    }
  }
  unsigned long long t1 = clock64();
  float s = 0;
  for(int t = 0; t < G::MAXT; t++)
    for(int ct = 0; ct < G::NCT; ct++)
      s += acc[t][ct][0] + acc[t][ct][3];
  out[blockIdx.x * G::NT + tid] = s;
  if(tid == 0)
    cyc[blockIdx.x] = t1 - t0;
}

template <class G, int MODE>
void run(const char* name, int wgPerCu, const h16x8* w, const uint16_t* tabs, float* out, unsigned long long* cyc) {
  const int grid = 256 * wgPerCu;
  KC_HIP(hipFuncSetAttribute((const void*)kConv<G, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
  for(int it = 0; it < 3; it++)
    hipLaunchKernelGGL((kConv<G, MODE>), dim3(grid), dim3(G::NT), G::LDS, 0, w, tabs, out, cyc);
  KC_HIP(hipDeviceSynchronize());
  std::vector<unsigned long long> c(grid);
  KC_HIP(hipMemcpy(c.data(), cyc, grid * 8, hipMemcpyDeviceToHost));
  double avg = 0;
  for(auto v : c)
    avg += v;
  avg /= grid;
  // MFMA issue floor per SIMD per conv: 27 K-steps x MAXT x NCT MFMAs x 16 cycles x waves per SIMD
  const double floor = 27.0 * G::MAXT * G::NCT * 16.0 * (G::NW * wgPerCu / 4);
  printf("NB%d/NW%d %-17s %8.0f cycles per conv (%.1f per K-step; MFMA floor %.0f)\n", G::NB, G::NW, name,
         avg / REPS, avg / REPS / 27, floor);
}

template <class G>
void runAll(int wgPerCu, const h16x8* w) {
  std::vector<uint16_t> tab = rowTables<G>();
  uint16_t* tabs;
  KC_HIP(hipMalloc(&tabs, tab.size() * 2));
  KC_HIP(hipMemcpy(tabs, tab.data(), tab.size() * 2, hipMemcpyHostToDevice));
  float* out;
  unsigned long long* cyc;
  KC_HIP(hipMalloc(&out, (size_t)512 * G::NT * 4));
  KC_HIP(hipMalloc(&cyc, 512 * 8));
  run<G, 0>("real", wgPerCu, w, tabs, out, cyc);
  run<G, 1>("nobar", wgPerCu, w, tabs, out, cyc);
  run<G, 2>("noload", wgPerCu, w, tabs, out, cyc);
  run<G, 3>("nodma", wgPerCu, w, tabs, out, cyc);
  run<G, 4>("dma-nowait-nobar", wgPerCu, w, tabs, out, cyc);
  run<G, 5>("dma-neverwait", wgPerCu, w, tabs, out, cyc);
}

int main() {
  using G8 = NNGeo<5, 5, 96, 8, 0>;
  std::vector<uint16_t> hw((size_t)9 * G8::WBUF * 8);
  for(size_t i = 0; i < hw.size(); i++)
    hw[i] = (uint16_t)(0x2000 + (i * 13 & 0x7ff));
  h16x8* w;
  KC_HIP(hipMalloc(&w, hw.size() * 2));
  KC_HIP(hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  runAll<G8>(1, w);
  runAll<NNGeo<5, 5, 96, NN_SMALL_NB, 0>>(1, w);

  return 0;
}
