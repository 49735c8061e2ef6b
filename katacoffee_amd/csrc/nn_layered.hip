// Layered residual-network forward: one MFMA implicit-GEMM launch per convolution
// over the whole leaf batch, for every CFNN architecture (b6c96, b10c128,
// b18c384nbt nested bottlenecks, ...) and board geometry (5x5, 7x7, 9x9).
//
// Semantics: eigenbackend.cpp (ConvLayer :270-680, BatchNormLayer :684-734,
// poolRowsGPool :141-166, poolRowsValueHead :168-186, ResidualBlock :888-931,
// GlobalPoolingResidualBlock :935-1015, Trunk :1169-1227, PolicyHead :1229-1299,
// ValueHead :1301-1377); nested bottleneck blocks model_pytorch.py:860-958.
//
// MI355X design (DESIGN.md §3 "kConvL"):
//  * activations live in HBM, NHWC: the residual trunk(s) in f32, activated conv
//    inputs in fp16 where an epilogue can produce them (BN-ReLU of a conv output);
//    BN-ReLU of a trunk is fused into the next conv's prologue (f32 -> fp16 while
//    staging into LDS), the residual add into the conv's epilogue;
//  * a 512-thread workgroup owns BPW whole boards (~250 output rows, 16 row tiles)
//    and 32*TN output channels per wave column; the K loop runs over 32-channel
//    slices: each slice of the boards' activations is staged (with a one-cell zero
//    border, so every 3x3 neighbour is a fixed LDS row offset) into a
//    double-buffered LDS stage while the previous slice's 9 taps run on
//    v_mfma_f32_16x16x32_f16 (computed transposed, weights x activations, so each
//    lane holds 4 consecutive output channels of one row);
//  * weights are pre-swizzled on the host into per-lane 16-byte B fragments in
//    [slice][tap][col tile] order and prefetched two K steps ahead into registers
//    straight from L2 (every workgroup reads the same few hundred KB);
//  * SPLIT ("accurate" precision): every operand is carried as an fp16 pair
//    hi + lo (lo = fp16(x - hi)), each product as hi*hi + lo*hi + hi*lo on three
//    MFMAs -> ~22-bit operands, logits within 1e-3 of the fp32 reference for any
//    net.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <functional>
#include <mutex>
#include <set>
#include <vector>

#include "engine.h"
#include "lds_dma.h"

namespace kc {

typedef _Float16 lh16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 lh16x4 __attribute__((ext_vector_type(4)));
typedef float lf32x4 __attribute__((ext_vector_type(4)));

constexpr int L_WAVES = 8, L_NT = L_WAVES * 64;
// fp16 per staged row: 32 channels + pad.  Fast: 48 (24 dwords: a 16-row tile's
// A-fragment ds_read_b128 lane groups hit distinct banks for contiguous rows, and the
// padded-board rows average 2 LDS cycles per group instead of 2.66 at 40).  Split: 40
// (two planes x two stages must fit the LDS).
constexpr int lStride(bool split) { return split ? 40 : 48; }

enum LPro : int { PRO_BITS = 0, PRO_F16 = 1, PRO_BN = 2, PRO_BN_GB = 3 };
enum LEpi : int { EPI_STORE = 0, EPI_ADD = 1, EPI_BNRELU16 = 2, EPI_STEM = 3 };

template <int X_, int Y_>
struct LGeo {
  static constexpr int X = X_, Y = Y_, A = X_ * Y_;
  static constexpr int BPW = 256 / A < 1 ? 1 : 256 / A;  // boards per workgroup
  static constexpr int ROWS = BPW * A;
  static constexpr int RT = (ROWS + 15) / 16;
  static constexpr int PX = X + 2, PY = Y + 2, PA = PX * PY;
  static constexpr int PROWS = BPW * PA;
  static constexpr int stage(bool split) { return PROWS * lStride(split) * 2; }  // bytes per staged slice
};

struct LConvArgs {
  // prologue: the conv input, channels [0, cinReal) of cin (multiple of 32)
  int pro, cin, cinReal;
  const void* src;
  int srcLd, srcOff;
  const float* ps;  // BN scale / bias (PRO_BN, PRO_BN_GB)
  const float* pb;
  const float* gb;  // per-board bias [board][gbLd] (PRO_BN_GB)
  int gbLd;
  const uint64_t* bits;  // PRO_BITS: packed V1 rows
  int inWords;
  const int* rowIdx;
  // weights: [cin/32][taps][coutPad/16][64] 16-byte fragments (hi, lo)
  const lh16x8* w;
  const lh16x8* wlo;
  int coutTiles;
  // epilogue: channels [0, cout)
  int epi, cout;
  void* dst;
  int dstLd, dstOff;
  const float* es;
  const float* eb;
  const float* glob;  // EPI_STEM: globInit [C] (gin == 1), times winLen
  float winLen;
  // batch
  int n;
  const int* countDev;
};

KC_D uint32_t packHalf2(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) |
         ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
}

// One 32-channel slice of the workgroup's boards into an LDS stage (hi and, for
// SPLIT, lo planes).  Rows are padded cells; borders stay zero (set once).  Split in
// two so the next slice's global loads are in flight while the current slice's
// MFMAs run: stageLoad issues a thread's (row, 8-channel) tasks into registers,
// stageStore applies the prologue (BN-ReLU, gpool bias) and writes fp16 to LDS.
template <class G>
struct StageRegs {
  static constexpr int TPT = (G::ROWS * 4 + L_NT - 1) / L_NT;  // tasks per thread
  float4 x0[TPT], x1[TPT];  // f32 source (PRO_BN*), or raw fp16 bits in x0 (PRO_F16)
};

template <class G>
KC_D void stageLoad(const LConvArgs& a, StageRegs<G>& R, int cb, int base, int nb, int tid) {
#pragma unroll
  for(int k = 0; k < StageRegs<G>::TPT; k++) {
    const int t = tid + k * L_NT;
    R.x0[k] = R.x1[k] = float4{0.0f, 0.0f, 0.0f, 0.0f};
    if(t >= G::ROWS * 4 || a.pro == PRO_BITS)
      continue;
    const int r = t >> 2, q = t & 3;
    const int brd = r / G::A;
    if(brd >= nb)
      continue;
    const size_t g = (size_t)base * G::A + r;
    const int c0 = cb * 32 + q * 8;
    if(a.pro == PRO_F16) {
      R.x0[k] = *reinterpret_cast<const float4*>(reinterpret_cast<const uint16_t*>(a.src) + g * a.srcLd + c0);
    } else {
      const float* sp = reinterpret_cast<const float*>(a.src) + g * a.srcLd + a.srcOff + c0;
      R.x0[k] = *reinterpret_cast<const float4*>(sp);
      R.x1[k] = *reinterpret_cast<const float4*>(sp + 4);
    }
  }
}

template <class G, bool SPLIT>
KC_D void stageStore(const LConvArgs& a, const StageRegs<G>& R, char* stHi, char* stLo, int cb, int base, int nb,
                     const float* sS, const float* sB, const float* sG, int tid) {
#pragma unroll
  for(int k = 0; k < StageRegs<G>::TPT; k++) {
    const int t = tid + k * L_NT;
    if(t >= G::ROWS * 4)
      continue;
    const int r = t >> 2, q = t & 3;
    const int brd = r / G::A, p = r - brd * G::A;
    const int pr = brd * G::PA + (p / G::X + 1) * G::PX + p % G::X + 1;
    const int c0 = cb * 32 + q * 8;
    char* dHi = stHi + (pr * lStride(SPLIT) + q * 8) * 2;
    if(a.pro == PRO_F16) {
      *reinterpret_cast<float4*>(dHi) = R.x0[k];  // already fp16 (zeros past the batch)
      continue;
    }
    float v[8];
    if(brd >= nb) {
#pragma unroll
      for(int j = 0; j < 8; j++)
        v[j] = 0.0f;
    } else if(a.pro == PRO_BITS) {
      const int src = a.rowIdx ? a.rowIdx[base + brd] : base + brd;
      const uint64_t* w = a.bits + (size_t)src * a.inWords;
#pragma unroll
      for(int j = 0; j < 8; j++) {
        const int c = c0 + j;
        float bit = 0.0f;
        if(c < a.cinReal) {
          const int i = c * G::A + p;
          bit = (float)((w[i >> 6] >> (i & 63)) & 1ULL);
        }
        v[j] = bit;
      }
    } else {
      const float xs[8] = {R.x0[k].x, R.x0[k].y, R.x0[k].z, R.x0[k].w, R.x1[k].x, R.x1[k].y, R.x1[k].z, R.x1[k].w};
#pragma unroll
      for(int j = 0; j < 8; j++) {
        const int c = c0 + j;
        float x = xs[j];
        if(a.pro == PRO_BN_GB && c < a.cinReal)
          x += sG[brd * a.gbLd + c];
        const float y = fmaxf(x * sS[c] + sB[c], 0.0f);
        v[j] = c < a.cinReal ? y : 0.0f;
      }
    }
    uint4 hi;
    hi.x = packHalf2(v[0], v[1]);
    hi.y = packHalf2(v[2], v[3]);
    hi.z = packHalf2(v[4], v[5]);
    hi.w = packHalf2(v[6], v[7]);
    *reinterpret_cast<uint4*>(dHi) = hi;
    if constexpr(SPLIT) {
      float lo[8];
#pragma unroll
      for(int j = 0; j < 8; j++)
        lo[j] = v[j] - (float)(_Float16)v[j];
      uint4 l4;
      l4.x = packHalf2(lo[0], lo[1]);
      l4.y = packHalf2(lo[2], lo[3]);
      l4.z = packHalf2(lo[4], lo[5]);
      l4.w = packHalf2(lo[6], lo[7]);
      *reinterpret_cast<uint4*>(stLo + (pr * lStride(SPLIT) + q * 8) * 2) = l4;
    }
  }
}

// Epilogue shared by the conv kernels: lane holds channels ch..ch+3 of row
// (lane & 15) of each of its tiles.
template <class G, int TM, int TN>
KC_D void convEpilogue(const LConvArgs& a, const lf32x4 (&acc)[TM][TN], int base, int nb, int wm, int ctBase,
                       int lane) {
  const int rowsValid = nb * G::A;
#pragma unroll
  for(int t = 0; t < TM; t++) {
    const int r = (wm * TM + t) * 16 + (lane & 15);
    if(r >= rowsValid)
      continue;
    const size_t g = (size_t)base * G::A + r;
#pragma unroll
    for(int c = 0; c < TN; c++) {
      const int ch = (ctBase + c) * 16 + 4 * (lane >> 4);
      if(ch >= a.cout)
        continue;
      const lf32x4 v = acc[t][c];
      if(a.epi == EPI_BNRELU16) {
        const float4 s4 = *reinterpret_cast<const float4*>(a.es + ch);
        const float4 b4 = *reinterpret_cast<const float4*>(a.eb + ch);
        uint2 h;
        h.x = packHalf2(fmaxf(v[0] * s4.x + b4.x, 0.0f), fmaxf(v[1] * s4.y + b4.y, 0.0f));
        h.y = packHalf2(fmaxf(v[2] * s4.z + b4.z, 0.0f), fmaxf(v[3] * s4.w + b4.w, 0.0f));
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(a.dst) + g * a.dstLd + a.dstOff + ch) = h;
      } else {
        float* d = reinterpret_cast<float*>(a.dst) + g * a.dstLd + a.dstOff + ch;
        float4 o = float4{v[0], v[1], v[2], v[3]};
        if(a.epi == EPI_ADD) {
          const float4 old = *reinterpret_cast<const float4*>(d);
          o = float4{old.x + o.x, old.y + o.y, old.z + o.z, old.w + o.w};
        } else if(a.epi == EPI_STEM) {
          const float4 g4 = *reinterpret_cast<const float4*>(a.glob + ch);
          o = float4{o.x + g4.x * a.winLen, o.y + g4.y * a.winLen, o.z + g4.z * a.winLen, o.w + g4.w * a.winLen};
        }
        *reinterpret_cast<float4*>(d) = o;
      }
    }
  }
}

// Cycle accounting of kConvLB and kConvL (profiling build, `make prof`; tools/convl_phase.py): wave 0
// of every workgroup adds its cycles per phase into g_convlProf (one atomic per slot and
// workgroup): 0 workgroups, 1 total, 2 prologue (entry to the first K-step), 3 weight
// waits (vmcnt + barrier per tap group; kConvL: the barrier per slice), 4 stage stores (incl. the wait for the slice's
// loads), 5 epilogue.
#ifdef KC_SEARCH_PROFILE
__device__ unsigned long long g_convlProf[8];
#define CLP_NOW() clock64()
#define CLP_ADD(i, v)                                                  \
  do {                                                                 \
    if(tid == 0)                                                       \
      atomicAdd(&g_convlProf[(i)], (unsigned long long)(v));           \
  } while(0)
#else
#define CLP_NOW() 0ll
#define CLP_ADD(i, v) \
  do {                \
  } while(0)
#endif

// Same-box A/B switches (tools/build_variant.sh): KC_CONVL_LATE_PRO 1 requests the first
// slice and weights after the prologue's barrier, KC_CONVL_LATE_STORE 1 runs the next
// slice's prologue after the last tap (both: the round-5 kernel); KC_CONVL_STORE_TAP the
// tap before which it runs otherwise
#ifndef KC_CONVL_LATE_PRO
#define KC_CONVL_LATE_PRO 0
#endif
#ifndef KC_CONVL_LATE_STORE
#define KC_CONVL_LATE_STORE 0
#endif
#ifndef KC_CONVL_STORE_TAP
#define KC_CONVL_STORE_TAP 5
#endif
template <int X, int Y, int KT, int TN, bool SPLIT, int WN>
__global__ void __launch_bounds__(L_NT, 2) kConvL(LConvArgs a) {
  using G = LGeo<X, Y>;
  constexpr int T = KT * KT;
  constexpr int WM = L_WAVES / WN, TM = (G::RT + WM - 1) / WM;  // wave grid WM x WN, row tiles per wave
  constexpr int NCT = TN * WN;                                   // column tiles per workgroup
  constexpr int PLANES = SPLIT ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int count = a.countDev ? min(*a.countDev, a.n) : a.n;
  const int base = blockIdx.x * G::BPW;
  if(base >= count)
    return;
  const int nb = min(G::BPW, count - base);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long tEntry = CLP_NOW();
  long long tWait = 0, tStore = 0;
  const int wm = wave / WN, wn = wave % WN;
  const int ctBase = blockIdx.y * NCT + wn * TN;  // this wave's first global column tile
  char* stage = smem;                                        // [2][PLANES][STAGE]
  float* sS = reinterpret_cast<float*>(smem + 2 * PLANES * G::stage(SPLIT));  // [cin]
  float* sB = sS + a.cin;
  float* sG = sB + a.cin;  // [BPW][gbLd]
  const int NCB = a.cin / 32;
  // B fragments: step s = cb*T + tap; a ring of R register slots loaded R-1 steps
  // ahead (3x3: R = 3, slot = tap % 3 since 9 % 3 == 0; 1x1: R = 2, slot = cb & 1)
  constexpr int R = T % 3 == 0 ? 3 : 2;
  const lh16x8* wl = a.w + (size_t)ctBase * 64 + lane;
  const lh16x8* wlo = SPLIT ? a.wlo + (size_t)ctBase * 64 + lane : nullptr;
  const size_t stepStride = (size_t)a.coutTiles * 64;
  lh16x8 bh[R][TN], bl[R][SPLIT ? TN : 1];
  auto loadB = [&](int s, int slot) {
#pragma unroll
    for(int c = 0; c < TN; c++) {
      bh[slot][c] = wl[(size_t)s * stepStride + c * 64];
      if constexpr(SPLIT)
        bl[slot][c] = wlo[(size_t)s * stepStride + c * 64];
    }
  };
  const int S = NCB * T;
  StageRegs<G> sr;
#if !KC_CONVL_LATE_PRO
  // the first slice's activations and the first K steps' weights are requested before the
  // LDS clear and the parameter copy, so their latency overlaps them (round 5 issued them
  // after that barrier: 10.2 k of the split conv's 100.9 k cycles per workgroup were its
  // prologue, tools/convl_phase.py)
  stageLoad<G>(a, sr, 0, base, nb, tid);
#pragma unroll
  for(int i = 0; i < R - 1; i++)
    if(i < S)
      loadB(i, i);
#endif
  // zero both stages (borders and boards past the batch stay zero), parameters to LDS
  for(int i = tid; i < 2 * PLANES * G::stage(SPLIT) / 16; i += L_NT)
    reinterpret_cast<uint4*>(smem)[i] = uint4{0u, 0u, 0u, 0u};
  if(a.pro == PRO_BN || a.pro == PRO_BN_GB)
    for(int i = tid; i < a.cin; i += L_NT) {
      sS[i] = i < a.cinReal ? a.ps[i] : 0.0f;
      sB[i] = i < a.cinReal ? a.pb[i] : 0.0f;
    }
  if(a.pro == PRO_BN_GB)
    for(int i = tid; i < nb * a.gbLd; i += L_NT)
      sG[i] = a.gb[(size_t)base * a.gbLd + i];
  __syncthreads();
#if KC_CONVL_LATE_PRO
  stageLoad<G>(a, sr, 0, base, nb, tid);
#endif
  stageStore<G, SPLIT>(a, sr, stage, stage + G::stage(SPLIT), 0, base, nb, sS, sB, sG, tid);

  // per-lane A row bases (bytes, shifted to the (-r,-r) neighbour), padding rows -> row 0
  int ab[TM];
#pragma unroll
  for(int t = 0; t < TM; t++) {
    int r = (wm * TM + t) * 16 + (lane & 15);
    if(r >= G::ROWS)
      r = 0;
    const int brd = r / G::A, p = r - brd * G::A;
    const int pr = brd * G::PA + (p / G::X + 1) * G::PX + p % G::X + 1;
    const int shift = KT == 3 ? G::PX + 1 : 0;
    ab[t] = ((pr - shift) * lStride(SPLIT)) * 2 + 16 * (lane >> 4);
  }
  lf32x4 acc[TM][TN];
#pragma unroll
  for(int t = 0; t < TM; t++)
#pragma unroll
    for(int c = 0; c < TN; c++)
      acc[t][c] = lf32x4{0.0f, 0.0f, 0.0f, 0.0f};

#if KC_CONVL_LATE_PRO
#pragma unroll
  for(int i = 0; i < R - 1; i++)
    if(i < S)
      loadB(i, i);
#endif
  __syncthreads();

  // one K step: tap of slice cb from the stage at stHi/stLo, B slot `slot`
  auto step = [&](int cb, int tap, int slot, const char* stHi, const char* stLo) {
    const int s = cb * T + tap;
    if(s + R - 1 < S)
      loadB(s + R - 1, (slot + R - 1) % R);
    const int dy = KT == 3 ? tap / 3 : 0, dx = KT == 3 ? tap % 3 : 0;
    const int aoff = (dy * G::PX + dx) * lStride(SPLIT) * 2;
    lh16x8 ah[TM], al[SPLIT ? TM : 1];
#pragma unroll
    for(int t = 0; t < TM; t++) {
      ah[t] = *reinterpret_cast<const lh16x8*>(stHi + ab[t] + aoff);
      if constexpr(SPLIT)
        al[t] = *reinterpret_cast<const lh16x8*>(stLo + ab[t] + aoff);
    }
#pragma unroll
    for(int t = 0; t < TM; t++)
#pragma unroll
      for(int c = 0; c < TN; c++) {
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[slot][c], ah[t], acc[t][c], 0, 0, 0);
        if constexpr(SPLIT) {
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[slot][c], ah[t], acc[t][c], 0, 0, 0);
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[slot][c], al[t], acc[t][c], 0, 0, 0);
        }
      }
  };
  // one slice: the next slice's global loads, its taps, then the next slice's
  // prologue into the other stage buffer
  auto slice = [&](int cb, int parity) {
    const char* stHi = stage + (cb & 1) * PLANES * G::stage(SPLIT);
    const char* stLo = stHi + G::stage(SPLIT);
    if(cb + 1 < NCB)
      stageLoad<G>(a, sr, cb + 1, base, nb, tid);
    // the next slice's prologue (BN-ReLU, hi/lo split, LDS stores into the other stage,
    // which no wave reads during this slice) runs between this slice's taps STORE_TAP - 1
    // and STORE_TAP, so its VALU work and LDS writes overlap the MFMAs in flight instead
    // of running after them (round 5: after the last tap, 9.1 k cycles per workgroup)
    constexpr int STORE_TAP = KC_CONVL_LATE_STORE ? T : (T % 3 == 0 ? KC_CONVL_STORE_TAP : T);
    auto storeNext = [&]() {
      if(cb + 1 < NCB) {
        char* nHi = stage + ((cb + 1) & 1) * PLANES * G::stage(SPLIT);
        const long long t0 = CLP_NOW();
        stageStore<G, SPLIT>(a, sr, nHi, nHi + G::stage(SPLIT), cb + 1, base, nb, sS, sB, sG, tid);
        tStore += CLP_NOW() - t0;
      }
    };
    if constexpr(T % 3 == 0) {
#pragma unroll
      for(int tap = 0; tap < T; tap++) {
        if(tap == STORE_TAP)
          storeNext();
        step(cb, tap, tap % 3, stHi, stLo);
      }
    } else {
      step(cb, 0, parity, stHi, stLo);
    }
    if(STORE_TAP == T)
      storeNext();
    const long long t1 = CLP_NOW();
    __syncthreads();
    tWait += CLP_NOW() - t1;
  };
  const long long tLoop = CLP_NOW();
  int cb = 0;
  for(; cb + 1 < NCB; cb += 2) {
    slice(cb, 0);
    slice(cb + 1, 1);
  }
  if(cb < NCB)
    slice(cb, 0);

  const long long tEpi = CLP_NOW();
  convEpilogue<G, TM, TN>(a, acc, base, nb, wm, ctBase, lane);
  CLP_ADD(0, 1);
  CLP_ADD(1, CLP_NOW() - tEntry);
  CLP_ADD(2, tLoop - tEntry);
  CLP_ADD(3, tWait);
  CLP_ADD(4, tStore);
  CLP_ADD(5, CLP_NOW() - tEpi);
  (void)tEntry;
  (void)tLoop;
  (void)tEpi;
  (void)tWait;
  (void)tStore;
}


// 3x3 fast convolutions with the weights in LDS: the workgroup's B fragments of three
// taps (3 x NCT pieces of 1 KiB) stream by LDS-DMA into one of two ring slots, so
// each fragment crosses the L1 once per workgroup instead of once per wave that uses
// it (kConvL's register ring: 4 or 2 waves per fragment).  Group q (slice cb, taps
// 3g..3g+2, q = 3cb + g) lives in slot q & 1; group q+1 is requested at the start of
// group q and published by the barrier before group q's last K-step, which also
// frees slot q & 1's previous group and, at a slice's end, publishes the next
// slice's stage.  Fragments of the next K-step (A from the stage, B from the ring)
// are read before the current step's MFMAs.  Same staging, tiles and epilogues as
// kConvL.
template <int X, int Y, int TN, int WN>
__global__ void __launch_bounds__(L_NT, 2) kConvLB(LConvArgs a) {
  using G = LGeo<X, Y>;
  constexpr int WM = L_WAVES / WN, TM = (G::RT + WM - 1) / WM;
  constexpr int NCT = TN * WN;
  constexpr int GPIECES = 3 * NCT;            // 1-KiB pieces per tap group
  constexpr int GBYTES = GPIECES * 1024;      // one ring slot
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int count = a.countDev ? min(*a.countDev, a.n) : a.n;
  const int base = blockIdx.x * G::BPW;
  if(base >= count)
    return;
  const int nb = min(G::BPW, count - base);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long tEntry = CLP_NOW();
  long long tWait = 0, tStore = 0;
  const int wm = wave / WN, wn = wave % WN;
  const int ctBase = blockIdx.y * NCT + wn * TN;
  char* stage = smem;                          // [2][STAGE]
  char* ring = smem + 2 * G::stage(false);            // [2][GBYTES]
  float* sS = reinterpret_cast<float*>(ring + 2 * GBYTES);
  float* sB = sS + a.cin;
  float* sG = sB + a.cin;
  const int NCB = a.cin / 32;
  // group q's pieces: tap 3g + j, column tile blockIdx.y * NCT + ct -> slot offset (j * NCT + ct) KiB
  const lh16x8* wg = a.w + (size_t)blockIdx.y * NCT * 64 + lane;
  const uint32_t ringAddr = ldsAddr(ring);
  auto request = [&](int q) {
    const int cb = q / 3, g = q - 3 * cb;
    for(int pc = wave; pc < GPIECES; pc += L_WAVES) {
      const int j = pc / NCT, ct = pc - j * NCT;
      glds16(wg + ((size_t)(cb * 9 + 3 * g + j) * a.coutTiles + ct) * 64, ringAddr + (q & 1) * GBYTES + pc * 1024);
    }
  };
  request(0);
  for(int i = tid; i < 2 * G::stage(false) / 16; i += L_NT)
    reinterpret_cast<uint4*>(smem)[i] = uint4{0u, 0u, 0u, 0u};
  if(a.pro == PRO_BN || a.pro == PRO_BN_GB)
    for(int i = tid; i < a.cin; i += L_NT) {
      sS[i] = i < a.cinReal ? a.ps[i] : 0.0f;
      sB[i] = i < a.cinReal ? a.pb[i] : 0.0f;
    }
  if(a.pro == PRO_BN_GB)
    for(int i = tid; i < nb * a.gbLd; i += L_NT)
      sG[i] = a.gb[(size_t)base * a.gbLd + i];
  __syncthreads();  // (drains group 0's DMA too)
  StageRegs<G> sr;
  stageLoad<G>(a, sr, 0, base, nb, tid);
  stageStore<G, false>(a, sr, stage, nullptr, 0, base, nb, sS, sB, sG, tid);
  int ab[TM];
#pragma unroll
  for(int t = 0; t < TM; t++) {
    int r = (wm * TM + t) * 16 + (lane & 15);
    if(r >= G::ROWS)
      r = 0;
    const int brd = r / G::A, p = r - brd * G::A;
    const int pr = brd * G::PA + (p / G::X + 1) * G::PX + p % G::X + 1;
    ab[t] = ((pr - G::PX - 1) * lStride(false)) * 2 + 16 * (lane >> 4);
  }
  lf32x4 acc[TM][TN];
#pragma unroll
  for(int t = 0; t < TM; t++)
#pragma unroll
    for(int c = 0; c < TN; c++)
      acc[t][c] = lf32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int Q = NCB * 3;  // tap groups
  __syncthreads();        // stage 0 published
  lh16x8 af[2][TM], bf[2][TN];
  // fragments of K-step (slice parity par, tap) into buffer buf
  auto loadFr = [&](int par, int tap, int buf) {
    const char* st = stage + par * G::stage(false);
    const int aoff = ((tap / 3) * G::PX + tap % 3) * lStride(false) * 2;
    const char* rb = ring + ((par + tap / 3) & 1) * GBYTES + ((tap % 3) * NCT + wn * TN) * 1024 + lane * 16;
#pragma unroll
    for(int c = 0; c < TN; c++)
      bf[buf][c] = *reinterpret_cast<const lh16x8*>(rb + c * 1024);
#pragma unroll
    for(int t = 0; t < TM; t++)
      af[buf][t] = *reinterpret_cast<const lh16x8*>(st + ab[t] + aoff);
  };
  loadFr(0, 0, 0);
  const long long tLoop = CLP_NOW();
  // one slice; par = cb & 1 (compile-time: slices run in pairs)
  auto slice = [&](int cb, int par) {
    const bool more = cb + 1 < NCB;
    if(more)
      stageLoad<G>(a, sr, cb + 1, base, nb, tid);
#pragma unroll
    for(int tap = 0; tap < 9; tap++) {
      const int q = 3 * cb + tap / 3;
      if(tap % 3 == 0 && q + 1 < Q)
        request(q + 1);
      const int buf = (par + tap) & 1;  // K-step s = 9 cb + tap alternates buffers
      if(tap == 8 && more) {
        const long long t0 = CLP_NOW();
        stageStore<G, false>(a, sr, stage + (par ^ 1) * G::stage(false), nullptr, cb + 1, base, nb, sS, sB, sG, tid);
        tStore += CLP_NOW() - t0;
      }
      if(tap % 3 == 2 && q + 1 < Q) {
        const long long t0 = CLP_NOW();
        waitVm<0>();
        barrierKeepDma();
        tWait += CLP_NOW() - t0;
      }
      if(tap < 8)
        loadFr(par, tap + 1, buf ^ 1);
      else if(more)
        loadFr(par ^ 1, 0, buf ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for(int t = 0; t < TM; t++)
#pragma unroll
        for(int c = 0; c < TN; c++)
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[buf][c], af[buf][t], acc[t][c], 0, 0, 0);
    }
  };
  int cb = 0;
  for(; cb + 1 < NCB; cb += 2) {
    slice(cb, 0);
    slice(cb + 1, 1);
  }
  if(cb < NCB)
    slice(cb, 0);
  const long long tEpi = CLP_NOW();
  convEpilogue<G, TM, TN>(a, acc, base, nb, wm, ctBase, lane);
  CLP_ADD(0, 1);
  CLP_ADD(1, CLP_NOW() - tEntry);
  CLP_ADD(2, tLoop - tEntry);
  CLP_ADD(3, tWait);
  CLP_ADD(4, tStore);
  CLP_ADD(5, CLP_NOW() - tEpi);
  (void)tEntry;
  (void)tLoop;
  (void)tEpi;
  (void)tWait;
  (void)tStore;
}

// 1x1 convolutions, split precision (fast: kConv1LP below): no halo, so a stage holds 128
// channels of the workgroup's rows unpadded (four 32-channel K steps per stage,
// staged synchronously with all of a thread's loads in flight), the stage count is
// a quarter of the 32-channel slices and a stage's load latency is paid once per
// four K steps.  Same wave grid, fragments, prologues and epilogues as kConvL.
constexpr int L1_SW = 4;                  // 32-channel slices per stage
constexpr int l1Stride(bool) { return 32 * L1_SW + 8; }  // fp16 per staged row (272 B)

template <class G, bool SPLIT>
constexpr int l1StageBytes() {
  return G::ROWS * l1Stride(SPLIT) * 2;
}

template <int X, int Y, int TN, bool SPLIT, int WN>
__global__ void __launch_bounds__(L_NT, 2) kConv1L(LConvArgs a) {
  using G = LGeo<X, Y>;
  constexpr int WM = L_WAVES / WN, TM = (G::RT + WM - 1) / WM;
  constexpr int NCT = TN * WN;
  constexpr int SB = l1StageBytes<G, SPLIT>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int count = a.countDev ? min(*a.countDev, a.n) : a.n;
  const int base = blockIdx.x * G::BPW;
  if(base >= count)
    return;
  const int nb = min(G::BPW, count - base);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int ctBase = blockIdx.y * NCT + wn * TN;
  char* stHi = smem;
  char* stLo = smem + SB;
  float* sS = reinterpret_cast<float*>(smem + (SPLIT ? 2 : 1) * SB);
  float* sB = sS + a.cin;
  for(int i = tid; i < a.cin; i += L_NT) {
    sS[i] = i < a.cinReal ? a.ps[i] : 0.0f;
    sB[i] = i < a.cinReal ? a.pb[i] : 0.0f;
  }
  int ab[TM];
#pragma unroll
  for(int t = 0; t < TM; t++) {
    int r = (wm * TM + t) * 16 + (lane & 15);
    if(r >= G::ROWS)
      r = 0;
    ab[t] = r * l1Stride(SPLIT) * 2 + 16 * (lane >> 4);
  }
  lf32x4 acc[TM][TN];
#pragma unroll
  for(int t = 0; t < TM; t++)
#pragma unroll
    for(int c = 0; c < TN; c++)
      acc[t][c] = lf32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const lh16x8* wl = a.w + (size_t)ctBase * 64 + lane;
  const lh16x8* wlo = SPLIT ? a.wlo + (size_t)ctBase * 64 + lane : nullptr;
  const size_t stepStride = (size_t)a.coutTiles * 64;
  const int NCB = a.cin / 32;
  lh16x8 bh[2][TN], bl[2][SPLIT ? TN : 1];
  auto loadB = [&](int s, int slot) {
#pragma unroll
    for(int c = 0; c < TN; c++) {
      bh[slot][c] = wl[(size_t)s * stepStride + c * 64];
      if constexpr(SPLIT)
        bl[slot][c] = wlo[(size_t)s * stepStride + c * 64];
    }
  };
  loadB(0, 0);
  constexpr int TASKS = G::ROWS * 4 * L1_SW;  // (row, 8-channel chunk) of a stage
  for(int st = 0; st * L1_SW < NCB; st++) {
    __syncthreads();  // previous stage consumed
    // stage: channels [128 st, 128 st + 128) of every row, prologue BN-ReLU -> fp16;
    // every load of the stage is issued before the first conversion
    constexpr int TPT = (TASKS + L_NT - 1) / L_NT;
    float4 x0[TPT], x1[TPT];
#pragma unroll
    for(int k = 0; k < TPT; k++) {
      const int t = tid + k * L_NT;
      const int r = t / (4 * L1_SW), q = t - r * (4 * L1_SW);
      const int c0 = st * 32 * L1_SW + q * 8;
      x0[k] = x1[k] = float4{0.0f, 0.0f, 0.0f, 0.0f};
      if(t < TASKS && r / G::A < nb && c0 < a.cin) {
        const float* sp = reinterpret_cast<const float*>(a.src) + ((size_t)base * G::A + r) * a.srcLd + a.srcOff + c0;
        x0[k] = *reinterpret_cast<const float4*>(sp);
        x1[k] = *reinterpret_cast<const float4*>(sp + 4);
      }
    }
#pragma unroll
    for(int k = 0; k < TPT; k++) {
      const int t = tid + k * L_NT;
      if(t >= TASKS)
        continue;
      const int r = t / (4 * L1_SW), q = t - r * (4 * L1_SW);
      const int brd = r / G::A;
      const int c0 = st * 32 * L1_SW + q * 8;
      float v[8];
      const float xs[8] = {x0[k].x, x0[k].y, x0[k].z, x0[k].w, x1[k].x, x1[k].y, x1[k].z, x1[k].w};
#pragma unroll
      for(int j = 0; j < 8; j++)
        v[j] = (brd < nb && c0 + j < a.cinReal) ? fmaxf(xs[j] * sS[c0 + j] + sB[c0 + j], 0.0f) : 0.0f;
      uint4 hi;
      hi.x = packHalf2(v[0], v[1]);
      hi.y = packHalf2(v[2], v[3]);
      hi.z = packHalf2(v[4], v[5]);
      hi.w = packHalf2(v[6], v[7]);
      *reinterpret_cast<uint4*>(stHi + (r * l1Stride(SPLIT) + q * 8) * 2) = hi;
      if constexpr(SPLIT) {
        float lo[8];
#pragma unroll
        for(int j = 0; j < 8; j++)
          lo[j] = v[j] - (float)(_Float16)v[j];
        uint4 l4;
        l4.x = packHalf2(lo[0], lo[1]);
        l4.y = packHalf2(lo[2], lo[3]);
        l4.z = packHalf2(lo[4], lo[5]);
        l4.w = packHalf2(lo[6], lo[7]);
        *reinterpret_cast<uint4*>(stLo + (r * l1Stride(SPLIT) + q * 8) * 2) = l4;
      }
    }
    __syncthreads();
#pragma unroll
    for(int j = 0; j < L1_SW; j++) {
      const int s = st * L1_SW + j;
      if(s >= NCB)
        break;
      if(s + 1 < NCB)
        loadB(s + 1, (j + 1) & 1);
      lh16x8 ah[TM], al[SPLIT ? TM : 1];
#pragma unroll
      for(int t = 0; t < TM; t++) {
        ah[t] = *reinterpret_cast<const lh16x8*>(stHi + ab[t] + 64 * j);
        if constexpr(SPLIT)
          al[t] = *reinterpret_cast<const lh16x8*>(stLo + ab[t] + 64 * j);
      }
#pragma unroll
      for(int t = 0; t < TM; t++)
#pragma unroll
        for(int c = 0; c < TN; c++) {
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j & 1][c], ah[t], acc[t][c], 0, 0, 0);
          if constexpr(SPLIT) {
            acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[j & 1][c], ah[t], acc[t][c], 0, 0, 0);
            acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j & 1][c], al[t], acc[t][c], 0, 0, 0);
          }
        }
    }
  }
  convEpilogue<G, TM, TN>(a, acc, base, nb, wm, ctBase, lane);
}

// 1x1 convolutions, pipelined: 64-channel stages, double-buffered in LDS; the next stage's
// global loads are issued before the current stage's MFMAs and converted (BN-ReLU -> fp16,
// and for SPLIT the lo = x - fp16(x) plane) into the other buffer after them, so the HBM
// latency of the f32 input overlaps the MFMAs (kConv1L waits for each stage before any
// MFMA: 5 % MFMA busy on b18c384nbt's bottleneck convs).  Rows are 40 dwords (64 channels +
// 16 pad: 10 mod 16 chunks, conflict-free A-fragment reads for contiguous rows).  SPLIT
// (round 6): a stage holds a hi and a lo plane, each K step issues
// hi*hi, lo(w)*hi(x), hi(w)*lo(x) -- kConv1L's products in kConv1L's order (an A/B
// option: see kConv1PipeFor).
constexpr int L1P_SW = 2;                  // 32-channel slices per stage
constexpr int L1P_STRIDE = 32 * L1P_SW + 16;  // fp16 per staged row

template <int X, int Y, bool SPLIT>
constexpr size_t l1pLds(int cin) {
  return 2 * (SPLIT ? 2 : 1) * (size_t)LGeo<X, Y>::ROWS * L1P_STRIDE * 2 + 2 * (size_t)cin * 4;
}

template <int X, int Y, int TN, bool SPLIT, int WN>
__global__ void __launch_bounds__(L_NT, 2) kConv1LP(LConvArgs a) {
  using G = LGeo<X, Y>;
  constexpr int WM = L_WAVES / WN, TM = (G::RT + WM - 1) / WM;
  constexpr int NCT = TN * WN;
  constexpr int SB = G::ROWS * L1P_STRIDE * 2;  // one plane of one stage buffer
  constexpr int PL = SPLIT ? 2 : 1;
  constexpr int CPR = 4 * L1P_SW;           // 8-channel chunks per staged row
  constexpr int TASKS = G::ROWS * CPR;
  constexpr int TPT = (TASKS + L_NT - 1) / L_NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int count = a.countDev ? min(*a.countDev, a.n) : a.n;
  const int base = blockIdx.x * G::BPW;
  if(base >= count)
    return;
  const int nb = min(G::BPW, count - base);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int ctBase = blockIdx.y * NCT + wn * TN;
  float* sS = reinterpret_cast<float*>(smem + 2 * PL * SB);
  float* sB = sS + a.cin;
  for(int i = tid; i < a.cin; i += L_NT) {
    sS[i] = i < a.cinReal ? a.ps[i] : 0.0f;
    sB[i] = i < a.cinReal ? a.pb[i] : 0.0f;
  }
  const int NCB = a.cin / 32, NST = (NCB + L1P_SW - 1) / L1P_SW;
  float4 x0[TPT], x1[TPT];
  auto load = [&](int st) {
#pragma unroll
    for(int k = 0; k < TPT; k++) {
      const int t = tid + k * L_NT;
      const int r = t / CPR, q = t - r * CPR;
      const int c0 = st * 32 * L1P_SW + q * 8;
      x0[k] = x1[k] = float4{0.0f, 0.0f, 0.0f, 0.0f};
      if(t < TASKS && r / G::A < nb && c0 < a.cin) {
        const float* sp = reinterpret_cast<const float*>(a.src) + ((size_t)base * G::A + r) * a.srcLd + a.srcOff + c0;
        x0[k] = *reinterpret_cast<const float4*>(sp);
        x1[k] = *reinterpret_cast<const float4*>(sp + 4);
      }
    }
  };
  auto store = [&](int st, char* buf) {
#pragma unroll
    for(int k = 0; k < TPT; k++) {
      const int t = tid + k * L_NT;
      if(t >= TASKS)
        continue;
      const int r = t / CPR, q = t - r * CPR;
      const int brd = r / G::A;
      const int c0 = st * 32 * L1P_SW + q * 8;
      const float xs[8] = {x0[k].x, x0[k].y, x0[k].z, x0[k].w, x1[k].x, x1[k].y, x1[k].z, x1[k].w};
      float v[8];
#pragma unroll
      for(int j = 0; j < 8; j++)
        v[j] = (brd < nb && c0 + j < a.cinReal) ? fmaxf(xs[j] * sS[c0 + j] + sB[c0 + j], 0.0f) : 0.0f;
      uint4 hi;
      hi.x = packHalf2(v[0], v[1]);
      hi.y = packHalf2(v[2], v[3]);
      hi.z = packHalf2(v[4], v[5]);
      hi.w = packHalf2(v[6], v[7]);
      *reinterpret_cast<uint4*>(buf + (r * L1P_STRIDE + q * 8) * 2) = hi;
      if constexpr(SPLIT) {
        float lo[8];
#pragma unroll
        for(int j = 0; j < 8; j++)
          lo[j] = v[j] - (float)(_Float16)v[j];
        uint4 l4;
        l4.x = packHalf2(lo[0], lo[1]);
        l4.y = packHalf2(lo[2], lo[3]);
        l4.z = packHalf2(lo[4], lo[5]);
        l4.w = packHalf2(lo[6], lo[7]);
        *reinterpret_cast<uint4*>(buf + SB + (r * L1P_STRIDE + q * 8) * 2) = l4;
      }
    }
  };
  int ab[TM];
#pragma unroll
  for(int t = 0; t < TM; t++) {
    int r = (wm * TM + t) * 16 + (lane & 15);
    if(r >= G::ROWS)
      r = 0;
    ab[t] = r * L1P_STRIDE * 2 + 16 * (lane >> 4);
  }
  lf32x4 acc[TM][TN];
#pragma unroll
  for(int t = 0; t < TM; t++)
#pragma unroll
    for(int c = 0; c < TN; c++)
      acc[t][c] = lf32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const lh16x8* wl = a.w + (size_t)ctBase * 64 + lane;
  const lh16x8* wlo = SPLIT ? a.wlo + (size_t)ctBase * 64 + lane : nullptr;
  const size_t stepStride = (size_t)a.coutTiles * 64;
  lh16x8 bh[2][TN], bl[2][SPLIT ? TN : 1];
  auto loadB = [&](int s, int slot) {
#pragma unroll
    for(int c = 0; c < TN; c++) {
      bh[slot][c] = wl[(size_t)s * stepStride + c * 64];
      if constexpr(SPLIT)
        bl[slot][c] = wlo[(size_t)s * stepStride + c * 64];
    }
  };
  load(0);
  loadB(0, 0);
  __syncthreads();  // sS / sB
  store(0, smem);
  __syncthreads();
  for(int st = 0; st < NST; st++) {
    const char* cur = smem + (st & 1) * PL * SB;
    if(st + 1 < NST)
      load(st + 1);
#pragma unroll
    for(int j = 0; j < L1P_SW; j++) {
      const int s = st * L1P_SW + j;
      if(s >= NCB)
        break;
      if(s + 1 < NCB)
        loadB(s + 1, (j + 1) & 1);
      lh16x8 ah[TM], al[SPLIT ? TM : 1];
#pragma unroll
      for(int t = 0; t < TM; t++) {
        ah[t] = *reinterpret_cast<const lh16x8*>(cur + ab[t] + 64 * j);
        if constexpr(SPLIT)
          al[t] = *reinterpret_cast<const lh16x8*>(cur + SB + ab[t] + 64 * j);
      }
#pragma unroll
      for(int t = 0; t < TM; t++)
#pragma unroll
        for(int c = 0; c < TN; c++) {
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j & 1][c], ah[t], acc[t][c], 0, 0, 0);
          if constexpr(SPLIT) {
            acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[j & 1][c], ah[t], acc[t][c], 0, 0, 0);
            acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j & 1][c], al[t], acc[t][c], 0, 0, 0);
          }
        }
    }
    if(st + 1 < NST)
      store(st + 1, smem + ((st + 1) & 1) * PL * SB);
    __syncthreads();
  }
  convEpilogue<G, TM, TN>(a, acc, base, nb, wm, ctBase, lane);
}

// Gpool branch of a gpool block: g = relu(T[:, Cr:Cr+Cg] * s + b), KataGPool
// (mean, mean*(sqrt(A)-14)/10, max), bias[Cr] = linG x pooled.  One workgroup per
// board; the pooling splits the cells over 256/Cg thread groups (consecutive lanes
// read consecutive channels of a row).
__global__ void __launch_bounds__(256) kGpoolBias(const float* __restrict__ T, int ld, int A, int Cr, int Cg,
                                                  const float* __restrict__ gs, const float* __restrict__ gbias,
                                                  const float* __restrict__ linGT /*[3Cg][Cr]*/, float* __restrict__ out,
                                                  int n, const int* __restrict__ countDev) {
  __shared__ float pooled[3 * 128], ps[256], pm[256];
  const int count = countDev ? min(*countDev, n) : n;
  const int b = blockIdx.x;
  if(b >= count)
    return;
  const float sqOff = sqrtf((float)A) - 14.0f;
  const float* Tb = T + (size_t)b * A * ld + Cr;
  const int parts = 256 / Cg, tid = threadIdx.x;
  const int c = tid % Cg, part = tid / Cg;
  float sum = 0.0f, mx = 0.0f;
  if(part < parts) {
    const float sc = gs[c], bi = gbias[c];
    for(int p = part; p < A; p += parts) {
      const float v = fmaxf(Tb[(size_t)p * ld + c] * sc + bi, 0.0f);
      sum += v;
      mx = fmaxf(mx, v);
    }
  }
  ps[tid] = sum;
  pm[tid] = mx;
  __syncthreads();
  if(tid < Cg) {
    float s2 = 0.0f, m2 = 0.0f;
    for(int k = 0; k < parts; k++) {
      s2 += ps[k * Cg + tid];
      m2 = fmaxf(m2, pm[k * Cg + tid]);
    }
    const float mean = s2 / (float)A;
    pooled[tid] = mean;
    pooled[Cg + tid] = mean * (sqOff / 10.0f);
    pooled[2 * Cg + tid] = m2;
  }
  __syncthreads();
  for(int o = tid; o < Cr; o += blockDim.x) {
    float s3 = 0.0f;
    for(int k = 0; k < 3 * Cg; k++)
      s3 += linGT[(size_t)k * Cr + o] * pooled[k];
    out[(size_t)b * Cr + o] = s3;
  }
}

struct LHeadW {
  const float *pBiasG, *pLinGT, *pBias2, *pConv2, *vBias1, *vLin2T, *vB2, *vLin3, *vB3, *vLinM, *vBM;
  int p1, g1, v1, v2;
};

// Policy and value heads from T = [p | g | v] (raw 1x1 conv outputs of the tip),
// PolicyHead::apply :1265-1299 / ValueHead::apply :1341-1377 with Coffee outputs:
// out[dst] = policy [4][A] (direction-major), value (2), misc (2).  One workgroup per board.
__global__ void __launch_bounds__(256) kHeadsL(const float* __restrict__ T, int ld, int A, LHeadW h,
                                               float* __restrict__ out, const int* __restrict__ rowIdx, int n,
                                               const int* __restrict__ countDev) {
  __shared__ float pp[3 * 64], vp[3 * 128], pb[64], vh[256], ps[256], pm[256];
  const int count = countDev ? min(*countDev, n) : n;
  const int b = blockIdx.x;
  if(b >= count)
    return;
  const float sqOff = sqrtf((float)A) - 14.0f;
  const float* Tb = T + (size_t)b * A * ld;
  const int tid = threadIdx.x;
  // pooled g (policy) and v (value) channels: 256 / (g1 + v1) thread groups split the cells
  const int NCH = h.g1 + h.v1, parts = 256 / NCH;
  const int c = tid % NCH, part = tid / NCH;
  const bool isG = c < h.g1;
  const int cc = isG ? c : c - h.g1;
  float sum = 0.0f, mx = 0.0f;
  if(part < parts) {
    const int col = isG ? h.p1 + cc : h.p1 + h.g1 + cc;
    const float bias = isG ? h.pBiasG[cc] : h.vBias1[cc];
    for(int p = part; p < A; p += parts) {
      const float v = fmaxf(Tb[(size_t)p * ld + col] + bias, 0.0f);
      sum += v;
      mx = fmaxf(mx, v);
    }
  }
  ps[tid] = sum;
  pm[tid] = mx;
  __syncthreads();
  if(tid < NCH) {
    float s2 = 0.0f, m2 = 0.0f;
    for(int k = 0; k < parts; k++) {
      s2 += ps[k * NCH + tid];
      m2 = fmaxf(m2, pm[k * NCH + tid]);
    }
    const float mean = s2 / (float)A;
    if(isG) {
      pp[cc] = mean;
      pp[h.g1 + cc] = mean * (sqOff / 10.0f);
      pp[2 * h.g1 + cc] = m2;
    } else {
      vp[cc] = mean;
      vp[h.v1 + cc] = mean * (sqOff / 10.0f);
      vp[2 * h.v1 + cc] = mean * ((sqOff * sqOff) / 100.0f - 0.1f);
    }
  }
  __syncthreads();
  for(int o = tid; o < h.p1 + h.v2; o += blockDim.x) {
    if(o < h.p1) {
      float s = 0.0f;
      for(int k = 0; k < 3 * h.g1; k++)
        s += h.pLinGT[(size_t)k * h.p1 + o] * pp[k];
      pb[o] = s + h.pBias2[o];
    } else {
      const int q = o - h.p1;
      float s = h.vB2[q];
      for(int k = 0; k < 3 * h.v1; k++)
        s += h.vLin2T[(size_t)k * h.v2 + q] * vp[k];
      vh[q] = fmaxf(s, 0.0f);
    }
  }
  __syncthreads();
  float* o = out + (size_t)(rowIdx ? rowIdx[b] : b) * (4 * A + 4);
  for(int i = tid; i < 4 * A; i += blockDim.x) {
    const int d = i / A, p = i - d * A;
    const float* tp = Tb + (size_t)p * ld;
    float s = 0.0f;
    for(int k = 0; k < h.p1; k++)
      s += h.pConv2[d * h.p1 + k] * fmaxf(tp[k] + pb[k], 0.0f);
    o[i] = s;
  }
  if(tid < 4) {
    const float* w = tid < 2 ? h.vLin3 + tid * h.v2 : h.vLinM + (tid - 2) * h.v2;
    float s = tid < 2 ? h.vB3[tid] : h.vBM[tid - 2];
    for(int k = 0; k < h.v2; k++)
      s += w[k] * vh[k];
    o[4 * A + tid] = s;
  }
}

// ---------------------------------------------------------------------------
// Host side

namespace {

uint16_t lf2h(float f) {
  const _Float16 h = (_Float16)f;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

#ifdef KC_NO_LDSB  // (A/B builds)
constexpr bool kConvLdsB = false;
#else
constexpr bool kConvLdsB = true;
#endif
// the fast path's 1x1 convs always run the pipelined kernel; the split path's run kConv1L
// unless built with -DKC_SPLIT_1X1_PIPE (round 6: the pipelined split instance is correct --
// test_gpu_nn / test_gpu_train green -- but measured equal: b18c384nbt accurate 54.95 vs
// 54.99 ms, b10c128 1.99-2.02 ms either way, profiles/r06/split_1x1_pipe_ab.txt)
#ifdef KC_SPLIT_1X1_PIPE
template <bool SPLIT>
constexpr bool kConv1PipeFor = true;
#else
template <bool SPLIT>
constexpr bool kConv1PipeFor = !SPLIT;
#endif

template <int X, int Y, int KT, int TN, bool SPLIT, int WN>
void launchConvT(const LConvArgs& a, int grid, hipStream_t st) {
  using G = LGeo<X, Y>;
  size_t lds;
  const void* fnp;
  if constexpr(KT == 1) {
    if(a.pro != PRO_BN)
      throw std::invalid_argument("1x1 convolutions take a BN-ReLU prologue");
    if(kConv1PipeFor<SPLIT> && l1pLds<X, Y, SPLIT>(a.cin) <= 160 * 1024) {
      lds = l1pLds<X, Y, SPLIT>(a.cin);
      fnp = (const void*)kConv1LP<X, Y, TN, SPLIT, WN>;
    } else {
      lds = (SPLIT ? 2 : 1) * l1StageBytes<G, SPLIT>() + 2 * (size_t)a.cin * 4;
      fnp = (const void*)kConv1L<X, Y, TN, SPLIT, WN>;
    }
  } else if constexpr(kConvLdsB && !SPLIT && WN == 2) {
    lds = 2 * G::stage(SPLIT) + 2 * 3 * TN * WN * 1024 + (2 * a.cin + G::BPW * (a.gbLd > 0 ? a.gbLd : 0)) * 4;
    fnp = (const void*)kConvLB<X, Y, TN, WN>;
  } else {
    lds = 2 * (SPLIT ? 2 : 1) * G::stage(SPLIT) + (2 * a.cin + G::BPW * (a.gbLd > 0 ? a.gbLd : 0)) * 4;
    fnp = (const void*)kConvL<X, Y, KT, TN, SPLIT, WN>;
  }
  if(lds > 160 * 1024)
    throw std::invalid_argument("layered conv: LDS budget exceeded");
  static std::mutex mu;
  // (device, kernel) pairs whose attribute is set (per device; an instance may
  // choose between two 1x1 kernels by its input width)
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  KC_HIP(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> lk(mu);
    if(!done.count({dev, fnp})) {
      KC_HIP(hipFuncSetAttribute(fnp, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      done.insert({dev, fnp});
    }
  }
  const int gy = (a.coutTiles + TN * WN - 1) / (TN * WN);
  if constexpr(KT == 1) {
    if(fnp == (const void*)kConv1LP<X, Y, TN, SPLIT, WN>)
      hipLaunchKernelGGL((kConv1LP<X, Y, TN, SPLIT, WN>), dim3(grid, gy), dim3(L_NT), lds, st, a);
    else
      hipLaunchKernelGGL((kConv1L<X, Y, TN, SPLIT, WN>), dim3(grid, gy), dim3(L_NT), lds, st, a);
  }
  else if constexpr(kConvLdsB && !SPLIT && WN == 2)
    hipLaunchKernelGGL((kConvLB<X, Y, TN, WN>), dim3(grid, gy), dim3(L_NT), lds, st, a);
  else
    hipLaunchKernelGGL((kConvL<X, Y, KT, TN, SPLIT, WN>), dim3(grid, gy), dim3(L_NT), lds, st, a);
  KC_HIP(hipGetLastError());
}

// (kt, tn, wn) of a conv -> its instance (chooseGrid).
template <int X, int Y, bool SPLIT>
void launchConvG(const LConvArgs& a, int kt, int tn, int wn, int grid, hipStream_t st) {
  if constexpr(!SPLIT) {
    if(wn == 4) {
      if(kt == 3)
        tn == 2 ? launchConvT<X, Y, 3, 2, false, 4>(a, grid, st) : launchConvT<X, Y, 3, 3, false, 4>(a, grid, st);
      else
        tn == 2 ? launchConvT<X, Y, 1, 2, false, 4>(a, grid, st) : launchConvT<X, Y, 1, 3, false, 4>(a, grid, st);
      return;
    }
  }
  if(kt == 3) {
    if(tn == 2) launchConvT<X, Y, 3, 2, SPLIT, 2>(a, grid, st);
    else if(tn == 3) launchConvT<X, Y, 3, 3, SPLIT, 2>(a, grid, st);
    else launchConvT<X, Y, 3, 4, SPLIT, 2>(a, grid, st);
  } else {
    if(tn == 2) launchConvT<X, Y, 1, 2, SPLIT, 2>(a, grid, st);
    else if(tn == 3) launchConvT<X, Y, 1, 3, SPLIT, 2>(a, grid, st);
    else launchConvT<X, Y, 1, 4, SPLIT, 2>(a, grid, st);
  }
}

int lBoardsPerWG(int X, int Y) {
  if(X == 5 && Y == 5) return LGeo<5, 5>::BPW;
  if(X == 7 && Y == 7) return LGeo<7, 7>::BPW;
  return LGeo<9, 9>::BPW;
}

}  // namespace

bool NNLayered::supportedGeometry(int X, int Y) { return (X == 5 && Y == 5) || (X == 7 && Y == 7) || (X == 9 && Y == 9); }

// Wave grid and column tiles per wave for a conv with `cout` outputs.  Default: the
// 4 x 2 grid (4 row groups x 2 column groups) with the widest TN of 4/3/2 that tiles
// the (padded) outputs in 32*TN-wide workgroup columns.  A fast conv whose output
// tiles then need more column groups (blockIdx.y, each re-staging the whole input)
// than a 2 x 4 grid with TN 3 or 2 takes that grid instead: 8 row tiles per wave,
// each B fragment shared by 2 waves instead of 4 -- b18c384nbt's 192-wide convs run
// in one column group instead of two and its 384-wide 1x1 in two instead of three
// (9x9 forward 25 % faster); at equal column groups (b10c128) the 4 x 2 grid is faster.
static void chooseGrid(int cout, bool split, int& tn, int& wn) {
  const int tiles = (cout + 15) / 16;
  wn = 2;
  tn = cout % 128 == 0 ? 4 : cout % 96 == 0 ? 3 : 2;
  const int gy2 = (tiles + 2 * tn - 1) / (2 * tn);
#ifndef KC_LAYERED_WN2  // (A/B builds: csrc/Makefile `alt` target, ALT_FLAGS=-DKC_LAYERED_WN2)
  if(split)
    return;
  for(int t : {3, 2})
    if(tiles % (4 * t) == 0 && tiles / (4 * t) < gy2) {
      tn = t;
      wn = 4;
      return;
    }
#else
  (void)split;
  (void)gy2;
#endif
}

NNLayered::NNLayered(const ModelHost& m, int X, int Y, int W, bool split)
    : cfg_(m.cfg), X_(X), Y_(Y), W_(W), split_(split) {
  if(!supportedGeometry(X, Y))
    throw std::invalid_argument("NNLayered: board geometry must be 5x5, 7x7 or 9x9");
  if(cfg_.gin != 1 || cfg_.cin > 32 || cfg_.p1 > 64 || cfg_.g1 > 64 || cfg_.v1 > 128 || cfg_.v2 > 256 ||
     cfg_.Cg > 128)
    throw std::invalid_argument("NNLayered: head/gpool widths out of range");
  const int A = X * Y;
  std::vector<uint16_t> wh, wl;  // fragments (8 fp16 each), hi / lo
  std::vector<float> wf;
  auto f32 = [&](const std::vector<float>& v) {
    const int off = (int)wf.size();
    wf.insert(wf.end(), v.begin(), v.end());
    while(wf.size() % 4)
      wf.push_back(0.0f);
    return off;
  };
  auto transpose = [](const std::vector<float>& w, int O, int I) {  // [O][I] -> [I][O]
    std::vector<float> t((size_t)O * I);
    for(int o = 0; o < O; o++)
      for(int i = 0; i < I; i++)
        t[(size_t)i * O + o] = w[(size_t)o * I + i];
    return t;
  };
  // Conv weights W(co, ci, tap) -> fragments [cb][tap][ct][lane][8]
  auto packConvL = [&](int kt, int cin, int cout, const std::function<float(int, int, int)>& Wf) {
    Conv c;
    c.kt = kt;
    c.cinReal = cin;
    c.cin = (cin + 31) / 32 * 32;
    c.cout = cout;
    chooseGrid(cout, split_, c.tn, c.wn);
    const int ncw = 16 * c.tn * c.wn;
    c.coutTiles = (cout + ncw - 1) / ncw * ncw / 16;
    c.wOff = (long)(wh.size() / 8);
    const int taps = kt * kt;
    for(int cb = 0; cb < c.cin / 32; cb++)
      for(int tap = 0; tap < taps; tap++)
        for(int ct = 0; ct < c.coutTiles; ct++)
          for(int l = 0; l < 64; l++)
            for(int j = 0; j < 8; j++) {
              const int co = ct * 16 + (l & 15), ci = cb * 32 + 8 * (l >> 4) + j;
              const float v = (co < cout && ci < cin) ? Wf(co, ci, tap) : 0.0f;
              const uint16_t h = lf2h(v);
              _Float16 hf;
              memcpy(&hf, &h, 2);
              wh.push_back(h);
              wl.push_back(lf2h(v - (float)hf));
            }
    return c;
  };
  auto conv3 = [&](const std::vector<float>& w, int cin, int cout) {
    return packConvL(3, cin, cout, [&](int co, int ci, int tap) { return w[((size_t)co * cin + ci) * 9 + tap]; });
  };
  auto conv1 = [&](const std::vector<float>& w, int cin, int cout) {
    return packConvL(1, cin, cout, [&](int co, int ci, int) { return w[(size_t)co * cin + ci]; });
  };
  // regular / gpool block at trunk width Wd
  std::function<void(const ModelBlock&, int, Block&)> buildBlock = [&](const ModelBlock& b, int Wd, Block& o) {
    o.kind = b.kind;
    o.width = Wd;
    if(b.kind >= 2) {
      const int mid = cfg_.mid;
      o.bnPs = f32(b.bnPs);
      o.bnPb = f32(b.bnPb);
      o.convP = conv1(b.convP, Wd, mid);
      o.inner.resize(2);
      buildBlock(b.inner[0], mid, o.inner[0]);
      buildBlock(b.inner[1], mid, o.inner[1]);
      o.bnQs = f32(b.bnQs);
      o.bnQb = f32(b.bnQb);
      o.convQ = conv1(b.convQ, mid, Wd);
      return;
    }
    o.bn1s = f32(b.bn1s);
    o.bn1b = f32(b.bn1b);
    if(b.kind == 0) {
      o.conv1 = conv3(b.conv1, Wd, Wd);
      o.bn2s = f32(b.bn2s);
      o.bn2b = f32(b.bn2b);
      o.conv2 = conv3(b.conv2, Wd, Wd);
    } else {
      const int Cg = cfg_.Cg, Cr = Wd - Cg;
      o.conv1 = packConvL(3, Wd, Wd, [&](int co, int ci, int tap) {
        return co < Cr ? b.conv1[((size_t)co * Wd + ci) * 9 + tap] : b.conv1g[((size_t)(co - Cr) * Wd + ci) * 9 + tap];
      });
      o.bngs = f32(b.bngs);
      o.bngb = f32(b.bngb);
      o.linGT = f32(transpose(b.linG, Cr, 3 * Cg));
      o.bn2s = f32(b.bn2s);
      o.bn2b = f32(b.bn2b);
      o.conv2 = conv3(b.conv2, Cr, Wd);
    }
  };
  const int C = cfg_.C;
  stem_ = packConvL(3, cfg_.cin, C, [&](int co, int ci, int tap) {
    return m.convInit[((size_t)co * cfg_.cin + ci) * 9 + tap];
  });
  globInit_ = f32(m.globInit);
  blocks_.resize(cfg_.kinds.size());
  for(size_t i = 0; i < blocks_.size(); i++)
    buildBlock(m.blocks[i], C, blocks_[i]);
  tips_ = f32(m.tips);
  tipb_ = f32(m.tipb);
  const int HWd = cfg_.p1 + cfg_.g1 + cfg_.v1;
  head_ = packConvL(1, C, HWd, [&](int co, int ci, int) {
    if(co < cfg_.p1)
      return m.pConv1[(size_t)co * C + ci];
    if(co < cfg_.p1 + cfg_.g1)
      return m.pConvG[(size_t)(co - cfg_.p1) * C + ci];
    return m.vConv1[(size_t)(co - cfg_.p1 - cfg_.g1) * C + ci];
  });
  hw_.pBiasG = f32(m.pBiasG);
  hw_.pLinGT = f32(transpose(m.pLinG, cfg_.p1, 3 * cfg_.g1));
  hw_.pBias2 = f32(m.pBias2);
  hw_.pConv2 = f32(m.pConv2);
  hw_.vBias1 = f32(m.vBias1);
  hw_.vLin2T = f32(transpose(m.vLin2, cfg_.v2, 3 * cfg_.v1));
  hw_.vB2 = f32(m.vB2);
  hw_.vLin3 = f32(m.vLin3);
  hw_.vB3 = f32(m.vB3);
  hw_.vLinM = f32(m.vLinM);
  hw_.vBM = f32(m.vBM);
  // widest activation buffers
  maxW_ = C;
  if(cfg_.mid > maxW_)
    maxW_ = cfg_.mid;
  tW_ = std::max(maxW_, HWd);
  // pad T / H widths so every column tile of the widest conv stays in bounds
  tW_ = (tW_ + 127) / 128 * 128;
  hW_ = (maxW_ + 127) / 128 * 128;
  KC_HIP(hipMalloc(&wHi_, wh.size() * 2));
  KC_HIP(hipMemcpy(wHi_, wh.data(), wh.size() * 2, hipMemcpyHostToDevice));
  if(split_) {
    KC_HIP(hipMalloc(&wLo_, wl.size() * 2));
    KC_HIP(hipMemcpy(wLo_, wl.data(), wl.size() * 2, hipMemcpyHostToDevice));
  }
  KC_HIP(hipMalloc(&wF_, wf.size() * 4));
  KC_HIP(hipMemcpy(wF_, wf.data(), wf.size() * 4, hipMemcpyHostToDevice));
  flops_ = modelFlopsPerEval(cfg_, A);
}

NNLayered::~NNLayered() {
  (void)hipFree(wHi_);
  (void)hipFree(wLo_);
  (void)hipFree(wF_);
  (void)hipFree(act_);
}

void NNLayered::ensure(int n) {
  if(n <= cap_)
    return;
  (void)hipFree(act_);
  act_ = nullptr;
  const int bpw = lBoardsPerWG(X_, Y_);
  const int nPad = (n + bpw - 1) / bpw * bpw;
  const size_t rows = (size_t)nPad * X_ * Y_;
  // X f32 [rows][C] | Y f32 [rows][mid] | T f32 [rows][tW] | H f16 [rows][hW] | gb f32 [nPad][C]
  const size_t bytes = rows * (cfg_.C + cfg_.mid + tW_) * 4 + rows * hW_ * 2 + (size_t)nPad * maxW_ * 4 + 256;
  KC_HIP(hipMalloc(&act_, bytes));
  char* p = reinterpret_cast<char*>(act_);
  bufX_ = reinterpret_cast<float*>(p);
  p += rows * cfg_.C * 4;
  bufY_ = reinterpret_cast<float*>(p);
  p += rows * cfg_.mid * 4;
  bufT_ = reinterpret_cast<float*>(p);
  p += rows * tW_ * 4;
  bufH_ = reinterpret_cast<uint16_t*>(p);
  p += rows * hW_ * 2;
  bufGB_ = reinterpret_cast<float*>(p);
  cap_ = nPad;
}

void NNLayered::conv(const Conv& c, int pro, const void* src, int srcLd, int srcOff, int psOff, int pbOff,
                     const float* gb, int gbLd, int epi, void* dst, int dstLd, int esOff, int ebOff, int n,
                     const int* countDev, const uint64_t* bits, const int* rowIdx, hipStream_t st) {
  LConvArgs a;
  memset(&a, 0, sizeof(a));
  a.pro = pro;
  a.cin = c.cin;
  a.cinReal = c.cinReal;
  a.src = src;
  a.srcLd = srcLd;
  a.srcOff = srcOff;
  a.ps = psOff >= 0 ? wF_ + psOff : nullptr;
  a.pb = pbOff >= 0 ? wF_ + pbOff : nullptr;
  a.gb = gb;
  a.gbLd = gb ? gbLd : 0;
  a.bits = bits;
  a.inWords = (NUM_SPATIAL * X_ * Y_ + 63) / 64;
  a.rowIdx = rowIdx;
  a.w = reinterpret_cast<const lh16x8*>(wHi_) + c.wOff;
  a.wlo = split_ ? reinterpret_cast<const lh16x8*>(wLo_) + c.wOff : nullptr;
  a.coutTiles = c.coutTiles;
  a.epi = epi;
  a.cout = c.cout;
  a.dst = dst;
  a.dstLd = dstLd;
  a.dstOff = 0;
  a.es = esOff >= 0 ? wF_ + esOff : nullptr;
  a.eb = ebOff >= 0 ? wF_ + ebOff : nullptr;
  a.glob = wF_ + globInit_;
  a.winLen = (float)W_;
  a.n = n;
  a.countDev = countDev;
  const int bpw = lBoardsPerWG(X_, Y_);
  const int grid = (n + bpw - 1) / bpw;
  const bool sp = split_;
  if(X_ == 5)
    sp ? launchConvG<5, 5, true>(a, c.kt, c.tn, c.wn, grid, st)
       : launchConvG<5, 5, false>(a, c.kt, c.tn, c.wn, grid, st);
  else if(X_ == 7)
    sp ? launchConvG<7, 7, true>(a, c.kt, c.tn, c.wn, grid, st)
       : launchConvG<7, 7, false>(a, c.kt, c.tn, c.wn, grid, st);
  else
    sp ? launchConvG<9, 9, true>(a, c.kt, c.tn, c.wn, grid, st)
       : launchConvG<9, 9, false>(a, c.kt, c.tn, c.wn, grid, st);
}

// x: trunk (f32, width = block width) updated in place.
void NNLayered::runBlock(const Block& b, float* x, int n, const int* countDev, hipStream_t st) {
  const int Wd = b.width;
  if(b.kind >= 2) {
    const int mid = cfg_.mid;
    conv(b.convP, PRO_BN, x, Wd, 0, b.bnPs, b.bnPb, nullptr, 0, EPI_STORE, bufY_, mid, -1, -1, n, countDev, nullptr,
         nullptr, st);
    for(const Block& in : b.inner)
      runBlock(in, bufY_, n, countDev, st);
    conv(b.convQ, PRO_BN, bufY_, mid, 0, b.bnQs, b.bnQb, nullptr, 0, EPI_ADD, x, Wd, -1, -1, n, countDev, nullptr,
         nullptr, st);
    return;
  }
  if(b.kind == 0 && !split_) {
    // mid activation BN2-ReLU'd in conv1's epilogue, stored fp16 (the conv2 operand)
    conv(b.conv1, PRO_BN, x, Wd, 0, b.bn1s, b.bn1b, nullptr, 0, EPI_BNRELU16, bufH_, hW_, b.bn2s, b.bn2b, n,
         countDev, nullptr, nullptr, st);
    conv(b.conv2, PRO_F16, bufH_, hW_, 0, -1, -1, nullptr, 0, EPI_ADD, x, Wd, -1, -1, n, countDev, nullptr, nullptr,
         st);
  } else if(b.kind == 0) {
    // split precision: the mid activation stays f32 so conv2's prologue can form hi + lo
    conv(b.conv1, PRO_BN, x, Wd, 0, b.bn1s, b.bn1b, nullptr, 0, EPI_STORE, bufT_, tW_, -1, -1, n, countDev, nullptr,
         nullptr, st);
    conv(b.conv2, PRO_BN, bufT_, tW_, 0, b.bn2s, b.bn2b, nullptr, 0, EPI_ADD, x, Wd, -1, -1, n, countDev, nullptr,
         nullptr, st);
  } else {
    const int Cg = cfg_.Cg, Cr = Wd - Cg;
    conv(b.conv1, PRO_BN, x, Wd, 0, b.bn1s, b.bn1b, nullptr, 0, EPI_STORE, bufT_, tW_, -1, -1, n, countDev, nullptr,
         nullptr, st);
    hipLaunchKernelGGL(kGpoolBias, dim3(n), dim3(256), 0, st, bufT_, tW_, X_ * Y_, Cr, Cg, wF_ + b.bngs,
                       wF_ + b.bngb, wF_ + b.linGT, bufGB_, n, countDev);
    KC_HIP(hipGetLastError());
    conv(b.conv2, PRO_BN_GB, bufT_, tW_, 0, b.bn2s, b.bn2b, bufGB_, Cr, EPI_ADD, x, Wd, -1, -1, n, countDev, nullptr,
         nullptr, st);
  }
}

void NNLayered::forward(int n, const uint64_t* in, float* out, hipStream_t st, const int* countDev, const int* rowIdx) {
  if(n <= 0)
    return;
  ensure(n);
  const int C = cfg_.C;
  conv(stem_, PRO_BITS, nullptr, 0, 0, -1, -1, nullptr, 0, EPI_STEM, bufX_, C, -1, -1, n, countDev, in, rowIdx, st);
  for(const Block& b : blocks_)
    runBlock(b, bufX_, n, countDev, st);
  conv(head_, PRO_BN, bufX_, C, 0, tips_, tipb_, nullptr, 0, EPI_STORE, bufT_, tW_, -1, -1, n, countDev, nullptr,
       nullptr, st);
  LHeadW h;
  h.pBiasG = wF_ + hw_.pBiasG;
  h.pLinGT = wF_ + hw_.pLinGT;
  h.pBias2 = wF_ + hw_.pBias2;
  h.pConv2 = wF_ + hw_.pConv2;
  h.vBias1 = wF_ + hw_.vBias1;
  h.vLin2T = wF_ + hw_.vLin2T;
  h.vB2 = wF_ + hw_.vB2;
  h.vLin3 = wF_ + hw_.vLin3;
  h.vB3 = wF_ + hw_.vB3;
  h.vLinM = wF_ + hw_.vLinM;
  h.vBM = wF_ + hw_.vBM;
  h.p1 = cfg_.p1;
  h.g1 = cfg_.g1;
  h.v1 = cfg_.v1;
  h.v2 = cfg_.v2;
  hipLaunchKernelGGL(kHeadsL, dim3(n), dim3(256), 0, st, bufT_, tW_, X_ * Y_, h, out, rowIdx, n, countDev);
  KC_HIP(hipGetLastError());
}

#ifdef KC_SEARCH_PROFILE
// kConvLB cycle accounting (profiling build): the 8 slots of g_convlProf, then reset.
extern "C" void coffee_debug_convl_profile(unsigned long long* out, int reset) {
  KC_HIP(hipDeviceSynchronize());
  KC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_convlProf), 8 * sizeof(unsigned long long)));
  if(reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    KC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_convlProf), z, sizeof(z)));
  }
}
#endif

}  // namespace kc
