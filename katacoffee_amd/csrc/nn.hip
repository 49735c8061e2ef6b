// Fused residual-network forward for Coffee leaf batches (one launch per batch).
//
// Semantics: eigenbackend.cpp (ConvLayer :270-680, BatchNormLayer :684-734,
// poolRowsGPool :141-166, poolRowsValueHead :168-186, ResidualBlock :888-931,
// GlobalPoolingResidualBlock :935-1015, Trunk :1169-1227, PolicyHead :1229-1299,
// ValueHead :1301-1377), Coffee head contract nninputs.h:75-118.
//
// MI355X design ("The fused network at C2 batch sizes"):
//  * one 512-thread workgroup (8 waves, 2 per SIMD, one workgroup per CU) per 8
//    boards, or per 5 boards when the batch fits 5 per CU (125 positions in the 128
//    rows the waves compute; 185 VGPRs, so one search wave of the other game group
//    still fits on each SIMD beside it);
//  * 3x3 convolutions are implicit GEMMs on v_mfma_f32_16x16x32_f16 (fp16
//    operands, f32 accumulation; same rate as bf16 on gfx950, 3 more mantissa
//    bits), computed transposed (weights x activations):
//    A = activations gathered from LDS by neighbour offset (fp16, NHWC, zero-bordered
//    boards, conflict-free ds_read_b128), B = weights pre-swizzled on the host into
//    per-lane 16-byte fragments streamed into an LDS ring by LDS-DMA across the
//    convolution boundaries;
//  * the f32 residual trunk lives in the accumulators between blocks; during each
//    block's first conv it is parked in registers (5-board instance) or in a
//    workgroup-private L2-resident scratch (8-board instance);
//  * BN + ReLU, global pooling, the gpool bias and both heads are fused epilogues.
// Waves: rg = wave>>1 owns a contiguous range of 16-row tiles, cg = wave&1 owns
// half of the output channels.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <mutex>
#include <vector>

#include "detmath.h"
#include "engine.h"
#include "kc_board.h"
#include "lds_dma.h"

namespace kc {

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Operand precision of an instance (MODE): 0 fp16 operands ("fast"); 1 fp16 hi/lo pairs,
// three MFMAs per product ("accurate"); 2 fp16 hi * hi plus the two cross terms on one
// block-scaled fp8 MFMA at twice the fp16 rate ("corrected", below).
enum { NN_MODE_F16 = 0, NN_MODE_SPLIT3 = 1, NN_MODE_F8C = 2 };
// Corrected mode: w x = hi(w) hi(x) + lo(w) x + w lo(x) + lo(w) lo(x), with lo(v) = v - fp16(v)
// (|lo(v)| <= 2^-11 |v|).  The first product runs on v_mfma_f32_16x16x32_f16; the two
// cross terms (the last is below f32 rounding) on v_mfma_scale_f32_16x16x128_f8f6f4 with
// e4m3 operands over two K-steps: A = [e4m3(lo(w) 2^(11-sw)) | e4m3(hi(w) 2^-sw)] with
// E8M0 scale 2^(sw-11), sw the convolution's block exponent (f8Exp of its largest |w|: the
// largest weight lands in (224, 448], so no weight saturates and small weights stay in
// e4m3's normal range), B = [e4m3(hi(x)) | e4m3(lo(x) 2^11)] with scale 1 (the e4m3 of
// w and x is taken of their fp16 values, hi(v) = fp16(v), as oracle/ora_nn.cpp restates).  Each cross term
// carries e4m3's 2^-4 relative error on a value 2^-11 below the product, so a product is
// good to ~2^-14 (fp16 operands: 2^-10): tools/precision_study.py.  An activation past
// e4m3's 448 (its conversion gives NaN) flags its board, and that board is re-evaluated by
// the accurate (split) instance in a second launch (kNNForward's `hot` argument) -- on
// realistic nets that launch finds no flag and every workgroup exits at once.
// (Per-board activation exponents instead of the flag were tried in round 5: their board
// maxima must be published by a barrier before each epilogue, and the capped instance's
// spill reloads then wait for the weight DMA in flight: 8 % slower)
constexpr int F8C_SHIFT = 11;
constexpr float F8C_MAX = 448.0f;  // largest finite e4m3fn
// The corrected instance is register-capped so that a 128-VGPR search wave of the other
// game group fits on each SIMD beside its two network waves (2 x 192 + 128 = 512):
// it is compiled separately (nn_corr.hip) as kNNForwardCap with amdgpu_num_vgpr
// KC_F8C_VGPR, which gfx950 counts in register pairs (96 = 192 VGPRs; 0: uncapped, the
// plain kNNForward instance).  KC_F8C_PARK 1: the f32 trunk is parked in the
// workgroup-private global scratch during a block's first conv (24 registers);
// KC_F8C_LATE 1: a K-step's fragments are read after the previous step's MFMAs issue
// (one fragment buffer).  (A/B builds: tools/Makefile alt, ALT_FLAGS=-DKC_F8C_VGPR=0 ...)
// Measured (C2 corrected bench, one box, 20 steps): uncapped 19.0 k rows/s (network 144 us,
// other group's select 105 us: no room beside the network's 233-256-VGPR waves); capped +
// late 19.5 k (network 163 us, select 71 us, backup 50 -> 59 us: the search waves now share
// the network's CUs); capped + late + parked trunk 19.3 k; late + parked, uncapped 18.1 k.
// Second box: capped + late 19.4 k, capped + parked 19.3 k, capped alone 19.7 k (network
// 154 us; 49 registers spilled, reloaded outside the K loops): the default.
#ifndef KC_F8C_VGPR
#define KC_F8C_VGPR 96
#endif
// KC_ACC_CAP 1: the accurate (split) borderless instance runs under the same cap (222 VGPRs
// uncapped: no search wave of the other game group fits beside it); 0: uncapped (A/B)
#ifndef KC_ACC_CAP
#define KC_ACC_CAP 1
#endif
// KC_ACC_LATE 1: the accurate borderless instance reads a K-step's fragments after the
// previous step's MFMAs issue (one fragment buffer, like KC_F8C_LATE); 0: double-buffered.
// Measured (round 6, profiles/r06/acc_late_ab.txt): 182 VGPRs and no spills against 17 spilled,
// but the network alone 3 % slower and the C2 bench equal within noise: off
#ifndef KC_ACC_LATE
#define KC_ACC_LATE 0
#endif
#ifndef KC_F8C_PARK
#define KC_F8C_PARK 0
#endif
#ifndef KC_F8C_LATE
#define KC_F8C_LATE 0
#endif
// KC_F8C_CVTW 1: the weights' e4m3(hi(w) 2^-sw) is converted from the fp16 fragments in
// registers (the ring slot holds fp16 hi + e4m3 lo(w): 27 KiB per 96-channel tap), 0: the
// slot holds host-packed e4m3 [lo(w) | hi(w)] pairs (36 KiB).  KC_F8C_CVTX 1: e4m3(hi(x))
// is converted from the activation fragments (the second plane holds e4m3 lo(x) only, one
// byte per channel), 0: the plane holds [hi(x) | lo(x)] pairs.  Either conversion frees
// the LDS for a 3-slot weight ring (both off: the 2-slot ring, the default).  Measured
// (round 5, tools/ab_nn.sh, 960 boards): 2-slot 153 us; both converted 191-348 us
// (register pressure: 72-96 spilled VGPRs under the cap), activations only 186 us,
// weights only 331 us.  tools/cvt_rate.hip: one v_cvt_scalef32_pk_fp8_f16 costs 13.8
// cycles per wave at 2 waves per SIMD (v_add_f32: 5.1) and each adds ~11 cycles to the
// K-step's MFMA stream -- it does not co-issue beside the MFMAs, so the 8-20 conversions
// per K-step cost more than the deeper ring and the smaller LDS footprint save.
#ifndef KC_F8C_CVTW
#define KC_F8C_CVTW 0
#endif
// KC_FAST_BL 1: the fast (fp16) small-batch instance is borderless too, with ring slots of
// three taps (one barrier per three taps instead of per pair; 192-VGPR cap, 17 spilled;
// the branch scratch in ring slot 1); 0: the bordered 5-board instance with the paired
// 4-slot ring (rounds 3-4, the default).  Measured (round 5, same box): network alone
// 77.7 vs 75.3 us at 960 boards, C2 bench 22.9-23.1 k vs 24.0 k rows/s (in-bench network
// 94 vs 84 us: its 149 KB of LDS leaves the other group's search blocks less room).
#ifndef KC_FAST_BL
#define KC_FAST_BL 0
#endif
#ifndef KC_F8C_CVTX
#define KC_F8C_CVTX 0
#endif
constexpr float F8C_SCALE = 2048.0f;  // 2^F8C_SHIFT
// Block exponent of the corrected precision's e4m3 weights (oracle/ora_nn.cpp f8Exp, the
// same integer arithmetic): m 2^-s in (224, 448] for m > 0 (m = f 2^e, f in [0.5, 1):
// s = e - 9, or e - 8 when f > 0.875, since 448 = 0.875 2^9); 0 for m == 0.
inline int f8Exp(float m) {
  if(!(m > 0.0f))
    return 0;
  int e;
  const float f = std::frexp(m, &e);
  const int s = e - 9 + (f > 0.875f ? 1 : 0);
  return s < -100 ? -100 : (s > 100 ? 100 : s);
}

template <int X_, int Y_, int C_, int NB_ = NN_BOARDS_PER_WG, int MODE_ = 0, bool BL_ = false>
struct NNGeo {
  static constexpr int X = X_, Y = Y_, C = C_, A = X_ * Y_;
  // boards per workgroup: 8, or NN_SMALL_NB (5) for batches of at most 5 per CU; one
  // 8-wave workgroup per CU, 2 waves per SIMD (tools/conv_bench.hip measured the alternatives:
  // 2 boards on 4 waves at two workgroups per CU streams every weight twice per CU, and
  // 4 boards on 4 waves with one wave per SIMD cuts the LDS reads per MFMA by 30 % but
  // exposes every LDS and barrier latency: both slower)
  static constexpr int NB = NB_;
  static constexpr int NW = 8, NT = NW * 64;  // waves / threads per workgroup
  static constexpr int MODE = MODE_;
  // SPLIT (modes 1 and 2): every conv operand carries a second LDS plane and every weight
  // tap a second block after the hi one -- fp16 lo values (mode 1), or e4m3 pairs
  // (mode 2: activations [x | lo(x) 2^11], weights [lo(w) 2^11 | w], per 8 channels).
  static constexpr bool SPLIT = MODE_ != NN_MODE_F16;
  static constexpr int PLANES = SPLIT ? 2 : 1;
  // BL ("borderless", the 5-board split instances): activations are stored one row per
  // position, no zero border; a 3x3 tap whose neighbour is off the board reads a shared
  // zero row instead (per-lane address select per tap).  That halves the activation
  // planes (129 rows instead of 5 x 49), so two planes of 5 boards and a 2-slot ring of
  // 36 KiB taps fit the 160 KiB.
  static constexpr bool BL = BL_;
  // weight ring slots.  3 (8-board and 2-board SPLIT instances, whose LDS holds no more): tap
  // k+2 is requested at the start of tap k, one barrier per tap.  4 (small-batch
  // instance): taps move in pairs (g, g+1), g even in the stream's global tap count;
  // pair j+1 is requested at the start of pair j and published by one barrier per pair.
  // 2 (BL split): chunks (one 36 KiB slot: a 96-channel tap, or 3 stem taps) alternate;
  // chunk j+2 is requested right after the barrier that publishes chunk j+1 and frees
  // chunk j.  3 (BL corrected: 27 KiB slots, the e4m3 weights derived from the fp16
  // fragments in registers): chunk j+3 is requested after that barrier, so a chunk's DMA
  // has two chunks of MFMAs to land in.  (6 slots, one barrier per 3 taps, would fill all
  // 160 KiB and keep the other game group's search kernels off the CU while the network
  // runs.)
  static constexpr bool F8W = MODE_ == NN_MODE_F8C && KC_F8C_CVTW;  // e4m3(w) converted in registers
  static constexpr bool F8X = MODE_ == NN_MODE_F8C && KC_F8C_CVTX;  // e4m3(x) converted in registers
  static constexpr int RING = BL ? ((F8W || F8X) ? 3 : 2) : ((NB_ == NN_SMALL_NB && !SPLIT) ? 4 : 3);
  static constexpr bool PAIRS = RING == 4;
  static constexpr int ROWS = NB * A;
  static constexpr int RT = (ROWS + 15) / 16;
  // Every wave owns MAXT whole tiles (uniform, branch-free MFMA loops): output
  // rows [ROWS, 64*MAXT) are padding (computed from arbitrary data, never stored).
  static constexpr int RGROUPS = NW / 2;  // row groups (x 2 column halves)
  static constexpr int MAXT = (RT + RGROUPS - 1) / RGROUPS;
  static constexpr int MROWS = RGROUPS * MAXT * 16;  // computed output rows
  // Activations in LDS are stored per board with a one-cell zero border
  // ((Y+2) x (X+2) cells), so every 3x3 neighbour of an on-board cell is a fixed
  // row offset away and the implicit-GEMM A reads need no bounds checks (BL: row r is
  // output row r, and row ZROW = MROWS is all zeros).
  static constexpr int PX = X + 2, PY = Y + 2, PA = PX * PY;
  static constexpr int ZROW = MROWS;
  static constexpr int PROWS = BL ? MROWS + 1 : NB * PA;
  // fp16 per activation row: 56-dword rows make the A-fragment ds_read_b128 (lane
  // groups {0-3,12-15,20-27}, ... ; 16 rows x 4 k-quarters) bank-conflict free.
  static constexpr int ASTR = C + 16;
  static constexpr int ROWB = ASTR * 2;  // bytes per activation row
  static constexpr int NCT = C / 32;     // 16-col tiles per wave
  static constexpr int NCT_ALL = C / 16;
  static constexpr int P = 4 * A;
  static constexpr int PLANE_BYTES = (PROWS * ROWB + 15) / 16 * 16;  // the hi plane
  // the second plane: fp16 lo values (mode 1, rows like the hi plane); e4m3(lo(x) 2^11)
  // (mode 2: one byte per channel, rows of ROWB / 2 bytes, so a lane's address there is
  // half its hi-plane address; e4m3(x) is converted from the hi fragment in registers)
  static constexpr int ROWB2 = F8X ? ROWB / 2 : ROWB;
  static constexpr int PLANE2_BYTES = SPLIT ? (PROWS * ROWB2 + 15) / 16 * 16 : 0;
  static constexpr int ACT_BYTES = PLANE_BYTES + PLANE2_BYTES;
  // f32 [MROWS][SCR] scratch for the g / value branches: aliases act (dead then)
  static constexpr int SCR = 36;  // f32 scratch row stride: 4-row lane groups hit distinct banks
  // (at least the gpool linear weights' [96][64] f32, staged below it)
  static constexpr int OFF_SCR = MROWS * SCR * 4 > 96 * 64 * 4 ? MROWS * SCR * 4 : 96 * 64 * 4;
  static constexpr int OFF_POOL = ACT_BYTES;
  static constexpr int OFF_BIAS = OFF_POOL + 2 * NB * 96 * 4;
  static constexpr int WBUF = (C / 32) * NCT_ALL * 64;  // 16-B weight fragments per tap and plane
  // a tap's second weight block: fp16 lo fragments (mode 1); e4m3(lo(w) 2^(11-sw)) only, 8 B
  // per lane and fragment (mode 2: e4m3(w 2^-sw) is converted from the hi fragment)
  static constexpr int WBUF2 = !SPLIT ? 0 : (F8W ? WBUF / 2 : WBUF);
  // one ring slot (16-B units): a tap's blocks, or three fp16 taps (fast borderless)
  static constexpr int WSLOT = (BL && !SPLIT) ? 3 * WBUF : WBUF + WBUF2;
  static constexpr int SLOT_PIECES = WSLOT / 64;  // its 1-KiB pieces
  // 1-KiB pieces of one tap of a conv with ncb 32-channel input blocks
  static constexpr int tapPieces(int ncb) { return ncb * NCT_ALL * (!SPLIT ? 2 : (F8W ? 3 : 4)) / 2; }
  // BL ring chunks of a conv with ntaps taps of ncb blocks: taps per chunk, chunks, and the
  // pieces of its first chunk (what the previous conv requests ahead)
  static constexpr int chunkTaps(int ncb, int ntaps) {
    return SLOT_PIECES / tapPieces(ncb) < 1 ? 1 : (SLOT_PIECES / tapPieces(ncb) < ntaps ? SLOT_PIECES / tapPieces(ncb) : ntaps);
  }
  static constexpr int chunks(int ncb, int ntaps) { return (ntaps + chunkTaps(ncb, ntaps) - 1) / chunkTaps(ncb, ntaps); }
  static constexpr int firstChunkPieces(int ncb, int ntaps) { return chunkTaps(ncb, ntaps) * tapPieces(ncb); }
  // row tables (u16): rowPa[MROWS], rowBP[MROWS], bpRow[ROWS] -- built on the host
  static constexpr int NTAB = 2 * MROWS + ROWS;
  static constexpr int OFF_TAB = OFF_BIAS + NB * 64 * 4;
  // the value head's hidden layer [NB][64] f32 lives in the (idle) ring during the
  // heads, after the policy-gpool and value linear weights staged there
  static constexpr int RING_VH = (32 + 64) * 96 * 4;
  // per-block f32 parameter slabs (double buffered, filled one block ahead)
  static constexpr int NPRM = NN_PRM;
  static constexpr int OFF_PRM = (OFF_TAB + NTAB * 2 + 15) / 16 * 16;
  static constexpr int OFF_W = OFF_PRM + 2 * NPRM * 4;
  static constexpr int LDS = OFF_W + RING * WSLOT * 16;
  // the f32 scratch of the g / value branches: in act (dead then), or -- fast borderless,
  // whose one-plane act is too small -- in ring slot 1, which holds only a consumed chunk
  // during the gpool mids (conv1's last chunk; conv2's first is in slot 0) and the heads
  // (the head conv's chunk; the heads' linear weights use slot 0)
  static constexpr bool SCR_IN_RING = BL && !SPLIT;
  static constexpr int SCR_OFF = SCR_IN_RING ? OFF_W + WSLOT * 16 : OFF_SCR;
  static_assert(C % 32 == 0, "C must be a multiple of 32");
  static_assert(SCR_IN_RING ? (MROWS * SCR * 4 <= WSLOT * 16 && RING == 2 && RING_VH + NB * 64 * 4 <= WSLOT * 16)
                            : OFF_SCR + MROWS * SCR * 4 <= ACT_BYTES,
                "f32 branch scratch must fit in act (or in ring slot 1)");
  static_assert(96 * 64 * 4 <= OFF_SCR, "gpool linear weights must fit below scr");
  static_assert(RING * WSLOT * 16 >= RING_VH + NB * 64 * 4, "head linear weights and vh must fit in the ring");
  static_assert((PLANES - 1) * PLANE_BYTES + (BL ? 0 : 2 * PA * ROWB) + 2 * 64 < 65536,
                "A-read offsets must fit the ds_read immediate");
  static_assert(!BL || C == 96, "borderless instances: b6c96");
  static_assert(LDS <= 163840, "LDS budget");
};

#ifdef KC_NN_PROFILE
// Phase timestamps (shader clock) of the first workgroups: tools/nn_phase.hip.
__device__ unsigned long long g_nnPhase[4][64];
#define NN_PHASE(i)                                  \
  do {                                               \
    if(blockIdx.x < 4 && threadIdx.x == 0) {         \
      g_nnPhase[blockIdx.x][(i)] = clock64();        \
      if((i) == 0 || (i) == 42)                      \
        g_nnPhase[blockIdx.x][(i) == 0 ? 62 : 63] =  \
            __builtin_amdgcn_s_memrealtime();        \
    }                                                \
  } while(0)
#else
#define NN_PHASE(i) \
  do {              \
  } while(0)
#endif

KC_D uint16_t f16bits(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }  // v_cvt_f16_f32, RNE

// Padded LDS row of cell p of board b.
template <class G>
KC_D int padCell(int b, int p) {
  const int y = p / G::X, x = p - y * G::X;
  return b * G::PA + (y + 1) * G::PX + x + 1;
}

// Byte address of this lane's activation-fragment row for tile t, shifted to the
// (-1,-1) neighbour so every tap / channel block is a non-negative immediate
// offset.  Padding rows read row 0's cells (their outputs are never stored).
template <class G>
KC_D void aBases(int (&ab)[G::MAXT], const uint16_t* rowPa, int tstart, int lane) {
#pragma unroll
  for(int t = 0; t < G::MAXT; t++) {
    const int r = (tstart + t) * 16 + (lane & 15);
    ab[t] = ((int)rowPa[r] - G::PX - 1) * G::ROWB + 16 * (lane >> 4);
  }
}

// A tap's weights (CH pieces of 64 fragments) into its ring slot; piece c by wave
// (c + rot) % nw (rot spreads two taps' remainders over different waves).
template <int NW>
KC_D void stageTapDma(const h16x8* __restrict__ src, uint32_t slotAddr, int ch, int wave, int lane, int rot = 0) {
  for(int c = (wave + NW - rot % NW) % NW; c < ch; c += NW)
    glds16s(src + c * 64, (uint32_t)lane * 16u, slotAddr + c * 1024);
}

// Implicit-GEMM convolution over the wave's tiles, computed transposed:
// acc[t][ct] += W(ct, K) * act(K, t), so each lane's accumulator holds 4
// consecutive output channels of one position (16-byte-friendly epilogues).
//
// Weights stream through a 3-slot LDS ring shared by the workgroup's 8 waves by
// LDS-DMA: tap k lives in slot k%3, and tap k+2 is requested at the start of tap k,
// two taps ahead of its use.  The stream runs across convolutions: taps 7 and 8
// request the NEXT convolution's taps 0 and 1 (wNext, chNext pieces per tap,
// nextTaps), so only the first convolution pays an L2 round trip up front.  One
// barrier per tap, before its last K-step: it publishes tap k+1 (each wave first
// retires its own pieces of it) and frees slot k%3 for the request of tap k+3.
// Within a wave the A/B fragments of the next K-step are read from LDS while the
// current step's MFMAs issue.  Fully unrolled: slot and fragment-buffer indices
// are compile-time constants and every LDS read a per-lane base plus an immediate.
// The caller keeps the ring slots of the next convolution's first taps untouched
// between convolutions and separates them with __syncthreads() (which also retires
// the requests for those taps).
// DBG (tools/conv_bench.hip ablations only): bit 0 skips the weight requests, bit 1
// the per-tap barriers, bit 3 the vmcnt waits, bit 8 the entry wait + barrier.
//
// G::PAIRS (4-slot ring): the weight stream's taps are counted globally across the
// convolutions (g0 = this conv's first tap: the stem 0, block b's conv1 9 + 18b and
// conv2 18 + 18b, the head 9 + 18 nblocks; PAR = g0 & 1 fixes the pair boundaries at
// compile time); tap g lives in slot g & 3.  At the start of each pair (g even) the
// next pair (g+2, g+3: this conv's or the next conv's first taps) is requested into the
// slots that the previous pair's barrier freed; the barrier before the pair's last
// K-step retires every wave's pieces of the next pair (vmcnt 0: nothing newer is in
// flight) and frees this pair's slots -- one barrier per two taps instead of one per tap.
// ENTRY = false: the caller already retired its DMA (waitVm<0>) before the barrier that
// published the conv's input, which then also publishes the first taps (one barrier
// fewer per conv).
template <class G, int NTAPS, int NCB, int PAR = 0, int DBG = 0, bool ENTRY = true>
KC_D void convTiles(const uint16_t* __restrict__ act, const h16x8* __restrict__ w, h16x8* __restrict__ wl,
                    f32x4 (&acc)[G::MAXT][G::NCT], const int (&ab)[G::MAXT], int cg, int lane, int tid,
                    const h16x8* __restrict__ wNext, int chNext, int nextTaps, int g0 = 0) {
  constexpr int CHP = NCB * G::NCT_ALL;  // 1-KiB pieces per tap and plane
  constexpr int CH = CHP * G::PLANES;    // 1-KiB pieces per tap (the lo block after the hi one)
  constexpr int UNITS = CH * 64;         // 16-B fragments per tap
  constexpr int STEPS = NTAPS * NCB;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t ring = ldsAddr(wl);
  // ring slot of local tap t (the 3-slot ring's taps start at slot 0 in every conv)
  auto slotOf = [&](int tap) { return G::PAIRS ? (g0 + tap) & 3 : tap % 3; };
  if(ENTRY && !(DBG & 256)) {
    waitVm<0>();
    __syncthreads();
  }
  const char* actB = reinterpret_cast<const char*>(act);
  const h16x8* wlane = wl + (cg * G::NCT) * 64 + lane;
  h16x8 af[2][G::MAXT], bf[2][G::NCT];
  h16x8 afl[G::SPLIT ? 2 : 1][G::MAXT], bfl[G::SPLIT ? 2 : 1][G::NCT];  // lo planes (SPLIT)
  auto loadStep = [&](int st, int buf) {
    const int tap = st / NCB, cb = st - tap * NCB;
    const int tb = NTAPS == 9 ? tap : 4;  // 1x1: the centre tap
    const int aoff = ((tb / 3) * G::PX + tb % 3) * G::ROWB + cb * 64;
    const h16x8* wb = wlane + slotOf(tap) * G::WSLOT + cb * G::NCT_ALL * 64;
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++) {
      bf[buf][ct] = wb[ct * 64];
      if constexpr(G::SPLIT)
        bfl[buf][ct] = wb[CHP * 64 + ct * 64];
    }
#pragma unroll
    for(int t = 0; t < G::MAXT; t++) {
      af[buf][t] = *reinterpret_cast<const h16x8*>(actB + ab[t] + aoff);
      if constexpr(G::SPLIT)
        afl[buf][t] = *reinterpret_cast<const h16x8*>(actB + G::PLANE_BYTES + ab[t] + aoff);
    }
  };
  loadStep(0, 0);
#pragma unroll
  for(int tap = 0; tap < NTAPS; tap++) {
    const bool pairStart = ((PAR + tap) & 1) == 0;
    if(DBG & 1) {
    } else if(G::PAIRS) {
      if(pairStart) {
        // request the next pair: stream taps tap+2, tap+3 (this conv's or the next's)
#pragma unroll
        for(int k = 2; k <= 3; k++) {
          const int u = tap + k;
          const uint32_t dst = ring + (uint32_t)(((g0 + u) & 3) * G::WSLOT * 16);
          if(u < NTAPS)
            stageTapDma<G::NW>(w + (size_t)u * UNITS, dst, CH, wave, lane, (k - 2) * CH);
          else if(u - NTAPS < nextTaps)
            stageTapDma<G::NW>(wNext + (size_t)(u - NTAPS) * chNext * 64, dst, chNext, wave, lane, (k - 2) * chNext);
        }
      }
    } else if(tap + 2 < NTAPS)
      // request stream tap tap+2 (this conv's, or the next conv's tap 0 / 1)
      stageTapDma<G::NW>(w + (size_t)(tap + 2) * UNITS, ring + slotOf(tap + 2) * G::WSLOT * 16, CH, wave, lane);
    else if(NTAPS == 9 && tap == 7)
      stageTapDma<G::NW>(wNext, ring, chNext, wave, lane);
    else if(NTAPS == 9 && tap == 8 && nextTaps > 1)
      stageTapDma<G::NW>(wNext + chNext * 64, ring + G::WSLOT * 16, chNext, wave, lane);
#pragma unroll
    for(int cb = 0; cb < NCB; cb++) {
      const int st = tap * NCB + cb;
      if(G::PAIRS && cb == NCB - 1 && !pairStart && tap + 1 < NTAPS) {
        // end of a pair: retire this wave's pieces of the next pair, publish them and
        // free this pair's slots
        if(!(DBG & 8))
          waitVm<0>();
        if(!(DBG & 2))
          barrierKeepDma();
      } else if(!G::PAIRS && cb == NCB - 1 && tap + 1 < NTAPS) {
        // retire this wave's pieces of tap+1 (only the tap+2 request, >= N pieces per
        // wave, may stay in flight), then publish them / free slot tap%3
        if(DBG & 8) {
        } else if(tap + 2 < NTAPS)
          waitVm<CH / G::NW>();
        else
          waitVm<(2 * G::NCT_ALL * G::PLANES) / G::NW>();  // next conv's tap 0: at least 12 pieces per plane
        if(!(DBG & 2))
          barrierKeepDma();
      }
      if(st + 1 < STEPS)
        loadStep(st + 1, (st + 1) & 1);
      // keep the next step's LDS reads ahead of this step's MFMAs (the scheduler
      // otherwise sinks them behind the MFMAs to shorten live ranges)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for(int t = 0; t < G::MAXT; t++)
#pragma unroll
        for(int ct = 0; ct < G::NCT; ct++)
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[st & 1][ct], af[st & 1][t], acc[t][ct], 0, 0, 0);
      if constexpr(G::SPLIT) {
        // + lo(w) * hi(x), then + hi(w) * lo(x) (the layered kernels' order)
#pragma unroll
        for(int t = 0; t < G::MAXT; t++)
#pragma unroll
          for(int ct = 0; ct < G::NCT; ct++)
            acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bfl[st & 1][ct], af[st & 1][t], acc[t][ct], 0, 0, 0);
#pragma unroll
        for(int t = 0; t < G::MAXT; t++)
#pragma unroll
          for(int ct = 0; ct < G::NCT; ct++)
            acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[st & 1][ct], afl[st & 1][t], acc[t][ct], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ---- borderless (BL) instances ----------------------------------------------
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2x __attribute__((ext_vector_type(2)));

// Per tile: the byte address of this lane's A-fragment row (row r = output row r, plus
// the lane's k-quarter) and a 9-bit mask of the 3x3 taps whose neighbour is on the
// board (padding rows: none).  Tap ky*3 + kx reads row r + (ky-1) X + (kx-1).
template <class G>
KC_D void aRowsBL(int (&rb)[G::MAXT], uint32_t (&vm)[G::MAXT], int tstart, int lane) {
#pragma unroll
  for(int t = 0; t < G::MAXT; t++) {
    const int r = (tstart + t) * 16 + (lane & 15);
    const int p = r % G::A, y = p / G::X, x = p - y * G::X;
    uint32_t m = 0;
#pragma unroll
    for(int tap = 0; tap < 9; tap++) {
      const int ny = y + tap / 3 - 1, nx = x + tap % 3 - 1;
      if(r < G::ROWS && ny >= 0 && ny < G::Y && nx >= 0 && nx < G::X)
        m |= 1u << tap;
    }
    rb[t] = r * G::ROWB + 16 * (lane >> 4);
    vm[t] = m;
  }
}

// A weight chunk (`pieces` 1-KiB pieces, contiguous in the stream) into a ring slot.
template <int NW>
KC_D void stageChunk(const h16x8* __restrict__ src, uint32_t slotAddr, int pieces, int wave, int lane) {
  for(int c = wave; c < pieces; c += NW)
    glds16s(src + c * 64, (uint32_t)lane * 16u, slotAddr + c * 1024);
}

// Implicit-GEMM convolution of a BL instance, computed transposed like convTiles.
// Weights stream through the RING-slot ring in chunks of TPC taps (one slot: a 96-channel
// tap, or three stem taps); chunk j of this conv lives in slot (PAR + j) % RING, PAR the
// index mod RING of the conv's first chunk in the whole stream.  On entry chunks
// 0 .. RING-2 were requested and are resident and published (the caller retired its DMA
// before the barrier that published the conv's input), and the slot of chunk RING-1 is
// free: it is requested at once.  One barrier per chunk, before the chunk's last K-step:
// every wave retires its pieces of chunk j+1 (the younger requests -- chunk j+2 with three
// slots -- stay in flight: a counted vmcnt), the barrier publishes them and frees chunk j's
// slot (all its fragment reads are complete: lgkmcnt(0)), and chunk j+RING is requested
// into it (this conv's, or the next conv's chunk j+RING-NCH: nextPieces pieces each,
// nextNCH chunks).  A-fragment addresses are formed per tap: the neighbour row, or the
// zero row when the neighbour is off the board.
//   MODE 1: acc += hi(w) hi(x) + lo(w) hi(x) + hi(w) lo(x)  (three f16 MFMAs per step)
//   MODE 2: acc += hi(w) hi(x) per step (f16 MFMA), and per pair of steps one scaled e4m3
//           MFMA over [lo(w) 2^(11-sw) | hi(w) 2^-sw] x [hi(x) | lo(x) 2^11] of both steps,
//           A scale 2^(sw-11): lo(w) and lo(x) are read from the second weight block /
//           activation plane (8 bytes per lane and fragment), e4m3 of the hi fragments
//           is converted in registers (v_cvt_scalef32_pk_fp8_f16, which divides by its
//           scale: 2^sw for the weights, 1 for the activations).
//   sA (mode 2): the A operand's E8M0 scale byte, 127 - 11 + the conv's weight exponent sw.
// DBG (tools/convb_bench.hip ablations only): bit 0 skips the weight requests, bit 1 the
// chunk waits and barriers, bit 2 the scaled e4m3 MFMAs, bit 3 the second-plane fragment
// reads, bit 4 every fragment read after the first K-step, bit 5 the chunk waits only.
template <class G, int NTAPS, int NCB, int PAR, int DBG = 0>
KC_D void convTilesB(const uint16_t* __restrict__ act, const h16x8* __restrict__ w, h16x8* __restrict__ wl,
                     f32x4 (&acc)[G::MAXT][G::NCT], const int (&rb)[G::MAXT], const uint32_t (&vm)[G::MAXT],
                     int cg, int lane, int tid, const h16x8* __restrict__ wNext, int nextPieces, int nextNCH,
                     int sA = 0) {
  constexpr int CHP = NCB * G::NCT_ALL;  // 1-KiB pieces per tap of the hi block
  constexpr int CH = G::tapPieces(NCB);  // per tap
  constexpr int TPC = G::SLOT_PIECES / CH >= 1 ? G::SLOT_PIECES / CH : 1;
  static_assert(TPC * CH <= G::SLOT_PIECES, "a tap must fit one ring slot");
  constexpr int NCH = (NTAPS + TPC - 1) / TPC;
  constexpr int STEPS = NTAPS * NCB;
  constexpr int R = G::RING;
  constexpr bool F8C = G::MODE == NN_MODE_F8C;
  // fewest pieces any wave issues for a chunk of the next conv (a 64-channel tap: 2 blocks)
  constexpr int NEXT_MIN = G::tapPieces(2) / G::NW;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t ring = ldsAddr(wl);
  auto slotOf = [&](int j) { return (PAR + j) % R; };
  auto chunkPieces = [&](int j) { return (NTAPS - j * TPC < TPC ? NTAPS - j * TPC : TPC) * CH; };
  // the request of stream chunk j of this conv (j >= NCH: the next conv's chunk j - NCH)
  auto request = [&](int j) {
    if(DBG & 1)
      return;
    const uint32_t dst = ring + (uint32_t)(slotOf(j) * G::WSLOT * 16);
    if(j < NCH)
      stageChunk<G::NW>(w + (size_t)j * TPC * CH * 64, dst, chunkPieces(j), wave, lane);
    else if(j - NCH < nextNCH && nextPieces > 0)
      stageChunk<G::NW>(wNext + (size_t)(j - NCH) * nextPieces * 64, dst, nextPieces, wave, lane);
  };
  request(R - 1);
  const char* actB = reinterpret_cast<const char*>(act);
  const int zb = G::ZROW * G::ROWB + 16 * (lane >> 4);
  const h16x8* wlane = wl + (cg * G::NCT) * 64 + lane;
  int at[G::MAXT];  // this tap's A-fragment row addresses (hi plane; mode 2's plane: half)
  auto tapAddr = [&](int tap) {
    const int tb = NTAPS == 9 ? tap : 4;  // 1x1: the centre tap
    const int off = ((tb / 3 - 1) * G::X + (tb % 3 - 1)) * G::ROWB;
#pragma unroll
    for(int t = 0; t < G::MAXT; t++)
      at[t] = ((vm[t] >> tb) & 1u) ? rb[t] + off : zb;
  };
  h16x8 af[2][G::MAXT], bf[2][G::NCT];
  // second planes: fp16 lo fragments, double buffered (mode 1); e4m3 (mode 2), the two
  // steps of an MFMA pair in the low / high half of one 8-register operand, so the scaled
  // MFMA reads its operands in place (the halves are the double buffer): per step
  // bq = [lo(w) (loaded) | hi(w) (converted)], aq = [hi(x) (converted) | lo(x) (loaded)]
  h16x8 afl[G::MODE == NN_MODE_SPLIT3 ? 2 : 1][G::MAXT], bfl[G::MODE == NN_MODE_SPLIT3 ? 2 : 1][G::NCT];
  i32x8 aq[G::MAXT], bq[G::NCT];
  // 2^sw: the weights' conversion scale (the conversion divides by it)
  const float wScale = __builtin_bit_cast(float, (uint32_t)(sA - 127 + F8C_SHIFT + 127) << 23);
  auto loadStep = [&](int st, int buf) {
    const int tap = st / NCB, cb = st - tap * NCB;
    const int chunk = tap / TPC, tc = tap - chunk * TPC;
    const int slot = slotOf(chunk);
    const h16x8* wb = wlane + slot * G::WSLOT + tc * CH * 64 + cb * G::NCT_ALL * 64;
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++) {
      bf[buf][ct] = wb[ct * 64];
      if constexpr((DBG & 8) || G::MODE == NN_MODE_F16) {
      } else if constexpr(G::MODE == NN_MODE_SPLIT3) {
        bfl[buf][ct] = wb[CHP * 64 + ct * 64];
      } else if constexpr(!G::F8W) {
        const i32x4 v = __builtin_bit_cast(i32x4, wb[CHP * 64 + ct * 64]);  // [lo(w) | w] pairs
        if(buf)
          bq[ct].hi = v;
        else
          bq[ct].lo = v;
      } else {
        // this lane's 8 bytes of the fragment in the tap's e4m3 block (512 B per fragment)
        const int frag = cb * G::NCT_ALL + cg * G::NCT + ct;
        const int2 v = *reinterpret_cast<const int2*>(reinterpret_cast<const char*>(wl) +
                                                      (size_t)(slot * G::WSLOT + tc * CH * 64) * 16 + CHP * 1024 +
                                                      frag * 512 + lane * 8);
        bq[ct][4 * buf] = v.x;
        bq[ct][4 * buf + 1] = v.y;
      }
    }
#pragma unroll
    for(int t = 0; t < G::MAXT; t++) {
      af[buf][t] = *reinterpret_cast<const h16x8*>(actB + at[t] + cb * 64);
      if constexpr((DBG & 8) || G::MODE == NN_MODE_F16) {
      } else if constexpr(G::MODE == NN_MODE_SPLIT3) {
        afl[buf][t] = *reinterpret_cast<const h16x8*>(actB + G::PLANE_BYTES + at[t] + cb * 64);
      } else if constexpr(!G::F8X) {
        const i32x4 v = __builtin_bit_cast(i32x4, *reinterpret_cast<const h16x8*>(actB + G::PLANE_BYTES + at[t] + cb * 64));
        if(buf)
          aq[t].hi = v;
        else
          aq[t].lo = v;
      } else {
        const int2 v = *reinterpret_cast<const int2*>(actB + G::PLANE_BYTES + (at[t] >> 1) + cb * 32);
        aq[t][4 * buf + 2] = v.x;
        aq[t][4 * buf + 3] = v.y;
      }
    }
  };
  // mode 2: e4m3 of a step's hi fragments (8 fp16 values -> 8 bytes in two registers)
  auto e4m3x8 = [](const h16x8& h, float scale, int oldA, int oldB) {
    // (both halves of each register are written: the old contents only save a zeroing move)
    s16x2 a = __builtin_bit_cast(s16x2, oldA), b = __builtin_bit_cast(s16x2, oldB);
    a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(a, h2x{h[0], h[1]}, scale, false);
    a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(a, h2x{h[2], h[3]}, scale, true);
    b = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(b, h2x{h[4], h[5]}, scale, false);
    b = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(b, h2x{h[6], h[7]}, scale, true);
    return int2{__builtin_bit_cast(int, a), __builtin_bit_cast(int, b)};
  };
  auto convertStep = [&](int buf) {
    if constexpr(G::F8W) {
#pragma unroll
      for(int ct = 0; ct < G::NCT; ct++) {
        const int2 v = e4m3x8(bf[buf][ct], wScale, bq[ct][4 * buf + 2], bq[ct][4 * buf + 3]);
        bq[ct][4 * buf + 2] = v.x;
        bq[ct][4 * buf + 3] = v.y;
      }
    }
    if constexpr(G::F8X) {
#pragma unroll
      for(int t = 0; t < G::MAXT; t++) {
        const int2 v = e4m3x8(af[buf][t], 1.0f, aq[t][4 * buf], aq[t][4 * buf + 1]);
        aq[t][4 * buf] = v.x;
        aq[t][4 * buf + 1] = v.y;
      }
    }
  };
  auto f8pair = [&]() {
    // one scaled e4m3 MFMA over the pair of steps held in aq / bq
#pragma unroll
    for(int t = 0; t < G::MAXT; t++)
#pragma unroll
      for(int ct = 0; ct < G::NCT; ct++)
        acc[t][ct] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bq[ct], aq[t], acc[t][ct], 0, 0, 0, sA, 0,
                                                                       127);
  };
  tapAddr(0);
  loadStep(0, 0);
#pragma unroll
  for(int st = 0; st < STEPS; st++) {
    const int tap = st / NCB, cb = st - tap * NCB;
    const int chunk = tap / TPC;
    const bool chunkEnd = cb == NCB - 1 && (tap == NTAPS - 1 || (tap + 1) % TPC == 0);
    if(chunkEnd && chunk + 1 < NCH && !(DBG & 2)) {
      // retire this wave's pieces of chunk+1 (with three slots chunk+2's requests, at
      // least NW2 per wave, may stay in flight), publish them, free chunk's slot, request
      // chunk+R
      if constexpr(DBG & 32) {
      } else if constexpr(R == 3) {
        // (chunk is a constant after unrolling: one branch remains; the next conv's chunk
        // exists unless nextPieces / nextNCH say otherwise -- then nothing younger is in
        // flight and every request must be retired)
        static_assert(NTAPS % TPC == 0, "three-slot ring: whole chunks");
        if(chunk + 2 < NCH)
          waitVm<TPC * CH / G::NW>();
        else if(nextPieces > 0 && chunk + 2 - NCH < nextNCH)
          waitVm<NEXT_MIN>();
        else
          waitVm<0>();
      } else {
        waitVm<0>();
      }
      barrierKeepDma();
      request(chunk + R);
    }
    if constexpr(F8C) {
      convertStep(st & 1);  // this step's fragments were read in the previous iteration
      if((st & 1) && !(DBG & 4))
        f8pair();  // steps st - 1 (low halves) and st (high halves)
    }
    if(chunkEnd && chunk + 1 < NCH && (DBG & 2) && !(DBG & 1))
      request(chunk + R);  // ablation: the requests without their waits / barriers
    constexpr bool LATE = (F8C && KC_F8C_LATE) || (G::MODE == NN_MODE_SPLIT3 && G::BL && KC_ACC_LATE);
    if(!LATE && st + 1 < STEPS && !(DBG & 16)) {
      if(cb == NCB - 1)
        tapAddr(tap + 1);
      loadStep(st + 1, (st + 1) & 1);
    }
    // keep the next step's LDS reads ahead of this step's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    const int b = st & 1;
#pragma unroll
    for(int t = 0; t < G::MAXT; t++)
#pragma unroll
      for(int ct = 0; ct < G::NCT; ct++)
        acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[b][ct], af[b][t], acc[t][ct], 0, 0, 0);
    if constexpr(G::MODE == NN_MODE_SPLIT3) {
      // + lo(w) * hi(x), then + hi(w) * lo(x) (the other split kernels' order)
#pragma unroll
      for(int t = 0; t < G::MAXT; t++)
#pragma unroll
        for(int ct = 0; ct < G::NCT; ct++)
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bfl[b][ct], af[b][t], acc[t][ct], 0, 0, 0);
#pragma unroll
      for(int t = 0; t < G::MAXT; t++)
#pragma unroll
        for(int ct = 0; ct < G::NCT; ct++)
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[b][ct], afl[b][t], acc[t][ct], 0, 0, 0);
    }
    if(LATE && st + 1 < STEPS) {
      // the next step's fragments, read once this step's MFMAs are issued
      __builtin_amdgcn_sched_barrier(0);
      if(cb == NCB - 1)
        tapAddr(tap + 1);
      loadStep(st + 1, (st + 1) & 1);
    }
    if constexpr(F8C) {
      if(st == STEPS - 1 && !(st & 1) && !(DBG & 4)) {
        // an odd step count: the last step pairs with zeros (stale weights x 0)
#pragma unroll
        for(int t = 0; t < G::MAXT; t++)
          aq[t].hi = i32x4{0, 0, 0, 0};
        f8pair();
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// Copies a [96][rows] f32 matrix (a [rows][96] linear layer the host stored
// transposed; global, 16-B aligned) into LDS: consecutive output rows of one wave
// read consecutive banks in the dot-product loops.  16-byte stores, no conflicts.
template <int NT>
KC_D void stage96(float* __restrict__ dst, const float* __restrict__ src, int rows, int tid) {
  const int n4 = rows * 24;
  for(int q = tid; q < n4; q += NT)
    reinterpret_cast<float4*>(dst)[q] = reinterpret_cast<const float4*>(src)[q];
}

// The residual trunk is f32.  Between blocks it lives in the accumulators; while
// a block's first convolution owns them it is parked in a workgroup-private global
// scratch in accumulator-fragment order (1 KiB contiguous per wave and tile, an
// L2-resident round trip per block), so trained nets keep f32 trunk precision
// without the 24 VGPRs a register copy would cost.
template <class G>
KC_D f32x4* trunkBase(float* trunk, int wave, int lane) {
  return reinterpret_cast<f32x4*>(trunk) + ((size_t)blockIdx.x * G::NW + wave) * (G::MAXT * G::NCT * 64) + lane;
}
// With at most 2 x 3 accumulator tiles per wave (the small-batch instance: 185 VGPRs) the
// parked trunk fits in 24 more registers (< 256, no spill): kept in `reg`, no scratch.
template <class G>
constexpr bool regTrunk() {
  return G::MAXT * G::NCT <= 6 && !(G::MODE == NN_MODE_F8C && KC_F8C_PARK);
}
template <class G>
KC_D void storeTrunk(float* trunk, f32x4 (&reg)[G::MAXT][G::NCT], const f32x4 (&a)[G::MAXT][G::NCT], int wave,
                     int lane) {
  if(regTrunk<G>()) {
#pragma unroll
    for(int t = 0; t < G::MAXT; t++)
#pragma unroll
      for(int ct = 0; ct < G::NCT; ct++)
        reg[t][ct] = a[t][ct];
    return;
  }
  f32x4* p = trunkBase<G>(trunk, wave, lane);
#pragma unroll
  for(int t = 0; t < G::MAXT; t++)
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++)
      p[(t * G::NCT + ct) * 64] = a[t][ct];
}
template <class G>
KC_D void loadTrunk(f32x4 (&a)[G::MAXT][G::NCT], const f32x4 (&reg)[G::MAXT][G::NCT], float* trunk, int wave,
                    int lane) {
  if(regTrunk<G>()) {
#pragma unroll
    for(int t = 0; t < G::MAXT; t++)
#pragma unroll
      for(int ct = 0; ct < G::NCT; ct++)
        a[t][ct] = reg[t][ct];
    return;
  }
  const f32x4* p = trunkBase<G>(trunk, wave, lane);
#pragma unroll
  for(int t = 0; t < G::MAXT; t++)
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++)
      a[t][ct] = p[(t * G::NCT + ct) * 64];
}

template <class G>
KC_D void zeroAcc(f32x4 (&a)[G::MAXT][G::NCT]) {
#pragma unroll
  for(int t = 0; t < G::MAXT; t++)
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++)
      a[t][ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

// First of the 4 consecutive channels lane `lane` holds in column tile ct.
template <class G>
KC_D int chOf(int cg, int ct, int lane) {
  return cg * (G::C / 2) + ct * 16 + 4 * (lane >> 4);
}

KC_D uint2 packH4(float a, float b, float c, float d) {
  return uint2{(uint32_t)f16bits(a) | ((uint32_t)f16bits(b) << 16), (uint32_t)f16bits(c) | ((uint32_t)f16bits(d) << 16)};
}
// lo = fp16(x - f32(fp16(x))) of four values (SPLIT activations' second plane)
KC_D uint2 packH4lo(float a, float b, float c, float d) {
  auto lo = [](float x) { return x - (float)(_Float16)x; };
  return packH4(lo(a), lo(b), lo(c), lo(d));
}
// e4m3 (OCP e4m3fn, round to nearest even) of two values in the low (HI false) or high half
// of `old`: byte 0 / 2 = a, byte 1 / 3 = b; past 448 the conversion gives NaN (the epilogue
// flags the board: the accurate instance re-evaluates it)
template <bool HI>
KC_D int e4m3x2(float a, float b, int old) {
  return __builtin_amdgcn_cvt_pk_fp8_f32(a, b, old, HI);
}
// Corrected instance: boards of the lane's tile rows whose activations reached past e4m3's
// range (m[t] = the lane's largest |value| in tile t) are flagged in hot[base + board].
template <class G>
KC_D void flagHot(int* hot, int base, int nb, int tstart, int lane, const float (&m)[G::MAXT]) {
  if constexpr(G::MODE == NN_MODE_F8C) {
#pragma unroll
    for(int t = 0; t < G::MAXT; t++) {
      const int row = (tstart + t) * 16 + (lane & 15);
      if(!(m[t] <= F8C_MAX) && row < nb * G::A)  // rare; NaN counts as past the range
        __hip_atomic_store(hot + base + row / G::A, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
// Four activated channels of one row into act: the hi plane, and the second plane --
// fp16 lo (mode 1), or e4m3(lo(x) 2^11), one byte per channel (mode 2; e4m3(x) is
// converted from the hi plane's fp16 value inside the convolution).
template <class G>
KC_D void storeAct4(uint16_t* act, int row, int ch, float y0, float y1, float y2, float y3) {
  *reinterpret_cast<uint2*>(act + row * G::ASTR + ch) = packH4(y0, y1, y2, y3);
  if constexpr(G::MODE == NN_MODE_SPLIT3)
    *reinterpret_cast<uint2*>(act + G::PLANE_BYTES / 2 + row * G::ASTR + ch) = packH4lo(y0, y1, y2, y3);
  if constexpr(G::MODE == NN_MODE_F8C) {
    auto lo = [](float x) { return (x - (float)(_Float16)x) * F8C_SCALE; };
    if constexpr(G::F8X) {
      *reinterpret_cast<int*>(reinterpret_cast<char*>(act) + G::PLANE_BYTES + row * G::ROWB2 + ch) =
          e4m3x2<true>(lo(y2), lo(y3), e4m3x2<false>(lo(y0), lo(y1), 0));
    } else {
      // the channel octet's 16 bytes: [hi(x) of its 8 channels | lo(x) 2^11 of its 8 channels]
      auto hi = [](float x) { return (float)(_Float16)x; };
      char* q = reinterpret_cast<char*>(act) + G::PLANE_BYTES + row * G::ROWB + (ch >> 3) * 16 + (ch & 7);
      *reinterpret_cast<int*>(q) = e4m3x2<true>(hi(y2), hi(y3), e4m3x2<false>(hi(y0), hi(y1), 0));
      *reinterpret_cast<int*>(q + 8) = e4m3x2<true>(lo(y2), lo(y3), e4m3x2<false>(lo(y0), lo(y1), 0));
    }
  }
}
// BL: zero the shared zero row in every plane (after act was used as f32 scratch).
template <class G>
KC_D void zeroRowBL(uint16_t* act, int tid) {
  constexpr int N = G::ROWB / 16, N2 = G::SPLIT ? G::ROWB2 / 16 : 0;
  char* a = reinterpret_cast<char*>(act);
  if(tid < N)
    reinterpret_cast<uint4*>(a + G::ZROW * G::ROWB)[tid] = uint4{0u, 0u, 0u, 0u};
  else if(tid < N + N2)
    reinterpret_cast<uint4*>(a + G::PLANE_BYTES + G::ZROW * G::ROWB2)[tid - N] = uint4{0u, 0u, 0u, 0u};
}

// act[pad(row)][ch..ch+3] = f16(relu(v * s[ch] + b[ch])) for on-board rows, all channels.
template <class G, class V>
KC_D void storeBnRelu(uint16_t* act, const uint16_t* rowPa, const V (&v)[G::MAXT][G::NCT], const float* __restrict__ s,
                      const float* __restrict__ bb, int tstart, int cg, int lane, int* hot = nullptr, int base = 0,
                      int nb = 0) {
  float4 sc[G::NCT], bi[G::NCT];
#pragma unroll
  for(int ct = 0; ct < G::NCT; ct++) {
    const int ch = chOf<G>(cg, ct, lane);
    sc[ct] = *reinterpret_cast<const float4*>(s + ch);
    bi[ct] = *reinterpret_cast<const float4*>(bb + ch);
  }
  float m[G::MAXT];
#pragma unroll
  for(int t = 0; t < G::MAXT; t++) {
    m[t] = 0.0f;
    const int row = (tstart + t) * 16 + (lane & 15);
    if(row >= G::ROWS)
      continue;
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++) {
      const float y0 = fmaxf((float)v[t][ct][0] * sc[ct].x + bi[ct].x, 0.0f);
      const float y1 = fmaxf((float)v[t][ct][1] * sc[ct].y + bi[ct].y, 0.0f);
      const float y2 = fmaxf((float)v[t][ct][2] * sc[ct].z + bi[ct].z, 0.0f);
      const float y3 = fmaxf((float)v[t][ct][3] * sc[ct].w + bi[ct].w, 0.0f);
      storeAct4<G>(act, (int)rowPa[row], chOf<G>(cg, ct, lane), y0, y1, y2, y3);
      if constexpr(G::MODE == NN_MODE_F8C)
        m[t] = fmaxf(m[t], fmaxf(fmaxf(y0, y1), fmaxf(y2, y3)));  // >= 0 (ReLU)
    }
  }
  flagHot<G>(hot, base, nb, tstart, lane, m);
}

// Zero the border cells of every board (all channels) after act was used as f32
// scratch; 16-byte stores.
template <class G>
KC_D void zeroBorders(uint16_t* act, int tid) {
  constexpr int CH = G::ASTR / 8;  // 16-B chunks per row
  constexpr int NBORD = G::PA - G::A;
  for(int idx = tid; idx < G::NB * NBORD * CH; idx += G::NT) {
    const int q = idx / CH, c = idx - q * CH;
    const int b = q / NBORD, k = q - b * NBORD;
    // k-th border cell: top row, bottom row, then left/right columns
    int cell;
    if(k < G::PX)
      cell = k;
    else if(k < 2 * G::PX)
      cell = (G::PY - 1) * G::PX + (k - G::PX);
    else {
      const int m = k - 2 * G::PX;
      cell = (1 + (m >> 1)) * G::PX + ((m & 1) ? G::PX - 1 : 0);
    }
#pragma unroll
    for(int pl = 0; pl < G::PLANES; pl++)
      reinterpret_cast<uint4*>(act + pl * (G::PLANE_BYTES / 2) + (b * G::PA + cell) * G::ASTR)[c] = uint4{0u, 0u, 0u, 0u};
  }
}

// KataGPool over 32 f32 channels of scr ([b*A+p][SCR]) per board: mean,
// mean * (sqrt(A)-14)/10, max (model_pytorch.py:326-352); with vsrc also the value
// head's mean, mean * (sqrt(A)-14)/10, mean * ((sqrt(A)-14)^2/100 - 0.1).
// A lane pair per (board, channel), each summing half of the board's cells.
template <class G>
KC_D void poolBoards(const float* scr, const float* vsrc, float* poolP, float* poolV, float sqOff, int tid) {
  for(int idx = tid; idx < G::NB * 64; idx += G::NT) {
    const int pr = idx >> 1, half = idx & 1;
    const int b = pr >> 5, c = pr & 31;
    const int p0 = half ? (G::A + 1) / 2 : 0, p1 = half ? G::A : (G::A + 1) / 2;
    float s = 0.0f, m = 0.0f, sv = 0.0f;
#pragma unroll 4
    for(int p = p0; p < p1; p++) {
      const int o = (b * G::A + p) * G::SCR + c;
      const float v = scr[o];
      s += v;
      m = v > m ? v : m;
      if(vsrc)
        sv += vsrc[o];
    }
    s = s + asF(partner<5>(bitsF(s)));  // lane ^ 1 (DPP)
    m = fmaxf(m, asF(partner<5>(bitsF(m))));
    if(vsrc)
      sv = sv + asF(partner<5>(bitsF(sv)));
    if(half == 0) {
      const float mean = s / (float)G::A;
      poolP[b * 96 + c] = mean;
      poolP[b * 96 + 32 + c] = mean * (sqOff / 10.0f);
      poolP[b * 96 + 64 + c] = m;
      if(vsrc) {
        const float meanv = sv / (float)G::A;
        poolV[b * 96 + c] = meanv;
        poolV[b * 96 + 32 + c] = meanv * (sqOff / 10.0f);
        poolV[b * 96 + 64 + c] = meanv * ((sqOff * sqOff) / 100.0f - 0.1f);
      }
    }
  }
}

// out[b*ostr + o] = f(bias[o] + sum_i wT[i*O + o] * in[b*96 + i]) for every board,
// O % 4 == 0, wT staged transposed in LDS.  A lane owns 4 consecutive outputs and
// a quarter of the 96 inputs; the quarters are reduced across lanes.
// O = 32 or 64 (the gpool and value linears): lanes run over the outputs first, then
// the quarter, then the board, so each 16-lane ds_read_b128 group reads 16 consecutive
// float4 (conflict-free; quarter-major lanes put the 4 quarters of an output on one
// bank: 4-way conflicts) and the quarters, O/4 lanes apart, are reduced by DPP /
// permlane swaps -- in the same order, (q0 + q1) + (q2 + q3), as the fallback below.
template <class G>
KC_D void linear96(const float* wT, int O, const float* in, float* out, int ostr, const float* bias, bool relu,
                   int tid) {
  const int quads = O >> 2;
  auto dot = [&](int q, int ks, int b) {
    float4 s = float4{0.0f, 0.0f, 0.0f, 0.0f};
    const float* xi = in + b * 96 + ks * 24;
    const float* wi = wT + (ks * 24) * O + 4 * q;
#pragma unroll 4
    for(int i = 0; i < 24; i++) {
      const float4 w4 = *reinterpret_cast<const float4*>(wi + i * O);
      const float xv = xi[i];
      s.x += w4.x * xv;
      s.y += w4.y * xv;
      s.z += w4.z * xv;
      s.w += w4.w * xv;
    }
    return s;
  };
  auto emit = [&](const float4& s, int q, int b) {
    float r[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for(int j = 0; j < 4; j++) {
      float v = bias ? bias[4 * q + j] + r[j] : r[j];
      out[b * ostr + 4 * q + j] = relu ? fmaxf(v, 0.0f) : v;
    }
  };
  auto add2 = [](float& x, int lvl) {  // x += x of the lane 16 (lvl 1) / 32 (lvl 0) apart
    int a0, a1;
    if(lvl == 0)
      swapPair<0>(bitsF(x), a0, a1);
    else
      swapPair<1>(bitsF(x), a0, a1);
    x = asF(a0) + asF(a1);
  };
  if(quads == 16 || quads == 8) {
    const int per = 4 * quads;  // lanes per board: a whole wave (O 64) or half of one (O 32)
    for(int idx = tid; idx < G::NB * per; idx += G::NT) {
      const int q = idx & (quads - 1), ks = (idx / quads) & 3, b = idx / per;
      float4 s = dot(q, ks, b);
      if(quads == 16) {
        add2(s.x, 1);
        add2(s.y, 1);
        add2(s.z, 1);
        add2(s.w, 1);
        add2(s.x, 0);
        add2(s.y, 0);
        add2(s.z, 0);
        add2(s.w, 0);
      } else {
        s.x += asF(partner<2>(bitsF(s.x)));  // lane ^8 (row rotation by 8)
        s.y += asF(partner<2>(bitsF(s.y)));
        s.z += asF(partner<2>(bitsF(s.z)));
        s.w += asF(partner<2>(bitsF(s.w)));
        add2(s.x, 1);
        add2(s.y, 1);
        add2(s.z, 1);
        add2(s.w, 1);
      }
      if(ks == 0)
        emit(s, q, b);
    }
    return;
  }
  for(int idx = tid; idx < G::NB * quads * 4; idx += G::NT) {
    const int ks = idx & 3, q = (idx >> 2) % quads, b = (idx >> 2) / quads;
    float4 s = dot(q, ks, b);
    // quarters reduced over lanes ^1 then ^2 (DPP quad permutes)
    s.x += asF(partner<5>(bitsF(s.x)));
    s.y += asF(partner<5>(bitsF(s.y)));
    s.z += asF(partner<5>(bitsF(s.z)));
    s.w += asF(partner<5>(bitsF(s.w)));
    s.x += asF(partner<4>(bitsF(s.x)));
    s.y += asF(partner<4>(bitsF(s.y)));
    s.z += asF(partner<4>(bitsF(s.z)));
    s.w += asF(partner<4>(bitsF(s.w)));
    if(ks == 0)
      emit(s, q, b);
  }
}

// Element `tid` of parameter slab k: block k's BN1/BN2 scale+bias and gpool BN
// ([0,96) bn1s [96,192) bn1b [192,288) bn2s [288,384) bn2b [384,416) bngs
// [416,448) bngb), or for k == nblocks the tip BN and head biases ([0,96) tips
// [96,192) tipb [192,224) pBiasG [224,256) vBias1 [256,288) pBias2).  The slabs are
// gathered on the host (paramSlabSource), so this is one coalesced load: the per-thread
// source arithmetic it replaces stayed live across the block loop and, in the
// register-capped corrected instance, was spilled and reloaded behind the weight DMA.
KC_D float loadParam(const NNLayout* __restrict__ L, const float* __restrict__ WF, int k, int tid) {
  return tid < NN_PRM ? WF[L->prmSlabs + k * NN_PRM + tid] : 0.0f;
}
// Host: the f32 offset (in the weight image) of slab k's element `tid`, -1 for zero.
static int paramSlabSource(const NNLayout& L, int k, int tid) {
  const int f = tid < 384 ? tid / 96 : (tid < 416 ? 4 : 5), i = tid < 384 ? tid - 96 * f : (tid - 384) & 31;
  if(k < L.nblocks) {
    if(f == 0) return L.bn1s[k] + i;
    if(f == 1) return L.bn1b[k] + i;
    if(f == 2) return L.bn2s[k] + i;
    if(f == 3) return L.bn2b[k] + i;
    if(tid < NN_PRM && L.kinds[k] == 1) return (f == 4 ? L.bngs[k] : L.bngb[k]) + i;
    return -1;
  }
  if(tid >= 288) return -1;
  if(tid < 96) return L.tips + tid;
  if(tid < 192) return L.tipb + tid - 96;
  if(tid < 224) return L.pBiasG + tid - 192;
  if(tid < 256) return L.vBias1 + tid - 224;
  return L.pBias2 + tid - 256;
}

#ifndef KC_NN_KERNEL
#define KC_NN_KERNEL kNNForward
#define KC_NN_KERNEL_ATTR
#endif
template <int X, int Y, int C, int NB, int MODE, bool BL>
__global__ void __launch_bounds__(512, 2) KC_NN_KERNEL_ATTR
    KC_NN_KERNEL(const NNLayout* __restrict__ L, const h16x8* __restrict__ WB, const float* __restrict__ WF,
               const uint16_t* __restrict__ tabs, int n, const int* __restrict__ countDev,
               const int* __restrict__ rowIdx, int inWords, float winLen, const uint64_t* __restrict__ in,
               float* __restrict__ out, float* __restrict__ trunk, int* __restrict__ hot) {
  // hot (batch positions): the corrected instance flags boards with activations past e4m3's
  // range there; the split instance launched with it re-evaluates the workgroup's boards
  // only when one of them is flagged (and clears the flags), else exits at once
  using G = NNGeo<X, Y, C, NB, MODE, BL>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  NN_PHASE(0);
  const int count = countDev ? min(*countDev, n) : n;
  const int base = blockIdx.x * G::NB;
  if(base >= count)
    return;
  const int nb = min(G::NB, count - base);
  // split instance re-evaluating flagged boards: only those boards' outputs are written
  // (a row's logits stay a function of that row alone)
  uint32_t hotMask = ~0u;
  if(G::MODE == NN_MODE_SPLIT3 && hot) {
    hotMask = 0;
    for(int b = 0; b < nb; b++)
      hotMask |= __hip_atomic_load(hot + base + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 1u << b : 0u;
    if(!hotMask)
      return;  // uniform: every thread read the same flags
  }
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rg = wave >> 1, cg = wave & 1;
  const int tstart = rg * G::MAXT;
  uint16_t* act = reinterpret_cast<uint16_t*>(smem);
  float* actF = reinterpret_cast<float*>(smem);
  float* scr = reinterpret_cast<float*>(smem + G::SCR_OFF);
  float* poolP = reinterpret_cast<float*>(smem + G::OFF_POOL);
  float* poolV = poolP + G::NB * 96;
  float* biasS = reinterpret_cast<float*>(smem + G::OFF_BIAS);
  float* vh = reinterpret_cast<float*>(smem + G::OFF_W + G::RING_VH);  // heads only (ring idle)
  uint16_t* rowPa = reinterpret_cast<uint16_t*>(smem + G::OFF_TAB);  // [MROWS] padded cell of row
  uint16_t* rowBP = rowPa + G::MROWS;                                 // [MROWS] b*A+p (0xFFFF: padding)
  float* prm = reinterpret_cast<float*>(smem + G::OFF_PRM);  // [2][NPRM] parameter slabs
  h16x8* wl = reinterpret_cast<h16x8*>(smem + G::OFF_W);
  const float sqOff = sqrtf((float)G::A) - 14.0f;

  // the stem's first weight taps (as many as the ring prefetches) stream into the ring
  // while the input is unpacked
  {
    constexpr int CH0 = G::tapPieces(1);  // 1-KiB pieces per stem tap (one 32-channel block)
    const uint32_t ring = ldsAddr(wl);
    if constexpr(G::BL) {
      // the stem's chunks 0 .. RING-2 into slots 0 .. RING-2 (its chunks are whole: 3 or 9 taps)
      constexpr int SC = G::firstChunkPieces(1, 9);
#pragma unroll
      for(int j = 0; j + 1 < G::RING && j < G::chunks(1, 9); j++)
        stageChunk<G::NW>(WB + L->wInit + (size_t)j * SC * 64, ring + j * G::WSLOT * 16, SC, wave, lane);
    } else {
#pragma unroll
      for(int tap = 0; tap < 2; tap++)
        stageTapDma<G::NW>(WB + L->wInit + (size_t)tap * CH0 * 64, ring + tap * G::WSLOT * 16, CH0, wave, lane);
    }
  }
  // ---- row tables; unpack the packed V1 planes into the zero-bordered act ----
  constexpr int NPK = (G::NPRM + G::NT - 1) / G::NT;  // parameter-slab elements per thread
  float pre[NPK];
#pragma unroll
  for(int j = 0; j < NPK; j++)
    pre[j] = loadParam(L, WF, 0, tid + j * G::NT);  // block 0's slab, stored after the stem conv
  for(int i = tid; i < G::NTAB; i += G::NT)
    rowPa[i] = tabs[i];
  for(int idx = tid; idx < G::ACT_BYTES / 16; idx += G::NT)
    reinterpret_cast<uint4*>(smem)[idx] = uint4{0u, 0u, 0u, 0u};
  __syncthreads();
  {
    // wave w unpacks board w: its row index and all its packed words are loaded up
    // front (two round trips), then lane l sets bits l, l+64, ... (plane-major bits)
    static_assert(G::NB <= G::NW, "one wave per board");
    constexpr int NBITS = G::A * NUM_SPATIAL, NWD = (NBITS + 63) / 64;
    const int b = __builtin_amdgcn_readfirstlane(wave);
    if(b < nb) {
      const int src = rowIdx ? rowIdx[base + b] : base + b;
      uint64_t words[NWD];
#pragma unroll
      for(int k = 0; k < NWD; k++)
        words[k] = in[(size_t)src * inWords + k];
#pragma unroll
      for(int k = 0; k < NWD; k++) {
        const int i = k * 64 + lane;
        if(i < NBITS && ((words[k] >> lane) & 1ULL)) {
          const int c = i / G::A, p = i - c * G::A;
          const int row = G::BL ? b * G::A + p : padCell<G>(b, p);
          act[row * G::ASTR + c] = (uint16_t)0x3c00;  // 1.0 (its lo planes stay 0)
          if constexpr(G::MODE == NN_MODE_F8C && !G::F8X)  // e4m3 1.0 in the pair plane
            reinterpret_cast<uint8_t*>(act)[G::PLANE_BYTES + row * G::ROWB + (c >> 3) * 16 + (c & 7)] = 0x38;
        }
      }
    }
  }
  waitVm<0>();  // the stem's first taps (convTiles skips its entry barrier)
  __syncthreads();

  NN_PHASE(1);
  int ab[G::MAXT];
  int rb[G::MAXT];
  uint32_t vm[G::MAXT];
  if constexpr(G::BL)
    aRowsBL<G>(rb, vm, tstart, lane);
  else
    aBases<G>(ab, rowPa, tstart, lane);
  f32x4 acc[G::MAXT][G::NCT];  // the f32 residual trunk between blocks
  f32x4 park[G::MAXT][G::NCT];  // the trunk while a block's first conv owns acc (regTrunk)
  zeroAcc<G>(acc);
  if constexpr(G::BL)
    convTilesB<G, 9, 1, 0>(act, WB + L->wInit, wl, acc, rb, vm, cg, lane, tid,
                           L->nblocks > 0 ? WB + L->wConv1[0] : WB + L->wHead,
                           L->nblocks > 0 ? G::firstChunkPieces(G::C / 32, 9) : G::firstChunkPieces(G::C / 32, 1),
                           L->nblocks > 0 ? G::chunks(G::C / 32, 9) : 1, L->sInit);
  else
    convTiles<G, 9, 1, 0, 0, false>(act, WB + L->wInit, wl, acc, ab, cg, lane, tid,
                                    L->nblocks > 0 ? WB + L->wConv1[0] : WB + L->wHead, 3 * G::NCT_ALL * G::PLANES,
                                    L->nblocks > 0 ? 9 : 1, 0);
  {
    // + linear_global(input_global) broadcast (model_pytorch.py:1587-1589); gin == 1
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++) {
      const float4 g4 = *reinterpret_cast<const float4*>(WF + L->globInit + chOf<G>(cg, ct, lane));
#pragma unroll
      for(int t = 0; t < G::MAXT; t++) {
        acc[t][ct][0] += g4.x * winLen;
        acc[t][ct][1] += g4.y * winLen;
        acc[t][ct][2] += g4.z * winLen;
        acc[t][ct][3] += g4.w * winLen;
      }
    }
  }
  if(L->nblocks > 0)
    storeTrunk<G>(trunk, park, acc, wave, lane);
#pragma unroll
  for(int j = 0; j < NPK; j++)
    if(tid + j * G::NT < G::NPRM)
      prm[tid + j * G::NT] = pre[j];
  const int Cr = G::C - L->Cg;
  NN_PHASE(2);
  const int tidK = tid;
  for(int blk = 0; blk < L->nblocks; blk++) {
    // the wave index as a scalar (fewer long-lived VGPRs: the corrected instance's cap)
    const int tid = tidK;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int cg = wave & 1, tstart = (wave >> 1) * G::MAXT;
    // previous conv finished reading act; the parked trunk's stores (and the next
    // conv's weight requests) stay in flight behind the epilogue below
    barrierKeepDma();
    NN_PHASE(3 + 4 * blk);
    const float* P = prm + (blk & 1) * G::NPRM;
    storeBnRelu<G>(act, rowPa, acc, P, P + 96, tstart, cg, lane, hot, base, nb);
    waitVm<0>();
    __syncthreads();
    zeroAcc<G>(acc);
#pragma unroll
    for(int j = 0; j < NPK; j++)
      pre[j] = loadParam(L, WF, blk + 1, tid + j * G::NT);  // next slab: its latency hides behind conv1
    NN_PHASE(4 + 4 * blk);
    if constexpr(G::BL)
      // first chunk mod RING: stem 3 chunks, each block's convs 9 + 9 (a 64-channel tap is one
      // chunk too), so conv1 starts at 3 + 18 blk (1 mod 2, 0 mod 3) and conv2 at 12 + 18 blk (0)
      convTilesB<G, 9, G::C / 32, G::RING == 2 ? 1 : 0>(act, WB + L->wConv1[blk], wl, acc, rb, vm, cg, lane, tid,
                                                       WB + L->wConv2[blk],
                                                       L->kinds[blk] == 0 ? G::firstChunkPieces(3, 9)
                                                                          : G::firstChunkPieces(2, 9),
                                                       L->kinds[blk] == 0 ? G::chunks(3, 9) : G::chunks(2, 9),
                                                       L->sConv1[blk]);
    else
      convTiles<G, 9, G::C / 32, 1, 0, false>(act, WB + L->wConv1[blk], wl, acc, ab, cg, lane, tid,
                                              WB + L->wConv2[blk],
                                              (L->kinds[blk] == 0 ? 3 : 2) * G::NCT_ALL * G::PLANES, 9, 9 + 18 * blk);
#pragma unroll
    for(int j = 0; j < NPK; j++)
      if(tid + j * G::NT < G::NPRM)
        prm[((blk + 1) & 1) * G::NPRM + tid + j * G::NT] = pre[j];
    __syncthreads();
    NN_PHASE(5 + 4 * blk);
    const bool lastBlk = blk + 1 == L->nblocks;
    const h16x8* nextW = lastBlk ? WB + L->wHead : WB + L->wConv1[lastBlk ? 0 : blk + 1];
    const int nextTaps = lastBlk ? 1 : 9;
    if(L->kinds[blk] == 0) {
      // the parked trunk is requested before the epilogue, whose LDS work hides its latency
      f32x4 tr[G::MAXT][G::NCT];
      loadTrunk<G>(tr, park, trunk, wave, lane);
      storeBnRelu<G>(act, rowPa, acc, P + 192, P + 288, tstart, cg, lane, hot, base, nb);
#pragma unroll
      for(int t = 0; t < G::MAXT; t++)
#pragma unroll
        for(int ct = 0; ct < G::NCT; ct++)
          acc[t][ct] = tr[t][ct];
      waitVm<0>();
      __syncthreads();
      NN_PHASE(6 + 4 * blk);
      if constexpr(G::BL)
        convTilesB<G, 9, G::C / 32, 0>(act, WB + L->wConv2[blk], wl, acc, rb, vm, cg, lane, tid, nextW,
                                       G::firstChunkPieces(G::C / 32, nextTaps), G::chunks(G::C / 32, nextTaps),
                                       L->sConv2[blk]);
      else
        convTiles<G, 9, G::C / 32, 0, 0, false>(act, WB + L->wConv2[blk], wl, acc, ab, cg, lane, tid, nextW,
                                                3 * G::NCT_ALL * G::PLANES, nextTaps, 18 + 18 * blk);
      if(!lastBlk)
        storeTrunk<G>(trunk, park, acc, wave, lane);
    } else {
      // g branch: BN-ReLU into scr (f32, aliases the dead conv input), then
      // KataGPool per board (model_pytorch.py:326-352)
      const float* gs = P + 384;
      const float* gbias = P + 416;
      // the gpool linear weights ([96][Cr] f32) are requested now and land in LDS
      // after the epilogue's barrier
      constexpr int LW = (96 * 64 / 4 + G::NT - 1) / G::NT;  // float4 per thread (Cr <= 64)
      float4 lw[LW];
      {
        const float4* src = reinterpret_cast<const float4*>(WF + L->linG[blk]);
#pragma unroll
        for(int k = 0; k < LW; k++) {
          const int q = tid + k * G::NT;
          lw[k] = q < Cr * 24 ? src[q] : float4{0.0f, 0.0f, 0.0f, 0.0f};
        }
      }
#pragma unroll
      for(int ct = 0; ct < G::NCT; ct++) {
        const int ch = chOf<G>(cg, ct, lane);
        if(cg * (G::C / 2) + ct * 16 < Cr)
          continue;
        const int gc = ch - Cr;
        const float4 sc = *reinterpret_cast<const float4*>(gs + gc);
        const float4 bi = *reinterpret_cast<const float4*>(gbias + gc);
#pragma unroll
        for(int t = 0; t < G::MAXT; t++) {
          const int row = (tstart + t) * 16 + (lane & 15);
          if(row >= G::ROWS)
            continue;
          *reinterpret_cast<float4*>(scr + (int)rowBP[row] * G::SCR + gc) =
              float4{fmaxf(acc[t][ct][0] * sc.x + bi.x, 0.0f), fmaxf(acc[t][ct][1] * sc.y + bi.y, 0.0f),
                     fmaxf(acc[t][ct][2] * sc.z + bi.z, 0.0f), fmaxf(acc[t][ct][3] * sc.w + bi.w, 0.0f)};
        }
      }
      __syncthreads();
      NN_PHASE(50);
      float* lgT = actF;  // transposed linear weights in the idle front of act
#pragma unroll
      for(int k = 0; k < LW; k++) {
        const int q = tid + k * G::NT;
        if(q < Cr * 24)
          reinterpret_cast<float4*>(lgT)[q] = lw[k];
      }
      poolBoards<G>(scr, nullptr, poolP, poolV, sqOff, tid);
      __syncthreads();
      NN_PHASE(51);
      linear96<G>(lgT, Cr, poolP, biasS, Cr, nullptr, false, tid);
      __syncthreads();
      f32x4 tr[G::MAXT][G::NCT];  // the parked trunk, in flight during the epilogue
      loadTrunk<G>(tr, park, trunk, wave, lane);
      if constexpr(G::BL)
        zeroRowBL<G>(act, tid);  // the f32 scratch overwrote the zero row
      else
        zeroBorders<G>(act, tid);  // the f32 scratch overwrote border cells (disjoint from r-epi cells)
      NN_PHASE(52);
      {
        // r branch + gpool bias -> BN2-ReLU -> f16 act (channels < Cr)
        const float* s2 = P + 192;
        const float* b2 = P + 288;
        float m[G::MAXT] = {};
#pragma unroll
        for(int ct = 0; ct < G::NCT; ct++) {
          if(cg * (G::C / 2) + ct * 16 >= Cr)
            continue;
          const int ch = chOf<G>(cg, ct, lane);
          const float4 sc = *reinterpret_cast<const float4*>(s2 + ch);
          const float4 bi = *reinterpret_cast<const float4*>(b2 + ch);
#pragma unroll
          for(int t = 0; t < G::MAXT; t++) {
            const int row = (tstart + t) * 16 + (lane & 15);
            if(row >= G::ROWS)
              continue;
            const float4 gb = *reinterpret_cast<const float4*>(biasS + ((int)rowBP[row] / G::A) * Cr + ch);
            const float y0 = fmaxf((acc[t][ct][0] + gb.x) * sc.x + bi.x, 0.0f);
            const float y1 = fmaxf((acc[t][ct][1] + gb.y) * sc.y + bi.y, 0.0f);
            const float y2 = fmaxf((acc[t][ct][2] + gb.z) * sc.z + bi.z, 0.0f);
            const float y3 = fmaxf((acc[t][ct][3] + gb.w) * sc.w + bi.w, 0.0f);
            storeAct4<G>(act, (int)rowPa[row], ch, y0, y1, y2, y3);
            if constexpr(G::MODE == NN_MODE_F8C)
              m[t] = fmaxf(m[t], fmaxf(fmaxf(y0, y1), fmaxf(y2, y3)));
          }
        }
        flagHot<G>(hot, base, nb, tstart, lane, m);
      }
#pragma unroll
      for(int t = 0; t < G::MAXT; t++)
#pragma unroll
        for(int ct = 0; ct < G::NCT; ct++)
          acc[t][ct] = tr[t][ct];
      waitVm<0>();
      __syncthreads();
      NN_PHASE(6 + 4 * blk);
      if constexpr(G::BL)
        convTilesB<G, 9, (G::C - 32) / 32, 0>(act, WB + L->wConv2[blk], wl, acc, rb, vm, cg, lane, tid, nextW,
                                              G::firstChunkPieces(G::C / 32, nextTaps),
                                              G::chunks(G::C / 32, nextTaps), L->sConv2[blk]);
      else
        convTiles<G, 9, (G::C - 32) / 32, 0, 0, false>(act, WB + L->wConv2[blk], wl, acc, ab, cg, lane, tid, nextW,
                                                       3 * G::NCT_ALL * G::PLANES, nextTaps, 18 + 18 * blk);
      if(!lastBlk)
        storeTrunk<G>(trunk, park, acc, wave, lane);
    }
  }
  // ---- trunk tip ----
  __syncthreads();
  NN_PHASE(40);
  const float* PT = prm + (L->nblocks & 1) * G::NPRM;  // tip slab
  storeBnRelu<G>(act, rowPa, acc, PT, PT + 96, tstart, cg, lane, hot, base, nb);
  waitVm<0>();
  __syncthreads();
  // ---- heads: one 1x1 conv C -> [p1 | g1 | v1] ----
  zeroAcc<G>(acc);
  if constexpr(G::BL)
    convTilesB<G, 1, G::C / 32, G::RING == 2 ? 1 : 0>(act, WB + L->wHead, wl, acc, rb, vm, cg, lane, tid, nullptr, 0,
                                                      0, L->sHead);
  else
    convTiles<G, 1, G::C / 32, 1, 0, false>(act, WB + L->wHead, wl, acc, ab, cg, lane, tid, nullptr, 0, 0,
                                            9 + 18 * L->nblocks);
  __syncthreads();  // act dead from here: f32 [MROWS][SCR] value branch at actF, g branch at scr
  NN_PHASE(41);
  {
    const float* pbg = PT + 192;
    const float* vb1 = PT + 224;
#pragma unroll
    for(int ct = 0; ct < G::NCT; ct++) {
      const int c0 = cg * (G::C / 2) + ct * 16;
      if(c0 < 32)
        continue;
      const bool isG = c0 < 64;
      const int hc = chOf<G>(cg, ct, lane) - (isG ? 32 : 64);
      const float4 bi = *reinterpret_cast<const float4*>((isG ? pbg : vb1) + hc);
      float* dst = isG ? scr : actF;
#pragma unroll
      for(int t = 0; t < G::MAXT; t++) {
        const int row = (tstart + t) * 16 + (lane & 15);
        if(row >= G::ROWS)
          continue;
        *reinterpret_cast<float4*>(dst + (int)rowBP[row] * G::SCR + hc) =
            float4{fmaxf(acc[t][ct][0] + bi.x, 0.0f), fmaxf(acc[t][ct][1] + bi.y, 0.0f),
                   fmaxf(acc[t][ct][2] + bi.z, 0.0f), fmaxf(acc[t][ct][3] + bi.w, 0.0f)};
      }
    }
  }
  __syncthreads();
  NN_PHASE(53);
  float* plgT = reinterpret_cast<float*>(wl);
  float* l2T = plgT + 32 * 96;
  // value / misc output weights [4][v2], then their 4 biases: in the idle parameter slab
  float* w3 = prm + ((L->nblocks + 1) & 1) * G::NPRM;
  static_assert(4 * 64 + 4 <= G::NPRM, "value weights fit a parameter slab");
  stage96<G::NT>(plgT, WF + L->pLinG, 32, tid);
  stage96<G::NT>(l2T, WF + L->vLin2, L->v2, tid);
  {
    const int v2 = L->v2;
    for(int i = tid; i < 4 * v2 + 4; i += G::NT) {
      float w;
      if(i < 2 * v2)
        w = WF[L->vLin3 + i];
      else if(i < 4 * v2)
        w = WF[L->vLinM + i - 2 * v2];
      else
        w = i - 4 * v2 < 2 ? WF[L->vB3 + i - 4 * v2] : WF[L->vBM + i - 4 * v2 - 2];
      w3[i] = w;
    }
  }
  poolBoards<G>(scr, actF, poolP, poolV, sqOff, tid);
  __syncthreads();
  NN_PHASE(54);
  linear96<G>(plgT, 32, poolP, biasS, 32, nullptr, false, tid);
  linear96<G>(l2T, L->v2, poolV, vh, 64, WF + L->vB2, true, tid);
  __syncthreads();
  {
    // value (2) and misc (2) outputs: a 16-lane group per (board, output), each lane
    // summing every 16th term, reduced across the group
    static_assert(G::NB * 4 * 16 <= G::NT, "one 16-lane group per (board, output)");
    const int k = tid & 15, o = (tid >> 4) & 3, b = tid >> 6;
    const int v2 = L->v2;
    const int bv = b < G::NB ? b : 0;  // waves past the boards compute a discarded copy
    float s = 0.0f;
    for(int i = k; i < v2; i += 16)
      s += w3[o * v2 + i] * vh[bv * 64 + i];
    // lanes ^8, ^4, ^2, ^1 of the 16-lane group (DPP; after ^8 a partial depends only
    // on lane mod 8, so the row rotation by 4 reaches the ^4 partner's value)
    s += asF(partner<2>(bitsF(s)));
    s += asF(partner<3>(bitsF(s)));
    s += asF(partner<4>(bitsF(s)));
    s += asF(partner<5>(bitsF(s)));
    if(k == 0 && b < nb && ((hotMask >> b) & 1u)) {
      const int dst = rowIdx ? rowIdx[base + b] : base + b;
      out[(size_t)dst * (G::P + 4) + G::P + o] = s + w3[4 * v2 + o];
    }
  }
  NN_PHASE(42);
  if(cg == 0) {
    // policy: relu(p + gpool bias + bias2) -> 1x1 conv p1 -> 4 direction logits.
    // Channels 0..31 live in column tiles 0 and 1: 8 per lane, reduced over the
    // four lane groups (lane >> 4).
    const float* pb2 = PT + 256;
    const float* w2 = WF + L->pConv2;
    const int c0 = chOf<G>(0, 0, lane), c1 = chOf<G>(0, 1, lane);
#pragma unroll
    for(int t = 0; t < G::MAXT; t++) {
      const int row = (tstart + t) * 16 + (lane & 15);
      const int bp = row < G::ROWS ? (int)rowBP[row] : 0;
      const int brd = bp / G::A;
      float pv[8];
#pragma unroll
      for(int j = 0; j < 4; j++) {
        pv[j] = fmaxf(acc[t][0][j] + biasS[brd * 32 + c0 + j] + pb2[c0 + j], 0.0f);
        pv[4 + j] = fmaxf(acc[t][1][j] + biasS[brd * 32 + c1 + j] + pb2[c1 + j], 0.0f);
      }
      float part[4];
#pragma unroll
      for(int d = 0; d < 4; d++) {
        float s = 0.0f;
#pragma unroll
        for(int j = 0; j < 4; j++)
          s += pv[j] * w2[d * 32 + c0 + j] + pv[4 + j] * w2[d * 32 + c1 + j];
        {
          int a0, a1;  // lanes ^16 then ^32 (permlane swaps)
          swapPair<1>(bitsF(s), a0, a1);
          s = asF(a0) + asF(a1);
          swapPair<0>(bitsF(s), a0, a1);
          s = asF(a0) + asF(a1);
        }
        part[d] = s;
      }
      if((lane >> 4) == 0 && row < G::ROWS && brd < nb && ((hotMask >> brd) & 1u)) {
        const int pp = bp - brd * G::A;
        float* o = out + (size_t)(rowIdx ? rowIdx[base + brd] : base + brd) * (G::P + 4);
#pragma unroll
        for(int d = 0; d < 4; d++)
          o[d * G::A + pp] = part[d];
      }
    }
  }
  if(G::MODE == NN_MODE_SPLIT3 && hot && tid < nb)
    hot[base + tid] = 0;  // this workgroup re-evaluated its boards (one was flagged)
}

#ifndef KC_NN_KERNEL_ONLY
#if KC_F8C_VGPR
// the register-capped corrected instance (nn_corr.hip)
template <int X, int Y, int C, int NB, int MODE, bool BL>
__global__ void kNNForwardCap(const NNLayout* __restrict__ L, const h16x8* __restrict__ WB,
                              const float* __restrict__ WF, const uint16_t* __restrict__ tabs, int n,
                              const int* __restrict__ countDev, const int* __restrict__ rowIdx, int inWords,
                              float winLen, const uint64_t* __restrict__ in, float* __restrict__ out,
                              float* __restrict__ trunk, int* __restrict__ hot);
#endif
template <class G>
constexpr auto nnKernel() {
#if KC_F8C_VGPR
  if constexpr(G::MODE == NN_MODE_F8C || (G::MODE == NN_MODE_F16 && G::BL) ||
               (KC_ACC_CAP && G::MODE == NN_MODE_SPLIT3 && G::BL))
    return kNNForwardCap<G::X, G::Y, G::C, G::NB, G::MODE, G::BL>;
  else
#endif
    return kNNForward<G::X, G::Y, G::C, G::NB, G::MODE, G::BL>;
}

// ---------------------------------------------------------------------------
// Host: pack weights into B-fragment order and launch.

// float -> IEEE binary16 bits, round to nearest even (weights; saturates to inf).
static uint16_t f2h(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u, a = u & 0x7fffffffu;
  if(a >= 0x7f800000u)
    return (uint16_t)(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));
  if(a < 0x38800000u) {  // subnormal half: quantum 2^-24
    float m;
    memcpy(&m, &a, 4);
    return (uint16_t)(sign | (uint32_t)nearbyintf(m * 16777216.0f));
  }
  uint32_t r = a + 0xfffu + ((a >> 13) & 1u);
  if(r >= 0x47800000u)
    return (uint16_t)(sign | 0x7c00u);
  return (uint16_t)(sign | (((r >> 23) - 112u) << 10) | ((r >> 13) & 0x3ffu));
}

// B fragment order for one conv: [kstep = tap*NCB + cb][coltile][lane][8],
// element = W(co = ct*16 + (lane&15), cin = cb*32 + 8*(lane>>4) + j, tap).
// IEEE binary16 bits -> float (exact).
static float h2f(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  float f;
  if(e == 0) {
    f = ldexpf((float)m, -24);
  } else if(e == 31) {
    const uint32_t u = 0x7f800000u | (m << 13);
    memcpy(&f, &u, 4);
  } else {
    const uint32_t u = ((e + 112u) << 23) | (m << 13);
    memcpy(&f, &u, 4);
  }
  uint32_t u;
  memcpy(&u, &f, 4);
  u |= sign;
  memcpy(&f, &u, 4);
  return f;
}

// float -> OCP e4m3fn (bias 7, max 448), round to nearest even, saturating at +-448
// (the device's e4m3x2 on activations).
static uint8_t f2e4m3(float f) {
  const uint8_t sign = std::signbit(f) ? 0x80 : 0x00;
  const float a = std::fabs(f);
  if(!(a < 448.0f))
    return sign | 0x7e;
  if(a < 0.015625f)  // below 2^-6: subnormal, quantum 2^-9 (a carry into 0x08 is 2^-6 itself)
    return sign | (uint8_t)std::nearbyint(a * 512.0f);
  int e;
  const float m = std::frexp(a, &e);  // a = m 2^e, m in [0.5, 1)
  int q = (int)std::nearbyint((m * 2.0f - 1.0f) * 8.0f);
  int E = e - 1;
  if(q == 8) {
    q = 0;
    E++;
  }
  if(E + 7 > 15 || (E + 7 == 15 && q == 7))
    return sign | 0x7e;
  return sign | (uint8_t)(((E + 7) << 3) | q);
}

// mode 1: after each tap's hi fragments the same fragments of lo = fp16(w - hi);
// mode 2: after them e4m3(lo(w) 2^(11-sw)) of each fragment's 8 k, 8 bytes per lane (512 B
// per fragment; e4m3(hi(w) 2^-sw) is converted from the hi fragment on the device), sw the
// conv's block exponent (f8Exp of its largest |w|), and *sA = the A operand's E8M0 scale
// byte, 127 - 11 + sw (convTiles' / convTilesB's SPLIT ring slot layout).
static void packConv(std::vector<uint16_t>& dst, int ntaps, int cinPad, int cout,
                     const std::function<float(int, int, int)>& W, int mode = NN_MODE_F16, int* sA = nullptr) {
  const int ncb = cinPad / 32, nct = cout / 16;
  int sw = 0;
  if(mode == NN_MODE_F8C) {
    float mx = 0.0f;
    for(int co = 0; co < cout; co++)
      for(int tap = 0; tap < ntaps; tap++)
        for(int ci = 0; ci < cinPad; ci++)
          mx = std::max(mx, std::fabs(W(co, ci, tap)));
    sw = f8Exp(mx);
    if(sA)
      *sA = 127 - F8C_SHIFT + sw;
  }
  for(int tap = 0; tap < ntaps; tap++)
    for(int part = 0; part < (mode != NN_MODE_F16 ? 2 : 1); part++)
      for(int cb = 0; cb < ncb; cb++)
        for(int ct = 0; ct < nct; ct++)
          for(int l = 0; l < 64; l++) {
            float w[8];
            for(int j = 0; j < 8; j++)
              w[j] = W(ct * 16 + (l & 15), cb * 32 + 8 * (l >> 4) + j, tap);
            if(part == 0 || mode == NN_MODE_SPLIT3) {
              for(int j = 0; j < 8; j++) {
                const uint16_t hi = f2h(w[j]);
                dst.push_back(part == 0 ? hi : f2h(w[j] - h2f(hi)));
              }
            } else if(KC_F8C_CVTW) {
              uint8_t b[8];
              for(int j = 0; j < 8; j++)
                b[j] = f2e4m3(ldexpf((w[j] - h2f(f2h(w[j]))) * F8C_SCALE, -sw));
              for(int j = 0; j < 4; j++)
                dst.push_back((uint16_t)(b[2 * j] | (b[2 * j + 1] << 8)));
            } else {
              uint8_t b[16];
              for(int j = 0; j < 8; j++) {
                b[j] = f2e4m3(ldexpf((w[j] - h2f(f2h(w[j]))) * F8C_SCALE, -sw));
                b[8 + j] = f2e4m3(ldexpf(h2f(f2h(w[j])), -sw));
              }
              for(int j = 0; j < 8; j++)
                dst.push_back((uint16_t)(b[2 * j] | (b[2 * j + 1] << 8)));
            }
          }
}

// Output-row order of a workgroup's NB boards: row r takes a cell whose padded
// LDS row is congruent to r mod 8 where possible.  With 224-byte activation rows
// the 16 lanes of each ds_read_b128 lane group then hit 16 distinct 16-byte bank
// slots (rows {0-3,12-15} and {4-11} of a tile each cover all residues).
template <class G>
static std::vector<uint16_t> rowTables() {
  std::vector<uint16_t> tab(G::NTAB, 0);
  uint16_t* rowPa = tab.data();
  uint16_t* rowBP = rowPa + G::MROWS;
  uint16_t* bpRow = rowBP + G::MROWS;
  if(G::BL) {  // borderless: output row r is activation row r, position r
    for(int r = 0; r < G::MROWS; r++) {
      rowPa[r] = (uint16_t)(r < G::ROWS ? r : G::ZROW);
      rowBP[r] = (uint16_t)(r < G::ROWS ? r : 0xFFFF);
    }
    for(int r = 0; r < G::ROWS; r++)
      bpRow[r] = (uint16_t)r;
    return tab;
  }
  std::vector<std::vector<int>> bucket(8);
  for(int b = 0; b < G::NB; b++)
    for(int p = 0; p < G::A; p++) {
      const int pa = b * G::PA + (p / G::X + 1) * G::PX + p % G::X + 1;
      bucket[pa % 8].push_back(b * G::A + p);
    }
  std::vector<size_t> next(8, 0);
  for(int r = 0; r < G::ROWS; r++) {
    int m = r % 8;
    for(int k = 0; k < 8 && next[m] >= bucket[m].size(); k++)
      m = (m + 1) % 8;
    const int bp = bucket[m][next[m]++];
    const int b = bp / G::A, p = bp % G::A;
    rowPa[r] = (uint16_t)(b * G::PA + (p / G::X + 1) * G::PX + p % G::X + 1);
    rowBP[r] = (uint16_t)bp;
    bpRow[bp] = (uint16_t)r;
  }
  for(int r = G::ROWS; r < G::MROWS; r++) {
    rowPa[r] = rowPa[0];
    rowBP[r] = 0xFFFF;
  }
  return tab;
}

bool NNEngine::fusedSupported(const ModelCfg& c, int X, int Y) {
  for(int k : c.kinds)
    if(k > 1)
      return false;
  return X == 5 && Y == 5 && c.C == 96 && c.Cg == 32 && c.p1 == 32 && c.g1 == 32 && c.v1 == 32 && c.v2 <= 64 && c.v2 % 4 == 0 &&
         c.cin == NUM_SPATIAL && c.gin == 1 && (int)c.kinds.size() <= NN_MAX_BLOCKS;
}

// Calibration positions of the default precision's check: n positions of seeded uniform
// random legal play from the empty board (position i after i % (A + 1) moves, or fewer if
// the game ends), symmetry i % 8, encoded on the device (kEncodeBatch).
static void calibrationBatch(int X, int Y, int W, int n, uint64_t* packedDev, hipStream_t st) {
  const DTables& T = hostTables(X, Y, W);
  const int A = X * Y;
  std::vector<uint8_t> cells((size_t)n * A), pla(n);
  std::vector<int8_t> hc((size_t)n * HIST), hd((size_t)n * HIST);
  std::vector<int32_t> sym(n);
  uint64_t rng = 0x243f6a8885a308d3ULL;
  auto next = [&]() {
    rng = rng * 6364136223846793005ULL + 1442695040888963407ULL;
    return (uint32_t)(rng >> 33);
  };
  for(int i = 0; i < n; i++) {
    DBoard b;
    boardInit(T, b);
    for(int k = 0; k < i % (A + 1) && !b.finished; k++) {
      int legal[4 * MAX_AREA], nl = 0;
      for(int c = 0; c < A; c++)
        for(int d = 0; d < 4; d++)
          if(isLegal(T, b, c, d))
            legal[nl++] = d * A + c;
      if(nl == 0)
        break;
      const int mv = legal[next() % nl];
      playMoveSerial(T, b, mv % A, mv / A);
    }
    for(int c = 0; c < A; c++)
      cells[(size_t)i * A + c] = (uint8_t)colorAt(b, c);
    for(int h = 0; h < HIST; h++) {
      hc[(size_t)i * HIST + h] = (int8_t)hCell(b, h);
      hd[(size_t)i * HIST + h] = (int8_t)hDir(b, h);
    }
    pla[i] = (uint8_t)b.pla;
    sym[i] = i % 8;
  }
  void* buf = nullptr;
  const size_t bytes = cells.size() + pla.size() + hc.size() + hd.size() + sym.size() * 4;
  KC_HIP(hipMalloc(&buf, bytes));
  char* p = static_cast<char*>(buf);
  auto up = [&](const void* src, size_t len) {
    KC_HIP(hipMemcpy(p, src, len, hipMemcpyHostToDevice));
    char* at = p;
    p += len;
    return at;
  };
  int32_t* symD = reinterpret_cast<int32_t*>(up(sym.data(), sym.size() * 4));
  uint8_t* cellsD = reinterpret_cast<uint8_t*>(up(cells.data(), cells.size()));
  int8_t* hcD = reinterpret_cast<int8_t*>(up(hc.data(), hc.size()));
  int8_t* hdD = reinterpret_cast<int8_t*>(up(hd.data(), hd.size()));
  uint8_t* plaD = reinterpret_cast<uint8_t*>(up(pla.data(), pla.size()));
  launchEncodeBatch(deviceTables(X, Y, W), n, cellsD, hcD, hdD, plaD, symD, packedDev, nullptr, st);
  KC_HIP(hipStreamSynchronize(st));
  (void)hipFree(buf);
}

// Largest |logit| difference between this engine and `ref` on the calibration batch, and
// (corrected instance) how many of its boards had activations past e4m3's range.
float NNEngine::calibrationError(NNEngine& ref, int* hotBoards) {
  constexpr int n = 256;
  const int inWords = (NUM_SPATIAL * X_ * Y_ + 63) / 64, P = 4 * X_ * Y_;
  uint64_t* in = nullptr;
  float* out = nullptr;
  KC_HIP(hipMalloc(&in, (size_t)n * inWords * 8));
  KC_HIP(hipMalloc(&out, (size_t)2 * n * (P + 4) * 4));
  float err = 0.0f;
  try {
    calibrationBatch(X_, Y_, W_, n, in, nullptr);
    if(mode_ == NN_CORRECTED) {
      // the corrected kernel alone first: the boards it flags (the re-evaluation clears them)
      fallback_ = false;
      forward(n, in, out, nullptr);
      fallback_ = true;
      std::vector<int> h(n);
      KC_HIP(hipMemcpy(h.data(), hot_, (size_t)n * 4, hipMemcpyDeviceToHost));
      *hotBoards = 0;
      for(int v : h)
        *hotBoards += v != 0;
      KC_HIP(hipMemset(hot_, 0, (size_t)n * 4));
    }
    forward(n, in, out, nullptr);
    ref.forward(n, in, out + (size_t)n * (P + 4), nullptr);
    std::vector<float> h((size_t)2 * n * (P + 4));
    KC_HIP(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
    for(size_t i = 0; i < h.size() / 2; i++)
      err = std::max(err, std::fabs(h[i] - h[i + h.size() / 2]));
    if(!std::isfinite(err))
      err = INFINITY;
  } catch(...) {
    (void)hipFree(in);
    (void)hipFree(out);
    throw;
  }
  (void)hipFree(in);
  (void)hipFree(out);
  return err;
}

NNEngine::NNEngine(const ModelHost& m, int X, int Y, int W, int path) : cfg_(m.cfg), X_(X), Y_(Y), W_(W) {
  flops_ = modelFlopsPerEval(cfg_, X * Y);
  if(path < NN_DEFAULT || path > NN_FAST)
    throw std::invalid_argument("NNEngine: unknown precision/path");
  // a constructor that throws runs no destructor: whatever build() or the calibration
  // allocated before the failure is released here (this path also runs on every hot reload)
  try {
    if(path != NN_DEFAULT) {
      build(m, path);
      return;
    }
    // the default (north-star 1e-3) precision: the corrected instance, unless on the
    // calibration batch its logits differ from the accurate (split) instance's by more than
    // NN_AUTO_TOL or any board needs the re-evaluation (activations past e4m3's range) --
    // corrected products are good to ~2^-14 relative, which deep-trained nets with large
    // logits push towards 1e-3; the split path is good to ~2^-21
    build(m, NN_CORRECTED);
    if(layered_)
      return;  // the layered kernels run "corrected" as the split path already
    int hotBoards = 0;
    calibErr_ = calibrationError(*fallbackNet_, &hotBoards);
    if(!(calibErr_ <= NN_AUTO_TOL) || hotBoards > 0) {
      release();
      build(m, NN_ACCURATE);
    }
  } catch(...) {
    release();
    throw;
  }
}

void NNEngine::build(const ModelHost& m, int path) {
  const int X = X_, Y = Y_, W = W_;
  if(path == NN_FAST_LAYERED || !fusedSupported(m.cfg, X, Y)) {
    // the layered kernels have fp16 and hi/lo split operands; corrected maps to split
    layered_.reset(new NNLayered(m, X, Y, W, path != NN_FAST && path != NN_FAST_LAYERED));
    return;
  }
  mode_ = path;
  if(path == NN_CORRECTED)  // the re-evaluation of boards past e4m3's range (forward)
    fallbackNet_.reset(new NNEngine(m, X, Y, W, NN_ACCURATE));
  // the fused kernel's operand mode: fp16, fp16 hi/lo pairs (accurate: the borderless
  // 5-board instance, or the 2-board one for A/B), fp16 + e4m3 cross terms (corrected)
  const int wmode = path == NN_CORRECTED ? NN_MODE_F8C : (path == NN_FAST ? NN_MODE_F16 : NN_MODE_SPLIT3);
  const int C = cfg_.C, Cr = C - cfg_.Cg;
  std::vector<uint16_t> wb;
  std::vector<float> wf;
  NNLayout& L = layout_;
  memset(&L, 0, sizeof(L));
  L.nblocks = (int)cfg_.kinds.size();
  L.C = C; L.Cg = cfg_.Cg; L.p1 = cfg_.p1; L.g1 = cfg_.g1; L.v1 = cfg_.v1; L.v2 = cfg_.v2;
  auto f32 = [&](const std::vector<float>& v) {
    int off = (int)wf.size();
    wf.insert(wf.end(), v.begin(), v.end());
    while(wf.size() % 4)
      wf.push_back(0.0f);
    return off;
  };
  // a [rows][96] linear layer stored transposed ([96][rows]): the kernel copies it
  // into LDS as is (stage96), the layout its dot products read
  auto f32T = [&](const std::vector<float>& v, int rows) {
    std::vector<float> t(v.size());
    for(int r = 0; r < rows; r++)
      for(int i = 0; i < 96; i++)
        t[(size_t)i * rows + r] = v[(size_t)r * 96 + i];
    return f32(t);
  };
  auto bfOff = [&]() { return (int)(wb.size() / 8); };
  L.wInit = bfOff();
  packConv(wb, 9, 32, C, [&](int co, int ci, int tap) {
    return ci < cfg_.cin ? m.convInit[((size_t)co * cfg_.cin + ci) * 9 + tap] : 0.0f;
  }, wmode, &L.sInit);
  L.globInit = f32(m.globInit);
  for(int i = 0; i < L.nblocks; i++) {
    const ModelBlock& b = m.blocks[i];
    L.kinds[i] = b.kind;
    L.bn1s[i] = f32(b.bn1s);
    L.bn1b[i] = f32(b.bn1b);
    L.wConv1[i] = bfOff();
    if(b.kind == 0) {
      packConv(wb, 9, C, C, [&](int co, int ci, int tap) { return b.conv1[((size_t)co * C + ci) * 9 + tap]; }, wmode,
               &L.sConv1[i]);
      L.bn2s[i] = f32(b.bn2s);
      L.bn2b[i] = f32(b.bn2b);
      L.wConv2[i] = bfOff();
      packConv(wb, 9, C, C, [&](int co, int ci, int tap) { return b.conv2[((size_t)co * C + ci) * 9 + tap]; }, wmode,
               &L.sConv2[i]);
    } else {
      packConv(wb, 9, C, C, [&](int co, int ci, int tap) {
        return co < Cr ? b.conv1[((size_t)co * C + ci) * 9 + tap] : b.conv1g[((size_t)(co - Cr) * C + ci) * 9 + tap];
      }, wmode, &L.sConv1[i]);
      L.bngs[i] = f32(b.bngs);
      L.bngb[i] = f32(b.bngb);
      L.linG[i] = f32T(b.linG, Cr);
      L.bn2s[i] = f32(b.bn2s);
      L.bn2b[i] = f32(b.bn2b);
      L.wConv2[i] = bfOff();
      packConv(wb, 9, Cr, C, [&](int co, int ci, int tap) { return b.conv2[((size_t)co * Cr + ci) * 9 + tap]; },
               wmode, &L.sConv2[i]);
    }
  }
  L.tips = f32(m.tips);
  L.tipb = f32(m.tipb);
  L.wHead = bfOff();
  packConv(wb, 1, C, C, [&](int co, int ci, int) {
    if(co < 32)
      return m.pConv1[(size_t)co * C + ci];
    if(co < 64)
      return m.pConvG[(size_t)(co - 32) * C + ci];
    return m.vConv1[(size_t)(co - 64) * C + ci];
  }, wmode, &L.sHead);
  L.pBiasG = f32(m.pBiasG);
  L.pLinG = f32T(m.pLinG, 32);
  L.pBias2 = f32(m.pBias2);
  L.pConv2 = f32(m.pConv2);
  L.vBias1 = f32(m.vBias1);
  L.vLin2 = f32T(m.vLin2, cfg_.v2);
  L.vB2 = f32(m.vB2);
  L.vLin3 = f32(m.vLin3);
  L.vB3 = f32(m.vB3);
  L.vLinM = f32(m.vLinM);
  L.vBM = f32(m.vBM);
  {
    std::vector<float> slabs((size_t)(L.nblocks + 1) * NN_PRM);
    for(int k = 0; k <= L.nblocks; k++)
      for(int t = 0; t < NN_PRM; t++) {
        const int src = paramSlabSource(L, k, t);
        slabs[(size_t)k * NN_PRM + t] = src >= 0 ? wf[src] : 0.0f;
      }
    L.prmSlabs = f32(slabs);
  }
  KC_HIP(hipMalloc(&wHalf_, wb.size() * 2));
  KC_HIP(hipMemcpy(wHalf_, wb.data(), wb.size() * 2, hipMemcpyHostToDevice));
  KC_HIP(hipMalloc(&wF32_, wf.size() * 4));
  KC_HIP(hipMemcpy(wF32_, wf.data(), wf.size() * 4, hipMemcpyHostToDevice));
  KC_HIP(hipMalloc(&layoutDev_, sizeof(NNLayout)));
  KC_HIP(hipMemcpy(layoutDev_, &L, sizeof(NNLayout), hipMemcpyHostToDevice));
  using G8 = NNGeo<5, 5, 96, 8, 0>;
  using G4 = NNGeo<5, 5, 96, NN_SMALL_NB, 0>;
  using GS = NNGeo<5, 5, 96, 2, NN_MODE_SPLIT3>;
  using GB = NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_SPLIT3, true>;
  using GC = NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_F8C, true>;
  const std::vector<uint16_t> tab8 = rowTables<G8>(), tab4 = rowTables<G4>(), tabS = rowTables<GS>(),
                              tabB = rowTables<GB>();
  KC_HIP(hipMalloc(&tabDevB_, tabB.size() * 2));
  KC_HIP(hipMemcpy(tabDevB_, tabB.data(), tabB.size() * 2, hipMemcpyHostToDevice));
  KC_HIP(hipMalloc(&tabDev_, tab8.size() * 2));
  KC_HIP(hipMemcpy(tabDev_, tab8.data(), tab8.size() * 2, hipMemcpyHostToDevice));
  KC_HIP(hipMalloc(&tabDevSm_, tab4.size() * 2));
  KC_HIP(hipMemcpy(tabDevSm_, tab4.data(), tab4.size() * 2, hipMemcpyHostToDevice));
  KC_HIP(hipMalloc(&tabDevS_, tabS.size() * 2));
  KC_HIP(hipMemcpy(tabDevS_, tabS.data(), tabS.size() * 2, hipMemcpyHostToDevice));

  // function attributes are per device: every engine sets it on its own device
  KC_HIP(hipFuncSetAttribute((const void*)kNNForward<5, 5, 96, 8, 0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             G8::LDS));
  KC_HIP(hipFuncSetAttribute((const void*)kNNForward<5, 5, 96, NN_SMALL_NB, 0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             G4::LDS));
  KC_HIP(hipFuncSetAttribute((const void*)kNNForward<5, 5, 96, 2, NN_MODE_SPLIT3, false>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, GS::LDS));
  KC_HIP(hipFuncSetAttribute((const void*)kNNForward<5, 5, 96, NN_SMALL_NB, NN_MODE_SPLIT3, true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, GB::LDS));
  KC_HIP(hipFuncSetAttribute((const void*)nnKernel<GC>(), hipFuncAttributeMaxDynamicSharedMemorySize, GC::LDS));
  using GF = NNGeo<5, 5, 96, NN_SMALL_NB, 0, true>;
  KC_HIP(hipFuncSetAttribute((const void*)nnKernel<GF>(), hipFuncAttributeMaxDynamicSharedMemorySize, GF::LDS));
#ifdef KC_AB_HOOKS
  // A/B builds only (tools/Makefile alt, -DKC_AB_HOOKS): KATACOFFEE_NN_SMALL=8 runs small
  // batches on the 8-board instance too; the product library never reads the variable
  const char* small = getenv("KATACOFFEE_NN_SMALL");
  small_ = small ? atoi(small) : 0;
#endif
  int dev = 0;
  KC_HIP(hipGetDevice(&dev));
  KC_HIP(hipDeviceGetAttribute(&cus_, hipDeviceAttributeMultiprocessorCount, dev));
}

NNEngine::~NNEngine() { release(); }

void NNEngine::release() {
  for(void* p : {(void*)trunk_, wHalf_, (void*)wF32_, (void*)layoutDev_, (void*)tabDev_, (void*)tabDevSm_,
                 (void*)tabDevS_, (void*)tabDevB_, (void*)hot_})
    (void)hipFree(p);
  trunk_ = nullptr;
  trunkBytes_ = 0;
  hot_ = nullptr;
  hotCap_ = 0;
  wHalf_ = nullptr;
  wF32_ = nullptr;
  layoutDev_ = nullptr;
  tabDev_ = tabDevSm_ = tabDevS_ = tabDevB_ = nullptr;
  layered_.reset();
  fallbackNet_.reset();
}

int NNEngine::precision() const {
  if(layered_)
    return layered_->split() ? NN_ACCURATE : NN_FAST_LAYERED;
  return mode_;
}

void NNEngine::forward(int n, const uint64_t* in, float* out, hipStream_t st, const int* countDev,
                       const int* rowIdx, hipEvent_t e0, hipEvent_t e1) {
  if(n <= 0)
    return;
  if(layered_) {
    if(e0)
      KC_HIP(hipEventRecord(e0, st));
    layered_->forward(n, in, out, st, countDev, rowIdx);
    if(e1)
      KC_HIP(hipEventRecord(e1, st));
    return;
  }
  const int inWords = (NUM_SPATIAL * X_ * Y_ + 63) / 64;
  // A launch costs about one workgroup's latency per wave of workgroups (one per CU):
  // a batch bound that fits NN_SMALL_NB boards per CU (e.g. each of two game groups'
  // batches) runs that many boards per workgroup, half the MFMA work on each
  // workgroup's path.
  // accurate / corrected: one instance for every batch size (results never depend on n)
  if(mode_ == NN_ACCURATE)
    launch<NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_SPLIT3, true>>(n, inWords, tabDevB_, in, out, st, countDev, rowIdx,
                                                               e0, e1);
  else if(mode_ == NN_CORRECTED) {
    // the corrected kernel flags boards whose activations pass e4m3's range; the accurate
    // kernel then re-evaluates the workgroups holding one (the others exit at once)
    const int grid = (n + NN_SMALL_NB - 1) / NN_SMALL_NB;
    if(grid * NN_SMALL_NB > hotCap_) {
      if(hot_)
        KC_HIP(hipStreamSynchronize(st));
      (void)hipFree(hot_);
      hot_ = nullptr;
      KC_HIP(hipMalloc(&hot_, (size_t)grid * NN_SMALL_NB * 4));
      KC_HIP(hipMemsetAsync(hot_, 0, (size_t)grid * NN_SMALL_NB * 4, st));
      hotCap_ = grid * NN_SMALL_NB;
    }
#ifdef KC_AB_NO_FALLBACK
    launch<NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_F8C, true>>(n, inWords, tabDevB_, in, out, st, countDev, rowIdx, e0, e1,
                                                            hot_);
#else
    launch<NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_F8C, true>>(n, inWords, tabDevB_, in, out, st, countDev, rowIdx, e0,
                                                            fallback_ ? nullptr : e1, hot_);
#endif
#ifdef KC_AB_NO_FALLBACK  // A/B builds: the cost of the (empty) re-evaluation launch
    if(false)
#else
    if(fallback_)  // the accurate engine's split weights, this engine's flags
#endif
      fallbackNet_->launch<NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_SPLIT3, true>>(
          n, inWords, fallbackNet_->tabDevB_, in, out, st, countDev, rowIdx, nullptr, e1, hot_);
  }
  else if(mode_ == NN_ACCURATE_NB2)
    launch<NNGeo<5, 5, 96, 2, NN_MODE_SPLIT3, false>>(n, inWords, tabDevS_, in, out, st, countDev, rowIdx, e0, e1);
  else if(n <= NN_SMALL_NB * cus_ && small_ != 8) {
    if(KC_FAST_BL)
      launch<NNGeo<5, 5, 96, NN_SMALL_NB, 0, true>>(n, inWords, tabDevB_, in, out, st, countDev, rowIdx, e0, e1);
    else
      launch<NNGeo<5, 5, 96, NN_SMALL_NB, 0>>(n, inWords, tabDevSm_, in, out, st, countDev, rowIdx, e0, e1);
  }
  else
    launch<NNGeo<5, 5, 96, 8, 0>>(n, inWords, tabDev_, in, out, st, countDev, rowIdx, e0, e1);
}

template <class G>
void NNEngine::launch(int n, int inWords, const uint16_t* tab, const uint64_t* in, float* out, hipStream_t st,
                      const int* countDev, const int* rowIdx, hipEvent_t e0, hipEvent_t e1, int* hot) {
  const int grid = (n + G::NB - 1) / G::NB;
  const size_t bytes = regTrunk<G>() ? 0 : (size_t)grid * G::NW * G::MAXT * G::NCT * 64 * 16;
  if(bytes > trunkBytes_) {
    // stream-ordered: a launch still using the old scratch finishes before the free
    if(trunk_)
      KC_HIP(hipStreamSynchronize(st));
    (void)hipFree(trunk_);
    trunk_ = nullptr;
    KC_HIP(hipMalloc(&trunk_, bytes));
    trunkBytes_ = bytes;
  }
  auto kern = nnKernel<G>();
  if(e0 || e1)
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(G::NT), G::LDS, st, e0, e1, 0, layoutDev_, (const h16x8*)wHalf_,
                          wF32_, tab, n, countDev, rowIdx, inWords, (float)W_, in, out, trunk_, hot);
  else
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G::NT), G::LDS, st, layoutDev_, (const h16x8*)wHalf_, wF32_, tab, n,
                       countDev, rowIdx, inWords, (float)W_, in, out, trunk_, hot);
  KC_HIP(hipGetLastError());
}

// Self-play audit of the default precision: the largest |difference| of
// two network outputs over the batch rows [0, min(n, *countDev)) (rows addressed through
// rowIdx like the network's), folded into *maxBits as float bits (non-negative floats
// order like their bits; NaN and infinity count as infinity).  One wave per row.
__global__ void __launch_bounds__(64) kAuditDiff(int n, const int* __restrict__ countDev, const int* __restrict__ rowIdx,
                                                 const float* __restrict__ a, const float* __restrict__ b, int width,
                                                 unsigned* __restrict__ maxBits) {
  const int count = countDev ? min(*countDev, n) : n;
  if((int)blockIdx.x >= count)
    return;
  const size_t row = (size_t)(rowIdx ? rowIdx[blockIdx.x] : (int)blockIdx.x) * width;
  float m = 0.0f;
  for(int j = threadIdx.x; j < width; j += 64) {
    const float d = fabsf(a[row + j] - b[row + j]);
    m = fmaxf(m, d <= 3.0e38f ? d : INFINITY);
  }
  for(int o = 32; o > 0; o >>= 1)
    m = fmaxf(m, __shfl_xor(m, o));
  if(threadIdx.x == 0)
    atomicMax(maxBits, __float_as_uint(m));
}

void NNEngine::audit(int n, const uint64_t* in, const float* out, float* scratch, unsigned* maxBits, hipStream_t st,
                     const int* countDev, const int* rowIdx) {
  if(layered_ || mode_ != NN_CORRECTED || !fallbackNet_ || n <= 0)
    return;
  const int m = std::min(n, NN_AUDIT_ROWS);
  const int inWords = (NUM_SPATIAL * X_ * Y_ + 63) / 64;
  // the accurate instance over the same rows (every board evaluated: no hot flags)
  fallbackNet_->launch<NNGeo<5, 5, 96, NN_SMALL_NB, NN_MODE_SPLIT3, true>>(m, inWords, fallbackNet_->tabDevB_, in, scratch,
                                                                           st, countDev, rowIdx, nullptr, nullptr);
  hipLaunchKernelGGL(kAuditDiff, dim3(m), dim3(64), 0, st, m, countDev, rowIdx, out, scratch, 4 * X_ * Y_ + 4, maxBits);
  KC_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Deterministic stand-in network (oracle fakeNet).
__global__ void __launch_bounds__(64) kFakeNet(const DTables* __restrict__ Tp, int n, const int* countDev,
                                               const int* __restrict__ rowIdx, const uint64_t* __restrict__ in,
                                               float* __restrict__ out) {
  const DTables& T = *Tp;
  const int count = countDev ? min(*countDev, n) : n;
  if((int)blockIdx.x >= count)
    return;
  const int i = rowIdx ? rowIdx[blockIdx.x] : (int)blockIdx.x;
  uint64_t h = 0x243f6a8885a308d3ULL;
  for(int w = 0; w < T.inWords; w++)
    h = mix64(h ^ in[(size_t)i * T.inWords + w]);
  float* o = out + (size_t)i * (T.P + 4);
  for(int j = threadIdx.x; j < T.P + 4; j += 64) {
    uint64_t v = mix64(h + (uint64_t)j * 0x9e3779b97f4a7c15ULL);
    int q = (int)((v >> 40) & 0xffffu);
    float scale = j < T.P ? (1.0f / 8192.0f) : (1.0f / 16384.0f);
    o[j] = ((float)q - 32768.0f) * scale;
  }
}

void launchFakeNet(const DTables* T, int n, const uint64_t* in, float* out, hipStream_t st, const int* countDev,
                   const int* rowIdx) {
  if(n <= 0)
    return;
  hipLaunchKernelGGL(kFakeNet, dim3(n), dim3(64), 0, st, T, n, countDev, rowIdx, in, out);
  KC_HIP(hipGetLastError());
}
#endif  // KC_NN_KERNEL_ONLY

}  // namespace kc
