// Batched Coffee rules and V1 encoder kernels (the C-ABI's coffee_rules_batch,
// coffee_play_batch, coffee_encode_batch).  The self-play engine calls the same
// device functions (kc_board.h) from its select/backup kernels.
#include "engine.h"
#include "kc_board.h"

namespace kc {

KC_D DBoard boardFromCells(const DTables& T, const uint8_t* cells, int lastCell, int lastDir, int pla,
                           const int8_t* histCell, const int8_t* histDir) {
  DBoard b;
  boardInit(T, b);
  for(int c = 0; c < T.A; c++) {
    int col = cells[c];
    if(col == 1 || col == 2) {
      if(col == 2)
        bbSet(b.stones[1], c);
      else
        bbSet(b.stones[0], c);
      b.h0 ^= T.zBoard[c][col][0];
      b.h1 ^= T.zBoard[c][col][1];
    }
  }
  b.lastCell = lastCell;
  b.lastDir = lastDir;
  b.pla = pla;
  uint64_t hc = 0, hd = 0;
#pragma unroll
  for(int i = HIST - 1; i >= 0; i--) {
    int c = histCell ? histCell[i] : (i == 0 ? lastCell : -1);
    int d = histDir ? histDir[i] : (i == 0 ? lastDir : 4);
    hc = (hc << 8) | (uint64_t)(uint8_t)c;
    hd = (hd << 8) | (uint64_t)(uint8_t)d;
  }
  b.histC = hc;
  b.histD = hd;
  return b;
}

// One wave per position; lanes enumerate the 4A moves (wave-ballot enumeration).
__global__ void __launch_bounds__(64) kRulesBatch(const DTables* __restrict__ Tp, int n, const uint8_t* cells,
                                                  const int8_t* lastCell, const int8_t* lastDir, const uint8_t* pla,
                                                  uint8_t* legal, uint8_t* hasLegal) {
  const DTables& T = *Tp;
  int i = blockIdx.x;
  if(i >= n)
    return;
  DBoard b = boardFromCells(T, cells + (size_t)i * T.A, lastCell[i], lastDir[i], pla[i], nullptr, nullptr);
  bool any = false;
  for(int pos = laneId(); pos < T.P; pos += 64) {
    bool ok = (b.pla == 1 || b.pla == 2) && isLegal(T, b, pos % T.A, pos / T.A);
    legal[(size_t)i * T.P + pos] = ok ? 1 : 0;
    any = any || ok;
  }
  uint64_t m = ballot(any);
  if(laneId() == 0)
    hasLegal[i] = m != 0 ? 1 : 0;
}

__global__ void __launch_bounds__(64) kPlayBatch(const DTables* __restrict__ Tp, int n, const uint8_t* cells,
                                                 const int8_t* lastCell, const int8_t* lastDir, const uint8_t* pla,
                                                 const int32_t* move, uint8_t* outCells, uint8_t* finished,
                                                 uint8_t* winner, int32_t* maxRunOut, uint64_t* posHash,
                                                 uint64_t* stHash) {
  const DTables& T = *Tp;
  int i = blockIdx.x;
  if(i >= n)
    return;
  DBoard b = boardFromCells(T, cells + (size_t)i * T.A, lastCell[i], lastDir[i], pla[i], nullptr, nullptr);
  int mv = move[i];
  int cell = mv % T.A, dir = mv / T.A;
  playMoveWave(T, b, cell, dir);
  for(int c = laneId(); c < T.A; c += 64)
    outCells[(size_t)i * T.A + c] = (uint8_t)colorAt(b, c);
  if(laneId() == 0) {
    finished[i] = (uint8_t)b.finished;
    winner[i] = (uint8_t)b.winner;
    maxRunOut[i] = maxRun(T, b, cell);
    posHash[2 * i] = b.h0;
    posHash[2 * i + 1] = b.h1;
    uint64_t k0, k1;
    stateHash(T, b, k0, k1);
    stHash[2 * i] = k0;
    stHash[2 * i + 1] = k1;
  }
}

__global__ void __launch_bounds__(64) kEncodeBatch(const DTables* __restrict__ Tp, int n, const uint8_t* cells,
                                                   const int8_t* histCell, const int8_t* histDir, const uint8_t* pla,
                                                   const int32_t* sym, uint64_t* packed, float* planes) {
  const DTables& T = *Tp;
  int i = blockIdx.x;
  if(i >= n)
    return;
  const int8_t* hc = histCell + (size_t)i * HIST;
  const int8_t* hd = histDir + (size_t)i * HIST;
  DBoard b = boardFromCells(T, cells + (size_t)i * T.A, hc[0], hd[0], pla[i], hc, hd);
  uint64_t* out = packed + (size_t)i * T.inWords;
  encodePackedWave(T, b, sym[i], out);
  if(planes) {
    __syncthreads();
    for(int j = laneId(); j < NUM_SPATIAL * T.A; j += 64) {
      uint64_t w = out[j >> 6];
      planes[(size_t)i * NUM_SPATIAL * T.A + j] = ((w >> (j & 63)) & 1ULL) ? 1.0f : 0.0f;
    }
  }
}

// Network rows back to the canonical frame (coffee_nn_forward2; the reference backend's
// SymmetryHelpers::copyOutputsWithSymmetry in NeuralNet::getOutput, eigenbackend.cpp:
// 1776-1796): canonical[d][cell] = symmetric[symDir[s][d]][symCell[s][cell]], in place,
// one 64-lane workgroup per row staged through LDS; value / misc logits unchanged.
__global__ void __launch_bounds__(64) kCanonicalRows(const DTables* __restrict__ Tp, int n, const int32_t* sym,
                                                     float* out) {
  const DTables& T = *Tp;
  __shared__ float row[4 * MAX_AREA + 4];
  const int i = blockIdx.x;
  if(i >= n)
    return;
  const int P = T.P, A = T.A;
  int s = sym[i] & 7;
  if(T.X != T.Y)
    s &= 3;
  float* o = out + (size_t)i * (P + 4);
  for(int j = laneId(); j < P; j += 64)
    row[j] = o[j];
  __syncthreads();
  for(int pos = laneId(); pos < P; pos += 64) {
    const int d = pos / A, cell = pos - d * A;
    o[pos] = row[T.symDir[s][d] * A + T.symCell[s][cell]];
  }
}

void launchCanonicalRows(const DTables* T, int n, const int32_t* sym, float* out, hipStream_t st) {
  if(n <= 0)
    return;
  hipLaunchKernelGGL(kCanonicalRows, dim3(n), dim3(64), 0, st, T, n, sym, out);
  KC_HIP(hipGetLastError());
}

void launchRulesBatch(const DTables* T, int n, const uint8_t* cells, const int8_t* lastCell, const int8_t* lastDir,
                      const uint8_t* pla, uint8_t* legal, uint8_t* hasLegal, hipStream_t st) {
  if(n <= 0)
    return;
  hipLaunchKernelGGL(kRulesBatch, dim3(n), dim3(64), 0, st, T, n, cells, lastCell, lastDir, pla, legal, hasLegal);
  KC_HIP(hipGetLastError());
}

void launchPlayBatch(const DTables* T, int n, const uint8_t* cells, const int8_t* lastCell, const int8_t* lastDir,
                     const uint8_t* pla, const int32_t* move, uint8_t* outCells, uint8_t* finished, uint8_t* winner,
                     int32_t* maxRunOut, uint64_t* posHash, uint64_t* stHash, hipStream_t st) {
  if(n <= 0)
    return;
  hipLaunchKernelGGL(kPlayBatch, dim3(n), dim3(64), 0, st, T, n, cells, lastCell, lastDir, pla, move, outCells,
                     finished, winner, maxRunOut, posHash, stHash);
  KC_HIP(hipGetLastError());
}

void launchEncodeBatch(const DTables* T, int n, const uint8_t* cells, const int8_t* histCell, const int8_t* histDir,
                       const uint8_t* pla, const int32_t* sym, uint64_t* packed, float* planes, hipStream_t st) {
  if(n <= 0)
    return;
  hipLaunchKernelGGL(kEncodeBatch, dim3(n), dim3(64), 0, st, T, n, cells, histCell, histDir, pla, sym, packed,
                     planes);
  KC_HIP(hipGetLastError());
}

}  // namespace kc
