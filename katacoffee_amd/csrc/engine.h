// Host-side declarations shared by the HIP translation units and the C ABI.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "kc_common.h"
#include "model.h"

namespace kc {

// ---- rules.hip ----
void launchRulesBatch(const DTables* T, int n, const uint8_t* cells, const int8_t* lastCell, const int8_t* lastDir,
                      const uint8_t* pla, uint8_t* legal, uint8_t* hasLegal, hipStream_t st);
void launchPlayBatch(const DTables* T, int n, const uint8_t* cells, const int8_t* lastCell, const int8_t* lastDir,
                     const uint8_t* pla, const int32_t* move, uint8_t* outCells, uint8_t* finished, uint8_t* winner,
                     int32_t* maxRunOut, uint64_t* posHash, uint64_t* stHash, hipStream_t st);
void launchEncodeBatch(const DTables* T, int n, const uint8_t* cells, const int8_t* histCell, const int8_t* histDir,
                       const uint8_t* pla, const int32_t* sym, uint64_t* packed, float* planes, hipStream_t st);

// Device copy of the geometry tables, cached per (X, Y, W).
const DTables* deviceTables(int X, int Y, int W);
const DTables& hostTables(int X, int Y, int W);

// ---- nn.hip ----
// Boards per network workgroup (one workgroup per compute unit at a time).
constexpr int NN_BOARDS_PER_WG = 8;
// Offsets (elements) into the packed weight buffers; see nn.hip.
constexpr int NN_MAX_BLOCKS = 16;
struct NNLayout {
  int nblocks, C, Cg, p1, g1, v1, v2, pad;
  int kinds[NN_MAX_BLOCKS];
  // bf16 B-fragment offsets (units of 8 bf16 = 16 bytes)
  int wInit, wHead;
  int wConv1[NN_MAX_BLOCKS], wConv2[NN_MAX_BLOCKS];
  // f32 offsets
  int globInit, tips, tipb, pBiasG, pLinG, pBias2, pConv2, vBias1, vLin2, vB2, vLin3, vB3, vLinM, vBM;
  int bn1s[NN_MAX_BLOCKS], bn1b[NN_MAX_BLOCKS], bn2s[NN_MAX_BLOCKS], bn2b[NN_MAX_BLOCKS];
  int bngs[NN_MAX_BLOCKS], bngb[NN_MAX_BLOCKS], linG[NN_MAX_BLOCKS];
};

class NNEngine {
 public:
  // Builds device weights for geometry X x Y (winLen W feeds the global input).
  NNEngine(const ModelHost& m, int X, int Y, int W);
  ~NNEngine();
  // in: packed V1 words [n][inWords] (device); out: [n][P+4] f32 (device):
  // policy logits [4][A] in the symmetric frame, value logits (win, loss), misc[2].
  // rows [0, min(n, *countDev)) of the batch; with rowIdx, batch row r is game row rowIdx[r]
  // (input in[rowIdx[r]], output out[rowIdx[r]]), otherwise r.
  void forward(int n, const uint64_t* in, float* out, hipStream_t st, const int* countDev = nullptr,
               const int* rowIdx = nullptr);
  const ModelCfg& cfg() const { return cfg_; }
  double flopsPerEval() const { return flops_; }
  static bool supported(const ModelCfg& c, int X, int Y);

 private:
  ModelCfg cfg_;
  int X_, Y_, W_;
  double flops_;
  NNLayout layout_;
  void* wHalf_ = nullptr;  // device
  float* wF32_ = nullptr;  // device
  NNLayout* layoutDev_ = nullptr;
  uint16_t* tabDev_ = nullptr;  // device row tables (nn.hip rowTables)
};

// Deterministic stand-in network (see oracle fakeNet); same I/O as NNEngine.
void launchFakeNet(const DTables* T, int n, const uint64_t* in, float* out, hipStream_t st,
                   const int* countDev = nullptr, const int* rowIdx = nullptr);

}  // namespace kc
