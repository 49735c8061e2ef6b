// Host-side declarations shared by the HIP translation units and the C ABI.
#pragma once
#include <algorithm>
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
// Policy logits of n network rows [n][P+4] from each row's symmetric frame sym[n] to
// the canonical frame, in place (coffee_nn_forward2).
void launchCanonicalRows(const DTables* T, int n, const int32_t* sym, float* out, hipStream_t st);

// Device copy of the geometry tables, cached per (X, Y, W).
const DTables* deviceTables(int X, int Y, int W);
const DTables& hostTables(int X, int Y, int W);

// ---- nn.hip ----
// Boards per network workgroup (one workgroup per compute unit at a time).
constexpr int NN_BOARDS_PER_WG = 8;
// Boards per workgroup of the small-batch instance (batches of at most that many per
// CU): 5 boards = 125 positions fill the 128 rows its 8 waves compute as exactly as 4
// (100 rows) do, so a launch takes one workgroup's latency on a fifth fewer CUs; the
// other game group's search waves take the free CUs (nn.hip NNGeo).
#ifndef NN_SMALL_BOARDS
#define NN_SMALL_BOARDS 5
#endif
constexpr int NN_SMALL_NB = NN_SMALL_BOARDS;
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
  // corrected instance: each convolution's A scale byte, 127 - 11 + its weights' block exponent
  int sInit, sHead, sConv1[NN_MAX_BLOCKS], sConv2[NN_MAX_BLOCKS];
  // f32 offset of the parameter slabs, [nblocks + 1][NN_PRM] (nn.hip loadParam's layout,
  // gathered on the host so a slab element is one coalesced load)
  int prmSlabs;
};
constexpr int NN_PRM = 448;  // floats per parameter slab (NNGeo::NPRM)

// Layered forward (nn_layered.hip): one implicit-GEMM MFMA launch per convolution
// over the whole batch; any CFNN architecture (incl. nested bottlenecks) at 5x5,
// 7x7 and 9x9.  split = "accurate" precision (fp16 hi/lo operand pairs).
class NNLayered {
 public:
  NNLayered(const ModelHost& m, int X, int Y, int W, bool split);
  ~NNLayered();
  void forward(int n, const uint64_t* in, float* out, hipStream_t st, const int* countDev, const int* rowIdx);
  static bool supportedGeometry(int X, int Y);
  bool split() const { return split_; }

 private:
  struct Conv {
    int kt = 3, cin = 0, cinReal = 0, cout = 0, tn = 3, wn = 2, coutTiles = 0;
    long wOff = 0;  // 16-byte fragments into wHi_/wLo_
  };
  struct Block {
    int kind = 0, width = 0;
    int bn1s = -1, bn1b = -1, bn2s = -1, bn2b = -1, bngs = -1, bngb = -1, linGT = -1;
    int bnPs = -1, bnPb = -1, bnQs = -1, bnQb = -1;
    Conv conv1, conv2, convP, convQ;
    std::vector<Block> inner;
  };
  struct HeadOff {
    int pBiasG, pLinGT, pBias2, pConv2, vBias1, vLin2T, vB2, vLin3, vB3, vLinM, vBM;
  };
  void ensure(int n);
  void conv(const Conv& c, int pro, const void* src, int srcLd, int srcOff, int psOff, int pbOff, const float* gb,
            int gbLd, int epi, void* dst, int dstLd, int esOff, int ebOff, int n, const int* countDev,
            const uint64_t* bits, const int* rowIdx, hipStream_t st);
  void runBlock(const Block& b, float* x, int n, const int* countDev, hipStream_t st);
  ModelCfg cfg_;
  int X_, Y_, W_;
  bool split_;
  double flops_ = 0.0;
  Conv stem_, head_;
  std::vector<Block> blocks_;
  int globInit_ = 0, tips_ = 0, tipb_ = 0;
  HeadOff hw_{};
  int maxW_ = 0, tW_ = 0, hW_ = 0;
  void* wHi_ = nullptr;
  void* wLo_ = nullptr;
  float* wF_ = nullptr;
  void* act_ = nullptr;
  int cap_ = 0;
  float *bufX_ = nullptr, *bufY_ = nullptr, *bufT_ = nullptr, *bufGB_ = nullptr;
  uint16_t* bufH_ = nullptr;
};

// Network precision / path (coffee_nn_create2, coffee_selfplay_config.nn_precision)
enum NNPath : int {
  NN_DEFAULT = 0,       // the 1e-3 path: NN_CORRECTED (which runs the layered split kernels where the
                        // fused kernel does not cover the net)
  NN_ACCURATE = 1,      // fp16 hi/lo operand pairs (fused kernel when it covers the net, else layered):
                        // logits within 1e-3 of fp32 for any net
  NN_FAST_LAYERED = 2,  // fp16 operands on the layered path (comparison / any architecture)
  NN_CORRECTED = 3,     // fp16 products plus the two cross terms on block-scaled e4m3 MFMAs (2 fp16-MFMA
                        // equivalents per product, ~2^-14 per product): fused kernel when it covers the
                        // net, else the layered accurate path
  NN_ACCURATE_NB2 = 4,  // the 2-board bordered split instance (A/B reference of the borderless one)
  NN_FAST = 5,          // fp16 operands, f32 accumulation and trunk: fused kernel when it covers the net
};

class NNEngine {
 public:
  // Builds device weights for geometry X x Y (winLen W feeds the global input).
  NNEngine(const ModelHost& m, int X, int Y, int W, int path = NN_DEFAULT);
  ~NNEngine();
  // in: packed V1 words [n][inWords] (device); out: [n][P+4] f32 (device):
  // policy logits [4][A] in the symmetric frame, value logits (win, loss), misc[2].
  // rows [0, min(n, *countDev)) of the batch; with rowIdx, batch row r is game row rowIdx[r]
  // (input in[rowIdx[r]], output out[rowIdx[r]]), otherwise r.
  // e0/e1 (optional): timing events, recorded by the fused kernel's dispatch itself
  // (kernel-only time), around the layered kernels otherwise
  void forward(int n, const uint64_t* in, float* out, hipStream_t st, const int* countDev = nullptr,
               const int* rowIdx = nullptr, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
  const ModelCfg& cfg() const { return cfg_; }
  double flopsPerEval() const { return flops_; }
  bool fused() const { return !layered_; }
  // rows per launch worth batching for one of `engines` engines sharing the device: the
  // fused kernel costs one workgroup's latency per wave of workgroups (one per CU), so a
  // launch is capped at one wave: cus x 8 boards of the fast kernel split between the
  // engines (two engines each launch up to cus x 4, one wave of its 5-board workgroups);
  // the accurate / corrected kernels have only the 5-board instance, so at most cus x 5
  // (cus x 8 was 1.6 waves for a lone engine); the 2-board A/B instance cus x 2
  int batchCap(int cus, int engines) const {
    if(layered_)
      return 1 << 30;
    if(mode_ == NN_ACCURATE_NB2)
      return std::max(1, cus * 2 / engines);
    const int split = std::max(1, cus * NN_BOARDS_PER_WG / engines);
    return (mode_ == NN_ACCURATE || mode_ == NN_CORRECTED) ? std::min(cus * NN_SMALL_NB, split) : split;
  }
  static bool fusedSupported(const ModelCfg& c, int X, int Y);
  // the precision the engine runs (NNPath; NN_DEFAULT resolved): NN_CORRECTED or NN_ACCURATE
  // for the default, NN_ACCURATE / NN_FAST_LAYERED on the layered kernels
  int precision() const;
  // the default precision's check: largest |logit| difference between the corrected and
  // accurate instances on the calibration batch (0 when not run)
  float calibrationError() const { return calibErr_; }
  // the default precision takes the corrected instance when that difference is at most this
  // (a quarter of north_star's 1e-3)
  static constexpr float NN_AUTO_TOL = 2.5e-4f;
  // Self-play audit of the corrected instance (the default precision's check on the
  // positions self-play actually evaluates, not only the calibration batch): re-evaluates
  // rows [0, min(n, NN_AUDIT_ROWS)) of a batch `forward` just wrote to `out` on the
  // accurate instance into `scratch` (rows addressed like `out`) and folds the largest
  // |difference| into *maxBits (float bits, device).  No-op unless the engine runs the
  // corrected instance.
  static constexpr int NN_AUDIT_ROWS = 256;
  void audit(int n, const uint64_t* in, const float* out, float* scratch, unsigned* maxBits, hipStream_t st,
             const int* countDev, const int* rowIdx);

 private:
  void build(const ModelHost& m, int path);
  void release();
  float calibrationError(NNEngine& ref, int* hotBoards);
  float calibErr_ = 0.0f;
  ModelCfg cfg_;
  int X_, Y_, W_;
  double flops_;
  NNLayout layout_;
  void* wHalf_ = nullptr;  // device
  float* wF32_ = nullptr;  // device
  NNLayout* layoutDev_ = nullptr;
  uint16_t* tabDev_ = nullptr;   // device row tables (nn.hip rowTables), 8 boards per workgroup
  uint16_t* tabDevSm_ = nullptr; // the same for the small-batch instance (NN_SMALL_NB boards)
  uint16_t* tabDevS_ = nullptr;  // the same for the 2-board split instance (NN_ACCURATE_NB2)
  uint16_t* tabDevB_ = nullptr;  // the same for the borderless 5-board instances (accurate, corrected)
  int mode_ = NN_FAST;           // NNPath of the fused kernel
  int small_ = 0;                // KATACOFFEE_NN_SMALL=8: small batches on the 8-board instance (A/B runs)
  float* trunk_ = nullptr;       // f32 residual trunk scratch, [workgroup][fragment] (nn.hip)
  size_t trunkBytes_ = 0;        // its size
  int cus_ = 1;                  // compute units of the engine's device
  template <class G>
  void launch(int n, int inWords, const uint16_t* tab, const uint64_t* in, float* out, hipStream_t st,
              const int* countDev, const int* rowIdx, hipEvent_t e0, hipEvent_t e1, int* hot = nullptr);
  int* hot_ = nullptr;      // corrected: per batch position, activations past e4m3 (nn.hip kNNForward)
  int hotCap_ = 0;
  bool fallback_ = true;    // corrected: re-evaluate flagged boards on the accurate instance
  std::unique_ptr<NNEngine> fallbackNet_;  // corrected: that instance (split-packed weights)
  std::unique_ptr<NNLayered> layered_;
};

// Deterministic stand-in network (see oracle fakeNet); same I/O as NNEngine.
void launchFakeNet(const DTables* T, int n, const uint64_t* in, float* out, hipStream_t st,
                   const int* countDev = nullptr, const int* rowIdx = nullptr);

}  // namespace kc
