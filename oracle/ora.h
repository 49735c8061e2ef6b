// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.
// A plain single-threaded CPU restatement of the reference (kennychenfs/KataCoffee)
// self-play hot path: Coffee rules, V1 encoder, residual-net forward, MCTS
// (KataGo search semantics restated for Coffee), move choice and training rows.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// it; the product (katacoffee_amd/) never links or calls it.
//
// Parity pinning (see DESIGN.md "Oracle"):
//   rules / zobrist / state hash : bit-exact vs tests/golden/rules_*.npz, produced
//                                  by the reference's own cpp/game (oracle/_ref)
//   Rand / t-dist CDF table      : tests/golden/rand_kat.npz, tdist3.npz (reference)
//   NN layers                    : tests/golden/nnlayers_kat.npz (the reference's
//                                  cpp/tests/testnn.cpp layer KATs) and
//                                  tests/golden/nnblocks_pytorch.npz (python/model_pytorch.py
//                                  ResBlock / gpool / nested-bottleneck blocks), see
//                                  tests/test_oracle_nn.py
//   encoder / search / rows      : "parity unpinned" by any reference test — the
//                                  reference does not compile for these (SURVEY §0,
//                                  §8c); pinned by SPEC decisions in DESIGN.md.
// ============================================================================
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace ora {

constexpr int MAX_LEN = 10;
constexpr int MAX_AREA = MAX_LEN * MAX_LEN;
constexpr int MAX_P = 4 * MAX_AREA;
constexpr int ARR = (MAX_LEN + 1) * (MAX_LEN + 2) + 1;
constexpr int NUM_SPATIAL = 15;  // README "V1" table (SPEC a6)
constexpr int NUM_GLOBAL = 1;
constexpr int HIST = 5;

struct H128 {
  uint64_t h0 = 0, h1 = 0;
  H128 operator^(const H128& o) const { return H128{h0 ^ o.h0, h1 ^ o.h1}; }
  bool operator==(const H128& o) const { return h0 == o.h0 && h1 == o.h1; }
};

struct Tables {
  H128 board[ARR][4];
  H128 board2[ARR][4];
  H128 player[4];
  H128 sizeX[MAX_LEN + 1];
  H128 sizeY[MAX_LEN + 1];
  H128 gameOver;
  float cdf[2000];  // t-dist(3) CDF on [-50,50] (search.cpp:111-116)
  bool loaded = false;
};
extern Tables T;

struct Geom {
  int X, Y, W, A, P;
  Geom(int x = 5, int y = 5, int w = 4) : X(x), Y(y), W(w), A(x * y), P(4 * x * y) {}
};

// Board state (board.h:112-228 + the parts of BoardHistory the hot path reads).
struct Board {
  uint8_t c[MAX_AREA];   // 0 empty, 1 black, 2 white; cell = y*X + x
  int8_t lastCell;       // -1 = none
  int8_t lastDir;        // 0 N, 1 W, 2 NW, 3 NE, 4 NONE (board.h:41-47)
  uint8_t pla;           // player to move
  uint8_t finished;      // BoardHistory::isGameFinished
  uint8_t winner;        // 0 = draw / none
  int16_t turn;          // moves played from the start
  int8_t histCell[HIST]; // [0] = last move ... [4] = 5 moves ago, -1 absent
  int8_t histDir[HIST];
  H128 posHash;          // Board::pos_hash
};

void boardInit(const Geom& g, Board& b);
bool isLegal(const Geom& g, const Board& b, int cell, int dir);
bool hasAnyLegal(const Geom& g, const Board& b);
int maxRun(const Geom& g, const Board& b, int cell);
void playMove(const Geom& g, Board& b, int cell, int dir);  // updates finished/winner (SPEC B16)
H128 stateHash(const Geom& g, const Board& b);               // graph-search key (SPEC a20)
int spotOf(const Geom& g, int cell);
void encodeV1(const Geom& g, const Board& b, int sym, float* bin /*15*A*/, float* glob /*1*/);
int symCell(const Geom& g, int cell, int sym);
int symDir(int dir, int sym);

// --------------------------------------------------------------------------
// Neural net (Coffee b-blocks x c-channels; eigenbackend.cpp:888-1377 semantics,
// nested bottleneck blocks model_pytorch.py:860-958).  CFNN v1/v2 file layout:
// katacoffee_amd/csrc/model.h.
struct ModelCfg {
  int cin = NUM_SPATIAL, gin = NUM_GLOBAL;
  int C = 96, Cg = 32, p1 = 32, g1 = 32, v1 = 32, v2 = 64;
  int mid = 0;  // nested-bottleneck inner width (0: no bottleneck blocks)
  int nblocks = 6;
  int kinds[64] = {0, 0, 1, 0, 1, 0};  // 0 regular, 1 gpool, 2 bottleneck, 3 bottleneck (gpool inner 0)
};
// A convolution's weights [cout][cin][ky][kx] plus GEMM-packed copies (fp32 and
// fp16-rounded) for the blocked CPU forward.
struct PackedConv {
  int ky = 0, kx = 0, cin = 0, cout = 0;
  std::vector<float> w, p32, p16;
  // corrected-precision emulation: [3K][cout] = fp16(w) ; E(lo(w) 2^11, sw) / 2^11 ; E(w, sw)
  // (ora_nn.cpp: e4m3 at the convolution's block exponent sw)
  std::vector<float> pC;
  void pack();
};
struct Model {
  ModelCfg cfg;
  PackedConv convInit;
  std::vector<float> globInit;
  struct Block {
    int kind = 0;
    // regular / gpool (width = the block's trunk width)
    std::vector<float> bn1s, bn1b, bngs, bngb, linG, bn2s, bn2b;
    PackedConv conv1;  // gpool blocks: the r and g output channels concatenated [r | g]
    PackedConv conv1g; // optional separate gpool conv (then conv1 holds only r)
    PackedConv conv2;
    // nested bottleneck: p = 1x1 C->mid, two inner blocks at width mid, q = 1x1 mid->C
    std::vector<float> bnPs, bnPb, bnQs, bnQb;
    PackedConv convP, convQ;
    std::vector<Block> inner;
  };
  std::vector<Block> blocks;
  std::vector<float> tips, tipb;
  PackedConv head;  // 1x1 C -> [pConv1 | pConvG | vConv1]
  std::vector<float> pBiasG, pLinG, pBias2, pConv2;
  std::vector<float> vBias1, vLin2, vB2, vLin3, vB3, vLinM, vBM;
};
bool modelLoad(const char* path, Model& m);
// n boards of size X*Y; bin NCHW [n][cin][A], glob [n][gin];
// outputs: policy logits [n][4][A], value logits [n][2], misc [n][2].
// mode 0: fp32; mode 1: emulate the GPU kernels' fp16 rounding points (every
// convolution weight and convolution input rounded to fp16, residual trunks f32).
void nnForward(const Model& m, int X, int Y, int n, const float* bin, const float* glob,
               float* policy, float* value, float* misc, int mode, int threads);

// Layer library (the forward above is built from these; tests pin them to the
// reference's testnn.cpp known-answer vectors and model_pytorch.py blocks).
// Activations NHWC [n][A][C]; mask [n][A] (nullptr = all cells on board).
struct NNBatch {
  int n, X, Y, A;
  const float* mask;
  int mode;  // convolution operands: 0 fp32, 1 fp16 (fast), 2 fp16 + e4m3 cross terms (corrected)
  int threads;
  int* hot = nullptr;  // mode 2: [n] set for boards with a convolution input past e4m3's 448
};
void convApply(const NNBatch& b, const PackedConv& cv, const float* in, float* out, bool accumulate);
// BatchNormLayer::apply (eigenbackend.cpp:717-734): (x [+ perBoard]) * s + b, act, mask
void bnAct(const NNBatch& b, int C, const float* s, const float* bias, const float* in, int ldIn, float* out,
           bool relu, const float* perBoard = nullptr);
// poolRowsGPool / poolRowsValueHead (eigenbackend.cpp:141-186): out [n][3C]
void gpoolRows(const NNBatch& b, int C, const float* in, int ldIn, float* out, bool valueHead);
// residual blocks (ResidualBlock :888-931, GlobalPoolingResidualBlock :935-1015,
// NestedBottleneckResBlock model_pytorch.py:943-958): x [n][A][width] updated in place
void blockApply(const NNBatch& b, const Model::Block& blk, float* x);
// One block from its CFNN tensor sequence (kind 0-3 at trunk width W).
bool blockFromBlob(const float* blob, size_t count, int kind, int W, int Cg, int mid, Model::Block& b);

}  // namespace ora
