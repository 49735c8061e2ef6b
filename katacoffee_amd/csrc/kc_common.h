// Shared host/device definitions for the MI355X Coffee self-play engine.
// Board geometry, the SoA game state, device lookup tables and error handling.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#define KC_HD __host__ __device__ __forceinline__
#define KC_D __device__ __forceinline__

namespace kc {

constexpr int MAX_LEN = 10;          // COMPILE_MAX_BOARD_LEN, board.h:14-16
constexpr int MAX_AREA = MAX_LEN * MAX_LEN;
constexpr int MAX_P = 4 * MAX_AREA;  // NNPos::MAX_NN_POLICY_SIZE (nninputs.h:16)
constexpr int NUM_SPATIAL = 15;      // V1 planes (README "V1", SPEC a6)
constexpr int HIST = 5;
constexpr int CDF_SIZE = 2000;       // DistributionTable(-50, 50, 2000), search.cpp:111-116
constexpr int SVB_Z_SIZE = 2 * (MAX_P + 1) + 3 + 4 * 25;
constexpr int MAX_IN_WORDS = (NUM_SPATIAL * MAX_AREA + 63) / 64;

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
// invariant violation detected on the device (COFFEE_EINTERNAL at the C ABI)
struct InternalError : std::exception {
  std::string msg;
  explicit InternalError(std::string m) : msg(std::move(m)) {}
  const char* what() const noexcept override { return msg.c_str(); }
};

#define KC_HIP(call)                                                                                      \
  do {                                                                                                    \
    hipError_t e_ = (call);                                                                               \
    if(e_ != hipSuccess)                                                                                  \
      throw ::kc::HipError(std::string(#call) + " failed: " + hipGetErrorString(e_) + " @" __FILE__ ":" + \
                           std::to_string(__LINE__));                                                     \
  } while(0)

// 128-bit cell set (cell = y*X + x, up to 100 cells).
struct BB {
  uint64_t lo, hi;
};
KC_HD bool bbTest(const BB& b, int c) { return c < 64 ? ((b.lo >> c) & 1ULL) : ((b.hi >> (c - 64)) & 1ULL); }
KC_HD void bbSet(BB& b, int c) {
  if(c < 64)
    b.lo |= 1ULL << c;
  else
    b.hi |= 1ULL << (c - 64);
}
KC_HD BB bbOr(const BB& a, const BB& b) { return BB{a.lo | b.lo, a.hi | b.hi}; }
KC_HD BB bbAnd(const BB& a, const BB& b) { return BB{a.lo & b.lo, a.hi & b.hi}; }
KC_HD BB bbAndNot(const BB& a, const BB& b) { return BB{a.lo & ~b.lo, a.hi & ~b.hi}; }
KC_HD bool bbAny(const BB& a) { return (a.lo | a.hi) != 0; }

// Coffee position (board.h:112-228 + the BoardHistory fields the hot path reads).
// Plain scalar fields only (no small arrays), so boards stay in registers.
struct DBoard {
  BB stones[2];          // [0] black, [1] white
  uint64_t h0, h1;       // Board::pos_hash
  uint64_t histC;        // last five move cells, byte i = i-th most recent (0xFF none)
  uint64_t histD;        // their directions, byte i (4 = none)
  int32_t lastCell;      // -1 none
  int32_t lastDir;       // 0 N, 1 W, 2 NW, 3 NE, 4 NONE
  int32_t pla;           // 1 black, 2 white (to move)
  int32_t finished;      // BoardHistory::isGameFinished
  int32_t winner;        // 0 none/draw
  int32_t turn;
};
static_assert(sizeof(DBoard) == 88, "DBoard layout");
KC_HD int hCell(const DBoard& b, int i) { return (int)(int8_t)(uint8_t)(b.histC >> (8 * i)); }
KC_HD int hDir(const DBoard& b, int i) { return (int)(uint8_t)(b.histD >> (8 * i)); }

// Device-resident lookup tables for one board geometry (built by tables.cpp).
struct DTables {
  int X, Y, W, A, P, inWords;
  int pad[2];
  BB lineMask[MAX_AREA][4];     // cells on the line through c along dir, excluding c
  uint64_t zBoard[MAX_AREA][3][2];  // ZOBRIST_BOARD_HASH[spot(c)][color] (board.cpp:145-157)
  uint64_t zBoard2[MAX_AREA][4][2]; // ZOBRIST_BOARD_HASH2[spot(c)][dir]: last-move term of the state key
  uint64_t zPlayer[3][2];
  uint64_t zInit[2];            // ZOBRIST_SIZE_X_HASH[X] ^ ZOBRIST_SIZE_Y_HASH[Y]
  uint64_t zGameOver[2];
  float cdf[CDF_SIZE];
  uint64_t svbZ[SVB_Z_SIZE];
  uint8_t symCell[8][MAX_AREA];
  uint8_t invSymCell[8][MAX_AREA];
  int8_t symDir[8][5];
  int8_t pad2[24];
};

DTables buildTables(int X, int Y, int W);

}  // namespace kc
