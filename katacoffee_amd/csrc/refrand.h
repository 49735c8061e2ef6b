// Host-side, reference-compatible random stream used ONLY to derive the Zobrist
// tables bit-exactly (board.cpp:134-178 `Board::initHash`), so that position
// hashes produced on the GPU equal the reference's `Board::pos_hash`.
//
// Algorithm restated from the reference's published behaviour (independent code):
//   seeding   rand.cpp:290-333  MD5(seed)[0] and SHA-256 chains -> 16+1 nonzero u64
//   stream    rand.h:140-160    nextUInt = PCG32 + xorshift1024*  (rand_helpers.h)
//   nextUInt64 rand.h:176-181   lower | upper<<32
// Verified against tests/golden/rand_kat.npz (reference output).
#pragma once
#include <cstdint>
#include <string>

namespace kc {

void sha256(const uint8_t* msg, size_t len, uint8_t out[32]);
void md5(const uint8_t* msg, size_t len, uint32_t out[4]);

class RefRand {
 public:
  explicit RefRand(const std::string& seed) { init(seed); }
  void init(const std::string& seed);
  uint32_t nextUInt();
  uint64_t nextUInt64() {
    uint64_t lo = nextUInt();
    uint64_t hi = (uint64_t)nextUInt() << 32;
    return lo | hi;
  }
  double nextDouble();

 private:
  uint64_t xs[16];
  uint64_t xsIdx;
  uint64_t pcg;
};

struct Hash128 {
  uint64_t h0, h1;
};

// Same mixers as core/hash.cpp (murmur3 fmix64 / splitmix64 finalizers).
uint64_t murmurMix(uint64_t x);
uint64_t splitMix64(uint64_t x);

// Board::initHash() tables for COMPILE_MAX_BOARD_LEN = 10 (board.h:14-16, 120-135).
struct ZobristTables {
  static constexpr int MAX_LEN = 10;
  static constexpr int ARR = (MAX_LEN + 1) * (MAX_LEN + 2) + 1;  // 133
  Hash128 player[4];
  Hash128 sizeX[MAX_LEN + 1];
  Hash128 sizeY[MAX_LEN + 1];
  Hash128 board[ARR][4];
  Hash128 board2[ARR][4];
  Hash128 gameOver;
};
const ZobristTables& zobrist();

}  // namespace kc
