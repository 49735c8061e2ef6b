// See refrand.h.  SHA-256 (FIPS 180-4) and MD5 (RFC 1321) are written from the
// standards; the seeding/stream composition follows rand.cpp:290-333 and
// rand_helpers.h (PCG32 "XSH RR", xorshift1024* with multiplier 1181783497276652981).
#include "refrand.h"

#include <cstring>
#include <mutex>
#include <vector>

namespace kc {

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

void sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  static const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t padded = ((len + 9 + 63) / 64) * 64;
  std::vector<uint8_t> buf(padded, 0);
  if(len)
    memcpy(buf.data(), msg, len);
  buf[len] = 0x80;
  uint64_t bits = (uint64_t)len * 8;
  for(int i = 0; i < 8; i++)
    buf[padded - 1 - i] = (uint8_t)(bits >> (8 * i));
  for(size_t off = 0; off < padded; off += 64) {
    uint32_t w[64];
    for(int i = 0; i < 16; i++)
      w[i] = ((uint32_t)buf[off + 4 * i] << 24) | ((uint32_t)buf[off + 4 * i + 1] << 16) |
             ((uint32_t)buf[off + 4 * i + 2] << 8) | (uint32_t)buf[off + 4 * i + 3];
    for(int i = 16; i < 64; i++) {
      uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for(int i = 0; i < 64; i++) {
      uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
      uint32_t ch = (e & f) ^ (~e & g);
      uint32_t t1 = hh + S1 + ch + K[i] + w[i];
      uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
      uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  for(int i = 0; i < 8; i++)
    for(int j = 0; j < 4; j++)
      out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
}

void md5(const uint8_t* msg, size_t len, uint32_t out[4]) {
  static const uint32_t S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
  static uint32_t T[64];
  static bool init = false;
  if(!init) {
    // T[i] = floor(2^32 * |sin(i+1)|), RFC 1321 section 3.4
    static const uint32_t t[64] = {
      0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
      0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
      0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
      0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
      0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
      0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
      0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
      0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    memcpy(T, t, sizeof(T));
    init = true;
  }
  uint32_t a0 = 0x67452301, b0 = 0xefcdab89, c0 = 0x98badcfe, d0 = 0x10325476;
  size_t padded = ((len + 8) / 64 + 1) * 64;
  std::vector<uint8_t> buf(padded, 0);
  if(len)
    memcpy(buf.data(), msg, len);
  buf[len] = 0x80;
  uint64_t bits = (uint64_t)len * 8;
  for(int i = 0; i < 8; i++)
    buf[padded - 8 + i] = (uint8_t)(bits >> (8 * i));
  for(size_t off = 0; off < padded; off += 64) {
    uint32_t M[16];
    for(int i = 0; i < 16; i++)
      M[i] = (uint32_t)buf[off + 4 * i] | ((uint32_t)buf[off + 4 * i + 1] << 8) |
             ((uint32_t)buf[off + 4 * i + 2] << 16) | ((uint32_t)buf[off + 4 * i + 3] << 24);
    uint32_t A = a0, B = b0, C = c0, D = d0;
    for(int i = 0; i < 64; i++) {
      uint32_t F;
      int g;
      if(i < 16) { F = (B & C) | (~B & D); g = i; }
      else if(i < 32) { F = (D & B) | (~D & C); g = (5 * i + 1) % 16; }
      else if(i < 48) { F = B ^ C ^ D; g = (3 * i + 5) % 16; }
      else { F = C ^ (B | ~D); g = (7 * i) % 16; }
      uint32_t tmp = D;
      D = C;
      C = B;
      B = B + rotl(A + F + T[i] + M[g], (int)S[i]);
      A = tmp;
    }
    a0 += A; b0 += B; c0 += C; d0 += D;
  }
  out[0] = a0; out[1] = b0; out[2] = c0; out[3] = d0;
}

void RefRand::init(const std::string& seed) {
  uint32_t m[4];
  md5((const uint8_t*)seed.data(), seed.size(), m);
  std::string s = "|" + std::to_string(m[0]) + "|" + seed;
  int counter = 0;
  int next = 4;
  uint64_t hv[4] = {0, 0, 0, 0};
  auto nonzero = [&]() -> uint64_t {
    uint64_t v;
    do {
      if(next >= 4) {
        std::string tmp = std::to_string(counter) + s;
        counter += 37;
        uint8_t dg[32];
        sha256((const uint8_t*)tmp.data(), tmp.size(), dg);
        for(int i = 0; i < 4; i++) {
          uint64_t x = 0;
          for(int j = 0; j < 8; j++)
            x = (x << 8) | dg[8 * i + j];
          hv[i] = x;
        }
        next = 0;
      }
      v = hv[next++];
    } while(v == 0);
    return v;
  };
  for(int i = 0; i < 16; i++)
    xs[i] = nonzero();
  xsIdx = 0;
  pcg = nonzero();
}

uint32_t RefRand::nextUInt() {
  // PCG32 XSH-RR
  pcg = pcg * 6364136223846793005ULL + 1442695040888963407ULL;
  uint32_t x = (uint32_t)(((pcg >> 18) ^ pcg) >> 27);
  int rot = (int)(pcg >> 59);
  uint32_t p = rot == 0 ? x : ((x >> rot) | (x << (32 - rot)));
  // xorshift1024*
  uint64_t a0 = xs[xsIdx];
  xsIdx = (xsIdx + 1) & 15;
  uint64_t a1 = xs[xsIdx];
  a1 ^= a1 << 31;
  a1 ^= a1 >> 11;
  a0 ^= a0 >> 30;
  xs[xsIdx] = a0 ^ a1;
  uint32_t q = (uint32_t)((xs[xsIdx] * 1181783497276652981ULL) >> 32);
  return p + q;
}

double RefRand::nextDouble() {
  double x;
  do {
    uint64_t bits = nextUInt64() & ((1ULL << 53) - 1ULL);
    x = (double)bits / (double)(1ULL << 53);
  } while(!(x >= 0.0 && x < 1.0));
  return x;
}

uint64_t murmurMix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

uint64_t splitMix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

const ZobristTables& zobrist() {
  static ZobristTables z;
  static std::once_flag once;
  std::call_once(once, [] {
    RefRand r("Board::initHash()");
    auto next = [&r]() {
      Hash128 h;
      h.h0 = r.nextUInt64();
      h.h1 = r.nextUInt64();
      return h;
    };
    for(int i = 0; i < 4; i++)
      z.player[i] = next();
    for(int i = 0; i < ZobristTables::ARR; i++)
      for(int j = 0; j < 4; j++)
        z.board[i][j] = (j == 0 || j == 3) ? Hash128{0, 0} : next();
    r.init("Board::initHash() for ZOBRIST_SIZE hashes");
    for(int i = 0; i <= ZobristTables::MAX_LEN; i++) {
      z.sizeX[i] = next();
      z.sizeY[i] = next();
    }
    r.init("Board::initHash() for second set of ZOBRIST hashes");
    for(int i = 0; i < ZobristTables::ARR; i++)
      for(int j = 0; j < 4; j++) {
        Hash128 h = next();
        h.h0 = murmurMix(h.h0);
        h.h1 = splitMix64(h.h1);
        z.board2[i][j] = h;
      }
    // board.cpp:26-27, sha256-derived constant
    z.gameOver = Hash128{0xb6f9e465597a77eeULL, 0xf1d583d960a4ce7fULL};
  });
  return z;
}

}  // namespace kc
