// Device-side Coffee rules over bitboards (DBoard), wave-cooperative where the
// work is per-move.  Semantics restated from the reference:
//   Board::isLegal           board.cpp:185-227  (line constraint + "other empty cell on the line")
//   Board::playMoveAssumeLegal board.cpp:427-435, BoardHistory::makeBoardMoveAssumeLegal
//                            boardhistory.cpp:157-176 (+ SPEC B16 draw when stuck, B18 history)
//   Board::maxConsecutives   board.cpp:315-335
//   NNInputs::fillRowV1      nninputs.cpp:508-657 (SPEC a6 15-plane V1)
#pragma once
#include "detmath.h"
#include "kc_common.h"

namespace kc {

// ADJS (board.cpp:82-85) as steps: N (0,-1), W (-1,0), NW (-1,-1), NE (1,-1).
KC_HD int dirDx(int d) { return d == 0 ? 0 : (d == 3 ? 1 : -1); }
KC_HD int dirDy(int d) { return d == 1 ? 0 : -1; }

// Stones of one colour, chosen by an opaque mask rather than by indexing
// stones[]: an index (or a select the optimizer turns into one) would force
// the whole board out of registers into scratch memory.
KC_HD BB stonesOf(const DBoard& b, bool white) {
  uint64_t m = white ? ~0ULL : 0ULL;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(m));
#endif
  return BB{(b.stones[0].lo & ~m) | (b.stones[1].lo & m), (b.stones[0].hi & ~m) | (b.stones[1].hi & m)};
}

KC_HD BB occupied(const DBoard& b) { return bbOr(b.stones[0], b.stones[1]); }
KC_HD int colorAt(const DBoard& b, int c) {
  return bbTest(b.stones[0], c) ? 1 : (bbTest(b.stones[1], c) ? 2 : 0);
}

KC_HD bool isLegal(const DTables& T, const DBoard& b, int cell, int dir) {
  BB occ = occupied(b);
  if(bbTest(occ, cell))
    return false;
  if(b.lastCell >= 0 && b.lastDir < 4 && !bbTest(T.lineMask[b.lastCell][b.lastDir], cell))
    return false;
  return bbAny(bbAndNot(T.lineMask[cell][dir], occ));
}

KC_HD int maxRun(const DTables& T, const DBoard& b, int cell) {
  const int X = T.X, Y = T.Y;
  const BB own = stonesOf(b, colorAt(b, cell) == 2);
  int x = cell % X, y = cell / X, best = 1;
  for(int d = 0; d < 4; d++) {
    int n = 1;
    for(int s = -1; s <= 1; s += 2) {
      int cx = x + s * dirDx(d), cy = y + s * dirDy(d);
      while(cx >= 0 && cx < X && cy >= 0 && cy < Y && bbTest(own, cy * X + cx)) {
        n++;
        cx += s * dirDx(d);
        cy += s * dirDy(d);
      }
    }
    best = n > best ? n : best;
  }
  return best;
}

// Longest run of the cell's colour along axis d through the cell (0 if empty).
KC_HD int runAlong(const DTables& T, const DBoard& b, int cell, int d) {
  int col = colorAt(b, cell);
  if(col == 0)
    return 0;
  const BB own = stonesOf(b, col == 2);
  int x = cell % T.X, y = cell / T.X, n = 1;
  for(int s = -1; s <= 1; s += 2) {
    int cx = x + s * dirDx(d), cy = y + s * dirDy(d);
    while(cx >= 0 && cx < T.X && cy >= 0 && cy < T.Y && bbTest(own, cy * T.X + cx)) {
      n++;
      cx += s * dirDx(d);
      cy += s * dirDy(d);
    }
  }
  return n;
}

KC_HD void boardInit(const DTables& T, DBoard& b) {
  b.stones[0] = BB{0, 0};
  b.stones[1] = BB{0, 0};
  b.h0 = T.zInit[0];
  b.h1 = T.zInit[1];
  b.lastCell = -1;
  b.lastDir = 4;
  b.pla = 1;
  b.finished = 0;
  b.winner = 0;
  b.turn = 0;
  b.histC = 0xFFFFFFFFFFULL;  // five "none" cells
  b.histD = 0x0404040404ULL;
}

// State part of playMove (everything except the end-of-game test).
KC_HD void applyMove(const DTables& T, DBoard& b, int cell, int dir) {
  int pla = b.pla;
  if(pla == 2)
    bbSet(b.stones[1], cell);
  else
    bbSet(b.stones[0], cell);
  b.h0 ^= T.zBoard[cell][pla][0];
  b.h1 ^= T.zBoard[cell][pla][1];
  b.lastCell = cell;
  b.lastDir = dir;
  b.histC = ((b.histC << 8) | (uint64_t)(uint8_t)cell) & 0xFFFFFFFFFFULL;
  b.histD = ((b.histD << 8) | (uint64_t)(uint8_t)dir) & 0xFFFFFFFFFFULL;
  b.turn++;
  b.pla = 3 - pla;
  b.finished = 0;
  b.winner = 0;
}

KC_HD bool hasAnyLegalSerial(const DTables& T, const DBoard& b) {
  for(int c = 0; c < T.A; c++)
    for(int d = 0; d < 4; d++)
      if(isLegal(T, b, c, d))
        return true;
  return false;
}

// Serial (single-thread) full move: host tools and per-lane use.
KC_HD void playMoveSerial(const DTables& T, DBoard& b, int cell, int dir) {
  int mover = b.pla;
  applyMove(T, b, cell, dir);
  if(maxRun(T, b, cell) >= T.W) {
    b.finished = 1;
    b.winner = mover;
  } else if(!hasAnyLegalSerial(T, b)) {
    b.finished = 1;
    b.winner = 0;
  }
}

// GraphHash::getStateHash graphhash.cpp:3-12 + last-move term (SPEC a20).
KC_HD void stateHash(const DTables& T, const DBoard& b, uint64_t& k0, uint64_t& k1) {
  k0 = b.h0 ^ T.zPlayer[b.pla][0];
  k1 = b.h1 ^ T.zPlayer[b.pla][1];
  if(b.lastCell >= 0) {
    k0 ^= T.zBoard2[b.lastCell][b.lastDir][0];
    k1 ^= T.zBoard2[b.lastCell][b.lastDir][1];
  }
  if(b.finished) {
    k0 ^= T.zGameOver[0];
    k1 ^= T.zGameOver[1];
  }
}

// Wave-cooperative: every lane calls with the same board; result is uniform.
KC_D bool hasAnyLegalWave(const DTables& T, const DBoard& b) {
  bool any = false;
  for(int pos = laneId(); pos < T.P; pos += 64)
    any = any || isLegal(T, b, pos % T.A, pos / T.A);
  return ballot(any) != 0;
}

KC_D void playMoveWave(const DTables& T, DBoard& b, int cell, int dir) {
  int mover = b.pla;
  applyMove(T, b, cell, dir);
  if(maxRun(T, b, cell) >= T.W) {
    b.finished = 1;
    b.winner = mover;
  } else if(!hasAnyLegalWave(T, b)) {
    b.finished = 1;
    b.winner = 0;
  }
}

// The 15 V1 feature bits of ORIGINAL cell c (bit p = plane p); sd0 is the
// symmetric direction of the last move (-1 when there is none).
KC_D uint32_t v1CellFeatures(const DTables& T, const DBoard& b, int c, int sd0) {
  const int col = colorAt(b, c);
  uint32_t f = 1u;
  if(col != 0)
    f |= col == b.pla ? 2u : 4u;
  if(hCell(b, 0) == c && sd0 >= 0 && sd0 < 4)
    f |= 1u << (3 + sd0);
#pragma unroll
  for(int k = 1; k < 5; k++)
    if(hCell(b, k) == c)
      f |= 1u << (6 + k);
  bool legal = false, run[3] = {false, false, false};
  for(int d = 0; d < 4; d++) {
    legal = legal || isLegal(T, b, c, d);
    const int n = runAlong(T, b, c, d);
#pragma unroll
    for(int j = 0; j < 3; j++)
      run[j] = run[j] || (n >= 1 && n == T.W - 1 - j);
  }
  f |= (legal ? 1u : 0u) << 11;
#pragma unroll
  for(int j = 0; j < 3; j++)
    f |= (run[j] ? 1u : 0u) << (12 + j);
  return f;
}

// Packs the 15 V1 planes (symmetric frame) into T.inWords words: bit i of the
// flat [plane][cell] index lands in word i>>6, bit i&63 (oracle packPlanes).
// Lane s evaluates all 15 features of symmetric cell s (one table lookup, the
// four axes once), one ballot per plane collects them, and lane w assembles
// word w from the uniform plane masks.
KC_D void encodePackedWave(const DTables& T, const DBoard& b, int sym, uint64_t* out) {
  if(T.X != T.Y)
    sym &= 3;
  const int A = T.A, lane = laneId();
  const int h0 = hCell(b, 0);
  const int sd0 = h0 >= 0 ? T.symDir[sym][hDir(b, 0)] : -1;
  uint64_t word = 0;
  for(int base = 0; base < A; base += 64) {
    const int s = base + lane;
    const uint32_t f = s < A ? v1CellFeatures(T, b, T.invSymCell[sym][s], sd0) : 0u;
    // plane p's chunk covers flat bits [p*A + base, p*A + base + 64): OR the part
    // falling into this lane's word [64*lane, 64*lane + 64)
#pragma unroll
    for(int p = 0; p < NUM_SPATIAL; p++) {
      const uint64_t m = ballot((f >> p) & 1u);
      const int o = p * A + base - 64 * lane;
      if(o >= 0 && o < 64)
        word |= m << o;
      else if(o < 0 && o > -64)
        word |= m >> (-o);
    }
  }
  if(lane < T.inWords)
    out[lane] = word;
}

// Training-row bin planes (trainingwrite.cpp:218-232 packBits, identity symmetry):
// plane p occupies ceil(A/8) bytes, cell 8j+i at bit 7-i of byte j.  Wave-
// cooperative: lane s computes cell s's features, one ballot per plane and chunk,
// lanes j < ceil(A/8) store the bytes.  out = the row's NUM_SPATIAL*ceil(A/8) bytes.
KC_D void packRowBinWave(const DTables& T, const DBoard& b, uint8_t* out) {
  const int A = T.A, pb = (A + 7) / 8, lane = laneId();
  const int h0 = hCell(b, 0);
  const int sd0 = h0 >= 0 ? T.symDir[0][hDir(b, 0)] : -1;
  const uint32_t f0 = lane < A ? v1CellFeatures(T, b, lane, sd0) : 0u;
  const uint32_t f1 = 64 + lane < A ? v1CellFeatures(T, b, 64 + lane, sd0) : 0u;
  const int c0 = 8 * lane;
#pragma unroll
  for(int p = 0; p < NUM_SPATIAL; p++) {
    const uint64_t m0 = ballot((f0 >> p) & 1u), m1 = ballot((f1 >> p) & 1u);
    if(lane < pb) {
      const uint64_t m = c0 < 64 ? m0 : m1;
      const uint32_t bits = (uint32_t)(m >> (c0 & 63)) & 0xFFu;
      out[p * pb + lane] = (uint8_t)(__builtin_bitreverse32(bits) >> 24);
    }
  }
}

}  // namespace kc
