// ORACLE (test infrastructure only) — Coffee rules and the V1 encoder.
// Restates board.cpp / boardhistory.cpp / graphhash.cpp / nninputs.cpp with the
// SPEC decisions recorded in DESIGN.md ("Bug decisions B1-B25").
#include "ora.h"

#include <cstring>

namespace ora {

Tables T;

// Location::getSpot, board.cpp:30-32 — the padded index the Zobrist tables use.
int spotOf(const Geom& g, int cell) {
  int x = cell % g.X, y = cell / g.X;
  return (x + 1) + (y + 1) * (g.X + 1);
}

// Board::init, board.cpp:111-132 (pos_hash = size hashes; lastLoc = NULL/NONE)
// + BoardHistory::clear, boardhistory.cpp:172-193.
void boardInit(const Geom& g, Board& b) {
  memset(&b, 0, sizeof(b));
  b.lastCell = -1;
  b.lastDir = 4;
  b.pla = 1;
  for(int i = 0; i < HIST; i++) {
    b.histCell[i] = -1;
    b.histDir[i] = 4;
  }
  b.posHash = T.sizeX[g.X] ^ T.sizeY[g.Y];
}

// Board::isLegal, board.cpp:185-227 (with the P3 `tempSpot` fix).  The two
// line walks are "some OTHER empty cell exists on the line through `cell`
// along `dir`", walking through stones and stopping at the wall.
static const int DX[4] = {0, -1, -1, 1};  // ADJ1..ADJ4 board.cpp:82-85: N, W, NW, NE
static const int DY[4] = {-1, 0, -1, -1};

bool isLegal(const Geom& g, const Board& b, int cell, int dir) {
  if(b.pla != 1 && b.pla != 2)
    return false;
  if(b.c[cell] != 0)
    return false;
  int x = cell % g.X, y = cell / g.X;
  if(b.lastCell >= 0 && b.lastDir < 4) {
    int dx = x - b.lastCell % g.X, dy = y - b.lastCell / g.X;
    switch(b.lastDir) {
      case 0: if(dx != 0 || dy == 0) return false; break;
      case 1: if(dx == 0 || dy != 0) return false; break;
      case 2: if(dx != dy) return false; break;
      case 3: if(dx != -dy) return false; break;
    }
  }
  for(int s = -1; s <= 1; s += 2) {
    int cx = x + s * DX[dir], cy = y + s * DY[dir];
    while(cx >= 0 && cx < g.X && cy >= 0 && cy < g.Y) {
      if(b.c[cy * g.X + cx] == 0)
        return true;
      cx += s * DX[dir];
      cy += s * DY[dir];
    }
  }
  return false;
}

bool hasAnyLegal(const Geom& g, const Board& b) {
  for(int cell = 0; cell < g.A; cell++)
    for(int d = 0; d < 4; d++)
      if(isLegal(g, b, cell, d))
        return true;
  return false;
}

// Board::maxConsecutives, board.cpp:315-335.
int maxRun(const Geom& g, const Board& b, int cell) {
  int color = b.c[cell];
  int x = cell % g.X, y = cell / g.X;
  int best = 1;
  for(int d = 0; d < 4; d++) {
    int n = 1;
    for(int s = -1; s <= 1; s += 2) {
      int cx = x + s * DX[d], cy = y + s * DY[d];
      while(cx >= 0 && cx < g.X && cy >= 0 && cy < g.Y && b.c[cy * g.X + cx] == color) {
        n++;
        cx += s * DX[d];
        cy += s * DY[d];
      }
    }
    if(n > best)
      best = n;
  }
  return best;
}

// Board::playMoveAssumeLegal board.cpp:427-435 + BoardHistory::makeBoardMoveAssumeLegal
// boardhistory.cpp:157-176 (win => winner = mover).  SPEC B16: if the game is not
// won and the player to move next has no legal move, the game ends as a draw.
// SPEC B18: the move IS recorded in the history (histCell/histDir).
void playMove(const Geom& g, Board& b, int cell, int dir) {
  int pla = b.pla;
  b.c[cell] = (uint8_t)pla;
  b.posHash = b.posHash ^ T.board[spotOf(g, cell)][pla];
  b.lastCell = (int8_t)cell;
  b.lastDir = (int8_t)dir;
  for(int i = HIST - 1; i > 0; i--) {
    b.histCell[i] = b.histCell[i - 1];
    b.histDir[i] = b.histDir[i - 1];
  }
  b.histCell[0] = (int8_t)cell;
  b.histDir[0] = (int8_t)dir;
  b.turn++;
  b.pla = (uint8_t)(3 - pla);
  b.finished = 0;
  b.winner = 0;
  if(maxRun(g, b, cell) >= g.W) {
    b.finished = 1;
    b.winner = (uint8_t)pla;
  } else if(!hasAnyLegal(g, b)) {
    b.finished = 1;
    b.winner = 0;
  }
}

// GraphHash::getStateHash graphhash.cpp:3-12 (sitHash ^ GAME_IS_OVER) extended
// with the last move (SPEC a20: legality depends on lastLoc, so it must be part
// of a transposition key); ZOBRIST_BOARD_HASH2[spot][dir] supplies that term.
H128 stateHash(const Geom& g, const Board& b) {
  H128 h = b.posHash ^ T.player[b.pla];
  if(b.lastCell >= 0)
    h = h ^ T.board2[spotOf(g, b.lastCell)][b.lastDir];
  if(b.finished)
    h = h ^ T.gameOver;
  return h;
}

// SymmetryHelpers::getSymSpot nninputs.cpp:377-391: flipX, flipY, then transpose
// (transpose ignored on non-square boards, as copyWithSymmetry does).
int symCell(const Geom& g, int cell, int sym) {
  int x = cell % g.X, y = cell / g.X;
  if(sym & 2) x = g.X - 1 - x;
  if(sym & 1) y = g.Y - 1 - y;
  if((sym & 4) && g.X == g.Y) {
    int t = x; x = y; y = t;
  }
  return y * g.X + x;
}

// SymmetryHelpers::getSymDir nninputs.cpp:409-433, fixed (B12): a flip of one
// axis swaps the two diagonals, a transpose swaps N and W.
int symDir(int dir, int sym) {
  if(dir >= 4)
    return dir;
  bool t = (sym & 4) != 0;
  bool fx = (sym & 2) != 0, fy = (sym & 1) != 0;
  if(fx != fy) {
    if(dir == 2) dir = 3;
    else if(dir == 3) dir = 2;
  }
  if(t) {
    if(dir == 0) dir = 1;
    else if(dir == 1) dir = 0;
  }
  return dir;
}

// Runs of stones of EXACT length len along any axis: per-(cell, axis) maximal
// run (SPEC B8 fix of Board::fillRowWithLine board.cpp:392-420).
static void lineRuns(const Geom& g, const Board& b, int runLen, uint8_t* mark) {
  for(int cell = 0; cell < g.A; cell++) {
    int col = b.c[cell];
    if(col == 0)
      continue;
    int x = cell % g.X, y = cell / g.X;
    for(int d = 0; d < 4; d++) {
      int n = 1;
      for(int s = -1; s <= 1; s += 2) {
        int cx = x + s * DX[d], cy = y + s * DY[d];
        while(cx >= 0 && cx < g.X && cy >= 0 && cy < g.Y && b.c[cy * g.X + cx] == col) {
          n++;
          cx += s * DX[d];
          cy += s * DY[d];
        }
      }
      if(n == runLen)
        mark[cell] = 1;
    }
  }
}

// NNInputs::fillRowV1 nninputs.cpp:508-657 restated as the README "V1" table:
//   0 on-board | 1 own | 2 opp | 3-6 last move by dir | 7-10 moves 2..5 ago
//   11 legal cells (any dir) | 12-14 runs of exact length W-1, W-2, W-3
// written in the symmetric frame `sym` (copyInputsWithSymmetry nninputs.cpp:337).
void encodeV1(const Geom& g, const Board& b, int sym, float* bin, float* glob) {
  const int A = g.A;
  if(g.X != g.Y)
    sym &= 3;  // copyWithSymmetry ignores transpose on non-square boards
  memset(bin, 0, sizeof(float) * NUM_SPATIAL * A);
  int pla = b.pla, opp = 3 - pla;
  uint8_t lines[3][MAX_AREA];
  memset(lines, 0, sizeof(lines));
  for(int j = 0; j < 3; j++)
    if(g.W - 1 - j >= 1)
      lineRuns(g, b, g.W - 1 - j, lines[j]);
  for(int cell = 0; cell < A; cell++) {
    int s = symCell(g, cell, sym);
    bin[0 * A + s] = 1.0f;
    if(b.c[cell] == pla) bin[1 * A + s] = 1.0f;
    else if(b.c[cell] == opp) bin[2 * A + s] = 1.0f;
    bool anyLegal = false;
    for(int d = 0; d < 4 && !anyLegal; d++)
      anyLegal = isLegal(g, b, cell, d);
    if(anyLegal) bin[11 * A + s] = 1.0f;
    for(int j = 0; j < 3; j++)
      if(lines[j][cell]) bin[(12 + j) * A + s] = 1.0f;
  }
  if(b.histCell[0] >= 0)
    bin[(3 + symDir(b.histDir[0], sym)) * A + symCell(g, b.histCell[0], sym)] = 1.0f;
  for(int k = 1; k < HIST; k++)
    if(b.histCell[k] >= 0)
      bin[(7 + k - 1) * A + symCell(g, b.histCell[k], sym)] = 1.0f;
  glob[0] = (float)g.W;
}

}  // namespace ora
