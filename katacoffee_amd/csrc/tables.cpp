// Host construction of the per-geometry device tables (DTables).
//   lineMask  : the line walks of Board::isLegal (board.cpp:213-226) and the
//               lastLoc line constraint (board.cpp:190-212) as cell sets
//   zobrist   : Board::initHash (board.cpp:134-178) via the Rand port (refrand.cpp)
//   cdf       : DistributionTable(tdistpdf/tdistcdf nu=3, -50..50, 2000) (search.cpp:111-116),
//               Student-t nu=3 CDF in closed form, rounded to f32
//   sym       : SymmetryHelpers::getSymSpot/getSymDir (nninputs.cpp:377-433, B12 fixed)
#include <cmath>
#include <cstring>

#include "detmath.h"
#include "kc_common.h"
#include "refrand.h"

namespace kc {

static const int DXS[4] = {0, -1, -1, 1};  // N, W, NW, NE (board.cpp:82-85)
static const int DYS[4] = {-1, 0, -1, -1};

static double tdist3Cdf(double t) {
  // nu = 3: F(t) = 1/2 + (1/pi) * ( t/(sqrt(3)(1+t^2/3)) + atan(t/sqrt(3)) )
  const double s3 = std::sqrt(3.0);
  return 0.5 + (1.0 / M_PI) * (t / (s3 * (1.0 + t * t / 3.0)) + std::atan(t / s3));
}

static int symCellOf(int X, int Y, int cell, int sym) {
  int x = cell % X, y = cell / X;
  if(sym & 2) x = X - 1 - x;
  if(sym & 1) y = Y - 1 - y;
  if((sym & 4) && X == Y) {
    int t = x; x = y; y = t;
  }
  return y * X + x;
}

static int symDirOf(int dir, int sym) {
  if(dir >= 4)
    return dir;
  bool fx = (sym & 2) != 0, fy = (sym & 1) != 0, t = (sym & 4) != 0;
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

DTables buildTables(int X, int Y, int W) {
  if(X < 2 || Y < 2 || X > MAX_LEN || Y > MAX_LEN || W < 2 || W > std::max(X, Y))
    throw std::invalid_argument("buildTables: unsupported board " + std::to_string(X) + "x" + std::to_string(Y) +
                                " winLen " + std::to_string(W));
  DTables t;
  memset(&t, 0, sizeof(t));
  t.X = X;
  t.Y = Y;
  t.W = W;
  t.A = X * Y;
  t.P = 4 * X * Y;
  t.inWords = (NUM_SPATIAL * t.A + 63) / 64;
  for(int c = 0; c < t.A; c++)
    for(int d = 0; d < 4; d++) {
      BB m{0, 0};
      int x = c % X, y = c / X;
      for(int s = -1; s <= 1; s += 2) {
        int cx = x + s * DXS[d], cy = y + s * DYS[d];
        while(cx >= 0 && cx < X && cy >= 0 && cy < Y) {
          bbSet(m, cy * X + cx);
          cx += s * DXS[d];
          cy += s * DYS[d];
        }
      }
      t.lineMask[c][d] = m;
    }
  const ZobristTables& z = zobrist();
  for(int c = 0; c < t.A; c++) {
    int spot = (c % X + 1) + (c / X + 1) * (X + 1);
    for(int col = 0; col < 3; col++) {
      t.zBoard[c][col][0] = z.board[spot][col].h0;
      t.zBoard[c][col][1] = z.board[spot][col].h1;
    }
    for(int d = 0; d < 4; d++) {
      t.zBoard2[c][d][0] = z.board2[spot][d].h0;
      t.zBoard2[c][d][1] = z.board2[spot][d].h1;
    }
  }
  for(int p = 0; p < 3; p++) {
    t.zPlayer[p][0] = z.player[p].h0;
    t.zPlayer[p][1] = z.player[p].h1;
  }
  t.zInit[0] = z.sizeX[X].h0 ^ z.sizeY[Y].h0;
  t.zInit[1] = z.sizeX[X].h1 ^ z.sizeY[Y].h1;
  t.zGameOver[0] = z.gameOver.h0;
  t.zGameOver[1] = z.gameOver.h1;
  for(int i = 0; i < CDF_SIZE; i++) {
    double zz = -50.0 + i * (100.0) / (CDF_SIZE - 1);
    t.cdf[i] = (float)tdist3Cdf(zz);
  }
  // SVB pattern zobrist: one stream with a fixed seed (SPEC a19).
  DRng r{0x5b5b5b5b5b5b5b5bULL, 0};
  for(int i = 0; i < SVB_Z_SIZE; i++)
    t.svbZ[i] = r.next();
  for(int s = 0; s < 8; s++) {
    for(int c = 0; c < t.A; c++) {
      int sc = symCellOf(X, Y, c, s);
      t.symCell[s][c] = (uint8_t)sc;
      t.invSymCell[s][sc] = (uint8_t)c;
    }
    for(int d = 0; d < 5; d++)
      t.symDir[s][d] = (int8_t)symDirOf(d, (X == Y) ? s : (s & 3));
  }
  return t;
}

}  // namespace kc
