// refgen: golden-vector generator that drives the REFERENCE implementation
// (kennychenfs/KataCoffee cpp/core + cpp/game, compiled by build_ref.sh).
// It is test infrastructure only: tests/golden/make_golden.py runs it and
// stores its outputs as .npz fixtures; nothing in the product links it.
//
// Modes (all write little-endian binary files):
//   refgen rules  X Y WIN NGAMES SEED OUT   random legal games, per-position records
//   refgen zobrist OUT                      Board::initHash() tables (board.cpp:134-178)
//   refgen rand OUT                         Rand KAT streams for fixed seeds (rand.cpp)
//   refgen tdist OUT                        FancyMath::tdistcdf(z,3) on the search table grid
//                                           (search.cpp:111-116, distributiontable.h)
//   refgen selftest                         Rand::runTests() (rand.cpp:511+)
#include "../core/rand.h"
#include "../core/fancymath.h"
#include "../game/boardhistory.h"
#include "../game/graphhash.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace refgen {

static uint64_t sm64(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

static void put(FILE* f, const void* p, size_t n) {
  if(fwrite(p, 1, n, f) != n) {
    fprintf(stderr, "write failed\n");
    exit(1);
  }
}

// One record per position (before the move) of a random game:
//   int32  game, turn, pla, lastX, lastY, lastDir, hasLegal, movePos
//   uint8  colors[X*Y]      (0 empty, 1 black, 2 white; pos = y*X+x)
//   uint8  legal[4*X*Y]     (pos = dir*X*Y + y*X + x, NNPos::xydToPos order)
//   uint64 posHashBefore[2]
//   --- after the move (only meaningful if movePos >= 0):
//   int32  finished, winner, maxConsecutive
//   uint64 posHashAfter[2], sitHashAfter[2] (next player), stateHashAfter[2]
static int rules(int X, int Y, int W, int ngames, uint64_t seed, const char* out) {
  Board::initHash();
  FILE* f = fopen(out, "wb");
  if(!f)
    return 1;
  int32_t hdr[4] = {X, Y, W, ngames};
  put(f, hdr, sizeof(hdr));
  uint64_t s = seed;
  const int A = X * Y;
  std::vector<uint8_t> colors(A), legal(4 * A);
  int64_t totalRecords = 0;
  for(int g = 0; g < ngames; g++) {
    Board board(X, Y, W);
    BoardHistory hist(board, P_BLACK);
    Player pla = P_BLACK;
    for(int turn = 0;; turn++) {
      int legalCount = 0;
      std::vector<int> legalPos;
      for(int d = 0; d < 4; d++)
        for(int y = 0; y < Y; y++)
          for(int x = 0; x < X; x++) {
            Spot sp = Location::getSpot(x, y, X);
            bool ok = board.isLegal(Loc(sp, (Direction)d), pla);
            legal[d * A + y * X + x] = ok ? 1 : 0;
            if(ok) {
              legalCount++;
              legalPos.push_back(d * A + y * X + x);
            }
          }
      for(int y = 0; y < Y; y++)
        for(int x = 0; x < X; x++)
          colors[y * X + x] = (uint8_t)board.colors[Location::getSpot(x, y, X)];
      int32_t lastX = -1, lastY = -1, lastDir = board.lastLoc.dir;
      if(board.lastLoc.spot != Board::NULL_LOC) {
        lastX = Location::getX(board.lastLoc.spot, X);
        lastY = Location::getY(board.lastLoc.spot, X);
      }
      int32_t movePos = legalCount > 0 ? legalPos[sm64(s) % legalPos.size()] : -1;
      int32_t rec[8] = {g, turn, pla, lastX, lastY, lastDir, legalCount > 0 ? 1 : 0, movePos};
      put(f, rec, sizeof(rec));
      put(f, colors.data(), A);
      put(f, legal.data(), 4 * A);
      uint64_t hb[2] = {board.pos_hash.hash0, board.pos_hash.hash1};
      put(f, hb, sizeof(hb));
      int32_t after[3] = {0, 0, 0};
      uint64_t ha[6] = {0, 0, 0, 0, 0, 0};
      if(movePos >= 0) {
        int d = movePos / A, p = movePos % A;
        Spot sp = Location::getSpot(p % X, p / X, X);
        hist.makeBoardMoveAssumeLegal(board, Loc(sp, (Direction)d), pla);
        Player next = getOpp(pla);
        after[0] = hist.isGameFinished ? 1 : 0;
        after[1] = hist.winner;
        after[2] = board.maxConsecutives(sp);
        Hash128 sit = board.getSitHash(next);
        Hash128 st = GraphHash::getStateHash(hist, next);
        ha[0] = board.pos_hash.hash0;
        ha[1] = board.pos_hash.hash1;
        ha[2] = sit.hash0;
        ha[3] = sit.hash1;
        ha[4] = st.hash0;
        ha[5] = st.hash1;
        pla = next;
      }
      put(f, after, sizeof(after));
      put(f, ha, sizeof(ha));
      totalRecords++;
      if(movePos < 0 || after[0])
        break;
    }
  }
  fclose(f);
  fprintf(stderr, "rules %dx%d/%d: %d games, %lld records\n", X, Y, W, ngames, (long long)totalRecords);
  return 0;
}

static int zobrist(const char* out) {
  Board::initHash();
  FILE* f = fopen(out, "wb");
  if(!f)
    return 1;
  int32_t hdr[2] = {Board::MAX_LEN, Board::MAX_ARR_SIZE};
  put(f, hdr, sizeof(hdr));
  for(int i = 0; i < 4; i++)
    put(f, &Board::ZOBRIST_PLAYER_HASH[i], 16);
  for(int i = 0; i <= Board::MAX_LEN; i++)
    put(f, &Board::ZOBRIST_SIZE_X_HASH[i], 16);
  for(int i = 0; i <= Board::MAX_LEN; i++)
    put(f, &Board::ZOBRIST_SIZE_Y_HASH[i], 16);
  for(int i = 0; i < Board::MAX_ARR_SIZE; i++)
    for(int j = 0; j < 4; j++)
      put(f, &Board::ZOBRIST_BOARD_HASH[i][j], 16);
  for(int i = 0; i < Board::MAX_ARR_SIZE; i++)
    for(int j = 0; j < 4; j++)
      put(f, &Board::ZOBRIST_BOARD_HASH2[i][j], 16);
  put(f, &Board::ZOBRIST_GAME_IS_OVER, 16);
  fclose(f);
  return 0;
}

// For each seed string: 64 x nextUInt, 64 x nextUInt64, 64 x nextDouble,
// 64 x nextGaussian, 16 x nextGamma(a) for a in {0.05,0.3,1,2.5,10}.
static int randKats(const char* out) {
  const char* seeds[] = {"Board::initHash()", "abc", "coffee-bench:0:0", "", "$searchThread$0$"};
  FILE* f = fopen(out, "wb");
  if(!f)
    return 1;
  int32_t n = (int32_t)(sizeof(seeds) / sizeof(seeds[0]));
  put(f, &n, 4);
  for(int i = 0; i < n; i++) {
    int32_t len = (int32_t)strlen(seeds[i]);
    put(f, &len, 4);
    put(f, seeds[i], len);
    Rand r(seeds[i]);
    for(int k = 0; k < 64; k++) {
      uint32_t v = r.nextUInt();
      put(f, &v, 4);
    }
    for(int k = 0; k < 64; k++) {
      uint64_t v = r.nextUInt64();
      put(f, &v, 8);
    }
    for(int k = 0; k < 64; k++) {
      double v = r.nextDouble();
      put(f, &v, 8);
    }
    for(int k = 0; k < 64; k++) {
      double v = r.nextGaussian();
      put(f, &v, 8);
    }
    double as[5] = {0.05, 0.3, 1.0, 2.5, 10.0};
    for(int a = 0; a < 5; a++)
      for(int k = 0; k < 16; k++) {
        double v = r.nextGamma(as[a]);
        put(f, &v, 8);
      }
  }
  fclose(f);
  return 0;
}

static int tdist(const char* out) {
  // Search::Search builds DistributionTable(tdistpdf, tdistcdf, -50, 50, 2000)
  // with VALUE_WEIGHT_DEGREES_OF_FREEDOM = 3 (search.cpp:65, :111-116).
  const int size = 2000;
  const double minZ = -50.0, maxZ = 50.0;
  FILE* f = fopen(out, "wb");
  if(!f)
    return 1;
  int32_t hdr[1] = {size};
  put(f, hdr, 4);
  put(f, &minZ, 8);
  put(f, &maxZ, 8);
  for(int i = 0; i < size; i++) {
    double z = minZ + i * (maxZ - minZ) / (size - 1);
    double c = FancyMath::tdistcdf(z, 3.0);
    double p = FancyMath::tdistpdf(z, 3.0);
    put(f, &c, 8);
    put(f, &p, 8);
  }
  fclose(f);
  return 0;
}

}  // namespace refgen

int main(int argc, char** argv) {
  if(argc < 2) {
    fprintf(stderr, "usage: refgen rules|zobrist|rand|tdist|selftest ...\n");
    return 2;
  }
  std::string mode = argv[1];
  if(mode == "rules" && argc == 8)
    return refgen::rules(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), strtoull(argv[6], 0, 10), argv[7]);
  if(mode == "zobrist" && argc == 3)
    return refgen::zobrist(argv[2]);
  if(mode == "rand" && argc == 3)
    return refgen::randKats(argv[2]);
  if(mode == "tdist" && argc == 3)
    return refgen::tdist(argv[2]);
  if(mode == "selftest") {
    Rand::runTests();
    printf("Rand::runTests passed\n");
    return 0;
  }
  fprintf(stderr, "bad args\n");
  return 2;
}
