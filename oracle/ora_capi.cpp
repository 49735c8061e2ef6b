// ORACLE (test infrastructure only) — extern "C" surface for the Python test
// harness (ctypes) and bench.py's cpu_baseline leg.  Never linked by the product.
#include <cmath>
#include <cstdio>
#include <cstring>

#include "ora.h"
#include "ora_search.h"

using namespace ora;

extern "C" {

int ora_load_tables(const uint64_t* board, const uint64_t* board2, const uint64_t* player, const uint64_t* sizeX,
                    const uint64_t* sizeY, const uint64_t* gameOver, const float* cdf) {
  memcpy(T.board, board, sizeof(T.board));
  memcpy(T.board2, board2, sizeof(T.board2));
  memcpy(T.player, player, sizeof(T.player));
  memcpy(T.sizeX, sizeX, sizeof(T.sizeX));
  memcpy(T.sizeY, sizeY, sizeof(T.sizeY));
  memcpy(&T.gameOver, gameOver, sizeof(T.gameOver));
  memcpy(T.cdf, cdf, sizeof(T.cdf));
  T.loaded = true;
  return 0;
}

static void toBoard(const Geom& g, Board& b, const uint8_t* colors, int lastCell, int lastDir, int pla,
                    const int8_t* histCell, const int8_t* histDir) {
  boardInit(g, b);
  H128 h = b.posHash;
  for(int c = 0; c < g.A; c++) {
    b.c[c] = colors[c];
    if(colors[c] == 1 || colors[c] == 2)
      h = h ^ T.board[spotOf(g, c)][colors[c]];
  }
  b.posHash = h;
  b.lastCell = (int8_t)lastCell;
  b.lastDir = (int8_t)lastDir;
  b.pla = (uint8_t)pla;
  for(int i = 0; i < HIST; i++) {
    b.histCell[i] = histCell ? histCell[i] : (i == 0 ? (int8_t)lastCell : (int8_t)-1);
    b.histDir[i] = histDir ? histDir[i] : (i == 0 ? (int8_t)lastDir : (int8_t)4);
  }
}

// Legal mask for n positions: legal[i][dir*A + cell] (NNPos::xydToPos order).
int ora_rules_batch(int X, int Y, int W, int n, const uint8_t* colors, const int8_t* lastCell, const int8_t* lastDir,
                    const uint8_t* pla, uint8_t* legal, uint8_t* hasLegal) {
  Geom g(X, Y, W);
  for(int i = 0; i < n; i++) {
    Board b;
    toBoard(g, b, colors + (size_t)i * g.A, lastCell[i], lastDir[i], pla[i], nullptr, nullptr);
    bool any = false;
    for(int p = 0; p < g.P; p++) {
      bool ok = isLegal(g, b, p % g.A, p / g.A);
      legal[(size_t)i * g.P + p] = ok ? 1 : 0;
      any = any || ok;
    }
    hasLegal[i] = any ? 1 : 0;
  }
  return 0;
}

// Plays move[i] (pos = dir*A + cell) on each position; reports the post-move state.
int ora_play_batch(int X, int Y, int W, int n, const uint8_t* colors, const int8_t* lastCell, const int8_t* lastDir,
                   const uint8_t* pla, const int32_t* move, uint8_t* outColors, uint8_t* finished, uint8_t* winner,
                   int32_t* maxRunOut, uint64_t* posHash, uint64_t* stHash) {
  Geom g(X, Y, W);
  for(int i = 0; i < n; i++) {
    Board b;
    toBoard(g, b, colors + (size_t)i * g.A, lastCell[i], lastDir[i], pla[i], nullptr, nullptr);
    int cell = move[i] % g.A, dir = move[i] / g.A;
    playMove(g, b, cell, dir);
    memcpy(outColors + (size_t)i * g.A, b.c, g.A);
    finished[i] = b.finished;
    winner[i] = b.winner;
    maxRunOut[i] = maxRun(g, b, cell);
    posHash[2 * i] = b.posHash.h0;
    posHash[2 * i + 1] = b.posHash.h1;
    H128 s = stateHash(g, b);
    stHash[2 * i] = s.h0;
    stHash[2 * i + 1] = s.h1;
  }
  return 0;
}

int ora_encode_batch(int X, int Y, int W, int n, const uint8_t* colors, const int8_t* histCell, const int8_t* histDir,
                     const uint8_t* pla, const int32_t* sym, float* bin, float* glob) {
  Geom g(X, Y, W);
  for(int i = 0; i < n; i++) {
    Board b;
    const int8_t* hc = histCell + (size_t)i * HIST;
    const int8_t* hd = histDir + (size_t)i * HIST;
    toBoard(g, b, colors + (size_t)i * g.A, hc[0], hd[0], pla[i], hc, hd);
    encodeV1(g, b, sym[i], bin + (size_t)i * NUM_SPATIAL * g.A, glob + i);
  }
  return 0;
}

int ora_fake_net(int X, int Y, int W, int n, const float* bin, float* out /*[n][P+4]*/) {
  Geom g(X, Y, W);
  for(int i = 0; i < n; i++) {
    float* o = out + (size_t)i * (g.P + 4);
    fakeNet(g, bin + (size_t)i * NUM_SPATIAL * g.A, o, o + g.P, o + g.P + 2);
  }
  return 0;
}

void* ora_model_load(const char* path) {
  Model* m = new Model();
  if(!modelLoad(path, *m)) {
    delete m;
    return nullptr;
  }
  return m;
}
void ora_model_free(void* m) { delete(Model*)m; }

int ora_nn_forward(void* m, int X, int Y, int n, const float* bin, const float* glob, float* policy, float* value,
                   float* misc, int mode, int threads) {
  nnForward(*(Model*)m, X, Y, n, bin, glob, policy, value, misc, mode, threads);
  return 0;
}

// ---- NN layer library (tests/test_oracle_nn.py) ----
// BatchNormLayer merge (eigenbackend.cpp:700-706): scale / sqrt(var + eps), bias - scale * mean.
void ora_bn_merge(int C, float eps, const float* mean, const float* var, const float* scale, const float* bias,
                  float* outS, float* outB) {
  for(int c = 0; c < C; c++) {
    outS[c] = scale[c] / sqrtf(var[c] + eps);
    outB[c] = bias[c] - outS[c] * mean[c];
  }
}

static PackedConv mkConv(int ky, int kx, int cin, int cout, const float* w) {
  PackedConv c;
  c.ky = ky;
  c.kx = kx;
  c.cin = cin;
  c.cout = cout;
  c.w.assign(w, w + (size_t)ky * kx * cin * cout);
  c.pack();
  return c;
}

int ora_conv_apply(int ky, int kx, int cin, int cout, const float* w, int n, int X, int Y, const float* in, float* out,
                   int mode) {
  NNBatch b{n, X, Y, X * Y, nullptr, mode, 1};
  convApply(b, mkConv(ky, kx, cin, cout, w), in, out, false);
  return 0;
}

int ora_bn_apply(int C, const float* s, const float* bias, int relu, int n, int X, int Y, const float* in,
                 const float* mask, float* out) {
  NNBatch b{n, X, Y, X * Y, mask, 0, 1};
  bnAct(b, C, s, bias, in, C, out, relu != 0);
  return 0;
}

int ora_gpool_apply(int C, int valueHead, int n, int X, int Y, const float* in, const float* mask, float* out) {
  NNBatch b{n, X, Y, X * Y, mask, 0, 1};
  gpoolRows(b, C, in, C, out, valueHead != 0);
  return 0;
}

// One residual block given its pieces (any kernel sizes): conv k = (ky, kx, cin, cout).
// kind 0: preBN, conv1, midBN, conv2.  kind 1 (gpool): conv1 the regular conv, kg/wg
// the gpool conv, gS/gB the gpool BN, linG [Cr][3Cg] (Cr = conv2 cin).
int ora_block_apply_parts(int kind, int n, int X, int Y, const float* mask, float* x, const float* preS,
                          const float* preB, const int* k1, const float* w1, const int* kg, const float* wg,
                          const float* gS, const float* gB, const float* linG, const float* midS, const float* midB,
                          const int* k2, const float* w2, int mode) {
  NNBatch b{n, X, Y, X * Y, mask, mode, 1};
  Model::Block blk;
  blk.kind = kind;
  blk.conv1 = mkConv(k1[0], k1[1], k1[2], k1[3], w1);
  blk.conv2 = mkConv(k2[0], k2[1], k2[2], k2[3], w2);
  if(kind == 1)
    blk.conv1g = mkConv(kg[0], kg[1], kg[2], kg[3], wg);
  const int W = k1[2], H = k1[3] + (kind == 1 ? kg[3] : 0), M = k2[2];
  blk.bn1s.assign(preS, preS + W);
  blk.bn1b.assign(preB, preB + W);
  blk.bn2s.assign(midS, midS + M);
  blk.bn2b.assign(midB, midB + M);
  if(kind == 1) {
    const int Cg = H - M;
    blk.bngs.assign(gS, gS + Cg);
    blk.bngb.assign(gB, gB + Cg);
    blk.linG.assign(linG, linG + (size_t)M * 3 * Cg);
  }
  blockApply(b, blk, x);
  return 0;
}

// One block (kind 0-3; 2/3 = nested bottleneck, model_pytorch.py:860-958) from its
// CFNN tensor sequence (csrc/model.h) at trunk width W, bottleneck width mid, gpool Cg.
int ora_block_apply_blob(int kind, int W, int mid, int Cg, const float* blob, long long count, int n, int X, int Y,
                         float* x, int mode) {
  Model::Block blk;
  if(!blockFromBlob(blob, (size_t)count, kind, W, Cg, mid, blk))
    return 1;
  NNBatch b{n, X, Y, X * Y, nullptr, mode, 1};
  blockApply(b, blk, x);
  return 0;
}

// play: NULL or the 13 play settings in coffee_search_params order (cheap_search_prob,
// cheap_search_visits, cheap_search_target_weight, reduce_visits, reduce_visits_threshold,
// reduce_visits_threshold_lookback, reduced_visits_min, reduced_visits_weight,
// policy_surprise_data_weight, value_surprise_data_weight, init_games_with_policy,
// policy_init_area_prop, policy_init_area_temperature, early_fork_game_prob,
// early_fork_game_expected_move_prop, fork_game_prob, fork_game_min_choices,
// early_fork_game_max_choices, fork_game_max_choices, side_position_prob,
// record_tree_positions, record_tree_threshold, record_tree_target_weight) and the
// search's cpuct_exploration.
void* ora_sp_create(int X, int Y, int W, int games, int maxVisits, int nodeCap, uint64_t seed, int slotBase,
                    int nnMode, void* model, int nnThreads, int cacheLog2, const float* play, int nnCap) {
  if(!T.loaded)
    return nullptr;
  Selfplay* s = new Selfplay();
  SelfplayCfg cfg;
  cfg.g = Geom(X, Y, W);
  cfg.sp.maxVisits = maxVisits;
  if(play) {
    cfg.sp.cheapSearchProb = play[0];
    cfg.sp.cheapSearchVisits = (int)play[1];
    cfg.sp.cheapSearchTargetWeight = play[2];
    cfg.sp.reduceVisits = (int)play[3];
    cfg.sp.reduceVisitsThreshold = play[4];
    cfg.sp.reduceVisitsThresholdLookback = (int)play[5];
    cfg.sp.reducedVisitsMin = (int)play[6];
    cfg.sp.reducedVisitsWeight = play[7];
    cfg.sp.policySurpriseDataWeight = play[8];
    cfg.sp.valueSurpriseDataWeight = play[9];
    cfg.sp.initGamesWithPolicy = (int)play[10];
    cfg.sp.policyInitAreaProp = play[11];
    cfg.sp.policyInitAreaTemperature = play[12];
    cfg.sp.earlyForkGameProb = play[13];
    cfg.sp.earlyForkGameExpectedMoveProp = play[14];
    cfg.sp.forkGameProb = play[15];
    cfg.sp.forkGameMinChoices = (int)play[16];
    cfg.sp.earlyForkGameMaxChoices = (int)play[17];
    cfg.sp.forkGameMaxChoices = (int)play[18];
    cfg.sp.sidePositionProb = play[19];
    cfg.sp.recordTreePositions = (int)play[20];
    cfg.sp.recordTreeThreshold = (int)play[21];
    cfg.sp.recordTreeTargetWeight = play[22];
    cfg.sp.cpuctExploration = play[23];
  }
  cfg.nodeCap = nodeCap;
  cfg.seed = seed;
  cfg.slotBase = slotBase;
  cfg.nnMode = nnMode;
  cfg.model = (const Model*)model;
  cfg.nnThreads = nnThreads;
  if(cacheLog2 < 0 || cacheLog2 > 26)
    return nullptr;
  cfg.cacheLog2 = cacheLog2;
  if(nnCap > 0)
    cfg.nnCap = nnCap;
  selfplayInit(*s, cfg, games);
  return s;
}
void ora_sp_free(void* h) { delete(Selfplay*)h; }
// Composition tests: every later round's network batch goes to fn (nnMode 3).
void ora_sp_set_netfn(void* h, void (*fn)(int, const uint64_t*, float*)) {
  Selfplay* s = (Selfplay*)h;
  s->cfg.netFn = fn;
  s->cfg.nnMode = fn ? 3 : 0;
}
// CPU baseline: threads over games in select / backup (numGameThreads, selfplay.cpp:90)
void ora_sp_set_parallel(void* h, int threads) { ((Selfplay*)h)->cfg.parallelGames = threads; }

// n rounds on the device engine's schedule (selfplay.cpp SelfplayEngine::step): moves
// are committed in rounds r with (r + 1) % commitInterval == 0 and in the call's last round.
int ora_sp_rounds(void* h, int n) {
  Selfplay* s = (Selfplay*)h;
  const uint64_t ci = (uint64_t)s->cfg.commitInterval;
  for(int i = 0; i < n; i++)
    selfplayRound(*s, ci <= 1 || (s->rounds + 1) % ci == 0 || i == n - 1);
  return 0;
}
// Round schedule, before the first round: commit interval (coffee_selfplay_config
// commit_interval) and staggered starts (start_stagger).
int ora_sp_set_schedule(void* h, int commitInterval, int startStagger) {
  Selfplay* s = (Selfplay*)h;
  if(s->rounds != 0 || commitInterval < 1 || startStagger < 0)
    return -1;
  selfplaySchedule(*s, commitInterval, startStagger);
  return 0;
}

// info[16]: phase, rootK, nodeCount, rootIdx, turn, pla, gameNum, playouts, nnEvals,
//           movesMade, gamesFinished, rngCtr, leafKind, rootVisits, lastCell, lastDir
int ora_sp_game_info(void* h, int slot, int64_t* info) {
  Selfplay* s = (Selfplay*)h;
  Game& gm = s->games[slot];
  int64_t v[16] = {gm.phase, gm.rootK, gm.nodeCount, gm.rootIdx, gm.root.turn, gm.root.pla, gm.gameNum,
                   (int64_t)gm.playouts, (int64_t)gm.nnEvals, (int64_t)gm.movesMade, (int64_t)gm.gamesFinished,
                   (int64_t)gm.rng.ctr, gm.leafKind, gm.rootIdx >= 0 ? (int64_t)gm.nodes[gm.rootIdx].visits : 0,
                   gm.root.lastCell, gm.root.lastDir};
  memcpy(info, v, sizeof(v));
  return 0;
}

// Copies the node pool of a game: nodes as raw 64-byte records (see ora::Node),
// and edges child/visits/move for the first nodeCount nodes.
int ora_sp_game_nodes(void* h, int slot, void* nodes, uint32_t* edgeChild, uint32_t* edgeVisits, uint16_t* edgeMove,
                      float* policy) {
  Selfplay* s = (Selfplay*)h;
  Game& gm = s->games[slot];
  const int P = s->cfg.g.P;
  memcpy(nodes, gm.nodes.data(), sizeof(Node) * gm.nodeCount);
  memcpy(edgeChild, gm.edgeChild.data(), sizeof(uint32_t) * (size_t)gm.nodeCount * P);
  memcpy(edgeVisits, gm.edgeVisits.data(), sizeof(uint32_t) * (size_t)gm.nodeCount * P);
  memcpy(edgeMove, gm.edgeMove.data(), sizeof(uint16_t) * (size_t)gm.nodeCount * P);
  memcpy(policy, gm.policy.data(), sizeof(float) * (size_t)gm.nodeCount * P);
  return gm.nodeCount;
}

int ora_sp_root_noised(void* h, int slot, float* out) {
  Selfplay* s = (Selfplay*)h;
  memcpy(out, s->games[slot].rootNoised.data(), sizeof(float) * s->cfg.g.P);
  return 0;
}

int ora_sp_rows_count(void* h) { return ((Selfplay*)h)->rows.n; }
int ora_sp_rows(void* h, uint8_t* bin, float* globIn, int16_t* policy, float* globT, int8_t* value, int32_t* meta) {
  Rows& R = ((Selfplay*)h)->rows;
  memcpy(meta, R.meta.data(), R.meta.size() * 4);
  memcpy(bin, R.bin.data(), R.bin.size());
  memcpy(globIn, R.globIn.data(), R.globIn.size() * 4);
  memcpy(policy, R.policy.data(), R.policy.size() * 2);
  memcpy(globT, R.globT.data(), R.globT.size() * 4);
  memcpy(value, R.value.data(), R.value.size());
  return R.n;
}
int ora_sizeof_node() { return (int)sizeof(Node); }

// Canonical breadth-first export (same algorithm and word layout as the device
// kGameTree): nodes [maxNodes][24] u32, edges [maxNodes][P][3] u32.
int ora_sp_game_tree(void* h, int slot, int maxNodes, uint32_t* out, uint32_t* edges) {
  Selfplay* s = (Selfplay*)h;
  Game& gm = s->games[slot];
  const int P = s->cfg.g.P;
  if(gm.rootIdx < 0)
    return 0;
  std::vector<int> order;
  order.push_back(gm.rootIdx);
  auto f2u = [](float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
  };
  size_t head = 0;
  while(head < order.size() && (int)head < maxNodes) {
    const int idx = order[head];
    const Node& x = gm.nodes[idx];
    uint32_t* o = out + head * 24;
    memset(o, 0, 24 * 4);
    o[0] = x.visits;
    o[1] = f2u(x.weightSum);
    o[2] = f2u(x.weightSqSum);
    o[3] = f2u(x.utilityAvg);
    o[4] = f2u(x.utilitySqAvg);
    o[5] = f2u(x.winLossAvg);
    o[6] = f2u(x.nnWin);
    o[7] = f2u(x.nnLoss);
    o[8] = f2u(x.lastSvbDelta);
    o[9] = f2u(x.lastSvbWeight);
    o[10] = (uint32_t)x.numChildren | ((uint32_t)x.nextPla << 16) | ((uint32_t)x.flags << 24);
    o[11] = (uint32_t)x.key0;
    o[12] = (uint32_t)(x.key0 >> 32);
    o[13] = (uint32_t)x.key1;
    o[14] = (uint32_t)(x.key1 >> 32);
    if(x.svbEntry >= 0) {
      uint64_t sk = gm.svbKey[x.svbEntry];
      uint64_t sd = (uint64_t)gm.svbDelta[x.svbEntry], sw = (uint64_t)gm.svbWeight[x.svbEntry];
      o[15] = (uint32_t)sk;
      o[16] = (uint32_t)(sk >> 32);
      o[17] = (uint32_t)sd;
      o[18] = (uint32_t)(sd >> 32);
      o[19] = (uint32_t)sw;
      o[20] = (uint32_t)(sw >> 32);
    }
    for(int i = 0; i < x.numChildren; i++) {
      const int c = (int)gm.edgeChild[(size_t)idx * P + i];
      int ci = -1;
      for(size_t q = 0; q < order.size(); q++)
        if(order[q] == c) {
          ci = (int)q;
          break;
        }
      if(ci < 0 && (int)order.size() < maxNodes) {
        order.push_back(c);
        ci = (int)order.size() - 1;
      }
      uint32_t* eo = edges + (head * P + i) * 3;
      eo[0] = (uint32_t)ci;
      eo[1] = gm.edgeVisits[(size_t)idx * P + i];
      eo[2] = gm.edgeMove[(size_t)idx * P + i];
    }
    head++;
  }
  return (int)order.size();
}

}  // extern "C"
