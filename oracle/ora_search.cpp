// ORACLE (test infrastructure only) — MCTS and self-play restatement.
// Semantics follow the reference search with Coffee utility (win/loss only):
//   playoutDescend            search.cpp:936-1165
//   allocateOrFindNode        search.cpp:704-759   (graph search, SVB attach)
//   maybeCatchUpEdgeVisits    search.cpp:1169-1207
//   selectBestChildToDescend  searchexplorehelpers.cpp:304-451
//   getExploreSelectionValue* searchexplorehelpers.cpp:27-207
//   getFpuValueForChildren... searchexplorehelpers.cpp:245-301
//   addLeafValue / recompute  searchupdatehelpers.cpp:12-328
//   downweightBadChildren...  searchupdatehelpers.cpp:330-419
//   maybeAddPolicyNoiseAndTemp searchhelpers.cpp:51-222
//   getPlaySelectionValues    searchresults.cpp:63-309, LCB searchhelpers.cpp:469-521
//   getChosenMoveLoc          searchresults.cpp:435-453, chooseIndexWithTemperature searchhelpers.cpp:11-49
//   makeMove (tree reuse)     search.cpp:262-330, beginSearch :514-694
//   Play::runGame targets     play.cpp:635-704, :1262-1460
//   TrainingWriteBuffers::addRow trainingwrite.cpp:316-565
// plus SPEC decisions.  Reductions over children use treeSum64.
#include "ora_search.h"

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstring>

namespace ora {

// std::min / std::max over the search's arithmetic type (mixed float / real operands)
template <class A, class B>
inline real rmin(A a, B b) {
  return std::min<real>((real)a, (real)b);
}
template <class A, class B>
inline real rmax(A a, B b) {
  return std::max<real>((real)a, (real)b);
}

// Transposition and SVB tables: nextPow2(2 * nodeCap) entries each, as the device
// (selfplay.cpp ttCap / svbCap).  Both hold at most one entry per live node, so a
// power-of-two size above 2 x nodeCap keeps every linear probe short and terminating.
static int tableCapFor(int nodeCap) {
  int c = 1;
  while(c < 2 * nodeCap)
    c <<= 1;
  return c;
}

// SPEC B27: subtree-value-bias sums are kept in 64-bit fixed point (2^-32 units)
// so that concurrent/unordered updates are exact and order independent.
inline int64_t svbQ(real x) { return std::llrint(x * 4294967296.0f); }
inline real svbF(int64_t v) { return (real)v * (1.0f / 4294967296.0f); }
static const uint64_t SVB_SEED = 0x5b5b5b5b5b5b5b5bULL;

// ---------------------------------------------------------------------------
// Fake network: a deterministic function of the (symmetrised) input planes.
void packPlanes(const Geom& g, const float* bin, uint64_t* words) {
  int nbits = NUM_SPATIAL * g.A, nw = (nbits + 63) / 64;
  for(int i = 0; i < nw; i++)
    words[i] = 0;
  for(int i = 0; i < nbits; i++)
    if(bin[i] != 0.0f)
      words[i >> 6] |= 1ULL << (i & 63);
}

void fakeNet(const Geom& g, const float* bin, float* policy, float* value, float* misc) {
  uint64_t w[32];
  packPlanes(g, bin, w);
  int nw = (NUM_SPATIAL * g.A + 63) / 64;
  uint64_t h = 0x243f6a8885a308d3ULL;
  for(int i = 0; i < nw; i++)
    h = mix64(h ^ w[i]);
  for(int j = 0; j < g.P + 4; j++) {
    uint64_t v = mix64(h + (uint64_t)j * 0x9e3779b97f4a7c15ULL);
    int q = (int)((v >> 40) & 0xffffu);
    if(j < g.P)
      policy[j] = ((float)q - 32768.0f) * (1.0f / 8192.0f);
    else if(j < g.P + 2)
      value[j - g.P] = ((float)q - 32768.0f) * (1.0f / 16384.0f);
    else
      misc[j - g.P - 2] = ((float)q - 32768.0f) * (1.0f / 16384.0f);
  }
}

// ---------------------------------------------------------------------------
namespace {

inline int svbIdxMove0(int pos) { return pos; }
inline int svbIdxMove1(int pos) { return (MAX_P + 1) + pos; }
inline int svbIdxPla(int pla) { return 2 * (MAX_P + 1) + pla; }
inline int svbIdxPat(int color, int wy, int wx) { return 2 * (MAX_P + 1) + 3 + color * 25 + wy * 5 + wx; }

static void packBitsBE(const float* v, int len, uint8_t* out);

struct Ctx {
  Selfplay& s;
  Game& gm;
  const Geom& g;
  const SearchParams& sp;
  // sp: this move's parameters (a cheap search without recorded rows drops the root
  // noise and root-specific settings, play.cpp:1024-1037)
  Ctx(Selfplay& s_, Game& gm_) : s(s_), gm(gm_), g(s_.cfg.g), sp(gm_.noNoise ? s_.spCheap : s_.cfg.sp) {}
  Ctx(Selfplay& s_, Game& gm_, const SearchParams& p) : s(s_), gm(gm_), g(s_.cfg.g), sp(p) {}

  Node& N(int i) { return gm.nodes[i]; }
  uint32_t& EC(int n, int i) { return gm.edgeChild[(size_t)n * g.P + i]; }
  uint32_t& EV(int n, int i) { return gm.edgeVisits[(size_t)n * g.P + i]; }
  uint16_t& EM(int n, int i) { return gm.edgeMove[(size_t)n * g.P + i]; }
  float* POL(int n) { return &gm.policy[(size_t)n * g.P]; }

  // --- transposition table (SearchNodeTable, searchnodetable.h) ---
  int ttCap() const { return (int)gm.ttNode.size(); }
  int ttFind(uint64_t k0, uint64_t k1) {
    int mask = ttCap() - 1;
    for(int i = (int)(k0 & (uint64_t)mask);; i = (i + 1) & mask) {
      if(gm.ttNode[i] < 0)
        return -1;
      if(gm.ttKey0[i] == k0 && gm.ttKey1[i] == k1)
        return gm.ttNode[i];
    }
  }
  void ttInsert(uint64_t k0, uint64_t k1, int node) {
    int mask = ttCap() - 1;
    int i = (int)(k0 & (uint64_t)mask);
    while(gm.ttNode[i] >= 0)
      i = (i + 1) & mask;
    gm.ttKey0[i] = k0;
    gm.ttKey1[i] = k1;
    gm.ttNode[i] = node;
  }
  void ttClear() { std::fill(gm.ttNode.begin(), gm.ttNode.end(), -1); }

  // --- subtree value bias table (subtreevaluebiastable.cpp:61-78) ---
  int svbFindOrInsert(std::vector<uint64_t>& key, std::vector<int64_t>& d, std::vector<int64_t>& w,
                      std::vector<uint8_t>& used, uint64_t k) {
    int mask = (int)key.size() - 1;
    for(int i = (int)(k & (uint64_t)mask);; i = (i + 1) & mask) {
      if(!used[i]) {
        used[i] = 1;
        key[i] = k;
        d[i] = 0;
        w[i] = 0;
        return i;
      }
      if(key[i] == k)
        return i;
    }
  }
  // Key (SPEC a19): ZOBRIST_MOVE_LOCS[parentPrev][0] ^ [prev][1] ^ 5x5 local
  // pattern around `prev` on the board BEFORE it was played ^ mover.
  uint64_t svbKey(const Board& before, int parentPrevPos, int movePos, int mover) {
    const std::vector<uint64_t>& Z = s.svbZ;
    uint64_t h = Z[svbIdxMove0(parentPrevPos)] ^ Z[svbIdxMove1(movePos)] ^ Z[svbIdxPla(mover)];
    int cell = movePos % g.A;
    int x = cell % g.X, y = cell / g.X;
    for(int wy = 0; wy < 5; wy++)
      for(int wx = 0; wx < 5; wx++) {
        int xx = x + wx - 2, yy = y + wy - 2;
        int col = (xx >= 0 && xx < g.X && yy >= 0 && yy < g.Y) ? before.c[yy * g.X + xx] : 3;
        h ^= Z[svbIdxPat(col, wy, wx)];
      }
    return h != 0 ? h : 1;  // 0 is the device table's empty sentinel
  }

  int allocNode(uint8_t nextPla, H128 key, bool terminal) {
    int i = gm.nodeCount++;
    if(i >= (int)gm.nodes.size()) {
      fprintf(stderr, "oracle: node pool overflow\n");
      abort();
    }
    Node& n = N(i);
    memset(&n, 0, sizeof(Node));
    n.svbEntry = -1;
    n.nextPla = nextPla;
    n.flags = terminal ? 2 : 0;
    n.key0 = key.h0;
    n.key1 = key.h1;
    return i;
  }

  static real childWeight(uint32_t edgeVisits, uint32_t childVisits, real rawWeight) {
    // NodeStats::childWeight searchnode.h:59-61
    return rawWeight * ((real)edgeVisits / (real)std::max(childVisits, 1u));
  }

  // --- addLeafValue searchupdatehelpers.cpp:12-82 (weight 1, Coffee utility = winLoss) ---
  void addLeafValue(int ni, real wl, bool isTerminal, bool assumeNoExisting) {
    Node& n = N(ni);
    real utility = wl;
    if(sp.subtreeValueBiasFactor != 0.0f && !isTerminal && n.svbEntry >= 0) {
      real d = svbF(gm.svbDelta[n.svbEntry]), w = svbF(gm.svbWeight[n.svbEntry]);
      if(w > 0.001f)
        utility = utility + (sp.subtreeValueBiasFactor * d) / w;
    }
    real usq = utility * utility;
    if(assumeNoExisting) {
      n.winLossAvg = wl;
      n.utilityAvg = utility;
      n.utilitySqAvg = usq;
      n.weightSqSum = 1.0f;
      n.weightSum = 1.0f;
      n.visits += 1;
    } else {
      real oldW = n.weightSum, newW = oldW + 1.0f;
      n.winLossAvg = (n.winLossAvg * oldW + wl) / newW;
      n.utilityAvg = (n.utilityAvg * oldW + utility) / newW;
      n.utilitySqAvg = (n.utilitySqAvg * oldW + usq) / newW;
      n.weightSqSum = n.weightSqSum + 1.0f;
      n.weightSum = newW;
      n.visits += 1;
    }
  }

  real cdf(real z) {
    // DistributionTable::getCdf distributiontable.h (size 2000, [-50,50])
    real d = (1999.0f * (z - (-50.0f))) / 100.0f;
    if(d <= 0.0f)
      return 0.0f;
    int idx = (int)d;
    if(idx >= 1999)
      return 1.0f;
    real lambda = d - (real)idx;
    real y0 = T.cdf[idx], y1 = T.cdf[idx + 1];
    return y0 + lambda * (y1 - y0);
  }

  // --- recomputeNodeStats searchupdatehelpers.cpp:151-328 ---
  void recompute(int ni, int numVisitsToAdd, bool isRoot) {
    Node& n = N(ni);
    const int k = n.numChildren;
    real wAdj[MAX_P], selfU[MAX_P], wlv[MAX_P], uv[MAX_P], usqv[MAX_P], wsqv[MAX_P], tmp[MAX_P];
    bool good[MAX_P];
    int numGood = 0;
    real maxW = 0.0f;
    for(int i = 0; i < k; i++) {
      const Node& c = N((int)EC(ni, i));
      uint32_t ev = EV(ni, i);
      good[i] = c.visits > 0 && c.weightSum > 0.0f && ev > 0;
      if(good[i]) {
        numGood++;
        selfU[i] = n.nextPla == 2 ? c.utilityAvg : -c.utilityAvg;
        wAdj[i] = childWeight(ev, c.visits, c.weightSum);
        if(wAdj[i] > maxW)
          maxW = wAdj[i];
      } else {
        selfU[i] = 0.0f;
        wAdj[i] = 0.0f;
      }
    }
    real origTotal = treeSum64(wAdj, k);
    real currentTotal = origTotal;
    real amountToSubtract = 0.0f, amountToPrune = 0.0f;
    if(isRoot && sp.rootNoiseEnabled) {
      amountToSubtract = rmin(sp.chosenMoveSubtract, maxW / 64.0f);
      amountToPrune = rmin(sp.chosenMovePrune, maxW / 64.0f);
    }
    // downweightBadChildrenAndNormalizeWeight (valueWeightExponent != 0 branch)
    if(numGood > 0 && currentTotal > 0.0f) {
      real stdev[MAX_P];
      for(int i = 0; i < k; i++) {
        stdev[i] = good[i] ? std::sqrt(1e-8f + 1.0f / (1.5f * std::sqrt(wAdj[i]))) : 0.0f;
        tmp[i] = good[i] ? selfU[i] * wAdj[i] : 0.0f;
      }
      real simpleValue = treeSum64(tmp, k) / currentTotal;
      for(int i = 0; i < k; i++) {
        if(!good[i]) {
          tmp[i] = 0.0f;
          continue;
        }
        if(wAdj[i] < amountToPrune) {
          tmp[i] = 0.0f;
          continue;
        }
        real nw = wAdj[i] - amountToSubtract;
        if(nw <= 0.0f)
          nw = 0.0f;
        real z = (selfU[i] - simpleValue) / stdev[i];
        real p = cdf(z) + 0.0001f;
        real f = sp.valueWeightExponent == 0.5f ? std::sqrt(p) : kPowf(p, (real)sp.valueWeightExponent);
        tmp[i] = nw * f;
      }
      real totalNew = treeSum64(tmp, k);
      real factor = currentTotal / totalNew;
      for(int i = 0; i < k; i++)
        wAdj[i] = tmp[i] * factor;
    }
    for(int i = 0; i < k; i++) {
      if(!good[i]) {
        wlv[i] = uv[i] = usqv[i] = wsqv[i] = 0.0f;
        continue;
      }
      const Node& c = N((int)EC(ni, i));
      real ws = wAdj[i] / c.weightSum;
      wlv[i] = wAdj[i] * c.winLossAvg;
      uv[i] = wAdj[i] * c.utilityAvg;
      usqv[i] = wAdj[i] * c.utilitySqAvg;
      wsqv[i] = (ws * ws) * c.weightSqSum;
    }
    real winLossSum = treeSum64(wlv, k);
    real utilitySum = treeSum64(uv, k);
    real utilitySqSum = treeSum64(usqv, k);
    real weightSqSum = treeSum64(wsqv, k);
    real weightSum = currentTotal;
    real wl = n.nnWin - n.nnLoss;
    real utility = wl;
    if(sp.subtreeValueBiasFactor != 0.0f && n.svbEntry >= 0) {
      int e = n.svbEntry;
      if(currentTotal > 1e-10f) {
        real utilityChildren = utilitySum / currentTotal;
        real svbW = kPowf(origTotal, (real)sp.subtreeValueBiasWeightExponent);
        real svbD = (utilityChildren - utility) * svbW;
        gm.svbDelta[e] += svbQ(svbD) - svbQ(n.lastSvbDelta);
        gm.svbWeight[e] += svbQ(svbW) - svbQ(n.lastSvbWeight);
        n.lastSvbDelta = svbD;
        n.lastSvbWeight = svbW;
      }
      real d = svbF(gm.svbDelta[e]), w = svbF(gm.svbWeight[e]);
      if(w > 0.001f)
        utility = utility + (sp.subtreeValueBiasFactor * d) / w;
    }
    winLossSum = winLossSum + wl;
    utilitySum = utilitySum + utility;
    utilitySqSum = utilitySqSum + utility * utility;
    weightSqSum = weightSqSum + 1.0f;
    weightSum = weightSum + 1.0f;
    n.winLossAvg = winLossSum / weightSum;
    n.utilityAvg = utilitySum / weightSum;
    n.utilitySqAvg = utilitySqSum / weightSum;
    n.weightSqSum = weightSqSum;
    n.weightSum = weightSum;
    n.visits += (uint32_t)numVisitsToAdd;
  }

  // --- getFpuValueForChildrenAssumeVisited searchexplorehelpers.cpp:245-301 ---
  real fpuValue(int ni, int pla, bool isRoot, real probMass) {
    const Node& n = N(ni);
    real parentUtility = n.utilityAvg;
    real forFpu = parentUtility;
    if(sp.fpuParentWeightByVisitedPolicy) {
      real pw = sp.fpuParentWeightByVisitedPolicyPow == 2.0f ? probMass * probMass
                                                              : kPowf(probMass, (real)sp.fpuParentWeightByVisitedPolicyPow);
      real avgWeight = rmin(1.0f, pw);
      forFpu = avgWeight * parentUtility + (1.0f - avgWeight) * (n.nnWin - n.nnLoss);
    }
    real redMax = isRoot ? sp.rootFpuReductionMax : sp.fpuReductionMax;
    real lossProp = isRoot ? sp.rootFpuLossProp : sp.fpuLossProp;
    real reduction = redMax * std::sqrt(probMass);
    real fpu = pla == 2 ? forFpu - reduction : forFpu + reduction;
    real lossValue = pla == 2 ? -1.0f : 1.0f;
    fpu = fpu + (lossValue - fpu) * lossProp;
    return fpu;
  }

  real exploreScaling(real totalChildWeight) {
    real c = sp.cpuctExploration;
    if(sp.cpuctExplorationLog != 0.0f)
      c = c + sp.cpuctExplorationLog * kLogf((totalChildWeight + sp.cpuctExplorationBase) / sp.cpuctExplorationBase);
    return c * std::sqrt(totalChildWeight + 0.01f);
  }

  // --- selectBestChildToDescend searchexplorehelpers.cpp:304-451 ---
  // returns slot (k = new child), sets newPos; -1 if nothing selectable.
  int selectBest(int ni, const float* pol, bool isRoot, int& newPos) {
    const Node& n = N(ni);
    const int k = n.numChildren;
    int pla = n.nextPla;
    real probs[MAX_P], cw[MAX_P];
    bool hasChild[MAX_P];
    memset(hasChild, 0, sizeof(hasChild));
    for(int i = 0; i < k; i++) {
      const Node& c = N((int)EC(ni, i));
      real p = pol[EM(ni, i)];
      probs[i] = p < 0.0f ? 0.0f : p;
      cw[i] = p < 0.0f ? 0.0f : childWeight(EV(ni, i), c.visits, c.weightSum);
      hasChild[EM(ni, i)] = true;
    }
    real probMass = treeSum64(probs, k);
    real total = treeSum64(cw, k);
    real fpu = fpuValue(ni, pla, isRoot, probMass);
    real scaling = exploreScaling(total);
    real best = -INFINITY;
    int bestSlot = -1;
    for(int i = 0; i < k; i++) {
      const Node& c = N((int)EC(ni, i));
      real p = pol[EM(ni, i)];
      real v;
      if(p < 0.0f)
        v = -INFINITY;  // POLICY_ILLEGAL_SELECTION_VALUE
      else {
        real w = cw[i];
        real u = (c.visits == 0 || w <= 0.0f) ? fpu : c.utilityAvg;
        if(isRoot && sp.rootDesiredPerChildVisitsCoeff > 0.0f && p > 0.0f &&
           w < std::sqrt((p * total) * sp.rootDesiredPerChildVisitsCoeff))
          v = 1e20f;
        else
          v = (scaling * p) / (1.0f + w) + (pla == 2 ? u : -u);
      }
      if(v > best) {
        best = v;
        bestSlot = i;
      }
    }
    real bestNewProb = -1.0f;
    int bestNew = -1;
    for(int pos = 0; pos < g.P; pos++) {
      if(hasChild[pos])
        continue;
      real p = pol[pos];
      if(p < 0.0f)
        continue;
      if(p > bestNewProb) {
        bestNewProb = p;
        bestNew = pos;
      }
    }
    newPos = -1;
    if(bestNew >= 0) {
      real v = (scaling * bestNewProb) / 1.0f + (pla == 2 ? fpu : -fpu);
      if(v > best) {
        best = v;
        bestSlot = k;
        newPos = bestNew;
      }
    }
    return bestSlot;
  }

  // --- playoutDescend (select half) ---
  void descend() {
    gm.pathNode.clear();
    gm.pathSlot.clear();
    Board b = gm.root;
    int ni = gm.rootIdx;
    while(true) {
      Node& n = N(ni);
      if(n.flags & 2) {
        gm.leafKind = LEAF_TERMINAL;
        gm.leafNode = ni;
        gm.leafBoard = b;
        break;
      }
      bool isRoot = ni == gm.rootIdx;
      const float* pol = isRoot ? gm.rootNoised.data() : POL(ni);
      int newPos = -1;
      int slot = selectBest(ni, pol, isRoot, newPos);
      if(slot < 0) {
        gm.leafKind = LEAF_NOCHILD;
        gm.leafNode = ni;
        break;
      }
      if(slot == n.numChildren) {
        int cell = newPos % g.A, dir = newPos / g.A;
        Board before = b;
        playMove(g, b, cell, dir);
        H128 key = stateHash(g, b);
        int child = sp.useGraphSearch ? ttFind(key.h0, key.h1) : -1;
        if(child < 0) {
          child = allocNode(b.pla, key, b.finished != 0);
          if(sp.subtreeValueBiasFactor != 0.0f && before.histCell[0] >= 0) {
            int ppos = before.histDir[0] * g.A + before.histCell[0];
            uint64_t k = svbKey(before, ppos, newPos, before.pla);
            N(child).svbEntry = svbFindOrInsert(gm.svbKey, gm.svbDelta, gm.svbWeight, gm.svbUsed, k);
          }
          if(sp.useGraphSearch)
            ttInsert(key.h0, key.h1, child);
        }
        Node& nn = N(ni);  // (re-fetch: vector storage is fixed-size, no realloc)
        EC(ni, slot) = (uint32_t)child;
        EV(ni, slot) = 0;
        EM(ni, slot) = (uint16_t)newPos;
        nn.numChildren++;
        gm.pathNode.push_back(ni);
        gm.pathSlot.push_back(slot);
        if(N(child).visits > 0) {  // maybeCatchUpEdgeVisits: edgeVisits 0 < childVisits
          gm.leafKind = LEAF_CATCHUP;
          gm.leafNode = child;
          break;
        }
        gm.leafNode = child;
        gm.leafBoard = b;
        gm.leafKind = (N(child).flags & 2) ? LEAF_TERMINAL : LEAF_NN;
        break;
      }
      int child = (int)EC(ni, slot);
      gm.pathNode.push_back(ni);
      gm.pathSlot.push_back(slot);
      if(EV(ni, slot) < N(child).visits) {
        gm.leafKind = LEAF_CATCHUP;
        gm.leafNode = child;
        break;
      }
      int mv = EM(ni, slot);
      playMove(g, b, mv % g.A, mv / g.A);
      ni = child;
    }
  }

  // NNEvaluator::evaluate post-processing nneval.cpp:702-815 + inverse symmetry
  // (copyOutputsWithSymmetry nninputs.cpp:349-357).
  void postprocess(const Board& b, int sym, const float* out, float* pol, float& whiteWin, float& whiteLoss) {
    if(g.X != g.Y)
      sym &= 3;
    real logit[MAX_P];
    bool legal[MAX_P];
    real mx = -1e25f;  // maxPolicy init nneval.cpp:709
    for(int pos = 0; pos < g.P; pos++) {
      int d = pos / g.A, cell = pos % g.A;
      legal[pos] = isLegal(g, b, cell, d);
      real v = legal[pos] ? out[symDir(d, sym) * g.A + symCell(g, cell, sym)] : -1e30f;
      logit[pos] = v;
      if(v > mx)
        mx = v;
    }
    real e[MAX_P];
    for(int pos = 0; pos < g.P; pos++)
      e[pos] = kExpf(logit[pos] - mx);
    real sum = treeSum64(e, g.P);
    int legalCount = 0;
    for(int pos = 0; pos < g.P; pos++)
      legalCount += legal[pos] ? 1 : 0;
    if(sum <= 0.0f) {
      real uniform = 1.0f / (real)legalCount;
      for(int pos = 0; pos < g.P; pos++)
        pol[pos] = legal[pos] ? uniform : -1.0f;
    } else {
      for(int pos = 0; pos < g.P; pos++)
        pol[pos] = legal[pos] ? e[pos] / sum : -1.0f;
    }
    real wlg = out[g.P], llg = out[g.P + 1];
    real m = rmax(wlg, llg);
    real wp = kExpf(wlg - m), lp = kExpf(llg - m);
    real ps = wp + lp;
    wp = wp / ps;
    lp = lp / ps;
    if(b.pla == 2) {
      whiteWin = wp;
      whiteLoss = lp;
    } else {
      whiteWin = lp;
      whiteLoss = wp;
    }
  }

  real interpolateEarly(real halflife, real earlyValue, real value) {
    // Search::interpolateEarly searchhelpers.cpp:463-467
    real rawHalflives = (real)gm.root.turn / halflife;
    real halflives = rawHalflives * (19.0f / std::sqrt((real)(g.X * g.Y)));
    return value + (earlyValue - value) * kPowf((real)0.5f, halflives);
  }

  // maybeAddPolicyNoiseAndTemp searchhelpers.cpp:122-222 (root only)
  void noiseAndTemp(const float* raw, float* out) {
    for(int pos = 0; pos < g.P; pos++)
      out[pos] = raw[pos];
    if(sp.rootPolicyTemperature != 1.0f || sp.rootPolicyTemperatureEarly != 1.0f) {
      real t = interpolateEarly(sp.chosenMoveTemperatureHalflife, sp.rootPolicyTemperatureEarly, sp.rootPolicyTemperature);
      real mx = 0.0f;
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] > mx)
          mx = out[pos];
      real logMax = kLogf(mx);
      real invTemp = 1.0f / t;
      real sum = 0.0f;
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] > 0.0f) {
          real p = kExpf((kLogf(out[pos]) - logMax) * invTemp);
          out[pos] = p;
          sum = sum + p;
        }
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] >= 0.0f)
          out[pos] = out[pos] / sum;
    }
    if(sp.rootNoiseEnabled) {
      // computeDirichletAlphaDistribution searchhelpers.cpp:51-91
      real alpha[MAX_P];
      int legalCount = 0;
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] >= 0.0f)
          legalCount++;
      real logSum = 0.0f;
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] >= 0.0f) {
          alpha[pos] = kLogf(rmin(0.01f, out[pos]) + 1e-20f);
          logSum = logSum + alpha[pos];
        }
      real logMean = logSum / (real)legalCount;
      real propSum = 0.0f;
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] >= 0.0f) {
          alpha[pos] = rmax(0.0f, alpha[pos] - logMean);
          propSum = propSum + alpha[pos];
        }
      real uniform = 1.0f / (real)legalCount;
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] >= 0.0f)
          alpha[pos] = propSum <= 0.0f ? uniform : 0.5f * (alpha[pos] / propSum + uniform);
      // addDirichletNoise searchhelpers.cpp:93-120.  SPEC a24: one draw from the
      // game stream seeds an independent sub-stream per move (parallel on device).
      real r[MAX_P];
      real rSum = 0.0f;
      const uint64_t base = gm.rng.next();
      for(int pos = 0; pos < g.P; pos++) {
        if(out[pos] >= 0.0f) {
          Rng sub;
          sub.seed = mix64(base ^ ((uint64_t)(pos + 1) * 0x9e3779b97f4a7c15ULL));
          sub.ctr = 0;
          r[pos] = sub.gamma(alpha[pos] * sp.rootDirichletNoiseTotalConcentration);
          rSum = rSum + r[pos];
        } else
          r[pos] = 0.0f;
      }
      for(int pos = 0; pos < g.P; pos++)
        r[pos] = r[pos] / rSum;
      real w = sp.rootDirichletNoiseWeight;
      for(int pos = 0; pos < g.P; pos++)
        if(out[pos] >= 0.0f)
          out[pos] = r[pos] * w + out[pos] * (1.0f - w);
    }
  }

  // getSelfUtilityLCBAndRadius searchhelpers.cpp:469-521 (utilityRangeRadius = 1)
  void lcbAndRadius(int pla, int ci, uint32_t ev, real& lcb, real& radius) {
    const Node& c = N(ci);
    radius = 2.0f * 1.0f * sp.lcbStdevs;
    lcb = -radius;
    real ws = childWeight(ev, c.visits, c.weightSum);
    real wsq = childWeight(ev, c.visits, c.weightSqSum);
    if(c.visits == 0 || ws <= 0.0f || wsq <= 0.0f)
      return;
    real u = c.utilityAvg, usq = c.utilitySqAvg;
    real ess = (ws * ws) / wsq;
    real priorWeight = ws / ((ess * ess) * ess);
    usq = rmax(usq, u * u + 1e-8f);
    usq = (usq * ws + (usq + 1.0f) * priorWeight) / (ws + priorWeight);
    ws = ws + priorWeight;
    wsq = wsq + priorWeight * priorWeight;
    ess = (ws * ws) / wsq;
    real selfU = pla == 2 ? u : -u;
    real variance = usq - u * u;
    real stdev = std::sqrt(variance / ess);
    radius = stdev * sp.lcbStdevs;
    lcb = selfU - radius;
  }

  // getPlaySelectionValues searchresults.cpp:63-309 on the root.
  // Fills pos[] and vals[]; returns count (0 = failure).  useLcb: searchParams.useLcbForSelection
  // at the call (self-play turns it off for the move choice only, play.cpp:1040-1046, :1073-1076).
  int playSelectionValues(real scaleMaxToAtLeast, bool allowDirectPolicyMoves, int* posOut, real* vals,
                          bool useLcb) {
    return playSelectionValuesAt(gm.rootIdx, gm.rootNoised.data(), true, scaleMaxToAtLeast, allowDirectPolicyMoves,
                                 posOut, vals, useLcb);
  }

  // The same on any node (tree positions, play.cpp:736-745): the node's own network
  // policy (getPolicyProbsMaybeNoised: noise only at the root); the reduction of
  // over-explored children (:136-186) and direct policy moves (:242-276) are root-only.
  int playSelectionValuesAt(int ri, const float* pol, bool isRoot, real scaleMaxToAtLeast,
                            bool allowDirectPolicyMoves, int* posOut, real* vals, bool useLcb) {
    const Node& n = N(ri);
    const int k = n.numChildren;
    int pla = n.nextPla;
    real cw[MAX_P];
    for(int i = 0; i < k; i++) {
      const Node& c = N((int)EC(ri, i));
      cw[i] = childWeight(EV(ri, i), c.visits, c.weightSum);
      posOut[i] = EM(ri, i);
      vals[i] = cw[i];
    }
    real total = treeSum64(cw, k);
    int numChildren = k;
    int bestIdx = 0;
    real bestWeight = -1e30f;
    {
      real maxGood = -1e30f;
      for(int i = 0; i < k; i++) {
        real ev = (real)EV(ri, i);
        real gdn = vals[i] * rmax(0.0f, ev - 1.0f) / rmax(1.0f, ev) + 2.0f * pol[posOut[i]];
        if(gdn > maxGood) {
          maxGood = gdn;
          bestWeight = vals[i];
          bestIdx = i;
        }
      }
    }
    if(isRoot && k > 0) {
      real fpu = fpuValue(ri, pla, true, 1.0f);
      real scaling = exploreScaling(total);
      // getExploreSelectionValueOfChild for the best child, isDuringSearch = false
      const Node& bc = N((int)EC(ri, bestIdx));
      real bp = pol[posOut[bestIdx]];
      real bw = cw[bestIdx];
      real bu = (bc.visits == 0 || bw <= 0.0f) ? fpu : bc.utilityAvg;
      real bestValue = bp < 0.0f ? -INFINITY : (scaling * bp) / (1.0f + bw) + (pla == 2 ? bu : -bu);
      for(int i = 0; i < k; i++) {
        if(i == bestIdx)
          continue;
        // getReducedPlaySelectionWeight searchexplorehelpers.cpp:209-243
        const Node& c = N((int)EC(ri, i));
        real w = cw[i];
        real reduced;
        if(c.visits == 0 || w <= 0.0f)
          reduced = 0.0f;
        else {
          real p = pol[posOut[i]];
          real wanted;
          if(p < 0.0f)
            wanted = 0.0f;
          else {
            real valueComponent = pla == 2 ? c.utilityAvg : -c.utilityAvg;
            real exploreComponent = bestValue - valueComponent;
            real exploreComponentScaling = scaling * p;
            if(exploreComponent <= 0.0f)
              wanted = INFINITY;
            else {
              wanted = exploreComponentScaling / exploreComponent - 1.0f;
              if(wanted < 0.0f)
                wanted = 0.0f;
            }
          }
          reduced = w > wanted ? wanted : w;
        }
        vals[i] = std::ceil(reduced);
      }
    }
    if(useLcb && k > 0) {
      real lcb[MAX_P], rad[MAX_P];
      real bestLcb = -1e10f;
      int bestLcbIdx = -1;
      for(int i = 0; i < k; i++) {
        lcbAndRadius(pla, (int)EC(ri, i), EV(ri, i), lcb[i], rad[i]);
        real w = vals[i];
        if(w > 0.0f && w >= sp.minVisitPropForLCB * bestWeight && lcb[i] > bestLcb) {
          bestLcb = lcb[i];
          bestLcbIdx = i;
        }
      }
      if(bestLcbIdx >= 0) {
        real adjusted = vals[bestLcbIdx];
        for(int i = 0; i < k; i++) {
          if(i == bestLcbIdx)
            continue;
          real excess = bestLcb - lcb[i];
          if(excess < 0.0f)
            continue;
          real rf = (rad[i] + excess) / (rad[i] + 0.20f * excess);
          real lbound = (rf * rf) * vals[i];
          if(lbound > adjusted)
            adjusted = lbound;
        }
        vals[bestLcbIdx] = adjusted;
      }
    }
    if(numChildren == 0) {
      if(!allowDirectPolicyMoves || !isRoot)
        return 0;
      for(int p = 0; p < g.P; p++) {
        if(!isLegal(g, gm.root, p % g.A, p / g.A) || pol[p] < 0.0f)
          continue;
        posOut[numChildren] = p;
        vals[numChildren] = pol[p];
        numChildren++;
      }
      if(numChildren == 0)
        return 0;
    }
    real mx = 0.0f;
    for(int i = 0; i < numChildren; i++)
      if(vals[i] > mx)
        mx = vals[i];
    if(mx <= 0.0f)
      return 0;
    real amountToSubtract = rmin(sp.chosenMoveSubtract, mx / 64.0f);
    real amountToPrune = rmin(sp.chosenMovePrune, mx / 64.0f);
    real newMax = mx - amountToSubtract;
    for(int i = 0; i < numChildren; i++) {
      if(vals[i] < amountToPrune)
        vals[i] = 0.0f;
      else {
        vals[i] = vals[i] - amountToSubtract;
        if(vals[i] <= 0.0f)
          vals[i] = 0.0f;
      }
    }
    if(newMax < scaleMaxToAtLeast)
      for(int i = 0; i < numChildren; i++)
        vals[i] = vals[i] * (scaleMaxToAtLeast / newMax);
    return numChildren;
  }

  // chooseIndexWithTemperature searchhelpers.cpp:11-49 with our stream.
  int chooseIndex(const real* vals, int n, real temperature) {
    real mx = 0.0f;
    for(int i = 0; i < n; i++)
      if(vals[i] > mx)
        mx = vals[i];
    if(temperature <= 1.0e-4f) {
      real best = vals[0];
      int bi = 0;
      for(int i = 1; i < n; i++)
        if(vals[i] > best) {
          best = vals[i];
          bi = i;
        }
      return bi;
    }
    real pr[MAX_P];
    real logMax = kLogf(mx);
    real sum = 0.0f;
    for(int i = 0; i < n; i++) {
      pr[i] = vals[i] <= 0.0f ? 0.0f : kExpf((kLogf(vals[i]) - logMax) / temperature);
      sum = sum + pr[i];
    }
    real d = gm.rng.uni() * sum;  // Rand::nextUInt(relProbs) rand.h:244-262
    real acc = 0.0f;
    for(int i = 0; i < n; i++) {
      acc = acc + pr[i];
      if(acc > d)
        return i;
    }
    return n - 1;
  }

  void mark(int root, std::vector<uint8_t>& live) {
    std::vector<int> st;
    st.push_back(root);
    live[root] = 1;
    while(!st.empty()) {
      int v = st.back();
      st.pop_back();
      for(int i = 0; i < N(v).numChildren; i++) {
        int c = (int)EC(v, i);
        if(!live[c]) {
          live[c] = 1;
          st.push_back(c);
        }
      }
    }
  }

  void clearTree() {
    gm.nodeCount = 0;
    gm.rootIdx = -1;
    ttClear();
    std::fill(gm.svbUsed.begin(), gm.svbUsed.end(), 0);
  }

  // Search::makeMove search.cpp:262-330 + deleteAllOld... :790-810 +
  // SubtreeValueBiasTable::clearUnusedSynchronous :47-59, as an in-place,
  // order-preserving compaction of the node pool (SPEC: GC).
  void reuseTree(int chosenPos) {
    int ri = gm.rootIdx;
    int child = -1;
    if(ri >= 0)
      for(int i = 0; i < N(ri).numChildren; i++)
        if(EM(ri, i) == chosenPos) {
          child = (int)EC(ri, i);
          break;
        }
    if(child < 0 || !(N(child).flags & 1)) {
      clearTree();
      return;
    }
    std::vector<uint8_t> live(gm.nodeCount, 0);
    mark(child, live);
    int liveCount = 0;
    for(int i = 0; i < gm.nodeCount; i++)
      liveCount += live[i];
    if(liveCount + sp.maxVisits + 2 > (int)gm.nodes.size()) {
      clearTree();
      return;
    }
    // removeSubtreeValueBias for every deleted table node and for the promoted
    // child (whose copy becomes the root without an SVB entry), in index order.
    for(int i = 0; i < gm.nodeCount; i++) {
      Node& n = N(i);
      if((live[i] && i != child) || n.svbEntry < 0)
        continue;
      int e = n.svbEntry;
      gm.svbDelta[e] -= svbQ(n.lastSvbDelta * sp.subtreeValueBiasFreeProp);
      gm.svbWeight[e] -= svbQ(n.lastSvbWeight * sp.subtreeValueBiasFreeProp);
    }
    N(child).svbEntry = -1;
    N(child).lastSvbDelta = 0.0f;
    N(child).lastSvbWeight = 0.0f;
    std::vector<int> newIdx(gm.nodeCount, -1);
    int j = 0;
    for(int i = 0; i < gm.nodeCount; i++)
      if(live[i])
        newIdx[i] = j++;
    for(int i = 0; i < gm.nodeCount; i++) {
      if(!live[i])
        continue;
      int d = newIdx[i];
      if(d != i) {
        gm.nodes[d] = gm.nodes[i];
        memcpy(&gm.edgeChild[(size_t)d * g.P], &gm.edgeChild[(size_t)i * g.P], sizeof(uint32_t) * g.P);
        memcpy(&gm.edgeVisits[(size_t)d * g.P], &gm.edgeVisits[(size_t)i * g.P], sizeof(uint32_t) * g.P);
        memcpy(&gm.edgeMove[(size_t)d * g.P], &gm.edgeMove[(size_t)i * g.P], sizeof(uint16_t) * g.P);
        memcpy(&gm.policy[(size_t)d * g.P], &gm.policy[(size_t)i * g.P], sizeof(float) * g.P);
      }
      for(int e = 0; e < N(d).numChildren; e++)
        EC(d, e) = (uint32_t)newIdx[EC(d, e)];
    }
    gm.nodeCount = liveCount;
    gm.rootIdx = newIdx[child];
    ttClear();
    for(int i = 0; i < gm.nodeCount; i++)
      if(i != gm.rootIdx)
        ttInsert(N(i).key0, N(i).key1, i);
    const size_t svbCap = gm.svbKey.size();
    std::vector<uint64_t> k2(svbCap, 0);
    std::vector<int64_t> d2(svbCap, 0), w2(svbCap, 0);
    std::vector<uint8_t> u2(svbCap, 0);
    for(int i = 0; i < gm.nodeCount; i++) {
      Node& n = N(i);
      if(n.svbEntry < 0)
        continue;
      int oe = n.svbEntry;
      int mask = (int)svbCap - 1;
      int slot = (int)(gm.svbKey[oe] & (uint64_t)mask);
      while(u2[slot] && k2[slot] != gm.svbKey[oe])
        slot = (slot + 1) & mask;
      if(!u2[slot]) {
        u2[slot] = 1;
        k2[slot] = gm.svbKey[oe];
        d2[slot] = gm.svbDelta[oe];
        w2[slot] = gm.svbWeight[oe];
      }
      n.svbEntry = slot;
    }
    gm.svbKey.swap(k2);
    gm.svbDelta.swap(d2);
    gm.svbWeight.swap(w2);
    gm.svbUsed.swap(u2);
  }

  // getSearchLimitsThisMove (play.cpp:871-1004) for the move about to be searched.
  // Returns clearBotBeforeSearchThisMove: self-play clears the tree before every
  // search (play.cpp:1941-1946, :1009-1010) except a cheap search whose rows are
  // not recorded (:920-925), which keeps the subtree of the previous move.
  bool setMoveLimits() {
    const SearchParams& b = s.cfg.sp;
    gm.visitLimit = b.maxVisits;
    gm.moveWeight = 1.0f;
    gm.noNoise = 0;
    bool clear = true;
    if(b.cheapSearchProb > 0.0f && gm.rng.uni() < b.cheapSearchProb) {
      gm.visitLimit = std::min(b.maxVisits, b.cheapSearchVisits);
      gm.moveWeight = 1.0f * b.cheapSearchTargetWeight;
      if(b.cheapSearchTargetWeight <= 0.0f) {
        clear = false;
        gm.noNoise = 1;
      }
    } else if(b.reduceVisits && (int)gm.turns.size() - gm.startTurn >= b.reduceVisitsThresholdLookback) {
      real mn = 1e20f, mx = -1e20f;
      for(int j = 0; j < b.reduceVisitsThresholdLookback; j++) {
        const real w = gm.turns[gm.turns.size() - 1 - j].rootWL;
        mn = w < mn ? w : mn;
        mx = w > mx ? w : mx;
      }
      real extreme = rmax(mn, -mx);
      if(extreme > 1.0f)
        extreme = 1.0f;
      const real through = extreme - b.reduceVisitsThreshold;
      if(through > 0.0f) {
        const real prop = through / (1.0f - b.reduceVisitsThreshold);
        const real red = prop * prop;
        const int v = (int)std::round((real)b.maxVisits + red * ((real)b.reducedVisitsMin - (real)b.maxVisits));
        gm.moveWeight = 1.0f + red * (b.reducedVisitsWeight - 1.0f);
        gm.visitLimit = std::max(v, b.reducedVisitsMin);
      }
    }
    return clear;
  }

  void startGame() {
    gm.rng.seed = mix64(s.cfg.seed ^ mix64(((uint64_t)(s.cfg.slotBase + gm.slot) << 32) | gm.gameNum));
    gm.rng.ctr = 0;
    boardInit(g, gm.root);
    clearTree();
    gm.turns.clear();
    gm.gameMode = 0;
    gm.side.clear();
    gm.sideNext = 0;
    gm.sideMode = 0;
    gm.gameHash0 = gm.rng.next();
    gm.gameHash1 = gm.rng.next();
    // initializeGameUsingPolicy (playutils.cpp:147-176): floor(Exp(1) * area * prop)
    // opening moves (nextExponential rand.h:299-305)
    gm.startTurn = 0;
    gm.initLeft = 0;
    const SearchParams& b = s.cfg.sp;
    if(b.initGamesWithPolicy && b.policyInitAreaProp > 0.0f) {
      real u = gm.rng.uni();
      while(u <= 0.0f)
        u = gm.rng.uni();
      gm.initLeft = (int)std::floor(-kLogf(u) * ((real)g.A * b.policyInitAreaProp));
    }
    if(gm.initLeft > 0) {
      gm.phase = PH_INIT;
    } else {
      setMoveLimits();
      gm.phase = PH_ROOTEVAL;
    }
    gm.rootK = 0;
  }

  // getGameInitializationMove (playutils.cpp:97-145) + the move of
  // initializeGameUsingPolicy (:163-175): a move sampled from the root's
  // post-processed policy raised to 1/temperature (2e-4 of the time uniformly among
  // the candidates), played without search, recorded as a turn without rows.
  // Returns true when the move ended the game.
  bool initMove(const float* out) {
    const SearchParams& b = s.cfg.sp;
    float pol[MAX_P], w, l;
    postprocess(gm.root, gm.leafSym, out, pol, w, l);
    int cpos[MAX_P];
    real cval[MAX_P];
    int n = 0;
    const real invT = 1.0f / b.policyInitAreaTemperature;
    for(int p = 0; p < g.P; p++)
      if(pol[p] > 0.0f) {
        cpos[n] = p;
        cval[n] = b.policyInitAreaTemperature == 1.0f ? pol[p] : kPowf((real)pol[p], (real)invT);
        n++;
      }
    int idx;
    if(gm.rng.uni() < 0.0002f) {
      idx = (int)gm.rng.below((uint32_t)n);
    } else {
      real sum = 0.0f;
      for(int i = 0; i < n; i++)
        sum = sum + cval[i];
      const real dd = gm.rng.uni() * sum;
      idx = n - 1;
      real acc = 0.0f;
      for(int i = 0; i < n; i++) {
        acc = acc + cval[i];
        if(acc > dd) {
          idx = i;
          break;
        }
      }
    }
    const int chosen = cpos[idx];
    TurnRec tr{};
    tr.cell = (int8_t)(chosen % g.A);
    tr.dir = (int8_t)(chosen / g.A);
    tr.policyTarget.assign(g.P, 0);
    gm.turns.push_back(tr);
    gm.startTurn++;
    gm.initLeft--;
    playMove(g, gm.root, chosen % g.A, chosen / g.A);
    if(gm.root.finished)
      return true;
    if(gm.initLeft == 0) {
      setMoveLimits();
      gm.phase = PH_ROOTEVAL;
      gm.rootK = 0;
    }
    return false;
  }

  // The slot's next game starts from the fork position b: the finished game's first
  // `prefix` moves plus `move` stay as unsearched turns, no policy init, mode FORK.
  void startForkGame(const Board& b, int prefix, int move) {
    gm.rng.seed = mix64(s.cfg.seed ^ mix64(((uint64_t)(s.cfg.slotBase + gm.slot) << 32) | gm.gameNum));
    gm.rng.ctr = 0;
    gm.root = b;
    clearTree();
    std::vector<TurnRec> keep;
    for(int t = 0; t <= prefix; t++) {
      TurnRec tr{};
      tr.cell = t < prefix ? gm.turns[t].cell : (int8_t)(move % g.A);
      tr.dir = t < prefix ? gm.turns[t].dir : (int8_t)(move / g.A);
      tr.policyTarget.assign(g.P, 0);
      keep.push_back(tr);
    }
    gm.turns.swap(keep);
    gm.startTurn = prefix + 1;
    gm.initLeft = 0;
    gm.gameMode = 2;
    gm.side.clear();
    gm.sideNext = 0;
    gm.sideMode = 0;
    gm.gameHash0 = gm.rng.next();
    gm.gameHash1 = gm.rng.next();
    setMoveLimits();
    gm.phase = PH_ROOTEVAL;
    gm.rootK = 0;
  }

  // Play::maybeForkGame (play.cpp:1741-1840) on the finished game's stream; candidates
  // are uniform draws with replacement from the legal moves in cell-major order
  // (chooseRandomLegalMoves playutils.cpp:33-60).  No draws when forks are off.
  bool maybeFork() {
    const SearchParams& b = s.cfg.sp;
    if(b.earlyForkGameProb <= 0.0f && b.forkGameProb <= 0.0f)
      return false;
    const bool early = gm.rng.uni() < b.earlyForkGameProb;
    const bool late = !early && b.forkGameProb > 0.0f && gm.rng.uni() < b.forkGameProb;
    if(!early && !late)
      return false;
    const int n = (int)gm.turns.size();
    int moveIdx;
    if(early) {
      real u = gm.rng.uni();
      while(u <= 0.0f)
        u = gm.rng.uni();
      moveIdx = (int)std::floor(-kLogf(u) * (b.earlyForkGameExpectedMoveProp * (real)g.A));
    } else {
      moveIdx = n <= 0 ? 0 : (int)gm.rng.below((uint32_t)n);
    }
    moveIdx = std::min(moveIdx, std::max(n - 1, 0));
    Board bd;
    boardInit(g, bd);
    for(int t = 0; t < moveIdx; t++) {
      playMove(g, bd, gm.turns[t].cell, gm.turns[t].dir);
      if(bd.finished)
        return false;
    }
    const int maxC = early ? b.earlyForkGameMaxChoices : b.forkGameMaxChoices;
    const int numChoices = b.forkGameMinChoices + (int)gm.rng.below((uint32_t)(maxC - b.forkGameMinChoices + 1));
    std::vector<int> legal;
    for(int cell = 0; cell < g.A; cell++)
      for(int dir = 0; dir < 4; dir++)
        if(isLegal(g, bd, cell, dir))
          legal.push_back(dir * g.A + cell);
    if(legal.empty())
      return false;
    gm.forkMoves.clear();
    for(int i = 0; i < numChoices; i++)
      gm.forkMoves.push_back(legal[gm.rng.below((uint32_t)legal.size())]);
    gm.forkBoard = bd;
    gm.forkNext = 0;
    gm.forkBest = -1;
    gm.forkBestWinrate = 0.0f;
    gm.forkPrefix = moveIdx;
    gm.phase = PH_FORK;
    return true;
  }

  // The value of the position after candidate forkNext (first best for the player at
  // the fork); after the last candidate the next game starts from the fork.
  void forkEval(const float* out) {
    float pol[MAX_P], w, l;
    postprocess(gm.leafBoard, gm.leafSym, out, pol, w, l);
    const real wr = 0.5f * (w - l + 1.0f);
    const int pla = gm.forkBoard.pla;
    if(gm.forkBest < 0 || (pla == 2 && wr > gm.forkBestWinrate) || (pla == 1 && wr < gm.forkBestWinrate)) {
      gm.forkBest = gm.forkNext;
      gm.forkBestWinrate = wr;
    }
    gm.forkNext++;
    if(gm.forkNext < (int)gm.forkMoves.size())
      return;
    const int move = gm.forkMoves[gm.forkBest];
    Board bd = gm.forkBoard;
    playMove(g, bd, move % g.A, move / g.A);
    if(bd.finished)
      startGame();
    else
      startForkGame(bd, gm.forkPrefix, move);
  }

  // chooseRandomForkingMove (play.cpp:615-633) over the post-processed policy `pol`
  // (chooseRandomPolicyMove playutils.cpp:62-95, chooseRandomLegalMove :10-31).
  // Returns the policy position, or -1.
  int forkingMove(const float* pol, const Board& b, int ban) {
    const real r = gm.rng.uni();
    if(r < 0.95f) {
      const real temp = r < 0.70f ? 1.0f : 2.0f;
      int cpos[MAX_P];
      real cval[MAX_P];
      int n = 0;
      for(int p = 0; p < g.P; p++)
        if(pol[p] > 0.0f && p != ban) {
          cpos[n] = p;
          cval[n] = pol[p];
          n++;
        }
      if(n <= 0)
        return -1;
      return cpos[chooseIndex(cval, n, temp)];
    }
    std::vector<int> legal;
    for(int cell = 0; cell < g.A; cell++)
      for(int dir = 0; dir < 4; dir++) {
        const int p = dir * g.A + cell;
        if(p != ban && isLegal(g, b, cell, dir))
          legal.push_back(p);
      }
    if(legal.empty())
      return -1;
    return legal[gm.rng.below((uint32_t)legal.size())];
  }

  void pushSide(const Board& b) {
    if(b.finished || (int)gm.side.size() >= MAX_SIDE)
      return;
    gm.side.push_back(b);
  }

  // The next side position: a full search from a cleared tree with the bot's own
  // parameters (play.cpp:1586-1590).
  void startSideSearch() {
    gm.root = gm.side[gm.sideNext];
    clearTree();
    gm.visitLimit = s.cfg.sp.maxVisits;
    gm.noNoise = 0;
    gm.moveWeight = 1.0f;
    gm.sideMode = 1;
    gm.phase = PH_ROOTEVAL;
    gm.rootK = 0;
  }

  // After a game's rows: its side positions, then the fork decision and the next game.
  void afterGame() {
    if(gm.sideNext < (int)gm.side.size()) {
      startSideSearch();
      return;
    }
    gm.sideMode = 0;
    if(!maybeFork())
      startGame();
  }

  // writeGame's side rows (trainingwrite.cpp:894-937, addRow with isSidePosition):
  // a searched side position (board = its root, after the game: gameNumMeta = the
  // finished game's number) or a tree position (board = the node's position).
  void emitSideRow(const TurnRec& tr) { emitSideRow(tr, gm.root, (int32_t)gm.gameNum - 1); }
  void emitSideRow(const TurnRec& tr, const Board& b, int32_t gameNumMeta) {
    const int A = g.A, P = g.P, pb = (A + 7) / 8;
    real hmv[5];
    bool h = true;
    for(int i = 0; i < 5; i++) {
      h = h && gm.rng.uni() < 0.98f;
      hmv[i] = h ? 1.0f : 0.0f;
    }
    Rows& R = s.rows;
    const int pla = b.pla;
    float bin[NUM_SPATIAL * MAX_AREA], glob[1];
    encodeV1(g, b, 0, bin, glob);
    const size_t r = (size_t)R.n;
    R.n++;
    R.bin.resize((size_t)R.n * NUM_SPATIAL * pb);
    R.globIn.resize((size_t)R.n);
    R.policy.resize((size_t)R.n * 2 * P);
    R.globT.resize((size_t)R.n * 64);
    R.value.resize((size_t)R.n * 5 * A);
    R.meta.resize((size_t)R.n * 4);
    R.meta[r * 4 + 0] = s.cfg.slotBase + gm.slot;
    R.meta[r * 4 + 1] = gameNumMeta;
    R.meta[r * 4 + 2] = b.turn;
    R.meta[r * 4 + 3] = (int32_t)gm.turns.size();
    for(int ch = 0; ch < NUM_SPATIAL; ch++)
      packBitsBE(bin + ch * A, A, &R.bin[(r * NUM_SPATIAL + ch) * pb]);
    R.globIn[r] = glob[0];
    for(int p = 0; p < P; p++) {
      R.policy[r * 2 * P + p] = tr.policyTarget[p];
      R.policy[r * 2 * P + P + p] = 1;
    }
    float* gt = &R.globT[r * 64];
    for(int i = 0; i < 64; i++)
      gt[i] = 0.0f;
    for(int f = 0; f < 5; f++) {
      gt[2 * f] = pla == 2 ? tr.whiteWin : tr.whiteLoss;
      gt[2 * f + 1] = pla == 2 ? tr.whiteLoss : tr.whiteWin;
    }
    gt[25] = 1.0f;
    gt[26] = 1.0f;
    gt[30] = tr.policySurprise;
    gt[31] = tr.policyEntropy;
    gt[32] = tr.searchEntropy;
    for(int i = 0; i < 5; i++)
      gt[36 + i] = hmv[i];
    gt[41] = (real)(gm.gameHash0 & 0x3FFFFF);
    gt[42] = (real)((gm.gameHash0 >> 22) & 0x3FFFFF);
    gt[43] = (real)((gm.gameHash0 >> 44) & 0xFFFFF);
    gt[44] = (real)(gm.gameHash1 & 0x3FFFFF);
    gt[45] = (real)((gm.gameHash1 >> 22) & 0x3FFFFF);
    gt[46] = (real)((gm.gameHash1 >> 44) & 0xFFFFF);
    gt[51] = (real)b.turn;
    gt[53] = (real)gm.startTurn;
    gt[55] = (real)gm.gameMode;
    gt[57] = pla == 2 ? tr.rawWhiteWL : -tr.rawWhiteWL;
    gt[59] = tr.rawPolicyEntropy;
    gt[60] = (real)tr.visits;
    gt[63] = 1.0f;
    for(int i = 0; i < 5 * A; i++)
      R.value[r * 5 * A + i] = 0;
  }

  // A search's targets at node ni with policy pol: extractPolicyTarget (play.cpp:635-672,
  // scaleMaxToAtLeast 10, no direct policy moves) and getPolicySurpriseAndEntropy
  // (searchresults.cpp:486-550, scaleMaxToAtLeast 1).
  void searchTargets(int ni, const float* pol, bool isRoot, TurnRec& tr) {
    int posv[MAX_P];
    real vals[MAX_P];
    tr.policyTarget.assign(g.P, 0);
    {
      int m = playSelectionValuesAt(ni, pol, isRoot, 10.0f, false, posv, vals, sp.useLcbForSelection);
      real mx = 0.0f;
      for(int i = 0; i < m; i++)
        if(vals[i] > mx)
          mx = vals[i];
      real factor = mx > 30000.0f ? 30000.0f / mx : 1.0f;
      for(int i = 0; i < m; i++)
        tr.policyTarget[posv[i]] = (int16_t)std::round(vals[i] * factor);
    }
    int m = playSelectionValuesAt(ni, pol, isRoot, 1.0f, true, posv, vals, sp.useLcbForSelection);
    real sumV = 0.0f;
    for(int i = 0; i < m; i++)
      sumV = sumV + vals[i];
    real surprise = 0.0f, searchEnt = 0.0f, polEnt = 0.0f;
    for(int i = 0; i < m; i++) {
      real p = rmax(pol[posv[i]], 1e-30f);
      real t = vals[i] / sumV;
      if(t > 1e-30f) {
        real lt = kLogf(t), lp = kLogf(p);
        surprise = surprise + t * (lt - lp);
        searchEnt = searchEnt + (-t * lt);
      }
    }
    for(int p = 0; p < g.P; p++)
      if(pol[p] > 1e-30f)
        polEnt = polEnt + (-pol[p] * kLogf(pol[p]));
    tr.policySurprise = rmax(0.0f, surprise);
    tr.searchEntropy = rmax(0.0f, searchEnt);
    tr.policyEntropy = rmax(0.0f, polEnt);
  }

  // extractValueTargets (play.cpp:674-682) via ReportedSearchValues (reportedsearchvalues.cpp:10-50).
  void valueTargets(int ni, TurnRec& tr) {
    real wl = rmax(-1.0f, rmin(1.0f, N(ni).winLossAvg));
    tr.whiteWin = rmax(0.0f, rmin(1.0f, 0.5f * (wl + 1.0f)));
    tr.whiteLoss = rmax(0.0f, rmin(1.0f, 0.5f * (-wl + 1.0f)));
    tr.rootWL = wl;
  }

  // computeNNRawStats (play.cpp:684-704) from a stored evaluation.
  void rawStats(real win, real loss, const float* pol, TurnRec& tr) {
    tr.rawWhiteWL = win - loss;
    real ent = 0.0f;
    for(int p = 0; p < g.P; p++) {
      real q = pol[p];
      if(q >= 1e-30f)
        ent = ent + (-q * kLogf(q));
    }
    tr.rawPolicyEntropy = ent;
  }

  // recordTreePositionsRec (play.cpp:710-814, maxDepth 5 from :832): a pre-order walk of
  // the finished search's tree that writes a side row at every non-root node reached
  // only through best moves of the player to move there; excl0/excl1 (the played move
  // and the side position's forking move) are skipped at the root.  SPEC: the raw
  // network stats are the node's stored evaluation (the reference re-evaluates the
  // position, :748); the weight resolves when the position is recorded
  // (resolveWeight :1683-1696: floor + a draw on the excess) and the rows are written
  // then (the tree is gone by the game's end), with the network-change fields of a
  // searched side row.
  void recordTreeRec(const Board& b, int ni, int depth, bool plaBest, bool oppBest, int excl0, int excl1,
                     uint32_t rootVisits, int32_t gameNumMeta) {
    const int k = N(ni).numChildren;
    if(k <= 0)
      return;
    if(plaBest && ni != gm.rootIdx) {
      TurnRec tr;
      searchTargets(ni, POL(ni), false, tr);
      valueTargets(ni, tr);
      rawStats(N(ni).nnWin, N(ni).nnLoss, POL(ni), tr);
      tr.visits = rootVisits;
      const real w = sp.recordTreeTargetWeight;
      const real fl = std::floor(w);
      const int copies = (int)fl + (gm.rng.uni() < w - fl ? 1 : 0);
      for(int c = 0; c < copies; c++)
        emitSideRow(tr, b, gameNumMeta);
    }
    if(depth >= 5)
      return;
    // the child with the most visits, children[0]'s count not consulted (:757-769)
    int best = 0;
    uint32_t bestVisits = 0;
    for(int i = 1; i < k; i++) {
      const uint32_t cv = N((int)EC(ni, i)).visits;
      if(cv > bestVisits) {
        bestVisits = cv;
        best = i;
      }
    }
    for(int i = 0; i < k; i++) {
      const bool newPla = oppBest, newOpp = plaBest && i == best;
      if(!newPla && !newOpp)
        continue;
      const int mv = EM(ni, i);
      if(mv == excl0 || mv == excl1)
        continue;
      const int ci = (int)EC(ni, i);
      if((int64_t)N(ci).visits < (int64_t)sp.recordTreeThreshold)
        continue;
      Board b2 = b;
      playMove(g, b2, mv % g.A, mv / g.A);
      recordTreeRec(b2, ci, depth + 1, newPla, newOpp, -1, -1, rootVisits, gameNumMeta);
    }
  }

  // The network's policy at a side position's continuation picks a forking move.
  void sideEval(const float* out) {
    float pol[MAX_P], w, l;
    postprocess(gm.leafBoard, gm.leafSym, out, pol, w, l);
    const int fm = forkingMove(pol, gm.leafBoard, -1);
    if(fm >= 0) {
      Board b3 = gm.leafBoard;
      playMove(g, b3, fm % g.A, fm / g.A);
      pushSide(b3);
    }
    gm.sideNext++;
    afterGame();
  }

  void finishGame();
  void commitMove();
  void commitPending();
};

// A game in PH_COMMIT at a commit round (device kCommit search.hip:3358-3507): a
// policy-initialisation move that ended the game finishes it (nothing searched, no rows,
// play.cpp:1262-1264); otherwise the search's move is committed.
void Ctx::commitPending() {
  if(gm.root.finished) {
    finishGame();
    gm.gamesFinished++;
    gm.gameNum++;
    gm.sideNext = 0;
    afterGame();
    return;
  }
  commitMove();
}

void Ctx::commitMove() {
  int posv[MAX_P];
  real vals[MAX_P];
  TurnRec tr;
  // a side position's search (play.cpp:1576-1662) ends like a move search, but writes
  // one row and plays nothing
  const bool side = gm.sideMode != 0;
  // getChosenMoveLoc (searchresults.cpp:435-453); runBotWithLimits disables LCB for the
  // game's moves in self-play (play.cpp:1040-1046), a side position's response keeps it
  int n = playSelectionValues(0.0f, true, posv, vals, side ? sp.useLcbForSelection != 0 : false);
  if(n <= 0) {
    fprintf(stderr, "oracle: no move selectable\n");
    abort();
  }
  real temp = interpolateEarly(sp.chosenMoveTemperatureHalflife, sp.chosenMoveTemperatureEarly, sp.chosenMoveTemperature);
  int chosen = posv[chooseIndex(vals, n, temp)];
  const Node& r = N(gm.rootIdx);
  valueTargets(gm.rootIdx, tr);
  tr.visits = r.visits;
  tr.rootNNWin = r.nnWin;
  tr.rootNNLoss = r.nnLoss;
  tr.targetWeight = gm.moveWeight;
  // the targets below run after runBotWithLimits restored the base parameters
  // (play.cpp:1066, :1307-1320)
  Ctx base(s, gm, s.cfg.sp);
  base.searchTargets(gm.rootIdx, gm.rootNoised.data(), true, tr);
  // computeNNRawStats play.cpp:684-704 (first root-symmetry eval)
  rawStats(gm.rawWin, gm.rawLoss, gm.rawPolicy.data(), tr);
  const bool recordTree = s.cfg.sp.recordTreePositions != 0 && s.cfg.sp.recordTreeTargetWeight > 0.0f;
  if(side) {
    emitSideRow(tr);
    // its subtree positions (play.cpp:1612-1628)
    if(recordTree)
      base.recordTreeRec(gm.root, gm.rootIdx, 0, true, true, -1, -1, r.visits, (int32_t)gm.gameNum - 1);
    // occasionally continue: the response, then a forking move (play.cpp:1632-1656)
    if(gm.rng.uni() < 0.25f) {
      Board b2 = gm.root;
      playMove(g, b2, chosen % g.A, chosen / g.A);
      if(!b2.finished) {
        gm.leafBoard = b2;
        gm.phase = PH_SIDEEVAL;
        return;
      }
    }
    gm.sideNext++;
    afterGame();
    return;
  }
  // a side position: the root policy's alternative to the move (play.cpp:1328-1345)
  int forkMove = -1;
  if(s.cfg.sp.sidePositionProb > 0.0f && gm.rng.uni() < s.cfg.sp.sidePositionProb) {
    const int fm = forkingMove(POL(gm.rootIdx), gm.root, chosen);
    forkMove = fm;
    if(fm >= 0) {
      Board b2 = gm.root;
      playMove(g, b2, fm % g.A, fm / g.A);
      pushSide(b2);
    }
  }
  // subtree positions of this search, except the played and the forked branches
  // (play.cpp:1347-1361)
  if(recordTree)
    base.recordTreeRec(gm.root, gm.rootIdx, 0, true, true, chosen, forkMove, r.visits, (int32_t)gm.gameNum);
  tr.cell = (int8_t)(chosen % g.A);
  tr.dir = (int8_t)(chosen / g.A);
  gm.turns.push_back(tr);
  playMove(g, gm.root, chosen % g.A, chosen / g.A);
  gm.movesMade++;
  if(gm.root.finished) {
    finishGame();
    gm.gamesFinished++;
    gm.gameNum++;
    gm.sideNext = 0;
    afterGame();
    return;
  }
  if(setMoveLimits())
    clearTree();
  else
    reuseTree(chosen);
  // SPEC B26: Search::recursivelyRecomputeStats (search.cpp:671, :834-910) is not
  // run after tree reuse; the kept subtree keeps its statistics.
  gm.phase = PH_ROOTEVAL;
  gm.rootK = 0;
}

static void packBitsBE(const float* v, int len, uint8_t* out) {
  // packBits trainingwrite.cpp:218-232 (big-endian within each byte)
  for(int i = 0; i < (len + 7) / 8; i++)
    out[i] = 0;
  for(int i = 0; i < len; i++)
    if(v[i] != 0.0f)
      out[i >> 3] |= (uint8_t)(1u << (7 - (i & 7)));
}

// Play::runGame row weights: value surprise (play.cpp:1470-1497), surprise-weighted
// target weights (:1498-1574) and their probabilistic resolution (:1683-1697), in f32
// with the loops' own order.  Fills turns[].rows.
static void resolveTurnWeights(const SearchParams& b, int A, std::vector<TurnRec>& turns, int t0, const real* tWin,
                               const real* tLoss, Rng& rng) {
  const int n = (int)turns.size();  // searched turns [t0, n)
  if(b.policySurpriseDataWeight > 0.0f || b.valueSurpriseDataWeight > 0.0f) {
    std::vector<real> vs(n);
    const real nowFactor = 1.0f / (1.0f + (real)A * 0.016f);
    real winV = tWin[n], lossV = tLoss[n];
    for(int i = n - 1; i >= t0; i--) {
      winV = winV + nowFactor * (tWin[i] - winV);
      lossV = lossV + nowFactor * (tLoss[i] - lossV);
      real v = 0.0f;
      if(winV > 1e-30f)
        v = v + winV * (kLogf(winV) - kLogf(rmax(turns[i].rootNNWin, 1e-30f)));
      if(lossV > 1e-30f)
        v = v + lossV * (kLogf(lossV) - kLogf(rmax(turns[i].rootNNLoss, 1e-30f)));
      if(v < 0.0f)
        v = 0.0f;
      vs[i] = rmin(v, 1.0f);
    }
    real sumW = 0.0f, sumPS = 0.0f, sumVS = 0.0f;
    for(int i = t0; i < n; i++) {
      const real tw = turns[i].targetWeight;
      sumW = sumW + tw;
      sumPS = sumPS + turns[i].policySurprise * tw;
      sumVS = sumVS + vs[i] * tw;
    }
    if(sumW >= 1.0f) {
      const real avgPS = sumPS / sumW, avgVS = sumVS / sumW;
      real vsdw = b.valueSurpriseDataWeight;
      if(avgVS < 0.010f)
        vsdw = vsdw * (avgVS / 0.010f);
      const real thr = avgPS * 1.5f;
      real sumPPV = 0.0f, sumVPV = 0.0f;
      for(int i = t0; i < n; i++) {
        const real tw = turns[i].targetWeight, ps = turns[i].policySurprise;
        sumPPV = sumPPV + (tw * ps + (1.0f - tw) * rmax(0.0f, ps - thr));
        sumVPV = sumVPV + tw * vs[i];
      }
      sumPPV = rmax(sumPPV, 1e-10f);
      sumVPV = rmax(sumVPV, 1e-10f);
      for(int i = t0; i < n; i++) {
        const real tw = turns[i].targetWeight, ps = turns[i].policySurprise;
        const real ppv = tw * ps + (1.0f - tw) * rmax(0.0f, ps - thr);
        const real vpv = tw * vs[i];
        turns[i].targetWeight = (1.0f - b.policySurpriseDataWeight - vsdw) * tw +
                                b.policySurpriseDataWeight * ppv * sumW / sumPPV + vsdw * vpv * sumW / sumVPV;
      }
    }
  }
  for(int i = t0; i < n; i++) {
    real w = turns[i].targetWeight;
    if(w <= 0.0f)
      w = 0.0f;
    const real fl = std::floor(w), excess = w - fl;
    turns[i].rows = (int)(rng.uni() < excess ? fl + 1.0f : fl);
  }
}

// Play::runGame finalisation play.cpp:1431-1460 + TrainingDataWriter::writeGame
// trainingwrite.cpp:774-890 + addRow :316-565: turn t is written turns[t].rows times.
void Ctx::finishGame() {
  const int numMoves = (int)gm.turns.size();
  const int A = g.A, P = g.P, pb = (A + 7) / 8;
  real finalWin = gm.root.winner == 2 ? 1.0f : (gm.root.winner == 1 ? 0.0f : 0.5f);
  std::vector<real> tWin(numMoves + 1), tLoss(numMoves + 1);
  for(int t = 0; t < numMoves; t++) {
    tWin[t] = gm.turns[t].whiteWin;
    tLoss[t] = gm.turns[t].whiteLoss;
  }
  tWin[numMoves] = finalWin;
  tLoss[numMoves] = 1.0f - finalWin;
  std::vector<Board> boards(numMoves + 1);
  boardInit(g, boards[0]);
  for(int t = 0; t < numMoves; t++) {
    boards[t + 1] = boards[t];
    playMove(g, boards[t + 1], gm.turns[t].cell, gm.turns[t].dir);
  }
  const Board& fin = boards[numMoves];
  // finalMaxLength (SPEC: per-cell longest same-colour run through the cell, 0 if empty)
  int8_t finalMaxLen[MAX_AREA];
  for(int c = 0; c < A; c++)
    finalMaxLen[c] = fin.c[c] == 0 ? 0 : (int8_t)maxRun(g, fin, c);
  resolveTurnWeights(s.cfg.sp, A, gm.turns, gm.startTurn, tWin.data(), tLoss.data(), gm.rng);
  // history-mask draws come from a copy of the game stream (the rows are written by a
  // separate device kernel from a snapshot), so the stream a fork continues from is
  // the one after the weight resolution
  Rng hmRng = gm.rng;
  std::vector<int> rowTurn;  // turn of each row, in row order
  for(int t = 0; t < numMoves; t++)
    for(int c = 0; c < gm.turns[t].rows; c++)
      rowTurn.push_back(t);
  Rows& R = s.rows;
  for(const int t : rowTurn) {
    const Board& b = boards[t];
    int pla = b.pla, opp = 3 - pla;
    float bin[NUM_SPATIAL * MAX_AREA], glob[1];
    encodeV1(g, b, 0, bin, glob);
    size_t r = (size_t)R.n;
    R.n++;
    R.bin.resize((size_t)R.n * NUM_SPATIAL * pb);
    R.globIn.resize((size_t)R.n);
    R.policy.resize((size_t)R.n * 2 * P);
    R.globT.resize((size_t)R.n * 64);
    R.value.resize((size_t)R.n * 5 * A);
    R.meta.resize((size_t)R.n * 4);
    R.meta[r * 4 + 0] = s.cfg.slotBase + gm.slot;
    R.meta[r * 4 + 1] = (int32_t)gm.gameNum;
    R.meta[r * 4 + 2] = t;
    R.meta[r * 4 + 3] = numMoves;
    for(int ch = 0; ch < NUM_SPATIAL; ch++)
      packBitsBE(bin + ch * A, A, &R.bin[(r * NUM_SPATIAL + ch) * pb]);
    R.globIn[r] = glob[0];
    int16_t* pol = &R.policy[r * 2 * P];
    for(int p = 0; p < P; p++) {
      pol[p] = gm.turns[t].policyTarget[p];
      pol[P + p] = t + 1 < numMoves ? gm.turns[t + 1].policyTarget[p] : (int16_t)1;
    }
    float* gt = &R.globT[r * 64];
    for(int i = 0; i < 64; i++)
      gt[i] = 0.0f;
    // fillValueTDTargets trainingwrite.cpp:286-314
    const real nowFactors[5] = {0.0f, 1.0f / (1.0f + (real)A * 0.176f), 1.0f / (1.0f + (real)A * 0.056f),
                                 1.0f / (1.0f + (real)A * 0.016f), 1.0f};
    for(int f = 0; f < 5; f++) {
      real win = 0.0f, loss = 0.0f, left = 1.0f;
      for(int i = t; i <= numMoves; i++) {
        real now;
        if(i == numMoves) {
          now = left;
          left = 0.0f;
        } else {
          now = left * nowFactors[f];
          left = left * (1.0f - nowFactors[f]);
        }
        win = win + now * (pla == 2 ? tWin[i] : tLoss[i]);
        loss = loss + now * (pla == 2 ? tLoss[i] : tWin[i]);
      }
      gt[2 * f] = win;
      gt[2 * f + 1] = loss;
    }
    {
      real sum = 0.0f;
      for(int i = t + 1; i <= numMoves; i++) {
        real prevWL = tWin[i - 1] - tLoss[i - 1], nextWL = tWin[i] - tLoss[i];
        real var = (nextWL - prevWL) * (nextWL - prevWL);
        sum = sum + (real)(i - t) * var;
      }
      gt[22] = sum;
    }
    gt[25] = 1.0f;
    gt[26] = 1.0f;
    gt[27] = 1.0f;
    gt[28] = t + 1 < numMoves ? 1.0f : 0.0f;
    gt[30] = gm.turns[t].policySurprise;
    gt[31] = gm.turns[t].policyEntropy;
    gt[32] = gm.turns[t].searchEntropy;
    gt[33] = 1.0f;
    bool h = true;
    for(int i = 0; i < 5; i++) {
      h = h && hmRng.uni() < 0.98f;
      gt[36 + i] = h ? 1.0f : 0.0f;
    }
    gt[41] = (real)(gm.gameHash0 & 0x3FFFFF);
    gt[42] = (real)((gm.gameHash0 >> 22) & 0x3FFFFF);
    gt[43] = (real)((gm.gameHash0 >> 44) & 0xFFFFF);
    gt[44] = (real)(gm.gameHash1 & 0x3FFFFF);
    gt[45] = (real)((gm.gameHash1 >> 22) & 0x3FFFFF);
    gt[46] = (real)((gm.gameHash1 >> 44) & 0xFFFFF);
    gt[51] = (real)t;
    gt[53] = (real)gm.startTurn;
    gt[55] = (real)gm.gameMode;
    gt[57] = pla == 2 ? gm.turns[t].rawWhiteWL : -gm.turns[t].rawWhiteWL;
    gt[59] = gm.turns[t].rawPolicyEntropy;
    gt[60] = (real)gm.turns[t].visits;
    gt[63] = 1.0f;
    int8_t* vt = &R.value[r * 5 * A];
    const Board& b2 = boards[std::min(t + 2, numMoves)];
    const Board& b3 = boards[std::min(t + 6, numMoves)];
    for(int c = 0; c < A; c++) {
      vt[c] = fin.c[c] == pla ? 1 : (fin.c[c] == opp ? -1 : 0);
      vt[A + c] = 0;
      vt[2 * A + c] = b2.c[c] == pla ? 1 : (b2.c[c] == opp ? -1 : 0);
      vt[3 * A + c] = b3.c[c] == pla ? 1 : (b3.c[c] == opp ? -1 : 0);
      vt[4 * A + c] = finalMaxLen[c];
    }
  }
}

}  // namespace

// Cache slot of a state key (SPEC a7): fold of the two key words, low bits.
static uint32_t cacheSlotOf(uint64_t k0, uint64_t k1, uint32_t mask) {
  const uint64_t h = k0 ^ ((k1 << 29) | (k1 >> 35));
  return (uint32_t)(h ^ (h >> 32)) & mask;
}

void selfplayInit(Selfplay& s, const SelfplayCfg& cfg, int numGames) {
  s.cfg = cfg;
  s.spCheap = cheapSearchParams(cfg.sp);
  const Geom& g = s.cfg.g;
  if(cfg.cacheLog2 > 0) {
    const size_t entries = (size_t)1 << cfg.cacheLog2;
    s.cacheKey.assign(2 * entries, 0);  // zero key: never a state
    s.cachePol.assign(entries * g.P, 0.0f);
    s.cacheVal.assign(2 * entries, 0.0f);
  }
  Rng zr;
  zr.seed = SVB_SEED;
  s.svbZ.resize(2 * (MAX_P + 1) + 3 + 4 * 25);
  for(auto& z : s.svbZ)
    z = zr.next();
  s.games.resize(numGames);
  for(int i = 0; i < numGames; i++) {
    Game& gm = s.games[i];
    gm.slot = i;
    gm.gameNum = 0;
    gm.nodes.resize(cfg.nodeCap);
    gm.edgeChild.assign((size_t)cfg.nodeCap * g.P, 0);
    gm.edgeVisits.assign((size_t)cfg.nodeCap * g.P, 0);
    gm.edgeMove.assign((size_t)cfg.nodeCap * g.P, 0);
    gm.policy.assign((size_t)cfg.nodeCap * g.P, 0.0f);
    gm.rootNoised.assign(g.P, 0.0f);
    gm.accPolicy.assign(g.P, 0.0f);
    gm.rawPolicy.assign(g.P, 0.0f);
    const int tcap = tableCapFor(cfg.nodeCap);
    gm.ttKey0.assign(tcap, 0);
    gm.ttKey1.assign(tcap, 0);
    gm.ttNode.assign(tcap, -1);
    gm.svbKey.assign(tcap, 0);
    gm.svbDelta.assign(tcap, 0);
    gm.svbWeight.assign(tcap, 0);
    gm.svbUsed.assign(tcap, 0);
    Ctx(s, gm).startGame();
  }
}

void selfplayRound(Selfplay& s, bool commitNow) {
  const Geom& g = s.cfg.g;
  const int G = (int)s.games.size();
  const int A = g.A;
  // encoded leaves, per game (a deferred leaf keeps its row across rounds)
  std::vector<float>& bin = s.nnBin;
  std::vector<float>& glob = s.nnGlob;
  bin.resize((size_t)G * NUM_SPATIAL * A);
  glob.resize((size_t)G);
  std::vector<int> need(G, 0);
  const bool cacheOn = s.cfg.cacheLog2 > 0;
  const uint32_t cacheMask = cacheOn ? (uint32_t)((1u << s.cfg.cacheLog2) - 1) : 0u;
  // ---- select (games are independent: threads over games for the CPU baseline,
  // cfg.parallelGames; the tests run it serially) ----
  const int par = s.cfg.parallelGames;
#pragma omp parallel for schedule(dynamic, 4) num_threads(par > 1 ? par : 1) if(par > 1)
  for(int i = 0; i < G; i++) {
    Game& gm = s.games[i];
    Ctx cx(s, gm);
    if(gm.nnDeferred) {  // the leaf (already encoded) waits for the network
      need[i] = 1;
      continue;
    }
    if(gm.phase == PH_COMMIT || gm.startDelay > 0) {
      // waits for the commit round, or for its staggered start (device kSelect)
      if(gm.startDelay > 0)
        gm.startDelay--;
      gm.leafKind = LEAF_NONE;
      continue;
    }
    if(gm.phase == PH_INIT) {
      gm.leafKind = LEAF_INIT;
      gm.leafSym = (int)gm.rng.below(8);
      gm.leafBoard = gm.root;
    } else if(gm.phase == PH_SIDEEVAL) {
      gm.leafKind = LEAF_SIDE;  // leafBoard: the continuation position set by commitMove
      gm.leafSym = (int)gm.rng.below(8);
    } else if(gm.phase == PH_FORK) {
      const int mv = gm.forkMoves[gm.forkNext];
      gm.leafBoard = gm.forkBoard;
      playMove(g, gm.leafBoard, mv % g.A, mv / g.A);
      gm.leafKind = LEAF_FORK;
      gm.leafSym = (int)gm.rng.below(8);
    } else if(gm.phase == PH_ROOTEVAL) {
      if(gm.rootK == 0) {
        int idx[8] = {0, 1, 2, 3, 4, 5, 6, 7};
        for(int k = 0; k < 4; k++) {
          int j = k + (int)gm.rng.below((uint32_t)(8 - k));
          std::swap(idx[k], idx[j]);
          gm.syms[k] = idx[k];
        }
      }
      gm.leafKind = LEAF_ROOTEVAL;
      gm.leafSym = gm.syms[gm.rootK];
      gm.leafBoard = gm.root;
    } else {
      cx.descend();
      if(gm.leafKind == LEAF_NN && cacheOn) {
        // lookups see the cache as it stood at the end of the previous round
        const Node& ln = cx.N(gm.leafNode);
        const uint32_t slot = cacheSlotOf(ln.key0, ln.key1, cacheMask);
        if(s.cacheKey[2 * slot] == ln.key0 && s.cacheKey[2 * slot + 1] == ln.key1) {
          gm.leafKind = LEAF_CACHED;
          gm.cacheSlot = (int)slot;
        }
      }
      if(gm.leafKind == LEAF_NN)
        gm.leafSym = (int)gm.rng.below(8);
    }
    if(gm.leafKind == LEAF_NN || gm.leafKind == LEAF_ROOTEVAL || gm.leafKind == LEAF_INIT ||
       gm.leafKind == LEAF_FORK || gm.leafKind == LEAF_SIDE) {
      encodeV1(g, gm.leafBoard, gm.leafSym, &bin[(size_t)i * NUM_SPATIAL * A], &glob[i]);
      need[i] = 1;
      gm.nnEvals++;
    }
  }
  // ---- NN ----
  std::vector<float> out((size_t)G * (g.P + 4));
  // the batch: needing games in cyclic order from the round-robin pointer, at most
  // nnCap rows; the rest are deferred, and the pointer moves past the last game taken
  // when the cap bites (device kCompact)
  std::vector<int> idx;
  int total = 0, lastTaken = -1;
  for(int k = 0; k < G; k++) {
    const int i = (s.nnRR + k) % G;
    if(!need[i]) {
      s.games[i].nnDeferred = 0;
      continue;
    }
    total++;
    const bool in = (int)idx.size() < s.cfg.nnCap;
    s.games[i].nnDeferred = in ? 0 : 1;
    if(in) {
      idx.push_back(i);
      lastTaken = i;
    }
  }
  if(total > s.cfg.nnCap)
    s.nnRR = (lastTaken + 1) % G;
  if(s.cfg.nnMode == 0) {
    for(int i : idx)
      fakeNet(g, &bin[(size_t)i * NUM_SPATIAL * A], &out[(size_t)i * (g.P + 4)], &out[(size_t)i * (g.P + 4) + g.P],
              &out[(size_t)i * (g.P + 4) + g.P + 2]);
  } else if(s.cfg.nnMode == 3) {
    if(!idx.empty()) {
      const int n = (int)idx.size(), nw = (NUM_SPATIAL * A + 63) / 64;
      std::vector<uint64_t> words((size_t)n * nw);
      std::vector<float> res((size_t)n * (g.P + 4));
      for(int j = 0; j < n; j++)
        packPlanes(g, &bin[(size_t)idx[j] * NUM_SPATIAL * A], &words[(size_t)j * nw]);
      s.cfg.netFn(n, words.data(), res.data());
      for(int j = 0; j < n; j++)
        memcpy(&out[(size_t)idx[j] * (g.P + 4)], &res[(size_t)j * (g.P + 4)], sizeof(float) * (g.P + 4));
    }
  } else if(!idx.empty()) {
    int n = (int)idx.size();
    std::vector<float> cb((size_t)n * NUM_SPATIAL * A), cg(n), pol((size_t)n * 4 * A), val((size_t)n * 2), misc((size_t)n * 2);
    for(int j = 0; j < n; j++) {
      memcpy(&cb[(size_t)j * NUM_SPATIAL * A], &bin[(size_t)idx[j] * NUM_SPATIAL * A], sizeof(float) * NUM_SPATIAL * A);
      cg[j] = glob[idx[j]];
    }
    nnForward(*s.cfg.model, g.X, g.Y, n, cb.data(), cg.data(), pol.data(), val.data(), misc.data(),
              s.cfg.nnMode == 2 ? 1 : 0, s.cfg.nnThreads);
    for(int j = 0; j < n; j++) {
      float* o = &out[(size_t)idx[j] * (g.P + 4)];
      memcpy(o, &pol[(size_t)j * 4 * A], sizeof(float) * g.P);
      o[g.P] = val[2 * j];
      o[g.P + 1] = val[2 * j + 1];
      o[g.P + 2] = misc[2 * j];
      o[g.P + 3] = misc[2 * j + 1];
    }
  }
  // ---- backup ----
  struct CacheWrite {
    uint32_t slot;
    uint64_t k0, k1;
    std::vector<float> pol;
    float w, l;
  };
  std::vector<CacheWrite> cacheWrites(G);  // fresh evaluations, by game (written in game order)
  std::vector<char> cacheWritten(G, 0);
  // moves, game ends and side/fork steps append to the shared row buffer: serialised
  // (in parallel mode the row order is thread order; the counts are the same)
#pragma omp parallel for schedule(dynamic, 4) num_threads(par > 1 ? par : 1) if(par > 1)
  for(int i = 0; i < G; i++) {
    Game& gm = s.games[i];
    if(gm.nnDeferred)  // backed up in the round its row is evaluated
      continue;
    if(gm.leafKind == LEAF_NONE)  // idle this round (PH_COMMIT or a staggered start)
      continue;
    Ctx cx(s, gm);
    const float* o = &out[(size_t)i * (g.P + 4)];
    if(gm.leafKind == LEAF_INIT || gm.leafKind == LEAF_FORK || gm.leafKind == LEAF_SIDE) {
#pragma omp critical(ora_rows)
      {
        if(gm.leafKind == LEAF_INIT) {
          if(cx.initMove(o))  // the opening ended the game: finished at the commit round
            gm.phase = PH_COMMIT;
        } else if(gm.leafKind == LEAF_FORK) {
          cx.forkEval(o);
        } else {
          cx.sideEval(o);
        }
      }
      continue;
    }
    if(gm.leafKind == LEAF_ROOTEVAL) {
      float pol[MAX_P], w, l;
      cx.postprocess(gm.root, gm.leafSym, o, pol, w, l);
      if(gm.rootK == 0) {
        for(int p = 0; p < g.P; p++) {
          gm.rawPolicy[p] = pol[p];
          gm.accPolicy[p] = 0.0f + pol[p];
        }
        gm.rawWin = w;
        gm.rawLoss = l;
        gm.accWin = 0.0f + w;
        gm.accLoss = 0.0f + l;
      } else {
        for(int p = 0; p < g.P; p++)
          gm.accPolicy[p] = gm.accPolicy[p] + pol[p];
        gm.accWin = gm.accWin + w;
        gm.accLoss = gm.accLoss + l;
      }
      gm.rootK++;
      if(gm.rootK == cx.sp.rootNumSymmetriesToSample) {
        real fl = (real)cx.sp.rootNumSymmetriesToSample;
        bool fresh = gm.rootIdx < 0;
        if(fresh)
          gm.rootIdx = cx.allocNode(gm.root.pla, stateHash(g, gm.root), false);
        Node& r = cx.N(gm.rootIdx);
        float* rp = cx.POL(gm.rootIdx);
        for(int p = 0; p < g.P; p++)
          rp[p] = gm.accPolicy[p] / fl;
        r.nnWin = gm.accWin / fl;
        r.nnLoss = gm.accLoss / fl;
        r.flags |= 1;
        if(fresh)
          cx.addLeafValue(gm.rootIdx, r.nnWin - r.nnLoss, false, true);
        cx.noiseAndTemp(rp, gm.rootNoised.data());
        gm.phase = PH_SEARCH;
        if(cx.N(gm.rootIdx).visits >= (uint32_t)gm.visitLimit)
          gm.phase = PH_COMMIT;
      }
      continue;
    }
    // PH_SEARCH leaf
    if(gm.leafKind == LEAF_NN || gm.leafKind == LEAF_CACHED) {
      Node& n = cx.N(gm.leafNode);
      float w, l;
      float* pol = cx.POL(gm.leafNode);
      if(gm.leafKind == LEAF_CACHED) {
        memcpy(pol, &s.cachePol[(size_t)gm.cacheSlot * g.P], sizeof(float) * g.P);
        w = s.cacheVal[2 * gm.cacheSlot];
        l = s.cacheVal[2 * gm.cacheSlot + 1];
      } else {
        cx.postprocess(gm.leafBoard, gm.leafSym, o, pol, w, l);
        if(cacheOn) {  // staged now: commitMove below may compact the node pool
          const uint32_t slot = cacheSlotOf(n.key0, n.key1, cacheMask);
          cacheWrites[i] = {slot, n.key0, n.key1, std::vector<float>(pol, pol + g.P), w, l};
          cacheWritten[i] = 1;
        }
      }
      n.nnWin = w;
      n.nnLoss = l;
      n.flags |= 1;
      cx.addLeafValue(gm.leafNode, w - l, false, true);
    } else if(gm.leafKind == LEAF_TERMINAL) {
      // search.cpp:943-953: value = 2*whiteWinsOfWinner - 1 (SPEC B16: draw = 0)
      real v = gm.leafBoard.winner == 2 ? 1.0f : (gm.leafBoard.winner == 1 ? -1.0f : 0.0f);
      cx.addLeafValue(gm.leafNode, v, true, false);
    } else if(gm.leafKind == LEAF_NOCHILD) {
      Node& n = cx.N(gm.leafNode);
      cx.addLeafValue(gm.leafNode, n.nnWin - n.nnLoss, false, false);
    }
    for(int j = (int)gm.pathNode.size() - 1; j >= 0; j--) {
      int pn = gm.pathNode[j];
      cx.EV(pn, gm.pathSlot[j]) += 1;
      cx.recompute(pn, 1, pn == gm.rootIdx);
    }
    gm.playouts++;
    if(cx.N(gm.rootIdx).visits >= (uint32_t)gm.visitLimit)
      gm.phase = PH_COMMIT;
  }
  // ---- cache write: after every read of this round; in game order, so a slot ends
  // up holding its highest-numbered evaluator (the device's atomicMax bid) ----
  for(int i = 0; i < G; i++) {
    if(!cacheWritten[i])
      continue;
    const CacheWrite& c = cacheWrites[i];
    s.cacheKey[2 * c.slot] = c.k0;
    s.cacheKey[2 * c.slot + 1] = c.k1;
    memcpy(&s.cachePol[(size_t)c.slot * g.P], c.pol.data(), sizeof(float) * g.P);
    s.cacheVal[2 * c.slot] = c.w;
    s.cacheVal[2 * c.slot + 1] = c.l;
  }
  // ---- commit (device kCommit after kBackup): every game waiting in PH_COMMIT; the
  // others stay idle until a commit round (cache writes above are staged copies, so
  // tree reuse / compaction here cannot touch them) ----
  if(commitNow) {
#pragma omp parallel for schedule(dynamic, 4) num_threads(par > 1 ? par : 1) if(par > 1)
    for(int i = 0; i < G; i++) {
      Game& gm = s.games[i];
      if(gm.phase != PH_COMMIT)
        continue;
      Ctx cx(s, gm);
#pragma omp critical(ora_rows)
      cx.commitPending();
    }
  }
  s.rounds++;
}

void selfplaySchedule(Selfplay& s, int commitInterval, int startStagger) {
  s.cfg.commitInterval = commitInterval > 0 ? commitInterval : 1;
  s.cfg.startStagger = startStagger > 0 ? startStagger : 0;
  // device kInit (search.hip:3640-3646): the slot's own seeded delay
  for(Game& gm : s.games)
    gm.startDelay = s.cfg.startStagger > 0
                        ? (int)(mix64(s.cfg.seed ^ 0x5a5a5a5a5a5a5a5aULL ^ (uint64_t)(s.cfg.slotBase + gm.slot)) %
                                (uint64_t)s.cfg.startStagger)
                        : 0;
}

}  // namespace ora
