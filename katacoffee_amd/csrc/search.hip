// Batched KataGo MCTS for Coffee: one wave (64 lanes) per game, thousands of games
// per launch.  A self-play round is three launches on one stream:
//   kSelect  — root-symmetry evaluation or one PUCT descent per game, leaf encoded
//              straight into the network batch (search.cpp:920-1165);
//   network  — fused residual net (nn.hip) or the stand-in net over the batch;
//   kBackup  — NN post-processing, leaf value and path backup (searchupdatehelpers.cpp);
// and every few rounds kCommit plays the chosen move for the games whose root reached
// maxVisits, reuses the subtree and writes finished games' training rows.
//
// Semantics are the oracle's (oracle/ora_search.cpp), which cites the reference
// lines; each function below names its oracle counterpart.  Every float result
// is reproduced bit-for-bit: reductions over children use waveSum (the treeSum64
// order), sequential sums run on lane 0 in the oracle's order, transcendental
// functions are detmath.h's dlog/dexp/dpow, and the file is compiled with
// -ffp-contract=off and correctly rounded division/sqrt.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "detmath.h"
#include "engine.h"
#include "kc_board.h"
#include "search.h"

namespace kc {

static constexpr int SVB_IDX_MOVE1 = MAX_P + 1;
static constexpr int SVB_IDX_PLA = 2 * (MAX_P + 1);
static constexpr int SVB_IDX_PAT = 2 * (MAX_P + 1) + 3;
static constexpr int BIG = 0x7fffffff;

KC_D int64_t svbQ(float x) { return llrintf(x * 4294967296.0f); }
KC_D float svbF(int64_t v) { return (float)v * (1.0f / 4294967296.0f); }

// Search blocks are a single wave and only that wave touches its game's arrays
// during a launch.  A wave's LDS and vector-memory instructions are performed in
// program order, so lane-to-lane visibility (one lane writes, all lanes read)
// needs only a compiler barrier; a __syncthreads() fence would additionally make
// every such step wait for all outstanding global stores to reach L2.
KC_D void waveSync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

#ifdef KC_SEARCH_PROFILE
// Cycle accounting of the search kernels (tools/search_phase.py; profiling build
// only): per-block phase cycles, accumulated in LDS during the kernel and added to
// the block's own slot at exit (no contended atomics inside the timed paths).
//  0 select blocks   1 select total   2 loadGame   3 descend   4 path levels
//  5 selectBest      6 expansion      7 encode
// 10 backup blocks  11 backup total  12 postprocess+order  13 path backup  14 leaf value
// 16 commit blocks  17 commit total  18 move choice+targets  19 tree reuse  20 finishGame
// 21 startGame      22 live nodes kept  23 finished games
constexpr int SPROF_N = 32;
constexpr int SPROF_MAXG = 16384;
__device__ unsigned long long g_searchProf[SPROF_MAXG * SPROF_N];
// NN-cache probe: every evaluated leaf's state key goes into an open-addressing set;
// a key already present counts as a potential cross-game cache hit (slot 9).
__device__ unsigned long long* g_probeKeys = nullptr;
__device__ unsigned long long g_probeMask = 0;
KC_D void probeLeafKey(uint64_t k0, uint64_t k1) {
  if(!g_probeKeys)
    return;
  uint64_t key = (k0 ^ (k1 * 0x9e3779b97f4a7c15ULL)) | 1ull;
  uint64_t i = (key >> 7) & g_probeMask;
  for(int probe = 0; probe < 64; probe++, i = (i + 1) & g_probeMask) {
    const unsigned long long prev = atomicCAS(&g_probeKeys[i], 0ull, (unsigned long long)key);
    if(prev == 0ull)
      return;
    if(prev == key) {
      atomicAdd(&g_searchProf[9], 1ull);
      return;
    }
  }
}
KC_D unsigned long long* sprofLds() {
  __shared__ unsigned long long c[SPROF_N];
  return c;
}
#define SPROF_NOW() clock64()
#define SPROF_INIT()                   \
  do {                                 \
    if(laneId() < SPROF_N)             \
      sprofLds()[laneId()] = 0;        \
    __syncthreads();                   \
  } while(0)
#define SPROF_ADD(i, v)                                 \
  do {                                                  \
    if(laneId() == 0)                                   \
      sprofLds()[(i)] += (unsigned long long)(v);       \
  } while(0)
#define SPROF_FLUSH()                                                           \
  do {                                                                          \
    __syncthreads();                                                            \
    if(laneId() < SPROF_N && blockIdx.x < SPROF_MAXG && laneId() < 24)          \
      g_searchProf[blockIdx.x * SPROF_N + laneId()] += sprofLds()[laneId()];    \
  } while(0)
// per-block maximum of a value over launches (slots 24..31; no contention)
#define SPROF_MAX(i, v)                                                                   \
  do {                                                                                    \
    if(laneId() == 0 && blockIdx.x < SPROF_MAXG) {                                        \
      unsigned long long* q_ = &g_searchProf[blockIdx.x * SPROF_N + (i)];                 \
      const unsigned long long v_ = (unsigned long long)(v);                              \
      if(v_ > *q_)                                                                        \
        *q_ = v_;                                                                         \
    }                                                                                     \
  } while(0)
#else
#define SPROF_NOW() 0ull
#define SPROF_INIT() \
  do {               \
  } while(0)
#define SPROF_ADD(i, v) \
  do {                  \
  } while(0)
#define SPROF_MAX(i, v) \
  do {                  \
  } while(0)
#define SPROF_FLUSH() \
  do {                \
  } while(0)
#endif

// A node's child slots: 0..INLINE_EDGES-1 stored with the node, the rest in its block
// of the game's edge pool (search.h).
struct NodeEdges {
  Edge* inl;
  Edge* pool;  // slot INLINE_EDGES of the node's pool block
  KC_D Edge& operator[](int i) const { return i < INLINE_EDGES ? inl[i] : pool[i - INLINE_EDGES]; }
};

// Per-game view of the SoA arrays.
struct GV {
  const SearchDev& d;
  const DTables& T;
  int g, lane;
  const SP* sp;  // this move's search parameters (moveParams after loadGame)
  mutable int esel = 0;  // the game's current edge-pool buffer (GameDev::edgeSel; setEdgeSel)
  KC_D GV(const SearchDev& d_, int g_) : d(d_), T(*d_.T), g(g_), lane(laneId()), sp(&d_.sp) {}
  // tables through a readonly noalias kernel argument: uniform reads become scalar loads
  KC_D GV(const SearchDev& d_, const DTables& t_, int g_) : d(d_), T(t_), g(g_), lane(laneId()), sp(&d_.sp) {}
  KC_D Node* nodes() const { return d.nodes + (size_t)g * d.cap; }
  KC_D Edge* inlineEdges(int n) const { return d.edges + ((size_t)g * d.cap + n) * INLINE_EDGES; }
  KC_D Edge* edgePool() const { return d.edgePool + ((size_t)g * 2 + esel) * d.edgePoolCap; }
  KC_D void setEdgeSel(int sel) const { esel = __builtin_amdgcn_readfirstlane(sel); }
  // child slots of node n whose pool block starts at ebase (Node::edgeBase)
  KC_D NodeEdges edges(int n, uint32_t ebase) const { return NodeEdges{inlineEdges(n), edgePool() + ebase}; }
  KC_D NodeEdges edges(int n) const { return edges(n, nodes()[n].edgeBase); }
  KC_D uint64_t* nodeKey(int n) const { return d.nodeKey + ((size_t)g * d.cap + n) * 2; }
  KC_D float* pol(int n) const { return d.policy + ((size_t)g * d.cap + n) * d.P; }
  KC_D uint32_t* freeList() const { return d.freeList + (size_t)g * d.cap; }
  KC_D uint32_t* allocBits() const { return d.allocBits + (size_t)g * (d.cap / 32); }
  KC_D uint64_t* ttKey() const { return d.ttKey + (size_t)g * d.ttCap * 2; }
  KC_D int32_t* ttNode() const { return d.ttNode + (size_t)g * d.ttCap; }
  KC_D size_t svbBase(int sel) const { return ((size_t)g * 2 + sel) * d.svbCap; }
  KC_D float* accPolicy() const { return d.accPolicy + (size_t)g * d.P; }
  KC_D float* rawPolicy() const { return d.rawPolicy + (size_t)g * d.P; }
  KC_D float* rootNoised() const { return d.rootNoised + (size_t)g * d.P; }
  KC_D int32_t* pathNode() const { return d.pathNode + (size_t)g * MAX_DEPTH; }
  KC_D int32_t* pathSlot() const { return d.pathSlot + (size_t)g * MAX_DEPTH; }
  KC_D TurnRec* turns() const { return d.turns + (size_t)g * d.maxTurns; }
  KC_D int16_t* turnPol(int t) const { return d.turnPol + ((size_t)g * d.maxTurns + t) * d.P; }
};

// The game's uniform state lives in LDS for the kernel's duration (one wave per
// block): every lane executes the same updates, so same-value LDS writes from
// all lanes are benign and program order keeps them visible to later reads.
// Keeping it out of registers roughly halves the kernels' VGPR use.
static_assert(sizeof(GameDev) % 4 == 0, "GameDev copy granularity");
KC_D void storeGame(const GV& v, const GameDev& s) {
  waveSync();
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&s);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&v.d.games[v.g]);
  for(int i = v.lane; i < (int)(sizeof(GameDev) / 4); i += 64)
    dst[i] = src[i];
}

// The view's per-game settings from the loaded state.
KC_D void bindGame(GV& v, const GameDev& s) {
  // a cheap search without recorded rows runs without root noise and root-specific
  // settings (runBotWithLimits play.cpp:1024-1037); the flag is uniform
  v.sp = __builtin_amdgcn_readfirstlane(s.noNoise) ? &v.d.spCheap : &v.d.sp;
  v.setEdgeSel(s.edgeSel);
}

KC_D void loadGame(GV& v, GameDev& s) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&v.d.games[v.g]);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&s);
  for(int i = v.lane; i < (int)(sizeof(GameDev) / 4); i += 64)
    dst[i] = src[i];
  waveSync();
  bindGame(v, s);
}

template <int NI>
KC_D float tsum(const float (&x)[NI], int n, int lane) {
  float a = 0.0f;
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int i = lane + 64 * j;
    if(i < n)
      a = j == 0 ? x[j] : a + x[j];
  }
  return waveSum(a);
}

KC_D int bcastI(int v, int srcLane) { return bcastLane(v, srcLane); }

// Child slots read speculatively with their node record (2 x 128-B lines of Edge).
constexpr int SPEC_EDGES = INLINE_EDGES;
// descend(): request the likely next node (most-visited inline child) with the children's
// records.  A/B switch, off: bit-exact but slower on the C2 bench (kSelect 64.9-65.1 vs
// 60.3-61.0 us, 23.4 k vs 24.0-24.2 k rows/s, same box: profiles/r05/spec_next_ab.txt) --
// the argmax sits on the critical path and kSelect<2> spills 7 more registers
#ifndef KC_SPEC_NEXT
#define KC_SPEC_NEXT 0
#endif
KC_D int firstLane(uint64_t m) { return __builtin_ctzll(m); }

KC_D float childWeight(uint32_t edgeVisits, uint32_t childVisits, float rawWeight) {
  return rawWeight * ((float)edgeVisits / (float)(childVisits > 1u ? childVisits : 1u));
}

// ---------------------------------------------------------------------------
// Transposition table (oracle ttFind / ttInsert): linear probing, PROBE_W slots per step.
// The node of key (k0, k1) or -1; on a miss emptySlot is where ttInsert would put it
// (the first free slot of the probe sequence; the table is not changed in between).
// A window's slot and key loads are issued together.  The tables are at most half full,
// so a probe almost always ends in its first few slots: a 16-slot window (lanes 0-15;
// 256 B of keys) instead of the whole wave's 64 (1 KB) keeps the same single round trip
// and cuts the bytes a probe pulls from HBM by 4 (PMC: kSelect read 15 MB per launch).
constexpr int PROBE_W = 16;
KC_D int ttFind(const GV& v, uint64_t k0, uint64_t k1, int& emptySlot) {
  const int mask = v.d.ttCap - 1;
  const int start = (int)(k0 & (uint64_t)mask);
  const uint64_t* key = v.ttKey();
  const int32_t* node = v.ttNode();
  emptySlot = -1;
  const bool act = v.lane < PROBE_W;
  for(int base = 0; base < v.d.ttCap; base += PROBE_W) {
    int s = (start + base + v.lane) & mask;
    const int nd = act ? node[s] : 0;
    const uint64_t ka = act ? key[2 * s] : 0ull, kb = act ? key[2 * s + 1] : 0ull;
    bool match = act && nd >= 0 && ka == k0 && kb == k1;
    uint64_t m = ballot(act && (nd < 0 || match));
    if(m) {
      int f = firstLane(m);
      emptySlot = bcastI(s, f);
      return bcastI(match ? nd : -1, f);
    }
  }
  return -1;
}

KC_D void ttInsertAt(const GV& v, int slot, uint64_t k0, uint64_t k1, int nodeIdx) {
  if(slot >= 0 && v.lane == 0) {
    v.ttKey()[2 * slot] = k0;
    v.ttKey()[2 * slot + 1] = k1;
    v.ttNode()[slot] = nodeIdx;
  }
}

// SVB table (oracle svbFindOrInsert), key 0 = empty.  first: this lane's key of the
// first probe window, loaded ahead by svbProbe (its latency overlaps other work).
KC_D uint64_t svbProbe(const GV& v, int sel, uint64_t k) {
  const int mask = v.d.svbCap - 1;
  return v.lane < PROBE_W ? v.d.svbKey[v.svbBase(sel) + (((int)(k & (uint64_t)mask) + v.lane) & mask)] : 0ull;
}
KC_D int svbFindOrInsert(const GV& v, int sel, uint64_t k, uint64_t first) {
  const int mask = v.d.svbCap - 1;
  const size_t b = v.svbBase(sel);
  const int start = (int)(k & (uint64_t)mask);
  const bool act = v.lane < PROBE_W;
  for(int base = 0; base < v.d.svbCap; base += PROBE_W) {
    int s = (start + base + v.lane) & mask;
    uint64_t kk = base == 0 ? first : (act ? v.d.svbKey[b + s] : 0ull);
    uint64_t m = ballot(act && (kk == 0 || kk == k));
    if(m) {
      int f = firstLane(m);
      int slot = bcastI(s, f);
      bool empty = bcastLane((int)(kk == 0), f) != 0;
      if(empty && v.lane == f) {
        v.d.svbKey[b + slot] = k;
        v.d.svbD[b + slot] = 0;
        v.d.svbW[b + slot] = 0;
      }
      return slot;
    }
  }
  return -1;
}

// SPEC a19 key (oracle svbKey): Zmove0[parentPrev] ^ Zmove1[move] ^ Zpla[mover] ^ 5x5 pattern.
KC_D uint64_t svbKeyOf(const GV& v, const DBoard& before, int parentPrevPos, int movePos, int mover) {
  const DTables& T = v.T;
  uint64_t h = 0;
  if(v.lane < 25) {
    int wy = v.lane / 5, wx = v.lane % 5;
    int cell = movePos % T.A;
    int xx = cell % T.X + wx - 2, yy = cell / T.X + wy - 2;
    int col = (xx >= 0 && xx < T.X && yy >= 0 && yy < T.Y) ? colorAt(before, yy * T.X + xx) : 3;
    h = T.svbZ[SVB_IDX_PAT + col * 25 + wy * 5 + wx];
  }
  h = waveXor64(h);
  h ^= T.svbZ[parentPrevPos] ^ T.svbZ[SVB_IDX_MOVE1 + movePos] ^ T.svbZ[SVB_IDX_PLA + mover];
  return h != 0 ? h : 1;
}

// freeIdx: freeList[freeTop - 1] when the caller loaded it ahead, else -1.
KC_D int allocNode(const GV& v, GameDev& s, int nextPla, uint64_t k0, uint64_t k1, bool terminal, int freeIdx = -1) {
  if(s.freeTop <= 0) {
    s.err = ERR_NODE_POOL;
    return -1;
  }
  s.freeTop--;
  int idx = freeIdx >= 0 ? freeIdx : (int)v.freeList()[s.freeTop];
  if(v.lane == 0) {
    Node n;
    n.visits = 0;
    n.weightSum = n.weightSqSum = n.utilityAvg = n.utilitySqAvg = n.winLossAvg = 0.0f;
    n.nnWin = n.nnLoss = n.lastSvbDelta = n.lastSvbWeight = 0.0f;
    n.svbEntry = -1;
    n.numChildren = 0;
    n.nextPla = (uint8_t)nextPla;
    n.flags = terminal ? 2 : 0;
    n.nextPrior = -1.0f;
    n.nextPos = 0xFFFF;
    n.pad0 = 0;
    n.edgeBase = 0;
    n.pad1 = 0;
    v.nodes()[idx] = n;
    v.nodeKey(idx)[0] = k0;
    v.nodeKey(idx)[1] = k1;
    atomicOr(&v.allocBits()[idx >> 5], 1u << (idx & 31));
  }
  s.liveCount++;
  return idx;
}

// ---------------------------------------------------------------------------
// A node's statistics after an update (what its parent's recompute reads).
struct NStats {
  uint32_t visits;
  float weightSum, weightSqSum, utilityAvg, utilitySqAvg, winLossAvg;
};

// oracle addLeafValue (searchupdatehelpers.cpp:12-82); returns the new statistics.
KC_D NStats addLeafValue(const GV& v, const GameDev& s, int ni, float wl, bool isTerminal, bool assumeNoExisting) {
  const SP& sp = *v.sp;
  Node* np = &v.nodes()[ni];
  const int svbEntry = np->svbEntry;
  uint32_t visits = np->visits;
  float weightSum = np->weightSum, weightSqSum = np->weightSqSum;
  float utilityAvg = np->utilityAvg, utilitySqAvg = np->utilitySqAvg, winLossAvg = np->winLossAvg;
  float utility = wl;
  if(sp.svbFactor != 0.0f && !isTerminal && svbEntry >= 0) {
    size_t e = v.svbBase(s.svbSel) + svbEntry;
    float dd = svbF(v.d.svbD[e]), ww = svbF(v.d.svbW[e]);
    if(ww > 0.001f)
      utility = utility + (sp.svbFactor * dd) / ww;
  }
  float usq = utility * utility;
  if(assumeNoExisting) {
    winLossAvg = wl;
    utilityAvg = utility;
    utilitySqAvg = usq;
    weightSqSum = 1.0f;
    weightSum = 1.0f;
    visits += 1;
  } else {
    float oldW = weightSum, newW = oldW + 1.0f;
    winLossAvg = (winLossAvg * oldW + wl) / newW;
    utilityAvg = (utilityAvg * oldW + utility) / newW;
    utilitySqAvg = (utilitySqAvg * oldW + usq) / newW;
    weightSqSum = weightSqSum + 1.0f;
    weightSum = newW;
    visits += 1;
  }
  waveSync();
  if(v.lane == 0) {
    np->visits = visits;
    np->weightSum = weightSum;
    np->weightSqSum = weightSqSum;
    np->utilityAvg = utilityAvg;
    np->utilitySqAvg = utilitySqAvg;
    np->winLossAvg = winLossAvg;
  }
  waveSync();
  return NStats{visits, weightSum, weightSqSum, utilityAvg, utilitySqAvg, winLossAvg};
}

KC_D float cdfT(const DTables& T, float z) {
  float dd = (1999.0f * (z - (-50.0f))) / 100.0f;
  if(dd <= 0.0f)
    return 0.0f;
  int idx = (int)dd;
  if(idx >= 1999)
    return 1.0f;
  float lambda = dd - (float)idx;
  float y0 = T.cdf[idx], y1 = T.cdf[idx + 1];
  return y0 + lambda * (y1 - y0);
}

// oracle recompute (recomputeNodeStats searchupdatehelpers.cpp:151-328 +
// downweightBadChildrenAndNormalizeWeight :330-419) for one path level, after the path
// edge `slot` gained a visit (the oracle's EV(pn, slot) += 1).  Split in three so the
// backup can run the levels as a pipeline: loadLevel (the node record and its first 64
// edges), loadKids (child records, remaining edges, the node's SVB sums), computeLevel
// (arithmetic and stores).  A level's loads are issued while the level below it is
// computed, so the path child's record and (when the two levels share an SVB entry)
// the SVB sums can be stale: computeLevel takes both from the level below (`below`),
// which is exactly what the sequential order would read.
template <int NI>
struct PathLevel {
  int ni, slot, k, nextPla, svbEntry;
  uint32_t ebase;
  float nnWin, nnLoss, lastSvbDelta, lastSvbWeight;
  uint32_t visits0;
  uint32_t ech[NI], evis[NI];  // edge child and visits
  uint32_t cv[NI];
  float cws[NI], cwsq[NI], cu[NI], cusq[NI], cwl[NI];
  int64_t svbD0, svbW0;
};
// What a computed level hands to the level above it.
struct LevelOut {
  NStats st;
  int svbEntry;  // -1: the SVB sums were not written
  int64_t svbD, svbW;
};

template <int NI>
KC_D void loadLevel(const GV& v, int ni, int slot, PathLevel<NI>& L) {
  const Node nd = v.nodes()[ni];
  const Edge* E = v.inlineEdges(ni);
  // the first SPEC_EDGES slots speculatively with the record (slots past numChildren
  // are ignored); the rest once the record says how many there are
  const Edge e0 = v.lane < SPEC_EDGES && v.lane < v.d.P ? E[v.lane] : Edge{0u, 0u, 0.0f, 0u};
  L.ebase = nd.edgeBase;
  L.ech[0] = e0.child;
  L.evis[0] = e0.visits;
  L.ni = ni;
  L.slot = slot;
  L.k = nd.numChildren;
  L.nextPla = nd.nextPla;
  L.svbEntry = nd.svbEntry;
  L.nnWin = nd.nnWin;
  L.nnLoss = nd.nnLoss;
  L.lastSvbDelta = nd.lastSvbDelta;
  L.lastSvbWeight = nd.lastSvbWeight;
  L.visits0 = nd.visits;
}

template <int NI>
KC_D void loadKids(const GV& v, const GameDev& s, PathLevel<NI>& L) {
  const SP& sp = *v.sp;
  const NodeEdges E = v.edges(L.ni, L.ebase);
  const Node* NS = v.nodes();
#pragma unroll
  for(int j = 0; j < NI; j++) {
    const int i = v.lane + 64 * j;
    L.cv[j] = 0;
    L.cws[j] = L.cwsq[j] = L.cu[j] = L.cusq[j] = L.cwl[j] = 0.0f;
    if(j > 0 || i >= SPEC_EDGES)
      L.ech[j] = L.evis[j] = 0u;
    if(i < L.k) {
      if(j > 0 || i >= SPEC_EDGES) {
        const Edge e = E[i];
        L.ech[j] = e.child;
        L.evis[j] = e.visits;
      }
      const Node& c = NS[L.ech[j]];
      L.cv[j] = c.visits;
      L.cws[j] = c.weightSum;
      L.cwsq[j] = c.weightSqSum;
      L.cu[j] = c.utilityAvg;
      L.cusq[j] = c.utilitySqAvg;
      L.cwl[j] = c.winLossAvg;
    }
  }
  // unconditional (entry 0 when the node has none; ignored then): no branch between
  // the pipeline's loads and the waits on them
  const size_t e = v.svbBase(s.svbSel) + (L.svbEntry >= 0 ? L.svbEntry : 0);
  L.svbD0 = v.d.svbD[e];
  L.svbW0 = v.d.svbW[e];
  (void)sp;
}

// issueNext() issues the next levels' loads; it runs right after this level's t-CDF
// table reads, the last loads the level waits on (vmcnt counts in issue order, so a
// wait on a load also waits on every older one).
template <int NI, class F>
KC_D LevelOut computeLevel(const GV& v, const GameDev& s, PathLevel<NI>& L, const LevelOut& below, bool haveBelow,
                           int numVisitsToAdd, bool isRoot, F&& issueNext) {
  const SP& sp = *v.sp;
  const int k = L.k, slot = L.slot;
  const int nextPla = L.nextPla;
  const int svbEntry = L.svbEntry;
  const NodeEdges E = v.edges(L.ni, L.ebase);
  const bool svbOn = sp.svbFactor != 0.0f && svbEntry >= 0;
  int64_t svbD0 = L.svbD0, svbW0 = L.svbW0;
  if(svbOn && haveBelow && below.svbEntry == svbEntry) {
    svbD0 = below.svbD;
    svbW0 = below.svbW;
  }
  bool good[NI];
  float wAdj[NI], selfU[NI], cU[NI], cUsq[NI], cWl[NI], cWs[NI], cWsq[NI], tmp[NI];
  int numGood = 0;
  float maxW = 0.0f;
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int i = v.lane + 64 * j;
    good[j] = false;
    wAdj[j] = selfU[j] = cU[j] = cUsq[j] = cWl[j] = cWs[j] = cWsq[j] = 0.0f;
    if(i < k) {
      uint32_t evis = L.evis[j];
      uint32_t cv = L.cv[j];
      float ws = L.cws[j], wsq = L.cwsq[j], u = L.cu[j], usq = L.cusq[j], wl = L.cwl[j];
      if(i == slot) {
        evis += 1;
        E[i].visits = evis;
        if(haveBelow) {
          cv = below.st.visits;
          ws = below.st.weightSum;
          wsq = below.st.weightSqSum;
          u = below.st.utilityAvg;
          usq = below.st.utilitySqAvg;
          wl = below.st.winLossAvg;
        }
      }
      good[j] = cv > 0 && ws > 0.0f && evis > 0;
      if(good[j]) {
        cU[j] = u;
        cUsq[j] = usq;
        cWl[j] = wl;
        cWs[j] = ws;
        cWsq[j] = wsq;
        selfU[j] = nextPla == 2 ? cU[j] : -cU[j];
        wAdj[j] = childWeight(evis, cv, ws);
        maxW = wAdj[j] > maxW ? wAdj[j] : maxW;
      }
    }
    numGood += __popcll(ballot(good[j]));
  }
  maxW = waveMax(maxW);
  const float origTotal = tsum<NI>(wAdj, k, v.lane);
  const float currentTotal = origTotal;
  float amountToSubtract = 0.0f, amountToPrune = 0.0f;
  if(isRoot && sp.rootNoise) {
    amountToSubtract = fminf(sp.moveSubtract, maxW / 64.0f);
    amountToPrune = fminf(sp.movePrune, maxW / 64.0f);
  }
  if(numGood > 0 && currentTotal > 0.0f) {
    float stdev[NI];
#pragma unroll
    for(int j = 0; j < NI; j++) {
      if(j > 0 && 64 * j >= k) {  // uniform: no lane has an item here
        stdev[j] = tmp[j] = 0.0f;
        continue;
      }
      stdev[j] = good[j] ? sqrtf(1e-8f + 1.0f / (1.5f * sqrtf(wAdj[j]))) : 0.0f;
      tmp[j] = good[j] ? selfU[j] * wAdj[j] : 0.0f;
    }
    const float simpleValue = tsum<NI>(tmp, k, v.lane) / currentTotal;
    // cdfT split: the table reads of every item first, then the next levels' loads,
    // then the interpolation (same arithmetic)
    float y0[NI], y1[NI], lam[NI], pc[NI];
    int mode[NI];  // 0 skip, 1 table, 2 constant pc
#pragma unroll
    for(int j = 0; j < NI; j++) {
      mode[j] = 0;
      y0[j] = y1[j] = lam[j] = pc[j] = 0.0f;
      if(j > 0 && 64 * j >= k)
        continue;
      if(!good[j] || wAdj[j] < amountToPrune)
        continue;
      float z = (selfU[j] - simpleValue) / stdev[j];
      float dd = (1999.0f * (z - (-50.0f))) / 100.0f;
      if(dd <= 0.0f) {
        mode[j] = 2;
        pc[j] = 0.0f;
        continue;
      }
      int idx = (int)dd;
      if(idx >= 1999) {
        mode[j] = 2;
        pc[j] = 1.0f;
        continue;
      }
      mode[j] = 1;
      lam[j] = dd - (float)idx;
      y0[j] = v.T.cdf[idx];
      y1[j] = v.T.cdf[idx + 1];
    }
    issueNext();
#pragma unroll
    for(int j = 0; j < NI; j++) {
      if((j > 0 && 64 * j >= k) || mode[j] == 0) {
        tmp[j] = 0.0f;
        continue;
      }
      float nw = wAdj[j] - amountToSubtract;
      if(nw <= 0.0f)
        nw = 0.0f;
      const float c = mode[j] == 1 ? y0[j] + lam[j] * (y1[j] - y0[j]) : pc[j];
      float p = c + 0.0001f;
      float f = sp.valueWeightExp == 0.5f ? sqrtf(p) : dpow(p, sp.valueWeightExp);
      tmp[j] = nw * f;
    }
    const float totalNew = tsum<NI>(tmp, k, v.lane);
    const float factor = currentTotal / totalNew;
#pragma unroll
    for(int j = 0; j < NI; j++)
      wAdj[j] = tmp[j] * factor;
  } else {
    issueNext();
  }
  float wlv[NI], uv[NI], usqv[NI], wsqv[NI];
#pragma unroll
  for(int j = 0; j < NI; j++) {
    if((j > 0 && 64 * j >= k) || !good[j]) {
      wlv[j] = uv[j] = usqv[j] = wsqv[j] = 0.0f;
      continue;
    }
    float ws = wAdj[j] / cWs[j];
    wlv[j] = wAdj[j] * cWl[j];
    uv[j] = wAdj[j] * cU[j];
    usqv[j] = wAdj[j] * cUsq[j];
    wsqv[j] = (ws * ws) * cWsq[j];
  }
  float winLossSum = tsum<NI>(wlv, k, v.lane);
  float utilitySum = tsum<NI>(uv, k, v.lane);
  float utilitySqSum = tsum<NI>(usqv, k, v.lane);
  float weightSqSum = tsum<NI>(wsqv, k, v.lane);
  float weightSum = currentTotal;
  float wl = L.nnWin - L.nnLoss;
  float utility = wl;
  float newLastD = L.lastSvbDelta, newLastW = L.lastSvbWeight;
  LevelOut out;
  out.svbEntry = -1;
  out.svbD = out.svbW = 0;
  if(svbOn) {
    int64_t D = svbD0, Wt = svbW0;
    if(currentTotal > 1e-10f) {
      float utilityChildren = utilitySum / currentTotal;
      float svbWv = dpow(origTotal, sp.svbExp);
      float svbDv = (utilityChildren - utility) * svbWv;
      D += svbQ(svbDv) - svbQ(L.lastSvbDelta);
      Wt += svbQ(svbWv) - svbQ(L.lastSvbWeight);
      waveSync();
      if(v.lane == 0) {
        const size_t e = v.svbBase(s.svbSel) + svbEntry;
        v.d.svbD[e] = D;
        v.d.svbW[e] = Wt;
      }
      newLastD = svbDv;
      newLastW = svbWv;
      out.svbEntry = svbEntry;
      out.svbD = D;
      out.svbW = Wt;
    }
    float dd = svbF(D), ww = svbF(Wt);
    if(ww > 0.001f)
      utility = utility + (sp.svbFactor * dd) / ww;
  }
  winLossSum = winLossSum + wl;
  utilitySum = utilitySum + utility;
  utilitySqSum = utilitySqSum + utility * utility;
  weightSqSum = weightSqSum + 1.0f;
  weightSum = weightSum + 1.0f;
  out.st.winLossAvg = winLossSum / weightSum;
  out.st.utilityAvg = utilitySum / weightSum;
  out.st.utilitySqAvg = utilitySqSum / weightSum;
  out.st.weightSqSum = weightSqSum;
  out.st.weightSum = weightSum;
  out.st.visits = L.visits0 + (uint32_t)numVisitsToAdd;
  waveSync();
  if(v.lane == 0) {
    Node* np = &v.nodes()[L.ni];
    np->winLossAvg = out.st.winLossAvg;
    np->utilityAvg = out.st.utilityAvg;
    np->utilitySqAvg = out.st.utilitySqAvg;
    np->weightSqSum = out.st.weightSqSum;
    np->weightSum = out.st.weightSum;
    np->visits = out.st.visits;
    np->lastSvbDelta = newLastD;
    np->lastSvbWeight = newLastW;
  }
  waveSync();
  return out;
}

// The path from the deepest level to the root.  The loads of level j-1 (record and
// first edges, then child records) and the record of level j-2 are issued before
// level j is computed; with more than two items per lane (register budget) the
// levels run one at a time.
template <int NI>
KC_D void backupPath(const GV& v, const GameDev& s, int pathLen, NStats leaf, bool haveLeaf) {
  const int32_t* pn = v.pathNode();
  const int32_t* ps = v.pathSlot();
  // the path in registers (lane j holds level j; levels >= 64 re-read), one load
  const int myNode = v.lane < pathLen ? pn[v.lane] : 0, mySlot = v.lane < pathLen ? ps[v.lane] : 0;
  auto nodeAt = [&](int j) { return j < 64 ? bcastLane(myNode, j) : pn[j]; };
  auto slotAt = [&](int j) { return j < 64 ? bcastLane(mySlot, j) : ps[j]; };
  if(pathLen <= 0)
    return;
  LevelOut below;
  bool haveBelow = haveLeaf;
  below.st = leaf;
  below.svbEntry = -1;
  below.svbD = below.svbW = 0;
  int j = pathLen - 1;
  if constexpr(NI > 2) {
    // wide levels (7x7, 9x9): one level at a time
    for(; j >= 0; j--) {
      PathLevel<NI> cur;
      loadLevel<NI>(v, nodeAt(j), slotAt(j), cur);
      loadKids<NI>(v, s, cur);
      below = computeLevel<NI>(v, s, cur, below, haveBelow, 1, cur.ni == s.rootIdx, [] {});
      haveBelow = true;
    }
    return;
  }
  PathLevel<NI> cur, nxt;
  loadLevel<NI>(v, nodeAt(j), slotAt(j), cur);
  if(j > 0)
    loadLevel<NI>(v, nodeAt(j - 1), slotAt(j - 1), nxt);
  loadKids<NI>(v, s, cur);
  for(; j >= 0; j--) {
    PathLevel<NI> nn;
    // the child records of the level above and the record two levels up, issued
    // while this level is computed
    auto issueNext = [&] {
      if(j > 0)
        loadKids<NI>(v, s, nxt);
      if(j > 1)
        loadLevel<NI>(v, nodeAt(j - 2), slotAt(j - 2), nn);
    };
    below = computeLevel<NI>(v, s, cur, below, haveBelow, 1, cur.ni == s.rootIdx, issueNext);
    haveBelow = true;
    if(j > 0) {
      cur = nxt;
      nxt = nn;
    }
  }
}

// oracle fpuValue (searchexplorehelpers.cpp:245-301)
KC_D float fpuValue(const SP& sp, const Node& n, int pla, bool isRoot, float probMass) {
  float parentUtility = n.utilityAvg;
  float forFpu = parentUtility;
  if(sp.fpuByVisited) {
    float pw = sp.fpuByVisitedPow == 2.0f ? probMass * probMass : dpow(probMass, sp.fpuByVisitedPow);
    float avgWeight = fminf(1.0f, pw);
    forFpu = avgWeight * parentUtility + (1.0f - avgWeight) * (n.nnWin - n.nnLoss);
  }
  float redMax = isRoot ? sp.rootFpuRedMax : sp.fpuRedMax;
  float lossProp = isRoot ? sp.rootFpuLossProp : sp.fpuLossProp;
  float reduction = redMax * sqrtf(probMass);
  float fpu = pla == 2 ? forFpu - reduction : forFpu + reduction;
  float lossValue = pla == 2 ? -1.0f : 1.0f;
  fpu = fpu + (lossValue - fpu) * lossProp;
  return fpu;
}

KC_D float exploreScaling(const SP& sp, float totalChildWeight) {
  float c = sp.cpuct;
  if(sp.cpuctLog != 0.0f)
    c = c + sp.cpuctLog * dlog((totalChildWeight + sp.cpuctBase) / sp.cpuctBase);
  return c * sqrtf(totalChildWeight + 0.01f);
}

// oracle selectBest (selectBestChildToDescend searchexplorehelpers.cpp:304-451)
// Also returns the chosen existing child's edge and the child's visits and flags,
// broadcast from the lane that holds them (no reload of either after the choice).
template <int NI>
KC_D int selectBest(const GV& v, int ni, const Node& n, const float* pol, bool isRoot, int& newPos,
                    uint32_t* hasBits, const Edge& e0, Edge& ce, uint32_t& cVisits, uint32_t& cFlags, int* specChild = nullptr,
                    Edge* specE0 = nullptr, Node* specN = nullptr) {
  const SP& sp = *v.sp;
  const int P = v.d.P;
  const int k = n.numChildren;
  const int pla = n.nextPla;
  if(isRoot) {
    for(int w = v.lane; w < (P + 31) / 32; w += 64)
      hasBits[w] = 0;
    waveSync();
  }
  const NodeEdges E = v.edges(ni, n.edgeBase);
  const Node* NS = v.nodes();
  float probs[NI], cw[NI], pv[NI], cu[NI];
  uint32_t cvis[NI], cfl[NI];
  Edge ev[NI];
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int i = v.lane + 64 * j;
    probs[j] = cw[j] = pv[j] = cu[j] = 0.0f;
    cvis[j] = cfl[j] = 0;
    ev[j] = Edge{0u, 0u, 0.0f, 0u};
    if(j > 0 && 64 * j >= k)  // uniform: no lane has an item here
      continue;
    if(i < k) {
      const Edge e = j == 0 && i < SPEC_EDGES ? e0 : E[i];
      ev[j] = e;
      const Node& c = NS[e.child];
      float p = isRoot ? pol[e.move] : e.prior;
      cvis[j] = c.visits;
      cfl[j] = c.flags;
      cu[j] = c.utilityAvg;
      pv[j] = p;
      probs[j] = p < 0.0f ? 0.0f : p;
      cw[j] = p < 0.0f ? 0.0f : childWeight(e.visits, cvis[j], c.weightSum);
      if(isRoot)
        atomicOr(&hasBits[e.move >> 5], 1u << (e.move & 31));
    }
  }
  if(specChild) {
    // the next level, speculatively: the inline child with the most edge visits (the
    // usual pick once a node has visits) -- its record and inline edges are requested
    // behind the children's records, so a hit saves the next level's first round trip
    float sv = v.lane < k && v.lane < SPEC_EDGES ? (float)e0.visits : -1.0f;
    int si = v.lane;
    waveArgmax(sv, si);
    const int sc = sv >= 0.0f ? bcastLane((int)e0.child, si) : -1;
    *specChild = sc;
    if(sc >= 0) {
      *specE0 = v.lane < SPEC_EDGES && v.lane < v.d.P ? v.inlineEdges(sc)[v.lane] : Edge{0u, 0u, 0.0f, 0u};
      *specN = NS[sc];
    }
  }
  const float probMass = tsum<NI>(probs, k, v.lane);
  const float total = tsum<NI>(cw, k, v.lane);
  const float fpu = fpuValue(sp, n, pla, isRoot, probMass);
  const float scaling = exploreScaling(sp, total);
  float best = -__builtin_inff();
  int bestIdx = BIG;
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int i = v.lane + 64 * j;
    if((j > 0 && 64 * j >= k) || i >= k)
      continue;
    float p = pv[j];
    float val;
    if(p < 0.0f)
      val = -__builtin_inff();
    else {
      float w = cw[j];
      float u = (cvis[j] == 0 || w <= 0.0f) ? fpu : cu[j];
      if(isRoot && sp.rootDesiredCoeff > 0.0f && p > 0.0f && w < sqrtf((p * total) * sp.rootDesiredCoeff))
        val = 1e20f;
      else
        val = (scaling * p) / (1.0f + w) + (pla == 2 ? u : -u);
    }
    if(val > best) {
      best = val;
      bestIdx = i;
    }
  }
  waveArgmax(best, bestIdx);
  int bestSlot = best > -__builtin_inff() ? bestIdx : -1;
  if(bestSlot >= 0) {
    Edge me{0u, 0u, 0.0f, 0u};
    uint32_t mv = 0, mf = 0;
#pragma unroll
    for(int j = 0; j < NI; j++)
      if(j == (bestSlot >> 6)) {
        me = ev[j];
        mv = cvis[j];
        mf = cfl[j];
      }
    const int bl = bestSlot & 63;
    ce.child = (uint32_t)bcastLane((int)me.child, bl);
    ce.visits = (uint32_t)bcastLane((int)me.visits, bl);
    ce.move = (uint32_t)bcastLane((int)me.move, bl);
    ce.prior = 0.0f;
    cVisits = (uint32_t)bcastLane((int)mv, bl);
    cFlags = (uint32_t)bcastLane((int)mf, bl);
  }
  float bp = -1.0f;
  int bpos = BIG;
  if(isRoot) {
    // root priors carry noise: scan every unexpanded legal move
    waveSync();
    for(int pos = v.lane; pos < P; pos += 64) {
      if((hasBits[pos >> 5] >> (pos & 31)) & 1u)
        continue;
      float p = pol[pos];
      if(p < 0.0f)
        continue;
      if(p > bp) {
        bp = p;
        bpos = pos;
      }
    }
    waveArgmax(bp, bpos);
  } else if(n.nextPos != 0xFFFF) {
    // non-root: children are always created in prior order, so the best
    // unexpanded move is the k-th entry of the node's expansion order, which
    // the node record caches
    bp = n.nextPrior;
    bpos = n.nextPos;
  }
  newPos = -1;
  if(bpos != BIG) {
    float val = (scaling * bp) / 1.0f + (pla == 2 ? fpu : -fpu);
    if(val > best) {
      bestSlot = k;
      newPos = bpos;
    }
  }
  return bestSlot;
}

// A non-root node's expansion order is its legal moves by descending prior, ties by
// ascending position -- the order selectBest's new-child scan yields
// (selectBestChildToDescend searchexplorehelpers.cpp:304-451: "first strictly
// greater" over positions).  The node caches only its next entry (Node::nextPrior /
// nextPos); the entry after (curPrior, curPos) is found when that one is expanded by
// one scan of the node's policy: the highest prior below curPrior, or equal to it at a
// higher position.  pv: the node's policy, lane-strided (illegal = -1).  No entry:
// (-1, 0xFFFF).
template <int NI>
KC_D void nextExpansion(const GV& v, const float (&pv)[NI], float curPrior, int curPos, float& nPrior, int& nPos) {
  const int P = v.d.P;
  float best = -1.0f;
  int bi = BIG;
#pragma unroll
  for(int j = 0; j < NI; j++) {
    const int p = v.lane + 64 * j;
    const float x = pv[j];
    if(p < P && x >= 0.0f && (x < curPrior || (x == curPrior && p > curPos)) && x > best) {
      best = x;
      bi = p;
    }
  }
  waveArgmax(best, bi);
  nPrior = bi != BIG ? best : -1.0f;
  nPos = bi != BIG ? bi : 0xFFFF;
}

// oracle descend (playoutDescend search.cpp:936-1165, allocateOrFindNode :704-759,
// maybeCatchUpEdgeVisits :1169-1207)
// KC_TT_EARLY 1: an expansion that lands on a transposition requests the child's record
// right after the table probe; 0: after the edge and node stores.  Measured (round 6, C2
// fast, 4 groups, profiles/r06/tt_early_ab.txt): 25.81 / 25.84 k rows/s early against
// 25.97 / 25.94 k late, bit-exact either way: off
#ifndef KC_TT_EARLY
#define KC_TT_EARLY 0
#endif
template <int NI>
KC_D void descend(const GV& v, GameDev& s, uint32_t* hasBits, float* rootPol /* LDS [P] */) {
  const SP& sp = *v.sp;
  const DTables& T = v.T;
  s.pathLen = 0;
  DBoard b = s.root;
  int ni = s.rootIdx;
  uint32_t scanned = 0;  // children of the path nodes (tree-roofline accounting)
  // the first SPEC_EDGES child slots (two cache lines) are read speculatively,
  // together with the node record (slots past numChildren are ignored), saving
  // a dependent round trip; wider speculation would touch cold lines.  Each
  // level's loads are issued before anything waits on the previous level.
  auto loadE0 = [&](int node) {
    return v.lane < SPEC_EDGES && v.lane < v.d.P ? v.inlineEdges(node)[v.lane] : Edge{0u, 0u, 0.0f, 0u};
  };
  Edge e0 = loadE0(ni);
  Node n = v.nodes()[ni];
  // the node an expansion will take (one expansion ends a descent)
  const int freeIdx = s.freeTop > 0 ? (int)v.freeList()[s.freeTop - 1] : -1;
  {
    // the root's noised policy into LDS: the root selection gathers it per child and
    // scans it for the best unexpanded move
    const float* rn = v.rootNoised();
    float pr[NI];
#pragma unroll
    for(int j = 0; j < NI; j++) {
      const int p = v.lane + 64 * j;
      pr[j] = p < v.d.P ? rn[p] : 0.0f;
    }
#pragma unroll
    for(int j = 0; j < NI; j++) {
      const int p = v.lane + 64 * j;
      if(p < v.d.P)
        rootPol[p] = pr[j];
    }
    waveSync();
  }
  while(true) {
    if(n.flags & 2) {
      s.leafKind = LEAF_TERMINAL;
      s.leafNode = ni;
      s.leaf = b;
      break;
    }
    const bool isRoot = ni == s.rootIdx;
    const float* pol = isRoot ? rootPol : v.pol(ni);
    int newPos = -1;
    scanned += n.numChildren;
    const unsigned long long tSel = SPROF_NOW();
    Edge ce{0u, 0u, 0.0f, 0u};
    uint32_t cVisits = 0, cFlags = 0;
    int specChild = -1;
    Edge specE0{0u, 0u, 0.0f, 0u};
    Node specN;
    int slot = KC_SPEC_NEXT ? selectBest<NI>(v, ni, n, pol, isRoot, newPos, hasBits, e0, ce, cVisits, cFlags, &specChild,
                                             &specE0, &specN)
                            : selectBest<NI>(v, ni, n, pol, isRoot, newPos, hasBits, e0, ce, cVisits, cFlags);
    SPROF_ADD(5, SPROF_NOW() - tSel);
    (void)tSel;
    if(slot < 0) {
      s.leafKind = LEAF_NOCHILD;
      s.leafNode = ni;
      break;
    }
    if(slot == n.numChildren) {
      const unsigned long long tExp = SPROF_NOW();
      (void)tExp;
      // the node's policy (non-root: the scan for its following expansion candidate) or
      // the root move's raw prior, requested first: the loads fly while the move is
      // played and the SVB / transposition probes run, and are consumed afterwards
      float pvn[NI];
      float rootPrior = 0.0f;
      {
        const float* pp = v.pol(ni);
#pragma unroll
        for(int j = 0; j < NI; j++) {
          const int p = v.lane + 64 * j;
          pvn[j] = !isRoot && p < v.d.P ? pp[p] : -1.0f;
        }
        if(isRoot)
          rootPrior = pp[newPos];
      }
      // child slot `slot` past the inline ones lives in the node's edge-pool block,
      // allocated (16 -> 64 slots) or grown (-> P) here; pool exhaustion ends the
      // descent like node-pool exhaustion (a counted device error)
      uint32_t ebase = n.edgeBase;
      int reserved = 0;  // pool entries taken for this expansion (returned if it fails)
      if(slot == INLINE_EDGES || (slot == 64 && v.d.P > 64)) {
        const int need = edgeBlockCap(slot + 1, v.d.P);
        if(s.edgeTop + need > v.d.edgePoolCap) {
          s.err = ERR_EDGE_POOL;
          s.leafKind = LEAF_NOCHILD;
          s.leafNode = ni;
          break;
        }
        const uint32_t nb = (uint32_t)s.edgeTop;
        s.edgeTop += need;
        s.edgePeak = max(s.edgePeak, s.edgeTop);
        reserved = need;
        if(slot > INLINE_EDGES) {
          Edge* pool = v.edgePool();
          for(int i = v.lane; i < slot - INLINE_EDGES; i += 64)
            pool[nb + i] = pool[ebase + i];
        }
        ebase = nb;
      }
      const float prior = isRoot ? rootPrior : n.nextPrior;
      const int cell = newPos % T.A, dir = newPos / T.A;
      // SVB key of the expansion (needs the board before the move); computed
      // up front so no second board copy stays live across playMoveWave.
      const bool svbKeyed = sp.svbFactor != 0.0f && hCell(b, 0) >= 0;
      uint64_t svbKey = 0, svbFirst = 0;
      if(svbKeyed) {
        svbKey = svbKeyOf(v, b, hDir(b, 0) * T.A + hCell(b, 0), newPos, b.pla);
        svbFirst = svbProbe(v, s.svbSel, svbKey);
      }
      playMoveWave(T, b, cell, dir);
      uint64_t k0, k1;
      stateHash(T, b, k0, k1);
      int ttSlot = -1;
      int child = sp.useGraph ? ttFind(v, k0, k1, ttSlot) : -1;
      const bool fresh = child < 0;
      // a transposition's record (visits, terminal flag) is requested here, so its latency
      // overlaps the next-candidate scan and the stores below; nothing in this descent
      // writes it (a child always holds more stones than its parent: never ni)
      uint32_t tVisits = 0u, tFlags = 0u;
      if(KC_TT_EARLY && !fresh) {
        const Node& cn = v.nodes()[child];
        tVisits = cn.visits;
        tFlags = (uint32_t)cn.flags;
      }
      float nxtPrior = -1.0f;
      int nxtPos = 0xFFFF;
      if(!isRoot)
        nextExpansion<NI>(v, pvn, n.nextPrior, n.nextPos, nxtPrior, nxtPos);
      if(fresh) {
        child = allocNode(v, s, b.pla, k0, k1, b.finished != 0, freeIdx);
        if(child < 0) {
          s.edgeTop -= reserved;  // the block was never linked to the node
          s.leafKind = LEAF_NOCHILD;
          s.leafNode = ni;
          break;
        }
        if(svbKeyed) {
          int e = svbFindOrInsert(v, s.svbSel, svbKey, svbFirst);
          waveSync();
          if(v.lane == 0)
            v.nodes()[child].svbEntry = e;
        }
        if(sp.useGraph)
          ttInsertAt(v, ttSlot, k0, k1, child);
      }
      waveSync();
      if(v.lane == 0) {
        v.edges(ni, ebase)[slot] = Edge{(uint32_t)child, 0u, prior, (uint32_t)newPos};
        v.nodes()[ni].numChildren = (uint16_t)(slot + 1);
        v.nodes()[ni].edgeBase = ebase;
        if(!isRoot) {
          v.nodes()[ni].nextPos = (uint16_t)nxtPos;
          v.nodes()[ni].nextPrior = nxtPrior;
        }
        v.pathNode()[s.pathLen] = ni;
        v.pathSlot()[s.pathLen] = slot;
      }
      s.pathLen++;
      waveSync();
      SPROF_ADD(6, SPROF_NOW() - tExp);
      // a fresh node has no visits and the terminal flag of b; a transposition's
      // record is read
      const uint32_t cv = fresh ? 0u : (KC_TT_EARLY ? tVisits : v.nodes()[child].visits);
      const uint32_t cf = fresh ? (b.finished ? 2u : 0u) : (KC_TT_EARLY ? tFlags : (uint32_t)v.nodes()[child].flags);
      if(cv > 0) {
        s.leafKind = LEAF_CATCHUP;
        s.leafNode = child;
        break;
      }
      s.leafNode = child;
      s.leaf = b;
      s.leafKind = (cf & 2) ? LEAF_TERMINAL : LEAF_NN;
      break;
    }
    const int child = (int)ce.child;
    if(v.lane == 0) {
      v.pathNode()[s.pathLen] = ni;
      v.pathSlot()[s.pathLen] = slot;
    }
    s.pathLen++;
    if(ce.visits < cVisits) {
      s.leafKind = LEAF_CATCHUP;
      s.leafNode = child;
      break;
    }
    // existing child: its terminal flag already says whether the move ends the game
    const int mv = (int)ce.move, mover = b.pla;
    applyMove(T, b, mv % T.A, mv / T.A);
    if(cFlags & 2) {
      b.finished = 1;
      b.winner = maxRun(T, b, mv % T.A) >= T.W ? mover : 0;
    }
    ni = child;
    if(KC_SPEC_NEXT && child == specChild) {
      // (no node or edge is written before a descent's last level: the speculative
      // copies are what the loads would return)
      e0 = specE0;
      n = specN;
    } else {
      e0 = loadE0(ni);
      n = v.nodes()[ni];
    }
  }
  s.treeLevels += (uint64_t)s.pathLen;
  s.treeChildren += scanned;
}

// ---------------------------------------------------------------------------
// kSelect: root evaluation or one descent; NN leaves are encoded into the batch.

// NN evaluation cache lookup of an NN leaf (SPEC a7): a state evaluated in an earlier
// round by any game is taken from the cache instead of the network.  The payload is
// loaded with the key and a hit copies it into the leaf's policy.  fused (kBackupSelect):
// the slot's tag is loaded too -- a bid of this round (tag != 0) means this round's
// backups, running beside this selection, write the slot, so the lookup is left to
// kResolve (LEAF_PENDING); any other slot is not written during the kernel.
template <int NI>
KC_D void cacheLookup(const GV& v, GameDev& s, bool fused) {
  const SearchDev& d = v.d;
  const uint64_t k0 = v.nodeKey(s.leafNode)[0], k1 = v.nodeKey(s.leafNode)[1];
  const uint32_t slot = cacheSlot(k0, k1, d.cacheMask);
  const int P = d.P;
  const float* cp = d.cPol + (size_t)slot * P;
  float pv[NI];
#pragma unroll
  for(int j = 0; j < NI; j++) {
    const int pos = v.lane + 64 * j;
    pv[j] = pos < P ? cp[pos] : 0.0f;
  }
  const float cw = d.cVal[2 * (size_t)slot], cl = d.cVal[2 * (size_t)slot + 1];
  const uint32_t tag = fused ? d.cTag[slot] : 0u;
  s.cSlot = (int32_t)slot;
  if(tag != 0u) {
    s.leafKind = LEAF_PENDING;
    if(v.lane == 0)
      d.pendList[atomicAdd(d.pendCount, 1)] = v.g;  // rare: a same-round transposition
    return;
  }
  if(d.cKey[2 * (size_t)slot] == k0 && d.cKey[2 * (size_t)slot + 1] == k1) {
    s.leafKind = LEAF_CACHED;
    s.cHitWin = cw;
    s.cHitLoss = cl;
    float* pol = v.pol(s.leafNode);
#pragma unroll
    for(int j = 0; j < NI; j++) {
      const int pos = v.lane + 64 * j;
      if(pos < P)
        pol[pos] = pv[j];
    }
  }
}

// The end of a selection: an NN leaf draws its symmetry, the game's batch row is encoded
// when the leaf needs the network, and the game state is stored.
KC_D void finishSelect(const GV& v, GameDev& s, DRng& rng) {
  const SearchDev& d = v.d;
  const int g = v.g;
  if(s.leafKind == LEAF_NN)
    s.leafSym = (int)rng.below(8);
  s.rngCtr = rng.ctr;
  const bool needNN =
      s.leafKind == LEAF_NN || s.leafKind == LEAF_ROOTEVAL || s.leafKind == LEAF_INIT || s.leafKind == LEAF_FORK ||
      s.leafKind == LEAF_SIDE;
  if(v.lane == 0) {
    d.nnNeed[g] = needNN ? 1 : 0;
    if(needNN)
      d.nnBid[g] = s.leafKind == LEAF_NN && d.cacheOn ? (uint32_t)s.cSlot : ~0u;
  }
  if(needNN) {
    // the game's own batch row: no shared counter (a same-address atomic from
    // every block serialises at L2); kCompact lists the rows the network evaluates
    const int slot = g;
    s.nnSlot = slot;
    s.nnEvals++;
    encodePackedWave(v.T, s.leaf, s.leafSym, d.nnIn + (size_t)slot * d.inWords);
  }
  waveSync();
  storeGame(v, s);
}

// One game's selection.  s: the game's LDS copy, already holding its state when `loaded`
// (the fused kernel's backup just ran; every path below then stores it).  rootPol: LDS [MAX_P].
template <int NI>
KC_D void selectBody(const SearchDev& d, const DTables& T, int g, GameDev& s, bool loaded, bool fused,
                     uint32_t* hasBits, float* rootPol) {
  GV v(d, T, g);
  SPROF_INIT();
  const unsigned long long t0 = SPROF_NOW();
  if(d.nnDefer[g]) {
    // the leaf from an earlier round still waits for the network (kCompact); the
    // game state stays as it is
    if(v.lane == 0)
      d.nnNeed[g] = 1;
    return;
  }
  if(loaded)
    bindGame(v, s);
  else
    loadGame(v, s);
  if(s.phase == PH_COMMIT || s.startDelay > 0) {
    s.leafKind = LEAF_NONE;
    if(loaded) {
      // the fused kernel's backup left the state to be stored here
      if(s.startDelay > 0)
        s.startDelay = s.startDelay - 1;
      storeGame(v, s);
      if(v.lane == 0)
        d.nnNeed[g] = 0;
      return;
    }
    if(v.lane == 0) {
      d.games[g].leafKind = LEAF_NONE;
      if(s.startDelay > 0)
        d.games[g].startDelay = s.startDelay - 1;
      d.nnNeed[g] = 0;
    }
    return;
  }
  const unsigned long long t1 = SPROF_NOW();
  (void)t0;
  (void)t1;
  DRng rng = DRng{s.rngSeed, s.rngCtr};
  if(s.phase == PH_INIT) {
    // policy-initialisation move: one evaluation of the root, random symmetry
    s.leafKind = LEAF_INIT;
    s.leafSym = (int)rng.below(8);
    s.leaf = s.root;
  } else if(s.phase == PH_SIDEEVAL) {
    // side-position continuation: the position after the search's response (set by
    // kCommit in s.leaf), random symmetry
    s.leafKind = LEAF_SIDE;
    s.leafSym = (int)rng.below(8);
  } else if(s.phase == PH_FORK) {
    // fork candidate: the position after the next candidate move, random symmetry
    const ForkRec* f = d.fork + g;
    const int mv = f->moves[f->next];
    s.leaf = f->board;
    playMoveWave(v.T, s.leaf, mv % v.T.A, mv / v.T.A);
    s.leafKind = LEAF_FORK;
    s.leafSym = (int)rng.below(8);
  } else if(s.phase == PH_ROOTEVAL) {
    if(s.rootK == 0) {
      // partial Fisher-Yates over 0..7, kept as packed nibbles (no dynamic register indexing)
      uint32_t idx = 0x76543210u;
#pragma unroll
      for(int k = 0; k < 4; k++) {
        int j = k + (int)rng.below((uint32_t)(8 - k));
        uint32_t a = (idx >> (4 * k)) & 15u, b = (idx >> (4 * j)) & 15u;
        idx = (idx & ~(15u << (4 * k)) & ~(15u << (4 * j))) | (b << (4 * k)) | (a << (4 * j));
      }
      s.syms = idx & 0xFFFFu;
    }
    s.leafKind = LEAF_ROOTEVAL;
    s.leafSym = (int)((s.syms >> (4 * s.rootK)) & 15u);
    s.leaf = s.root;
  } else {
    descend<NI>(v, s, hasBits, rootPol);
    if(s.leafKind == LEAF_NN && d.cacheOn)
      cacheLookup<NI>(v, s, fused);
  }
  const unsigned long long t2 = SPROF_NOW();
  (void)t2;
  finishSelect(v, s, rng);
  SPROF_ADD(0, 1);
  SPROF_MAX(24, SPROF_NOW() - t0);
  SPROF_MAX(25, s.pathLen);
  SPROF_ADD(1, SPROF_NOW() - t0);
  SPROF_ADD(2, t1 - t0);
  SPROF_ADD(3, t2 - t1);
  SPROF_ADD(4, s.pathLen);
  SPROF_ADD(7, SPROF_NOW() - t2);
  SPROF_FLUSH();
}

template <int NI>
__global__ void __launch_bounds__(64, NI <= 2 ? 4 : 2) kSelect(const SearchDev* __restrict__ dp, const DTables* __restrict__ Tp,
                                                                int resetCommit) {
  const SearchDev& d = *dp;
  const int g = blockIdx.x;
  // the previous commit's list is consumed (kCommit/kRows ran before this kernel);
  // this round's kBackup appends to an empty one
  if(resetCommit && g == 0 && threadIdx.x == 0)
    *d.commitCount = 0;
  if(g >= d.G)
    return;
  __shared__ uint32_t hasBits[(MAX_P + 31) / 32];
  __shared__ GameDev s;
  __shared__ float rootPol[MAX_P];
  selectBody<NI>(d, *Tp, g, s, false, false, hasBits, rootPol);
}

// The selections a fused kernel left pending: the cache slot is final now (every backup
// of the round has run), so the lookup and the rest of the selection complete here, in
// the order kSelect runs them (the symmetry draw comes after the lookup).  Each round
// winner's tag is cleared too (before the next kCompact bids).  A small grid: block b
// clears the tags of games b, b + grid, ... and completes pending entries b, b + grid, ...
constexpr int RESOLVE_GRID = 64;
// The two halves of a resolve, shared by kResolve and the resolving kCompact: clearing
// the round winners' tags (entries first, first + stride, ...) and completing the pending
// selections (entries first, first + stride, ...; one wave each, s its LDS game copy).
KC_D void clearRoundTags(const SearchDev& d, int first, int stride) {
  for(int i = first; i < d.G; i += stride) {
    const uint32_t cc = d.cClear[i];
    if(cc != 0u) {
      d.cTag[cc - 1u] = 0u;
      d.cClear[i] = 0u;
    }
  }
}
template <int NI>
KC_D void completePending(const SearchDev& d, const DTables& T, int first, int stride, GameDev& s) {
  const int np = *d.pendCount;
  for(int k = first; k < np; k += stride) {
    const int g = __builtin_amdgcn_readfirstlane(d.pendList[k]);
    GV v(d, T, g);
    loadGame(v, s);
    s.leafKind = LEAF_NN;
    cacheLookup<NI>(v, s, false);
    DRng rng = DRng{s.rngSeed, s.rngCtr};
    finishSelect(v, s, rng);
  }
}
template <int NI>
__global__ void __launch_bounds__(64) kResolve(const SearchDev* __restrict__ dp, const DTables* __restrict__ Tp) {
  const SearchDev& d = *dp;
  clearRoundTags(d, blockIdx.x * 64 + laneId(), RESOLVE_GRID * 64);
  __shared__ GameDev s;
  completePending<NI>(d, *Tp, blockIdx.x, RESOLVE_GRID, s);
}

// oracle postprocess (nneval.cpp:702-815 + copyOutputsWithSymmetry nninputs.cpp:349-357)
template <int NI>
// The network row is staged in LDS (one coalesced read) and gathered from there in
// the symmetric frame; pv returns each lane's policy values for buildOrder.
// `stage` (>= P+4 floats) may alias polDst.
KC_D void postprocess(const GV& v, const DBoard& b, int sym, const float* out, float* polDst, float& whiteWin,
                      float& whiteLoss, float* stage, float (&pv)[NI]) {
  const DTables& T = v.T;
  const int P = T.P, A = T.A;
  if(T.X != T.Y)
    sym &= 3;
  float raw[NI + 1];
#pragma unroll
  for(int j = 0; j <= NI; j++) {
    const int i = v.lane + 64 * j;
    raw[j] = i < P + 4 ? out[i] : 0.0f;
  }
  int src[NI];
  bool legal[NI];
#pragma unroll
  for(int j = 0; j < NI; j++) {
    const int pos = v.lane + 64 * j;
    legal[j] = false;
    src[j] = 0;
    if(pos < P) {
      const int dd = pos / A, cell = pos % A;
      legal[j] = isLegal(T, b, cell, dd);
      src[j] = T.symDir[sym][dd] * A + T.symCell[sym][cell];
    }
  }
  waveSync();
#pragma unroll
  for(int j = 0; j <= NI; j++) {
    const int i = v.lane + 64 * j;
    if(i < P + 4)
      stage[i] = raw[j];
  }
  waveSync();
  float logit[NI];
  float mx = -1e25f;
  int legalCount = 0;
#pragma unroll
  for(int j = 0; j < NI; j++) {
    const int pos = v.lane + 64 * j;
    logit[j] = -1e30f;
    if(pos < P) {
      logit[j] = legal[j] ? stage[src[j]] : -1e30f;
      mx = logit[j] > mx ? logit[j] : mx;
    }
    legalCount += __popcll(ballot(legal[j]));
  }
  const float wlg = stage[P], llg = stage[P + 1];
  waveSync();
  mx = waveMax(mx);
  float e[NI];
#pragma unroll
  for(int j = 0; j < NI; j++)
    e[j] = dexp(logit[j] - mx);
  const float sum = tsum<NI>(e, P, v.lane);
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int pos = v.lane + 64 * j;
    pv[j] = legal[j] ? (sum <= 0.0f ? 1.0f / (float)legalCount : e[j] / sum) : -1.0f;
    if(pos < P)
      polDst[pos] = pv[j];
  }
  float m = wlg > llg ? wlg : llg;
  float wp = dexp(wlg - m), lp = dexp(llg - m);
  float ps = wp + lp;
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

KC_D float interpolateEarly(const DTables& T, int turn, float halflife, float earlyValue, float value) {
  float rawHalflives = (float)turn / halflife;
  float halflives = rawHalflives * (19.0f / sqrtf((float)(T.X * T.Y)));
  return value + (earlyValue - value) * dpow(0.5f, halflives);
}

// Sequential in-order sum of lds[0..n) (the oracle's plain loops), result to all lanes.
KC_D float seqSum(float* lds, int n, int lane) {
  waveSync();
  float acc = 0.0f;
  if(lane == 0)
    for(int i = 0; i < n; i++)
      acc = acc + lds[i];
  return bcastLaneF(acc, 0);
}

// oracle noiseAndTemp (maybeAddPolicyNoiseAndTemp searchhelpers.cpp:122-222)
KC_D void noiseAndTemp(const GV& v, GameDev& s, DRng& rng, const float* raw, float* out, float* scratch) {
  const SP& sp = *v.sp;
  const int P = v.d.P;
  for(int pos = v.lane; pos < P; pos += 64)
    out[pos] = raw[pos];
  waveSync();
  if(sp.rootTemp != 1.0f || sp.rootTempEarly != 1.0f) {
    float t = interpolateEarly(v.T, s.root.turn, sp.moveTempHalflife, sp.rootTempEarly, sp.rootTemp);
    float mx = 0.0f;
    for(int pos = v.lane; pos < P; pos += 64)
      mx = out[pos] > mx ? out[pos] : mx;
    mx = waveMax(mx);
    float logMax = dlog(mx);
    float invTemp = 1.0f / t;
    for(int pos = v.lane; pos < P; pos += 64) {
      float o = out[pos];
      float p = 0.0f;
      if(o > 0.0f) {
        p = dexp((dlog(o) - logMax) * invTemp);
        out[pos] = p;
      }
      scratch[pos] = p;  // zero terms do not change the in-order sum
    }
    float sum = seqSum(scratch, P, v.lane);
    waveSync();
    for(int pos = v.lane; pos < P; pos += 64)
      if(out[pos] >= 0.0f)
        out[pos] = out[pos] / sum;
    waveSync();
  }
  if(sp.rootNoise) {
    // computeDirichletAlphaDistribution searchhelpers.cpp:51-91
    int legalCount = 0;
    for(int base = 0; base < P; base += 64) {
      int pos = base + v.lane;
      legalCount += __popcll(ballot(pos < P && out[pos] >= 0.0f));
    }
    float* alpha = scratch;          // [P]
    float* r = scratch + MAX_P;      // [P]
    for(int pos = v.lane; pos < P; pos += 64)
      alpha[pos] = out[pos] >= 0.0f ? dlog(fminf(0.01f, out[pos]) + 1e-20f) : 0.0f;
    float logSum = seqSum(alpha, P, v.lane);
    float logMean = logSum / (float)legalCount;
    waveSync();
    for(int pos = v.lane; pos < P; pos += 64)
      alpha[pos] = out[pos] >= 0.0f ? fmaxf(0.0f, alpha[pos] - logMean) : 0.0f;
    float propSum = seqSum(alpha, P, v.lane);
    float uniform = 1.0f / (float)legalCount;
    waveSync();
    for(int pos = v.lane; pos < P; pos += 64)
      if(out[pos] >= 0.0f)
        alpha[pos] = propSum <= 0.0f ? uniform : 0.5f * (alpha[pos] / propSum + uniform);
    // addDirichletNoise searchhelpers.cpp:93-120; SPEC a24 per-move sub-streams
    const uint64_t base = rng.next();
    for(int pos = v.lane; pos < P; pos += 64) {
      float rv = 0.0f;
      if(out[pos] >= 0.0f) {
        DRng sub{mix64(base ^ ((uint64_t)(pos + 1) * 0x9e3779b97f4a7c15ULL)), 0};
        rv = sub.gamma(alpha[pos] * sp.dirConc);
      }
      r[pos] = rv;
    }
    float rSum = seqSum(r, P, v.lane);
    waveSync();
    float w = sp.dirWeight;
    for(int pos = v.lane; pos < P; pos += 64) {
      float rr = r[pos] / rSum;
      if(out[pos] >= 0.0f)
        out[pos] = rr * w + out[pos] * (1.0f - w);
    }
    waveSync();
  }
}

// A freshly evaluated node's first expansion candidate.
template <int NI>
KC_D void firstExpansion(const GV& v, int ni, const float (&pv)[NI]) {
  float pr;
  int pos;
  nextExpansion<NI>(v, pv, __builtin_inff(), -1, pr, pos);
  if(v.lane == 0) {
    v.nodes()[ni].nextPos = (uint16_t)pos;
    v.nodes()[ni].nextPrior = pr;
  }
  waveSync();
}

// kBackup: NN post-processing + leaf value + path backup.
KC_D bool setMoveLimits(const GV& v, GameDev& s, DRng& rng, float lastWL);
KC_D void finishGameRecord(const GV& v, const GameDev& s, DRng& rng, float* scratch);
KC_D void startGame(const GV& v, GameDev& s);
template <int NI>
KC_D void forkEval(const GV& v, GameDev& s, const float* o, float* scratch);
template <int NI>
KC_D void sideEval(const GV& v, GameDev& s, const float* o, float* scratch);

// oracle initMove (getGameInitializationMove playutils.cpp:97-145 + the move of
// initializeGameUsingPolicy :163-175): a move sampled from the root's post-processed
// policy raised to 1/temperature (2e-4 of the time uniformly among the candidates),
// played without search and recorded as a turn without rows.  Returns true when the
// move ended the game (kCommit then finishes it).
template <int NI>
KC_D bool initMove(const GV& v, GameDev& s, const float* o, float* scratch /* LDS [2*MAX_P] */) {
  const SP& b = v.d.sp;
  const int P = v.d.P, A = v.T.A;
  float* pol = scratch;
  float w, l;
  float pv[NI];
  postprocess<NI>(v, s.root, s.leafSym, o, pol, w, l, scratch, pv);
  waveSync();
  // candidates in ascending policy position: legal with probability > 0
  int* cpos = reinterpret_cast<int*>(scratch + MAX_P);
  float* cval = scratch;  // overwrites pol in place: candidate i <= its position
  int n = 0;
  const float invT = 1.0f / b.initTemp;
  for(int base = 0; base < P; base += 64) {
    const int p = base + v.lane;
    const float q = p < P ? pol[p] : -1.0f;
    const bool ok = q > 0.0f;
    const uint64_t m = ballot(ok);
    waveSync();
    if(ok) {
      const int i = n + __popcll(m & ((1ULL << v.lane) - 1ULL));
      cpos[i] = p;
      cval[i] = b.initTemp == 1.0f ? q : dpow(q, invT);
    }
    n += __popcll(m);
    waveSync();
  }
  DRng rng{s.rngSeed, s.rngCtr};
  int idx = 0;
  if(rng.uni() < 0.0002f) {
    idx = (int)rng.below((uint32_t)n);
  } else {
    const float sum = seqSum(cval, n, v.lane);
    const float dd = rng.uni() * sum;
    idx = n - 1;
    if(v.lane == 0) {
      float acc = 0.0f;
      for(int i = 0; i < n; i++) {
        acc = acc + cval[i];
        if(acc > dd) {
          idx = i;
          break;
        }
      }
    }
    idx = bcastI(idx, 0);
  }
  s.rngCtr = rng.ctr;
  const int chosen = cpos[idx];
  waveSync();
  if(v.lane == 0) {
    TurnRec rec;
    memset(&rec, 0, sizeof(rec));
    rec.gen = (uint8_t)*v.d.modelGen;
    rec.cell = (int8_t)(chosen % A);
    rec.dir = (int8_t)(chosen / A);
    v.turns()[s.numTurns] = rec;
  }
  s.numTurns++;
  s.startTurn++;
  s.initLeft--;
  playMoveWave(v.T, s.root, chosen % A, chosen / A);
  waveSync();
  if(s.root.finished)
    return true;
  if(s.initLeft == 0) {
    DRng r2{s.rngSeed, s.rngCtr};
    setMoveLimits(v, s, r2, 0.0f);
    s.rngCtr = r2.ctr;
    s.phase = PH_ROOTEVAL;
    s.rootK = 0;
  }
  return false;
}

// One game's backup; returns whether s holds the game's state afterwards (fused: not yet
// stored -- selectBody stores it on every path).
// fused (kBackupSelect): a cache-slot winner leaves the slot's tag set -- the selections
// running beside it treat the slot as being written -- and kResolve clears it.
template <int NI>
KC_D bool backupBody(const SearchDev& d, const DTables& T, int g, GameDev& s, bool fused, float* scratch) {
  if(d.nnDefer[g])  // a deferred leaf is backed up in a later round
    return false;
  GV v(d, T, g);
  SPROF_INIT();
  const unsigned long long t0 = SPROF_NOW();
  (void)t0;
  loadGame(v, s);
  if(s.leafKind == LEAF_NONE)
    return true;
  unsigned long long tPost = 0, tLeaf = 0, tPath = 0;
  (void)tPost;
  (void)tLeaf;
  (void)tPath;
  const SP& sp = *v.sp;
  const int P = d.P;
  const float* o = d.nnOut + (size_t)s.nnSlot * (P + 4);
  bool needCommit = false;
  if(s.leafKind == LEAF_INIT) {
    needCommit = initMove<NI>(v, s, o, scratch);
  } else if(s.leafKind == LEAF_FORK) {
    forkEval<NI>(v, s, o, scratch);
  } else if(s.leafKind == LEAF_SIDE) {
    sideEval<NI>(v, s, o, scratch);
  } else if(s.leafKind == LEAF_ROOTEVAL) {
    float* pol = scratch;
    float w, l;
    float pv[NI];
    postprocess<NI>(v, s.root, s.leafSym, o, pol, w, l, scratch, pv);
    waveSync();
    float* acc = v.accPolicy();
    if(s.rootK == 0) {
      for(int p = v.lane; p < P; p += 64) {
        v.rawPolicy()[p] = pol[p];
        acc[p] = 0.0f + pol[p];
      }
      s.rawWin = w;
      s.rawLoss = l;
      s.accWin = 0.0f + w;
      s.accLoss = 0.0f + l;
    } else {
      for(int p = v.lane; p < P; p += 64)
        acc[p] = acc[p] + pol[p];
      s.accWin = s.accWin + w;
      s.accLoss = s.accLoss + l;
    }
    s.rootK++;
    if(s.rootK == sp.rootSyms) {
      const float fl = (float)sp.rootSyms;
      const bool fresh = s.rootIdx < 0;
      if(fresh) {
        uint64_t k0, k1;
        stateHash(v.T, s.root, k0, k1);
        s.rootIdx = allocNode(v, s, s.root.pla, k0, k1, false);
      }
      waveSync();
      float* rp = v.pol(s.rootIdx);
      for(int p = v.lane; p < P; p += 64)
        rp[p] = acc[p] / fl;
      if(v.lane == 0) {
        Node* r = &v.nodes()[s.rootIdx];
        r->nnWin = s.accWin / fl;
        r->nnLoss = s.accLoss / fl;
        r->flags |= 1;
      }
      waveSync();
      if(fresh) {
        const Node& r = v.nodes()[s.rootIdx];
        addLeafValue(v, s, s.rootIdx, r.nnWin - r.nnLoss, false, true);
      }
      DRng rng{s.rngSeed, s.rngCtr};
      noiseAndTemp(v, s, rng, rp, v.rootNoised(), scratch);
      s.rngCtr = rng.ctr;
      s.phase = PH_SEARCH;
      needCommit = v.nodes()[s.rootIdx].visits >= (uint32_t)s.visitLimit;
    }
  } else {
    NStats leafSt{0u, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    bool haveLeaf = false;
    if(s.leafKind == LEAF_NN || s.leafKind == LEAF_CACHED) {
      float w, l;
      float* pol = v.pol(s.leafNode);
      const unsigned long long ta = SPROF_NOW();
      (void)ta;
      float pv[NI];
#ifdef KC_SEARCH_PROFILE
      if(v.lane == 0)
        probeLeafKey(v.nodeKey(s.leafNode)[0], v.nodeKey(s.leafNode)[1]);
#endif
      if(s.leafKind == LEAF_CACHED) {
        // copied from the cache into the leaf's policy by kSelect
#pragma unroll
        for(int j = 0; j < NI; j++) {
          const int pos = v.lane + 64 * j;
          pv[j] = pos < P ? pol[pos] : -1.0f;
        }
        w = s.cHitWin;
        l = s.cHitLoss;
      } else {
        postprocess<NI>(v, s.leaf, s.leafSym, o, pol, w, l, scratch, pv);
        if(d.cacheOn) {
          // kCompact bid this evaluation for the state's cache slot (atomicMax of
          // game + 1 over the round's batch); the highest bidder stores its payload
          // and clears the tag, deterministic whatever the block order.  Nothing
          // reads the table in this kernel (hits were copied by kSelect).
          const uint32_t slot = (uint32_t)s.cSlot;
          if(d.cTag[slot] == (uint32_t)g + 1u) {
            float* cp = d.cPol + (size_t)slot * P;
#pragma unroll
            for(int j = 0; j < NI; j++)
              if(v.lane + 64 * j < P)
                cp[v.lane + 64 * j] = pv[j];
            if(v.lane == 0) {
              d.cVal[2 * (size_t)slot] = w;
              d.cVal[2 * (size_t)slot + 1] = l;
              d.cKey[2 * (size_t)slot] = v.nodeKey(s.leafNode)[0];
              d.cKey[2 * (size_t)slot + 1] = v.nodeKey(s.leafNode)[1];
              if(fused)
                d.cClear[g] = slot + 1u;
              else
                d.cTag[slot] = 0;
            }
          }
        }
      }
      firstExpansion<NI>(v, s.leafNode, pv);
      if(v.lane == 0) {
        Node* n = &v.nodes()[s.leafNode];
        n->nnWin = w;
        n->nnLoss = l;
        n->flags |= 1;
      }
      waveSync();
      const unsigned long long tb = SPROF_NOW();
      (void)tb;
      leafSt = addLeafValue(v, s, s.leafNode, w - l, false, true);
      haveLeaf = true;
      tPost = tb - ta;
      tLeaf = SPROF_NOW() - tb;
    } else if(s.leafKind == LEAF_TERMINAL) {
      float val = s.leaf.winner == 2 ? 1.0f : (s.leaf.winner == 1 ? -1.0f : 0.0f);
      leafSt = addLeafValue(v, s, s.leafNode, val, true, false);
      haveLeaf = true;
    } else if(s.leafKind == LEAF_NOCHILD) {
      const Node& n = v.nodes()[s.leafNode];
      leafSt = addLeafValue(v, s, s.leafNode, n.nnWin - n.nnLoss, false, false);
      haveLeaf = true;
    }
    const unsigned long long tp0 = SPROF_NOW();
    (void)tp0;
    // an updated leaf is the deepest level's path child (a catch-up leaf is unchanged)
    backupPath<NI>(v, s, s.pathLen, leafSt, haveLeaf);
    tPath = SPROF_NOW() - tp0;
    s.playouts++;
    needCommit = v.nodes()[s.rootIdx].visits >= (uint32_t)s.visitLimit;
  }
  if(needCommit) {
    s.phase = PH_COMMIT;
    if(v.lane == 0)
      d.commitList[atomicAdd(d.commitCount, 1)] = g;
  }
  s.leafKind = LEAF_NONE;
  waveSync();
  if(!fused)  // fused: the selection that follows stores the state once (408 B per game less)
    storeGame(v, s);
  SPROF_ADD(10, 1);
  SPROF_MAX(26, SPROF_NOW() - t0);
  SPROF_ADD(11, SPROF_NOW() - t0);
  SPROF_ADD(12, tPost);
  SPROF_ADD(13, tPath);
  SPROF_ADD(14, tLeaf);
  SPROF_FLUSH();
  return true;
}

template <int NI>
__global__ void __launch_bounds__(64, NI <= 4 ? 4 : 3) kBackup(const SearchDev* __restrict__ dp, const DTables* __restrict__ Tp) {
  const SearchDev& d = *dp;
  const int g = blockIdx.x;
  if(g >= d.G)
    return;
  __shared__ __attribute__((aligned(16))) float scratch[3 * MAX_P];
  __shared__ GameDev s;
  backupBody<NI>(d, *Tp, g, s, false, scratch);
}

// Round r's backup and round r+1's selection of one game in one kernel (no commit between
// them).  Games only read and write their own trees and tables; the one table they share,
// the NN cache, is handled by the tags (backupBody / cacheLookup / kResolve), so every
// result is the one the two separate kernels give.  One kernel boundary less per round,
// and a game's slow backup and slow descent no longer each set a kernel's length.
// waves per SIMD the fused kernel is compiled for at 5x5 (A/B switch: 4 = 128 VGPRs, as
// kSelect / kBackup; beside a network workgroup's two waves a SIMD holds one such wave.
// 6 (80 VGPRs: two fit) spills 332 B per lane and ran 18.0 k against 24.4 k rows/s, 5
// 21.6 k: profiles/r05/fused_occupancy_ab.txt)
#ifndef KC_FUSED_OCC
#define KC_FUSED_OCC 4
#endif
// A/B switch: KC_SEARCH_PRIO > 0 raises the fused search waves' issue priority (s_setprio)
// over the other group's network waves sharing their SIMD
#ifndef KC_SEARCH_PRIO
#define KC_SEARCH_PRIO 0
#endif
template <int NI>
__global__ void __launch_bounds__(64, NI <= 2 ? KC_FUSED_OCC : 2) kBackupSelect(const SearchDev* __restrict__ dp,
                                                                      const DTables* __restrict__ Tp) {
  const SearchDev& d = *dp;
  const int g = blockIdx.x;
  if(g >= d.G)
    return;
  if constexpr(KC_SEARCH_PRIO > 0)
    __builtin_amdgcn_s_setprio(KC_SEARCH_PRIO);
  __shared__ __attribute__((aligned(16))) float scratch[3 * MAX_P];
  __shared__ uint32_t hasBits[(MAX_P + 31) / 32];
  __shared__ GameDev s;
  const bool loaded = backupBody<NI>(d, *Tp, g, s, true, scratch);
  // (the selection's root policy reuses the backup's scratch)
  selectBody<NI>(d, *Tp, g, s, loaded, true, hasBits, scratch);
}

#ifdef KC_SEARCH_PROFILE
}  // namespace kc
#include <algorithm>
#include <vector>
namespace kc {
extern "C" void coffee_debug_probe_table(void* keys, unsigned long long cap /* power of two */) {
  unsigned long long* k = (unsigned long long*)keys;
  unsigned long long m = cap ? cap - 1 : 0;
  KC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_probeKeys), &k, sizeof(k)));
  KC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_probeMask), &m, sizeof(m)));
}

extern "C" void coffee_debug_search_profile(unsigned long long* out, int reset) {
  std::vector<unsigned long long> all((size_t)SPROF_MAXG * SPROF_N);
  KC_HIP(hipDeviceSynchronize());
  KC_HIP(hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(g_searchProf), all.size() * 8));
  for(int i = 0; i < SPROF_N; i++)
    out[i] = 0;
  for(size_t k = 0; k < all.size(); k++) {
    const int i = (int)(k % SPROF_N);
    if(i < 24)
      out[i] += all[k];
    else if(i <= 26)
      out[i] = std::max(out[i], all[k]);
    if(i == 24)
      out[27] += all[k];  // sum of per-block maxima (their mean: the typical slowest descent)
    if(i == 26)
      out[28] += all[k];
  }
  if(reset) {
    std::fill(all.begin(), all.end(), 0ull);
    KC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_searchProf), all.data(), all.size() * 8));
  }
}
#endif

// ---------------------------------------------------------------------------
// Commit: move choice, targets, tree reuse, rows.

// oracle lcbAndRadius (getSelfUtilityLCBAndRadius searchhelpers.cpp:469-521)
KC_D void lcbAndRadius(const SP& sp, int pla, uint32_t cVisits, float cWs, float cWsq, float cU, float cUsq,
                       uint32_t ev, float& lcb, float& radius) {
  radius = 2.0f * 1.0f * sp.lcbStdevs;
  lcb = -radius;
  float ws = childWeight(ev, cVisits, cWs);
  float wsq = childWeight(ev, cVisits, cWsq);
  if(cVisits == 0 || ws <= 0.0f || wsq <= 0.0f)
    return;
  float u = cU, usq = cUsq;
  float ess = (ws * ws) / wsq;
  float priorWeight = ws / ((ess * ess) * ess);
  usq = fmaxf(usq, u * u + 1e-8f);
  usq = (usq * ws + (usq + 1.0f) * priorWeight) / (ws + priorWeight);
  ws = ws + priorWeight;
  wsq = wsq + priorWeight * priorWeight;
  ess = (ws * ws) / wsq;
  float selfU = pla == 2 ? u : -u;
  float variance = usq - u * u;
  float stdev = sqrtf(variance / ess);
  radius = stdev * sp.lcbStdevs;
  lcb = selfU - radius;
}

// oracle playSelectionValuesAt (getPlaySelectionValues searchresults.cpp:63-309) on node
// ri with policy pol; the over-explored-children reduction and direct policy moves are
// root-only.  posOut/vals are LDS arrays [P]; returns the count (uniform).
template <int NI>
KC_D int playSelectionValuesAt(const GV& v, const SP& sp, const GameDev& s, int ri, const float* pol, bool isRoot,
                               float scaleMaxToAtLeast, bool allowDirect, int* posOut, float* vals, bool useLcb) {
  const Node& n = v.nodes()[ri];
  const int k = n.numChildren;
  const int pla = n.nextPla;
  const NodeEdges E = v.edges(ri, n.edgeBase);
  float cw[NI], val[NI];
  uint32_t ev[NI];
  int posv[NI];
  uint32_t cvis[NI];
  float cws[NI], cwsq[NI], cu[NI], cusq[NI];
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int i = v.lane + 64 * j;
    cw[j] = val[j] = 0.0f;
    ev[j] = 0;
    posv[j] = 0;
    cvis[j] = 0;
    cws[j] = cwsq[j] = cu[j] = cusq[j] = 0.0f;
    if(i < k) {
      Edge e = E[i];
      const Node& c = v.nodes()[e.child];
      cvis[j] = c.visits;
      cws[j] = c.weightSum;
      cwsq[j] = c.weightSqSum;
      cu[j] = c.utilityAvg;
      cusq[j] = c.utilitySqAvg;
      ev[j] = e.visits;
      cw[j] = childWeight(e.visits, cvis[j], cws[j]);
      posv[j] = (int)e.move;
      val[j] = cw[j];
    }
  }
  const float total = tsum<NI>(cw, k, v.lane);
  int numChildren = k;
  // best child by "good" weight (first max)
  float maxGood = -1e30f;
  int bestIdx = BIG;
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int i = v.lane + 64 * j;
    if(i >= k)
      continue;
    float evf = (float)ev[j];
    float gdn = val[j] * fmaxf(0.0f, evf - 1.0f) / fmaxf(1.0f, evf) + 2.0f * pol[posv[j]];
    if(gdn > maxGood) {
      maxGood = gdn;
      bestIdx = i;
    }
  }
  waveArgmax(maxGood, bestIdx);
  if(bestIdx == BIG)
    bestIdx = 0;
  const int bestLane = bestIdx & 63, bestJ = bestIdx >> 6;
  float bestWeight = -1e30f;
  if(k > 0) {
    float bw = 0.0f;
#pragma unroll
    for(int j = 0; j < NI; j++)
      if(j == bestJ)
        bw = cw[j];
    bestWeight = bcastLaneF(bw, bestLane);
  }
  if(isRoot && k > 0) {
    const float fpu = fpuValue(sp, n, pla, true, 1.0f);
    const float scaling = exploreScaling(sp, total);
    float bp = 0.0f, bu = 0.0f;
    uint32_t bvis = 0;
#pragma unroll
    for(int j = 0; j < NI; j++)
      if(j == bestJ) {
        bp = pol[posv[j]];
        bu = cu[j];
        bvis = cvis[j];
      }
    bp = bcastLaneF(bp, bestLane);
    bu = bcastLaneF(bu, bestLane);
    bvis = (uint32_t)bcastLane((int)bvis, bestLane);
    const float bw = bestWeight;
    const float buu = (bvis == 0 || bw <= 0.0f) ? fpu : bu;
    const float bestValue = bp < 0.0f ? -__builtin_inff() : (scaling * bp) / (1.0f + bw) + (pla == 2 ? buu : -buu);
#pragma unroll
    for(int j = 0; j < NI; j++) {
      int i = v.lane + 64 * j;
      if(i >= k || i == bestIdx)
        continue;
      float w = cw[j];
      float reduced;
      if(cvis[j] == 0 || w <= 0.0f)
        reduced = 0.0f;
      else {
        float p = pol[posv[j]];
        float wanted;
        if(p < 0.0f)
          wanted = 0.0f;
        else {
          float valueComponent = pla == 2 ? cu[j] : -cu[j];
          float exploreComponent = bestValue - valueComponent;
          float exploreComponentScaling = scaling * p;
          if(exploreComponent <= 0.0f)
            wanted = __builtin_inff();
          else {
            wanted = exploreComponentScaling / exploreComponent - 1.0f;
            if(wanted < 0.0f)
              wanted = 0.0f;
          }
        }
        reduced = w > wanted ? wanted : w;
      }
      val[j] = ceilf(reduced);
    }
  }
  if(useLcb && k > 0) {
    float lcb[NI], rad[NI];
    float bestLcb = -1e10f;
    int bestLcbIdx = BIG;
#pragma unroll
    for(int j = 0; j < NI; j++) {
      int i = v.lane + 64 * j;
      lcb[j] = rad[j] = 0.0f;
      if(i >= k)
        continue;
      lcbAndRadius(sp, pla, cvis[j], cws[j], cwsq[j], cu[j], cusq[j], ev[j], lcb[j], rad[j]);
      float w = val[j];
      if(w > 0.0f && w >= sp.minVisitPropLcb * bestWeight && lcb[j] > bestLcb) {
        bestLcb = lcb[j];
        bestLcbIdx = i;
      }
    }
    waveArgmax(bestLcb, bestLcbIdx);
    if(bestLcbIdx != BIG) {
      float adj = 0.0f;
#pragma unroll
      for(int j = 0; j < NI; j++)
        if(j == (bestLcbIdx >> 6))
          adj = val[j];
      adj = bcastLaneF(adj, bestLcbIdx & 63);
      float lb = adj;
#pragma unroll
      for(int j = 0; j < NI; j++) {
        int i = v.lane + 64 * j;
        if(i >= k || i == bestLcbIdx)
          continue;
        float excess = bestLcb - lcb[j];
        if(excess < 0.0f)
          continue;
        float rf = (rad[j] + excess) / (rad[j] + 0.20f * excess);
        float lbound = (rf * rf) * val[j];
        if(lbound > lb)
          lb = lbound;
      }
      lb = waveMax(lb);
#pragma unroll
      for(int j = 0; j < NI; j++)
        if(v.lane + 64 * j == bestLcbIdx)
          val[j] = lb;
    }
  }
  // to LDS
#pragma unroll
  for(int j = 0; j < NI; j++) {
    int i = v.lane + 64 * j;
    if(i < k) {
      posOut[i] = posv[j];
      vals[i] = val[j];
    }
  }
  waveSync();
  if(numChildren == 0) {
    if(!allowDirect || !isRoot)
      return 0;
    const int P = v.d.P;
    for(int base = 0; base < P; base += 64) {
      int p = base + v.lane;
      bool ok = p < P && isLegal(v.T, s.root, p % v.T.A, p / v.T.A) && pol[p] >= 0.0f;
      uint64_t m = ballot(ok);
      if(ok) {
        int idx = numChildren + __popcll(m & ((1ULL << v.lane) - 1ULL));
        posOut[idx] = p;
        vals[idx] = pol[p];
      }
      numChildren += __popcll(m);
    }
    waveSync();
    if(numChildren == 0)
      return 0;
  }
  float mx = 0.0f;
  for(int i = v.lane; i < numChildren; i += 64)
    mx = vals[i] > mx ? vals[i] : mx;
  mx = waveMax(mx);
  if(mx <= 0.0f)
    return 0;
  const float amountToSubtract = fminf(sp.moveSubtract, mx / 64.0f);
  const float amountToPrune = fminf(sp.movePrune, mx / 64.0f);
  const float newMax = mx - amountToSubtract;
  for(int i = v.lane; i < numChildren; i += 64) {
    float x = vals[i];
    if(x < amountToPrune)
      x = 0.0f;
    else {
      x = x - amountToSubtract;
      if(x <= 0.0f)
        x = 0.0f;
    }
    if(newMax < scaleMaxToAtLeast)
      x = x * (scaleMaxToAtLeast / newMax);
    vals[i] = x;
  }
  waveSync();
  return numChildren;
}

// oracle playSelectionValues: the root with its noised policy.
template <int NI>
KC_D int playSelectionValues(const GV& v, const SP& sp, const GameDev& s, float scaleMaxToAtLeast, bool allowDirect,
                             int* posOut, float* vals, bool useLcb) {
  return playSelectionValuesAt<NI>(v, sp, s, s.rootIdx, v.rootNoised(), true, scaleMaxToAtLeast, allowDirect, posOut,
                                   vals, useLcb);
}

// oracle chooseIndex (chooseIndexWithTemperature searchhelpers.cpp:11-49)
KC_D int chooseIndex(const GV& v, DRng& rng, const float* vals, int n, float temperature, float* pr) {
  float mx = 0.0f;
  for(int i = v.lane; i < n; i += 64)
    mx = vals[i] > mx ? vals[i] : mx;
  mx = waveMax(mx);
  if(temperature <= 1.0e-4f) {
    float best = -__builtin_inff();
    int bi = BIG;
    for(int i = v.lane; i < n; i += 64)
      if(vals[i] > best) {
        best = vals[i];
        bi = i;
      }
    waveArgmax(best, bi);
    // oracle: best starts at vals[0]; strictly greater later values win
    return bi == BIG ? 0 : bi;
  }
  const float logMax = dlog(mx);
  for(int i = v.lane; i < n; i += 64)
    pr[i] = vals[i] <= 0.0f ? 0.0f : dexp((dlog(vals[i]) - logMax) / temperature);
  const float sum = seqSum(pr, n, v.lane);
  const float dd = rng.uni() * sum;
  int chosen = n - 1;
  if(v.lane == 0) {
    float acc = 0.0f;
    for(int i = 0; i < n; i++) {
      acc = acc + pr[i];
      if(acc > dd) {
        chosen = i;
        break;
      }
    }
  }
  return bcastI(chosen, 0);
}

// 16-byte stores where the arrays allow (every per-game slice starts 16-B aligned when
// its length is a multiple of 4 words), one word at a time otherwise.
KC_D void fillWords(uint32_t* p, int n, uint32_t val, int lane) {
  if((n & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    uint4* q = reinterpret_cast<uint4*>(p);
    for(int i = lane; i < n / 4; i += 64)
      q[i] = uint4{val, val, val, val};
  } else {
    for(int i = lane; i < n; i += 64)
      p[i] = val;
  }
}

KC_D void clearTables(const GV& v, GameDev& s) {
  const int cap = v.d.cap;
  uint32_t* fl = v.freeList();
  if((cap & 3) == 0 && (reinterpret_cast<uintptr_t>(fl) & 15) == 0) {
    uint4* q = reinterpret_cast<uint4*>(fl);
    for(int i = v.lane; i < cap / 4; i += 64) {
      const uint32_t b = (uint32_t)(cap - 1 - 4 * i);  // pop order: 0, 1, 2, ...
      q[i] = uint4{b, b - 1, b - 2, b - 3};
    }
  } else {
    for(int i = v.lane; i < cap; i += 64)
      fl[i] = (uint32_t)(cap - 1 - i);
  }
  fillWords(v.allocBits(), cap / 32, 0u, v.lane);
  fillWords(reinterpret_cast<uint32_t*>(v.ttNode()), v.d.ttCap, 0xFFFFFFFFu, v.lane);
  const size_t sb = v.svbBase(s.svbSel);
  fillWords(reinterpret_cast<uint32_t*>(&v.d.svbKey[sb]), 2 * v.d.svbCap, 0u, v.lane);
  s.freeTop = cap;
  s.edgeTop = 0;
  s.liveCount = 0;
  s.rootIdx = -1;
  waveSync();
}

// oracle reuseTree (Search::makeMove search.cpp:262-330 + deleteAllOld... :790-810 +
// SubtreeValueBiasTable::clearUnusedSynchronous :47-59) as mark / free / rebuild.
// lds: live bitmap [cap/32] u32 + BFS queue [cap] u16.
KC_D void reuseTree(const GV& v, GameDev& s, int chosenPos, uint32_t* liveBits, uint16_t* queue, int* qtail) {
  const SP& sp = *v.sp;
  const int cap = v.d.cap;
  const int ri = s.rootIdx;
  int child = -1;
  if(ri >= 0) {
    const Node& r = v.nodes()[ri];
    const NodeEdges E = v.edges(ri, r.edgeBase);
    for(int base = 0; base < r.numChildren; base += 64) {
      int i = base + v.lane;
      bool hit = i < r.numChildren && (int)E[i].move == chosenPos;
      uint64_t m = ballot(hit);
      if(m) {
        int f = firstLane(m);
        child = bcastI(hit ? (int)E[i].child : -1, f);
        break;
      }
    }
  }
  if(child < 0 || !(v.nodes()[child].flags & 1)) {
    clearTables(v, s);
    return;
  }
  // mark: parallel BFS over child slots
  for(int i = v.lane; i < cap / 32; i += 64)
    liveBits[i] = 0;
  waveSync();
  if(v.lane == 0) {
    liveBits[child >> 5] |= 1u << (child & 31);
    queue[0] = (uint16_t)child;
    *qtail = 1;
  }
  waveSync();
  int head = 0;
  while(true) {
    const int tail = *qtail;
    if(head >= tail)
      break;
    const int cnt = min(64, tail - head);
    if(v.lane < cnt) {
      const int nd = queue[head + v.lane];
      const Node& nr = v.nodes()[nd];
      const int kc = nr.numChildren;
      const Edge* inl = v.inlineEdges(nd);
      const Edge* pool = v.edgePool() + nr.edgeBase - INLINE_EDGES;  // indexed by child slot
      // four child loads in flight before the LDS atomics that consume them
      for(int i = 0; i < kc; i += 4) {
        int ch[4];
#pragma unroll
        for(int u = 0; u < 4; u++)
          ch[u] = i + u < kc ? (int)(i + u < INLINE_EDGES ? inl : pool)[i + u].child : -1;
#pragma unroll
        for(int u = 0; u < 4; u++) {
          const int c = ch[u];
          if(c < 0)
            continue;
          const uint32_t bit = 1u << (c & 31);
          uint32_t old = atomicOr(&liveBits[c >> 5], bit);
          if(!(old & bit))
            queue[atomicAdd(qtail, 1)] = (uint16_t)c;
        }
      }
    }
    head += cnt;
    waveSync();
  }
  int liveCount = 0;
  for(int i = v.lane; i < cap / 32; i += 64)
    liveCount += __popc(liveBits[i]);
#pragma unroll
  for(int off = 32; off >= 1; off >>= 1)
    liveCount += __shfl_xor(liveCount, off, 64);
  if(liveCount + sp.maxVisits + 2 > cap) {
    clearTables(v, s);
    return;
  }
  // removeSubtreeValueBias for dead table nodes and the promoted child (fixed point: any order).
  // The dead allocated nodes are compacted into the queue behind the live ones
  // (queue[0..liveCount) = live nodes in BFS order; dead <= cap - liveCount), so the
  // node reads below are independent and batched; lane 0 adds the child.
  const size_t sb = v.svbBase(s.svbSel);
  uint32_t* ab = v.allocBits();
  const int nw = cap / 32;
  uint16_t* dead = queue + liveCount;
  int nDead = 0;
  for(int wb = 0; wb < nw; wb += 64) {
    const int w = wb + v.lane;
    uint32_t m = 0;
    if(w < nw)
      m = ab[w] & ~liveBits[w];
    int cnt = __popc(m), incl = cnt;
#pragma unroll
    for(int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off, 64);
      if(v.lane >= off)
        incl += y;
    }
    int o = nDead + incl - cnt;
    while(m) {
      const int b = __builtin_ctz(m);
      m &= m - 1;
      dead[o++] = (uint16_t)(w * 32 + b);
    }
    nDead += __shfl(incl, 63, 64);
  }
  waveSync();
  for(int base = 0; base < nDead + 1; base += 256) {
    int32_t e[4];
    float dl[4], wl[4];
#pragma unroll
    for(int u = 0; u < 4; u++) {
      const int i = base + 64 * u + v.lane;  // i == nDead: the promoted child
      e[u] = -1;
      dl[u] = wl[u] = 0.0f;
      if(i <= nDead) {
        const Node& n = v.nodes()[i < nDead ? (int)dead[i] : child];
        e[u] = n.svbEntry;
        dl[u] = n.lastSvbDelta;
        wl[u] = n.lastSvbWeight;
      }
    }
#pragma unroll
    for(int u = 0; u < 4; u++) {
      if(e[u] < 0)
        continue;
      atomicAdd((unsigned long long*)&v.d.svbD[sb + e[u]], (unsigned long long)(-svbQ(dl[u] * sp.svbFreeProp)));
      atomicAdd((unsigned long long*)&v.d.svbW[sb + e[u]], (unsigned long long)(-svbQ(wl[u] * sp.svbFreeProp)));
    }
  }
  waveSync();
  if(v.lane == 0) {
    Node* c = &v.nodes()[child];
    c->svbEntry = -1;
    c->lastSvbDelta = 0.0f;
    c->lastSvbWeight = 0.0f;
  }
  // free list = every non-live index; allocBits = live
  int top = 0;
  uint32_t* fl = v.freeList();
  for(int base = 0; base < cap; base += 64) {
    int i = base + v.lane;
    bool live = (liveBits[i >> 5] >> (i & 31)) & 1u;
    uint64_t m = ballot(!live);
    if(!live)
      fl[top + __popcll(m & ((1ULL << v.lane) - 1ULL))] = (uint32_t)i;
    top += __popcll(m);
  }
  for(int i = v.lane; i < cap / 32; i += 64)
    ab[i] = liveBits[i];
  s.freeTop = top;
  s.liveCount = liveCount;
  s.rootIdx = child;
  // transposition table: clear, insert every live node but the root (CAS, any order)
  int32_t* tn = v.ttNode();
  uint64_t* tk = v.ttKey();
  for(int i = v.lane; i < v.d.ttCap; i += 64)
    tn[i] = -1;
  // new SVB table
  const int nsel = s.svbSel ^ 1;
  const size_t nb = v.svbBase(nsel);
  for(int i = v.lane; i < v.d.svbCap; i += 64)
    v.d.svbKey[nb + i] = 0;
  waveSync();
  const int tmask = v.d.ttCap - 1, smask = v.d.svbCap - 1;
  // live nodes, in the order of the BFS queue (queue[0..liveCount) holds them all)
  for(int i = v.lane; i < liveCount; i += 64) {
    const int ni = queue[i];
    Node* n = &v.nodes()[ni];
    const int32_t se = n->svbEntry;
    if(ni != child && v.d.sp.useGraph) {
      const uint64_t k0 = v.nodeKey(ni)[0], k1 = v.nodeKey(ni)[1];
      int sl = (int)(k0 & (uint64_t)tmask);
      while(atomicCAS(&tn[sl], -1, ni) != -1)
        sl = (sl + 1) & tmask;
      tk[2 * sl] = k0;
      tk[2 * sl + 1] = k1;
    }
    if(se >= 0) {
      const size_t oe = sb + se;
      const uint64_t key = v.d.svbKey[oe];
      int sl = (int)(key & (uint64_t)smask);
      while(true) {
        unsigned long long prev =
          atomicCAS((unsigned long long*)&v.d.svbKey[nb + sl], 0ULL, (unsigned long long)key);
        if(prev == 0ULL || prev == key)
          break;
        sl = (sl + 1) & smask;
      }
      v.d.svbD[nb + sl] = v.d.svbD[oe];
      v.d.svbW[nb + sl] = v.d.svbW[oe];
      n->svbEntry = sl;
    }
  }
  s.svbSel = nsel;
  // edge pool: the live nodes' blocks into the other buffer (queue order, prefix sums
  // of the block sizes), so the dead nodes' blocks are reclaimed
  {
    const int P = v.d.P;
    Edge* src = v.edgePool();
    Edge* dst = v.d.edgePool + ((size_t)v.g * 2 + (s.edgeSel ^ 1)) * v.d.edgePoolCap;
    int top = 0;
    for(int base = 0; base < liveCount; base += 64) {
      const int i = base + v.lane;
      const int nd = i < liveCount ? (int)queue[i] : -1;
      const Node* np = nd >= 0 ? &v.nodes()[nd] : nullptr;
      const int k = np ? (int)np->numChildren : 0;
      const int need = k > INLINE_EDGES ? edgeBlockCap(k, P) : 0;
      int incl = need;
#pragma unroll
      for(int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if(v.lane >= off)
          incl += y;
      }
      const int mine = top + incl - need;
      if(need) {
        const uint32_t ob = np->edgeBase;
        for(int e = 0; e < k - INLINE_EDGES; e++)
          dst[mine + e] = src[ob + e];
        v.nodes()[nd].edgeBase = (uint32_t)mine;
      }
      top += __shfl(incl, 63, 64);
    }
    const int nsel2 = s.edgeSel ^ 1;
    waveSync();
    s.edgeSel = nsel2;
    s.edgeTop = top;
    s.edgePeak = max(s.edgePeak, top);
    v.setEdgeSel(nsel2);
  }
  waveSync();
}

// oracle setMoveLimits (getSearchLimitsThisMove play.cpp:871-1004) for the move about
// to be searched; every lane runs it on the same state.  lastWL: the root value of the
// move just committed (the newest reduceVisits history entry).  Returns
// clearBotBeforeSearchThisMove (self-play clears before every search, play.cpp:1941-1946,
// except a cheap search whose rows are not recorded, :920-925).
KC_D bool setMoveLimits(const GV& v, GameDev& s, DRng& rng, float lastWL) {
  const SP& b = v.d.sp;
  s.visitLimit = b.maxVisits;
  s.moveWeight = 1.0f;
  s.noNoise = 0;
  bool clear = true;
  if(b.cheapProb > 0.0f && rng.uni() < b.cheapProb) {
    s.visitLimit = min(b.maxVisits, b.cheapVisits);
    s.moveWeight = 1.0f * b.cheapWeight;
    if(b.cheapWeight <= 0.0f) {
      clear = false;
      s.noNoise = 1;
    }
  } else if(b.reduceVisits && s.numTurns - s.startTurn >= b.reduceLookback) {
    const TurnRec* tr = v.turns();
    float mn = 1e20f, mx = -1e20f;
    for(int j = 0; j < b.reduceLookback; j++) {
      const float w = j == 0 ? lastWL : tr[s.numTurns - 1 - j].rootWL;
      mn = w < mn ? w : mn;
      mx = w > mx ? w : mx;
    }
    float extreme = fmaxf(mn, -mx);
    if(extreme > 1.0f)
      extreme = 1.0f;
    const float through = extreme - b.reduceThreshold;
    if(through > 0.0f) {
      const float prop = through / (1.0f - b.reduceThreshold);
      const float red = prop * prop;
      const int vl = (int)roundf((float)b.maxVisits + red * ((float)b.reducedMin - (float)b.maxVisits));
      s.moveWeight = 1.0f + red * (b.reducedWeight - 1.0f);
      s.visitLimit = max(vl, b.reducedMin);
    }
  }
  return clear;
}

KC_D void startGame(const GV& v, GameDev& s) {
  s.rngSeed = mix64(v.d.seed ^ mix64(((uint64_t)(v.d.slotBase + v.g) << 32) | (uint32_t)s.gameNum));
  s.rngCtr = 0;
  s.startGen = *v.d.modelGen;
  boardInit(v.T, s.root);
  clearTables(v, s);
  s.numTurns = 0;
  s.gameMode = 0;
  s.sideCount = 0;
  s.sideNext = 0;
  s.sideMode = 0;
  DRng rng{s.rngSeed, s.rngCtr};
  s.gameHash0 = rng.next();
  s.gameHash1 = rng.next();
  // initializeGameUsingPolicy (playutils.cpp:147-176): floor(Exp(1) * area * prop)
  // opening moves sampled from the raw policy (nextExponential rand.h:299-305)
  s.startTurn = 0;
  s.initLeft = 0;
  const SP& b = v.d.sp;
  if(b.initPolicy && b.initAreaProp > 0.0f) {
    float u = rng.uni();
    while(u <= 0.0f)
      u = rng.uni();
    s.initLeft = (int)floorf(-dlog(u) * ((float)v.T.A * b.initAreaProp));
  }
  if(s.initLeft > 0) {
    s.phase = PH_INIT;
  } else {
    setMoveLimits(v, s, rng, 0.0f);
    s.phase = PH_ROOTEVAL;
  }
  s.rngCtr = rng.ctr;
  s.rootK = 0;
  s.leafKind = LEAF_NONE;
}

// oracle startForkGame: the slot's next game starts from the fork position `b`
// (the finished game replayed to `prefix` moves plus the chosen move); those moves
// stay in the turn records as unsearched turns, no policy initialisation (play.cpp:
// 380-395), mode FORK in the rows (trainingwrite.cpp:468).
KC_D void startForkGame(const GV& v, GameDev& s, const DBoard& b, int prefix, int move) {
  s.rngSeed = mix64(v.d.seed ^ mix64(((uint64_t)(v.d.slotBase + v.g) << 32) | (uint32_t)s.gameNum));
  s.rngCtr = 0;
  s.startGen = *v.d.modelGen;
  s.root = b;
  clearTables(v, s);
  TurnRec* tr = v.turns();
  for(int t = v.lane; t <= prefix; t += 64) {
    const int8_t cell = t < prefix ? tr[t].cell : (int8_t)(move % v.T.A);
    const int8_t dir = t < prefix ? tr[t].dir : (int8_t)(move / v.T.A);
    TurnRec rec;
    memset(&rec, 0, sizeof(rec));
    rec.gen = (uint8_t)*v.d.modelGen;
    rec.cell = cell;
    rec.dir = dir;
    tr[t] = rec;
  }
  s.numTurns = prefix + 1;
  s.startTurn = prefix + 1;
  s.initLeft = 0;
  s.gameMode = 2;
  s.sideCount = 0;
  s.sideNext = 0;
  s.sideMode = 0;
  DRng rng{s.rngSeed, s.rngCtr};
  s.gameHash0 = rng.next();
  s.gameHash1 = rng.next();
  setMoveLimits(v, s, rng, 0.0f);
  s.rngCtr = rng.ctr;
  s.phase = PH_ROOTEVAL;
  s.rootK = 0;
  s.leafKind = LEAF_NONE;
  waveSync();
}

// oracle maybeFork (Play::maybeForkGame play.cpp:1741-1840) at the end of a game, on
// the finished game's stream: an early fork (position after floor(Exp(1) * A *
// earlyForkGameExpectedMoveProp) moves) or a late one (uniform move index); the
// candidates are numChoices uniform draws, with replacement, from the legal moves in
// cell-major order (chooseRandomLegalMoves playutils.cpp:33-60).  Returns true when a
// fork was set up (PH_FORK: one candidate evaluated per round).  No draws at all when
// both probabilities are 0 (SPEC: benchmark mode's streams stay as they are).
KC_D bool maybeFork(const GV& v, GameDev& s, DRng& rng, uint16_t* legal /* LDS [MAX_P] */) {
  const SP& b = v.d.sp;
  if(b.earlyForkProb <= 0.0f && b.forkProb <= 0.0f)
    return false;
  const DTables& T = v.T;
  const bool early = rng.uni() < b.earlyForkProb;
  const bool late = !early && b.forkProb > 0.0f && rng.uni() < b.forkProb;
  if(!early && !late)
    return false;
  const int n = s.numTurns;
  int moveIdx;
  if(early) {
    float u = rng.uni();
    while(u <= 0.0f)
      u = rng.uni();
    moveIdx = (int)floorf(-dlog(u) * (b.earlyForkMoveProp * (float)T.A));
  } else {
    moveIdx = n <= 0 ? 0 : (int)rng.below((uint32_t)n);
  }
  moveIdx = min(moveIdx, max(n - 1, 0));
  // replayGameUpToMove (play.cpp:1703-1739)
  const TurnRec* tr = v.turns();
  DBoard bd;
  boardInit(T, bd);
  for(int t = 0; t < moveIdx; t++) {
    playMoveWave(T, bd, tr[t].cell, tr[t].dir);
    if(bd.finished)
      return false;
  }
  const int maxC = early ? b.earlyForkMaxChoices : b.forkMaxChoices;
  const int numChoices = b.forkMinChoices + (int)rng.below((uint32_t)(maxC - b.forkMinChoices + 1));
  int numLegal = 0;
  for(int base = 0; base < T.P; base += 64) {
    const int q = base + v.lane;  // cell-major: q = cell * 4 + dir
    const bool ok = q < T.P && isLegal(T, bd, q >> 2, q & 3);
    const uint64_t m = ballot(ok);
    if(ok)
      legal[numLegal + __popcll(m & ((1ULL << v.lane) - 1ULL))] = (uint16_t)((q & 3) * T.A + (q >> 2));
    numLegal += __popcll(m);
  }
  waveSync();
  if(numLegal <= 0)
    return false;
  ForkRec* f = v.d.fork + v.g;
  for(int i = 0; i < numChoices; i++) {
    const int k = (int)rng.below((uint32_t)numLegal);
    if(v.lane == 0)
      f->moves[i] = legal[k];
  }
  if(v.lane == 0) {
    f->board = bd;
    f->numChoices = numChoices;
    f->next = 0;
    f->best = -1;
    f->bestWinrate = 0.0f;
    f->prefix = moveIdx;
  }
  s.phase = PH_FORK;
  s.leafKind = LEAF_NONE;
  waveSync();
  return true;
}

// oracle forkEval: the network's value for the position after candidate f.next; the
// best for the player at the fork (first of equals) wins; after the last candidate the
// slot's next game starts from the fork (or normally when the fork move ends the game).
template <int NI>
KC_D void forkEval(const GV& v, GameDev& s, const float* o, float* scratch) {
  ForkRec* f = v.d.fork + v.g;
  float w, l;
  float pv[NI];
  postprocess<NI>(v, s.leaf, s.leafSym, o, scratch, w, l, scratch, pv);
  const float wr = 0.5f * (w - l + 1.0f);
  const int pla = f->board.pla;
  const int next = f->next;
  int best = f->best;
  float bestWr = f->bestWinrate;
  if(best < 0 || (pla == 2 && wr > bestWr) || (pla == 1 && wr < bestWr)) {
    best = next;
    bestWr = wr;
  }
  waveSync();
  if(v.lane == 0) {
    f->best = best;
    f->bestWinrate = bestWr;
    f->next = next + 1;
  }
  if(next + 1 < f->numChoices)
    return;
  const int move = f->moves[best];
  DBoard bd = f->board;
  playMoveWave(v.T, bd, move % v.T.A, move / v.T.A);
  if(bd.finished)
    startGame(v, s);  // "if the game is over now, don't actually do anything"
  else
    startForkGame(v, s, bd, f->prefix, move);
}

// oracle forkingMove (chooseRandomForkingMove play.cpp:615-633): 70% a temperature-1
// policy move, 25% temperature 2 (chooseRandomPolicyMove playutils.cpp:62-95: policy
// positions in order, probability > 0, not `ban`, chooseIndexWithTemperature), 5% a
// uniform legal move in cell-major order (chooseRandomLegalMove :10-31).  pol: the
// post-processed policy (illegal < 0); cpos / cval / pr: LDS [MAX_P] scratch.
// Returns the policy position, or -1 when there is none.
KC_D int forkingMove(const GV& v, DRng& rng, const float* pol, const DBoard& b, int ban, int* cpos, float* cval,
                     float* pr) {
  const DTables& T = v.T;
  const float r = rng.uni();
  int n = 0;
  if(r < 0.95f) {
    const float temp = r < 0.70f ? 1.0f : 2.0f;
    for(int base = 0; base < T.P; base += 64) {
      const int p = base + v.lane;
      const float q = p < T.P ? pol[p] : -1.0f;
      const bool ok = q > 0.0f && p != ban;
      const uint64_t m = ballot(ok);
      if(ok) {
        const int i = n + __popcll(m & ((1ULL << v.lane) - 1ULL));
        cpos[i] = p;
        cval[i] = q;
      }
      n += __popcll(m);
    }
    waveSync();
    if(n <= 0)
      return -1;
    const int ci = chooseIndex(v, rng, cval, n, temp, pr);
    waveSync();
    return cpos[ci];
  }
  for(int base = 0; base < T.P; base += 64) {
    const int q = base + v.lane;  // cell-major
    const int p = (q & 3) * T.A + (q >> 2);
    const bool ok = q < T.P && p != ban && isLegal(T, b, q >> 2, q & 3);
    const uint64_t m = ballot(ok);
    if(ok)
      cpos[n + __popcll(m & ((1ULL << v.lane) - 1ULL))] = p;
    n += __popcll(m);
  }
  waveSync();
  if(n <= 0)
    return -1;
  const int k = (int)rng.below((uint32_t)n);
  return cpos[k];
}

// A side position `b` joins the game's queue unless it is finished or the queue is full.
KC_D void pushSide(const GV& v, GameDev& s, const DBoard& b) {
  if(b.finished || s.sideCount >= MAX_SIDE)
    return;
  if(v.lane == 0)
    v.d.side[(size_t)v.g * MAX_SIDE + s.sideCount] = b;
  s.sideCount++;
  waveSync();
}

// oracle startSideSearch: the next queued side position becomes the root of a full
// search from a cleared tree (play.cpp:1586-1590: setPosition + runWholeSearchAndGetMove
// with the bot's own parameters).
KC_D void startSideSearch(const GV& v, GameDev& s) {
  s.root = v.d.side[(size_t)v.g * MAX_SIDE + s.sideNext];
  clearTables(v, s);
  s.visitLimit = v.d.sp.maxVisits;
  s.noNoise = 0;
  s.moveWeight = 1.0f;
  s.sideMode = 1;
  s.phase = PH_ROOTEVAL;
  s.rootK = 0;
  s.leafKind = LEAF_NONE;
  waveSync();
}

// After a game's rows: its side positions are searched, then the fork decision and
// the slot's next game (play.cpp:1576-1662, selfplay gameLoop :2008).
KC_D void afterGame(const GV& v, GameDev& s, DRng& rng, uint16_t* scratch) {
  if(s.sideNext < s.sideCount) {
    startSideSearch(v, s);
    s.rngCtr = rng.ctr;
    return;
  }
  s.sideMode = 0;
  if(!maybeFork(v, s, rng, scratch))
    startGame(v, s);
  else
    s.rngCtr = rng.ctr;
}

// oracle emitSideRow (writeGame side rows trainingwrite.cpp:894-937 + addRow with
// isSidePosition, :316-565): the side position's search targets; one value target
// (the search's root value), no next-move policy, no ownership / future boards /
// final run lengths (the reference passes NULL for them; its finalMaxLength
// dereference is B15, here zeros).  History masks from the game stream.
KC_D void emitSideRow(const GV& v, const GameDev& s, const TurnRec& rec, DRng& rng, const DBoard& b, int gameNumMeta) {
  const SearchDev& d = v.d;
  const DTables& T = v.T;
  const int A = T.A, P = T.P, pb = (A + 7) / 8;
  bool h = true;
  uint32_t hm = 0;
  for(int i = 0; i < 5; i++) {
    h = h && rng.uni() < 0.98f;
    hm |= (h ? 1u : 0u) << i;
  }
  unsigned long long r = 0;
  if(v.lane == 0) {
    r = atomicAdd(d.rCount, 1ull);
    if(r >= (unsigned long long)d.rowCap) {
      atomicAdd(d.rCount, (unsigned long long)-1ll);
      atomicAdd(d.rDropped, 1ull);
      r = ~0ull;
    }
  }
  const uint32_t lo = (uint32_t)bcastLane((int)(uint32_t)r, 0), hi = (uint32_t)bcastLane((int)(uint32_t)(r >> 32), 0);
  r = ((unsigned long long)hi << 32) | lo;
  if(r == ~0ull)
    return;
  const int pla = b.pla;
  packRowBinWave(T, b, d.rBin + r * NUM_SPATIAL * pb);
  if(v.lane == 0)
    d.rGlob[r] = (float)T.W;
  const int16_t* sp0 = d.sidePol + (size_t)v.g * P;
  int16_t* pol = d.rPol + r * 2 * P;
  for(int p = v.lane; p < P; p += 64) {
    pol[p] = sp0[p];
    pol[P + p] = (int16_t)1;
  }
  const int li = v.lane;
  float gval = 0.0f;
  if(li < 10)
    gval = (li & 1) ? (pla == 2 ? rec.whiteLoss : rec.whiteWin) : (pla == 2 ? rec.whiteWin : rec.whiteLoss);
  else if(li == 25 || li == 26 || li == 63)
    gval = 1.0f;
  else if(li == 30)
    gval = rec.policySurprise;
  else if(li == 31)
    gval = rec.policyEntropy;
  else if(li == 32)
    gval = rec.searchEntropy;
  else if(li >= 36 && li <= 40)
    gval = ((hm >> (li - 36)) & 1u) ? 1.0f : 0.0f;
  else if(li == 41)
    gval = (float)(s.gameHash0 & 0x3FFFFF);
  else if(li == 42)
    gval = (float)((s.gameHash0 >> 22) & 0x3FFFFF);
  else if(li == 43)
    gval = (float)((s.gameHash0 >> 44) & 0xFFFFF);
  else if(li == 44)
    gval = (float)(s.gameHash1 & 0x3FFFFF);
  else if(li == 45)
    gval = (float)((s.gameHash1 >> 22) & 0x3FFFFF);
  else if(li == 46)
    gval = (float)((s.gameHash1 >> 44) & 0xFFFFF);
  else if(li == 51)
    gval = (float)b.turn;
  else if(li == 53)
    gval = (float)s.startTurn;
  else if(li == 49)
    gval = *d.modelGen != s.startGen ? 1.0f : 0.0f;  // [50]: 0 (searched with the current network)
  else if(li == 55)
    gval = (float)s.gameMode;
  else if(li == 57)
    gval = pla == 2 ? rec.rawWhiteWL : -rec.rawWhiteWL;
  else if(li == 59)
    gval = rec.rawPolicyEntropy;
  else if(li == 60)
    gval = (float)rec.visits;
  d.rGt[r * 64 + li] = gval;
  int8_t* vt = d.rVal + r * 5 * A;
  for(int i = v.lane; i < 5 * A; i += 64)
    vt[i] = 0;
  if(v.lane < 4) {
    const int m = v.lane == 0 ? d.slotBase + v.g : (v.lane == 1 ? gameNumMeta : (v.lane == 2 ? b.turn : s.numTurns));
    d.rMeta[r * 4 + v.lane] = m;
  }
}

// oracle searchTargets: extractPolicyTarget (play.cpp:635-672; scaleMaxToAtLeast 10, no
// direct policy moves) into pt (global [P]) and getPolicySurpriseAndEntropy
// (searchresults.cpp:486-550) at node ni with policy pol.
template <int NI>
KC_D void searchTargets(const GV& v, const SP& sp, const GameDev& s, int ni, const float* pol, bool isRoot,
                        int16_t* pt, TurnRec& rec, int* posv, float* vals, float* tmp, float* tmp2) {
  const int P = v.d.P;
  for(int p = v.lane; p < P; p += 64)
    pt[p] = 0;
  {
    int m = playSelectionValuesAt<NI>(v, sp, s, ni, pol, isRoot, 10.0f, false, posv, vals, sp.useLcb);
    float mx = 0.0f;
    for(int i = v.lane; i < m; i += 64)
      mx = vals[i] > mx ? vals[i] : mx;
    mx = waveMax(mx);
    float factor = mx > 30000.0f ? 30000.0f / mx : 1.0f;
    waveSync();
    for(int i = v.lane; i < m; i += 64)
      pt[posv[i]] = (int16_t)roundf(vals[i] * factor);
  }
  waveSync();
  int m = playSelectionValuesAt<NI>(v, sp, s, ni, pol, isRoot, 1.0f, true, posv, vals, sp.useLcb);
  const float sumV = seqSum(vals, m, v.lane);
  // per-child terms (0 where the oracle skips), summed in order on lane 0
  waveSync();
  for(int i = v.lane; i < m; i += 64) {
    float p = fmaxf(pol[posv[i]], 1e-30f);
    float tt = vals[i] / sumV;
    float st = 0.0f, et = 0.0f;
    if(tt > 1e-30f) {
      float lt = dlog(tt), lp = dlog(p);
      st = tt * (lt - lp);
      et = -tt * lt;
    }
    tmp[i] = st;
    tmp2[i] = et;
  }
  const float surprise = seqSum(tmp, m, v.lane);
  const float searchEnt = seqSum(tmp2, m, v.lane);
  waveSync();
  for(int p = v.lane; p < P; p += 64) {
    float q = pol[p];
    tmp[p] = q > 1e-30f ? -q * dlog(q) : 0.0f;
  }
  float polEnt = seqSum(tmp, P, v.lane);
  rec.policySurprise = fmaxf(0.0f, surprise);
  rec.searchEntropy = fmaxf(0.0f, searchEnt);
  rec.policyEntropy = fmaxf(0.0f, polEnt);
  waveSync();
}

// oracle valueTargets (extractValueTargets play.cpp:674-682, reportedsearchvalues.cpp:10-50)
KC_D void valueTargets(const Node& n, TurnRec& rec) {
  float wl = fmaxf(-1.0f, fminf(1.0f, n.winLossAvg));
  rec.whiteWin = fmaxf(0.0f, fminf(1.0f, 0.5f * (wl + 1.0f)));
  rec.whiteLoss = fmaxf(0.0f, fminf(1.0f, 0.5f * (-wl + 1.0f)));
  rec.rootWL = wl;
}

// oracle rawStats (computeNNRawStats play.cpp:684-704) from a stored evaluation
KC_D void rawStats(const GV& v, float win, float loss, const float* pol, TurnRec& rec, float* tmp) {
  rec.rawWhiteWL = win - loss;
  for(int p = v.lane; p < v.d.P; p += 64) {
    float q = pol[p];
    tmp[p] = q >= 1e-30f ? -q * dlog(q) : 0.0f;
  }
  // in-order sum of only the q >= 1e-30 terms: zero terms are exact no-ops
  rec.rawPolicyEntropy = seqSum(tmp, v.d.P, v.lane);
  waveSync();
}

// oracle recordTreeRec (recordTreePositionsRec play.cpp:710-814, maxDepth 5), as a
// pre-order walk with an explicit stack: a side row at every non-root node reached
// only through the best moves of the player to move there; excl0/excl1 skipped at the
// root.  Frames and boards live in LDS; every lane walks the same path.
template <int NI>
KC_D void recordTreePositions(const GV& v, const SP& sp, const GameDev& s, DRng& rng, int excl0, int excl1,
                              uint32_t rootVisits, int gameNumMeta, int* posv, float* vals, float* tmp, float* tmp2) {
  constexpr int MAXD = 5;
  __shared__ DBoard tb[MAXD + 1];
  __shared__ int fNode[MAXD + 1], fNext[MAXD + 1], fBest[MAXD + 1], fFlags[MAXD + 1];
  const SearchDev& d = v.d;
  const int A = d.A;
  int16_t* pt = d.sidePol + (size_t)v.g * d.P;
  tb[0] = s.root;
  fNode[0] = s.rootIdx;
  fFlags[0] = 3;  // bit 0: the player to move has played best so far; bit 1: the opponent
  waveSync();
  int depth = 0;
  bool enter = true;
  while(depth >= 0) {
    const int ni = fNode[depth];
    const int k = v.nodes()[ni].numChildren;
    const NodeEdges E = v.edges(ni);
    if(enter) {
      enter = false;
      if(k <= 0) {
        depth--;
        continue;
      }
      if((fFlags[depth] & 1) && ni != s.rootIdx) {
        TurnRec rec;
        searchTargets<NI>(v, sp, s, ni, v.pol(ni), false, pt, rec, posv, vals, tmp, tmp2);
        const Node& n = v.nodes()[ni];
        rawStats(v, n.nnWin, n.nnLoss, v.pol(ni), rec, tmp);
        valueTargets(n, rec);
        rec.visits = rootVisits;
        // resolveWeight (play.cpp:1683-1696) when the position is recorded
        const float w = sp.recordTreeWeight;
        const float fl = floorf(w);
        const int copies = (int)fl + (rng.uni() < w - fl ? 1 : 0);
        for(int c = 0; c < copies; c++)
          emitSideRow(v, s, rec, rng, tb[depth], gameNumMeta);
        waveSync();
      }
      if(depth >= MAXD) {
        depth--;
        continue;
      }
      // the most-visited child; children[0]'s count is not consulted (:757-769)
      float bv = -1.0f;
      int bi = BIG;
      for(int i = 1 + v.lane; i < k; i += 64) {
        const float cv = (float)v.nodes()[E[i].child].visits;
        if(cv > bv) {
          bv = cv;
          bi = i;
        }
      }
      waveArgmax(bv, bi);
      fBest[depth] = bv > 0.0f ? bi : 0;
      fNext[depth] = 0;
      waveSync();
    }
    const int flags = fFlags[depth], best = fBest[depth];
    const bool plaB = (flags & 1) != 0, oppB = (flags & 2) != 0;
    int found = -1, foundFlags = 0;
    for(int i = fNext[depth]; i < k; i++) {
      const bool np = oppB, no = plaB && i == best;
      if(!np && !no)
        continue;
      const Edge e = E[i];
      const int mv = (int)e.move;
      if(depth == 0 && (mv == excl0 || mv == excl1))
        continue;
      if((long long)v.nodes()[e.child].visits < (long long)sp.recordTreeThreshold)
        continue;
      found = i;
      foundFlags = (np ? 1 : 0) | (no ? 2 : 0);
      break;
    }
    if(found < 0) {
      depth--;
      continue;
    }
    const Edge e = E[found];
    waveSync();
    fNext[depth] = found + 1;
    tb[depth + 1] = tb[depth];
    waveSync();
    playMoveWave(v.T, tb[depth + 1], (int)e.move % A, (int)e.move / A);
    fNode[depth + 1] = (int)e.child;
    fFlags[depth + 1] = foundFlags;
    waveSync();
    depth++;
    enter = true;
  }
  waveSync();
}

// oracle sideEval: the network's policy at a side position's continuation picks a
// forking move (no ban); the result joins the queue; then the next side position.
template <int NI>
KC_D void sideEval(const GV& v, GameDev& s, const float* o, float* scratch /* LDS [3*MAX_P] */) {
  float w, l;
  float pv[NI];
  postprocess<NI>(v, s.leaf, s.leafSym, o, scratch, w, l, scratch, pv);
  waveSync();
  DRng rng{s.rngSeed, s.rngCtr};
  // candidates compact in place over the policy (candidate i <= its position)
  const int fm = forkingMove(v, rng, scratch, s.leaf, -1, reinterpret_cast<int*>(scratch + MAX_P), scratch,
                             scratch + 2 * MAX_P);
  if(fm >= 0) {
    DBoard b3 = s.leaf;
    playMoveWave(v.T, b3, fm % v.T.A, fm / v.T.A);
    pushSide(v, s, b3);
  }
  s.sideNext++;
  afterGame(v, s, rng, reinterpret_cast<uint16_t*>(scratch + MAX_P));
  waveSync();
}

// oracle finishGame (play.cpp:1431-1460 + trainingwrite.cpp:316-565, 774-890), commit
// part: the SGF move record, the row reservation and the FinRec kRows reads.  The
// turn records and per-turn policies stay in place until the game's next commit,
// so kRows (launched right after this kernel) reads them there.
// oracle resolveTurnWeights: value surprise (play.cpp:1470-1497), surprise-weighted
// target weights (:1498-1574), probabilistic resolution (:1683-1697).  Every lane runs
// the sequential loops on the same data; lane 0 stores each turn's row count.
// Returns the game's number of rows.
KC_D int resolveTurnWeights(const GV& v, const GameDev& s, DRng& rng, float* vs /* LDS [MAX_AREA] */) {
  const SP& b = v.d.sp;
  const int n = s.numTurns, t0 = s.startTurn, A = v.T.A;  // searched turns [t0, n)
  TurnRec* tr = v.turns();
  const float finalWin = s.root.winner == 2 ? 1.0f : (s.root.winner == 1 ? 0.0f : 0.5f);
  float psdw = b.policySurpriseWeight, vsdw = b.valueSurpriseWeight;
  bool reweight = false;
  float sumW = 0.0f, sumPPV = 0.0f, sumVPV = 0.0f, thr = 0.0f;
  if(psdw > 0.0f || vsdw > 0.0f) {
    if(v.lane == 0) {
      const float nowFactor = 1.0f / (1.0f + (float)A * 0.016f);
      float winV = finalWin, lossV = 1.0f - finalWin;
      for(int i = n - 1; i >= t0; i--) {
        winV = winV + nowFactor * (tr[i].whiteWin - winV);
        lossV = lossV + nowFactor * (tr[i].whiteLoss - lossV);
        float x = 0.0f;
        if(winV > 1e-30f)
          x = x + winV * (dlog(winV) - dlog(fmaxf(tr[i].rootNNWin, 1e-30f)));
        if(lossV > 1e-30f)
          x = x + lossV * (dlog(lossV) - dlog(fmaxf(tr[i].rootNNLoss, 1e-30f)));
        if(x < 0.0f)
          x = 0.0f;
        vs[i] = fminf(x, 1.0f);
      }
    }
    waveSync();
    float sumPS = 0.0f, sumVS = 0.0f;
    for(int i = t0; i < n; i++) {
      const float tw = tr[i].targetWeight;
      sumW = sumW + tw;
      sumPS = sumPS + tr[i].policySurprise * tw;
      sumVS = sumVS + vs[i] * tw;
    }
    if(sumW >= 1.0f) {
      reweight = true;
      const float avgPS = sumPS / sumW, avgVS = sumVS / sumW;
      if(avgVS < 0.010f)
        vsdw = vsdw * (avgVS / 0.010f);
      thr = avgPS * 1.5f;
      for(int i = t0; i < n; i++) {
        const float tw = tr[i].targetWeight, ps = tr[i].policySurprise;
        sumPPV = sumPPV + (tw * ps + (1.0f - tw) * fmaxf(0.0f, ps - thr));
        sumVPV = sumVPV + tw * vs[i];
      }
      sumPPV = fmaxf(sumPPV, 1e-10f);
      sumVPV = fmaxf(sumVPV, 1e-10f);
    }
  }
  int total = 0;
  for(int i = t0; i < n; i++) {
    float w = tr[i].targetWeight;
    if(reweight) {
      const float ps = tr[i].policySurprise;
      const float ppv = w * ps + (1.0f - w) * fmaxf(0.0f, ps - thr);
      const float vpv = w * vs[i];
      w = (1.0f - psdw - vsdw) * w + psdw * ppv * sumW / sumPPV + vsdw * vpv * sumW / sumVPV;
    }
    if(w <= 0.0f)
      w = 0.0f;
    const float fl = floorf(w), excess = w - fl;
    const int rows = (int)(rng.uni() < excess ? fl + 1.0f : fl);
    total += rows;
    waveSync();
    if(v.lane == 0)
      tr[i].rows = (uint8_t)rows;
  }
  waveSync();
  return total;
}

KC_D void finishGameRecord(const GV& v, const GameDev& s, DRng& rng, float* scratch) {
  const SearchDev& d = v.d;
  const int numMoves = s.numTurns;
  const TurnRec* tr = v.turns();
  const int numRows = resolveTurnWeights(v, s, rng, scratch);
  {
    // the game's move record (SGF)
    unsigned long long gi = 0;
    if(v.lane == 0) {
      gi = atomicAdd(d.gCount, 1ull);
      if(gi >= (unsigned long long)d.gCap) {
        atomicAdd(d.gCount, (unsigned long long)-1ll);
        atomicAdd(d.gDropped, 1ull);
      }
    }
    gi = (unsigned long long)(uint32_t)bcastLane((int)(uint32_t)gi, 0);
    if(gi < (unsigned long long)d.gCap) {
      GameRec* gr = d.gRec + gi;
      if(v.lane == 0) {
        gr->slot = d.slotBase + v.g;
        gr->gameNum = (int32_t)s.gameNum;
        gr->numMoves = numMoves;
        gr->winner = s.root.winner;
      }
      for(int t = v.lane; t < numMoves; t += 64) {
        gr->cell[t] = (uint8_t)tr[t].cell;
        gr->dir[t] = (uint8_t)tr[t].dir;
      }
    }
  }
  if(v.lane == 0) {
    unsigned long long base = atomicAdd(d.rCount, (unsigned long long)numRows);
    bool fits = true;
    if(base + (unsigned long long)numRows > (unsigned long long)d.rowCap) {
      atomicAdd(d.rCount, (unsigned long long)(-(long long)numRows));
      atomicAdd(d.rDropped, (unsigned long long)numRows);
      fits = false;
    }
    FinRec* f = d.fin + v.g;
    f->rngSeed = rng.seed;
    f->rngCtr = rng.ctr;
    f->gameHash0 = s.gameHash0;
    f->gameHash1 = s.gameHash1;
    f->rowBase = base;
    f->numMoves = numMoves;
    f->numRows = numRows;
    f->startTurn = s.startTurn;
    f->gameMode = s.gameMode;
    f->genStart = s.startGen;
    f->genEnd = *d.modelGen;
    f->winner = s.root.winner;
    f->gameNum = s.gameNum;
    f->pending = fits && numRows > 0 ? 1 : 0;
  }
}

// kRows: the training rows of the games the preceding kCommit finished
// (trainingwrite.cpp:316-565 addRow via writeGame :774-890; turn t is written
// TurnRec::rows times).  One 256-thread block per committed game; the boards after
// every move, the row -> turn map and the final board's per-cell max runs are built
// once in LDS, then wave w writes rows w, w + 4, ...
constexpr int ROWS_WAVES = 8;
__global__ void __launch_bounds__(64 * ROWS_WAVES) kRows(const SearchDev* __restrict__ dp,
                                                         const DTables* __restrict__ Tp) {
  const SearchDev& d = *dp;
  if((int)blockIdx.x >= *d.commitCount)
    return;
  const int g = d.commitList[blockIdx.x];
  FinRec* fp = d.fin + g;
  if(fp->pending != 1)
    return;
  const FinRec f = *fp;
  const DTables& T = *Tp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  GV v(d, T, g);
  __shared__ DBoard boards[MAX_AREA + 1];
  __shared__ float tWin[MAX_AREA + 1], tLoss[MAX_AREA + 1];
  __shared__ int8_t finRun[MAX_AREA];
  __shared__ uint8_t hMask[2 * MAX_AREA];
  __shared__ uint8_t rowTurn[2 * MAX_AREA];
  __shared__ uint8_t tCell[MAX_AREA], tDir[MAX_AREA], tRows[MAX_AREA];
  const int numMoves = f.numMoves, numRows = min(f.numRows, 2 * MAX_AREA);  // <= 2 numMoves by construction
  const int A = T.A, P = T.P, pb = (A + 7) / 8;
  const TurnRec* tr = v.turns();
  const float finalWin = f.winner == 2 ? 1.0f : (f.winner == 1 ? 0.0f : 0.5f);
  // the turn records into LDS in parallel; the serial steps below then read LDS only
  for(int t = threadIdx.x; t < numMoves; t += 64 * ROWS_WAVES) {
    const TurnRec rec = tr[t];
    tWin[t] = rec.whiteWin;
    tLoss[t] = rec.whiteLoss;
    tCell[t] = (uint8_t)rec.cell;
    tDir[t] = (uint8_t)rec.dir;
    tRows[t] = rec.rows;
  }
  __syncthreads();
  if(threadIdx.x == 0) {
    tWin[numMoves] = finalWin;
    tLoss[numMoves] = 1.0f - finalWin;
    DBoard b;
    boardInit(T, b);
    boards[0] = b;
    for(int t = 0; t < numMoves; t++) {
      applyMove(T, b, tCell[t], tDir[t]);
      boards[t + 1] = b;
    }
    int j = 0;
    for(int t = 0; t < numMoves; t++)
      for(int c = 0; c < (int)tRows[t] && j < 2 * MAX_AREA; c++)
        rowTurn[j++] = (uint8_t)t;
    // history-mask draws, in row order from the game's stream (the chain stops
    // drawing at its first failure, so the draws are consumed sequentially)
    DRng rng{f.rngSeed, f.rngCtr};
    for(int r = 0; r < numRows; r++) {
      bool h = true;
      uint32_t hm = 0;
      for(int i = 0; i < 5; i++) {
        h = h && rng.uni() < 0.98f;
        hm |= (h ? 1u : 0u) << i;
      }
      hMask[r] = (uint8_t)hm;
    }
  }
  __syncthreads();
  const DBoard& fin = boards[numMoves];
  for(int c = threadIdx.x; c < A; c += 64 * ROWS_WAVES)
    finRun[c] = colorAt(fin, c) == 0 ? 0 : (int8_t)maxRun(T, fin, c);
  __syncthreads();
  const float nowF1 = 1.0f / (1.0f + (float)A * 0.176f), nowF2 = 1.0f / (1.0f + (float)A * 0.056f),
              nowF3 = 1.0f / (1.0f + (float)A * 0.016f);
  for(int row = wave; row < numRows; row += ROWS_WAVES) {
    const int t = rowTurn[row];
    const uint32_t hm = hMask[row];
    const size_t r = (size_t)f.rowBase + row;
    const DBoard& b = boards[t];
    const int pla = b.pla, opp = 3 - pla;
    packRowBinWave(T, b, d.rBin + r * NUM_SPATIAL * pb);
    if(lane == 0)
      d.rGlob[r] = (float)T.W;
    const int16_t* p0 = v.turnPol(t);
    const int16_t* p1 = t + 1 < numMoves ? v.turnPol(t + 1) : nullptr;
    int16_t* pol = d.rPol + r * 2 * P;
    for(int p = lane; p < P; p += 64) {
      pol[p] = p0[p];
      pol[P + p] = p1 ? p1[p] : (int16_t)1;
    }
    float gval = 0.0f;
    const int li = lane;
    if(li < 10) {
      const int fi = li >> 1;
      const float nf = fi == 0 ? 0.0f : (fi == 1 ? nowF1 : (fi == 2 ? nowF2 : (fi == 3 ? nowF3 : 1.0f)));
      float win = 0.0f, loss = 0.0f, left = 1.0f;
      for(int i = t; i <= numMoves; i++) {
        float now;
        if(i == numMoves) {
          now = left;
          left = 0.0f;
        } else {
          now = left * nf;
          left = left * (1.0f - nf);
        }
        win = win + now * (pla == 2 ? tWin[i] : tLoss[i]);
        loss = loss + now * (pla == 2 ? tLoss[i] : tWin[i]);
      }
      gval = (li & 1) ? loss : win;
    } else if(li == 22) {
      float sum = 0.0f;
      for(int i = t + 1; i <= numMoves; i++) {
        float prevWL = tWin[i - 1] - tLoss[i - 1], nextWL = tWin[i] - tLoss[i];
        float var = (nextWL - prevWL) * (nextWL - prevWL);
        sum = sum + (float)(i - t) * var;
      }
      gval = sum;
    } else if(li == 25 || li == 26 || li == 27 || li == 33 || li == 63) {
      gval = 1.0f;
    } else if(li == 28) {
      gval = t + 1 < numMoves ? 1.0f : 0.0f;
    } else if(li == 30) {
      gval = tr[t].policySurprise;
    } else if(li == 31) {
      gval = tr[t].policyEntropy;
    } else if(li == 32) {
      gval = tr[t].searchEntropy;
    } else if(li >= 36 && li <= 40) {
      gval = ((hm >> (li - 36)) & 1u) ? 1.0f : 0.0f;
    } else if(li == 41) {
      gval = (float)(f.gameHash0 & 0x3FFFFF);
    } else if(li == 42) {
      gval = (float)((f.gameHash0 >> 22) & 0x3FFFFF);
    } else if(li == 43) {
      gval = (float)((f.gameHash0 >> 44) & 0xFFFFF);
    } else if(li == 44) {
      gval = (float)(f.gameHash1 & 0x3FFFFF);
    } else if(li == 45) {
      gval = (float)((f.gameHash1 >> 22) & 0x3FFFFF);
    } else if(li == 46) {
      gval = (float)((f.gameHash1 >> 44) & 0xFFFFF);
    } else if(li == 51) {
      gval = (float)t;
    } else if(li == 53) {
      gval = (float)f.startTurn;
    } else if(li == 49) {
      // earlier-network metadata (trainingwrite.cpp:459-461, :844-850): the game saw a
      // hot reload; reloads after this turn's commit
      gval = f.genEnd != f.genStart ? 1.0f : 0.0f;
    } else if(li == 50) {
      gval = (float)(uint8_t)((uint32_t)f.genEnd - (uint32_t)tr[t].gen);
    } else if(li == 55) {
      gval = (float)f.gameMode;
    } else if(li == 57) {
      gval = pla == 2 ? tr[t].rawWhiteWL : -tr[t].rawWhiteWL;
    } else if(li == 59) {
      gval = tr[t].rawPolicyEntropy;
    } else if(li == 60) {
      gval = (float)tr[t].visits;
    }
    d.rGt[r * 64 + li] = gval;
    int8_t* vt = d.rVal + r * 5 * A;
    const DBoard& b2 = boards[min(t + 2, numMoves)];
    const DBoard& b3 = boards[min(t + 6, numMoves)];
    for(int c = lane; c < A; c += 64) {
      int fc = colorAt(fin, c), c2 = colorAt(b2, c), c3 = colorAt(b3, c);
      vt[c] = fc == pla ? 1 : (fc == opp ? -1 : 0);
      vt[A + c] = 0;
      vt[2 * A + c] = c2 == pla ? 1 : (c2 == opp ? -1 : 0);
      vt[3 * A + c] = c3 == pla ? 1 : (c3 == opp ? -1 : 0);
      vt[4 * A + c] = finRun[c];
    }
    if(lane < 4) {
      int m = lane == 0 ? d.slotBase + g : (lane == 1 ? f.gameNum : (lane == 2 ? t : numMoves));
      d.rMeta[r * 4 + lane] = m;
    }
  }
  __syncthreads();
  if(threadIdx.x == 0)
    fp->pending = 0;
}

// oracle commitMove (getChosenMoveLoc searchresults.cpp:435-453, extract*Targets
// play.cpp:635-704, getPolicySurpriseAndEntropy searchresults.cpp:486-550, makeMove)
template <int NI>
__global__ void __launch_bounds__(64) kCommit(const SearchDev* __restrict__ dp, const DTables* __restrict__ Tp) {
  const SearchDev& d = *dp;
  if((int)blockIdx.x >= *d.commitCount)
    return;
  const int g = d.commitList[blockIdx.x];
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int* posv = reinterpret_cast<int*>(lds);                    // [MAX_P]
  float* vals = reinterpret_cast<float*>(posv + MAX_P);       // [MAX_P]
  float* tmp = vals + MAX_P;                                  // [MAX_P]
  float* tmp2 = tmp + MAX_P;                                  // [MAX_P]
  int* qtail = reinterpret_cast<int*>(tmp2 + MAX_P);
  uint32_t* liveBits = reinterpret_cast<uint32_t*>(qtail + 4);  // [cap/32]
  uint16_t* queue = reinterpret_cast<uint16_t*>(liveBits + d.cap / 32);     // [cap]
  __shared__ GameDev s;
  GV v(d, *Tp, g);
  SPROF_INIT();
  [[maybe_unused]] const unsigned long long t0 = SPROF_NOW();
  loadGame(v, s);
  const SP& sp = d.sp;
  const int P = d.P, A = d.A;
  DRng rng{s.rngSeed, s.rngCtr};
  if(s.root.finished) {
    // a policy-initialisation move ended the game: nothing was searched, no rows
    // (the reference's main loop does not run, play.cpp:1262-1264)
    finishGameRecord(v, s, rng, reinterpret_cast<float*>(lds) + 2 * MAX_P);
    s.gamesFinished++;
    s.gameNum++;
    s.sideNext = 0;
    afterGame(v, s, rng, reinterpret_cast<uint16_t*>(lds));
    waveSync();
    storeGame(v, s);
    return;
  }
  // a side position's search (play.cpp:1576-1662) ends like a move search, but
  // writes one row and plays nothing
  const bool side = s.sideMode != 0;
  // move choice: self-play disables LCB for the game's moves (runBotWithLimits
  // play.cpp:1040-1046), not for a side position's response (:1590)
  int n = playSelectionValues<NI>(v, *v.sp, s, 0.0f, true, posv, vals, side ? sp.useLcb != 0 : false);
  if(n <= 0) {
    s.err = ERR_NO_CANDIDATE;
    n = 1;
    posv[0] = 0;
  }
  const float temp = interpolateEarly(v.T, s.root.turn, sp.moveTempHalflife, sp.moveTempEarly, sp.moveTemp);
  int ci = chooseIndex(v, rng, vals, n, temp, tmp);
  waveSync();
  const int chosen = posv[ci];
  const Node& r = v.nodes()[s.rootIdx];
  TurnRec rec;
  valueTargets(r, rec);
  rec.visits = r.visits;
  rec.rootNNWin = r.nnWin;
  rec.rootNNLoss = r.nnLoss;
  rec.targetWeight = s.moveWeight;
  rec.rows = 0;
  rec.gen = (uint8_t)*v.d.modelGen;
  const int t = s.numTurns;
  int16_t* pt = side ? d.sidePol + (size_t)g * P : v.turnPol(t);
  waveSync();
  // the targets run after runBotWithLimits restored the base parameters (play.cpp:1066, :1307-1320)
  searchTargets<NI>(v, sp, s, s.rootIdx, v.rootNoised(), true, pt, rec, posv, vals, tmp, tmp2);
  rawStats(v, s.rawWin, s.rawLoss, v.rawPolicy(), rec, tmp);
  const bool recordTree = sp.recordTree != 0 && sp.recordTreeWeight > 0.0f;
  if(side) {
    emitSideRow(v, s, rec, rng, s.root, s.gameNum - 1);
    // its subtree positions (play.cpp:1612-1628)
    if(recordTree)
      recordTreePositions<NI>(v, sp, s, rng, -1, -1, r.visits, s.gameNum - 1, posv, vals, tmp, tmp2);
    // occasionally continue: the response, then a forking move from the network's
    // policy there becomes another side position (play.cpp:1632-1656)
    if(rng.uni() < 0.25f) {
      DBoard b2 = s.root;
      playMoveWave(v.T, b2, chosen % A, chosen / A);
      if(!b2.finished) {
        s.leaf = b2;
        s.phase = PH_SIDEEVAL;
        s.rngCtr = rng.ctr;
        waveSync();
        storeGame(v, s);
        return;
      }
    }
    s.sideNext++;
    afterGame(v, s, rng, reinterpret_cast<uint16_t*>(posv));
    waveSync();
    storeGame(v, s);
    return;
  }
  // a side position: the root policy's alternative to the move (play.cpp:1328-1345)
  int forkMove = -1;
  if(sp.sideProb > 0.0f && rng.uni() < sp.sideProb) {
    const int fm = forkingMove(v, rng, v.pol(s.rootIdx), s.root, chosen, posv, vals, tmp);
    forkMove = fm;
    if(fm >= 0) {
      DBoard b2 = s.root;
      playMoveWave(v.T, b2, fm % A, fm / A);
      pushSide(v, s, b2);
    }
  }
  // subtree positions of this search, except the played and the forked branches
  // (play.cpp:1347-1361)
  if(recordTree) {
    waveSync();
    recordTreePositions<NI>(v, sp, s, rng, chosen, forkMove, r.visits, s.gameNum, posv, vals, tmp, tmp2);
  }
  rec.cell = (int8_t)(chosen % A);
  rec.dir = (int8_t)(chosen / A);
  for(int i = 0; i < 5; i++)
    rec.pad[i] = 0;
  waveSync();
  if(v.lane == 0)
    v.turns()[t] = rec;
  s.numTurns++;
  [[maybe_unused]] const unsigned long long t1 = SPROF_NOW();
  SPROF_ADD(18, t1 - t0);
  playMoveWave(v.T, s.root, chosen % A, chosen / A);
  s.moves++;
  waveSync();
  if(s.root.finished) {
    [[maybe_unused]] const unsigned long long t3 = SPROF_NOW();
    finishGameRecord(v, s, rng, tmp);
    [[maybe_unused]] const unsigned long long t4 = SPROF_NOW();
    s.gamesFinished++;
    s.gameNum++;
    s.sideNext = 0;
    waveSync();
    afterGame(v, s, rng, reinterpret_cast<uint16_t*>(posv));
    SPROF_ADD(20, t4 - t3);
    SPROF_ADD(21, SPROF_NOW() - t4);
    SPROF_ADD(23, 1);
  } else {
    // the next move's limits decide whether its search starts from a cleared tree
    if(setMoveLimits(v, s, rng, rec.rootWL))
      clearTables(v, s);
    else
      reuseTree(v, s, chosen, liveBits, queue, qtail);
    [[maybe_unused]] const unsigned long long t2 = SPROF_NOW();
    SPROF_ADD(19, t2 - t1);
    SPROF_ADD(22, s.liveCount);
    s.rngCtr = rng.ctr;
    s.phase = PH_ROOTEVAL;
    s.rootK = 0;
  }
  waveSync();
  storeGame(v, s);
  SPROF_ADD(16, 1);
  SPROF_ADD(17, SPROF_NOW() - t0);
  SPROF_FLUSH();
}

// kCompact: the list of games whose row the network evaluates this round, at most
// d.nnCap rows (one full wave of network workgroups: a launch's cost steps with its
// number of workgroup waves).  The needing games are taken in cyclic game order from
// the round-robin pointer *d.nnRR, which moves past the last game taken whenever the
// cap bites, so a deferred row waits at most ceil(G / cap) rounds.  Rows past the cap
// are deferred (nnDefer): their games keep their leaf and skip the next select.  The
// oracle applies the same rule (ora_search.cpp selfplayRound).
// accumulate != 0: the count is also added to *d.nnTimedEvals (sampled kernel timing).
// Layout: the games are cut into 64-game chunks; wave w owns the contiguous chunks
// [w * cpw, (w + 1) * cpw) and lane l game l of each, so every load and every nnDefer
// store is one coalesced 256-byte access per chunk.  The need flags and cache bids of
// all of a lane's chunks are loaded before the first use (up to CP_CH chunks per wave),
// so the kernel waits for one round of loads.  Positions: a lane's packed count (high
// half: needing games at or past the round-robin pointer, low half: the others, G <
// 65536) is summed over the wave and scanned over the waves; inside a wave the chunks
// are walked in order with a ballot per chunk.
// (256 threads cover a group of 8192 games: a 4-wave workgroup finds room beside the
// other group's network kernels, where a 1024-thread one waited for a whole CU to
// drain: 34 us per launch at C3)
constexpr int CP_CH = 32;
// resolve != 0 (after a fused kBackupSelect): the block first does kResolve's work -- the
// round winners' tags cleared by every thread, the pending selections completed by waves
// 0-3 -- and the compaction below reads the need flags and bids those selections wrote
// after a workgroup barrier: one dispatch fewer on every fused round.
constexpr int CP_RESOLVE_WAVES = 4;
// (The resolving instance alone holds the LDS game copies: the plain one, which the separate
// round kernels and the default precision's network run beside, keeps its 132 bytes of LDS
// and fits on a CU next to any network workgroup.)
template <int NI, bool RESOLVE>
__global__ void __launch_bounds__(1024) kCompact(const SearchDev* __restrict__ dp, const DTables* __restrict__ Tp,
                                                 int accumulate) {
  const SearchDev& d = *dp;
  __shared__ uint32_t wsum[16], wpre[17];
  const int nt = blockDim.x, nw = nt >> 6;  // 256 or 1024 threads (launchCompact)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if constexpr(RESOLVE) {
    __shared__ GameDev rs[CP_RESOLVE_WAVES];
    clearRoundTags(d, t, nt);
    if(w < CP_RESOLVE_WAVES)
      completePending<NI>(d, *Tp, w, CP_RESOLVE_WAVES, rs[w]);
    __syncthreads();
  }
  const int nch = (d.G + 63) >> 6;
  const int cpw = (nch + nw - 1) / nw;  // chunks per wave (<= 64: G < 65536, >= 16 waves past 8192 games)
  const int g0 = w * cpw * 64 + lane;   // this lane's game in the wave's first chunk
  const int p = *d.nnRR;
  const bool vec = cpw <= CP_CH;
  uint64_t need = 0;  // bit k: game g0 + 64 k needs the network
  uint32_t bids[CP_CH];
  if(vec) {
#pragma unroll
    for(int k = 0; k < CP_CH; k++) {
      bids[k] = ~0u;
      if(k < cpw) {
        const int i = g0 + 64 * k;
        const int ic = i < d.G ? i : 0;
        bids[k] = d.nnBid[ic];
        need |= (uint64_t)(i < d.G && d.nnNeed[ic] ? 1u : 0u) << k;
      }
    }
  } else {
    for(int k = 0; k < cpw; k++) {
      const int i = g0 + 64 * k;
      need |= (uint64_t)(i < d.G && d.nnNeed[i] ? 1u : 0u) << k;
    }
  }
  // bit k of atOrPast: game g0 + 64 k >= p
  const uint64_t atOrPast = p <= g0 ? ~0ull : (p - g0 > 64 * 63 ? 0ull : ~0ull << ((p - g0 + 63) / 64));
  uint32_t c = ((uint32_t)__popcll(need & atOrPast) << 16) + (uint32_t)__popcll(need & ~atOrPast);
#pragma unroll
  for(int off = 32; off >= 1; off >>= 1)
    c += (uint32_t)__shfl_xor((int)c, off, 64);
  if(lane == 0)
    wsum[w] = c;
  __syncthreads();
  if(t < 64) {
    uint32_t x = t < nw ? wsum[t] : 0u, xi = x;
#pragma unroll
    for(int off = 1; off < 16; off <<= 1) {
      const uint32_t v = (uint32_t)__shfl_up((int)xi, off, 64);
      if(t >= off)
        xi += v;
    }
    if(t < 16)
      wpre[t] = xi - x;
    if(t == 15)
      wpre[16] = xi;
  }
  __syncthreads();
  const uint32_t all = wpre[16], excl = wpre[w];
  const int totalHi = (int)(all >> 16), total = totalHi + (int)(all & 0xFFFFu), cap = d.nnCap;
  int oh = (int)(excl >> 16), ol = totalHi + (int)(excl & 0xFFFFu);  // wave-uniform running positions
  const uint64_t below = (1ull << lane) - 1ull;
  auto chunk = [&](int k, uint32_t bid) {
    const int i = g0 + 64 * k;
    const bool nd = (need >> k) & 1u;
    const uint64_t b = ballot(nd), ge = ballot(nd && i >= p);
    if(nd) {
      const int pos = i >= p ? oh + __popcll(ge & below) : ol + __popcll(b & ~ge & below);
      const bool in = pos < cap;
      if(in) {
        d.nnIdx[pos] = i;
        // the evaluation's bid for its NN-cache slot (kBackup: the highest game stores it)
        if(bid != ~0u)
          atomicMax(&d.cTag[bid], (uint32_t)i + 1u);
      }
      d.nnDefer[i] = in ? 0 : 1;
      if(total > cap && pos == cap - 1)
        *d.nnRR = i + 1 < d.G ? i + 1 : 0;
    } else if(i < d.G) {
      d.nnDefer[i] = 0;
    }
    oh += __popcll(ge);
    ol += __popcll(b & ~ge);
  };
  if(vec) {
#pragma unroll
    for(int k = 0; k < CP_CH; k++)
      if(k < cpw)
        chunk(k, bids[k]);
  } else {
    for(int k = 0; k < cpw; k++) {
      const int i = g0 + 64 * k;
      chunk(k, i < d.G ? d.nnBid[i] : ~0u);
    }
  }
  if(t == nt - 1) {
    const int count = min(total, cap);
    *d.nnCount = count;
    *d.pendCount = 0;  // the pending list kResolve (or the resolve phase above) completed
    if(accumulate)
      *d.nnTimedEvals += (unsigned long long)count;
  }
}

__global__ void __launch_bounds__(64) kInit(const SearchDev* __restrict__ dp, const DTables* __restrict__ Tp) {
  const SearchDev& d = *dp;
  const int g = blockIdx.x;
  if(g >= d.G)
    return;
  __shared__ GameDev s;
  GV v(d, *Tp, g);
  for(int i = v.lane; i < (int)(sizeof(GameDev) / 4); i += 64)
    reinterpret_cast<uint32_t*>(&s)[i] = 0;
  waveSync();
  s.svbSel = 0;
  s.gameNum = 0;
  startGame(v, s);
  // benchmark stagger: idle rounds before the slot's first game, so game ends (and
  // row bursts) spread over the run instead of arriving in phase; own stream, so
  // the games themselves are unchanged
  s.startDelay = d.startStagger > 0
                     ? (int32_t)(mix64(d.seed ^ 0x5a5a5a5a5a5a5a5aULL ^ (uint64_t)(d.slotBase + g)) %
                                 (uint64_t)d.startStagger)
                     : 0;
  waveSync();
  storeGame(v, s);
}

// Canonical breadth-first export of one game's tree (tests / tools).
// nodesOut [maxNodes][24] u32, edgesOut [maxNodes][P][3] u32 (child bfs index, edge visits, move).
__global__ void kGameTree(const SearchDev* __restrict__ dp, int g, int maxNodes, uint32_t* nodesOut,
                          uint32_t* edgesOut, int32_t* count) {
  const SearchDev& d = *dp;
  if(threadIdx.x != 0)
    return;
  const GameDev& s = d.games[g];
  const Node* NS = d.nodes + (size_t)g * d.cap;
  if(s.rootIdx < 0) {
    *count = 0;
    return;
  }
  // canonical index map kept in nodesOut word 23 of each discovered node: store original idx
  int n = 0;
  int head = 0;
  nodesOut[23] = (uint32_t)s.rootIdx;
  n = 1;
  while(head < n && head < maxNodes) {
    const int idx = (int)nodesOut[(size_t)head * 24 + 23];
    const Node& x = NS[idx];
    uint32_t* o = nodesOut + (size_t)head * 24;
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
    const uint64_t* nk = d.nodeKey + ((size_t)g * d.cap + idx) * 2;
    o[11] = (uint32_t)nk[0];
    o[12] = (uint32_t)(nk[0] >> 32);
    o[13] = (uint32_t)nk[1];
    o[14] = (uint32_t)(nk[1] >> 32);
    uint64_t sk = 0;
    int64_t sd = 0, sw = 0;
    if(x.svbEntry >= 0) {
      size_t e = ((size_t)g * 2 + s.svbSel) * d.svbCap + x.svbEntry;
      sk = d.svbKey[e];
      sd = d.svbD[e];
      sw = d.svbW[e];
    }
    o[15] = (uint32_t)sk;
    o[16] = (uint32_t)(sk >> 32);
    o[17] = (uint32_t)(uint64_t)sd;
    o[18] = (uint32_t)((uint64_t)sd >> 32);
    o[19] = (uint32_t)(uint64_t)sw;
    o[20] = (uint32_t)((uint64_t)sw >> 32);
    o[21] = 0;
    o[22] = 0;
    const NodeEdges E{d.edges + ((size_t)g * d.cap + idx) * INLINE_EDGES,
                      d.edgePool + ((size_t)g * 2 + d.games[g].edgeSel) * d.edgePoolCap + x.edgeBase};
    for(int i = 0; i < x.numChildren; i++) {
      const int c = (int)E[i].child;
      int ci = -1;
      for(int q = 0; q < n; q++)
        if((int)nodesOut[(size_t)q * 24 + 23] == c) {
          ci = q;
          break;
        }
      if(ci < 0 && n < maxNodes) {
        nodesOut[(size_t)n * 24 + 23] = (uint32_t)c;
        ci = n++;
      }
      uint32_t* eo = edgesOut + ((size_t)head * d.P + i) * 3;
      eo[0] = (uint32_t)ci;
      eo[1] = E[i].visits;
      eo[2] = E[i].move;
    }
    head++;
  }
  // replace word 23 (original index) by 0 so the export is index independent
  for(int q = 0; q < n; q++)
    nodesOut[(size_t)q * 24 + 23] = 0;
  *count = n;
}

// ---------------------------------------------------------------------------
static int laneItems(int P) { return P <= 128 ? 2 : (P <= 256 ? 4 : 7); }

// ---------------------------------------------------------------------------
// Row staging for device-resident gathers (coffee_selfplay_stage_rows): one wave per
// row packs the row's six arrays into one contiguous record (rows.py FIELDS: bin u8
// [15][pb], glob f32, pol i16 [2][P], gt f32 [64], val i8 [5][A], meta i32 [4]), so a
// rank's rows leave as one device block for the RCCL gather.
__global__ void __launch_bounds__(256) kStageRows(const SearchDev* __restrict__ dp, uint8_t* __restrict__ dst,
                                                  int rb) {
  const SearchDev& d = *dp;
  const int A = d.A, P = d.P, pb = (A + 7) / 8;
  const unsigned long long n = *d.rCount;
  const int lane = threadIdx.x & 63;
  const int sz[6] = {NUM_SPATIAL * pb, 4, 4 * P, 256, 5 * A, 16};
  for(unsigned long long r = blockIdx.x * 4ull + (threadIdx.x >> 6); r < n; r += gridDim.x * 4ull) {
    const uint8_t* src[6] = {d.rBin + r * sz[0], reinterpret_cast<const uint8_t*>(d.rGlob + r),
                             reinterpret_cast<const uint8_t*>(d.rPol + r * 2 * P),
                             reinterpret_cast<const uint8_t*>(d.rGt + r * 64), reinterpret_cast<const uint8_t*>((const int8_t*)d.rVal) + r * sz[4],
                             reinterpret_cast<const uint8_t*>(d.rMeta + r * 4)};
    uint8_t* o = dst + r * (unsigned long long)rb;
#pragma unroll
    for(int f = 0; f < 6; f++) {
      for(int i = lane; i < sz[f]; i += 64)
        o[i] = src[f][i];
      o += sz[f];
    }
  }
}

__global__ void kStageDone(const SearchDev* __restrict__ dp, int discardGames) {
  const SearchDev& d = *dp;
  *d.rStaged += *d.rCount;
  *d.rCount = 0;
  if(discardGames)
    *d.gCount = 0;
}

void launchStageRows(const SearchDev& d, const SearchDev* dd, uint8_t* dst, unsigned long long* countOut,
                     bool discardGames, hipStream_t st) {
  hipLaunchKernelGGL(kStageRows, dim3(1024), dim3(256), 0, st, dd, dst, rowBytes(d.A));
  KC_HIP(hipGetLastError());
  KC_HIP(hipMemcpyAsync(countOut, d.rCount, 8, hipMemcpyDeviceToHost, st));
  hipLaunchKernelGGL(kStageDone, dim3(1), dim3(1), 0, st, dd, discardGames ? 1 : 0);
  KC_HIP(hipGetLastError());
}

void launchSelfplayInit(const SearchDev& d, const SearchDev* dd, hipStream_t st) {
  hipLaunchKernelGGL(kInit, dim3(d.G), dim3(64), 0, st, dd, d.T);
  KC_HIP(hipGetLastError());
}

// 256 threads (one wave per SIMD) while each wave keeps at most CP_CH chunks of 64 games: a workgroup
// that small fits beside a network workgroup of the other game group on its CU (1024
// threads need 4 waves per SIMD) and does not wait for a free one.
void launchCompact(const SearchDev& d, const SearchDev* dd, hipStream_t st, bool accumulate, bool resolve) {
  const int nt = d.G <= 4 * 64 * CP_CH ? 256 : 1024;  // 1024 only past 8192 games per engine
  const DTables* T = d.T;
  const int a = accumulate ? 1 : 0;
  if(!resolve)
    hipLaunchKernelGGL((kCompact<2, false>), dim3(1), dim3(nt), 0, st, dd, T, a);
  else
    switch(laneItems(d.P)) {
      case 2: hipLaunchKernelGGL((kCompact<2, true>), dim3(1), dim3(nt), 0, st, dd, T, a); break;
      case 4: hipLaunchKernelGGL((kCompact<4, true>), dim3(1), dim3(nt), 0, st, dd, T, a); break;
      default: hipLaunchKernelGGL((kCompact<7, true>), dim3(1), dim3(nt), 0, st, dd, T, a); break;
    }
  KC_HIP(hipGetLastError());
}

// A launch, with start/end events recorded by the dispatch itself when given.
template <class K, class... Args>
static void launchEv(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st, hipEvent_t e0, hipEvent_t e1,
                     Args... args) {
  if(e0)
    hipExtLaunchKernelGGL(kernel, grid, block, lds, st, e0, e1, 0, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
}

void launchSelect(const SearchDev& d, const SearchDev* dd, hipStream_t st, hipEvent_t e0, hipEvent_t e1,
                  bool resetCommit) {
  const DTables* T = d.T;
  const int rc = resetCommit ? 1 : 0;
  switch(laneItems(d.P)) {
    case 2: launchEv(kSelect<2>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T, rc); break;
    case 4: launchEv(kSelect<4>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T, rc); break;
    default: launchEv(kSelect<7>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T, rc); break;
  }
  KC_HIP(hipGetLastError());
}

void launchBackup(const SearchDev& d, const SearchDev* dd, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const DTables* T = d.T;
  switch(laneItems(d.P)) {
    case 2: launchEv(kBackup<2>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T); break;
    case 4: launchEv(kBackup<4>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T); break;
    default: launchEv(kBackup<7>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T); break;
  }
  KC_HIP(hipGetLastError());
}

void launchBackupSelect(const SearchDev& d, const SearchDev* dd, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const DTables* T = d.T;
  switch(laneItems(d.P)) {
    case 2: launchEv(kBackupSelect<2>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T); break;
    case 4: launchEv(kBackupSelect<4>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T); break;
    default: launchEv(kBackupSelect<7>, dim3(d.G), dim3(64), 0, st, e0, e1, dd, T); break;
  }
  KC_HIP(hipGetLastError());
}

void launchResolve(const SearchDev& d, const SearchDev* dd, hipStream_t st) {
  const DTables* T = d.T;
  switch(laneItems(d.P)) {
    case 2: hipLaunchKernelGGL(kResolve<2>, dim3(RESOLVE_GRID), dim3(64), 0, st, dd, T); break;
    case 4: hipLaunchKernelGGL(kResolve<4>, dim3(RESOLVE_GRID), dim3(64), 0, st, dd, T); break;
    default: hipLaunchKernelGGL(kResolve<7>, dim3(RESOLVE_GRID), dim3(64), 0, st, dd, T); break;
  }
  KC_HIP(hipGetLastError());
}

void launchCommit(const SearchDev& d, const SearchDev* dd, hipStream_t st) {
  const size_t lds = commitLdsBytes(d.cap);
  switch(laneItems(d.P)) {
    case 2: hipLaunchKernelGGL(kCommit<2>, dim3(d.G), dim3(64), lds, st, dd, d.T); break;
    case 4: hipLaunchKernelGGL(kCommit<4>, dim3(d.G), dim3(64), lds, st, dd, d.T); break;
    default: hipLaunchKernelGGL(kCommit<7>, dim3(d.G), dim3(64), lds, st, dd, d.T); break;
  }
  KC_HIP(hipGetLastError());
  hipLaunchKernelGGL(kRows, dim3(d.G), dim3(64 * ROWS_WAVES), 0, st, dd, d.T);
  KC_HIP(hipGetLastError());
}

void launchGameTree(const SearchDev* dd, int slot, int maxNodes, uint32_t* nodesOut, uint32_t* edgesOut,
                    int32_t* count, hipStream_t st) {
  hipLaunchKernelGGL(kGameTree, dim3(1), dim3(64), 0, st, dd, slot, maxNodes, nodesOut, edgesOut, count);
  KC_HIP(hipGetLastError());
}

}  // namespace kc
