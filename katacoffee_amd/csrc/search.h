// Device-resident self-play state: one wave (64 lanes) owns one game.
//
// Layout in HBM (DESIGN.md "Data layout"), every array indexed by game slot g:
//   GameDev   games[G]                         per-game scalars (boards, RNG, phase, counters)
//   Node      nodes[G][cap]                    64-B statistics record per search node
//   Edge      edges[G][cap][16]                (child, edgeVisits, prior, move) of child slots 0..15,
//                                              slots in expansion order (SearchChildPointer, searchnode.h)
//   Edge      edgePool[G][2][edgePoolCap]      slots 16.. of the nodes with more children: one block per
//                                              node at Node::edgeBase, grown 48 -> P-16 like the reference's
//                                              child arrays (8 -> 64 -> P, searchnode.h:172-174), double
//                                              buffered so tree reuse compacts the live blocks
//   uint64_t  nodeKey[G][cap][2]               transposition key per node (TT rebuild after tree reuse)
//   float     policy[G][cap][P]                NN policy of the node (NNOutput::policyProbs)
//   uint32_t  freeList[G][cap], allocBits[G][cap/32]   node allocator
//   TT        ttKey[G][ttCap][2], ttNode[G][ttCap]     transposition table (searchnodetable.h)
//   SVB       svbKey/svbD/svbW[G][2][svbCap]           subtree value bias tables (double buffered)
//   float     accPolicy/rawPolicy/rootNoised[G][P]     root symmetry accumulation / noised prior
//   int32     pathNode/pathSlot[G][MAX_DEPTH]          the current playout's path
//   TurnRec   turns[G][maxTurns], int16 turnPol[G][maxTurns][P]  per-move records for rows
// Node indices are an allocator detail: results depend only on child-slot order,
// which is the reference's expansion order.
#pragma once
#include "kc_common.h"

namespace kc {

constexpr int MAX_DEPTH = MAX_AREA + 2;
// Child slots stored with the node (the selection's speculative first read); more
// children go to a block in the game's edge pool
constexpr int INLINE_EDGES = 16;
// Capacity of a node's pool block once it has k > INLINE_EDGES children: 48 (to 64
// slots in all) then P - 16 (reference growth 8 -> 64 -> P, searchnode.cpp:160-235).
KC_HD int edgeBlockCap(int k, int P) {
  return (P > 64 && k <= 64) ? 64 - INLINE_EDGES : P - INLINE_EDGES;
}
// Pool entries per buffer for node cap `cap`, bounded through the edges: a node with
// k > 16 children holds 48 entries (<= 48/17 per edge), or 48 + P - 16 once k > 64
// (the abandoned 48-block included: <= (32 + P)/65 per edge, 5.5 at 9x9).  Every edge
// is one expansion of a playout and leads to a node or, with graph search, to a
// transposition of one, so a tree holds about as many edges as nodes; the pool takes
// max(48/17, (32 + P)/65) entries for each of 1.5 x cap edges (half again for
// transposition edges) plus two root-sized blocks.  Measured use is far below (only
// nodes with more than 16 visits have more than 16 children): coffee_selfplay_stats
// reports the high-water mark.  Exhaustion is counted as a device error of its own
// (errors_edge_pool), like node-pool exhaustion; it never writes out of bounds.
inline int edgePoolCapFor(int cap, int P) {
  const double perEdge = (32.0 + P) / 65.0 > 48.0 / 17.0 ? (32.0 + P) / 65.0 : 48.0 / 17.0;
  return (int)(perEdge * 1.5 * cap) + 2 * P;
}
// GameDev::err codes (coffee_selfplay_stats.errors counts slots with any of them)
enum { ERR_NODE_POOL = 1, ERR_NO_CANDIDATE = 2, ERR_EDGE_POOL = 3 };
constexpr int MAX_LANE_ITEMS = (MAX_P + 63) / 64;  // 7

enum LeafKind {
  LEAF_NONE = 0,
  LEAF_NN = 1,
  LEAF_TERMINAL = 2,
  LEAF_CATCHUP = 3,
  LEAF_NOCHILD = 4,
  LEAF_ROOTEVAL = 5,
  LEAF_CACHED = 6,  // NN output taken from the evaluation cache (SPEC a7)
  LEAF_INIT = 7,    // policy-initialisation move: the root evaluated for a sampled opening move
  LEAF_FORK = 8,    // fork candidate: the position after one candidate move evaluated
  LEAF_SIDE = 9,    // side-position continuation: the position after the search's response
  // fused backup + select (kBackupSelect): the leaf's cache slot is being written by this
  // round's backups, so the lookup waits for kResolve (which runs after them)
  LEAF_PENDING = 10
};

// NN evaluation cache slot of a state key (SPEC a7; oracle ora_search.cpp cacheSlot).
KC_HD uint32_t cacheSlot(uint64_t k0, uint64_t k1, uint32_t mask) {
  const uint64_t h = k0 ^ ((k1 << 29) | (k1 >> 35));
  return (uint32_t)(h ^ (h >> 32)) & mask;
}
enum Phase { PH_ROOTEVAL = 0, PH_SEARCH = 1, PH_COMMIT = 2, PH_INIT = 3, PH_FORK = 4, PH_SIDEEVAL = 5 };

// SearchParams (searchparams.h) restricted to Coffee self-play.
struct SP {
  int maxVisits;
  float cpuct, cpuctLog, cpuctBase;
  float fpuRedMax, rootFpuRedMax, fpuLossProp, rootFpuLossProp;
  int fpuByVisited;
  float fpuByVisitedPow;
  float valueWeightExp;
  int rootNoise;
  float dirConc, dirWeight;
  float rootTemp, rootTempEarly;
  float rootDesiredCoeff;
  int rootSyms;
  float moveTemp, moveTempEarly, moveTempHalflife;
  float moveSubtract, movePrune;
  int useLcb;
  float lcbStdevs, minVisitPropLcb;
  float svbFactor, svbExp, svbFreeProp;
  int useGraph;
  // PlaySettings per-move limits and row weighting (play.cpp:871-1004, :1470-1697)
  float cheapProb;
  int cheapVisits;
  float cheapWeight;
  int reduceVisits;
  float reduceThreshold;
  int reduceLookback, reducedMin;
  float reducedWeight;
  float policySurpriseWeight, valueSurpriseWeight;
  int initPolicy;            // initGamesWithPolicy
  float initAreaProp, initTemp;  // policyInitAreaProp, policyInitAreaTemperature
  float earlyForkProb, earlyForkMoveProp, forkProb;  // earlyForkGameProb, earlyForkGameExpectedMoveProp, forkGameProb
  int forkMinChoices, earlyForkMaxChoices, forkMaxChoices;
  float sideProb;            // sidePositionProb
  int recordTree, recordTreeThreshold;  // recordTreePositions, recordTreeThreshold
  float recordTreeWeight;               // recordTreeTargetWeight
};

// The parameters of a cheap search whose rows are not recorded (runBotWithLimits
// removeRootNoise, play.cpp:1024-1037).
inline SP cheapSearchSP(const SP& p) {
  SP c = p;
  c.rootNoise = 0;
  c.rootTemp = 1.0f;
  c.rootTempEarly = 1.0f;
  c.rootFpuLossProp = p.fpuLossProp;
  c.rootFpuRedMax = p.fpuRedMax;
  c.rootDesiredCoeff = 0.0f;
  c.rootSyms = 1;
  return c;
}

struct Node {
  uint32_t visits;
  float weightSum, weightSqSum, utilityAvg, utilitySqAvg, winLossAvg;
  float nnWin, nnLoss;            // white-perspective NN probabilities
  float lastSvbDelta, lastSvbWeight;
  int32_t svbEntry;               // slot in the current SVB table, -1 none
  uint16_t numChildren;
  uint8_t nextPla;
  uint8_t flags;                  // 1 expanded (NN output stored), 2 terminal
  // next expansion of a non-root node: the legal move with the highest prior among
  // the unexpanded ones (ties: lower position), cached here so the selection reads it
  // with the node record: prior and policy position (0xFFFF: every legal move expanded)
  float nextPrior;
  uint16_t nextPos;
  uint16_t pad0;
  uint32_t edgeBase;              // the node's block of child slots >= INLINE_EDGES in the edge pool
  uint32_t pad1;
};
static_assert(sizeof(Node) == 64, "Node layout");

struct Edge {
  uint32_t child, visits;
  float prior;    // parent's NN prior of the move (root selection reads the noised root policy)
  uint32_t move;  // policy position dir*A + cell
};

// A finished game's move record (SGF output): header then the moves in order.
struct GameRec {
  int32_t slot, gameNum, numMoves, winner;  // winner 0 draw, 1 black, 2 white
  uint8_t cell[MAX_AREA], dir[MAX_AREA];
};

struct TurnRec {
  float whiteWin, whiteLoss, rawWhiteWL, rawPolicyEntropy;
  float policySurprise, policyEntropy, searchEntropy;
  uint32_t visits;
  float rootWL;                // getRootValues winLossValue (reduceVisits history)
  float rootNNWin, rootNNLoss; // getRootRawNNValues (value surprise)
  float targetWeight;          // limits.targetWeight, surprise-weighted at the game's end
  int8_t cell, dir;
  uint8_t rows;                // resolved integer weight: copies of this turn's row
  uint8_t gen;                 // network generation (hot reloads so far, mod 256) at the move's commit
  int8_t pad[4];
};
static_assert(sizeof(TurnRec) == 56, "TurnRec layout");

// Side positions (play.cpp:1328-1345, :1576-1662): at most MAX_SIDE per game are
// queued (a rare overflow drops the extra ones); each is searched after the game.
constexpr int MAX_SIDE = 8;

// Fork in progress (Play::maybeForkGame play.cpp:1741-1840): the position the
// finished game is replayed to and the candidate moves, evaluated one per round;
// the best becomes the start of the slot's next game.
constexpr int MAX_FORK_CHOICES = 100;
struct ForkRec {
  DBoard board;                    // the position before the fork move
  int32_t numChoices, next, best, prefix;  // prefix: moves replayed (kept as the next game's first turns)
  float bestWinrate;
  int32_t pad;
  uint16_t moves[MAX_FORK_CHOICES];  // candidate policy positions (dir * A + cell)
};

// A game finished by kCommit whose training rows kRows emits right after it.
struct FinRec {
  uint64_t rngSeed, rngCtr;  // history-mask stream state after the game's last move choice
  uint64_t gameHash0, gameHash1;
  unsigned long long rowBase;
  int32_t numMoves, winner, gameNum, pending;  // pending 1: rows reserved at rowBase
  int32_t numRows, startTurn;                  // startTurn: unsearched moves before the searched ones
  int32_t gameMode;
  int32_t genStart, genEnd;  // network generations at the game's start / end (rows' [49], [50])
  int32_t pad;
};

struct GameDev {
  DBoard root;
  DBoard leaf;
  uint64_t rngSeed, rngCtr;
  uint64_t gameHash0, gameHash1;
  uint64_t playouts, nnEvals, moves, gamesFinished;
  // measurement (SURVEY §8d tree roofline): tree levels descended and children
  // scanned at those levels, summed over this slot's descents
  uint64_t treeLevels, treeChildren;
  int32_t phase, rootK;
  uint32_t syms;                  // four root symmetries, 4 bits each
  int32_t cSlot;                  // NN-cache slot of the leaf (hit or bid)
  float cHitWin, cHitLoss;        // a cache hit's values, read by kSelect with the key
  int32_t noNoise;                // this move is a cheap search without recorded rows
  int32_t visitLimit;             // this move's maxVisits (getSearchLimitsThisMove)
  float moveWeight;               // this move's target weight
  int32_t initLeft;               // policy-initialisation moves still to play (PH_INIT)
  int32_t startTurn;              // unsearched opening moves (policy init or fork prefix): turns [0, startTurn) have no rows
  int32_t gameMode;               // FinishedGameData mode: 0 normal, 2 fork (trainingwrite.h:97-104)
  int32_t sideCount, sideNext;    // queued side positions of this game, the one being searched
  int32_t sideMode;               // 1 while the finished game's side positions are searched
  int32_t startDelay;             // rounds this slot idles before its first game (bench stagger)
  int32_t startGen;               // network generation when the game started
  int32_t leafKind, leafNode, leafSym, nnSlot;
  int32_t rootIdx, liveCount, freeTop, pathLen;
  int32_t gameNum, numTurns, svbSel, err;
  int32_t edgeSel, edgeTop;       // current edge-pool buffer, its first free slot
  int32_t edgePeak, pad0;         // edge-pool high-water mark (stats)
  float accWin, accLoss, rawWin, rawLoss;
};

// Device array pointer of SearchDev: on the device every access goes through a
// global-address-space pointer, so the compiler emits global_load/store (ordered,
// vmcnt-only waits) instead of flat accesses, which it must assume may hit LDS and
// drain with vmcnt(0) lgkmcnt(0).  Same layout as a raw pointer.
// (The empty asm keeps the generic->global->generic cast pair from being folded
// away, so address-space inference sees a global pointer.)
template <class T>
KC_HD T* asGlobal(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  __attribute__((address_space(1))) T* q = (__attribute__((address_space(1))) T*)p;
  asm volatile("" : "+s"(q));
  return (T*)q;
#else
  return p;
#endif
}
template <class T>
struct DPtr {
  T* p;
  DPtr() = default;
  KC_HD DPtr(T* q) : p(q) {}
  KC_HD operator T*() const { return asGlobal(p); }
  KC_HD T* operator->() const { return asGlobal(p); }
};

struct SearchDev {
  DPtr<const DTables> T;
  SP sp;
  SP spCheap;            // cheapSearchSP(sp): parameters of games with noNoise set
  int G, cap, ttCap, svbCap, P, A, inWords, maxTurns;
  int rowCap, slotBase;
  int startStagger;      // first games start after a per-slot delay in [0, startStagger) rounds
  DPtr<int32_t> modelGen;     // network generation: hot reloads so far (coffee_selfplay_set_model)
  uint64_t seed;
  DPtr<GameDev> games;
  DPtr<Node> nodes;
  DPtr<Edge> edges;           // [G][cap][INLINE_EDGES]
  DPtr<Edge> edgePool;        // [G][2][edgePoolCap]
  int edgePoolCap;
  DPtr<uint64_t> nodeKey;     // [G][cap][2] transposition key of each node (TT rebuild after reuse)
  DPtr<float> policy;
  DPtr<uint32_t> freeList;
  DPtr<uint32_t> allocBits;
  DPtr<uint64_t> ttKey;
  DPtr<int32_t> ttNode;
  DPtr<uint64_t> svbKey;
  DPtr<int64_t> svbD;
  DPtr<int64_t> svbW;
  DPtr<float> accPolicy;
  DPtr<float> rawPolicy;
  DPtr<float> rootNoised;
  DPtr<int32_t> pathNode;
  DPtr<int32_t> pathSlot;
  DPtr<TurnRec> turns;
  DPtr<int16_t> turnPol;
  // network batch
  DPtr<uint64_t> nnIn;        // [G][inWords]
  DPtr<float> nnOut;          // [G][P+4]
  DPtr<int32_t> nnNeed;       // [G] 1 when the game's row needs the network this round
  DPtr<int32_t> nnIdx;        // [G] compacted rows to evaluate (kCompact)
  DPtr<int32_t> nnCount;      // rows in nnIdx
  DPtr<int32_t> nnDefer;      // [G] 1: the row did not fit this round's batch (kCompact); the game waits
  DPtr<uint32_t> nnBid;       // [G] cache slot the row's evaluation bids for (~0u: none), kCompact bids
  int nnCap;             // rows per network launch (batch cap: one full wave of network workgroups)
  DPtr<int32_t> nnRR;         // round-robin start of the next batch (kCompact)
  DPtr<unsigned long long> nnTimedEvals;  // summed nnCount of the rounds whose network launch was timed
  // NN evaluation cache (SPEC a7): direct-mapped by state key, written between rounds
  uint32_t cacheMask;    // entries - 1 (0 with cacheOn == 0)
  int32_t cacheOn;
  DPtr<uint64_t> cKey;        // [entries][2]
  DPtr<float> cPol;           // [entries][P] post-processed policy (illegal = -1)
  DPtr<float> cVal;           // [entries][2] white win / loss
  DPtr<uint32_t> cTag;        // [entries] this round's highest bidding game + 1 (0 = none)
  DPtr<uint32_t> cClear;      // [G] fused rounds: slot + 1 whose tag kResolve clears (0 = none)
  DPtr<int32_t> pendList;     // [G] fused rounds: games whose cache lookup waits for kResolve (LEAF_PENDING)
  DPtr<int32_t> pendCount;    // entries in pendList (zeroed by the next kCompact)
  // commit queue
  DPtr<FinRec> fin;           // [G] games finished by the current commit (kRows)
  DPtr<ForkRec> fork;         // [G] fork state (PH_FORK)
  DPtr<DBoard> side;          // [G][MAX_SIDE] queued side positions
  DPtr<int16_t> sidePol;      // [G][P] the policy target of the side position being written
  DPtr<int32_t> commitList;   // [G]
  DPtr<int32_t> commitCount;
  // rows
  DPtr<uint8_t> rBin;         // [rowCap][15][pb]
  DPtr<float> rGlob;          // [rowCap]
  DPtr<int16_t> rPol;         // [rowCap][2][P]
  DPtr<float> rGt;            // [rowCap][64]
  DPtr<int8_t> rVal;          // [rowCap][5][A]
  DPtr<int32_t> rMeta;        // [rowCap][4]
  DPtr<unsigned long long> rCount;
  DPtr<unsigned long long> rDropped;
  DPtr<unsigned long long> rStaged;  // rows handed out by coffee_selfplay_stage_rows so far
  // finished-game records (drained by the host for SGF files)
  int gCap;
  DPtr<GameRec> gRec;               // [gCap]
  DPtr<unsigned long long> gCount;
  DPtr<unsigned long long> gDropped;
};

// Kernel launchers (search.hip).
void launchSelfplayInit(const SearchDev& d, const SearchDev* dd, hipStream_t st);
// e0/e1 (optional): events recorded at the kernel's start and end (hipExtLaunchKernel),
// so the bench times the kernel itself, not the stream gaps around it
// resetCommit: zero the commit count first (the previous commit consumed its list)
void launchSelect(const SearchDev& d, const SearchDev* dd, hipStream_t st, hipEvent_t e0 = nullptr,
                  hipEvent_t e1 = nullptr, bool resetCommit = false);
// accumulate: add the batch size to *d.nnTimedEvals (rounds whose network launch is timed)
// resolve: do launchResolve's work first, in the same dispatch (after launchBackupSelect)
void launchCompact(const SearchDev& d, const SearchDev* dd, hipStream_t st, bool accumulate, bool resolve = false);
// Packs the device row buffer's rows into dst ([rowCap][rowBytes], rows.py FIELDS order),
// copies their count to countOut (host, asynchronously) and empties the buffer (and the
// finished-game records when discardGames); stream-ordered, no host synchronisation.
void launchStageRows(const SearchDev& d, const SearchDev* dd, uint8_t* dst, unsigned long long* countOut,
                     bool discardGames, hipStream_t st);
int rowBytes(int A);  // bytes of one packed row at board area A
void launchBackup(const SearchDev& d, const SearchDev* dd, hipStream_t st, hipEvent_t e0 = nullptr,
                  hipEvent_t e1 = nullptr);
// One kernel for round r's backup and round r+1's selection of every game (no commit in
// between); the selections whose NN-cache slot this round's backups write are finished by
// launchResolve, which must run before the next launchCompact.
void launchBackupSelect(const SearchDev& d, const SearchDev* dd, hipStream_t st, hipEvent_t e0 = nullptr,
                        hipEvent_t e1 = nullptr);
void launchResolve(const SearchDev& d, const SearchDev* dd, hipStream_t st);
void launchCommit(const SearchDev& d, const SearchDev* dd, hipStream_t st);  // + kRows
void launchGameTree(const SearchDev* dd, int slot, int maxNodes, uint32_t* nodesOut, uint32_t* edgesOut,
                    int32_t* count, hipStream_t st);
// Dynamic LDS bytes the commit kernel needs for node_cap `cap`.
size_t commitLdsBytes(int cap);

}  // namespace kc
