// ORACLE (test infrastructure only) — MCTS + self-play restatement.  See ora.h.
#pragma once
#include <vector>

#include "ora.h"
#include "ora_math.h"

namespace ora {

// Arithmetic type of the search statistics and selection values: float (the device's
// SPEC restatement, the default) or double (-DORA_REAL=double, liboracle_f64.so: the
// reference's own precision, searchnode.h:18-44; used to measure how far the f32
// search drifts from f64 semantics, tests/test_f64_divergence.py).
#ifndef ORA_REAL
#define ORA_REAL float
#endif
typedef ORA_REAL real;

// SearchParams (searchparams.h) restricted to what Coffee self-play reads, with
// the values of cpp/configs/training/selfplay1.cfg (SURVEY §8d benchmark mode).
struct SearchParams {
  int maxVisits = 600;
  float cpuctExploration = 1.1f, cpuctExplorationLog = 0.0f, cpuctExplorationBase = 500.0f;
  float fpuReductionMax = 0.2f, rootFpuReductionMax = 0.0f, fpuLossProp = 0.0f, rootFpuLossProp = 0.0f;
  int fpuParentWeightByVisitedPolicy = 1;
  float fpuParentWeightByVisitedPolicyPow = 2.0f;
  float valueWeightExponent = 0.5f;
  int rootNoiseEnabled = 1;
  float rootDirichletNoiseTotalConcentration = 10.83f, rootDirichletNoiseWeight = 0.25f;
  float rootPolicyTemperature = 1.1f, rootPolicyTemperatureEarly = 1.25f;
  float rootDesiredPerChildVisitsCoeff = 2.0f;
  int rootNumSymmetriesToSample = 4;
  float chosenMoveTemperature = 0.15f, chosenMoveTemperatureEarly = 0.75f, chosenMoveTemperatureHalflife = 19.0f;
  float chosenMoveSubtract = 0.0f, chosenMovePrune = 1.0f;
  int useLcbForSelection = 1;
  float lcbStdevs = 5.0f, minVisitPropForLCB = 0.15f;
  float subtreeValueBiasFactor = 0.30f, subtreeValueBiasWeightExponent = 0.8f, subtreeValueBiasFreeProp = 0.8f;
  int useGraphSearch = 1;
  // PlaySettings (playsettings.cpp) per-move search limits and row weighting; the
  // defaults are benchmark mode, selfplay1.cfg values in comments
  float cheapSearchProb = 0.0f;          // 0.75
  int cheapSearchVisits = 100;           // 100
  float cheapSearchTargetWeight = 0.0f;  // 0.0
  int reduceVisits = 0;                  // true
  float reduceVisitsThreshold = 0.9f;    // 0.9
  int reduceVisitsThresholdLookback = 3; // 3
  int reducedVisitsMin = 100;            // 100
  float reducedVisitsWeight = 0.1f;      // 0.1
  float policySurpriseDataWeight = 0.0f; // 0.5
  float valueSurpriseDataWeight = 0.0f;  // 0.1
  int initGamesWithPolicy = 0;           // true
  float policyInitAreaProp = 0.04f;      // 0.04
  float policyInitAreaTemperature = 1.0f;
  float earlyForkGameProb = 0.0f;        // 0.04
  float earlyForkGameExpectedMoveProp = 0.025f;
  float forkGameProb = 0.0f;             // 0.01
  int forkGameMinChoices = 3, earlyForkGameMaxChoices = 12, forkGameMaxChoices = 36;
  float sidePositionProb = 0.0f;         // 0.02
  // recordTreePositions (play.cpp:710-860): PlaySettings fields the selfplay config
  // loader leaves at their defaults (playsettings.cpp:14)
  int recordTreePositions = 0;
  int recordTreeThreshold = 0;
  float recordTreeTargetWeight = 0.0f;
};

// The search parameters of a cheap search whose rows are not recorded
// (runBotWithLimits removeRootNoise, play.cpp:1024-1037).
inline SearchParams cheapSearchParams(const SearchParams& p) {
  SearchParams c = p;
  c.rootNoiseEnabled = 0;
  c.rootPolicyTemperature = 1.0f;
  c.rootPolicyTemperatureEarly = 1.0f;
  c.rootFpuLossProp = p.fpuLossProp;
  c.rootFpuReductionMax = p.fpuReductionMax;
  c.rootDesiredPerChildVisitsCoeff = 0.0f;
  c.rootNumSymmetriesToSample = 1;
  return c;
}

// Node record; identical fields and pool layout to the HIP engine so whole
// pools can be compared bit-for-bit.
struct Node {
  uint32_t visits;
  real weightSum, weightSqSum, utilityAvg, utilitySqAvg, winLossAvg;
  float nnWin, nnLoss;             // white-perspective NN probs (NNOutput::whiteWinProb/LossProb)
  real lastSvbDelta, lastSvbWeight;
  int32_t svbEntry;                // -1 none
  uint16_t numChildren;
  uint8_t nextPla;
  uint8_t flags;                   // 1 = expanded (has NN output), 2 = terminal
  uint64_t key0, key1;             // transposition key (stateHash)
};

enum LeafKind { LEAF_NONE = 0, LEAF_NN = 1, LEAF_TERMINAL = 2, LEAF_CATCHUP = 3, LEAF_NOCHILD = 4, LEAF_ROOTEVAL = 5,
               LEAF_CACHED = 6, LEAF_INIT = 7, LEAF_FORK = 8, LEAF_SIDE = 9 };
// PH_COMMIT: the root reached its visit limit (or a policy-init move ended the game) and
// the game idles until the next commit round (device kBackup -> kCommit every
// commit_interval rounds, selfplay.cpp SelfplayEngine::step)
enum Phase { PH_ROOTEVAL = 0, PH_SEARCH = 1, PH_COMMIT = 2, PH_INIT = 3, PH_FORK = 4, PH_SIDEEVAL = 5 };
constexpr int MAX_SIDE = 8;  // side positions queued per game (device search.h)

struct TurnRec {
  int8_t cell, dir;
  std::vector<int16_t> policyTarget;  // [P]
  float whiteWin, whiteLoss;          // extractValueTargets (play.cpp:674-682)
  float rawWhiteWL, rawPolicyEntropy; // computeNNRawStats (play.cpp:684-704)
  float policySurprise, policyEntropy, searchEntropy;
  uint32_t visits;
  float rootWL;                       // getRootValues winLossValue (reduceVisits history, play.cpp:1381-1384)
  float rootNNWin, rootNNLoss;        // getRootRawNNValues (value surprise, play.cpp:1336)
  float targetWeight;                 // limits.targetWeight, then surprise-weighted (play.cpp:1498-1574)
  int rows = 0;                       // resolved integer weight (play.cpp:1683-1697)
};

struct Rows {
  int n = 0;
  std::vector<uint8_t> bin;      // [n][15][(A+7)/8]
  std::vector<float> globIn;     // [n][1]
  std::vector<int16_t> policy;   // [n][2][P]
  std::vector<float> globT;      // [n][64]
  std::vector<int8_t> value;     // [n][5][A]
  std::vector<int32_t> meta;     // [n][4] slot, game number, turn, num moves
};

struct SelfplayCfg {
  Geom g;
  SearchParams sp;
  int nodeCap = 2048;
  uint64_t seed = 1;
  int slotBase = 0;        // global index of this engine's first game slot (rank * games)
  int nnMode = 0;          // 0 fake deterministic net, 1 model fp32, 2 model bf16-emulation,
                           // 3 external network (netFn; composition tests)
  const Model* model = nullptr;
  // nnMode 3: called once per round with the batch's packed V1 rows [n][ceil(15A/64)]
  // (coffee_encode_batch layout, batch order) and fills out [n][P+4] (coffee_nn_forward
  // layout).  Tests plug the device network in here, so the oracle's search consumes the
  // very outputs the device engine's network produces for the same rows.
  void (*netFn)(int n, const uint64_t* packed, float* out) = nullptr;
  int nnThreads = 1;
  int cacheLog2 = 0;       // NN evaluation cache of 2^cacheLog2 entries, 0 = off (SPEC a7)
  int nnCap = 1 << 30;     // rows per network batch; the rest wait for the next round (device kCompact)
  int parallelGames = 0;   // > 1: select / backup threads over games (CPU baseline only)
  // Round schedule of the device engine (coffee_selfplay_config): moves are committed
  // in rounds r with (r + 1) % commitInterval == 0 and in the last round of every
  // rounds() call (ora_sp_rounds); startStagger > 0: each slot idles a seeded number of
  // rounds in [0, startStagger) before its first game (the bench's staggered starts).
  int commitInterval = 1;
  int startStagger = 0;
};

struct Game {
  int slot = 0;
  uint32_t gameNum = 0;
  Rng rng;
  Board root;
  int phase = PH_ROOTEVAL, rootK = 0;
  int syms[4];
  std::vector<float> accPolicy;  // [P]
  float accWin = 0, accLoss = 0;
  std::vector<float> rawPolicy;  // first root eval (raw stats)
  float rawWin = 0, rawLoss = 0;
  // this move's search limits (getSearchLimitsThisMove play.cpp:871-1004)
  int visitLimit = 0, noNoise = 0;
  float moveWeight = 1.0f;
  // policy-initialisation moves (initializeGameUsingPolicy playutils.cpp:147-176);
  // startTurn: unsearched moves at the start (policy init or fork prefix)
  int initLeft = 0, startTurn = 0;
  int gameMode = 0;                  // 0 normal, 2 fork (trainingwrite.h:97-104)
  // fork in progress (Play::maybeForkGame play.cpp:1741-1840)
  Board forkBoard;
  std::vector<int> forkMoves;
  int forkNext = 0, forkBest = -1, forkPrefix = 0;
  float forkBestWinrate = 0.0f;
  // side positions (play.cpp:1328-1345, :1576-1662) queued during the game, searched after it
  std::vector<Board> side;
  int sideNext = 0, sideMode = 0;
  // tree
  int nodeCount = 0, rootIdx = -1;
  std::vector<Node> nodes;
  std::vector<uint32_t> edgeChild, edgeVisits;
  std::vector<uint16_t> edgeMove;
  std::vector<float> policy;     // [cap][P]
  std::vector<float> rootNoised; // [P]
  std::vector<uint64_t> ttKey0, ttKey1;
  std::vector<int32_t> ttNode;
  std::vector<uint64_t> svbKey;
  std::vector<int64_t> svbDelta, svbWeight;  // fixed point, 2^-32 units (SPEC B27)
  std::vector<uint8_t> svbUsed;
  // playout scratch
  int leafKind = LEAF_NONE, leafNode = -1, leafSym = 0, cacheSlot = 0;
  int nnDeferred = 0;      // the leaf missed the previous batch and waits for the network
  int startDelay = 0;      // rounds this slot still idles before its first game (startStagger)
  Board leafBoard;
  std::vector<int> pathNode, pathSlot;
  // game record
  std::vector<TurnRec> turns;
  uint64_t gameHash0 = 0, gameHash1 = 0;
  // counters
  uint64_t playouts = 0, nnEvals = 0, movesMade = 0, gamesFinished = 0;
};

struct Selfplay {
  SelfplayCfg cfg;
  SearchParams spCheap;        // cheapSearchParams(cfg.sp)
  std::vector<Game> games;
  std::vector<uint64_t> svbZ;  // SVB pattern zobrist (SPEC a19)
  Rows rows;
  uint64_t rounds = 0;
  // NN evaluation cache (nneval.h:18 NNCacheTable, restated as a direct-mapped table
  // written once per round; SPEC a7): key pair, postprocessed policy row, white win/loss
  std::vector<uint64_t> cacheKey;
  std::vector<float> cachePol, cacheVal;
  std::vector<float> nnBin, nnGlob;  // [G][15][A], [G]: each game's encoded leaf
  int nnRR = 0;                      // round-robin start of the next network batch
};

void selfplayInit(Selfplay& s, const SelfplayCfg& cfg, int numGames);
// One round = select for every game, one batched NN eval, backup for every game, then
// (commitNow) the moves of every game in PH_COMMIT.
void selfplayRound(Selfplay& s, bool commitNow = true);
// Sets the round schedule (before the first round): commit interval and start stagger.
void selfplaySchedule(Selfplay& s, int commitInterval, int startStagger);
// The deterministic stand-in network (analogue of nneval.cpp:442-500 debugSkipNeuralNet).
void fakeNet(const Geom& g, const float* bin, float* policy, float* value, float* misc);
void packPlanes(const Geom& g, const float* bin, uint64_t* words);

}  // namespace ora
