// Host self-play engine (selfplay.cpp) behind coffee_selfplay_*.
#pragma once
#include <functional>
#include <memory>
#include <vector>

#include "../../include/katacoffee.h"
#include "engine.h"
#include "search.h"

namespace kc {

SP toSP(const coffee_search_params& p);

class SelfplayEngine {
 public:
  explicit SelfplayEngine(const coffee_selfplay_config& c);
  ~SelfplayEngine();
  void step(int rounds, hipStream_t st);
  void sync();
  void stats(coffee_selfplay_stats& out);
  int drain(int maxRows, uint8_t* bin, float* glob, int16_t* pol, float* gt, int8_t* val, int32_t* meta);
  int drainGames(int maxGames, int32_t* header, uint8_t* moves);
  // Stream-ordered row hand-off (no host synchronisation): packs every pending row into
  // dst (device, >= rowCap rows), their count into *countOut (host, valid once the
  // engine stream passes this point) and empties the buffer.
  void stageRows(uint8_t* dst, int maxRows, unsigned long long* countOut, bool discardGames);
  hipStream_t stream() const { return stream_; }
  // Replaces the network for all subsequent rounds (all games: switchNetsMidGame).
  void setModel(const char* path);
  // The same from a CFNN image in host memory (weights broadcast from another rank).
  void setModelBytes(const void* data, size_t bytes);
  void gameInfo(int slot, int64_t* info);
  int gameTree(int slot, int maxNodes, uint32_t* nodes, uint32_t* edges);
  void rootPolicy(int slot, float* out);
  // every = 0: off; N: time every N-th launch of each kernel group (HIP events;
  // each event pair costs a few microseconds of stream gap, so sampling keeps
  // the timed run representative)
  void setTiming(int every) { timingEvery_ = every > 0 ? every : 0; }
  void kernelTime(int which, double& ms, uint64_t& launches);
  uint64_t timedNNEvals();
  const SearchDev& dev() const { return hd_; }
  bool nnFused() const { return nn_ && nn_->fused(); }

 private:
  struct PendingTiming {
    int which;
    hipEvent_t a, b;
  };
  void switchModel(const ModelHost& m);
  void timed(int which, hipStream_t st, const std::function<void()>& f, bool on);
  void timedKernel(int which, bool on, const std::function<void(hipEvent_t, hipEvent_t)>& f);
  bool sampleNow(int which) { return timingEvery_ > 0 && groupLaunches_[which]++ % (uint64_t)timingEvery_ == 0; }
  hipEvent_t takeEvent();
  void resolveTiming();
  std::vector<PendingTiming> pending_;
  std::vector<hipEvent_t> evPool_;
  const DTables* T_ = nullptr;
  std::unique_ptr<NNEngine> nn_;
  SearchDev hd_;
  SearchDev* dd_ = nullptr;
  std::vector<void*> owned_;
  hipStream_t stream_ = nullptr;
  int commitInterval_ = 8;
  int xLen_ = 0, yLen_ = 0, winLen_ = 0;
  int nnPath_ = 0;  // NNPath of the network (kept across hot reloads)
  int userCap_ = 0;          // coffee_selfplay_config.nn_batch_cap (0 = the network's default)
  int enginesPerDevice_ = 1; // engines sharing the device's default fused batch cap
  int cus_ = 1;              // compute units of the device
  int nnCapFor(int G) const;
  int32_t modelGen_ = 0;  // hot reloads so far
  uint64_t rounds_ = 0;
  bool commitReset_ = false;  // a commit ran: the next kSelect zeroes the commit count
  uint64_t rowsDrained_ = 0;
  int timingEvery_ = 0;
  // kernel timing slots: 0 select, 1 network, 2 backup, 3 commit, 4 backup + next select (fused)
  uint64_t groupLaunches_[5] = {0, 0, 0, 0, 0};
  double kernelMs_[5] = {0, 0, 0, 0, 0};
  uint64_t kernelLaunches_[5] = {0, 0, 0, 0, 0};
  // a round's backup and the next round's selection run as one kernel unless a commit
  // comes between them -- with the fast fused network or the stand-in (measured: with the
  // corrected network, which bounds the round, the longer-lived search waves delay its
  // workgroups: 202 vs 161 us).  COFFEE_FUSED_ROUNDS=0: never, 1: always (same results)
  int fuseRounds_ = -1;  // -1 auto, 0 never, 1 always
  bool fuseNow() const;
  // after a fused round the pending selections are completed and the round's cache tags
  // cleared by the compaction's own dispatch (kCompact resolve phase) instead of a separate
  // kResolve launch; COFFEE_SEPARATE_RESOLVE=1 keeps the separate launch (same results)
  bool resolveInCompact_ = true;
  // Audit of the default precision on self-play's own positions: every
  // auditEvery_-th network launch of an engine whose default precision resolved to the
  // corrected instance is re-evaluated (its first NN_AUDIT_ROWS rows) on the accurate
  // instance; sync() -- every stats / drain / game-record call -- reads the largest
  // difference so far and, past auditTol_ (NNEngine::NN_AUTO_TOL), rebuilds the network
  // at the accurate precision (same model; the NN cache is cleared).  The switch happens
  // only at those host synchronisation points, so runs stay reproducible.
  // COFFEE_NN_AUDIT_EVERY (0 = off) and COFFEE_NN_AUDIT_TOL override the defaults.
  void auditCheck();
  std::unique_ptr<ModelHost> model_;  // the network's model (rebuilt on an audit switch)
  float* auditOut_ = nullptr;         // device [G][P+4]: the accurate instance's rows
  unsigned* auditMax_ = nullptr;      // device: largest difference so far (float bits)
  int auditEvery_ = 128;
  float auditTol_ = NNEngine::NN_AUTO_TOL;
  uint64_t nnLaunches_ = 0;
  uint64_t audits_ = 0;
  float auditSeen_ = 0.0f;            // largest difference read back so far
  int auditSwitches_ = 0;
};

}  // namespace kc
