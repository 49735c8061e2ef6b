// Host side of the self-play engine: device allocation, the round loop and the
// row drain.  Replaces the reference's per-thread game loop (selfplay.cpp:262-330
// gameLoop, Play::runGame play.cpp:1146-1701) and NNEvaluator batching
// (nneval.cpp:386-567): all games advance together, one playout per round.
#include "selfplay.h"

#include <algorithm>
#include <cstring>

namespace kc {

static int nextPow2(int v) {
  int p = 1;
  while(p < v)
    p <<= 1;
  return p;
}

SP toSP(const coffee_search_params& p) {
  SP s;
  s.maxVisits = p.max_visits;
  s.cpuct = p.cpuct_exploration;
  s.cpuctLog = p.cpuct_exploration_log;
  s.cpuctBase = p.cpuct_exploration_base;
  s.fpuRedMax = p.fpu_reduction_max;
  s.rootFpuRedMax = p.root_fpu_reduction_max;
  s.fpuLossProp = p.fpu_loss_prop;
  s.rootFpuLossProp = p.root_fpu_loss_prop;
  s.fpuByVisited = p.fpu_parent_weight_by_visited_policy;
  s.fpuByVisitedPow = p.fpu_parent_weight_by_visited_policy_pow;
  s.valueWeightExp = p.value_weight_exponent;
  s.rootNoise = p.root_noise_enabled;
  s.dirConc = p.root_dirichlet_noise_total_concentration;
  s.dirWeight = p.root_dirichlet_noise_weight;
  s.rootTemp = p.root_policy_temperature;
  s.rootTempEarly = p.root_policy_temperature_early;
  s.rootDesiredCoeff = p.root_desired_per_child_visits_coeff;
  s.rootSyms = p.root_num_symmetries_to_sample;
  s.moveTemp = p.chosen_move_temperature;
  s.moveTempEarly = p.chosen_move_temperature_early;
  s.moveTempHalflife = p.chosen_move_temperature_halflife;
  s.moveSubtract = p.chosen_move_subtract;
  s.movePrune = p.chosen_move_prune;
  s.useLcb = p.use_lcb_for_selection;
  s.lcbStdevs = p.lcb_stdevs;
  s.minVisitPropLcb = p.min_visit_prop_for_lcb;
  s.svbFactor = p.subtree_value_bias_factor;
  s.svbExp = p.subtree_value_bias_weight_exponent;
  s.svbFreeProp = p.subtree_value_bias_free_prop;
  s.useGraph = p.use_graph_search;
  s.cheapProb = p.cheap_search_prob;
  s.cheapVisits = p.cheap_search_visits;
  s.cheapWeight = p.cheap_search_target_weight;
  s.reduceVisits = p.reduce_visits;
  s.reduceThreshold = p.reduce_visits_threshold;
  s.reduceLookback = p.reduce_visits_threshold_lookback;
  s.reducedMin = p.reduced_visits_min;
  s.reducedWeight = p.reduced_visits_weight;
  s.policySurpriseWeight = p.policy_surprise_data_weight;
  s.valueSurpriseWeight = p.value_surprise_data_weight;
  s.initPolicy = p.init_games_with_policy;
  s.initAreaProp = p.policy_init_area_prop;
  s.initTemp = p.policy_init_area_temperature;
  s.earlyForkProb = p.early_fork_game_prob;
  s.earlyForkMoveProp = p.early_fork_game_expected_move_prop;
  s.forkProb = p.fork_game_prob;
  s.forkMinChoices = p.fork_game_min_choices;
  s.earlyForkMaxChoices = p.early_fork_game_max_choices;
  s.forkMaxChoices = p.fork_game_max_choices;
  s.sideProb = p.side_position_prob;
  s.recordTree = p.record_tree_positions;
  s.recordTreeThreshold = p.record_tree_threshold;
  s.recordTreeWeight = p.record_tree_target_weight;
  return s;
}

// Bytes of one staged row (kStageRows; rows.py FIELDS): bin, glob, pol, gtgt, value, meta.
int rowBytes(int A) {
  const int pb = (A + 7) / 8;
  return NUM_SPATIAL * pb + 4 + 2 * 4 * A * 2 + 64 * 4 + 5 * A + 16;
}

// Dynamic LDS of the commit kernel (kCommit's policy scratch, live-node bits and BFS queue).
size_t commitLdsBytes(int cap) {
  size_t b = (size_t)MAX_P * 4 * 4 + 16;
  b += (size_t)(cap / 32) * 4 + (size_t)cap * 2;
  return (b + 15) / 16 * 16;
}

template <class T>
static T* devAlloc(std::vector<void*>& owned, size_t count, bool zero = true) {
  void* p = nullptr;
  size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  KC_HIP(hipMalloc(&p, bytes));
  owned.push_back(p);
  if(zero)
    KC_HIP(hipMemset(p, 0, bytes));
  return reinterpret_cast<T*>(p);
}

SelfplayEngine::SelfplayEngine(const coffee_selfplay_config& c) {
  if(c.num_games <= 0)
    throw std::invalid_argument("num_games must be positive");
  if(c.num_games > 65535)  // kCompact packs two per-device game counts into 16-bit halves
    throw std::invalid_argument("num_games must be <= 65535 per device");
  const coffee_search_params& sp = c.search;
  if(sp.max_visits < 1 || sp.root_num_symmetries_to_sample < 1 || sp.root_num_symmetries_to_sample > 4)
    throw std::invalid_argument("search params: max_visits >= 1 and 1 <= root_num_symmetries_to_sample <= 4");
  // the reference's own checks (play.cpp:906-910, :925-930)
  if(sp.cheap_search_prob > 0.0f && (sp.cheap_search_visits <= 0 || sp.cheap_search_visits > sp.max_visits))
    throw std::invalid_argument("cheap_search_visits must be in [1, max_visits]");
  if(sp.reduce_visits && (sp.reduced_visits_min <= 0 || sp.reduced_visits_min > sp.max_visits))
    throw std::invalid_argument("reduced_visits_min must be in [1, max_visits]");
  if(sp.reduce_visits && (sp.reduce_visits_threshold < 0.0f || sp.reduce_visits_threshold >= 1.0f ||
                          sp.reduce_visits_threshold_lookback < 1 || sp.reduce_visits_threshold_lookback > 100))
    throw std::invalid_argument("reduce_visits_threshold must be in [0, 1) and lookback in [1, 100]");
  // playsettings.cpp:80-99 ranges
  auto unit = [](float x) { return x >= 0.0f && x <= 1.0f; };
  if(!unit(sp.cheap_search_prob) || !unit(sp.cheap_search_target_weight) || !unit(sp.reduced_visits_weight) ||
     !unit(sp.policy_surprise_data_weight) || !unit(sp.value_surprise_data_weight) ||
     sp.policy_surprise_data_weight + sp.value_surprise_data_weight > 1.0f)
    throw std::invalid_argument("play settings: probabilities and weights in [0, 1], surprise weights sum <= 1");
  if(sp.init_games_with_policy && (!unit(sp.policy_init_area_prop) || sp.policy_init_area_temperature < 0.1f ||
                                   sp.policy_init_area_temperature > 5.0f))
    throw std::invalid_argument("policy_init_area_prop in [0, 1], policy_init_area_temperature in [0.1, 5]");
  // playsettings.cpp:74-79 ranges; play.cpp:1783-1788 checks
  if(sp.early_fork_game_prob < 0.0f || sp.early_fork_game_prob > 0.5f || sp.fork_game_prob < 0.0f ||
     sp.fork_game_prob > 0.5f || !unit(sp.early_fork_game_expected_move_prop) || sp.fork_game_min_choices < 1 ||
     sp.early_fork_game_max_choices < sp.fork_game_min_choices || sp.fork_game_max_choices < sp.fork_game_min_choices ||
     sp.early_fork_game_max_choices > MAX_FORK_CHOICES || sp.fork_game_max_choices > MAX_FORK_CHOICES)
    throw std::invalid_argument("fork settings: probabilities in [0, 0.5], min <= max choices <= 100");
  if(!unit(sp.side_position_prob))
    throw std::invalid_argument("side_position_prob must be in [0, 1]");
  // play.cpp:1349-1350
  if(sp.record_tree_positions && sp.record_tree_target_weight > 1.0f)
    throw std::invalid_argument("record_tree_target_weight > 1");
  const DTables& ht = hostTables(c.x, c.y, c.win_len);
  T_ = deviceTables(c.x, c.y, c.win_len);
  commitInterval_ = c.commit_interval > 0 ? c.commit_interval : 8;
  int cap = c.node_cap > 0 ? c.node_cap : std::max(2048, 3 * sp.max_visits);
  cap = (cap + 63) / 64 * 64;
  if(cap > 65535)
    throw std::invalid_argument("node_cap must be <= 65535");
  if(cap < sp.max_visits + 4)
    throw std::invalid_argument("node_cap must exceed max_visits + 3");
  const int G = c.num_games, P = ht.P, A = ht.A;
  const int ttCap = nextPow2(2 * cap);
  const int rowCap = c.row_capacity > 0 ? c.row_capacity : 4 * G * A;
  if(!c.use_fake_net) {
    if(!c.model_path)
      throw std::invalid_argument("model_path required unless use_fake_net");
    model_.reset(new ModelHost(loadModel(c.model_path)));
    nn_.reset(new NNEngine(*model_, c.x, c.y, c.win_len, c.nn_precision));
  }
  nnPath_ = c.nn_precision;
  xLen_ = c.x;
  yLen_ = c.y;
  winLen_ = c.win_len;
  SearchDev& d = hd_;
  memset(&d, 0, sizeof(d));
  d.T = T_;
  d.sp = toSP(sp);
  d.spCheap = cheapSearchSP(d.sp);
  d.G = G;
  d.cap = cap;
  d.ttCap = ttCap;
  d.svbCap = ttCap;
  d.P = P;
  d.A = A;
  d.inWords = ht.inWords;
  d.maxTurns = A + 1;
  d.rowCap = rowCap;
  d.slotBase = c.slot_base;
  if(c.start_stagger < 0)
    throw std::invalid_argument("start_stagger must be >= 0");
  d.startStagger = c.start_stagger;
  d.seed = c.seed;
  d.games = devAlloc<GameDev>(owned_, G);
  d.nodes = devAlloc<Node>(owned_, (size_t)G * cap, false);
  d.edges = devAlloc<Edge>(owned_, (size_t)G * cap * INLINE_EDGES, false);
  d.edgePoolCap = edgePoolCapFor(cap, P);
  d.edgePool = devAlloc<Edge>(owned_, (size_t)G * 2 * d.edgePoolCap, false);
  d.policy = devAlloc<float>(owned_, (size_t)G * cap * P, false);
  d.nodeKey = devAlloc<uint64_t>(owned_, (size_t)G * cap * 2, false);
  d.freeList = devAlloc<uint32_t>(owned_, (size_t)G * cap, false);
  d.allocBits = devAlloc<uint32_t>(owned_, (size_t)G * (cap / 32));
  d.ttKey = devAlloc<uint64_t>(owned_, (size_t)G * ttCap * 2, false);
  d.ttNode = devAlloc<int32_t>(owned_, (size_t)G * ttCap, false);
  d.svbKey = devAlloc<uint64_t>(owned_, (size_t)G * 2 * ttCap);
  d.svbD = devAlloc<int64_t>(owned_, (size_t)G * 2 * ttCap);
  d.svbW = devAlloc<int64_t>(owned_, (size_t)G * 2 * ttCap);
  d.accPolicy = devAlloc<float>(owned_, (size_t)G * P);
  d.rawPolicy = devAlloc<float>(owned_, (size_t)G * P);
  d.rootNoised = devAlloc<float>(owned_, (size_t)G * P);
  d.pathNode = devAlloc<int32_t>(owned_, (size_t)G * MAX_DEPTH);
  d.pathSlot = devAlloc<int32_t>(owned_, (size_t)G * MAX_DEPTH);
  d.turns = devAlloc<TurnRec>(owned_, (size_t)G * d.maxTurns);
  d.turnPol = devAlloc<int16_t>(owned_, (size_t)G * d.maxTurns * P);
  d.nnIn = devAlloc<uint64_t>(owned_, (size_t)G * ht.inWords);
  d.nnOut = devAlloc<float>(owned_, (size_t)G * (P + 4));
  d.fin = devAlloc<FinRec>(owned_, G);
  d.fork = devAlloc<ForkRec>(owned_, G);
  d.side = devAlloc<DBoard>(owned_, (size_t)G * MAX_SIDE);
  d.sidePol = devAlloc<int16_t>(owned_, (size_t)G * P);
  d.commitList = devAlloc<int32_t>(owned_, G);
  d.nnTimedEvals = devAlloc<unsigned long long>(owned_, 1);
  d.commitCount = devAlloc<int32_t>(owned_, 1);
  const int pb = (A + 7) / 8;
  d.rBin = devAlloc<uint8_t>(owned_, (size_t)rowCap * NUM_SPATIAL * pb, false);
  d.rGlob = devAlloc<float>(owned_, (size_t)rowCap, false);
  d.rPol = devAlloc<int16_t>(owned_, (size_t)rowCap * 2 * P, false);
  d.rGt = devAlloc<float>(owned_, (size_t)rowCap * 64, false);
  d.rVal = devAlloc<int8_t>(owned_, (size_t)rowCap * 5 * A, false);
  d.rMeta = devAlloc<int32_t>(owned_, (size_t)rowCap * 4, false);
  d.rCount = devAlloc<unsigned long long>(owned_, 1);
  d.rDropped = devAlloc<unsigned long long>(owned_, 1);
  d.rStaged = devAlloc<unsigned long long>(owned_, 1);
  d.nnNeed = devAlloc<int32_t>(owned_, G);
  d.nnDefer = devAlloc<int32_t>(owned_, G);
  d.nnBid = devAlloc<uint32_t>(owned_, G);
  d.nnRR = devAlloc<int32_t>(owned_, 1);
  if(c.nn_batch_cap < 0)
    throw std::invalid_argument("nn_batch_cap must be >= 0");
  if(c.engines_per_device < 0)
    throw std::invalid_argument("engines_per_device must be >= 0");
  userCap_ = c.nn_batch_cap;
  enginesPerDevice_ = std::max(1, c.engines_per_device);
  {
    int dev = 0;
    KC_HIP(hipGetDevice(&dev));
    KC_HIP(hipDeviceGetAttribute(&cus_, hipDeviceAttributeMultiprocessorCount, dev));
    cus_ = std::max(1, cus_);
  }
  d.nnCap = nnCapFor(G);
  d.nnIdx = devAlloc<int32_t>(owned_, G);
  d.modelGen = devAlloc<int32_t>(owned_, 1);
  d.nnCount = devAlloc<int32_t>(owned_, 1);
  if(c.nn_cache_log2 < 0 || c.nn_cache_log2 > 26)
    throw std::invalid_argument("nn_cache_log2 must be in 0..26");
  d.cacheOn = c.nn_cache_log2 > 0 ? 1 : 0;
  {
    const size_t entries = d.cacheOn ? (size_t)1 << c.nn_cache_log2 : 1;
    d.cacheMask = (uint32_t)(entries - 1);
    d.cKey = devAlloc<uint64_t>(owned_, entries * 2);  // zero key: never a state
    d.cPol = devAlloc<float>(owned_, entries * P, false);
    d.cVal = devAlloc<float>(owned_, entries * 2, false);
    d.cTag = devAlloc<uint32_t>(owned_, entries);
  }
  d.cClear = devAlloc<uint32_t>(owned_, G);
  d.pendList = devAlloc<int32_t>(owned_, G, false);
  d.pendCount = devAlloc<int32_t>(owned_, 1);
  {
    const char* f = getenv("COFFEE_FUSED_ROUNDS");
    fuseRounds_ = f && f[0] == '0' ? 0 : (f && f[0] == '1' ? 1 : -1);
    const char* r = getenv("COFFEE_SEPARATE_RESOLVE");
    resolveInCompact_ = !(r && r[0] == '1');
  }
  {
    const char* e = getenv("COFFEE_NN_AUDIT_EVERY");
    if(e)
      auditEvery_ = std::max(0, atoi(e));
    const char* t = getenv("COFFEE_NN_AUDIT_TOL");
    if(t)
      auditTol_ = (float)atof(t);
  }
  auditOut_ = devAlloc<float>(owned_, (size_t)G * (P + 4), false);
  auditMax_ = devAlloc<unsigned>(owned_, 1);
  d.gCap = 2 * G;
  d.gRec = devAlloc<GameRec>(owned_, (size_t)d.gCap, false);
  d.gCount = devAlloc<unsigned long long>(owned_, 1);
  d.gDropped = devAlloc<unsigned long long>(owned_, 1);
  dd_ = devAlloc<SearchDev>(owned_, 1);
  KC_HIP(hipMemcpy(dd_, &d, sizeof(SearchDev), hipMemcpyHostToDevice));
  KC_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  const size_t lds = commitLdsBytes(cap);
  if(lds > 64 * 1024)
    throw std::invalid_argument("node_cap too large for the commit kernel's LDS");
  launchSelfplayInit(d, dd_, stream_);
  KC_HIP(hipStreamSynchronize(stream_));
}

SelfplayEngine::~SelfplayEngine() {
  if(stream_)
    (void)hipStreamSynchronize(stream_);
  for(const PendingTiming& p : pending_) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for(hipEvent_t e : evPool_)
    (void)hipEventDestroy(e);
  nn_.reset();
  for(void* p : owned_)
    (void)hipFree(p);
  if(stream_)
    (void)hipStreamDestroy(stream_);
}

// Kernel timing: an event pair per launch on the launch stream, resolved later
// (no host synchronisation inside the round loop).
hipEvent_t SelfplayEngine::takeEvent() {
  if(evPool_.empty()) {
    hipEvent_t e;
    KC_HIP(hipEventCreate(&e));
    return e;
  }
  hipEvent_t e = evPool_.back();
  evPool_.pop_back();
  return e;
}

void SelfplayEngine::timed(int which, hipStream_t st, const std::function<void()>& f, bool on) {
  if(!on) {
    f();
    return;
  }
  hipEvent_t a = takeEvent(), b = takeEvent();
  KC_HIP(hipEventRecord(a, st));
  f();
  KC_HIP(hipEventRecord(b, st));
  pending_.push_back({which, a, b});
}

void SelfplayEngine::timedKernel(int which, bool on, const std::function<void(hipEvent_t, hipEvent_t)>& f) {
  if(!on) {
    f(nullptr, nullptr);
    return;
  }
  hipEvent_t a = takeEvent(), b = takeEvent();
  f(a, b);
  pending_.push_back({which, a, b});
}

void SelfplayEngine::resolveTiming() {
  for(const PendingTiming& p : pending_) {
    KC_HIP(hipEventSynchronize(p.b));
    float ms = 0.0f;
    KC_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    kernelMs_[p.which] += ms;
    kernelLaunches_[p.which]++;
    evPool_.push_back(p.a);
    evPool_.push_back(p.b);
  }
  pending_.clear();
}

bool SelfplayEngine::fuseNow() const {
  if(fuseRounds_ >= 0)
    return fuseRounds_ == 1;
  return !nn_ || (nn_->fused() && nn_->precision() == NN_FAST);
}

void SelfplayEngine::step(int rounds, hipStream_t st) {
  if(!st)
    st = stream_;
  const SearchDev& d = hd_;
  const bool fuse = fuseNow();
  bool selected = false;  // this round's selections ran in the previous round's fused kernel
  for(int r = 0; r < rounds; r++) {
    const bool t1 = sampleNow(1);
    // select, network and backup are timed by their own dispatches (kernel start to
    // end, like rocprofv3); compact and cache write run untimed between them
    if(selected) {
      if(!resolveInCompact_)
        launchResolve(d, dd_, st);  // the selections whose cache slot was being written
    } else {
      const bool t0 = sampleNow(0);
      timedKernel(0, t0, [&](hipEvent_t a, hipEvent_t b) { launchSelect(d, dd_, st, a, b, commitReset_); });
    }
    commitReset_ = false;
    launchCompact(d, dd_, st, t1, selected && resolveInCompact_);
    timedKernel(1, t1, [&](hipEvent_t a, hipEvent_t b) {
      const int rows = std::min(d.G, d.nnCap);  // grid bound; the batch is *d.nnCount rows
      if(nn_) {
        nn_->forward(rows, d.nnIn, d.nnOut, st, d.nnCount, d.nnIdx, a, b);
      } else {
        if(a)
          KC_HIP(hipEventRecord(a, st));
        launchFakeNet(T_, rows, d.nnIn, d.nnOut, st, d.nnCount, d.nnIdx);
        if(b)
          KC_HIP(hipEventRecord(b, st));
      }
    });
    if(nn_ && nnPath_ == NN_DEFAULT && auditEvery_ > 0 && nn_->precision() == NN_CORRECTED &&
       nnLaunches_++ % (uint64_t)auditEvery_ == 0) {
      nn_->audit(std::min(d.G, d.nnCap), d.nnIn, d.nnOut, auditOut_, auditMax_, st, d.nnCount, d.nnIdx);
      audits_++;
    }
    const bool commitNow = (rounds_ + 1) % (uint64_t)commitInterval_ == 0 || r == rounds - 1;
    if(fuse && !commitNow) {
      const bool t4 = sampleNow(4);
      timedKernel(4, t4, [&](hipEvent_t a, hipEvent_t b) { launchBackupSelect(d, dd_, st, a, b); });
      selected = true;
    } else {
      const bool t2 = sampleNow(2);
      timedKernel(2, t2, [&](hipEvent_t a, hipEvent_t b) { launchBackup(d, dd_, st, a, b); });
      selected = false;
    }
    rounds_++;
    if(commitNow) {
      const bool t3 = sampleNow(3);
      timed(3, st, [&] { launchCommit(d, dd_, st); }, t3);
      commitReset_ = true;  // the next kSelect zeroes the count (no separate memset)
    }
  }
}

void SelfplayEngine::sync() {
  KC_HIP(hipStreamSynchronize(stream_));
  resolveTiming();
  auditCheck();
}

void SelfplayEngine::auditCheck() {
  if(!nn_ || audits_ == 0)
    return;
  unsigned bits = 0;
  KC_HIP(hipMemcpy(&bits, auditMax_, 4, hipMemcpyDeviceToHost));
  float m;
  memcpy(&m, &bits, 4);
  auditSeen_ = std::max(auditSeen_, m);
  if(!(auditSeen_ <= auditTol_) && nn_->precision() == NN_CORRECTED && nnPath_ == NN_DEFAULT) {
    // the corrected instance missed the default precision's bound on self-play positions:
    // the same model on the accurate instance from here on (cached evaluations cleared)
    nn_.reset(new NNEngine(*model_, xLen_, yLen_, winLen_, NN_ACCURATE));
    auditSwitches_++;
    const int cap = nnCapFor(hd_.G);
    if(cap != hd_.nnCap) {
      hd_.nnCap = cap;
      KC_HIP(hipMemcpy(&dd_->nnCap, &cap, sizeof(int), hipMemcpyHostToDevice));
    }
    if(hd_.cacheOn)
      KC_HIP(hipMemsetAsync(hd_.cKey, 0, sizeof(uint64_t) * 2 * ((size_t)hd_.cacheMask + 1), stream_));
    KC_HIP(hipStreamSynchronize(stream_));
  }
}

void SelfplayEngine::stats(coffee_selfplay_stats& out) {
  sync();
  std::vector<GameDev> g(hd_.G);
  KC_HIP(hipMemcpy(g.data(), hd_.games, sizeof(GameDev) * hd_.G, hipMemcpyDeviceToHost));
  memset(&out, 0, sizeof(out));
  out.rounds = rounds_;
  for(const GameDev& x : g) {
    out.playouts += x.playouts;
    out.nn_evals += x.nnEvals;
    out.moves += x.moves;
    out.games_finished += x.gamesFinished;
    out.errors += x.err != 0 ? 1 : 0;
    out.errors_node_pool += x.err == ERR_NODE_POOL ? 1 : 0;
    out.errors_edge_pool += x.err == ERR_EDGE_POOL ? 1 : 0;
    out.edge_pool_peak = std::max<uint64_t>(out.edge_pool_peak, (uint64_t)x.edgePeak);
    out.tree_levels += x.treeLevels;
    out.tree_children += x.treeChildren;
  }
  unsigned long long cnt = 0, dropped = 0;
  KC_HIP(hipMemcpy(&cnt, hd_.rCount, 8, hipMemcpyDeviceToHost));
  KC_HIP(hipMemcpy(&dropped, hd_.rDropped, 8, hipMemcpyDeviceToHost));
  unsigned long long staged = 0;
  KC_HIP(hipMemcpy(&staged, hd_.rStaged, 8, hipMemcpyDeviceToHost));
  out.rows_pending = cnt;
  out.rows_written = rowsDrained_ + staged + cnt;
  out.rows_dropped = dropped;
  unsigned long long gdrop = 0;
  KC_HIP(hipMemcpy(&gdrop, hd_.gDropped, 8, hipMemcpyDeviceToHost));
  out.games_dropped = gdrop;
  out.edge_pool_cap = (uint64_t)hd_.edgePoolCap;
  out.nn_precision = nn_ ? (uint64_t)nn_->precision() : 0;
  out.nn_audits = audits_;
  out.nn_audit_switches = (uint64_t)auditSwitches_;
  out.nn_audit_max_diff = auditSeen_;
  if(out.errors)
    throw InternalError("self-play device invariant violated in " + std::to_string(out.errors) +
                        " game slot(s): " + std::to_string(out.errors_node_pool) + " node pool exhausted, " +
                        std::to_string(out.errors_edge_pool) + " edge pool exhausted, " +
                        std::to_string(out.errors - out.errors_node_pool - out.errors_edge_pool) +
                        " without a move candidate (raise node_cap)");
}

int SelfplayEngine::drain(int maxRows, uint8_t* bin, float* glob, int16_t* pol, float* gt, int8_t* val,
                          int32_t* meta) {
  sync();
  unsigned long long cnt = 0;
  KC_HIP(hipMemcpy(&cnt, hd_.rCount, 8, hipMemcpyDeviceToHost));
  const int n = (int)std::min<unsigned long long>(cnt, (unsigned long long)std::max(maxRows, 0));
  const int A = hd_.A, P = hd_.P, pb = (A + 7) / 8;
  auto cp = [&](void* dst, const void* src, size_t rowBytes) {
    if(dst && n > 0)
      KC_HIP(hipMemcpy(dst, src, rowBytes * n, hipMemcpyDeviceToHost));
  };
  cp(bin, hd_.rBin, (size_t)NUM_SPATIAL * pb);
  cp(glob, hd_.rGlob, 4);
  cp(pol, hd_.rPol, (size_t)2 * P * 2);
  cp(gt, hd_.rGt, 64 * 4);
  cp(val, hd_.rVal, (size_t)5 * A);
  cp(meta, hd_.rMeta, 16);
  if(n > 0 && (unsigned long long)n < cnt) {
    // keep the undrained tail at the front of the buffer, in chunks of n rows so
    // no copy's source overlaps its destination
    const size_t rest = cnt - n;
    auto mv = [&](void* base, size_t rowBytes) {
      for(size_t off = 0; off < rest; off += (size_t)n) {
        const size_t k = std::min(rest - off, (size_t)n);
        KC_HIP(hipMemcpy((char*)base + rowBytes * off, (char*)base + rowBytes * (n + off), rowBytes * k,
                         hipMemcpyDeviceToDevice));
      }
    };
    mv(hd_.rBin, (size_t)NUM_SPATIAL * pb);
    mv(hd_.rGlob, 4);
    mv(hd_.rPol, (size_t)2 * P * 2);
    mv(hd_.rGt, 256);
    mv(hd_.rVal, (size_t)5 * A);
    mv(hd_.rMeta, 16);
  }
  unsigned long long left = cnt - (unsigned long long)n;
  KC_HIP(hipMemcpy(hd_.rCount, &left, 8, hipMemcpyHostToDevice));
  rowsDrained_ += n;
  return n;
}

void SelfplayEngine::stageRows(uint8_t* dst, int maxRows, unsigned long long* countOut, bool discardGames) {
  if(maxRows < hd_.rowCap)
    throw std::invalid_argument("stage_rows: the destination must hold the row capacity (" +
                                std::to_string(hd_.rowCap) + " rows)");
  launchStageRows(hd_, dd_, dst, countOut, discardGames, stream_);
  // kernel timings whose events completed are folded in without waiting (a run that
  // never drains synchronously would otherwise keep every event pending)
  size_t keep = 0;
  for(size_t i = 0; i < pending_.size(); i++) {
    const PendingTiming& p = pending_[i];
    if(hipEventQuery(p.b) == hipSuccess) {
      float ms = 0.0f;
      KC_HIP(hipEventElapsedTime(&ms, p.a, p.b));
      kernelMs_[p.which] += ms;
      kernelLaunches_[p.which]++;
      evPool_.push_back(p.a);
      evPool_.push_back(p.b);
    } else {
      pending_[keep++] = p;
    }
  }
  pending_.resize(keep);
}

int SelfplayEngine::drainGames(int maxGames, int32_t* header, uint8_t* moves) {
  sync();
  unsigned long long cnt = 0;
  KC_HIP(hipMemcpy(&cnt, hd_.gCount, 8, hipMemcpyDeviceToHost));
  const int n = (int)std::min<unsigned long long>(cnt, (unsigned long long)std::max(maxGames, 0));
  if(n > 0) {
    std::vector<GameRec> recs(n);
    KC_HIP(hipMemcpy(recs.data(), hd_.gRec, sizeof(GameRec) * n, hipMemcpyDeviceToHost));
    const int A = hd_.A;
    for(int i = 0; i < n; i++) {
      const GameRec& r = recs[i];
      if(header) {
        header[4 * i + 0] = r.slot;
        header[4 * i + 1] = r.gameNum;
        header[4 * i + 2] = r.numMoves;
        header[4 * i + 3] = r.winner;
      }
      if(moves)
        for(int t = 0; t < A; t++) {
          moves[((size_t)i * A + t) * 2 + 0] = t < r.numMoves ? r.cell[t] : 0xFF;
          moves[((size_t)i * A + t) * 2 + 1] = t < r.numMoves ? r.dir[t] : 0xFF;
        }
    }
    const size_t rest = cnt - n;
    for(size_t off = 0; off < rest; off += (size_t)n) {
      const size_t k = std::min(rest - off, (size_t)n);
      KC_HIP(hipMemcpy(hd_.gRec + off, hd_.gRec + n + off, sizeof(GameRec) * k, hipMemcpyDeviceToDevice));
    }
  }
  unsigned long long left = cnt - (unsigned long long)n;
  KC_HIP(hipMemcpy(hd_.gCount, &left, 8, hipMemcpyHostToDevice));
  return n;
}

// Rows per network launch: the configured cap, else the network's own (one wave of
// fused workgroups, split between the engines sharing the device; the layered path is
// uncapped), never more than the games.
int SelfplayEngine::nnCapFor(int G) const {
  if(userCap_ > 0)
    return userCap_;
  if(!nn_)
    return std::min(G, cus_ * NN_BOARDS_PER_WG);
  if(!nn_->fused())
    return G;
  return std::min(G, nn_->batchCap(cus_, enginesPerDevice_));
}

void SelfplayEngine::setModel(const char* path) {
  if(!nn_)
    throw std::invalid_argument("engine runs the stand-in network (use_fake_net)");
  switchModel(loadModel(path));  // throws on a bad file; the current network stays
}

void SelfplayEngine::setModelBytes(const void* data, size_t bytes) {
  if(!nn_)
    throw std::invalid_argument("engine runs the stand-in network (use_fake_net)");
  switchModel(loadModelBytes(data, bytes, "<model bytes>"));
}

void SelfplayEngine::switchModel(const ModelHost& m) {
  std::unique_ptr<NNEngine> next(new NNEngine(m, xLen_, yLen_, winLen_, nnPath_));
  std::unique_ptr<ModelHost> keep(new ModelHost(m));
  sync();
  nn_ = std::move(next);
  model_ = std::move(keep);
  // the audit starts over for the new model
  auditSeen_ = 0.0f;
  KC_HIP(hipMemset(auditMax_, 0, 4));
  // a reload may change the network path (fused <-> layered) and with it the default cap
  const int cap = nnCapFor(hd_.G);
  if(cap != hd_.nnCap) {
    hd_.nnCap = cap;
    KC_HIP(hipMemcpy(&dd_->nnCap, &cap, sizeof(int), hipMemcpyHostToDevice));
  }
  // network generation: rows of games that span the switch carry it in [49] / [50]
  // (ChangedNeuralNet, play.cpp:1210-1226; trainingwrite.cpp:459-461)
  modelGen_++;
  KC_HIP(hipMemcpy(hd_.modelGen, &modelGen_, sizeof(int32_t), hipMemcpyHostToDevice));
  // cached evaluations belong to the previous network (the reference builds a new
  // NNEvaluator, and with it a new cache, per model: cpp/command/selfplay.cpp:150-200)
  if(hd_.cacheOn)
    KC_HIP(hipMemsetAsync(hd_.cKey, 0, sizeof(uint64_t) * 2 * ((size_t)hd_.cacheMask + 1), stream_));
}

void SelfplayEngine::gameInfo(int slot, int64_t* info) {
  if(slot < 0 || slot >= hd_.G)
    throw std::invalid_argument("slot out of range");
  sync();
  GameDev g;
  KC_HIP(hipMemcpy(&g, hd_.games + slot, sizeof(GameDev), hipMemcpyDeviceToHost));
  int64_t v[16] = {g.phase, g.rootK, g.liveCount, g.rootIdx, g.gameNum, g.root.turn, g.root.pla,
                   g.root.finished, g.root.winner, (int64_t)g.playouts, (int64_t)g.nnEvals, (int64_t)g.moves,
                   (int64_t)g.gamesFinished, g.root.lastCell, g.root.lastDir, (int64_t)g.rngCtr};
  memcpy(info, v, sizeof(v));
}

int SelfplayEngine::gameTree(int slot, int maxNodes, uint32_t* nodes, uint32_t* edges) {
  if(slot < 0 || slot >= hd_.G || maxNodes <= 0)
    throw std::invalid_argument("slot/max_nodes out of range");
  sync();
  std::vector<void*> tmp;
  // zeroed on the engine stream: a null-stream hipMemset is not ordered before work
  // on the non-blocking engine stream
  uint32_t* dn = devAlloc<uint32_t>(tmp, (size_t)maxNodes * 24, false);
  uint32_t* de = devAlloc<uint32_t>(tmp, (size_t)maxNodes * hd_.P * 3, false);
  int32_t* dc = devAlloc<int32_t>(tmp, 1, false);
  KC_HIP(hipMemsetAsync(dn, 0, (size_t)maxNodes * 24 * 4, stream_));
  KC_HIP(hipMemsetAsync(de, 0, (size_t)maxNodes * hd_.P * 3 * 4, stream_));
  KC_HIP(hipMemsetAsync(dc, 0, 4, stream_));
  launchGameTree(dd_, slot, maxNodes, dn, de, dc, stream_);
  KC_HIP(hipStreamSynchronize(stream_));
  int n = 0;
  KC_HIP(hipMemcpy(&n, dc, 4, hipMemcpyDeviceToHost));
  if(nodes)
    KC_HIP(hipMemcpy(nodes, dn, (size_t)maxNodes * 24 * 4, hipMemcpyDeviceToHost));
  if(edges)
    KC_HIP(hipMemcpy(edges, de, (size_t)maxNodes * hd_.P * 3 * 4, hipMemcpyDeviceToHost));
  for(void* p : tmp)
    (void)hipFree(p);
  return n;
}

void SelfplayEngine::rootPolicy(int slot, float* out) {
  if(slot < 0 || slot >= hd_.G)
    throw std::invalid_argument("slot out of range");
  sync();
  KC_HIP(hipMemcpy(out, hd_.rootNoised + (size_t)slot * hd_.P, sizeof(float) * hd_.P, hipMemcpyDeviceToHost));
}

uint64_t SelfplayEngine::timedNNEvals() {
  sync();
  unsigned long long v = 0;
  KC_HIP(hipMemcpy(&v, hd_.nnTimedEvals, 8, hipMemcpyDeviceToHost));
  return v;
}

void SelfplayEngine::kernelTime(int which, double& ms, uint64_t& launches) {
  resolveTiming();
  if(which < 0 || which > 4)
    throw std::invalid_argument("which must be 0..4");
  ms = kernelMs_[which];
  launches = kernelLaunches_[which];
}

}  // namespace kc
