// C ABI (include/katacoffee.h): argument checking, error capture, dispatch.
// No C++ exception crosses this boundary; failures return COFFEE_E* with the
// message in coffee_last_error().
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>

#include "../../include/katacoffee.h"
#include "engine.h"
#include "model.h"
#include "npzwrite.h"
#include "selfplay.h"

namespace kc {

// ---- per-geometry table cache ----
namespace {
std::mutex gTablesMu;
std::map<std::tuple<int, int, int, int>, std::pair<DTables*, DTables*>> gTables;  // (dev,X,Y,W) -> host, device
}  // namespace

static std::pair<DTables*, DTables*> tablesFor(int X, int Y, int W) {
  int dev = 0;
  KC_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(gTablesMu);
  auto key = std::make_tuple(dev, X, Y, W);
  auto it = gTables.find(key);
  if(it != gTables.end())
    return it->second;
  DTables* h = new DTables(buildTables(X, Y, W));
  DTables* d = nullptr;
  KC_HIP(hipMalloc(&d, sizeof(DTables)));
  KC_HIP(hipMemcpy(d, h, sizeof(DTables), hipMemcpyHostToDevice));
  gTables[key] = {h, d};
  return {h, d};
}

const DTables* deviceTables(int X, int Y, int W) { return tablesFor(X, Y, W).second; }
const DTables& hostTables(int X, int Y, int W) { return *tablesFor(X, Y, W).first; }

}  // namespace kc

using namespace kc;

static thread_local std::string gLastError;

template <class F>
static int guarded(F&& f) {
  try {
    gLastError.clear();
    f();
    return COFFEE_OK;
  } catch(const HipError& e) {
    gLastError = e.what();
    return COFFEE_EHIP;
  } catch(const std::invalid_argument& e) {
    gLastError = e.what();
    return COFFEE_EINVAL;
  } catch(const InternalError& e) {
    gLastError = e.what();
    return COFFEE_EINTERNAL;
  } catch(const std::runtime_error& e) {
    gLastError = e.what();
    return COFFEE_EIO;
  } catch(const std::exception& e) {
    gLastError = e.what();
    return COFFEE_EINTERNAL;
  } catch(...) {
    gLastError = "unknown error";
    return COFFEE_EINTERNAL;
  }
}

static void need(bool ok, const char* what) {
  if(!ok)
    throw std::invalid_argument(what);
}

static void checkGeom(int x, int y, int w) {
  need(x >= 2 && y >= 2 && x <= MAX_LEN && y <= MAX_LEN, "board size must be 2..10 x 2..10");
  need(w >= 2 && w <= (x > y ? x : y), "win_len must be in 2..max(x, y)");
}

extern "C" {

const char* coffee_last_error(void) { return gLastError.c_str(); }
int coffee_abi_version(void) { return 108; }

int coffee_device_count(int* count) {
  return guarded([&] {
    need(count != nullptr, "count is NULL");
    KC_HIP(hipGetDeviceCount(count));
  });
}
int coffee_set_device(int device) {
  return guarded([&] { KC_HIP(hipSetDevice(device)); });
}
int coffee_device_compute_units(int device, int* cus) {
  return guarded([&] {
    need(cus != nullptr, "cus is NULL");
    KC_HIP(hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, device));
  });
}
int coffee_malloc(void** p, uint64_t bytes) {
  return guarded([&] {
    need(p != nullptr, "pointer is NULL");
    KC_HIP(hipMalloc(p, bytes ? bytes : 1));
  });
}
int coffee_free(void* p) {
  return guarded([&] { KC_HIP(hipFree(p)); });
}
int coffee_memcpy(void* dst, const void* src, uint64_t bytes, int kind) {
  return guarded([&] {
    need(kind >= 0 && kind <= 2, "kind must be 0, 1 or 2");
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
    KC_HIP(hipMemcpy(dst, src, bytes, k));
  });
}
int coffee_synchronize(void) {
  return guarded([&] { KC_HIP(hipDeviceSynchronize()); });
}

int coffee_rules_batch(int x, int y, int win_len, int n, const uint8_t* cells, const int8_t* last_cell,
                       const int8_t* last_dir, const uint8_t* pla, uint8_t* legal, uint8_t* has_legal, void* stream) {
  return guarded([&] {
    checkGeom(x, y, win_len);
    need(n >= 0, "n must be >= 0");
    need(n == 0 || (cells && last_cell && last_dir && pla && legal && has_legal), "NULL buffer");
    launchRulesBatch(deviceTables(x, y, win_len), n, cells, last_cell, last_dir, pla, legal, has_legal,
                     (hipStream_t)stream);
  });
}

int coffee_play_batch(int x, int y, int win_len, int n, const uint8_t* cells, const int8_t* last_cell,
                      const int8_t* last_dir, const uint8_t* pla, const int32_t* move, uint8_t* out_cells,
                      uint8_t* finished, uint8_t* winner, int32_t* max_run, uint64_t* pos_hash,
                      uint64_t* state_hash, void* stream) {
  return guarded([&] {
    checkGeom(x, y, win_len);
    need(n >= 0, "n must be >= 0");
    need(n == 0 || (cells && last_cell && last_dir && pla && move && out_cells && finished && winner && max_run &&
                    pos_hash && state_hash),
         "NULL buffer");
    launchPlayBatch(deviceTables(x, y, win_len), n, cells, last_cell, last_dir, pla, move, out_cells, finished,
                    winner, max_run, pos_hash, state_hash, (hipStream_t)stream);
  });
}

int coffee_encode_batch(int x, int y, int win_len, int n, const uint8_t* cells, const int8_t* hist_cell,
                        const int8_t* hist_dir, const uint8_t* pla, const int32_t* sym, uint64_t* packed,
                        float* planes, void* stream) {
  return guarded([&] {
    checkGeom(x, y, win_len);
    need(n >= 0, "n must be >= 0");
    need(n == 0 || (cells && hist_cell && hist_dir && pla && sym && packed), "NULL buffer");
    launchEncodeBatch(deviceTables(x, y, win_len), n, cells, hist_cell, hist_dir, pla, sym, packed, planes,
                      (hipStream_t)stream);
  });
}

int coffee_model_write_random(const char* arch, uint64_t seed, const char* path) {
  return guarded([&] {
    need(arch && path, "NULL argument");
    saveModel(path, randomModel(modelCfgByName(arch), seed));
  });
}

int coffee_model_flops(const char* path, int area, double* flops) {
  return guarded([&] {
    need(path && flops && area > 0, "bad argument");
    ModelHost m = loadModel(path);
    *flops = modelFlopsPerEval(m.cfg, area);
  });
}

struct coffee_nn {
  NNEngine* eng;
  int x, y, w;
};

int coffee_nn_create(const char* model_path, int x, int y, int win_len, coffee_nn** out) {
  return coffee_nn_create2(model_path, x, y, win_len, COFFEE_NN_DEFAULT, out);
}

int coffee_nn_create2(const char* model_path, int x, int y, int win_len, int precision, coffee_nn** out) {
  return guarded([&] {
    need(model_path && out, "NULL argument");
    need(precision >= COFFEE_NN_DEFAULT && precision <= COFFEE_NN_FAST, "unknown precision");
    checkGeom(x, y, win_len);
    ModelHost m = loadModel(model_path);
    (void)deviceTables(x, y, win_len);
    coffee_nn* h = new coffee_nn{nullptr, x, y, win_len};
    try {
      h->eng = new NNEngine(m, x, y, win_len, precision);
    } catch(...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int coffee_nn_forward(coffee_nn* h, int n, const uint64_t* in, float* out, void* stream) {
  return guarded([&] {
    need(h && h->eng, "NULL handle");
    need(n >= 0, "n must be >= 0");
    need(n == 0 || (in && out), "NULL buffer");
    h->eng->forward(n, in, out, (hipStream_t)stream);
  });
}

int coffee_nn_forward2(coffee_nn* h, int n, const uint64_t* in, const int32_t* sym, float* out, void* stream) {
  return guarded([&] {
    need(h && h->eng, "NULL handle");
    need(n >= 0, "n must be >= 0");
    need(n == 0 || (in && sym && out), "NULL buffer");
    h->eng->forward(n, in, out, (hipStream_t)stream);
    launchCanonicalRows(deviceTables(h->x, h->y, h->w), n, sym, out, (hipStream_t)stream);
  });
}

int coffee_nn_is_fused(coffee_nn* h, int* fused) {
  return guarded([&] {
    need(h && h->eng && fused, "NULL argument");
    *fused = h->eng->fused() ? 1 : 0;
  });
}

int coffee_nn_precision(coffee_nn* h, int* precision, float* calib_err) {
  return guarded([&] {
    need(h && h->eng && precision, "NULL argument");
    *precision = h->eng->precision();
    if(calib_err)
      *calib_err = h->eng->calibrationError();
  });
}

int coffee_nn_destroy(coffee_nn* h) {
  return guarded([&] {
    if(h) {
      delete h->eng;
      delete h;
    }
  });
}

int coffee_fake_net(int x, int y, int win_len, int n, const uint64_t* in, float* out, void* stream) {
  return guarded([&] {
    checkGeom(x, y, win_len);
    need(n >= 0, "n must be >= 0");
    need(n == 0 || (in && out), "NULL buffer");
    launchFakeNet(deviceTables(x, y, win_len), n, in, out, (hipStream_t)stream);
  });
}

void coffee_search_params_default(coffee_search_params* p) {
  if(!p)
    return;
  // cpp/configs/training/selfplay1.cfg (SURVEY §8d benchmark settings)
  p->max_visits = 600;
  p->cpuct_exploration = 1.1f;
  p->cpuct_exploration_log = 0.0f;
  p->cpuct_exploration_base = 500.0f;
  p->fpu_reduction_max = 0.2f;
  p->root_fpu_reduction_max = 0.0f;
  p->fpu_loss_prop = 0.0f;
  p->root_fpu_loss_prop = 0.0f;
  p->fpu_parent_weight_by_visited_policy = 1;
  p->fpu_parent_weight_by_visited_policy_pow = 2.0f;
  p->value_weight_exponent = 0.5f;
  p->root_noise_enabled = 1;
  p->root_dirichlet_noise_total_concentration = 10.83f;
  p->root_dirichlet_noise_weight = 0.25f;
  p->root_policy_temperature = 1.1f;
  p->root_policy_temperature_early = 1.25f;
  p->root_desired_per_child_visits_coeff = 2.0f;
  p->root_num_symmetries_to_sample = 4;
  p->chosen_move_temperature = 0.15f;
  p->chosen_move_temperature_early = 0.75f;
  p->chosen_move_temperature_halflife = 19.0f;
  p->chosen_move_subtract = 0.0f;
  p->chosen_move_prune = 1.0f;
  p->use_lcb_for_selection = 1;
  p->lcb_stdevs = 5.0f;
  p->min_visit_prop_for_lcb = 0.15f;
  p->subtree_value_bias_factor = 0.30f;
  p->subtree_value_bias_weight_exponent = 0.8f;
  p->subtree_value_bias_free_prop = 0.8f;
  p->use_graph_search = 1;
  // play settings: benchmark mode (one row per move at full visits)
  p->cheap_search_prob = 0.0f;
  p->cheap_search_visits = 100;
  p->cheap_search_target_weight = 0.0f;
  p->reduce_visits = 0;
  p->reduce_visits_threshold = 0.9f;
  p->reduce_visits_threshold_lookback = 3;
  p->reduced_visits_min = 100;
  p->reduced_visits_weight = 0.1f;
  p->policy_surprise_data_weight = 0.0f;
  p->value_surprise_data_weight = 0.0f;
  p->init_games_with_policy = 0;
  p->policy_init_area_prop = 0.04f;
  p->policy_init_area_temperature = 1.0f;
  p->early_fork_game_prob = 0.0f;
  p->early_fork_game_expected_move_prop = 0.025f;
  p->fork_game_prob = 0.0f;
  p->fork_game_min_choices = 3;
  p->early_fork_game_max_choices = 12;
  p->fork_game_max_choices = 36;
  p->side_position_prob = 0.0f;
  p->record_tree_positions = 0;
  p->record_tree_threshold = 0;
  p->record_tree_target_weight = 0.0f;
}

struct coffee_selfplay {
  SelfplayEngine* eng;
};

int coffee_selfplay_create(const coffee_selfplay_config* cfg, coffee_selfplay** out) {
  return guarded([&] {
    need(cfg && out, "NULL argument");
    checkGeom(cfg->x, cfg->y, cfg->win_len);
    coffee_selfplay* h = new coffee_selfplay{nullptr};
    try {
      h->eng = new SelfplayEngine(*cfg);
    } catch(...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int coffee_selfplay_step(coffee_selfplay* h, int rounds, void* stream) {
  return guarded([&] {
    need(h && h->eng, "NULL handle");
    need(rounds >= 0, "rounds must be >= 0");
    h->eng->step(rounds, (hipStream_t)stream);
  });
}

int coffee_selfplay_sync(coffee_selfplay* h) {
  return guarded([&] {
    need(h && h->eng, "NULL handle");
    h->eng->sync();
  });
}

int coffee_selfplay_stats_get(coffee_selfplay* h, coffee_selfplay_stats* out) {
  return guarded([&] {
    need(h && h->eng && out, "NULL argument");
    h->eng->stats(*out);
  });
}

int coffee_selfplay_drain_rows(coffee_selfplay* h, int max_rows, uint8_t* bin, float* glob, int16_t* pol,
                               float* gtgt, int8_t* value, int32_t* meta, int* n_out) {
  return guarded([&] {
    need(h && h->eng && n_out, "NULL argument");
    *n_out = h->eng->drain(max_rows, bin, glob, pol, gtgt, value, meta);
  });
}

int coffee_row_bytes(int x, int y, int* bytes) {
  return guarded([&] {
    need(bytes != nullptr, "NULL argument");
    need(x >= 2 && y >= 2 && x <= MAX_LEN && y <= MAX_LEN, "bad shape");
    *bytes = rowBytes(x * y);
  });
}

int coffee_selfplay_row_capacity(coffee_selfplay* h, int* rows) {
  return guarded([&] {
    need(h && h->eng && rows, "NULL argument");
    *rows = h->eng->dev().rowCap;
  });
}

int coffee_selfplay_stream(coffee_selfplay* h, void** stream) {
  return guarded([&] {
    need(h && h->eng && stream, "NULL argument");
    *stream = (void*)h->eng->stream();
  });
}

int coffee_selfplay_stage_rows(coffee_selfplay* h, void* dst, int max_rows, uint64_t* count, int flags) {
  return guarded([&] {
    need(h && h->eng && dst && count, "NULL argument");
    need((flags & ~COFFEE_STAGE_DISCARD_GAMES) == 0, "unknown flags");
    h->eng->stageRows((uint8_t*)dst, max_rows, (unsigned long long*)count, (flags & COFFEE_STAGE_DISCARD_GAMES) != 0);
  });
}

int coffee_selfplay_drain_games(coffee_selfplay* h, int max_games, int32_t* header, uint8_t* moves, int* n_out) {
  return guarded([&] {
    need(h && h->eng && n_out, "NULL argument");
    need(max_games >= 0, "max_games must be >= 0");
    *n_out = h->eng->drainGames(max_games, header, moves);
  });
}

int coffee_selfplay_set_model(coffee_selfplay* h, const char* model_path) {
  return guarded([&] {
    need(h && h->eng && model_path, "NULL argument");
    h->eng->setModel(model_path);
  });
}

int coffee_selfplay_set_model_bytes(coffee_selfplay* h, const void* data, uint64_t bytes) {
  return guarded([&] {
    need(h && h->eng && data, "NULL argument");
    h->eng->setModelBytes(data, (size_t)bytes);
  });
}

int coffee_selfplay_destroy(coffee_selfplay* h) {
  return guarded([&] {
    if(h) {
      delete h->eng;
      delete h;
    }
  });
}

int coffee_write_npz(const char* path, int n, int x, int y, const uint8_t* bin, const float* glob,
                     const int16_t* pol, const float* gtgt, const int8_t* value) {
  return guarded([&] {
    need(path != nullptr, "NULL path");
    need(n >= 0 && x >= 2 && y >= 2 && x <= MAX_LEN && y <= MAX_LEN, "bad shape");
    writeNpz(path, n, x, y, bin, glob, pol, gtgt, value);
  });
}

int coffee_selfplay_game_info(coffee_selfplay* h, int slot, int64_t* info) {
  return guarded([&] {
    need(h && h->eng && info, "NULL argument");
    h->eng->gameInfo(slot, info);
  });
}

int coffee_selfplay_game_tree(coffee_selfplay* h, int slot, int max_nodes, uint32_t* nodes, uint32_t* edges,
                              int* n_nodes) {
  return guarded([&] {
    need(h && h->eng && n_nodes, "NULL argument");
    *n_nodes = h->eng->gameTree(slot, max_nodes, nodes, edges);
  });
}

int coffee_selfplay_root_policy(coffee_selfplay* h, int slot, float* out) {
  return guarded([&] {
    need(h && h->eng && out, "NULL argument");
    h->eng->rootPolicy(slot, out);
  });
}

int coffee_debug_cdf_table(int x, int y, int win_len, float* out) {
  return guarded([&] {
    need(out != nullptr, "NULL argument");
    checkGeom(x, y, win_len);
    DTables t = buildTables(x, y, win_len);
    memcpy(out, t.cdf, sizeof(float) * CDF_SIZE);
  });
}

int coffee_debug_zobrist(int x, int y, int win_len, uint64_t* board, uint64_t* board2, uint64_t* player,
                         uint64_t* init, uint64_t* game_over) {
  return guarded([&] {
    need(board && board2 && player && init && game_over, "NULL argument");
    checkGeom(x, y, win_len);
    DTables t = buildTables(x, y, win_len);
    memcpy(board, t.zBoard, sizeof(uint64_t) * t.A * 3 * 2);
    memcpy(board2, t.zBoard2, sizeof(uint64_t) * t.A * 4 * 2);
    memcpy(player, t.zPlayer, sizeof(t.zPlayer));
    memcpy(init, t.zInit, sizeof(t.zInit));
    memcpy(game_over, t.zGameOver, sizeof(t.zGameOver));
  });
}

int coffee_selfplay_enable_timing(coffee_selfplay* h, int enable) {
  return guarded([&] {
    need(h && h->eng, "NULL handle");
    need(enable >= 0, "enable must be >= 0");
    h->eng->setTiming(enable);
  });
}

int coffee_selfplay_timed_nn_evals(coffee_selfplay* h, uint64_t* evals) {
  return guarded([&] {
    need(h && h->eng && evals, "NULL argument");
    *evals = h->eng->timedNNEvals();
  });
}

int coffee_selfplay_kernel_time(coffee_selfplay* h, int which, double* ms, uint64_t* launches) {
  return guarded([&] {
    need(h && h->eng && ms && launches, "NULL argument");
    h->eng->kernelTime(which, *ms, *launches);
  });
}

}  // extern "C"
