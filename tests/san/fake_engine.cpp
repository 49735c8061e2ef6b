// A host-only stand-in of the self-play C ABI (include/katacoffee.h) for ThreadSanitizer
// runs of the host programs' threads (tests/test_sanitizers.py): the CLI
// (csrc/cli_selfplay.cpp: one thread per engine, the shared models-directory watch, the
// game counter, the log) and bench_writer.cpp (bench.py's engine loop + .npz writer
// thread).  No GPU: "engines" produce deterministic rows and game records at a fixed
// rate per round; coffee_write_npz is the product's own writer (csrc/npzwrite.cpp).
// Like the real library it keeps a per-thread device and error string and one
// process-wide, mutex-guarded cache (the real one caches device tables per geometry).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <sys/stat.h>
#include <thread>

#include "../../include/katacoffee.h"
#include "../../katacoffee_amd/csrc/npzwrite.h"

static thread_local std::string tLastError;
static thread_local int tDevice = 0;
static std::mutex gGeomMu;
static std::map<int, int> gGeomUsers;  // geometry key -> engines using it

struct coffee_selfplay {
  coffee_selfplay_config cfg;
  std::string model;
  int device;
  uint64_t rounds = 0, moves = 0, games = 0, rowsMade = 0, rowsDrained = 0, gamesDrained = 0;
};

static int fail(const char* what) {
  tLastError = what;
  return COFFEE_EINVAL;
}

extern "C" {
const char* coffee_last_error(void) { return tLastError.c_str(); }
int coffee_device_count(int* count) {
  const char* e = getenv("FAKE_DEVICES");
  *count = e ? atoi(e) : 2;
  return COFFEE_OK;
}
int coffee_set_device(int device) {
  tDevice = device;
  return COFFEE_OK;
}
int coffee_device_compute_units(int, int* cus) {
  *cus = 256;
  return COFFEE_OK;
}
void coffee_search_params_default(coffee_search_params* p) {
  memset(p, 0, sizeof(*p));
  p->max_visits = 600;
}
int coffee_selfplay_create(const coffee_selfplay_config* cfg, coffee_selfplay** out) {
  struct stat st;
  if(!cfg || !out || cfg->num_games <= 0 || !cfg->model_path || stat(cfg->model_path, &st) != 0)
    return fail("bad config or model");
  coffee_selfplay* h = new coffee_selfplay;
  h->cfg = *cfg;
  h->model = cfg->model_path;
  h->device = tDevice;
  std::lock_guard<std::mutex> lk(gGeomMu);
  gGeomUsers[cfg->x * 100 + cfg->y]++;
  *out = h;
  return COFFEE_OK;
}
int coffee_selfplay_step(coffee_selfplay* h, int rounds, void*) {
  if(!h || rounds < 0)
    return fail("bad step");
  h->rounds += rounds;
  // one move per game every 50 rounds, a game end every 12 moves (one row per move)
  const uint64_t moves = h->rounds * h->cfg.num_games / 50;
  const uint64_t games = moves / 12;
  h->rowsMade += (games - h->games) * 12;
  h->moves = moves;
  h->games = games;
  std::this_thread::sleep_for(std::chrono::microseconds(200));
  return COFFEE_OK;
}
int coffee_selfplay_sync(coffee_selfplay*) { return COFFEE_OK; }
int coffee_selfplay_drain_rows(coffee_selfplay* h, int max_rows, uint8_t* bin, float* glob, int16_t* pol,
                               float* gt, int8_t* val, int32_t* meta, int* n_out) {
  const int A = h->cfg.x * h->cfg.y, pb = (A + 7) / 8, P = 4 * A;
  const uint64_t avail = h->rowsMade - h->rowsDrained;
  const int n = (int)(avail < (uint64_t)max_rows ? avail : (uint64_t)max_rows);
  for(int i = 0; i < n; i++) {
    const uint64_t r = h->rowsDrained + i;
    if(bin)
      memset(bin + (size_t)i * 15 * pb, (int)(r & 0xff), (size_t)15 * pb);
    if(glob)
      glob[i] = (float)h->cfg.win_len;
    if(pol)
      for(int k = 0; k < 2 * P; k++)
        pol[(size_t)i * 2 * P + k] = (int16_t)((r + k) % 7);
    if(gt)
      for(int k = 0; k < 64; k++)
        gt[(size_t)i * 64 + k] = k == 63 ? 1.0f : 0.0f;
    if(val)
      memset(val + (size_t)i * 5 * A, 0, (size_t)5 * A);
    if(meta) {
      meta[4 * i] = h->cfg.slot_base + (int)(r % h->cfg.num_games);
      meta[4 * i + 1] = (int)(r / 12);
      meta[4 * i + 2] = (int)(r % 12);
      meta[4 * i + 3] = 0;
    }
  }
  h->rowsDrained += n;
  *n_out = n;
  return COFFEE_OK;
}
int coffee_selfplay_drain_games(coffee_selfplay* h, int max_games, int32_t* hdr, uint8_t* mv, int* n_out) {
  const int A = h->cfg.x * h->cfg.y;
  const uint64_t avail = h->games - h->gamesDrained;
  const int n = (int)(avail < (uint64_t)max_games ? avail : (uint64_t)max_games);
  for(int i = 0; i < n; i++) {
    const uint64_t g = h->gamesDrained + i;
    if(hdr) {
      hdr[4 * i] = h->cfg.slot_base + (int)(g % h->cfg.num_games);
      hdr[4 * i + 1] = (int)g;
      hdr[4 * i + 2] = 12 < A ? 12 : A;
      hdr[4 * i + 3] = (int)(g % 3);
    }
    if(mv)
      for(int t = 0; t < A; t++) {
        mv[((size_t)i * A + t) * 2] = (uint8_t)(t < 12 ? t : 0xff);
        mv[((size_t)i * A + t) * 2 + 1] = (uint8_t)(t < 12 ? t % 4 : 0xff);
      }
  }
  h->gamesDrained += n;
  *n_out = n;
  return COFFEE_OK;
}
int coffee_selfplay_set_model(coffee_selfplay* h, const char* path) {
  struct stat st;
  if(!h || !path || stat(path, &st) != 0)
    return fail("cannot load model");
  h->model = path;
  return COFFEE_OK;
}
int coffee_selfplay_stats_get(coffee_selfplay* h, coffee_selfplay_stats* out) {
  memset(out, 0, sizeof(*out));
  out->rounds = h->rounds;
  out->playouts = h->rounds * h->cfg.num_games;
  out->moves = h->moves;
  out->games_finished = h->games;
  out->rows_written = h->rowsMade;
  out->rows_pending = h->rowsMade - h->rowsDrained;
  return COFFEE_OK;
}
int coffee_selfplay_destroy(coffee_selfplay* h) {
  {
    std::lock_guard<std::mutex> lk(gGeomMu);
    gGeomUsers[h->cfg.x * 100 + h->cfg.y]--;
  }
  delete h;
  return COFFEE_OK;
}
int coffee_write_npz(const char* path, int n, int x, int y, const uint8_t* bin, const float* glob,
                     const int16_t* pol, const float* gt, const int8_t* val) {
  if(!path || n < 0)
    return fail("bad npz arguments");
  kc::writeNpz(path, n, x, y, bin, glob, pol, gt, val);
  return COFFEE_OK;
}
}
