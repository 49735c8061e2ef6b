// `katago selfplay` for Coffee on MI355X: the process-level boundary of the hot path
// (command/selfplay.cpp:44-72 flags, :83-250 output layout).  Host C++ over the C ABI.
//
//   katago selfplay -config <cfg> -models-dir <dir> -output-dir <dir>
//                   [-max-games-total N] [-override-config k=v,k=v,...]
//
// Reads KataGo-style `key = value` config files (selfplay1.cfg keys that apply to this
// path, plus `winLen`, `numGpus`, `boardXLen`/`boardYLen`; `bSizes` first entry sets a
// square board).  Uses the newest model file in -models-dir (CFNN v1) and polls the
// directory every `modelPollSeconds` (default 10): a newer file is loaded into every
// engine and used by all games from their next round on (hot reload with
// switchNetsMidGame semantics, selfplay.cpp:135-260 / :366-384).  Writes
// <output-dir>/<modelName>/tdata/<hex>.npz (maxRowsPerTrainFile rows each, reference
// layout), <output-dir>/<modelName>/sgfs/<hex>.sgfs (one SGF per finished game per
// line, sgf.cpp:1526-1700 with Coffee's 3-letter moves, selfplaymanager.cpp:350-354)
// and <output-dir>/log<time>.log.  Rows and games drained after a switch go to the new
// model's directories.  Each GPU plays games [gpu*numGameThreads, (gpu+1)*numGameThreads)
// on ceil(numNNServerThreadsPerModel / numGpus) engines (default 1; 2 overlaps one
// engine's network with the other's search, +8 % rows/s at C2), each on its own thread
// writing its own files (SURVEY §8e fallback, no collective).  SIGINT/SIGTERM: flush
// rows and exit.
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/katacoffee.h"
#include "cli_config.h"

using namespace kccli;

static std::atomic<bool> gStop(false);
static void onSignal(int) { gStop = true; }

static std::mutex gLogMu;
static FILE* gLog = nullptr;
static void logf(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lk(gLogMu);
  time_t t = time(nullptr);
  char ts[32];
  strftime(ts, sizeof(ts), "%Y-%m-%d %H:%M:%S", localtime(&t));
  fprintf(stdout, "%s: %s\n", ts, buf);
  fflush(stdout);
  if(gLog) {
    fprintf(gLog, "%s: %s\n", ts, buf);
    fflush(gLog);
  }
}

static void die(const std::string& msg) {
  fprintf(stderr, "katago selfplay: %s\n", msg.c_str());
  exit(1);
}

static void check(int rc, const char* what) {
  if(rc != COFFEE_OK)
    die(std::string(what) + ": " + coffee_last_error());
}

// Newest regular file in dir ("" if none); its mtime in *mt.
static std::string newestModelOrEmpty(const std::string& dir, time_t* mt) {
  DIR* d = opendir(dir.c_str());
  if(!d)
    return "";
  std::string best;
  time_t bestT = 0;
  while(dirent* e = readdir(d)) {
    if(e->d_name[0] == '.')
      continue;
    std::string p = dir + "/" + e->d_name;
    struct stat st;
    if(stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode) && (best.empty() || st.st_mtime > bestT)) {
      best = p;
      bestT = st.st_mtime;
    }
  }
  closedir(d);
  if(mt)
    *mt = bestT;
  return best;
}

static std::string newestModel(const std::string& dir) {
  const std::string m = newestModelOrEmpty(dir, nullptr);
  if(m.empty())
    die("no model file in " + dir);
  return m;
}

static std::string modelNameOf(const std::string& path) {
  std::string n = path.substr(path.find_last_of('/') + 1);
  return n.find('.') != std::string::npos ? n.substr(0, n.find('.')) : n;
}

// The models directory as seen by all GPU threads: version bumps when a newer file
// (path or mtime) appears; each thread switches when its version lags.
struct ModelWatch {
  std::mutex mu;
  std::string dir, path;
  time_t mtime = 0;
  int version = 0;
  double pollSeconds = 10.0;
  std::chrono::steady_clock::time_point lastPoll = std::chrono::steady_clock::now();

  void current(std::string& p, int& v) {
    std::lock_guard<std::mutex> lk(mu);
    const auto now = std::chrono::steady_clock::now();
    if(std::chrono::duration<double>(now - lastPoll).count() >= pollSeconds) {
      lastPoll = now;
      time_t mt = 0;
      const std::string np = newestModelOrEmpty(dir, &mt);
      if(!np.empty() && (np != path || mt > mtime)) {
        path = np;
        mtime = mt;
        version++;
        logf("models dir: new model %s", path.c_str());
      }
    }
    p = path;
    v = version;
  }
};
static ModelWatch gModels;

static void mkdirs(const std::string& path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if(!path.empty() && path[0] == '/')
    cur = "/";
  while(std::getline(ss, part, '/')) {
    if(part.empty())
      continue;
    cur += part + "/";
    mkdir(cur.c_str(), 0755);
  }
}

struct RowSink {
  std::string dir;
  int x, y, maxRows;
  std::mt19937_64 rng;
  std::vector<uint8_t> bin;
  std::vector<float> glob, gt;
  std::vector<int16_t> pol;
  std::vector<int8_t> val;
  int n = 0;
  int64_t filesWritten = 0, rowsWritten = 0;

  void append(int k, const uint8_t* b, const float* g, const int16_t* p, const float* t, const int8_t* v) {
    const int A = x * y, pb = (A + 7) / 8;
    bin.insert(bin.end(), b, b + (size_t)k * 15 * pb);
    glob.insert(glob.end(), g, g + k);
    pol.insert(pol.end(), p, p + (size_t)k * 2 * 4 * A);
    gt.insert(gt.end(), t, t + (size_t)k * 64);
    val.insert(val.end(), v, v + (size_t)k * 5 * A);
    n += k;
  }
  void flush(bool all) {
    const int A = x * y, pb = (A + 7) / 8, P = 4 * A;
    while(n >= maxRows || (all && n > 0)) {
      int k = n < maxRows ? n : maxRows;
      char name[64];
      snprintf(name, sizeof(name), "%016llX.npz", (unsigned long long)rng());
      std::string path = dir + "/" + name;
      check(coffee_write_npz(path.c_str(), k, x, y, bin.data(), glob.data(), pol.data(), gt.data(), val.data()),
            "write npz");
      bin.erase(bin.begin(), bin.begin() + (size_t)k * 15 * pb);
      glob.erase(glob.begin(), glob.begin() + k);
      pol.erase(pol.begin(), pol.begin() + (size_t)k * 2 * P);
      gt.erase(gt.begin(), gt.begin() + (size_t)k * 64);
      val.erase(val.begin(), val.begin() + (size_t)k * 5 * A);
      n -= k;
      filesWritten++;
      rowsWritten += k;
      logf("wrote %s (%d rows)", path.c_str(), k);
    }
  }
};

// Finished games as SGF, one game per line of <dir>/<hex>.sgfs (sgf.cpp:1526-1700:
// FF[4] GM[Coffee] SZ WLL PB PW RE, moves B[xyd] / W[xyd] with d = a..d for N, W,
// NW, NE; Coffee draws — SPEC B16 — are RE[0]).
struct SgfSink {
  std::string dir, modelName;
  int x, y, winLen;
  uint64_t fileId;
  FILE* f = nullptr;
  int64_t games = 0;

  void write(int n, const int32_t* hdr, const uint8_t* mv) {
    if(n <= 0)
      return;
    if(!f) {
      char name[64];
      snprintf(name, sizeof(name), "%016llX.sgfs", (unsigned long long)fileId);
      f = fopen((dir + "/" + name).c_str(), "a");
      if(!f)
        die("cannot write sgfs in " + dir);
    }
    const int A = x * y;
    const char* coord = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ";
    for(int i = 0; i < n; i++) {
      const int32_t* h = hdr + 4 * i;
      const char* res = h[3] == 1 ? "B+" : (h[3] == 2 ? "W+" : "0");
      std::string g = "(;FF[4]GM[Coffee]";
      g += x == y ? "SZ[" + std::to_string(x) + "]" : "SZ[" + std::to_string(x) + ":" + std::to_string(y) + "]";
      g += "WLL[" + std::to_string(winLen) + "]PB[" + modelName + "]PW[" + modelName + "]RE[" + res + "]";
      g += "C[startTurnIdx=0,initTurnNum=0,gameId=" + std::to_string(h[0]) + ":" + std::to_string(h[1]) +
           ",gtype=normal]";
      for(int t = 0; t < h[2] && t < A; t++) {
        const int cell = mv[((size_t)i * A + t) * 2], d = mv[((size_t)i * A + t) * 2 + 1];
        g += t % 2 == 0 ? ";B[" : ";W[";
        g += coord[cell % x];
        g += coord[cell / x];
        g += (char)('a' + d);
        g += "]";
        if(t + 1 == h[2])
          g += std::string("C[result=") + res + "]";
      }
      g += ")\n";
      fputs(g.c_str(), f);
      games++;
    }
    fflush(f);
  }
  void close() {
    if(f)
      fclose(f);
    f = nullptr;
  }
};

static std::atomic<int64_t> gGamesDone(0);

// One self-play engine: `share` of GPU `gpu`'s games from slot `slot` on (the
// reference's NN server thread with its game threads).  Engines on one device run
// on their own streams, so one's network overlaps another's search kernels; they
// split the device's batch cap (one wave of fused-network workgroups).
static void runGpu(int gpu, int server, int perGpu, int slot, int share, const Settings& s,
                   const std::string& outDir) {
  check(coffee_set_device(gpu), "set device");
  std::string model;
  int version = 0;
  gModels.current(model, version);
  coffee_selfplay_config c;
  memset(&c, 0, sizeof(c));
  c.x = s.x;
  c.y = s.y;
  c.win_len = s.winLen;
  c.num_games = share;
  c.seed = s.seed;
  c.slot_base = slot;
  // engines sharing this GPU split the default batch cap of a fused network (one wave
  // of network workgroups); layered networks stay uncapped (the engine decides, also
  // after a hot reload that changes the network path)
  c.nn_batch_cap = 0;
  c.engines_per_device = perGpu;
  c.use_fake_net = 0;
  c.commit_interval = 16;  // moves committed every 16 rounds (bench.py's default)
  c.model_path = model.c_str();
  c.search = s.sp;
  c.nn_cache_log2 = s.nnCacheLog2;
  c.nn_precision = s.nnPrecision;
  coffee_selfplay* h = nullptr;
  check(coffee_selfplay_create(&c, &h), "create engine");
  std::mt19937_64 fileRng(s.seed ^ (0x9E3779B97F4A7C15ULL * (gpu + 1)) ^ ((uint64_t)server << 48));
  auto dirsFor = [&](const std::string& m, std::string& tdata, std::string& sgfs) {
    tdata = outDir + "/" + modelNameOf(m) + "/tdata";
    sgfs = outDir + "/" + modelNameOf(m) + "/sgfs";
    mkdirs(tdata);
    mkdirs(sgfs);
  };
  std::string tdata, sgfs;
  dirsFor(model, tdata, sgfs);
  RowSink sink{tdata, s.x, s.y, s.maxRowsPerFile, std::mt19937_64(fileRng())};
  SgfSink games{sgfs, modelNameOf(model), s.x, s.y, s.winLen, fileRng()};
  const int A = s.x * s.y, pb = (A + 7) / 8, P = 4 * A;
  const int chunk = 65536;
  std::vector<uint8_t> bin((size_t)chunk * 15 * pb);
  std::vector<float> glob(chunk), gt((size_t)chunk * 64);
  std::vector<int16_t> pol((size_t)chunk * 2 * P);
  std::vector<int8_t> val((size_t)chunk * 5 * A);
  std::vector<int32_t> meta((size_t)chunk * 4);
  const int gchunk = 2 * s.games;
  std::vector<int32_t> ghdr((size_t)gchunk * 4);
  std::vector<uint8_t> gmv((size_t)gchunk * A * 2);
  uint64_t lastGames = 0;
  int64_t filesBefore = 0, rowsBefore = 0, rowsDrained = 0;
  auto t0 = std::chrono::steady_clock::now();
  auto drainAll = [&]() {
    int got = 0;
    do {
      check(coffee_selfplay_drain_rows(h, chunk, bin.data(), glob.data(), pol.data(), gt.data(), val.data(),
                                       meta.data(), &got),
            "drain");
      if(got > 0) {
        sink.append(got, bin.data(), glob.data(), pol.data(), gt.data(), val.data());
        rowsDrained += got;
      }
    } while(got == chunk);
    check(coffee_selfplay_drain_games(h, gchunk, ghdr.data(), gmv.data(), &got), "drain games");
    games.write(got, ghdr.data(), gmv.data());
  };
  while(!gStop) {
    check(coffee_selfplay_step(h, 200, nullptr), "step");
    drainAll();
    sink.flush(false);
    std::string latest;
    int v = 0;
    gModels.current(latest, v);
    if(v != version) {
      // hot reload: finish the old model's files, then switch every game to the new net
      sink.flush(true);
      games.close();
      if(coffee_selfplay_set_model(h, latest.c_str()) == COFFEE_OK) {
        logf("gpu %d.%d: switched to model %s", gpu, server, latest.c_str());
        model = latest;
        filesBefore += sink.filesWritten;
        rowsBefore += sink.rowsWritten;
        dirsFor(model, tdata, sgfs);
        sink.dir = tdata;
        sink.filesWritten = sink.rowsWritten = 0;
        games.dir = sgfs;
        games.modelName = modelNameOf(model);
        games.fileId = fileRng();
      } else {
        logf("gpu %d.%d: cannot load %s (%s); keeping %s", gpu, server, latest.c_str(), coffee_last_error(), model.c_str());
      }
      version = v;
    }
    coffee_selfplay_stats st;
    check(coffee_selfplay_stats_get(h, &st), "stats");
    gGamesDone += (int64_t)(st.games_finished - lastGames);
    lastGames = st.games_finished;
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // rows/s counts the training rows drained for the .npz files (after weight
    // resolution: cheap searches, surprise weighting and side positions make it differ
    // from moves/s)
    logf("gpu %d.%d: %llu games, %llu moves, %lld rows, %.1f rows/s, %.1f moves/s, %.3g playouts/s, %llu rows dropped",
         gpu, server, (unsigned long long)st.games_finished, (unsigned long long)st.moves, (long long)rowsDrained,
         rowsDrained / secs, st.moves / secs, st.playouts / secs, (unsigned long long)st.rows_dropped);
    if(st.nn_audits > 0 || st.nn_audit_switches > 0)  // the default precision's audit
      logf("gpu %d.%d: network precision %llu, %llu audited launches, max |corrected - accurate| %.3g%s", gpu, server,
           (unsigned long long)st.nn_precision, (unsigned long long)st.nn_audits, st.nn_audit_max_diff,
           st.nn_audit_switches ? ", switched to accurate" : "");
    if(s.maxGamesTotal >= 0 && gGamesDone >= s.maxGamesTotal)
      gStop = true;
  }
  drainAll();
  sink.flush(true);
  games.close();
  coffee_selfplay_destroy(h);
  logf("gpu %d.%d done: %lld files, %lld rows, %lld games", gpu, server, (long long)(filesBefore + sink.filesWritten),
       (long long)(rowsBefore + sink.rowsWritten), (long long)games.games);
}

int main(int argc, char** argv) {
  if(argc < 2 || std::string(argv[1]) != "selfplay")
    die("usage: katago selfplay -config <cfg> -models-dir <dir> -output-dir <dir> [-max-games-total N] "
        "[-override-config k=v,...]");
  std::string cfgPath, modelsDir, outDir, overrides;
  int64_t maxGames = -1;
  for(int i = 2; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if(i + 1 >= argc)
        die("missing value for " + a);
      return argv[++i];
    };
    if(a == "-config")
      cfgPath = next();
    else if(a == "-models-dir")
      modelsDir = next();
    else if(a == "-output-dir")
      outDir = next();
    else if(a == "-max-games-total")
      maxGames = std::stoll(next());
    else if(a == "-override-config")
      overrides = next();
    else
      die("unknown argument " + a);
  }
  if(cfgPath.empty() || modelsDir.empty() || outDir.empty())
    die("-config, -models-dir and -output-dir are required");
  std::map<std::string, std::string> kv;
  if(!readConfig(cfgPath, kv))
    die("cannot read config " + cfgPath);
  std::stringstream os(overrides);
  std::string item;
  while(std::getline(os, item, ',')) {
    size_t eq = item.find('=');
    if(eq != std::string::npos)
      kv[trim(item.substr(0, eq))] = trim(item.substr(eq + 1));
  }
  Settings s;
  coffee_search_params_default(&s.sp);
  try {
    applyConfig(kv, s);
  } catch(const std::exception& e) {
    die(e.what());
  }
  s.maxGamesTotal = maxGames;
  s.seed = std::random_device{}() ^ ((uint64_t)std::random_device{}() << 32);
  mkdirs(outDir);
  char lname[64];
  time_t now = time(nullptr);
  strftime(lname, sizeof(lname), "log%Y%m%d-%H%M%S.log", localtime(&now));
  gLog = fopen((outDir + "/" + lname).c_str(), "w");
  std::signal(SIGINT, onSignal);
  std::signal(SIGTERM, onSignal);
  gModels.dir = modelsDir;
  gModels.path = newestModel(modelsDir);
  newestModelOrEmpty(modelsDir, &gModels.mtime);
  gModels.pollSeconds = s.modelPollSeconds;
  const std::string model = gModels.path;
  {
    // one HIP stream per engine: HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware
    // queues (4 by default) and streams sharing a queue serialise, so a GPU running more
    // engines than that gets more queues before the first HIP call (bench.py: 4 engines on
    // 4 queues ran at 60 % of their rate on 8)
    const int perGpu = std::max(1, (s.servers + std::max(1, s.gpus) - 1) / std::max(1, s.gpus));
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    const int have = q ? atoi(q) : 4;
    if(perGpu + 1 > have)
      setenv("GPU_MAX_HW_QUEUES", std::to_string(std::min(16, std::max(8, perGpu + 1))).c_str(), 1);
  }
  int ndev = 0;
  check(coffee_device_count(&ndev), "device count");
  if(s.gpus < 1 || s.gpus > ndev)
    die("numGpus must be in 1.." + std::to_string(ndev));
  logf("selfplay: model %s, %dx%d win %d, %d games/GPU x %d GPUs, %d visits", model.c_str(), s.x, s.y, s.winLen,
       s.games, s.gpus, s.sp.max_visits);
  // numNNServerThreadsPerModel engines spread over the GPUs: floor / ceil per GPU so the
  // total is exactly the configured count (the reference gives each server thread its
  // GPU, gpuToUseThreadN); every GPU runs at least one.  A GPU's games split evenly
  // between its engines.
  int engines = 0;
  for(int g = 0; g < s.gpus; g++)
    engines += std::max(1, s.servers / s.gpus + (g < s.servers % s.gpus ? 1 : 0));
  if(engines != s.servers)
    logf("selfplay: numNNServerThreadsPerModel %d < numGpus %d: running %d engines (one per GPU)", s.servers,
         s.gpus, engines);
  std::vector<std::thread> th;
  for(int g = 0; g < s.gpus; g++) {
    const int perGpu = std::max(1, s.servers / s.gpus + (g < s.servers % s.gpus ? 1 : 0));
    if(perGpu > s.games)
      die("numNNServerThreadsPerModel exceeds the games per GPU");
    for(int k = 0, off = 0; k < perGpu; k++) {
      const int share = s.games / perGpu + (k < s.games % perGpu ? 1 : 0);
      th.emplace_back(runGpu, g, k, perGpu, g * s.games + off, share, std::cref(s), std::cref(outDir));
      off += share;
    }
  }
  for(auto& t : th)
    t.join();
  if(gLog)
    fclose(gLog);
  return 0;
}
