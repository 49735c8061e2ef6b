// Sanitizer driver for the product's host code (tests/test_sanitizers.py builds it with
// host-side AddressSanitizer + UndefinedBehaviorSanitizer, tests/san/Makefile):
// CFNN model I/O (model.cpp), the .npz row writer (npzwrite.cpp), the geometry /
// Zobrist tables (tables.cpp, refrand.cpp) and the CLI config layer (cli_config.h).
//
//   host_check models DIR        write/load/re-write every named architecture; truncated
//                                and corrupted files must fail with an exception
//   host_check npz DIR           rows for 4 geometries x {0, 1, 37} rows: DIR/r_X_Y_N.npz
//                                plus the raw arrays (DIR/r_X_Y_N.<member>.bin) to compare
//   host_check tables            buildTables for every geometry 2..10 x 2..10
//   host_check config FILE...    parse each file; print the resolved settings or the error
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../katacoffee_amd/csrc/cli_config.h"
#include "../../katacoffee_amd/csrc/kc_common.h"
#include "../../katacoffee_amd/csrc/model.h"
#include "../../katacoffee_amd/csrc/npzwrite.h"

using namespace kc;

static std::vector<char> slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  return std::vector<char>(std::istreambuf_iterator<char>(f), {});
}
static void spit(const std::string& p, const char* d, size_t n) {
  std::ofstream f(p, std::ios::binary);
  f.write(d, (std::streamsize)n);
}

static int models(const std::string& dir) {
  int fails = 0;
  for(const char* arch : {"b2c32", "b2c32nbt", "b6c96", "b10c128", "b18c384nbt"}) {
    const std::string p = dir + "/" + arch + ".cfnn", q = p + ".2";
    ModelHost m = randomModel(modelCfgByName(arch), 0xC0FFEE);
    saveModel(p, m);
    ModelHost r = loadModel(p);
    saveModel(q, r);
    const std::vector<char> a = slurp(p), b = slurp(q);
    if(a != b) {
      printf("%s: re-written file differs\n", arch);
      fails++;
    }
    const double fl = modelFlopsPerEval(r.cfg, 25);
    // every proper prefix must be rejected, never read past the end
    int rejected = 0, tried = 0;
    for(size_t cut : {size_t(0), size_t(3), size_t(8), size_t(40), a.size() / 3, a.size() / 2, a.size() - 4,
                      a.size() - 1}) {
      spit(p + ".cut", a.data(), cut);
      tried++;
      try {
        loadModel(p + ".cut");
      } catch(const std::exception&) {
        rejected++;
      }
    }
    // corrupted header fields (sizes, block count, kinds): an exception or a model, never a crash
    int corrupt = 0;
    for(size_t off = 4; off < 64 && off + 4 <= a.size(); off += 4) {
      for(int32_t v : {-1, 0, 1 << 20, 7}) {
        std::vector<char> c = a;
        memcpy(&c[off], &v, 4);
        spit(p + ".bad", c.data(), c.size());
        try {
          loadModel(p + ".bad");
        } catch(const std::exception&) {
          corrupt++;
        }
      }
    }
    printf("%s: %zu bytes, %.4g flops/eval, %d/%d prefixes rejected, %d corrupt headers rejected\n", arch, a.size(),
           fl, rejected, tried, corrupt);
    if(rejected != tried)
      fails++;
  }
  return fails;
}

static int npz(const std::string& dir) {
  std::mt19937 rng(7);
  const int geoms[4][2] = {{5, 5}, {7, 7}, {9, 9}, {6, 4}};
  for(auto& gm : geoms)
    for(int n : {0, 1, 37}) {
      const int X = gm[0], Y = gm[1], A = X * Y, P = 4 * A, pb = (A + 7) / 8;
      std::vector<uint8_t> bin((size_t)n * 15 * pb);
      std::vector<float> glob((size_t)n), gt((size_t)n * 64);
      std::vector<int16_t> pol((size_t)n * 2 * P);
      std::vector<int8_t> val((size_t)n * 5 * A);
      for(auto& v : bin) v = (uint8_t)rng();
      for(auto& v : glob) v = (float)(rng() % 11);
      for(auto& v : gt) v = (float)(int)(rng() % 2001) / 1000.0f - 1.0f;
      for(auto& v : pol) v = (int16_t)(rng() % 1000);
      for(auto& v : val) v = (int8_t)((int)(rng() % 3) - 1);
      char base[256];
      snprintf(base, sizeof(base), "%s/r_%d_%d_%d", dir.c_str(), X, Y, n);
      writeNpz(std::string(base) + ".npz", n, X, Y, bin.data(), glob.data(), pol.data(), gt.data(), val.data());
      spit(std::string(base) + ".binaryInputNCHWPacked.bin", (const char*)bin.data(), bin.size());
      spit(std::string(base) + ".globalInputNC.bin", (const char*)glob.data(), glob.size() * 4);
      spit(std::string(base) + ".policyTargetsNCMove.bin", (const char*)pol.data(), pol.size() * 2);
      spit(std::string(base) + ".globalTargetsNC.bin", (const char*)gt.data(), gt.size() * 4);
      spit(std::string(base) + ".valueTargetsNCHW.bin", (const char*)val.data(), val.size());
    }
  printf("npz ok\n");
  return 0;
}

static int tables() {
  long n = 0;
  for(int X = 2; X <= MAX_LEN; X++)
    for(int Y = 2; Y <= MAX_LEN; Y++)
      for(int W = 2; W <= (X > Y ? X : Y); W++) {
        DTables t = buildTables(X, Y, W);
        n += t.A;
      }
  printf("tables ok %ld\n", n);
  return 0;
}

static int config(int argc, char** argv) {
  for(int i = 0; i < argc; i++) {
    std::map<std::string, std::string> kv;
    kccli::Settings s;
    memset(&s.sp, 0, sizeof(s.sp));
    if(!kccli::readConfig(argv[i], kv)) {
      printf("%s: unreadable\n", argv[i]);
      continue;
    }
    try {
      kccli::applyConfig(kv, s);
      printf("%s: x=%d y=%d win=%d games=%d gpus=%d servers=%d rows=%d cache=%d prec=%d visits=%d cpuct=%.4f "
             "noise=%d tree=%d\n",
             argv[i], s.x, s.y, s.winLen, s.games, s.gpus, s.servers, s.maxRowsPerFile, s.nnCacheLog2, s.nnPrecision,
             s.sp.max_visits, s.sp.cpuct_exploration, s.sp.root_noise_enabled, s.sp.record_tree_positions);
    } catch(const std::exception& e) {
      printf("%s: error: %s\n", argv[i], e.what());
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  if(argc < 2)
    return 2;
  const std::string cmd = argv[1];
  if(cmd == "models" && argc == 3)
    return models(argv[2]) ? 1 : 0;
  if(cmd == "npz" && argc == 3)
    return npz(argv[2]);
  if(cmd == "tables")
    return tables();
  if(cmd == "config")
    return config(argc - 2, argv + 2);
  return 2;
}
