// bench.py's host threading restated in C++ for ThreadSanitizer (tests/test_sanitizers.py):
// the main thread steps K engine groups in interleaved chunks (bench.py Groups.step),
// collects their rows after every step -- drained to host buffers, or (stage mode, the
// bench's multi-GPU path) staged on the "device" by coffee_selfplay_stage_rows and copied
// back once the engine stream has passed it -- and hands each step's block to a writer
// thread through a queue; the writer writes <dir>/rows%06d.npz via a .tmp file and rename
// (bench.py NpzWriter, trainingwrite.cpp:566-587 / :765-769) while the engines keep
// stepping; close() sends the sentinel and joins before the clock would stop.  Linked
// with the product's host code (capi.cpp, selfplay.cpp, npzwrite.cpp, ...) over
// fake_device.cpp (host memory for the GPU, stand-in kernels).
//   bench_writer <dir> [groups] [steps] [stage]
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/katacoffee.h"

struct Block {
  int n = 0;
  std::vector<uint8_t> bin;
  std::vector<float> glob, gt;
  std::vector<int16_t> pol;
  std::vector<int8_t> val;
};

class Writer {
 public:
  Writer(std::string dir, int x, int y) : dir_(std::move(dir)), x_(x), y_(y), t_([this] { run(); }) {}
  void put(Block* b) {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(b);
    cv_.notify_one();
  }
  // every queued block is on disk when close() returns
  void close() {
    put(nullptr);
    t_.join();
  }
  long rows() const { return rows_; }
  int files() const { return files_; }
  bool failed() const { return err_; }

 private:
  void run() {
    for(;;) {
      Block* b;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !q_.empty(); });
        b = q_.front();
        q_.pop_front();
      }
      if(!b)
        return;
      if(b->n) {
        char name[64];
        snprintf(name, sizeof(name), "/rows%06d.npz", files_);
        const std::string path = dir_ + name;
        if(coffee_write_npz((path + ".tmp").c_str(), b->n, x_, y_, b->bin.data(), b->glob.data(), b->pol.data(),
                            b->gt.data(), b->val.data()) != COFFEE_OK ||
           rename((path + ".tmp").c_str(), path.c_str()) != 0)
          err_ = true;
        files_++;
        rows_ += b->n;
      }
      delete b;
    }
  }
  std::string dir_;
  int x_, y_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Block*> q_;
  long rows_ = 0;
  int files_ = 0;
  bool err_ = false;
  std::thread t_;  // last: starts after the members it uses
};

int main(int argc, char** argv) {
  if(argc < 2)
    return 2;
  const std::string dir = argv[1];
  const int groups = argc > 2 ? atoi(argv[2]) : 2, steps = argc > 3 ? atoi(argv[3]) : 40;
  const bool stage = argc > 4 && std::string(argv[4]) == "stage";
  const int X = 5, Y = 5, A = X * Y, pb = (A + 7) / 8, P = 4 * A, games = 256, chunk = 16, rps = 200;
  const int rowCap = 4096;
  int rb = 0;
  if(coffee_row_bytes(X, Y, &rb) != COFFEE_OK)
    return 3;
  std::vector<coffee_selfplay*> g(groups);
  std::vector<void*> dst(groups, nullptr);
  for(int k = 0; k < groups; k++) {
    coffee_selfplay_config c = {};
    coffee_search_params_default(&c.search);
    c.x = X;
    c.y = Y;
    c.win_len = 4;
    c.num_games = games / groups;
    c.slot_base = k * (games / groups);
    c.use_fake_net = 1;
    c.row_capacity = rowCap;
    c.node_cap = 1024;
    c.commit_interval = 16;
    c.engines_per_device = groups;
    if(coffee_selfplay_create(&c, &g[k]) != COFFEE_OK) {
      fprintf(stderr, "create: %s\n", coffee_last_error());
      return 3;
    }
    if(stage && coffee_malloc(&dst[k], (uint64_t)rowCap * rb) != COFFEE_OK)
      return 3;
  }
  Writer w(dir, X, Y);
  long drained = 0;
  std::vector<uint8_t> staged((size_t)rowCap * rb);
  for(int s = 0; s < steps; s++) {
    for(int done = 0; done < rps; done += chunk)
      for(auto* e : g)
        coffee_selfplay_step(e, chunk, nullptr);
    Block* b = new Block;
    for(size_t k = 0; k < g.size(); k++) {
      coffee_selfplay* e = g[k];
      if(stage) {
        // the row buffer packed on the engine stream; the count is valid once the stream
        // has passed the call (coffee_selfplay_sync here; bench.py waits on an event)
        uint64_t n = 0;
        if(coffee_selfplay_stage_rows(e, dst[k], rowCap, &n, COFFEE_STAGE_DISCARD_GAMES) != COFFEE_OK ||
           coffee_selfplay_sync(e) != COFFEE_OK || coffee_memcpy(staged.data(), dst[k], n * rb, 1) != COFFEE_OK)
          return 4;
        for(uint64_t r = 0; r < n; r++) {
          const uint8_t* q = staged.data() + r * rb;
          auto take = [&](auto& vec, size_t count) {
            using T = typename std::remove_reference<decltype(vec)>::type::value_type;
            const T* src = reinterpret_cast<const T*>(q);
            vec.insert(vec.end(), src, src + count);
            q += count * sizeof(T);
          };
          take(b->bin, (size_t)15 * pb);
          take(b->glob, 1);
          take(b->pol, (size_t)2 * P);
          take(b->gt, 64);
          take(b->val, (size_t)5 * A);
        }
        b->n += (int)n;
        continue;
      }
      const int cap = 4096;
      std::vector<uint8_t> bin((size_t)cap * 15 * pb);
      std::vector<float> glob(cap), gt((size_t)cap * 64);
      std::vector<int16_t> pol((size_t)cap * 2 * P);
      std::vector<int8_t> val((size_t)cap * 5 * A);
      std::vector<int32_t> meta((size_t)cap * 4);
      int got = 0;
      do {
        coffee_selfplay_drain_rows(e, cap, bin.data(), glob.data(), pol.data(), gt.data(), val.data(), meta.data(), &got);
        b->bin.insert(b->bin.end(), bin.begin(), bin.begin() + (size_t)got * 15 * pb);
        b->glob.insert(b->glob.end(), glob.begin(), glob.begin() + got);
        b->gt.insert(b->gt.end(), gt.begin(), gt.begin() + (size_t)got * 64);
        b->pol.insert(b->pol.end(), pol.begin(), pol.begin() + (size_t)got * 2 * P);
        b->val.insert(b->val.end(), val.begin(), val.begin() + (size_t)got * 5 * A);
        b->n += got;
      } while(got == cap);
      int ng = 0;
      coffee_selfplay_drain_games(e, 1024, nullptr, nullptr, &ng);
    }
    drained += b->n;
    w.put(b);
  }
  w.close();
  for(auto* e : g)
    coffee_selfplay_destroy(e);
  for(void* p : dst)
    if(p)
      coffee_free(p);
  printf("bench writer: %ld rows drained, %ld written in %d files%s\n", drained, w.rows(), w.files(),
         w.failed() ? " (write error)" : "");
  return drained == w.rows() && !w.failed() ? 0 : 1;
}
