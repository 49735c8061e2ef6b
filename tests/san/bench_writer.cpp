// bench.py's host threading restated in C++ for ThreadSanitizer (tests/test_sanitizers.py):
// the main thread steps K engine groups in interleaved chunks (bench.py Groups.step),
// drains their rows after every step and hands each step's block to a writer thread
// through a queue; the writer writes <dir>/rows%06d.npz via a .tmp file and rename
// (bench.py NpzWriter, trainingwrite.cpp:566-587 / :765-769) while the engines keep
// stepping; close() sends the sentinel and joins before the clock would stop.  Linked
// with fake_engine.cpp (the C ABI without a GPU) and the product's npzwrite.cpp.
//   bench_writer <dir> [groups] [steps]
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
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
  const int X = 5, Y = 5, A = X * Y, pb = (A + 7) / 8, P = 4 * A, games = 256, chunk = 16, rps = 200;
  std::string model = dir + "/model.cfnn";
  FILE* f = fopen(model.c_str(), "w");
  if(!f)
    return 2;
  fputs("fake", f);
  fclose(f);
  std::vector<coffee_selfplay*> g(groups);
  for(int k = 0; k < groups; k++) {
    coffee_selfplay_config c = {};
    c.x = X;
    c.y = Y;
    c.win_len = 4;
    c.num_games = games / groups;
    c.slot_base = k * (games / groups);
    c.model_path = model.c_str();
    c.engines_per_device = groups;
    if(coffee_selfplay_create(&c, &g[k]) != COFFEE_OK)
      return 3;
  }
  Writer w(dir, X, Y);
  long drained = 0;
  for(int s = 0; s < steps; s++) {
    for(int done = 0; done < rps; done += chunk)
      for(auto* e : g)
        coffee_selfplay_step(e, chunk, nullptr);
    Block* b = new Block;
    for(auto* e : g) {
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
  printf("bench writer: %ld rows drained, %ld written in %d files%s\n", drained, w.rows(), w.files(),
         w.failed() ? " (write error)" : "");
  return drained == w.rows() && !w.failed() ? 0 : 1;
}
