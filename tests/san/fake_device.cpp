// A host-memory stand-in for the GPU under ThreadSanitizer (tests/test_sanitizers.py):
// the PRODUCT's host code -- csrc/capi.cpp (the C ABI: argument checks, thread-local
// error strings, the process-wide device-table cache), csrc/selfplay.cpp (engine
// allocation, the round loop, kernel-timing events, drain / stage / drain-games, model
// hot switch), model.cpp, tables.cpp, refrand.cpp and npzwrite.cpp -- is compiled with
// -fsanitize=thread and linked against this file instead of the HIP runtime and the
// kernels.  Test infrastructure only: nothing here is shipped.
//  * HIP API: device memory is host memory, every copy / memset / "kernel" runs at once
//    on the calling thread (so a stream is always idle and an event always complete),
//    the current device is per thread like the runtime's, events hold a timestamp;
//  * kernel launchers (search.hip, rules.hip, nn.hip): a round advances every game's
//    counters; a commit plays one move per game and ends a game every 12 moves, writing
//    its rows and its game record into the "device" buffers the host code then drains
//    or stages; the network and the rules batches touch nothing;
//  * NNEngine: the network object without device weights (precision as requested).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "../../katacoffee_amd/csrc/engine.h"
#include "../../katacoffee_amd/csrc/search.h"

struct ihipStream_t {
  int id;
};
struct ihipEvent_t {
  double ms;
};

namespace {
thread_local int tDevice = 0;
std::atomic<int> gStreams{0};
double nowMs() {
  using namespace std::chrono;
  static const steady_clock::time_point t0 = steady_clock::now();
  return duration<double, std::milli>(steady_clock::now() - t0).count();
}
}  // namespace

extern "C" {
hipError_t hipMalloc(void** ptr, size_t size) {
  *ptr = aligned_alloc(256, (size + 255) / 256 * 256);
  return *ptr ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* ptr) {
  free(ptr);
  return hipSuccess;
}
hipError_t hipMemcpy(void* dst, const void* src, size_t sizeBytes, hipMemcpyKind) {
  memmove(dst, src, sizeBytes);
  return hipSuccess;
}
hipError_t hipMemset(void* dst, int value, size_t sizeBytes) {
  memset(dst, value, sizeBytes);
  return hipSuccess;
}
hipError_t hipMemsetAsync(void* dst, int value, size_t sizeBytes, hipStream_t) {
  memset(dst, value, sizeBytes);
  return hipSuccess;
}
hipError_t hipGetDevice(int* deviceId) {
  *deviceId = tDevice;
  return hipSuccess;
}
hipError_t hipSetDevice(int deviceId) {
  int n = 0;
  hipGetDeviceCount(&n);
  if(deviceId < 0 || deviceId >= n)
    return hipErrorInvalidDevice;
  tDevice = deviceId;
  return hipSuccess;
}
hipError_t hipGetDeviceCount(int* count) {
  const char* e = getenv("FAKE_DEVICES");
  *count = e ? atoi(e) : 2;
  return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int* pi, hipDeviceAttribute_t attr, int) {
  *pi = attr == hipDeviceAttributeMultiprocessorCount ? 256 : 0;
  return hipSuccess;
}
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "fake device error"; }
hipError_t hipStreamCreateWithFlags(hipStream_t* stream, unsigned int) {
  *stream = new ihipStream_t{++gStreams};
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t stream) {
  delete stream;
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* event) {
  *event = new ihipEvent_t{0.0};
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t event) {
  delete event;
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t event, hipStream_t) {
  event->ms = nowMs();
  return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t start, hipEvent_t stop) {
  *ms = (float)(stop->ms - start->ms);
  return hipSuccess;
}
}

namespace kc {

static void stamp(hipEvent_t e) {
  if(e)
    hipEventRecord(e, nullptr);
}

void launchSelfplayInit(const SearchDev&, const SearchDev*, hipStream_t) {}

void launchSelect(const SearchDev& d, const SearchDev*, hipStream_t, hipEvent_t e0, hipEvent_t e1, bool resetCommit) {
  stamp(e0);
  if(resetCommit)
    *d.commitCount = 0;
  for(int g = 0; g < d.G; g++)
    d.games[g].playouts++;
  stamp(e1);
}

void launchCompact(const SearchDev& d, const SearchDev*, hipStream_t, bool accumulate, bool) {
  const int n = d.G < d.nnCap ? d.G : d.nnCap;
  *d.nnCount = n;
  for(int i = 0; i < n; i++)
    d.nnIdx[i] = i;
  if(accumulate)
    *d.nnTimedEvals += (unsigned long long)n;
}

void launchBackup(const SearchDev& d, const SearchDev*, hipStream_t, hipEvent_t e0, hipEvent_t e1) {
  stamp(e0);
  for(int i = 0; i < *d.nnCount; i++)
    d.games[d.nnIdx[i]].nnEvals++;
  stamp(e1);
}

void launchBackupSelect(const SearchDev& d, const SearchDev* dd, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  stamp(e0);
  launchBackup(d, dd, st, nullptr, nullptr);
  launchSelect(d, dd, st, nullptr, nullptr, false);
  stamp(e1);
}
void launchResolve(const SearchDev&, const SearchDev*, hipStream_t) {}

// one move per game; a game ends every 12 moves with one row per move and a record
void launchCommit(const SearchDev& d, const SearchDev*, hipStream_t) {
  const int A = d.A, P = d.P, pb = (A + 7) / 8;
  for(int g = 0; g < d.G; g++) {
    GameDev& s = d.games[g];
    s.moves++;
    if(s.moves % 12)
      continue;
    s.gamesFinished++;
    for(int t = 0; t < 12; t++) {
      const unsigned long long r = *d.rCount;
      if(r >= (unsigned long long)d.rowCap) {
        ++*d.rDropped;
        continue;
      }
      memset(d.rBin + r * NUM_SPATIAL * pb, (int)((g + t) & 0xff), (size_t)NUM_SPATIAL * pb);
      d.rGlob[r] = 4.0f;
      for(int k = 0; k < 2 * P; k++)
        d.rPol[r * 2 * P + k] = (int16_t)((g + t + k) % 7);
      for(int k = 0; k < 64; k++)
        d.rGt[r * 64 + k] = k == 63 ? 1.0f : 0.0f;
      memset(d.rVal + r * 5 * A, 0, (size_t)5 * A);
      d.rMeta[r * 4] = d.slotBase + g;
      d.rMeta[r * 4 + 1] = (int32_t)s.gamesFinished;
      d.rMeta[r * 4 + 2] = t;
      d.rMeta[r * 4 + 3] = 12;
      *d.rCount = r + 1;
    }
    const unsigned long long k = *d.gCount;
    if(k >= (unsigned long long)d.gCap) {
      ++*d.gDropped;
      continue;
    }
    GameRec& rec = d.gRec[k];
    rec.slot = d.slotBase + g;
    rec.gameNum = (int32_t)s.gamesFinished;
    rec.numMoves = 12 < A ? 12 : A;
    rec.winner = (int32_t)(s.gamesFinished % 3);
    for(int m = 0; m < MAX_AREA; m++) {
      rec.cell[m] = (uint8_t)(m % A);
      rec.dir[m] = (uint8_t)(m % 4);
    }
    *d.gCount = k + 1;
  }
}

void launchStageRows(const SearchDev& d, const SearchDev*, uint8_t* dst, unsigned long long* countOut, bool discardGames,
                     hipStream_t) {
  const int A = d.A, P = d.P, pb = (A + 7) / 8, rb = rowBytes(A);
  const unsigned long long n = *d.rCount;
  for(unsigned long long r = 0; r < n; r++) {
    uint8_t* o = dst + r * rb;
    auto put = [&](const void* src, size_t bytes) {
      memcpy(o, src, bytes);
      o += bytes;
    };
    put(d.rBin + r * NUM_SPATIAL * pb, (size_t)NUM_SPATIAL * pb);
    put(d.rGlob + r, 4);
    put(d.rPol + r * 2 * P, (size_t)4 * P);
    put(d.rGt + r * 64, 256);
    put(d.rVal + r * 5 * A, (size_t)5 * A);
    put(d.rMeta + r * 4, 16);
  }
  *countOut = n;
  *d.rStaged += n;
  *d.rCount = 0;
  if(discardGames)
    *d.gCount = 0;
}

void launchGameTree(const SearchDev*, int, int, uint32_t*, uint32_t*, int32_t* count, hipStream_t) { *count = 0; }
void launchFakeNet(const DTables*, int, const uint64_t*, float*, hipStream_t, const int*, const int*) {}
void launchCanonicalRows(const DTables*, int, const int*, float*, hipStream_t) {}
void launchEncodeBatch(const DTables*, int, const uint8_t*, const int8_t*, const int8_t*, const uint8_t*, const int32_t*,
                       uint64_t*, float*, hipStream_t) {}
void launchRulesBatch(const DTables*, int, const uint8_t*, const int8_t*, const int8_t*, const uint8_t*, uint8_t*, uint8_t*,
                      hipStream_t) {}
void launchPlayBatch(const DTables*, int, const uint8_t*, const int8_t*, const int8_t*, const uint8_t*, const int32_t*,
                     uint8_t*, uint8_t*, uint8_t*, int32_t*, uint64_t*, uint64_t*, hipStream_t) {}

NNEngine::NNEngine(const ModelHost& m, int X, int Y, int W, int path) : cfg_(m.cfg), X_(X), Y_(Y), W_(W) {
  flops_ = modelFlopsPerEval(cfg_, X * Y);
  if(path < NN_DEFAULT || path > NN_FAST)
    throw std::invalid_argument("NNEngine: unknown precision/path");
  mode_ = path == NN_DEFAULT ? NN_CORRECTED : path;
}
NNEngine::~NNEngine() {}
void NNEngine::forward(int, const uint64_t*, float*, hipStream_t, const int*, const int*, hipEvent_t e0, hipEvent_t e1) {
  stamp(e0);
  stamp(e1);
}
int NNEngine::precision() const { return mode_; }
void NNEngine::audit(int, const uint64_t*, const float*, float*, unsigned*, hipStream_t, const int*, const int*) {}
NNLayered::~NNLayered() {}

}  // namespace kc
