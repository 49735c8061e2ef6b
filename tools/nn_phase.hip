// Phase timing of the fused network kernel (shader-clock stamps from the first
// workgroups).  Build: make -C tools nn_phase ; run on the GPU box:
// tools/_build/nn_phase [boards] [path: 0 fast, 1 accurate, 3 corrected, 4 accurate-nb2]
#define KC_NN_PROFILE
#include "../katacoffee_amd/csrc/nn.hip"

#include <cstdio>
#include <random>

using namespace kc;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;  // <= 5 x CUs: the small-batch (5-board) instance
  ModelHost m = randomModel(modelCfgByName("b6c96"), 1);
  const int path = argc > 2 ? atoi(argv[2]) : NN_FAST;
  NNEngine eng(m, 5, 5, 4, path);
  const int words = (15 * 25 + 63) / 64;
  std::vector<uint64_t> in((size_t)n * words);
  std::mt19937_64 rng(1);
  for(auto& w : in)
    w = rng() & rng();
  uint64_t* din;
  float* dout;
  KC_HIP(hipMalloc(&din, in.size() * 8));
  KC_HIP(hipMalloc(&dout, (size_t)n * 104 * 4));
  KC_HIP(hipMemcpy(din, in.data(), in.size() * 8, hipMemcpyHostToDevice));
  for(int it = 0; it < 3; it++)
    eng.forward(n, din, dout, nullptr);
  KC_HIP(hipDeviceSynchronize());
  unsigned long long ph[4][64];
  KC_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_nnPhase), sizeof(ph)));
  const char* names[64] = {};
  names[0] = "start";
  names[1] = "input unpacked";
  names[2] = "stem conv";
  for(int b = 0; b < 6; b++) {
    static char buf[6][4][48];
    snprintf(buf[b][0], 48, "blk%d start (prev conv)", b);
    snprintf(buf[b][1], 48, "blk%d bn1", b);
    snprintf(buf[b][2], 48, "blk%d conv1", b);
    snprintf(buf[b][3], 48, "blk%d mid (bn2/gpool)", b);
    names[3 + 4 * b] = buf[b][0];
    names[4 + 4 * b] = buf[b][1];
    names[5 + 4 * b] = buf[b][2];
    names[6 + 4 * b] = buf[b][3];
  }
  names[40] = "last conv2";
  names[41] = "tip + head conv";
  names[42] = "pool+linear";
  int order[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 40, 41, 42};
  for(int wg = 0; wg < 2; wg++) {
    printf("gpool(last): g-epi->pool %lld  pool->linG %lld  linG->r-epi %lld ; head: conv->pool %lld pool->lin %lld lin->end %lld\n",
           (long long)(ph[wg][51] - ph[wg][50]), (long long)(ph[wg][52] - ph[wg][51]),
           (long long)(ph[wg][26] - ph[wg][52]), (long long)(ph[wg][54] - ph[wg][53]),
           (long long)(ph[wg][42] - ph[wg][54]), 0LL);
    printf("workgroup %d (cycles since previous mark)\n", wg);
    unsigned long long prev = ph[wg][0];
    for(int i : order) {
      // phase k+1 of block b is stamped before the next; skip unset slots
      if(ph[wg][i] == 0)
        continue;
      printf("  %-24s %8lld\n", names[i] ? names[i] : "?", (long long)(ph[wg][i] - prev));
      prev = ph[wg][i];
    }
    printf("  total %lld cycles\n", (long long)(prev - ph[wg][0]));
    printf("  wall %.1f us (s_memrealtime) -> tick %.3f GHz\n", (ph[wg][63] - ph[wg][62]) / 100.0,
           (double)(ph[wg][42] - ph[wg][0]) / ((ph[wg][63] - ph[wg][62]) * 10.0));
  }
  return 0;
}
