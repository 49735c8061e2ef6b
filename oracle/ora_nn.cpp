// ORACLE (test infrastructure only) — fp32 residual-net forward with the Eigen
// CPU backend's semantics (eigenbackend.cpp):
//   ConvLayer        :270-680  ("same" convolution of any odd kernel size, NHWC;
//                               here im2col + a register-blocked SGEMM, the
//                               reference's non-Winograd path :669-677)
//   BatchNormLayer   :684-734  (merged scale/bias, then activation, then mask)
//   poolRowsGPool    :141-166  (mean, mean*(sqrt(maskSum)-14)*0.1, masked max)
//   poolRowsValueHead:168-186  (mean, mean*(sqrt-14)*0.1, mean*((sqrt-14)^2*0.01-0.1))
//   ResidualBlock    :888-931, GlobalPoolingResidualBlock :935-1015
//   NestedBottleneckResBlock  model_pytorch.py:860-958 (1x1 in, two inner blocks, 1x1 out)
//   Trunk :1169-1227, PolicyHead :1229-1299 (Coffee: 4 direction logits, no pass),
//   ValueHead :1301-1377 (Coffee: win/loss logits + 2 misc).
// The layer functions are pinned to the reference's own known-answer vectors
// (cpp/tests/testnn.cpp:107-915 -> tests/golden/nnlayers_kat.npz) and to blocks
// of python/model_pytorch.py (tests/golden/nnblocks_pytorch.npz); see
// tests/test_oracle_nn.py.
// mode 1 rounds every convolution weight and convolution input to fp16 (RNE),
// exactly where the HIP kernels do; residual trunks stay f32 as in the kernels.
// mode 2 restates the "corrected" precision (csrc/nn.hip NN_MODE_F8C): each product is
//   fp16(w) fp16(x) + E(lo(w) 2^11, sw) e4m3(fp16(x)) / 2^11 + E(fp16(w), sw) e4m3(lo(x) 2^11) / 2^11,
// lo(v) = v - fp16(v), e4m3 = OCP e4m3fn, round to nearest even, E(v, s) = e4m3(v 2^-s) 2^s
// (the device converts e4m3(w) and e4m3(x) from the fp16 fragments in registers)
// with sw the convolution's block exponent (the E8M0 scale operand of the block-scaled
// MFMA; f8Exp: its largest |weight| lands in (224, 448]).  A board with a convolution input
// past e4m3's 448 is "hot": the device re-evaluates it on the accurate (split) instance,
// here its outputs are the fp32 forward's (mode 0; the split path is within ~1e-5 of it).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>

#include "ora.h"

namespace ora {

// float -> IEEE binary16 -> float, round to nearest even (v_cvt_f16_f32).
static inline float f16r(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  uint32_t sign = u & 0x80000000u, a = u & 0x7fffffffu;
  if(a >= 0x7f800000u)
    return f;
  float r;
  if(a < 0x38800000u) {  // below 2^-14: binary16 subnormal, quantum 2^-24
    float m;
    memcpy(&m, &a, 4);
    r = nearbyintf(m * 16777216.0f) * (1.0f / 16777216.0f);
  } else {
    uint32_t v = (a + 0xfffu + ((a >> 13) & 1u)) & ~0x1fffu;
    if(v >= 0x47800000u)
      v = 0x7f800000u;
    memcpy(&r, &v, 4);
  }
  uint32_t ru;
  memcpy(&ru, &r, 4);
  ru |= sign;
  memcpy(&r, &ru, 4);
  return r;
}

// float -> OCP e4m3fn -> float, round to nearest even, saturating at +-448 (the
// device's v_cvt_pk_fp8_f32 after a clamp; tools/mfma_f8_probe.hip pins the encoding).
static inline float e4m3r(float f) {
  const float a = fabsf(f);
  float r;
  if(!(a < 448.0f)) {
    r = 448.0f;
  } else if(a < 0.015625f) {  // subnormal: quantum 2^-9
    r = nearbyintf(a * 512.0f) * (1.0f / 512.0f);
  } else {
    int e;
    const float m = frexpf(a, &e);  // a = m 2^e, m in [0.5, 1): 3 mantissa bits below the leading one
    r = ldexpf(nearbyintf(m * 16.0f), e - 4);
    if(r > 448.0f)
      r = 448.0f;
  }
  return std::signbit(f) ? -r : r;
}
static const float F8C_SCALE = 2048.0f;
// Block exponent s of the corrected precision's e4m3 operands: m 2^-s in (224, 448] for
// m > 0 (m = f 2^e, f in [0.5, 1): s = e - 9, or e - 8 when f > 0.875, since 448 = 0.875 2^9),
// 0 for m == 0 (csrc/nn.hip f8Exp, the same integer arithmetic).
static inline int f8Exp(float m) {
  if(!(m > 0.0f))
    return 0;
  int e;
  const float f = frexpf(m, &e);
  int s = e - 9 + (f > 0.875f ? 1 : 0);
  return s < -100 ? -100 : (s > 100 ? 100 : s);
}
// e4m3 of v at block exponent s, back in v's units
static inline float e4m3s(float v, int s) { return ldexpf(e4m3r(ldexpf(v, -s)), s); }

// ---------------------------------------------------------------------------
// SGEMM: C[M][ldc] (+)= A[M][lda] * B, B packed in 16-column panels
// ([panel][K][16], zero padded).  6x16 register tile (12 x 8-wide accumulators),
// K blocked by 256 so a panel slice stays in L1.
typedef float v8 __attribute__((vector_size(32)));
typedef float v8u __attribute__((vector_size(32), aligned(4)));
constexpr int NR = 16, MR = 6, KC = 256;

static inline v8 ld8(const float* p) { return *reinterpret_cast<const v8u*>(p); }
static inline void st8(float* p, v8 v) { *reinterpret_cast<v8u*>(p) = v; }

static void packB(const float* B /*[K][N]*/, int K, int N, std::vector<float>& out) {
  const int np = (N + NR - 1) / NR;
  out.assign((size_t)np * K * NR, 0.0f);
  for(int p = 0; p < np; p++)
    for(int k = 0; k < K; k++)
      for(int j = 0; j < NR && p * NR + j < N; j++)
        out[((size_t)p * K + k) * NR + j] = B[(size_t)k * N + p * NR + j];
}

static void sgemm(int M, int N, int K, const float* A, int lda, const float* Bp, float* C, int ldc, bool accumulate) {
  const int np = (N + NR - 1) / NR;
  for(int k0 = 0; k0 < K; k0 += KC) {
    const int kc = K - k0 < KC ? K - k0 : KC;
    const bool acc0 = accumulate || k0 > 0;
    for(int p = 0; p < np; p++) {
      const float* bp = Bp + ((size_t)p * K + k0) * NR;
      const int nw = N - p * NR < NR ? N - p * NR : NR;
      for(int m0 = 0; m0 < M; m0 += MR) {
        const int mr = M - m0 < MR ? M - m0 : MR;
        v8 c[MR][2];
        for(int i = 0; i < MR; i++)
          c[i][0] = c[i][1] = v8{0, 0, 0, 0, 0, 0, 0, 0};
        const float* a = A + (size_t)m0 * lda + k0;
        if(mr == MR) {
          for(int k = 0; k < kc; k++) {
            const v8 b0 = ld8(bp + (size_t)k * NR), b1 = ld8(bp + (size_t)k * NR + 8);
            for(int i = 0; i < MR; i++) {
              const float av = a[(size_t)i * lda + k];
              c[i][0] += av * b0;
              c[i][1] += av * b1;
            }
          }
        } else {
          for(int k = 0; k < kc; k++) {
            const v8 b0 = ld8(bp + (size_t)k * NR), b1 = ld8(bp + (size_t)k * NR + 8);
            for(int i = 0; i < mr; i++) {
              const float av = a[(size_t)i * lda + k];
              c[i][0] += av * b0;
              c[i][1] += av * b1;
            }
          }
        }
        for(int i = 0; i < mr; i++) {
          float* cr = C + (size_t)(m0 + i) * ldc + p * NR;
          if(nw == NR) {
            if(acc0) {
              st8(cr, ld8(cr) + c[i][0]);
              st8(cr + 8, ld8(cr + 8) + c[i][1]);
            } else {
              st8(cr, c[i][0]);
              st8(cr + 8, c[i][1]);
            }
          } else {
            float t[NR];
            st8(t, c[i][0]);
            st8(t + 8, c[i][1]);
            for(int j = 0; j < nw; j++)
              cr[j] = acc0 ? cr[j] + t[j] : t[j];
          }
        }
      }
    }
  }
}

// B[k = (ky, kx, ci)][co] from w[co][ci][ky][kx]
void PackedConv::pack() {
  const int K = ky * kx * cin;
  std::vector<float> B((size_t)K * cout), B16((size_t)K * cout), BC((size_t)3 * K * cout);
  float mx = 0.0f;  // the convolution's block exponent (corrected precision)
  for(float v : w)
    mx = fmaxf(mx, fabsf(v));
  const int sw = f8Exp(mx);
  for(int co = 0; co < cout; co++) {
    for(int ci = 0; ci < cin; ci++)
      for(int y = 0; y < ky; y++)
        for(int x = 0; x < kx; x++) {
          const float v = w[(((size_t)co * cin + ci) * ky + y) * kx + x];
          const size_t k = ((size_t)y * kx + x) * cin + ci;
          B[k * cout + co] = v;
          B16[k * cout + co] = f16r(v);
          BC[k * cout + co] = f16r(v);
          BC[(K + k) * cout + co] = e4m3s((v - f16r(v)) * F8C_SCALE, sw) / F8C_SCALE;
          BC[(2 * K + k) * cout + co] = e4m3s(f16r(v), sw);
        }
  }
  packB(B.data(), K, cout, p32);
  packB(B16.data(), K, cout, p16);
  packB(BC.data(), 3 * K, cout, pC);
}

// ConvLayer::apply: "same" convolution, zero outside the board (the masked input is
// zero there in the reference, so the mask needs no separate handling here).
void convApply(const NNBatch& b, const PackedConv& cv, const float* in, float* out, bool accumulate) {
  const int A = b.A, rows = b.n * A, K = cv.ky * cv.kx * cv.cin;
  const int ry = cv.ky / 2, rx = cv.kx / 2;
  static const int emu = getenv("ORA_EMU") ? atoi(getenv("ORA_EMU")) : 3;
  const bool fp16 = b.mode == 1, corr = b.mode == 2;
  const float* Bp = corr ? cv.pC.data() : ((fp16 && (emu & 1)) ? cv.p16.data() : cv.p32.data());
  const int KC3 = corr ? 3 * K : K;  // corrected: im2col columns [fp16(x) | e4m3(x) | e4m3(lo(x) 2^11) / 2^11]
  constexpr int CH = 48;  // rows per im2col chunk
  const int chunks = (rows + CH - 1) / CH;
  if(corr && b.hot)  // corrected: boards whose convolution input passes e4m3's range
    for(int brd = 0; brd < b.n; brd++)
      for(size_t i = 0; i < (size_t)A * cv.cin; i++)
        if(!(fabsf(in[(size_t)brd * A * cv.cin + i]) <= 448.0f)) {
          b.hot[brd] = 1;
          break;
        }
#pragma omp parallel for schedule(dynamic, 1) num_threads(b.threads > 0 ? b.threads : 1)
  for(int ch = 0; ch < chunks; ch++) {
    const int r0 = ch * CH, r1 = r0 + CH < rows ? r0 + CH : rows;
    std::vector<float> col((size_t)(r1 - r0) * KC3);
    for(int r = r0; r < r1; r++) {
      const int brd = r / A, p = r - brd * A, y = p / b.X, x = p - y * b.X;
      float* cr = col.data() + (size_t)(r - r0) * KC3;
      for(int dy = 0; dy < cv.ky; dy++)
        for(int dx = 0; dx < cv.kx; dx++) {
          const int yy = y + dy - ry, xx = x + dx - rx;
          float* dst = cr + ((size_t)dy * cv.kx + dx) * cv.cin;
          if(yy < 0 || yy >= b.Y || xx < 0 || xx >= b.X) {
            memset(dst, 0, sizeof(float) * cv.cin);
            if(corr) {
              memset(dst + K, 0, sizeof(float) * cv.cin);
              memset(dst + 2 * K, 0, sizeof(float) * cv.cin);
            }
          } else {
            const float* src = in + ((size_t)brd * A + yy * b.X + xx) * cv.cin;
            if(corr) {
              for(int c = 0; c < cv.cin; c++) {
                const float h = f16r(src[c]);
                dst[c] = h;
                dst[K + c] = e4m3r(h);
                dst[2 * K + c] = e4m3r((src[c] - h) * F8C_SCALE) / F8C_SCALE;
              }
            } else if(fp16 && (emu & 2)) {
              for(int c = 0; c < cv.cin; c++)
                dst[c] = f16r(src[c]);
            } else {
              memcpy(dst, src, sizeof(float) * cv.cin);
            }
          }
        }
    }
    sgemm(r1 - r0, cv.cout, KC3, col.data(), KC3, Bp, out + (size_t)r0 * cv.cout, cv.cout, accumulate);
  }
}

void bnAct(const NNBatch& b, int C, const float* s, const float* bias, const float* in, int ldIn, float* out,
           bool relu, const float* perBoard) {
  const int rows = b.n * b.A;
  for(int r = 0; r < rows; r++) {
    const int brd = r / b.A;
    const float m = b.mask ? b.mask[r] : 1.0f;
    const float* pb = perBoard ? perBoard + (size_t)brd * C : nullptr;
    for(int c = 0; c < C; c++) {
      float x = in[(size_t)r * ldIn + c];
      if(pb)
        x += pb[c];
      float v = x * s[c] + bias[c];
      if(relu)
        v = v > 0.0f ? v : 0.0f;
      out[(size_t)r * C + c] = m == 1.0f ? v : 0.0f;
    }
  }
}

void gpoolRows(const NNBatch& b, int C, const float* in, int ldIn, float* out, bool valueHead) {
  for(int brd = 0; brd < b.n; brd++) {
    float div = 0.0f;
    for(int p = 0; p < b.A; p++)
      div += b.mask ? b.mask[(size_t)brd * b.A + p] : 1.0f;
    const float sqrtdiv = sqrtf(div);
    for(int c = 0; c < C; c++) {
      float s = 0.0f, m = -1.0f;
      for(int p = 0; p < b.A; p++) {
        const float x = in[((size_t)brd * b.A + p) * ldIn + c];
        const float mv = b.mask ? b.mask[(size_t)brd * b.A + p] : 1.0f;
        s += x;
        m = m > x + (mv - 1.0f) ? m : x + (mv - 1.0f);
      }
      const float mean = s / div;
      float* o = out + (size_t)brd * 3 * C;
      o[c] = mean;
      o[C + c] = mean * (sqrtdiv - 14.0f) * 0.1f;
      o[2 * C + c] = valueHead ? mean * ((sqrtdiv - 14.0f) * (sqrtdiv - 14.0f) * 0.01f - 0.1f) : m;
    }
  }
}

// out[n][O] = in[n][I] * W^T (W [O][I]) (+ bias)
static void matmulRows(int n, int I, int O, const float* in, const float* W, const float* bias, float* out) {
  for(int i = 0; i < n; i++)
    for(int o = 0; o < O; o++) {
      float s = bias ? bias[o] : 0.0f;
      for(int k = 0; k < I; k++)
        s += W[(size_t)o * I + k] * in[(size_t)i * I + k];
      out[(size_t)i * O + o] = s;
    }
}

// Widths come from the convolutions: trunk W = conv2.cout (bottleneck: convP.cin);
// regular: conv1 W -> M, conv2 M -> W; gpool: conv1 W -> [r | g] (Cr + Cg), conv2 Cr -> W.
void blockApply(const NNBatch& b, const Model::Block& blk, float* x) {
  const size_t rows = (size_t)b.n * b.A;
  if(blk.kind >= 2) {
    const int W = blk.convP.cin, mid = blk.convP.cout;
    std::vector<float> a(rows * W), y(rows * mid), aq(rows * mid);
    bnAct(b, W, blk.bnPs.data(), blk.bnPb.data(), x, W, a.data(), true);
    convApply(b, blk.convP, a.data(), y.data(), false);
    for(const Model::Block& in : blk.inner)
      blockApply(b, in, y.data());
    bnAct(b, mid, blk.bnQs.data(), blk.bnQb.data(), y.data(), mid, aq.data(), true);
    convApply(b, blk.convQ, aq.data(), x, true);
    return;
  }
  const int W = blk.conv1.cin, M = blk.conv2.cin;
  const bool split = blk.conv1g.cout > 0;  // separate gpool conv (any kernel sizes: testnn.cpp KAT)
  const int H = blk.conv1.cout + (split ? blk.conv1g.cout : 0);
  std::vector<float> a(rows * W), h(rows * blk.conv1.cout), a2(rows * M), hg;
  bnAct(b, W, blk.bn1s.data(), blk.bn1b.data(), x, W, a.data(), true);
  convApply(b, blk.conv1, a.data(), h.data(), false);
  if(blk.kind == 0) {
    bnAct(b, M, blk.bn2s.data(), blk.bn2b.data(), h.data(), H, a2.data(), true);
  } else {
    const int Cr = M, Cg = H - M;
    const float* graw = h.data() + Cr;
    int gld = H;
    if(split) {
      hg.resize(rows * Cg);
      convApply(b, blk.conv1g, a.data(), hg.data(), false);
      graw = hg.data();
      gld = Cg;
    }
    const int rld = split ? Cr : H;
    std::vector<float> g(rows * Cg), pooled((size_t)b.n * 3 * Cg), bias((size_t)b.n * Cr);
    bnAct(b, Cg, blk.bngs.data(), blk.bngb.data(), graw, gld, g.data(), true);
    gpoolRows(b, Cg, g.data(), Cg, pooled.data(), false);
    matmulRows(b.n, 3 * Cg, Cr, pooled.data(), blk.linG.data(), nullptr, bias.data());
    bnAct(b, Cr, blk.bn2s.data(), blk.bn2b.data(), h.data(), rld, a2.data(), true, bias.data());
  }
  convApply(b, blk.conv2, a2.data(), x, true);
}

// ---------------------------------------------------------------------------
// CFNN v1 / v2 (katacoffee_amd/csrc/model.h)
namespace {
struct Reader {
  const char* p;
  size_t len, pos = 0;
  bool ok = true;
  bool raw(void* dst, size_t bytes) {
    if(pos + bytes > len) {
      ok = false;
      return false;
    }
    memcpy(dst, p + pos, bytes);
    pos += bytes;
    return true;
  }
  void rd(std::vector<float>& v, size_t n) {
    v.assign(n, 0.0f);
    raw(v.data(), 4 * n);
  }
  void conv(PackedConv& c, int ky, int kx, int cin, int cout) {
    c.ky = ky;
    c.kx = kx;
    c.cin = cin;
    c.cout = cout;
    rd(c.w, (size_t)cout * cin * ky * kx);
  }
};

void readBlock(Reader& r, Model::Block& b, int kind, int W, int Cg, int mid) {  // CFNN tensor order
  b.kind = kind;
  if(kind >= 2) {
    r.rd(b.bnPs, W);
    r.rd(b.bnPb, W);
    r.conv(b.convP, 1, 1, W, mid);
    b.inner.resize(2);
    readBlock(r, b.inner[0], kind == 3 ? 1 : 0, mid, Cg, 0);
    readBlock(r, b.inner[1], 0, mid, Cg, 0);
    r.rd(b.bnQs, mid);
    r.rd(b.bnQb, mid);
    r.conv(b.convQ, 1, 1, mid, W);
    return;
  }
  const int Cr = kind == 1 ? W - Cg : W;
  r.rd(b.bn1s, W);
  r.rd(b.bn1b, W);
  if(kind == 0) {
    r.conv(b.conv1, 3, 3, W, W);
  } else {
    PackedConv cr, cg;
    r.conv(cr, 3, 3, W, Cr);
    r.conv(cg, 3, 3, W, Cg);
    b.conv1 = cr;
    b.conv1.cout = W;
    b.conv1.w.insert(b.conv1.w.end(), cg.w.begin(), cg.w.end());
    r.rd(b.bngs, Cg);
    r.rd(b.bngb, Cg);
    r.rd(b.linG, (size_t)Cr * 3 * Cg);
  }
  r.rd(b.bn2s, Cr);
  r.rd(b.bn2b, Cr);
  r.conv(b.conv2, 3, 3, Cr, W);
}

void packBlock(Model::Block& b) {
  if(b.kind >= 2) {
    b.convP.pack();
    b.convQ.pack();
    for(auto& in : b.inner)
      packBlock(in);
  } else {
    b.conv1.pack();
    b.conv2.pack();
  }
}
}  // namespace

bool modelLoad(const char* path, Model& m) {
  FILE* f = fopen(path, "rb");
  if(!f)
    return false;
  std::vector<char> data;
  char buf[1 << 16];
  size_t got;
  while((got = fread(buf, 1, sizeof(buf), f)) > 0)
    data.insert(data.end(), buf, buf + got);
  fclose(f);
  Reader r{data.data(), data.size()};
  char magic[4];
  int32_t ver = 0;
  if(!r.raw(magic, 4) || memcmp(magic, "CFNN", 4) != 0 || !r.raw(&ver, 4) || (ver != 1 && ver != 2))
    return false;
  int32_t hdr[10] = {0};
  if(!r.raw(hdr, 4 * (ver == 1 ? 9 : 10)))
    return false;
  ModelCfg& c = m.cfg;
  c.cin = hdr[0]; c.gin = hdr[1]; c.C = hdr[2]; c.Cg = hdr[3]; c.p1 = hdr[4]; c.g1 = hdr[5];
  c.v1 = hdr[6]; c.v2 = hdr[7]; c.nblocks = hdr[8]; c.mid = ver == 2 ? hdr[9] : 0;
  if(c.nblocks < 1 || c.nblocks > 64 || !r.raw(c.kinds, 4 * (size_t)c.nblocks))
    return false;
  const int C = c.C;
  r.conv(m.convInit, 3, 3, c.cin, C);
  r.rd(m.globInit, (size_t)C * c.gin);
  m.blocks.resize(c.nblocks);
  for(int i = 0; i < c.nblocks; i++) {
    if(c.kinds[i] < 0 || c.kinds[i] > 3 || (c.kinds[i] >= 2 && c.mid <= 0))
      return false;
    readBlock(r, m.blocks[i], c.kinds[i], C, c.Cg, c.mid);
  }
  r.rd(m.tips, C);
  r.rd(m.tipb, C);
  std::vector<float> pConv1, pConvG, vConv1;
  r.rd(pConv1, (size_t)c.p1 * C);
  r.rd(pConvG, (size_t)c.g1 * C);
  r.rd(m.pBiasG, c.g1);
  r.rd(m.pLinG, (size_t)c.p1 * 3 * c.g1);
  r.rd(m.pBias2, c.p1);
  r.rd(m.pConv2, (size_t)4 * c.p1);
  r.rd(vConv1, (size_t)c.v1 * C);
  r.rd(m.vBias1, c.v1);
  r.rd(m.vLin2, (size_t)c.v2 * 3 * c.v1);
  r.rd(m.vB2, c.v2);
  r.rd(m.vLin3, (size_t)2 * c.v2);
  r.rd(m.vB3, 2);
  r.rd(m.vLinM, (size_t)2 * c.v2);
  r.rd(m.vBM, 2);
  if(!r.ok || r.pos != r.len)
    return false;
  m.head.ky = m.head.kx = 1;
  m.head.cin = C;
  m.head.cout = c.p1 + c.g1 + c.v1;
  m.head.w = pConv1;
  m.head.w.insert(m.head.w.end(), pConvG.begin(), pConvG.end());
  m.head.w.insert(m.head.w.end(), vConv1.begin(), vConv1.end());
  m.convInit.pack();
  m.head.pack();
  for(auto& b : m.blocks)
    packBlock(b);
  return true;
}

bool blockFromBlob(const float* blob, size_t count, int kind, int W, int Cg, int mid, Model::Block& b) {
  Reader r{reinterpret_cast<const char*>(blob), count * 4};
  readBlock(r, b, kind, W, Cg, mid);
  if(!r.ok || r.pos != r.len)
    return false;
  packBlock(b);
  return true;
}

void nnForward(const Model& m, int X, int Y, int n, const float* bin, const float* glob, float* policy,
               float* value, float* misc, int mode, int threads) {
  const ModelCfg& c = m.cfg;
  const int A = X * Y, C = c.C;
  std::vector<int> hot(mode == 2 ? n : 0, 0);
  NNBatch b{n, X, Y, A, nullptr, mode, threads, mode == 2 ? hot.data() : nullptr};
  const size_t rows = (size_t)n * A;
  std::vector<float> in(rows * c.cin), x(rows * C), a(rows * C);
  for(int i = 0; i < n; i++)
    for(int ch = 0; ch < c.cin; ch++)
      for(int p = 0; p < A; p++)
        in[((size_t)i * A + p) * c.cin + ch] = bin[((size_t)i * c.cin + ch) * A + p];
  convApply(b, m.convInit, in.data(), x.data(), false);
  // + linear_global(input_global) broadcast (Trunk::apply :1218-1220)
  for(int i = 0; i < n; i++)
    for(int co = 0; co < C; co++) {
      float s = 0.0f;
      for(int gi = 0; gi < c.gin; gi++)
        s += m.globInit[(size_t)co * c.gin + gi] * glob[(size_t)i * c.gin + gi];
      for(int p = 0; p < A; p++)
        x[((size_t)i * A + p) * C + co] += s;
    }
  for(const Model::Block& blk : m.blocks)
    blockApply(b, blk, x.data());
  bnAct(b, C, m.tips.data(), m.tipb.data(), x.data(), C, a.data(), true);
  // heads: one 1x1 conv C -> [p1 | g1 | v1]
  const int HW = c.p1 + c.g1 + c.v1;
  std::vector<float> h(rows * HW);
  convApply(b, m.head, a.data(), h.data(), false);
  // policy (PolicyHead::apply :1265-1299)
  std::vector<float> pg(rows * c.g1), pp((size_t)n * 3 * c.g1), pb((size_t)n * c.p1);
  for(size_t r = 0; r < rows; r++)
    for(int o = 0; o < c.g1; o++) {
      const float v = h[r * HW + c.p1 + o] + m.pBiasG[o];
      pg[r * c.g1 + o] = v > 0.0f ? v : 0.0f;
    }
  gpoolRows(b, c.g1, pg.data(), c.g1, pp.data(), false);
  matmulRows(n, 3 * c.g1, c.p1, pp.data(), m.pLinG.data(), nullptr, pb.data());
  std::vector<float> p((size_t)c.p1);
  for(int i = 0; i < n; i++)
    for(int q = 0; q < A; q++) {
      const size_t r = (size_t)i * A + q;
      for(int o = 0; o < c.p1; o++) {
        const float v = h[r * HW + o] + pb[(size_t)i * c.p1 + o] + m.pBias2[o];
        p[o] = v > 0.0f ? v : 0.0f;
      }
      for(int d = 0; d < 4; d++) {
        float s = 0.0f;
        for(int k = 0; k < c.p1; k++)
          s += m.pConv2[(size_t)d * c.p1 + k] * p[k];
        policy[((size_t)i * 4 + d) * A + q] = s;
      }
    }
  // value (ValueHead::apply :1341-1377)
  std::vector<float> v(rows * c.v1), vp((size_t)n * 3 * c.v1), vh((size_t)n * c.v2);
  for(size_t r = 0; r < rows; r++)
    for(int o = 0; o < c.v1; o++) {
      const float t = h[r * HW + c.p1 + c.g1 + o] + m.vBias1[o];
      v[r * c.v1 + o] = t > 0.0f ? t : 0.0f;
    }
  gpoolRows(b, c.v1, v.data(), c.v1, vp.data(), true);
  matmulRows(n, 3 * c.v1, c.v2, vp.data(), m.vLin2.data(), m.vB2.data(), vh.data());
  for(float& t : vh)
    t = t > 0.0f ? t : 0.0f;
  matmulRows(n, c.v2, 2, vh.data(), m.vLin3.data(), m.vB3.data(), value);
  matmulRows(n, c.v2, 2, vh.data(), m.vLinM.data(), m.vBM.data(), misc);
  if(mode == 2) {
    // hot boards: the accurate re-evaluation, i.e. the fp32 forward's outputs
    std::vector<float> hb, hg;
    std::vector<int> idx;
    for(int i = 0; i < n; i++)
      if(hot[i]) {
        idx.push_back(i);
        hb.insert(hb.end(), bin + (size_t)i * c.cin * A, bin + (size_t)(i + 1) * c.cin * A);
        hg.insert(hg.end(), glob + (size_t)i * c.gin, glob + (size_t)(i + 1) * c.gin);
      }
    if(!idx.empty()) {
      const int k = (int)idx.size();
      std::vector<float> p((size_t)k * 4 * A), v((size_t)k * 2), mi((size_t)k * 2);
      nnForward(m, X, Y, k, hb.data(), hg.data(), p.data(), v.data(), mi.data(), 0, threads);
      for(int j = 0; j < k; j++) {
        memcpy(policy + (size_t)idx[j] * 4 * A, &p[(size_t)j * 4 * A], sizeof(float) * 4 * A);
        memcpy(value + (size_t)idx[j] * 2, &v[(size_t)j * 2], sizeof(float) * 2);
        memcpy(misc + (size_t)idx[j] * 2, &mi[(size_t)j * 2], sizeof(float) * 2);
      }
    }
  }
}

}  // namespace ora
