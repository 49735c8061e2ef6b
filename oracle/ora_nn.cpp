// ORACLE (test infrastructure only) — fp32 residual-net forward with the Eigen
// CPU backend's semantics (eigenbackend.cpp):
//   ConvLayer        :270-680  ("same" 3x3 / 1x1 convolution, NHWC)
//   BatchNormLayer   :684-734  (merged scale/bias, then activation, then mask)
//   poolRowsGPool    :141-166  (mean, mean*(sqrt(area)-14)/10, max)
//   poolRowsValueHead:168-186  (mean, mean*(sqrt(area)-14)/10, mean*((sqrt-14)^2/100-0.1))
//   ResidualBlock    :888-931, GlobalPoolingResidualBlock :935-1015
//   Trunk :1169-1227, PolicyHead :1229-1299 (Coffee: 4 direction logits, no pass),
//   ValueHead :1301-1377 (Coffee: win/loss logits + 2 misc).
// Boards always fill the NN input here (nnLen == board size), so the mask is 1.
// mode 1 rounds every convolution weight and convolution input to fp16 (RNE)
// and the residual trunk to fp16 (RNE) after the stem and after every block,
// exactly where the HIP kernel does, to compare with it at accumulation-order
// precision.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>

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

bool modelLoad(const char* path, Model& m) {
  FILE* f = fopen(path, "rb");
  if(!f)
    return false;
  char magic[4];
  int32_t ver;
  bool ok = fread(magic, 1, 4, f) == 4 && memcmp(magic, "CFNN", 4) == 0 && fread(&ver, 4, 1, f) == 1 && ver == 1;
  int32_t hdr[9];
  ok = ok && fread(hdr, 4, 9, f) == 9;
  if(!ok) {
    fclose(f);
    return false;
  }
  ModelCfg& c = m.cfg;
  c.cin = hdr[0]; c.gin = hdr[1]; c.C = hdr[2]; c.Cg = hdr[3]; c.p1 = hdr[4]; c.g1 = hdr[5];
  c.v1 = hdr[6]; c.v2 = hdr[7]; c.nblocks = hdr[8];
  if(c.nblocks > 32 || fread(c.kinds, 4, c.nblocks, f) != (size_t)c.nblocks) {
    fclose(f);
    return false;
  }
  auto rd = [&](std::vector<float>& v, size_t n) {
    v.resize(n);
    if(fread(v.data(), 4, n, f) != n)
      ok = false;
  };
  const int C = c.C, Cr = c.C - c.Cg;
  rd(m.convInit, (size_t)C * c.cin * 9);
  rd(m.globInit, (size_t)C * c.gin);
  m.blocks.resize(c.nblocks);
  for(int i = 0; i < c.nblocks; i++) {
    Model::Block& b = m.blocks[i];
    b.kind = c.kinds[i];
    rd(b.bn1s, C);
    rd(b.bn1b, C);
    if(b.kind == 0) {
      rd(b.conv1, (size_t)C * C * 9);
      rd(b.bn2s, C);
      rd(b.bn2b, C);
      rd(b.conv2, (size_t)C * C * 9);
    } else {
      rd(b.conv1, (size_t)Cr * C * 9);
      rd(b.conv1g, (size_t)c.Cg * C * 9);
      rd(b.bngs, c.Cg);
      rd(b.bngb, c.Cg);
      rd(b.linG, (size_t)Cr * 3 * c.Cg);
      rd(b.bn2s, Cr);
      rd(b.bn2b, Cr);
      rd(b.conv2, (size_t)C * Cr * 9);
    }
  }
  rd(m.tips, C);
  rd(m.tipb, C);
  rd(m.pConv1, (size_t)c.p1 * C);
  rd(m.pConvG, (size_t)c.g1 * C);
  rd(m.pBiasG, c.g1);
  rd(m.pLinG, (size_t)c.p1 * 3 * c.g1);
  rd(m.pBias2, c.p1);
  rd(m.pConv2, (size_t)4 * c.p1);
  rd(m.vConv1, (size_t)c.v1 * C);
  rd(m.vBias1, c.v1);
  rd(m.vLin2, (size_t)c.v2 * 3 * c.v1);
  rd(m.vB2, c.v2);
  rd(m.vLin3, (size_t)2 * c.v2);
  rd(m.vB3, 2);
  rd(m.vLinM, (size_t)2 * c.v2);
  rd(m.vBM, 2);
  fclose(f);
  return ok;
}

namespace {

struct Ctx {
  int X, Y, A;
  bool bf;
};

// 3x3 "same" convolution, NHWC single board: out[a][co] (+)= sum in[nb][ci]*w[co][ci][ky][kx]
// Weight layout [Cout][Cin][3][3] (ConvLayerDesc, desc.h).  The k-sum is
// ordered tap-major, channel-minor as the GPU kernel's K steps are.
void conv3(const Ctx& cx, const float* in, int cin, const float* w, int cout, float* out, bool accumulate) {
  std::vector<float> wt((size_t)9 * cin * cout);  // [tap][ci][co]
  for(int co = 0; co < cout; co++)
    for(int ci = 0; ci < cin; ci++)
      for(int t = 0; t < 9; t++) {
        float v = w[((size_t)co * cin + ci) * 9 + t];
        wt[((size_t)t * cin + ci) * cout + co] = cx.bf ? f16r(v) : v;
      }
  std::vector<float> acc((size_t)cout);
  for(int y = 0; y < cx.Y; y++)
    for(int x = 0; x < cx.X; x++) {
      std::fill(acc.begin(), acc.end(), 0.0f);
      for(int t = 0; t < 9; t++) {
        int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        if(yy < 0 || yy >= cx.Y || xx < 0 || xx >= cx.X)
          continue;
        const float* ip = in + (size_t)(yy * cx.X + xx) * cin;
        const float* wp = wt.data() + (size_t)t * cin * cout;
        for(int ci = 0; ci < cin; ci++) {
          float v = ip[ci];
          if(cx.bf)
            v = f16r(v);
          const float* wr = wp + (size_t)ci * cout;
          for(int co = 0; co < cout; co++)
            acc[co] += v * wr[co];
        }
      }
      float* op = out + (size_t)(y * cx.X + x) * cout;
      for(int co = 0; co < cout; co++)
        op[co] = accumulate ? op[co] + acc[co] : acc[co];
    }
}

// 1x1 convolution, weight [Cout][Cin].
void conv1(const Ctx& cx, const float* in, int cin, const float* w, int cout, float* out, bool roundBf) {
  for(int a = 0; a < cx.A; a++)
    for(int co = 0; co < cout; co++) {
      float s = 0.0f;
      for(int ci = 0; ci < cin; ci++) {
        float v = in[(size_t)a * cin + ci], ww = w[(size_t)co * cin + ci];
        if(roundBf) {
          v = f16r(v);
          ww = f16r(ww);
        }
        s += v * ww;
      }
      out[(size_t)a * cout + co] = s;
    }
}

void bnRelu(const Ctx& cx, const float* in, int C, const float* s, const float* b, float* out) {
  for(int a = 0; a < cx.A; a++)
    for(int c = 0; c < C; c++) {
      float v = in[(size_t)a * C + c] * s[c] + b[c];
      out[(size_t)a * C + c] = v > 0.0f ? v : 0.0f;
    }
}

void gpool(const Ctx& cx, const float* in, int C, float* out /*3C*/, bool valueHead) {
  float sq = sqrtf((float)cx.A) - 14.0f;
  for(int c = 0; c < C; c++) {
    float sum = 0.0f, mx = 0.0f;  // inputs are post-ReLU (>= 0) and mask == 1
    for(int a = 0; a < cx.A; a++) {
      float v = in[(size_t)a * C + c];
      sum += v;
      if(v > mx)
        mx = v;
    }
    float mean = sum / (float)cx.A;
    out[c] = mean;
    out[C + c] = mean * (sq / 10.0f);
    out[2 * C + c] = valueHead ? mean * ((sq * sq) / 100.0f - 0.1f) : mx;
  }
}

void forwardOne(const Model& m, const Ctx& cx, const float* binNCHW, const float* glob, float* policy,
                float* value, float* misc) {
  const ModelCfg& c = m.cfg;
  const int A = cx.A, C = c.C, Cr = c.C - c.Cg;
  std::vector<float> in((size_t)A * c.cin), x((size_t)A * C), a((size_t)A * C), h((size_t)A * C),
    g((size_t)A * C);
  for(int ch = 0; ch < c.cin; ch++)
    for(int p = 0; p < A; p++)
      in[(size_t)p * c.cin + ch] = binNCHW[(size_t)ch * A + p];
  conv3(cx, in.data(), c.cin, m.convInit.data(), C, x.data(), false);
  for(int co = 0; co < C; co++) {
    float s = 0.0f;
    for(int gi = 0; gi < c.gin; gi++)
      s += m.globInit[(size_t)co * c.gin + gi] * glob[gi];
    for(int p = 0; p < A; p++)
      x[(size_t)p * C + co] += s;
  }
  auto roundTrunk = [&]() {
    if(cx.bf)
      for(float& v : x)
        v = f16r(v);
  };
  roundTrunk();
  std::vector<float> pooled(3 * (size_t)C), bias(C);
  for(const Model::Block& b : m.blocks) {
    bnRelu(cx, x.data(), C, b.bn1s.data(), b.bn1b.data(), a.data());
    if(b.kind == 0) {
      conv3(cx, a.data(), C, b.conv1.data(), C, h.data(), false);
      bnRelu(cx, h.data(), C, b.bn2s.data(), b.bn2b.data(), a.data());
      conv3(cx, a.data(), C, b.conv2.data(), C, x.data(), true);
    } else {
      conv3(cx, a.data(), C, b.conv1.data(), Cr, h.data(), false);
      conv3(cx, a.data(), C, b.conv1g.data(), c.Cg, g.data(), false);
      bnRelu(cx, g.data(), c.Cg, b.bngs.data(), b.bngb.data(), g.data());
      gpool(cx, g.data(), c.Cg, pooled.data(), false);
      for(int o = 0; o < Cr; o++) {
        float s = 0.0f;
        for(int i = 0; i < 3 * c.Cg; i++)
          s += b.linG[(size_t)o * 3 * c.Cg + i] * pooled[i];
        bias[o] = s;
      }
      for(int p = 0; p < A; p++)
        for(int o = 0; o < Cr; o++)
          h[(size_t)p * Cr + o] += bias[o];
      bnRelu(cx, h.data(), Cr, b.bn2s.data(), b.bn2b.data(), a.data());
      conv3(cx, a.data(), Cr, b.conv2.data(), C, x.data(), true);
    }
    roundTrunk();
  }
  bnRelu(cx, x.data(), C, m.tips.data(), m.tipb.data(), a.data());
  // Policy head
  std::vector<float> p((size_t)A * c.p1), pg((size_t)A * c.g1), pp(3 * (size_t)c.g1), pb(c.p1);
  conv1(cx, a.data(), C, m.pConv1.data(), c.p1, p.data(), cx.bf);
  conv1(cx, a.data(), C, m.pConvG.data(), c.g1, pg.data(), cx.bf);
  for(int q = 0; q < A; q++)
    for(int o = 0; o < c.g1; o++) {
      float v = pg[(size_t)q * c.g1 + o] + m.pBiasG[o];
      pg[(size_t)q * c.g1 + o] = v > 0.0f ? v : 0.0f;
    }
  gpool(cx, pg.data(), c.g1, pp.data(), false);
  for(int o = 0; o < c.p1; o++) {
    float s = 0.0f;
    for(int i = 0; i < 3 * c.g1; i++)
      s += m.pLinG[(size_t)o * 3 * c.g1 + i] * pp[i];
    pb[o] = s;
  }
  for(int q = 0; q < A; q++)
    for(int o = 0; o < c.p1; o++) {
      float v = p[(size_t)q * c.p1 + o] + pb[o] + m.pBias2[o];
      p[(size_t)q * c.p1 + o] = v > 0.0f ? v : 0.0f;
    }
  for(int d = 0; d < 4; d++)
    for(int q = 0; q < A; q++) {
      float s = 0.0f;
      for(int i = 0; i < c.p1; i++)
        s += m.pConv2[(size_t)d * c.p1 + i] * p[(size_t)q * c.p1 + i];
      policy[(size_t)d * A + q] = s;
    }
  // Value head
  std::vector<float> v((size_t)A * c.v1), vp(3 * (size_t)c.v1), vh(c.v2);
  conv1(cx, a.data(), C, m.vConv1.data(), c.v1, v.data(), cx.bf);
  for(int q = 0; q < A; q++)
    for(int o = 0; o < c.v1; o++) {
      float t = v[(size_t)q * c.v1 + o] + m.vBias1[o];
      v[(size_t)q * c.v1 + o] = t > 0.0f ? t : 0.0f;
    }
  gpool(cx, v.data(), c.v1, vp.data(), true);
  for(int o = 0; o < c.v2; o++) {
    float s = m.vB2[o];
    for(int i = 0; i < 3 * c.v1; i++)
      s += m.vLin2[(size_t)o * 3 * c.v1 + i] * vp[i];
    vh[o] = s > 0.0f ? s : 0.0f;
  }
  for(int o = 0; o < 2; o++) {
    float s = m.vB3[o], t = m.vBM[o];
    for(int i = 0; i < c.v2; i++) {
      s += m.vLin3[(size_t)o * c.v2 + i] * vh[i];
      t += m.vLinM[(size_t)o * c.v2 + i] * vh[i];
    }
    value[o] = s;
    misc[o] = t;
  }
}

}  // namespace

void nnForward(const Model& m, int X, int Y, int n, const float* bin, const float* glob, float* policy,
               float* value, float* misc, int mode, int threads) {
  Ctx cx{X, Y, X * Y, mode == 1};
  const int A = X * Y, cin = m.cfg.cin, gin = m.cfg.gin;
  auto work = [&](int lo, int hi) {
    for(int i = lo; i < hi; i++)
      forwardOne(m, cx, bin + (size_t)i * cin * A, glob + (size_t)i * gin, policy + (size_t)i * 4 * A,
                 value + (size_t)i * 2, misc + (size_t)i * 2);
  };
  if(threads <= 1 || n <= 1) {
    work(0, n);
    return;
  }
  std::vector<std::thread> ts;
  for(int t = 0; t < threads; t++) {
    int lo = (int)((int64_t)n * t / threads), hi = (int)((int64_t)n * (t + 1) / threads);
    if(hi > lo)
      ts.emplace_back(work, lo, hi);
  }
  for(auto& th : ts)
    th.join();
}

}  // namespace ora
