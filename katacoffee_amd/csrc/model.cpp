#include "model.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "detmath.h"

namespace kc {

ModelCfg modelCfgByName(const std::string& name) {
  ModelCfg c;
  if(name == "b6c96") {
    // modelconfigs.py:129-152
    c.C = 96; c.Cg = 32; c.p1 = 32; c.g1 = 32; c.v1 = 32; c.v2 = 64;
    c.kinds = {0, 0, 1, 0, 1, 0};
  } else if(name == "b10c128") {
    // modelconfigs.py:156-180
    c.C = 128; c.Cg = 32; c.p1 = 32; c.g1 = 32; c.v1 = 32; c.v2 = 80;
    c.kinds = {0, 0, 0, 0, 1, 0, 0, 1, 0, 0};
  } else if(name == "b18c384nbt") {
    // modelconfigs.py:887-924: 18 "bottlenest2" blocks (every third from rconv3 with a
    // gpool inner block), trunk 384, bottleneck 192, gpool 64
    c.C = 384; c.mid = 192; c.Cg = 64; c.p1 = 48; c.g1 = 48; c.v1 = 96; c.v2 = 128;
    c.kinds = {2, 2, 3, 2, 2, 3, 2, 2, 3, 2, 2, 3, 2, 2, 3, 2, 2, 2};
  } else if(name == "b2c32nbt") {
    // small nested-bottleneck net for tests
    c.C = 64; c.mid = 32; c.Cg = 16; c.p1 = 16; c.g1 = 16; c.v1 = 16; c.v2 = 32;
    c.kinds = {3, 2};
  } else if(name == "b2c32") {
    c.C = 32; c.Cg = 16; c.p1 = 16; c.g1 = 16; c.v1 = 16; c.v2 = 32;
    c.kinds = {0, 1};
  } else {
    throw std::invalid_argument("unknown model architecture: " + name);
  }
  return c;
}

namespace {
struct Init {
  DRng r;
  std::vector<float> normal(size_t n, float std) {
    std::vector<float> v(n);
    for(auto& x : v)
      x = r.gauss() * std;
    return v;
  }
  std::vector<float> around(size_t n, float center, float std) {
    std::vector<float> v(n);
    for(auto& x : v)
      x = center + r.gauss() * std;
    return v;
  }
};
}  // namespace

static ModelBlock randomBlock(Init& in, int k, int W, int Cg, int mid) {
  auto he = [](int fanIn) { return std::sqrt(2.0f / (float)fanIn); };
  ModelBlock b;
  b.kind = k;
  if(k >= 2) {
    b.bnPs = in.around(W, 1.0f, 0.1f);
    b.bnPb = in.normal(W, 0.1f);
    b.convP = in.normal((size_t)mid * W, he(W));
    b.inner.push_back(randomBlock(in, k == 3 ? 1 : 0, mid, Cg, 0));
    b.inner.push_back(randomBlock(in, 0, mid, Cg, 0));
    b.bnQs = in.around(mid, 1.0f, 0.1f);
    b.bnQb = in.normal(mid, 0.1f);
    b.convQ = in.normal((size_t)W * mid, 0.5f * he(mid));
    return b;
  }
  const int Cr = W - Cg;
  b.bn1s = in.around(W, 1.0f, 0.1f);
  b.bn1b = in.normal(W, 0.1f);
  if(k == 0) {
    b.conv1 = in.normal((size_t)W * W * 9, he(W * 9));
    b.bn2s = in.around(W, 1.0f, 0.1f);
    b.bn2b = in.normal(W, 0.1f);
    b.conv2 = in.normal((size_t)W * W * 9, 0.5f * he(W * 9));
  } else {
    b.conv1 = in.normal((size_t)Cr * W * 9, 0.8f * he(W * 9));
    b.conv1g = in.normal((size_t)Cg * W * 9, he(W * 9));
    b.bngs = in.around(Cg, 1.0f, 0.1f);
    b.bngb = in.normal(Cg, 0.1f);
    b.linG = in.normal((size_t)Cr * 3 * Cg, 0.6f * he(3 * Cg));
    b.bn2s = in.around(Cr, 1.0f, 0.1f);
    b.bn2b = in.normal(Cr, 0.1f);
    b.conv2 = in.normal((size_t)W * Cr * 9, 0.5f * he(Cr * 9));
  }
  return b;
}

// He-normal convolutions, near-identity merged BN (SURVEY §8d synthetic init),
// residual branches scaled by 0.5 so the trunk stays O(1) without fixup zeros.
ModelHost randomModel(const ModelCfg& cfg, uint64_t seed) {
  ModelHost m;
  m.cfg = cfg;
  Init in{DRng{mix64(seed ^ 0xC0FFEEULL), 0}};
  const int C = cfg.C;
  auto he = [](int fanIn) { return std::sqrt(2.0f / (float)fanIn); };
  m.convInit = in.normal((size_t)C * cfg.cin * 9, he(cfg.cin * 9));
  m.globInit = in.normal((size_t)C * cfg.gin, 0.1f);
  for(int k : cfg.kinds)
    m.blocks.push_back(randomBlock(in, k, C, cfg.Cg, cfg.mid));
  m.tips = in.around(C, 1.0f, 0.1f);
  m.tipb = in.normal(C, 0.1f);
  m.pConv1 = in.normal((size_t)cfg.p1 * C, 0.8f * he(C));
  m.pConvG = in.normal((size_t)cfg.g1 * C, he(C));
  m.pBiasG = in.normal(cfg.g1, 0.1f);
  m.pLinG = in.normal((size_t)cfg.p1 * 3 * cfg.g1, 0.6f * he(3 * cfg.g1));
  m.pBias2 = in.normal(cfg.p1, 0.1f);
  m.pConv2 = in.normal((size_t)4 * cfg.p1, 0.3f / std::sqrt((float)cfg.p1));
  m.vConv1 = in.normal((size_t)cfg.v1 * C, he(C));
  m.vBias1 = in.normal(cfg.v1, 0.1f);
  m.vLin2 = in.normal((size_t)cfg.v2 * 3 * cfg.v1, he(3 * cfg.v1));
  m.vB2 = in.normal(cfg.v2, 0.1f);
  m.vLin3 = in.normal((size_t)2 * cfg.v2, 1.0f / std::sqrt((float)cfg.v2));
  m.vB3 = in.normal(2, 0.1f);
  m.vLinM = in.normal((size_t)2 * cfg.v2, 1.0f / std::sqrt((float)cfg.v2));
  m.vBM = in.normal(2, 0.1f);
  return m;
}

static bool hasBottleneck(const ModelCfg& c) {
  for(int k : c.kinds)
    if(k >= 2)
      return true;
  return false;
}

static void writeBlock(FILE* f, const ModelBlock& b) {
  auto w = [&](const std::vector<float>& v) { fwrite(v.data(), 4, v.size(), f); };
  if(b.kind >= 2) {
    w(b.bnPs); w(b.bnPb); w(b.convP);
    writeBlock(f, b.inner[0]);
    writeBlock(f, b.inner[1]);
    w(b.bnQs); w(b.bnQb); w(b.convQ);
    return;
  }
  w(b.bn1s);
  w(b.bn1b);
  if(b.kind == 0) {
    w(b.conv1); w(b.bn2s); w(b.bn2b); w(b.conv2);
  } else {
    w(b.conv1); w(b.conv1g); w(b.bngs); w(b.bngb); w(b.linG); w(b.bn2s); w(b.bn2b); w(b.conv2);
  }
}

void saveModel(const std::string& path, const ModelHost& m) {
  FILE* f = fopen(path.c_str(), "wb");
  if(!f)
    throw std::runtime_error("cannot write model " + path);
  fwrite("CFNN", 1, 4, f);
  const ModelCfg& c = m.cfg;
  const bool v2 = hasBottleneck(c);
  int32_t ver = v2 ? 2 : 1;
  fwrite(&ver, 4, 1, f);
  int32_t hdr[10] = {c.cin, c.gin, c.C, c.Cg, c.p1, c.g1, c.v1, c.v2, (int32_t)c.kinds.size(), c.mid};
  fwrite(hdr, 4, v2 ? 10 : 9, f);
  for(int k : c.kinds) {
    int32_t kk = k;
    fwrite(&kk, 4, 1, f);
  }
  auto w = [&](const std::vector<float>& v) { fwrite(v.data(), 4, v.size(), f); };
  w(m.convInit);
  w(m.globInit);
  for(const ModelBlock& b : m.blocks)
    writeBlock(f, b);
  w(m.tips); w(m.tipb);
  w(m.pConv1); w(m.pConvG); w(m.pBiasG); w(m.pLinG); w(m.pBias2); w(m.pConv2);
  w(m.vConv1); w(m.vBias1); w(m.vLin2); w(m.vB2); w(m.vLin3); w(m.vB3); w(m.vLinM); w(m.vBM);
  fclose(f);
}

namespace {
// Reads a CFNN image in memory (a file's bytes, or weights broadcast from another rank).
struct FileReader {
  const unsigned char* p;
  size_t left;  // bytes left in the image: no tensor is sized past its end
  bool ok = true;
  bool raw(void* dst, size_t bytes) {
    if(!ok || bytes > left) {
      ok = false;
      return false;
    }
    memcpy(dst, p, bytes);
    p += bytes;
    left -= bytes;
    return true;
  }
  void r(std::vector<float>& v, size_t n) {
    if(!ok || n > left / 4) {
      ok = false;
      return;
    }
    v.resize(n);
    raw(v.data(), n * 4);
  }
  void block(ModelBlock& b, int k, int W, int Cg, int mid) {
    b.kind = k;
    if(k >= 2) {
      r(b.bnPs, W); r(b.bnPb, W); r(b.convP, (size_t)mid * W);
      b.inner.resize(2);
      block(b.inner[0], k == 3 ? 1 : 0, mid, Cg, 0);
      block(b.inner[1], 0, mid, Cg, 0);
      r(b.bnQs, mid); r(b.bnQb, mid); r(b.convQ, (size_t)W * mid);
      return;
    }
    const int Cr = W - Cg;
    r(b.bn1s, W);
    r(b.bn1b, W);
    if(k == 0) {
      r(b.conv1, (size_t)W * W * 9); r(b.bn2s, W); r(b.bn2b, W); r(b.conv2, (size_t)W * W * 9);
    } else {
      r(b.conv1, (size_t)Cr * W * 9); r(b.conv1g, (size_t)Cg * W * 9); r(b.bngs, Cg); r(b.bngb, Cg);
      r(b.linG, (size_t)Cr * 3 * Cg); r(b.bn2s, Cr); r(b.bn2b, Cr); r(b.conv2, (size_t)W * Cr * 9);
    }
  }
};
}  // namespace

ModelHost loadModelBytes(const void* data, size_t bytes, const std::string& name) {
  FileReader rd{static_cast<const unsigned char*>(data), data ? bytes : 0};
  char magic[4];
  int32_t ver = 0, hdr[10] = {0};
  if(!rd.raw(magic, 4) || memcmp(magic, "CFNN", 4) != 0 || !rd.raw(&ver, 4) || (ver != 1 && ver != 2) ||
     !rd.raw(hdr, 4 * (ver == 1 ? 9 : 10)) || hdr[8] < 1 || hdr[8] > 64)
    throw std::runtime_error("not a CFNN v1/v2 model: " + name);
  // header sizes: positive and bounded (a corrupted field must not size a tensor)
  bool sane = true;
  for(int i = 0; i < 8; i++)
    sane = sane && hdr[i] >= 1 && hdr[i] <= 4096;
  sane = sane && hdr[3] < hdr[2] && (ver == 1 || (hdr[9] >= 1 && hdr[9] <= hdr[2]));
  if(!sane)
    throw std::runtime_error("bad header sizes in model " + name);
  ModelHost m;
  ModelCfg& c = m.cfg;
  c.cin = hdr[0]; c.gin = hdr[1]; c.C = hdr[2]; c.Cg = hdr[3]; c.p1 = hdr[4]; c.g1 = hdr[5]; c.v1 = hdr[6];
  c.v2 = hdr[7];
  c.mid = ver == 2 ? hdr[9] : 0;
  c.kinds.resize(hdr[8]);
  rd.raw(c.kinds.data(), 4 * (size_t)hdr[8]);
  for(int k : c.kinds)
    if(k < 0 || k > 3 || (k >= 2 && c.mid <= 0))
      rd.ok = false;
  if(!rd.ok)
    throw std::runtime_error("bad block kinds in model " + name);
  const int C = c.C;
  rd.r(m.convInit, (size_t)C * c.cin * 9);
  rd.r(m.globInit, (size_t)C * c.gin);
  for(int k : c.kinds) {
    ModelBlock b;
    rd.block(b, k, C, c.Cg, c.mid);
    m.blocks.push_back(std::move(b));
  }
  rd.r(m.tips, C); rd.r(m.tipb, C);
  rd.r(m.pConv1, (size_t)c.p1 * C); rd.r(m.pConvG, (size_t)c.g1 * C); rd.r(m.pBiasG, c.g1);
  rd.r(m.pLinG, (size_t)c.p1 * 3 * c.g1); rd.r(m.pBias2, c.p1); rd.r(m.pConv2, (size_t)4 * c.p1);
  rd.r(m.vConv1, (size_t)c.v1 * C); rd.r(m.vBias1, c.v1); rd.r(m.vLin2, (size_t)c.v2 * 3 * c.v1); rd.r(m.vB2, c.v2);
  rd.r(m.vLin3, (size_t)2 * c.v2); rd.r(m.vB3, 2); rd.r(m.vLinM, (size_t)2 * c.v2); rd.r(m.vBM, 2);
  if(!rd.ok || rd.left != 0)
    throw std::runtime_error("truncated or oversized model " + name);
  return m;
}

ModelHost loadModel(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if(!f)
    throw std::runtime_error("cannot open model " + path);
  std::vector<unsigned char> img;
  unsigned char buf[1 << 16];
  size_t got;
  while((got = fread(buf, 1, sizeof(buf), f)) > 0)
    img.insert(img.end(), buf, buf + got);
  const bool err = ferror(f) != 0;
  fclose(f);
  if(err)
    throw std::runtime_error("cannot read model " + path);
  return loadModelBytes(img.data(), img.size(), path);
}

static double blockMacs(int k, double A, double W, double Cg, double mid) {
  if(k >= 2)
    return A * W * mid + blockMacs(k == 3 ? 1 : 0, A, mid, Cg, 0) + blockMacs(0, A, mid, Cg, 0) + A * mid * W;
  if(k == 0)
    return 2.0 * A * W * W * 9.0;
  const double Cr = W - Cg;
  return A * W * W * 9.0 + Cr * 3.0 * Cg + A * W * Cr * 9.0;
}

double modelFlopsPerEval(const ModelCfg& c, int A) {
  const double C = c.C;
  double macs = A * C * c.cin * 9.0 + C * c.gin;
  for(int k : c.kinds)
    macs += blockMacs(k, A, C, c.Cg, c.mid);
  macs += A * C * (c.p1 + c.g1) + 3.0 * c.g1 * c.p1 + A * 4.0 * c.p1;
  macs += A * C * c.v1 + 3.0 * c.v1 * c.v2 + 4.0 * c.v2;
  return 2.0 * macs;
}

}  // namespace kc
