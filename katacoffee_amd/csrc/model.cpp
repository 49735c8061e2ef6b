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

// He-normal convolutions, near-identity merged BN (SURVEY §8d synthetic init),
// residual branches scaled by 0.5 so the trunk stays O(1) without fixup zeros.
ModelHost randomModel(const ModelCfg& cfg, uint64_t seed) {
  ModelHost m;
  m.cfg = cfg;
  Init in{DRng{mix64(seed ^ 0xC0FFEEULL), 0}};
  const int C = cfg.C, Cr = cfg.C - cfg.Cg;
  auto he = [](int fanIn) { return std::sqrt(2.0f / (float)fanIn); };
  m.convInit = in.normal((size_t)C * cfg.cin * 9, he(cfg.cin * 9));
  m.globInit = in.normal((size_t)C * cfg.gin, 0.1f);
  for(int k : cfg.kinds) {
    ModelBlock b;
    b.kind = k;
    b.bn1s = in.around(C, 1.0f, 0.1f);
    b.bn1b = in.normal(C, 0.1f);
    if(k == 0) {
      b.conv1 = in.normal((size_t)C * C * 9, he(C * 9));
      b.bn2s = in.around(C, 1.0f, 0.1f);
      b.bn2b = in.normal(C, 0.1f);
      b.conv2 = in.normal((size_t)C * C * 9, 0.5f * he(C * 9));
    } else {
      b.conv1 = in.normal((size_t)Cr * C * 9, 0.8f * he(C * 9));
      b.conv1g = in.normal((size_t)cfg.Cg * C * 9, he(C * 9));
      b.bngs = in.around(cfg.Cg, 1.0f, 0.1f);
      b.bngb = in.normal(cfg.Cg, 0.1f);
      b.linG = in.normal((size_t)Cr * 3 * cfg.Cg, 0.6f * he(3 * cfg.Cg));
      b.bn2s = in.around(Cr, 1.0f, 0.1f);
      b.bn2b = in.normal(Cr, 0.1f);
      b.conv2 = in.normal((size_t)C * Cr * 9, 0.5f * he(Cr * 9));
    }
    m.blocks.push_back(std::move(b));
  }
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

void saveModel(const std::string& path, const ModelHost& m) {
  FILE* f = fopen(path.c_str(), "wb");
  if(!f)
    throw std::runtime_error("cannot write model " + path);
  fwrite("CFNN", 1, 4, f);
  int32_t ver = 1;
  fwrite(&ver, 4, 1, f);
  const ModelCfg& c = m.cfg;
  int32_t hdr[9] = {c.cin, c.gin, c.C, c.Cg, c.p1, c.g1, c.v1, c.v2, (int32_t)c.kinds.size()};
  fwrite(hdr, 4, 9, f);
  for(int k : c.kinds) {
    int32_t kk = k;
    fwrite(&kk, 4, 1, f);
  }
  auto w = [&](const std::vector<float>& v) { fwrite(v.data(), 4, v.size(), f); };
  w(m.convInit);
  w(m.globInit);
  for(const ModelBlock& b : m.blocks) {
    w(b.bn1s);
    w(b.bn1b);
    if(b.kind == 0) {
      w(b.conv1); w(b.bn2s); w(b.bn2b); w(b.conv2);
    } else {
      w(b.conv1); w(b.conv1g); w(b.bngs); w(b.bngb); w(b.linG); w(b.bn2s); w(b.bn2b); w(b.conv2);
    }
  }
  w(m.tips); w(m.tipb);
  w(m.pConv1); w(m.pConvG); w(m.pBiasG); w(m.pLinG); w(m.pBias2); w(m.pConv2);
  w(m.vConv1); w(m.vBias1); w(m.vLin2); w(m.vB2); w(m.vLin3); w(m.vB3); w(m.vLinM); w(m.vBM);
  fclose(f);
}

ModelHost loadModel(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if(!f)
    throw std::runtime_error("cannot open model " + path);
  char magic[4];
  int32_t ver = 0, hdr[9];
  if(fread(magic, 1, 4, f) != 4 || memcmp(magic, "CFNN", 4) != 0 || fread(&ver, 4, 1, f) != 1 || ver != 1 ||
     fread(hdr, 4, 9, f) != 9 || hdr[8] < 1 || hdr[8] > 64) {
    fclose(f);
    throw std::runtime_error("not a CFNN v1 model: " + path);
  }
  ModelHost m;
  ModelCfg& c = m.cfg;
  c.cin = hdr[0]; c.gin = hdr[1]; c.C = hdr[2]; c.Cg = hdr[3]; c.p1 = hdr[4]; c.g1 = hdr[5]; c.v1 = hdr[6];
  c.v2 = hdr[7];
  c.kinds.resize(hdr[8]);
  bool ok = fread(c.kinds.data(), 4, hdr[8], f) == (size_t)hdr[8];
  auto r = [&](std::vector<float>& v, size_t n) {
    v.resize(n);
    if(fread(v.data(), 4, n, f) != n)
      ok = false;
  };
  const int C = c.C, Cr = c.C - c.Cg;
  r(m.convInit, (size_t)C * c.cin * 9);
  r(m.globInit, (size_t)C * c.gin);
  for(int k : c.kinds) {
    ModelBlock b;
    b.kind = k;
    r(b.bn1s, C);
    r(b.bn1b, C);
    if(k == 0) {
      r(b.conv1, (size_t)C * C * 9); r(b.bn2s, C); r(b.bn2b, C); r(b.conv2, (size_t)C * C * 9);
    } else {
      r(b.conv1, (size_t)Cr * C * 9); r(b.conv1g, (size_t)c.Cg * C * 9); r(b.bngs, c.Cg); r(b.bngb, c.Cg);
      r(b.linG, (size_t)Cr * 3 * c.Cg); r(b.bn2s, Cr); r(b.bn2b, Cr); r(b.conv2, (size_t)C * Cr * 9);
    }
    m.blocks.push_back(std::move(b));
  }
  r(m.tips, C); r(m.tipb, C);
  r(m.pConv1, (size_t)c.p1 * C); r(m.pConvG, (size_t)c.g1 * C); r(m.pBiasG, c.g1);
  r(m.pLinG, (size_t)c.p1 * 3 * c.g1); r(m.pBias2, c.p1); r(m.pConv2, (size_t)4 * c.p1);
  r(m.vConv1, (size_t)c.v1 * C); r(m.vBias1, c.v1); r(m.vLin2, (size_t)c.v2 * 3 * c.v1); r(m.vB2, c.v2);
  r(m.vLin3, (size_t)2 * c.v2); r(m.vB3, 2); r(m.vLinM, (size_t)2 * c.v2); r(m.vBM, 2);
  fclose(f);
  if(!ok)
    throw std::runtime_error("truncated model file " + path);
  return m;
}

double modelFlopsPerEval(const ModelCfg& c, int A) {
  const double C = c.C, Cr = c.C - c.Cg;
  double macs = A * C * c.cin * 9.0 + C * c.gin;
  for(int k : c.kinds) {
    if(k == 0)
      macs += 2.0 * A * C * C * 9.0;
    else
      macs += A * C * C * 9.0 + Cr * 3.0 * c.Cg + A * C * Cr * 9.0;
  }
  macs += A * C * (c.p1 + c.g1) + 3.0 * c.g1 * c.p1 + A * 4.0 * c.p1;
  macs += A * C * c.v1 + 3.0 * c.v1 * c.v2 + 4.0 * c.v2;
  return 2.0 * macs;
}

}  // namespace kc
