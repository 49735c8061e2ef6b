// Coffee network weights: the "CFNN" v1 file format and a seeded initializer.
//
// The reference has no Coffee model format (desc.cpp:800-914 only reads
// KataGo Go nets).  This format carries exactly the tensors of the Coffee head
// contract (NNOutput, nninputs.h:75-118) on a KataGo-style trunk
// (model_pytorch.py:678-1152; eigenbackend.cpp:888-1377):
//
//   "CFNN" u32 version (1, or 2 when any block is a nested bottleneck)
//   i32 cin gin C Cg p1 g1 v1 v2 nblocks [v2: mid], i32 kinds[nblocks]
//   (0 regular, 1 gpool, 2 nested bottleneck, 3 nested bottleneck whose first
//   inner block is a gpool block; model_pytorch.py:860-958 "bottlenest2[gpool]")
//   f32 tensors, in this order:
//     convInit[C][cin][3][3]  globInit[C][gin]
//     per block: bn1s[C] bn1b[C]
//        regular: conv1[C][C][3][3] bn2s[C] bn2b[C] conv2[C][C][3][3]
//        gpool  : conv1r[C-Cg][C][3][3] conv1g[Cg][C][3][3] bngs[Cg] bngb[Cg]
//                 linG[C-Cg][3Cg] bn2s[C-Cg] bn2b[C-Cg] conv2[C][C-Cg][3][3]
//        bottleneck: bnPs[C] bnPb[C] convP[mid][C] (1x1), inner block 0 (gpool for
//                 kind 3, else regular) and inner block 1 (regular), both at width
//                 mid in the layouts above, bnQs[mid] bnQb[mid] convQ[C][mid] (1x1)
//     tips[C] tipb[C]
//     pConv1[p1][C] pConvG[g1][C] pBiasG[g1] pLinG[p1][3g1] pBias2[p1] pConv2[4][p1]
//     vConv1[v1][C] vBias1[v1] vLin2[v2][3v1] vB2[v2] vLin3[2][v2] vB3[2] vLinM[2][v2] vBM[2]
// BatchNorm layers are stored merged (scale = gamma/sqrt(var+eps), bias = beta -
// scale*mean, eigenbackend.cpp:684-734).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace kc {

struct ModelCfg {
  int cin = 15, gin = 1, C = 96, Cg = 32, p1 = 32, g1 = 32, v1 = 32, v2 = 64;
  int mid = 0;             // nested-bottleneck width (0: none)
  std::vector<int> kinds;  // per block
};

struct ModelBlock {
  int kind = 0;
  std::vector<float> bn1s, bn1b, conv1, conv1g, bngs, bngb, linG, bn2s, bn2b, conv2;
  // nested bottleneck (kinds 2, 3)
  std::vector<float> bnPs, bnPb, convP, bnQs, bnQb, convQ;
  std::vector<ModelBlock> inner;
};

struct ModelHost {
  ModelCfg cfg;
  std::vector<float> convInit, globInit;
  std::vector<ModelBlock> blocks;
  std::vector<float> tips, tipb;
  std::vector<float> pConv1, pConvG, pBiasG, pLinG, pBias2, pConv2;
  std::vector<float> vConv1, vBias1, vLin2, vB2, vLin3, vB3, vLinM, vBM;
};

// Named architectures: "b6c96" (BASELINE C1/C2), "b10c128" (C3/C4), "b18c384nbt" (C5).
ModelCfg modelCfgByName(const std::string& name);
ModelHost randomModel(const ModelCfg& cfg, uint64_t seed);
void saveModel(const std::string& path, const ModelHost& m);
ModelHost loadModel(const std::string& path);
// The same from a CFNN image in memory (e.g. weights broadcast from rank 0); name labels errors.
ModelHost loadModelBytes(const void* data, size_t bytes, const std::string& name);
// FLOPs per evaluation at area A (2 x MACs of every conv / matmul).
double modelFlopsPerEval(const ModelCfg& cfg, int A);

}  // namespace kc
