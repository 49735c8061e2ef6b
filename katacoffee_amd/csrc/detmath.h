// Deterministic f32 math, the per-game counter RNG and 64-lane wave reductions.
// SPEC (DESIGN.md "Numerics"): every search-side float result is defined by
// these exact operation sequences (compiled with -ffp-contract=off), so the
// device search is reproducible bit-for-bit and checkable against the CPU oracle.
#pragma once
#include "kc_common.h"

namespace kc {

KC_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
KC_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

KC_HD float dlog(float x) {
  if(!(x > 0.0f))
    return x == 0.0f ? -__builtin_inff() : __builtin_nanf("");
  if(x == __builtin_inff())
    return x;
  int e = 0;
  uint32_t u = f2u(x);
  if(u < 0x00800000u) {
    x = x * 8388608.0f;
    u = f2u(x);
    e = -23;
  }
  e += (int)((u >> 23) & 0xffu) - 127;
  float m = u2f((u & 0x007fffffu) | 0x3f800000u);
  if(m > 1.41421356f) {
    m = m * 0.5f;
    e += 1;
  }
  float s = (m - 1.0f) / (m + 1.0f);
  float s2 = s * s;
  float poly = s2 * (0.333333343f + s2 * (0.2f + s2 * (0.142857149f + s2 * 0.111111112f)));
  float logm = (s + s * poly) * 2.0f;
  float fe = (float)e;
  return fe * 0.693145752f + (logm + fe * 1.42860677e-06f);
}

KC_HD float dexp(float x) {
  if(x != x)
    return x;
  if(x > 88.7228f)
    return __builtin_inff();
  if(x < -103.97f)
    return 0.0f;
  float n = floorf(x * 1.44269504f + 0.5f);
  float r = (x - n * 0.693145752f) - n * 1.42860677e-06f;
  float p = 1.0f + r * (1.0f + r * (0.5f + r * (0.166666672f + r * (0.0416666679f +
            r * (0.00833333377f + r * (0.00138888892f + r * 0.000198412701f))))));
  int ni = (int)n;
  if(ni > 127) {
    p = p * 1.70141183e38f;
    ni -= 127;
  }
  if(ni < -126) {
    p = p * 1.17549435e-38f;
    ni += 126;
  }
  return p * u2f((uint32_t)(ni + 127) << 23);
}

KC_HD float dpow(float x, float y) {
  if(x == 0.0f)
    return y > 0.0f ? 0.0f : (y == 0.0f ? 1.0f : __builtin_inff());
  return dexp(y * dlog(x));
}

KC_HD uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// Per-game counter-based stream (SPEC a24).
struct DRng {
  uint64_t seed, ctr;
  KC_HD uint64_t next() { return mix64(seed ^ (++ctr * 0xd1342543de82ef95ULL)); }
  KC_HD float uni() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }
  KC_HD uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  KC_HD float gauss() {
    float u, v, s;
    do {
      u = 2.0f * uni() - 1.0f;
      v = 2.0f * uni() - 1.0f;
      s = u * u + v * v;
    } while(s >= 1.0f || s == 0.0f);
    return u * sqrtf((-2.0f * dlog(s)) / s);
  }
  // Marsaglia-Tsang (rand.cpp:335-363) in f32; a <= 1 boosts through a + 1.
  KC_HD float gammaGt1(float a) {
    float d = a - 0.333333343f;
    float c = 0.333333343f / sqrtf(d);
    while(true) {
      float x = gauss();
      float vt = 1.0f + c * x;
      if(vt <= 0.0f)
        continue;
      float v = vt * vt * vt;
      float u = uni();
      float xx = x * x;
      if(u < 1.0f - 0.0331f * xx * xx)
        return d * v;
      if(u == 0.0f || dlog(u) < 0.5f * xx + d * ((1.0f - v) + dlog(v)))
        return d * v;
    }
  }
  KC_HD float gamma(float a) {
    if(a <= 1.0f) {
      float r = gammaGt1(a + 1.0f);
      float inva = 1.0f / a;
      float u = uni();
      return r * dpow(u, inva);
    }
    return gammaGt1(a);
  }
};

KC_D int laneId() { return (int)(threadIdx.x & 63); }

// Cross-lane exchanges of the xor butterfly without the LDS: lanes i and i^32 /
// i^16 via v_permlane32_swap / v_permlane16_swap (both results of the swap hold
// the two partners' values), i^8 / i^4 via DPP row_ror:8 / row_ror:4 (after the
// wider levels a partial depends only on lane mod 16 / mod 8, so rotating a row
// by 8 / 4 reaches the xor partner's value), i^2 / i^1 via DPP quad_perm.  Every
// combine below is commutative, so each level pairs exactly the butterfly's
// partials: the results are bit-identical to the shuffle butterfly (treeSum64).
KC_D int bitsF(float x) { return __builtin_bit_cast(int, x); }
KC_D float asF(int x) { return __builtin_bit_cast(float, x); }
template <int CTRL>
KC_D int dppMov(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
constexpr int DPP_ROR8 = 0x128, DPP_ROR4 = 0x124, DPP_X2 = 0x4e, DPP_X1 = 0xb1;
// The partner value at butterfly level LVL (0: i^32, 1: i^16, 2: i^8, 3: i^4, 4: i^2,
// 5: i^1) for the DPP levels; the permlane levels go through swapPair.
template <int LVL>
KC_D int partner(int x) {
  static_assert(LVL >= 2 && LVL <= 5, "DPP levels");
  if constexpr(LVL == 2)
    return dppMov<DPP_ROR8>(x);
  else if constexpr(LVL == 3)
    return dppMov<DPP_ROR4>(x);
  else if constexpr(LVL == 4)
    return dppMov<DPP_X2>(x);
  else
    return dppMov<DPP_X1>(x);
}
// {own-half value, partner-half value} for levels 0/1 (order differs by half; the
// combines are commutative).
template <int LVL>
KC_D void swapPair(int x, int& a, int& b) {
  if constexpr(LVL == 0) {
    auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    a = r[0];
    b = r[1];
  } else {
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    a = r[0];
    b = r[1];
  }
}

// treeSum64 (oracle/ora_math.h): the lane's in-order partial, then xor butterfly.
KC_D float waveSum(float s) {
  int a, b;
  swapPair<0>(bitsF(s), a, b);
  s = asF(a) + asF(b);
  swapPair<1>(bitsF(s), a, b);
  s = asF(a) + asF(b);
  s = s + asF(partner<2>(bitsF(s)));
  s = s + asF(partner<3>(bitsF(s)));
  s = s + asF(partner<4>(bitsF(s)));
  s = s + asF(partner<5>(bitsF(s)));
  return s;
}
KC_D float waveMax(float s) {
  int a, b;
  swapPair<0>(bitsF(s), a, b);
  s = fmaxf(asF(a), asF(b));
  swapPair<1>(bitsF(s), a, b);
  s = fmaxf(asF(a), asF(b));
  s = fmaxf(s, asF(partner<2>(bitsF(s))));
  s = fmaxf(s, asF(partner<3>(bitsF(s))));
  s = fmaxf(s, asF(partner<4>(bitsF(s))));
  s = fmaxf(s, asF(partner<5>(bitsF(s))));
  return s;
}
KC_D int waveMinI(int s) {
  int a, b;
  swapPair<0>(s, a, b);
  s = min(a, b);
  swapPair<1>(s, a, b);
  s = min(a, b);
  s = min(s, partner<2>(s));
  s = min(s, partner<3>(s));
  s = min(s, partner<4>(s));
  s = min(s, partner<5>(s));
  return s;
}
// argmax with "first strictly greater wins" semantics (lowest index on ties).
KC_D void argmaxCombine(float& v, int& idx, float ov, int oi) {
  if(ov > v || (ov == v && oi < idx)) {
    v = ov;
    idx = oi;
  }
}
template <int LVL>
KC_D void argmaxSwapLevel(float& v, int& idx) {
  int va, vb, ia, ib;
  swapPair<LVL>(bitsF(v), va, vb);
  swapPair<LVL>(idx, ia, ib);
  v = asF(va);
  idx = ia;
  argmaxCombine(v, idx, asF(vb), ib);
}
template <int LVL>
KC_D void argmaxDppLevel(float& v, int& idx) {
  const float ov = asF(partner<LVL>(bitsF(v)));
  const int oi = partner<LVL>(idx);
  argmaxCombine(v, idx, ov, oi);
}
KC_D void waveArgmax(float& v, int& idx) {
  argmaxSwapLevel<0>(v, idx);
  argmaxSwapLevel<1>(v, idx);
  argmaxDppLevel<2>(v, idx);
  argmaxDppLevel<3>(v, idx);
  argmaxDppLevel<4>(v, idx);
  argmaxDppLevel<5>(v, idx);
}
// XOR of every lane's value (order-free), in every lane.
KC_D uint64_t waveXor64(uint64_t h) {
  int lo = (int)(uint32_t)h, hi = (int)(uint32_t)(h >> 32), a, b;
  swapPair<0>(lo, a, b);
  lo = a ^ b;
  swapPair<0>(hi, a, b);
  hi = a ^ b;
  swapPair<1>(lo, a, b);
  lo = a ^ b;
  swapPair<1>(hi, a, b);
  hi = a ^ b;
  lo ^= partner<2>(lo);
  hi ^= partner<2>(hi);
  lo ^= partner<3>(lo);
  hi ^= partner<3>(hi);
  lo ^= partner<4>(lo);
  hi ^= partner<4>(hi);
  lo ^= partner<5>(lo);
  hi ^= partner<5>(hi);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
// v of lane srcLane (uniform) in every lane, through a scalar register.
KC_D int bcastLane(int v, int srcLane) {
  return __builtin_amdgcn_readlane(v, __builtin_amdgcn_readfirstlane(srcLane));
}
KC_D float bcastLaneF(float v, int srcLane) { return asF(bcastLane(bitsF(v), srcLane)); }
KC_D uint64_t ballot(bool b) { return __ballot(b); }

}  // namespace kc
