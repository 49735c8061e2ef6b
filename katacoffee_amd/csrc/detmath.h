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

// treeSum64 (oracle/ora_math.h): the lane's in-order partial, then xor butterfly.
KC_D float waveSum(float s) {
#pragma unroll
  for(int off = 32; off >= 1; off >>= 1)
    s = s + __shfl_xor(s, off, 64);
  return s;
}
KC_D float waveMax(float s) {
#pragma unroll
  for(int off = 32; off >= 1; off >>= 1)
    s = fmaxf(s, __shfl_xor(s, off, 64));
  return s;
}
KC_D int waveMinI(int s) {
#pragma unroll
  for(int off = 32; off >= 1; off >>= 1)
    s = min(s, __shfl_xor(s, off, 64));
  return s;
}
// argmax with "first strictly greater wins" semantics (lowest index on ties).
KC_D void waveArgmax(float& v, int& idx) {
#pragma unroll
  for(int off = 32; off >= 1; off >>= 1) {
    float ov = __shfl_xor(v, off, 64);
    int oi = __shfl_xor(idx, off, 64);
    if(ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
}
KC_D uint64_t ballot(bool b) { return __ballot(b); }

}  // namespace kc
