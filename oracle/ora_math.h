// ORACLE (test infrastructure only) — deterministic float math + counter RNG.
// SPEC (DESIGN.md "Numerics"): all search arithmetic is IEEE f32 with no FMA
// contraction; log/exp/pow are the fixed polynomial sequences below; sums over
// a node's children use the 64-lane xor-butterfly order of treeSum64.  The HIP
// kernels implement the same sequences independently
// (katacoffee_amd/csrc/detmath.h), so GPU and oracle searches agree bit-for-bit.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

namespace ora {

inline uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
inline float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

inline float kLogf(float x) {
  if(!(x > 0.0f))
    return x == 0.0f ? -INFINITY : NAN;
  if(x == INFINITY)
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

inline float kExpf(float x) {
  if(x != x)
    return x;
  if(x > 88.7228f)
    return INFINITY;
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

inline float kPowf(float x, float y) {
  if(x == 0.0f)
    return y > 0.0f ? 0.0f : (y == 0.0f ? 1.0f : INFINITY);
  return kExpf(y * kLogf(x));
}
// double overloads (liboracle_f64: the reference's <cmath> in double)
inline double kLogf(double x) { return std::log(x); }
inline double kExpf(double x) { return std::exp(x); }
inline double kPowf(double x, double y) { return std::pow(x, y); }

// 64-lane xor butterfly: lane l first accumulates v[l], v[l+64], v[l+128], ...
// in order (lanes with l >= n start from +0), then xor-butterfly 32,16,..,1.
template <class T>
inline T treeSum64(const T* v, int n) {
  T s[64];
  for(int l = 0; l < 64; l++) {
    T a = l < n ? v[l] : T(0);
    for(int j = l + 64; j < n; j += 64)
      a = a + v[j];
    s[l] = a;
  }
  for(int off = 32; off >= 1; off >>= 1) {
    T t[64];
    for(int l = 0; l < 64; l++)
      t[l] = s[l] + s[l ^ off];
    memcpy(s, t, sizeof(s));
  }
  return s[0];
}

inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// Counter-based per-game stream (replaces the reference's per-thread Rand for
// search noise, symmetry choice, move temperature and row metadata: SPEC a24).
struct Rng {
  uint64_t seed = 0, ctr = 0;
  uint64_t next() { return mix64(seed ^ (++ctr * 0xd1342543de82ef95ULL)); }
  float uni() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  bool nextBool(float p) { return uni() < p; }
  // Marsaglia polar method.
  float gauss() {
    float u, v, s;
    do {
      u = 2.0f * uni() - 1.0f;
      v = 2.0f * uni() - 1.0f;
      s = u * u + v * v;
    } while(s >= 1.0f || s == 0.0f);
    return u * sqrtf((-2.0f * kLogf(s)) / s);
  }
  // Rand::nextGamma, rand.cpp:335-363 (Marsaglia & Tsang), restated in f32.
  float gamma(float a) {
    if(a <= 1.0f) {
      float r = gammaGt1(a + 1.0f);
      float inva = 1.0f / a;
      float u = uni();
      return r * kPowf(u, inva);
    }
    return gammaGt1(a);
  }
  float gammaGt1(float a) {
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
      if(u == 0.0f || kLogf(u) < 0.5f * xx + d * ((1.0f - v) + kLogf(v)))
        return d * v;
    }
  }
};

}  // namespace ora
