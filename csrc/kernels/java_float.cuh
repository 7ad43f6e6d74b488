// Java Float.toString text of a binary32 on the device (JDK 19+ shortest-digit rules): shared by
// the standalone formatting kernel (format.hip) and the whole-network forward kernels that
// format their softmax rows in their own epilogue (resnet20_fused.hip, lenet5_fused.hip).
// See format.hip for the algorithm and the slot layout.
#pragma once
#include "common.cuh"
#include "exact_decimal.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

struct F32Parts {
  uint64_t m;  // significand (with the hidden bit for normals)
  int e2;      // v = m * 2^e2
  uint64_t upK, loK;  // rounding interval [loK * 2^loE, upK * 2^upE]
  int upE, loE;
  bool incl;  // the interval's ends belong to it (m even: a tie parses back to v)
};

__device__ __forceinline__ F32Parts f32_parts(uint32_t bits) {
  F32Parts f;
  const uint32_t be = (bits >> 23) & 0xffu, frac = bits & 0x7fffffu;
  f.m = be ? (uint64_t)(frac | 0x800000u) : (uint64_t)frac;
  f.e2 = be ? (int)be - 150 : -149;
  f.upK = 2 * f.m + 1;
  f.upE = f.e2 - 1;
  if (frac == 0 && be > 1) {  // power of two: the predecessor is half an ulp closer
    f.loK = 4 * f.m - 1;
    f.loE = f.e2 - 2;
  } else {
    f.loK = 2 * f.m - 1;
    f.loE = f.e2 - 1;
  }
  f.incl = (f.m & 1) == 0;
  return f;
}

// Every comparison is first made in double: d * 10^-q carries a relative error below 2^-50
// (10^|k| from at most 6 exact powers, one reciprocal, one product), so a difference larger
// than 2^-44 of the magnitude decides it; only a closer call (a decimal within 2^-44 of a
// rounding boundary: rare) takes the exact 256-bit comparison.
constexpr double kTol = 0x1p-44;

// out of line: the 256-bit temporaries (dynamically indexed limbs) live in scratch memory,
// which only this rarely taken call should touch
__device__ __noinline__ int cmp_exact(uint64_t d, int q10, uint64_t K, int E) {
  return cmp_decimal_dyadic(d, q10, K, E);
}

__device__ __forceinline__ double p10(int k) {  // 10^k, |k| <= 63
  const int a = k < 0 ? -k : k;
  const double r = (((a & 1) ? 1e1 : 1.0) * ((a & 2) ? 1e2 : 1.0)) *
                   (((a & 4) ? 1e4 : 1.0) * ((a & 8) ? 1e8 : 1.0)) *
                   (((a & 16) ? 1e16 : 1.0) * ((a & 32) ? 1e32 : 1.0));
  return k < 0 ? 1.0 / r : r;
}

// sign of d * 10^-q - K * 2^E, given x ~ d * 10^-q and y = K * 2^E (exact)
__device__ __forceinline__ int cmp_fast(double x, double y, uint64_t d, int q, uint64_t K,
                                        int E) {
  const double diff = x - y;
  if (fabs(diff) > fabs(y) * kTol) return diff > 0 ? 1 : -1;
  return cmp_exact(d, -q, K, E);
}

// d * 10^-q lies in v's rounding interval
__device__ __forceinline__ bool in_interval(const F32Parts& f, uint64_t d, int q) {
  const double x = (double)d * p10(-q);
  const int cu = cmp_fast(x, ldexp((double)f.upK, f.upE), d, q, f.upK, f.upE);
  if (cu > 0 || (cu == 0 && !f.incl)) return false;
  const int cl = cmp_fast(x, ldexp((double)f.loK, f.loE), d, q, f.loK, f.loE);
  return cl > 0 || (cl == 0 && f.incl);
}

// floor(v * 10^q), exactly
__device__ __forceinline__ uint64_t floor_scaled(const F32Parts& f, float v, int q) {
  const double est = (double)v * p10(q);
  uint64_t d = (uint64_t)est;
  const double fr = est - (double)d;
  if (fr > est * kTol && 1.0 - fr > est * kTol) return d;
  for (int it = 0; it < 4 && d > 0 && cmp_exact(d, -q, f.m, f.e2) > 0; ++it) --d;
  for (int it = 0; it < 4 && cmp_exact(d + 1, -q, f.m, f.e2) <= 0; ++it) ++d;
  return d;
}

// the member of T at length p (q = p - 1 - E10), or false when no p-digit decimal is in R
__device__ bool pick(const F32Parts& f, float v, int q, uint64_t* out) {
  const uint64_t d0 = floor_scaled(f, v, q);
  const bool in0 = d0 > 0 && in_interval(f, d0, q);
  const bool in1 = in_interval(f, d0 + 1, q);
  if (!in0 && !in1) return false;
  if (in0 != in1) {
    *out = in0 ? d0 : d0 + 1;
    return true;
  }
  // both: the closer one; sign of (2 d0 + 1) * 10^-q - 2 v
  const int s = cmp_fast((double)(2 * d0 + 1) * p10(-q), 2.0 * (double)v, 2 * d0 + 1, q, f.m,
                         f.e2 + 1);
  *out = s > 0 ? d0 : s < 0 ? d0 + 1 : ((d0 & 1) ? d0 + 1 : d0);
  return true;
}

// The text is assembled in two 64-bit registers (byte k of the slot = byte k of lo:hi): a
// per-lane char array indexed by a running position would live in scratch memory, and its
// dependent byte stores/loads cost more than all the arithmetic.
struct Text16 {
  uint64_t lo = 0, hi = 0;
  __device__ __forceinline__ void put(int pos, uint32_t c) {
    const uint64_t v = (uint64_t)(c & 0xffu);
    lo |= pos < 8 ? v << (8 * (pos & 7)) : 0ull;
    hi |= pos >= 8 ? v << (8 * (pos & 7)) : 0ull;
  }
};

__device__ __forceinline__ int ndigits(uint64_t d) {  // d < 10^10
  int n = 1;
#pragma unroll
  for (int k = 1; k < 10; ++k) n += d >= (uint64_t)p10(k) ? 1 : 0;
  return n;
}

__device__ Text16 format_java(float v, int* len_out) {
  Text16 t;
  const uint32_t bits = __float_as_uint(v);
  if ((bits & 0x7f800000u) == 0x7f800000u && (bits & 0x7fffffu)) {
    t.lo = 0x4e614eull;  // "NaN"
    *len_out = 3;
    return t;
  }
  const int sg = (int)(bits >> 31);
  if (sg) t.put(0, '-');
  const uint32_t ab = bits & 0x7fffffffu;
  if (ab == 0x7f800000u) {
    const uint64_t inf = 0x7974696e69666e49ull;  // "Infinity"
    t.lo |= sg ? inf << 8 : inf;
    t.hi |= sg ? inf >> 56 : 0ull;
    *len_out = sg + 8;
    return t;
  }
  if (ab == 0) {
    t.put(sg, '0'); t.put(sg + 1, '.'); t.put(sg + 2, '0');
    *len_out = sg + 3;
    return t;
  }
  const float a = __uint_as_float(ab);
  const F32Parts f = f32_parts(ab);
  // E10 = floor(log10 a), made exact: 10^E10 <= a < 10^(E10+1)
  const double ad = (double)a;
  int E = (int)floorf(log10f(a));
  for (int it = 0; it < 3 && cmp_fast(p10(E), ad, 1, -E, f.m, f.e2) > 0; ++it) --E;
  for (int it = 0; it < 3 && cmp_fast(p10(E + 1), ad, 1, -E - 1, f.m, f.e2) <= 0; ++it) ++E;
  // minimal length by bisection (9 always succeeds)
  int lo = 1, hi = 9;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    uint64_t u;
    if (pick(f, a, mid - 1 - E, &u)) hi = mid;
    else lo = mid + 1;
  }
  const int p = lo == 1 ? 2 : lo;  // JDK 19+: a one-digit shortest -> closest 2-digit member
  int q = p - 1 - E;
  uint64_t d = 0;
  pick(f, a, q, &d);  // (membership is monotone in p: a member exists at p >= lo)
  while (d >= 10 && d % 10 == 0) {  // strip trailing zeros: value = d * 10^-q
    d /= 10;
    --q;
  }
  const int nd = ndigits(d);
  const int e = nd - 1 - q;  // a = d1.d2.. * 10^e
  const int dec_exp = e + 1;
  // layout (FloatingDecimal): where digit i (0 = most significant) goes, what else is written
  const int mode = (dec_exp > 0 && dec_exp < 8) ? 0 : (dec_exp <= 0 && dec_exp > -3) ? 1 : 2;
  const int o = sg;  // after the sign
  int len;
  uint64_t r = d;
  for (int i = nd - 1; i >= 0; --i) {  // least significant digit first
    const uint32_t c = '0' + (uint32_t)(r % 10);
    r /= 10;
    int pos;
    if (mode == 0) pos = i < dec_exp ? i : i + 1;
    else if (mode == 1) pos = 2 - dec_exp + i;
    else pos = i == 0 ? 0 : i + 1;
    t.put(o + pos, c);
  }
  if (mode == 0) {
    if (nd <= dec_exp) {
      for (int k = nd; k < dec_exp; ++k) t.put(o + k, '0');
      t.put(o + dec_exp, '.');
      t.put(o + dec_exp + 1, '0');
      len = dec_exp + 2;
    } else {
      t.put(o + dec_exp, '.');
      len = nd + 1;
    }
  } else if (mode == 1) {
    t.put(o, '0');
    t.put(o + 1, '.');
    for (int k = 0; k < -dec_exp; ++k) t.put(o + 2 + k, '0');
    len = 2 - dec_exp + nd;
  } else {
    t.put(o + 1, '.');
    int m = nd + 1;
    if (nd == 1) t.put(o + m++, '0');
    t.put(o + m++, 'E');
    int x = e;
    if (x < 0) {
      t.put(o + m++, '-');
      x = -x;
    }
    if (x >= 10) t.put(o + m++, '0' + (uint32_t)(x / 10));
    t.put(o + m++, '0' + (uint32_t)(x % 10));
    len = m;
  }
  *len_out = o + len;
  return t;
}

// One prediction slot: the text from byte 0, its length in byte 15 (at most 14 characters).
__device__ __forceinline__ uint4 java_float_slot(float v) {
  int len = 0;
  Text16 t = format_java(v, &len);
  t.hi |= (uint64_t)len << 56;
  return make_uint4((uint32_t)t.lo, (uint32_t)(t.lo >> 32), (uint32_t)t.hi,
                    (uint32_t)(t.hi >> 32));
}

// The step graph's verdict hand-off (StepOut): this workgroup's threads copy the parse's record
// statuses to the host-mapped array and clear them for the slot's next batch.
__device__ __forceinline__ void step_verdicts(const StepOut& so) {
  const int n = *so.nrec;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    so.status_out[i] = so.status[i];
    so.status[i] = 0;
  }
}

}  // namespace
}  // namespace gale
