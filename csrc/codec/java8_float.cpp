// Java 8 Float.toString (--float-format java8): the reference serializes its predictions with
// Jackson 2.10 on Java 1.8 (/root/reference/pom.xml:113-114, InferenceBolt.java:90-91), whose
// float[] writer calls Float.toString -> sun.misc.FloatingDecimal. Before JDK 19 that is the
// Steele & White / dtoa free-format digit loop with a symmetric half-ulp stopping test, an
// estimated decimal exponent and two special rules (at least two digits in E-form, a halved
// margin at powers of two), which sometimes prints more digits than the shortest round-trip
// form (JDK-4511638, fixed in 19: format_float_java implements the JDK 19 rule).
//
// This is a re-derivation of that algorithm's arithmetic - int, long (with Java's wrap-around
// on overflow) and big-integer paths chosen by the same bit-size estimates - written from the
// algorithm's description, not from JDK source. There is no JVM in this environment to compare
// against, so parity with Java 8's output is unpinned; tests/test_codec.py checks the
// properties that must hold (round trip, never shorter than the shortest form, the fixed
// documented cases).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "json_codec.h"

namespace gale {
namespace codec {
namespace {

// ---- minimal unsigned big integer (little-endian 32-bit limbs) for the wide path ----
struct Big {
  std::vector<uint32_t> d;
  static Big from(uint64_t v) {
    Big b;
    while (v) {
      b.d.push_back((uint32_t)v);
      v >>= 32;
    }
    return b;
  }
  void trim() {
    while (!d.empty() && d.back() == 0) d.pop_back();
  }
  void mul_small(uint32_t m) {
    uint64_t c = 0;
    for (uint32_t& x : d) {
      const uint64_t v = (uint64_t)x * m + c;
      x = (uint32_t)v;
      c = v >> 32;
    }
    if (c) d.push_back((uint32_t)c);
  }
  void mul_pow5(int n) {
    for (; n >= 13; n -= 13) mul_small(1220703125u);  // 5^13
    uint32_t p = 1;
    for (int i = 0; i < n; ++i) p *= 5u;
    if (p > 1) mul_small(p);
  }
  void shl(int s) {
    if (d.empty() || s <= 0) return;
    const int w = s / 32, b = s % 32;
    std::vector<uint32_t> r(d.size() + (size_t)w + 1, 0);
    for (size_t i = 0; i < d.size(); ++i) {
      r[i + (size_t)w] |= d[i] << b;
      if (b) r[i + (size_t)w + 1] |= d[i] >> (32 - b);
    }
    d.swap(r);
    trim();
  }
  static int cmp(const Big& a, const Big& b) {
    if (a.d.size() != b.d.size()) return a.d.size() < b.d.size() ? -1 : 1;
    for (size_t i = a.d.size(); i-- > 0;)
      if (a.d[i] != b.d[i]) return a.d[i] < b.d[i] ? -1 : 1;
    return 0;
  }
  void sub(const Big& b) {  // *this >= b
    int64_t br = 0;
    for (size_t i = 0; i < d.size(); ++i) {
      int64_t v = (int64_t)d[i] - br - (i < b.d.size() ? (int64_t)b.d[i] : 0);
      br = v < 0;
      d[i] = (uint32_t)(v + (br << 32));
    }
    trim();
  }
  static Big add(const Big& a, const Big& b) {
    Big r;
    uint64_t c = 0;
    for (size_t i = 0; i < std::max(a.d.size(), b.d.size()); ++i) {
      const uint64_t v = (uint64_t)(i < a.d.size() ? a.d[i] : 0) +
                         (i < b.d.size() ? b.d[i] : 0) + c;
      r.d.push_back((uint32_t)v);
      c = v >> 32;
    }
    if (c) r.d.push_back((uint32_t)c);
    return r;
  }
};

Big pow52(uint64_t m, int p5, int p2) {
  Big b = Big::from(m);
  b.mul_pow5(p5);
  b.shl(p2);
  return b;
}

int bitlen64(uint64_t v) { return v ? 64 - __builtin_clzll(v) : 0; }

// bits of 5^i (0 for i = 0), i < 27: the digit-loop size estimates
int n5bits(int i) {
  if (i == 0) return 0;
  uint64_t p = 1;
  for (int k = 0; k < i; ++k) p *= 5u;
  return bitlen64(p);
}
constexpr int kN5 = 27;
uint64_t pow5_64(int i) {
  uint64_t p = 1;
  for (int k = 0; k < i; ++k) p *= 5u;
  return p;
}

struct Digits {
  char d[24];
  int first = 0, n = 0, dec_exp = 0;  // value = 0.d[first..first+n) x 10^dec_exp
  void roundup() {
    int i = first + n - 1;
    char q = d[i];
    if (q == '9') {
      while (q == '9' && i > first) {
        d[i] = '0';
        q = d[--i];
      }
      if (q == '9') {  // carry out of the leading digit
        dec_exp += 1;
        d[first] = '1';
        return;
      }
    }
    d[i] = (char)(q + 1);
  }
};

// integer values below 2^63 (no fraction bits): exact digits, rounded to the significant ones
void long_digits(Digits& D, int dec_exp, uint64_t v, int insignificant) {
  if (insignificant) {
    uint64_t p10 = 1;
    for (int k = 0; k < insignificant; ++k) p10 *= 10u;
    const uint64_t res = v % p10;
    v /= p10;
    dec_exp += insignificant;
    if (res >= (p10 >> 1)) ++v;
  }
  int pos = 23;
  int c = (int)(v % 10);
  v /= 10;
  while (c == 0) {  // trailing zeros move into the exponent
    ++dec_exp;
    c = (int)(v % 10);
    v /= 10;
  }
  while (v != 0) {
    D.d[pos--] = (char)('0' + c);
    ++dec_exp;
    c = (int)(v % 10);
    v /= 10;
  }
  D.d[pos] = (char)('0' + c);
  D.dec_exp = dec_exp + 1;
  D.first = pos;
  D.n = 24 - pos;
}

// floor of the decimal exponent estimate (a linear fit of log10 over the binade)
int estimate_dec_exp(uint64_t fract_bits, int bin_exp) {
  uint64_t bits = 0x3ff0000000000000ull | (fract_bits & 0x000fffffffffffffull);
  double d2;
  memcpy(&d2, &bits, 8);
  const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + (double)bin_exp * 0.301029995663981;
  return (int)floor(d);
}

// the digit loop on machine integers with Java's wrap-around semantics (T = int32 / int64)
template <typename T, typename U>
void small_loop(Digits& D, int& dec_exp, T b, T s, T m, bool& low, bool& high, int64_t& ldd) {
  const T tens = (T)((U)s * 10u);
  auto mul10 = [](T x) { return (T)((U)x * 10u); };
  int nd = 0;
  int q = (int)(b / s);
  b = mul10(b % s);
  m = mul10(m);
  low = b < m;
  high = (T)((U)b + (U)m) > tens;
  if (q == 0 && !high)
    --dec_exp;  // the estimate was one too high
  else
    D.d[nd++] = (char)('0' + q);
  if (dec_exp < -3 || dec_exp >= 8) high = low = false;  // E-form: at least two digits
  while (!low && !high) {
    q = (int)(b / s);
    b = mul10(b % s);
    m = mul10(m);
    if (m > 0) {
      low = b < m;
      high = (T)((U)b + (U)m) > tens;
    } else {  // m wrapped: both conditions
      low = high = true;
    }
    D.d[nd++] = (char)('0' + q);
  }
  ldd = (int64_t)(T)((U)((U)b << 1) - (U)tens);
  D.n = nd;
}

void dtoa(Digits& D, int bin_exp, uint64_t fract_bits, int n_sig_bits) {
  const int tail_zeros = __builtin_ctzll(fract_bits);
  const int n_fract_bits = 53 - tail_zeros;
  const int n_tiny_bits = std::max(0, n_fract_bits - bin_exp - 1);
  if (bin_exp <= 62 && bin_exp >= -21 && n_tiny_bits == 0) {
    // an integer: exact digits (insignificant low-order ones rounded off)
    int insig = 0;
    if (bin_exp > n_sig_bits) {
      const int p2 = bin_exp - n_sig_bits - 1;
      if (p2 > 1 && p2 < 64) insig = (int)((int64_t)p2 * 30103 / 100000);  // floor(p2 log10 2)
    }
    const uint64_t v = bin_exp >= 52 ? fract_bits << (bin_exp - 52) : fract_bits >> (52 - bin_exp);
    long_digits(D, 0, v, insig);
    return;
  }
  int dec_exp = estimate_dec_exp(fract_bits, bin_exp);
  const int B5 = std::max(0, -dec_exp);
  int B2 = B5 + n_tiny_bits + bin_exp;
  const int S5 = std::max(0, dec_exp);
  int S2 = S5 + n_tiny_bits;
  const int M5 = B5;
  int M2 = B2 - n_sig_bits;
  fract_bits >>= tail_zeros;
  B2 -= n_fract_bits - 1;
  const int common2 = std::min(B2, S2);
  B2 -= common2;
  S2 -= common2;
  M2 -= common2;
  if (n_fract_bits == 1) M2 -= 1;  // a power of two: the neighbour below is half as far
  if (M2 < 0) {
    B2 -= M2;
    S2 -= M2;
    M2 = 0;
  }
  const int Bbits = n_fract_bits + B2 + (B5 < kN5 ? n5bits(B5) : B5 * 3);
  const int tenSbits = S2 + 1 + (S5 + 1 < kN5 ? n5bits(S5 + 1) : (S5 + 1) * 3);
  bool low = false, high = false;
  int64_t ldd = 0;
  if (Bbits < 64 && tenSbits < 64) {
    if (Bbits < 32 && tenSbits < 32) {
      const int32_t b = (int32_t)(((uint32_t)fract_bits * (uint32_t)pow5_64(B5)) << B2);
      const int32_t s = (int32_t)((uint32_t)pow5_64(S5) << S2);
      const int32_t m = (int32_t)((uint32_t)pow5_64(M5) << M2);
      small_loop<int32_t, uint32_t>(D, dec_exp, b, s, m, low, high, ldd);
    } else {
      const int64_t b = (int64_t)((fract_bits * pow5_64(B5)) << B2);
      const int64_t s = (int64_t)(pow5_64(S5) << S2);
      const int64_t m = (int64_t)(pow5_64(M5) << M2);
      small_loop<int64_t, uint64_t>(D, dec_exp, b, s, m, low, high, ldd);
    }
  } else {
    Big S = pow52(1, S5, S2);
    Big B = pow52(fract_bits, B5, B2);
    Big M = pow52(1, M5 + 1, M2 + 1);  // 10 M
    const Big tenS = pow52(1, S5 + 1, S2 + 1);
    auto quo_rem = [&]() {  // q = B / S, B = 10 (B % S)
      int q = 0;
      while (Big::cmp(B, S) >= 0) {
        B.sub(S);
        ++q;
      }
      B.mul_small(10);
      return q;
    };
    int nd = 0;
    int q = quo_rem();
    low = Big::cmp(B, M) < 0;
    high = Big::cmp(tenS, Big::add(B, M)) <= 0;
    if (q == 0 && !high)
      --dec_exp;
    else
      D.d[nd++] = (char)('0' + q);
    if (dec_exp < -3 || dec_exp >= 8) high = low = false;
    while (!low && !high) {
      q = quo_rem();
      M.mul_small(10);
      low = Big::cmp(B, M) < 0;
      high = Big::cmp(tenS, Big::add(B, M)) <= 0;
      D.d[nd++] = (char)('0' + q);
    }
    if (high && low) {
      Big B2x = B;
      B2x.shl(1);
      ldd = Big::cmp(B2x, tenS);
    }
    D.n = nd;
  }
  D.dec_exp = dec_exp + 1;
  D.first = 0;
  if (high) {  // the last digit, rounded by the stopping condition
    if (low) {
      if (ldd == 0) {
        if ((D.d[D.first + D.n - 1] & 1) != 0) D.roundup();  // tie: to even
      } else if (ldd > 0) {
        D.roundup();
      }
    } else {
      D.roundup();
    }
  }
}

}  // namespace

int format_float_java8(float v, char* out) {
  uint32_t bits;
  memcpy(&bits, &v, 4);
  const bool neg = bits >> 31;
  uint32_t fract = bits & 0x7fffff;
  int bin_exp = (int)((bits >> 23) & 0xff);
  char* o = out;
  if (bin_exp == 0xff) {
    if (fract) {
      memcpy(o, "NaN", 3);
      return 3;
    }
    if (neg) *o++ = '-';
    memcpy(o, "Infinity", 8);
    return (int)(o - out) + 8;
  }
  if (neg) *o++ = '-';
  int n_sig;
  if (bin_exp == 0) {
    if (fract == 0) {
      memcpy(o, "0.0", 3);
      return (int)(o - out) + 3;
    }
    const int lz = __builtin_clz(fract);
    const int shift = lz - (31 - 23);
    fract <<= shift;
    bin_exp = 1 - shift;
    n_sig = 32 - lz;
  } else {
    fract |= 1u << 23;
    n_sig = 24;
  }
  bin_exp -= 127;
  Digits D;
  dtoa(D, bin_exp, (uint64_t)fract << (52 - 23), n_sig);
  const char* dg = D.d + D.first;
  const int nd = D.n, de = D.dec_exp;
  if (de > 0 && de < 8) {
    const int c = std::min(nd, de);
    memcpy(o, dg, (size_t)c);
    o += c;
    if (c < de) {
      for (int k = c; k < de; ++k) *o++ = '0';
      *o++ = '.';
      *o++ = '0';
    } else {
      *o++ = '.';
      if (c < nd) {
        memcpy(o, dg + c, (size_t)(nd - c));
        o += nd - c;
      } else {
        *o++ = '0';
      }
    }
  } else if (de <= 0 && de > -3) {
    *o++ = '0';
    *o++ = '.';
    for (int k = 0; k < -de; ++k) *o++ = '0';
    memcpy(o, dg, (size_t)nd);
    o += nd;
  } else {
    *o++ = dg[0];
    *o++ = '.';
    if (nd > 1) {
      memcpy(o, dg + 1, (size_t)(nd - 1));
      o += nd - 1;
    } else {
      *o++ = '0';
    }
    *o++ = 'E';
    int e;
    if (de <= 0) {
      *o++ = '-';
      e = -de + 1;
    } else {
      e = de - 1;
    }
    if (e >= 100) {
      *o++ = (char)('0' + e / 100);
      e %= 100;
      *o++ = (char)('0' + e / 10);
      *o++ = (char)('0' + e % 10);
    } else if (e >= 10) {
      *o++ = (char)('0' + e / 10);
      *o++ = (char)('0' + e % 10);
    } else {
      *o++ = (char)('0' + e);
    }
  }
  return (int)(o - out);
}

}  // namespace codec
}  // namespace gale
