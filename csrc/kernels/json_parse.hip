// GPU decoder for the InstObj JSON contract ({"instances": float[N][H][W][C]},
// /root/reference/src/main/java/dke/model/data/InstObj.java:8).
//
// The reference decodes every record with Jackson on a CPU worker thread
// (InferenceBolt.java:76-77) and then copies the nested float arrays into a native tensor
// (Tensor.create, :80). At ~35 KB of text per CIFAR image that float parsing is the dominant host
// cost of the whole pipeline, so gale moves it to the GPU. The host only validates
// the envelope and counts '[' to get N (codec::scan_instances) and stages the raw bytes of the
// instances array; the device then
//   * splits every record's text into kJsonTileBytes = 2 KiB tiles, ONE WAVE PER TILE (64 lanes
//     x 32 contiguous bytes; 4 tiles per 256-thread workgroup, so a 256-record CIFAR batch is
//     ~4600 waves and no kernel here has a workgroup barrier),
//   * classifies 4 bytes per VALU op with a nibble lookup (two v_perm_b32 tables, as in SIMD JSON
//     scanners) into delimiter / number-alphabet / digit bit masks,
//   * pass 1 (json_count_kernel): counts the number tokens of each tile (a token starts at a
//     non-delimiter byte that follows a delimiter) and rejects bytes outside the number alphabet,
//   * pass 2 (json_parse_kernel): stages the tile (+ halos) in LDS, a wave prefix sum over the
//     lanes' token counts gives every token its element index (the record's earlier tiles are
//     summed from pass 1), the token start offsets are compacted into an LDS list and then every
//     lane parses tokens lane, lane+64, ... - balanced work, no per-lane divergence from uneven
//     token density. A token is parsed from a 16-byte register window (v_alignbyte realignment
//     of 5 LDS dwords) with bit-mask arithmetic for the strict JSON grammar
//     -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)? and two 32-bit digit accumulators; anything
//     the window cannot decide (tokens >= 16 bytes, whitespace in the gap, the first/last token of
//     a record) takes the sequential byte-by-byte path, which is the definitive check,
//   * checks that the delimiters in front of token i are exactly what a rectangular
//     [N][H][W][C] array requires ("," inside a pixel, "],[" between pixels, "]],[[" between
//     rows, "]]],[[[" between images, "[[[[" before the first and "]]]]" after the last) and that
//     the token count is N*H*W*C, so ragged or wrong-rank input is rejected like Jackson would.
// Per-record status is the max over the flags raised by its tiles (atomicMax): 1 count mismatch,
// 2 malformed number / element, 3 bad structure; the host zeroes it before the launch.
//
// Each record's bytes start 16-byte aligned; the buffer must be readable 16 bytes past the last
// record. Positions below are record-relative: 0 = the record's 16-byte-aligned start.
#include "common.cuh"
#include "crc32c.cuh"
#include "gale/kernels.h"
#include "exact_decimal.cuh"
#include "text_expand.cuh"

namespace gale {
namespace {

constexpr int kTile = kJsonTileBytes;           // bytes per tile = per wave
constexpr int kLaneBytes = kTile / 64;          // contiguous bytes per lane
constexpr int kChunks = kLaneBytes / 16;        // 16-byte chunks per lane
static_assert(kChunks >= 1 && kChunks * 16 * 64 == kTile, "tile = 64 lanes x 16-byte chunks");
constexpr int kHalo = 64;                       // LDS halo on each side of the tile
constexpr int kWaves = 4;                       // tiles (waves) per workgroup
constexpr int kText = kTile + 2 * kHalo + 16;   // LDS text bytes per wave (+16: window over-read)
constexpr int kMaxTok = kTile / 2;              // a token start needs a delimiter before it

__device__ __forceinline__ bool is_ws(unsigned c) {
  return c == ' ' || c == '\n' || c == '\r' || c == '\t';
}
__device__ __forceinline__ bool is_delim(unsigned c) {
  return c == '[' || c == ']' || c == ',' || is_ws(c);
}

// 10^k for 0 <= k <= 31 from its binary digits, in registers: a per-lane index into a __constant__
// table is a vector memory load (hundreds of cycles per token), this is 5 selects + 4 multiplies.
// Exact for k <= 22 (every partial product is a power of ten that a double represents exactly).
__device__ __forceinline__ double pow10_exact(int k) {
  const double a = (k & 1) ? 1e1 : 1.0, b = (k & 2) ? 1e2 : 1.0, c = (k & 4) ? 1e4 : 1.0,
               d = (k & 8) ? 1e8 : 1.0, e = (k & 16) ? 1e16 : 1.0;
  return ((a * b) * (c * d)) * e;
}

// ---- 4-bytes-per-op classification ------------------------------------------------------------
// Byte groups: g0 {\t \n \r} 0x01, g1 {' ' ','} 0x02, g2 {+ - .} 0x04, g3 digits 0x08,
// g4 {E e} 0x10, g5 {[ ]} 0x20. class(c) = HI[c >> 4] & LO[c & 15] (0 for bytes >= 0x80):
// delimiter = g0|g1|g5, number alphabet = g2|g3|g4, anything else is an invalid byte.
constexpr uint32_t kHi03 = 0x08060001u, kHi47 = 0x00102010u;
constexpr uint32_t kLo03 = 0x0808080Au, kLo47 = 0x08081808u, kLo8B = 0x24010908u,
                   kLoCF = 0x00042502u;
constexpr uint32_t kDelimG = 0x23232323u, kNumG = 0x1C1C1C1Cu, kDigitG = 0x08080808u;

__device__ __forceinline__ uint32_t classify4(uint32_t x) {
  const uint32_t hi = __builtin_amdgcn_perm(kHi47, kHi03, (x >> 4) & 0x07070707u);
  const uint32_t l = x & 0x0F0F0F0Fu;
  const uint32_t s = l & 0x07070707u;
  const uint32_t p0 = __builtin_amdgcn_perm(kLo47, kLo03, s);
  const uint32_t p1 = __builtin_amdgcn_perm(kLoCF, kLo8B, s);
  const uint32_t m = ((l >> 3) & 0x01010101u) * 0xFFu;
  const uint32_t lo = (m & p1) | (~m & p0);
  const uint32_t ascii = ~(((x >> 7) & 0x01010101u) * 0xFFu);
  return hi & lo & ascii;
}

// one bit per byte (bit j = byte j of x has a group bit in g): bytes of (cls & g) are < 0x80
__device__ __forceinline__ uint32_t nz4(uint32_t cls, uint32_t g) {
  const uint32_t t = ((cls & g) + 0x7F7F7F7Fu) & 0x80808080u;
  return ((t >> 7) * 0x01020408u) >> 24;
}

struct Masks16 {
  uint32_t delim, num, digit;  // 16-bit masks, bit j = byte j
};

__device__ __forceinline__ Masks16 classify16(uint32_t w0, uint32_t w1, uint32_t w2,
                                              uint32_t w3) {
  const uint32_t c0 = classify4(w0), c1 = classify4(w1), c2 = classify4(w2), c3 = classify4(w3);
  Masks16 m;
  m.delim = nz4(c0, kDelimG) | nz4(c1, kDelimG) << 4 | nz4(c2, kDelimG) << 8 |
            nz4(c3, kDelimG) << 12;
  m.num = nz4(c0, kNumG) | nz4(c1, kNumG) << 4 | nz4(c2, kNumG) << 8 | nz4(c3, kNumG) << 12;
  m.digit = nz4(c0, kDigitG) | nz4(c1, kDigitG) << 4 | nz4(c2, kDigitG) << 8 |
            nz4(c3, kDigitG) << 12;
  return m;
}

// bits [a, b) of a 32-bit mask, 0 <= a, b <= 16
__device__ __forceinline__ uint32_t bits_range(int a, int b) {
  return b > a ? ((1u << b) - 1u) & ~((1u << a) - 1u) : 0u;
}

// valid-byte mask of the 16 bytes at p for the record extent [beg, end)
__device__ __forceinline__ uint32_t valid16(int p, int beg, int end) {
  return bits_range(min(max(beg - p, 0), 16), min(max(end - p, 0), 16));
}

// Packed masks of one 16-byte chunk at p: low half = delimiter bits (bytes outside the record
// count as delimiters), high half = digit bits (inside the record).
__device__ __forceinline__ uint32_t chunk_masks(const Masks16& m, int p, int beg, int end) {
  const uint32_t vm = valid16(p, beg, end);
  return ((m.delim | ~vm) & 0xFFFFu) | (m.digit & vm) << 16;
}

// Token starts of the lane's kChunks contiguous chunks at o and their packed chunk masks; *bad gets the
// invalid bytes. prev_delim: the byte before o is a delimiter (or outside the record).
__device__ __forceinline__ void token_starts(const uint4 (&v)[kChunks], int o, int beg, int end,
                                             bool prev_delim, uint32_t (&st)[kChunks],
                                             uint32_t (&cm)[kChunks], bool* bad) {
  uint32_t carry = prev_delim ? 1u : 0u;
  bool b = false;
#pragma unroll
  for (int i = 0; i < kChunks; ++i) {
    const Masks16 m = classify16(v[i].x, v[i].y, v[i].z, v[i].w);
    cm[i] = chunk_masks(m, o + 16 * i, beg, end);
    const uint32_t dx = cm[i] & 0xFFFFu;
    const uint32_t tokb = ~dx & 0xFFFFu;
    b |= (tokb & ~m.num) != 0;
    st[i] = tokb & ((dx << 1) | carry) & 0xFFFFu;
    carry = dx >> 15;
  }
  *bad = b;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---- sequential (definitive) path ---------------------------------------------------------
// The record text as seen by one wave: [lo, hi) is mirrored in LDS at text[q - lbase], anything
// else (a very long token or whitespace run) falls back to global memory.
struct Text {
  const uint8_t* g;
  const uint8_t* l;
  int lbase, lo, hi;
  __device__ __forceinline__ unsigned at(int q) const {
    return (q >= lo && q < hi) ? (unsigned)l[q - lbase] : (unsigned)g[q];
  }
};

// ---- correctly rounded decimal -> binary32 (Java Float.parseFloat semantics) ----------------
// x = w * 10^q (w < 2^64 holds the first 19 significant digits; sticky = a nonzero digit was
// dropped after them). A double approximation d of x gives the candidate f = (float)d; f is
// already the correctly rounded result unless d lies within its error bound of a binary32
// rounding midpoint (one rounding of an exact product: only d == midpoint is ambiguous). Those
// rare tokens are decided exactly: x is compared with the midpoint (2M+1) * 2^(e-1) as big
// integers (w * 5^|q| left-aligned in 256 bits against the midpoint's significand), ties to
// even. With dropped digits, w * 10^q < x < (w + 1) * 10^q brackets x; only a midpoint strictly
// inside that bracket (x within 1e-19 relative of it) needs the dropped digits, and then every
// digit of the token is compared with the midpoint's finite decimal expansion (<= 115 digits for
// binary32) - exact for any length, like Java's Float.parseFloat.
// (The 5^k table and the 256-bit comparison live in exact_decimal.cuh.)

// N *= m (base-1e9 limbs, little-endian; m < 2^32)
__device__ __forceinline__ void limbs_mul(uint32_t* N, int* nl, uint32_t m) {
  uint64_t carry = 0;
  for (int i = 0; i < *nl; ++i) {
    const uint64_t v = (uint64_t)N[i] * m + carry;
    N[i] = (uint32_t)(v % 1000000000ull);
    carry = v / 1000000000ull;
  }
  while (carry) {
    N[(*nl)++] = (uint32_t)(carry % 1000000000ull);
    carry /= 1000000000ull;
  }
}

// Sign of x - K * 2^E, x the decimal token at [i0, end) with all of its digits. K * 2^E is
// written as N * 10^-s (N = K * 5^-E, s = -E for E < 0; N = K * 2^E, s = 0 otherwise) and its
// decimal digits are walked against the token's, after comparing the decimal magnitudes.
__device__ __noinline__ int cmp_token_dyadic(const Text& t, int i0, int end, uint64_t K, int E) {
  uint32_t N[16];
  int nl = 0, s = 0;
  for (uint64_t k = K; k || nl == 0; k /= 1000000000ull) N[nl++] = (uint32_t)(k % 1000000000ull);
  if (E >= 0) {
    for (int k = E; k > 0; k -= 29) limbs_mul(N, &nl, 1u << (k < 29 ? k : 29));
  } else {
    s = -E;
    for (int k = s; k > 0; k -= 13) {
      uint32_t p = 1;
      for (int j = 0; j < (k < 13 ? k : 13); ++j) p *= 5u;
      limbs_mul(N, &nl, p);
    }
  }
  int top = 1;
  for (uint32_t v = N[nl - 1]; v >= 10; v /= 10) ++top;
  const int nd = 9 * (nl - 1) + top;  // decimal digits of N
  // token: leading-digit position Lx (x in [10^(Lx-1), 10^Lx)) and exponent
  int k = i0;
  if (t.at(k) == '-') ++k;
  int int_sig = 0, lead_zeros = 0, first = -1;
  unsigned c = k < end ? t.at(k) : 0u;
  for (; c >= '0' && c <= '9'; c = ++k < end ? t.at(k) : 0u)
    if (first >= 0 || c != '0') {
      if (first < 0) first = k;
      ++int_sig;
    }
  if (c == '.')
    for (c = ++k < end ? t.at(k) : 0u; c >= '0' && c <= '9'; c = ++k < end ? t.at(k) : 0u)
      if (first < 0) {
        if (c == '0') ++lead_zeros;
        else first = k;
      }
  int ex = 0;
  if (c == 'e' || c == 'E') {
    c = ++k < end ? t.at(k) : 0u;
    const bool eneg = c == '-';
    if (c == '+' || c == '-') c = ++k < end ? t.at(k) : 0u;
    for (; c >= '0' && c <= '9'; c = ++k < end ? t.at(k) : 0u)
      if (ex < 100000) ex = ex * 10 + (int)(c - '0');
    if (eneg) ex = -ex;
  }
  if (first < 0) return -1;  // x == 0 < K * 2^E
  const int Lx = (int_sig > 0 ? int_sig : -lead_zeros) + ex, Lm = nd - s;
  if (Lx != Lm) return Lx > Lm ? 1 : -1;
  // digit walk from the leading digits
  int j = nd - 1;  // next digit of N, from the top
  for (k = first; k < end; ++k) {
    c = t.at(k);
    if (c == '.') continue;
    if (c < '0' || c > '9') break;
    int dm = 0;
    if (j >= 0) {
      uint32_t v = N[j / 9];
      for (int r = j % 9; r > 0; --r) v /= 10;
      dm = (int)(v % 10);
    }
    const int dx = (int)(c - '0');
    if (dx != dm) return dx > dm ? 1 : -1;
    --j;
  }
  for (; j >= 0; --j) {  // the token ended: x < K * 2^E iff N has a nonzero digit left
    uint32_t v = N[j / 9];
    for (int r = j % 9; r > 0; --r) v /= 10;
    if (v % 10) return -1;
  }
  return 0;
}

// sign of x - K * 2^E for x = w * 10^q (+ dropped digits when sticky)
__device__ __forceinline__ int cmp_x_dyadic(uint64_t w, int q, bool sticky, uint64_t K, int E,
                                            const Text* tok, int i0, int end) {
  const int c = cmp_decimal_dyadic(w, q, K, E);
  if (!sticky) return c;
  if (c >= 0) return 1;                                    // x > w * 10^q >= midpoint
  if (cmp_decimal_dyadic(w + 1, q, K, E) <= 0) return -1;  // x < (w + 1) * 10^q <= midpoint
  return cmp_token_dyadic(*tok, i0, end, K, E);
}

// binary32 value M * 2^e, 0 <= M <= 2^24 (M = 2^24 at e = 104 stands for +inf)
__device__ __forceinline__ void f32_split(float f, uint64_t* M, int* e) {
  const uint32_t b = __float_as_uint(f);
  const uint32_t ex = (b >> 23) & 0xff, fr = b & 0x7fffff;
  if (ex == 0xff) { *M = 1u << 24; *e = 104; }
  else if (ex == 0) { *M = fr; *e = -149; }
  else { *M = fr | 0x800000u; *e = (int)ex - 150; }
}

__device__ __forceinline__ float f32_join(uint64_t M, int e) {
  if (M >= (1u << 24)) { M >>= 1; ++e; }
  if (e > 104) return __uint_as_float(0x7f800000u);
  if (M < (1u << 23)) return __uint_as_float((uint32_t)M);  // subnormal (e == -149)
  return __uint_as_float(((uint32_t)(e + 150) << 23) | ((uint32_t)M & 0x7fffff));
}

__device__ float exact_f32(uint64_t w, int q, bool sticky, double d, const Text* tok, int i0,
                          int end) {
  float f = (float)d;
  uint64_t M;
  int e;
  f32_split(f, &M, &e);
  for (int it = 0; it < 4; ++it) {
    if (M < (1u << 24)) {  // upper neighbour and the midpoint to it
      const int c = cmp_x_dyadic(w, q, sticky, 2 * M + 1, e - 1, tok, i0, end);
      if (c > 0 || (c == 0 && (M & 1))) {
        ++M;
        if (M == (1u << 24) && e < 104) { M = 1u << 23; ++e; }
        continue;
      }
    }
    if (M > 0) {  // lower neighbour and the midpoint to it
      uint64_t Mp = M - 1;
      int ep = e;
      if (M == (1u << 23) && e > -149) { Mp = (1u << 24) - 1; ep = e - 1; }
      if (M == (1u << 24)) { Mp = (1u << 24) - 1; }  // below +inf: FLT_MAX
      const int c = cmp_x_dyadic(w, q, sticky, 2 * Mp + 1, ep - 1, tok, i0, end);
      if (c < 0 || (c == 0 && (M & 1))) {
        M = Mp;
        e = ep;
        continue;
      }
    }
    break;
  }
  return f32_join(M, e);
}

// tok / i0 / end: the token, read again only when sticky and a midpoint is within 1e-19
__device__ __forceinline__ float scale10(uint64_t w, int q, bool neg, bool sticky,
                                         const Text* tok = nullptr, int i0 = 0, int end = 0) {
  float r;
  if (w == 0 || q < -66) {
    r = 0.f;
  } else if (q > 39) {
    r = __uint_as_float(0x7f800000u);
  } else {
    const bool exact_in = w < (1ull << 53) && q >= -22 && q <= 22 && !sticky;
    double d = (double)w;
    if (q >= 0) {
      d = q <= 22 ? d * pow10_exact(q) : d * pow10_exact(22) * pow10_exact(q - 22);
    } else {
      int k = -q;  // <= 66: at most three exact divisions
      while (k > 22) {
        d /= pow10_exact(22);
        k -= 22;
      }
      d /= pow10_exact(k);
    }
    r = (float)d;
    // d within its error bound of a binary32 midpoint (or at the overflow edge) -> exact path
    bool ambiguous = !(r < 3.4028234e38f);
    const uint64_t db = (uint64_t)__double_as_longlong(d);
    const int dexp = (int)((db >> 52) & 0x7ff);
    if (!ambiguous && exact_in && dexp >= 1023 - 126) {
      // normal binary32 range: a midpoint keeps 24 significand bits + the half bit, so the low
      // 29 bits of the double's 52-bit fraction are exactly 1 << 28 (one integer compare)
      ambiguous = (db & 0x1fffffffull) == 0x10000000ull;
    } else if (!ambiguous) {
      const uint32_t rb = __float_as_uint(r);
      const double lo = 0.5 * ((double)r + (double)__uint_as_float(rb - (rb ? 1u : 0u)));
      const double hi = 0.5 * ((double)r + (double)__uint_as_float(rb + 1u));
      if (exact_in) {
        ambiguous = d == lo || d == hi;
      } else {
        const double tol = fabs(d) * 0x1p-50;  // a few double ulps of accumulated error
        ambiguous = fabs(d - lo) <= tol || fabs(d - hi) <= tol;
      }
    }
    if (ambiguous) r = exact_f32(w, q, sticky, d, tok, i0, end);
  }
  return neg ? -r : r;
}

// Strict JSON number starting at i0 and ending at a delimiter or `end`; *len = token length.
__device__ float parse_number(const Text& t, int i0, int end, bool* ok, int* len) {
  int i = i0;
  bool neg = false;
  unsigned c = i < end ? t.at(i) : 0u;
  if (c == '-') { neg = true; ++i; c = i < end ? t.at(i) : 0u; }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool good = true, sticky = false;
  if (i >= end) {
    good = false;
  } else if (c == '0') {
    ++i;
    c = i < end ? t.at(i) : 0u;
    if (c >= '0' && c <= '9') good = false;  // leading zero
  } else if (c >= '1' && c <= '9') {
    while (c >= '0' && c <= '9') {
      if (digits < 19) { mant = mant * 10 + (c - '0'); ++digits; }
      else { ++exp10; sticky |= c != '0'; }
      ++i;
      c = i < end ? t.at(i) : 0u;
    }
  } else {
    good = false;
  }
  if (good && c == '.') {
    ++i;
    c = i < end ? t.at(i) : 0u;
    int fd = 0;
    while (c >= '0' && c <= '9') {
      if (digits < 19) {
        if (mant != 0 || c != '0') ++digits;
        mant = mant * 10 + (c - '0');
        --exp10;
      } else {
        sticky |= c != '0';
      }
      ++fd;
      ++i;
      c = i < end ? t.at(i) : 0u;
    }
    if (fd == 0) good = false;
  }
  if (good && (c == 'e' || c == 'E')) {
    ++i;
    c = i < end ? t.at(i) : 0u;
    bool eneg = false;
    if (c == '+' || c == '-') {
      eneg = c == '-';
      ++i;
      c = i < end ? t.at(i) : 0u;
    }
    int e = 0, ed = 0;
    while (c >= '0' && c <= '9') {
      if (e < 100000) e = e * 10 + (c - '0');
      ++ed;
      ++i;
      c = i < end ? t.at(i) : 0u;
    }
    if (ed == 0) good = false;
    exp10 += eneg ? -e : e;
  }
  while (i < end && !is_delim(c)) {  // trailing garbage in the token
    good = false;
    ++i;
    c = i < end ? t.at(i) : 0u;
  }
  *ok = good;
  *len = i - i0;
  return good ? scale10(mant, exp10, neg, sticky, &t, i0, i) : 0.f;
}

// n / d for n < 2^32, d < 2^20 from a double reciprocal rd = 1/d: the product is below the true
// quotient by < 1 (never above it by a whole unit), so one correction step is exact.
__device__ __forceinline__ uint32_t udiv_rcp(uint32_t n, uint32_t d, double rd) {
  uint32_t q = (uint32_t)((double)n * rd);
  if (n - q * d >= d) ++q;
  return q;
}

struct Dims {
  uint32_t C, W, H;
  double rC, rW, rH;
};

// number of array dimensions that close between element idx-1 and idx (idx > 0)
__device__ __forceinline__ int wraps(uint32_t idx, const Dims& d) {
  const uint32_t px = udiv_rcp(idx, d.C, d.rC);
  if (idx - px * d.C) return 0;
  const uint32_t row = udiv_rcp(px, d.W, d.rW);
  if (px - row * d.W) return 1;
  return (row - udiv_rcp(row, d.H, d.rH) * d.H) ? 2 : 3;
}

// Delimiters in front of token `idx` (scanning back from pos-1). Between tokens the text must be
// ws* (']' ws*)^k ',' ws* ('[' ws*)^k with k = wraps(idx).
__device__ bool gap_ok(const Text& t, int beg, int pos, uint32_t idx, int k) {
  int opens = 0, closes = 0, commas = 0;
  int q = pos - 1;
  for (; q >= beg; --q) {
    const unsigned c = t.at(q);
    if (is_ws(c)) continue;
    if (c == '[') {
      if (commas) return false;
      ++opens;
    } else if (c == ',') {
      if (commas) return false;
      ++commas;
    } else if (c == ']') {
      if (!commas) return false;
      ++closes;
    } else {
      break;
    }
  }
  if (idx == 0) return q < beg && opens == 4 && commas == 0 && closes == 0;
  return q >= beg && commas == 1 && opens == k && closes == k;
}

// After the last token: ws* (']' ws*)^4 up to the end of the array text.
__device__ bool tail_ok(const Text& t, int pos, int end) {
  int closes = 0;
  for (int q = pos; q < end; ++q) {
    const unsigned c = t.at(q);
    if (is_ws(c)) continue;
    if (c != ']') return false;
    ++closes;
  }
  return closes == 4;
}

// ---- window (fast) path ---------------------------------------------------------------------
__device__ __forceinline__ uint32_t byte_at(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                            int k) {
  const uint32_t lo = (k & 4) ? w1 : w0;
  const uint32_t hi = (k & 4) ? w3 : w2;
  return (((k & 8) ? hi : lo) >> ((k & 3) * 8)) & 0xFFu;
}

// Parses the token at LDS offset x from a 16-byte window; m0/m1 = packed masks of the chunk
// holding the token start and the next one, off = the start's offset in its chunk. Returns false
// when the window cannot decide (the caller then runs parse_number).
__device__ __forceinline__ bool parse_window(const uint8_t* text, int x, uint32_t m0, uint32_t m1,
                                             int off, float* out) {
  const uint32_t* tw = reinterpret_cast<const uint32_t*>(text) + (x >> 2);
  const uint32_t sh = (uint32_t)(x & 3);
  const uint32_t d0 = tw[0], d1 = tw[1], d2 = tw[2], d3 = tw[3], d4 = tw[4];
  const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
  const uint32_t w3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
  const uint32_t delim = (((m1 << 16) | (m0 & 0xFFFFu)) >> off) & 0xFFFFu;
  const uint32_t D = (((m1 & 0xFFFF0000u) | (m0 >> 16)) >> off) & 0xFFFFu;
  const uint32_t tok = ~delim & 0xFFFFu;
  const int L = __builtin_ctz(~tok);  // token length (a delimiter or the record end follows)
  if (L >= 16) return false;
  const int s = byte_at(w0, w1, w2, w3, 0) == '-' ? 1 : 0;
  const int ie = s + __builtin_ctz(~(D >> s));
  bool ok = ie > s && !(byte_at(w0, w1, w2, w3, s) == '0' && ie > s + 1);
  int fb = ie, fe = ie;
  if (byte_at(w0, w1, w2, w3, ie) == '.' && ie < L) {
    fb = ie + 1;
    fe = fb + __builtin_ctz(~(D >> fb));
    ok &= fe > fb;
  }
  int eb = fe, ee = fe;
  bool eneg = false;
  const uint32_t ce = byte_at(w0, w1, w2, w3, fe);
  if (fe < L && (ce == 'e' || ce == 'E')) {
    int p = fe + 1;
    const uint32_t c2 = byte_at(w0, w1, w2, w3, p);
    if (p < L && (c2 == '+' || c2 == '-')) {
      eneg = c2 == '-';
      ++p;
    }
    eb = p;
    ee = p + __builtin_ctz(~(D >> p));
    ok &= ee > eb;
  }
  if (!ok || ee != L) return false;
  const uint32_t mm = bits_range(s, ie) | bits_range(fb, fe);  // mantissa digits
  // <= 15 mantissa digits (the window): exact in a 64-bit accumulator and in a double
  uint64_t a = 0;
  const uint32_t wd[4] = {w0, w1, w2, w3};
#pragma unroll
  for (int j = 0; j < 15; ++j) {
    const uint32_t d = ((wd[j >> 2] >> ((j & 3) * 8)) & 0xFFu) - '0';
    a = ((mm >> j) & 1u) ? a * 10u + d : a;
  }
  uint32_t e = 0;
  for (int p = eb; p < ee; ++p)
    if (e < 100000u) e = e * 10u + (byte_at(w0, w1, w2, w3, p) - '0');
  const int exp10 = (eneg ? -(int)e : (int)e) - (fe - fb);
  *out = scale10(a, exp10, s != 0, false);
  return true;
}

// The k-wrap separator (",", "],[", "]],[[", "]]],[[[") directly in front of x with a digit
// before it; false = undecided (whitespace, other bytes): the caller runs gap_ok.
__device__ __forceinline__ bool gap_window(const uint8_t* text, int x, int k) {
  const uint32_t* tw = reinterpret_cast<const uint32_t*>(text) + ((x - 8) >> 2);
  const uint32_t sh = (uint32_t)(x & 3);
  const uint32_t d0 = tw[0], d1 = tw[1], d2 = tw[2];
  const uint64_t g = (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32 |
                     __builtin_amdgcn_alignbyte(d1, d0, sh);  // bytes x-8 .. x-1
  const int plen = 2 * k + 1;
  const uint64_t pat = k == 0 ? 0x2Cull : k == 1 ? 0x5B2C5Dull
                     : k == 2 ? 0x5B5B2C5D5Dull : 0x5B5B5B2C5D5D5Dull;
  if ((g >> (8 * (8 - plen))) != pat) return false;
  const uint32_t prev = (uint32_t)(g >> (8 * (7 - plen))) & 0xFFu;
  return prev - '0' < 10u;
}

// Number tokens of record-relative tile tl of record r (one wave, the count on every lane);
// *bad: the tile holds a byte outside the number / delimiter alphabet.
__device__ __forceinline__ int tile_tokens(const JsonRecord& r, int tl, const uint8_t* bytes,
                                           bool* bad) {
  const int lane = threadIdx.x & 63;
  const int64_t abeg = r.off & ~(int64_t)15;
  const uint8_t* rb = bytes + abeg;
  const int beg = (int)(r.off - abeg), end = beg + r.len;
  const int o = tl * kTile + kLaneBytes * lane;
  uint4 v[kChunks];
#pragma unroll
  for (int i = 0; i < kChunks; ++i)
    v[i] = (o + 16 * i < end) ? *reinterpret_cast<const uint4*>(rb + o + 16 * i)
                              : make_uint4(0, 0, 0, 0);
  unsigned prevb = __shfl_up(v[kChunks - 1].w >> 24, 1, 64);
  if (lane == 0 && o - 1 >= beg) prevb = rb[o - 1];
  const bool pd = (o - 1 < beg) || is_delim(prevb);
  uint32_t st[kChunks], cm[kChunks];
  token_starts(v, o, beg, end, pd, st, cm, bad);
  int lc = 0;
#pragma unroll
  for (int i = 0; i < kChunks; ++i) lc += __builtin_popcount(st[i]);
  return wave_sum_i(lc);
}

// tile_tokens over a nibble-packed fetch buffer (the fused GPU ingest): each lane expands its
// chunks from the packed stream in registers, stores them into the text image at `bytes` (the
// mirror the parse reads later; tiles of a record are disjoint and cover its 16-byte-aligned
// extent, so every byte the parse reads is stored exactly once) and counts as tile_tokens.
__device__ __forceinline__ int tile_tokens_packed(const JsonRecord& r, int tl, uint8_t* bytes,
                                                  const PackedText& pt, bool* bad) {
  const int lane = threadIdx.x & 63;
  const int64_t abeg = r.off & ~(int64_t)15;
  uint8_t* rb = bytes + abeg;
  const int beg = (int)(r.off - abeg), end = beg + r.len;
  const int o = tl * kTile + kLaneBytes * lane;
  uint4 v[kChunks];
#pragma unroll
  for (int i = 0; i < kChunks; ++i) {
    if (o + 16 * i < end) {
      v[i] = expand16(pt, abeg + o + 16 * i);
      *reinterpret_cast<uint4*>(rb + o + 16 * i) = v[i];
    } else {
      v[i] = make_uint4(0, 0, 0, 0);
    }
  }
  unsigned prevb = __shfl_up(v[kChunks - 1].w >> 24, 1, 64);
  if (lane == 0 && o - 1 >= beg) prevb = expand16(pt, abeg + o - 16).w >> 24;  // (another tile's)
  const bool pd = (o - 1 < beg) || is_delim(prevb);
  uint32_t st[kChunks], cm[kChunks];
  token_starts(v, o, beg, end, pd, st, cm, bad);
  int lc = 0;
#pragma unroll
  for (int i = 0; i < kChunks; ++i) lc += __builtin_popcount(st[i]);
  return wave_sum_i(lc);
}

// tiles of a record: json_tile_count on the device
__device__ __forceinline__ int record_tiles(const JsonRecord& r) {
  const int64_t abeg = r.off & ~(int64_t)15;
  return (int)((r.off + r.len - abeg + kTile - 1) / kTile);
}

// The parse's counting pass for global tile t (one wave): counts[t]. A record whose counts the
// ingest pass already left on the device (has_cnt) is skipped.
__device__ __forceinline__ void count_tile(JsonRecord* recs, const int* tile_rec, int t,
                                           const uint8_t* bytes, int* counts, int* status) {
  const int ri = tile_rec[t];
  const JsonRecord r = recs[ri];
  if (r.has_cnt) return;
  bool bad;
  const int cnt = tile_tokens(r, t - r.tile0, bytes, &bad);
  if ((threadIdx.x & 63) == 0) counts[t] = cnt;
  if (bad) atomicMax(status ? &status[ri] : &recs[ri].status, 2);
}

// The ingest pass's counting of one tile group (one workgroup: wave w counts tile tl0 + w of the
// record, up to kGroupTiles = kWaves tiles). The record's count block (at counts + tile0 + grp0)
// gets its nt tile counts, then one sum per group; gsum[g] (contiguous, read back by the host)
// gets the group's sum too, and the host adds a record's group sums for its image count. The
// parse finds a tile's first element index from nt / kGroupTiles group sums plus < kGroupTiles
// tile counts. (Per-tile atomics on one record counter serialise: an ImageNet record is ~850
// tiles, 80 of the 92 us of a 15 MB fetch's ingest launch, tools/bench_ingest.py.)
// gbad non-null: the group's verdict goes to gbad[g] (0 / 2) with a plain store instead of an
// atomic on the record's status - the plan and the results may then live in host memory (the
// GPU ingest reads them over the link and writes them back without copies; device atomics on
// fine-grained host memory are not something to rely on).
template <bool PACKED>
__device__ __forceinline__ void count_group(JsonRecord* recs, const int2* groups, int g,
                                            uint8_t* bytes, const PackedText& pt, int* counts,
                                            int* gsum, int* gbad, int* lds8) {
  const int wave = threadIdx.x >> 6;
  const int2 gr = groups[g];  // (record, record-relative first tile)
  const JsonRecord r = recs[gr.x];
  const int nt = record_tiles(r);
  const int tl = gr.y + wave;
  int cnt = 0;
  bool bad = false;
  if (tl < nt) {
    cnt = PACKED ? tile_tokens_packed(r, tl, bytes, pt, &bad)
                 : tile_tokens(r, tl, bytes, &bad);  // (bad: this lane's bytes)
    if ((threadIdx.x & 63) == 0) counts[r.tile0 + (int)r.grp0 + tl] = cnt;
    if (bad && !gbad) atomicMax(&recs[gr.x].status, 2);
    bad = __ballot(bad) != 0;  // the wave's verdict, for lane 0 below
  }
  if ((threadIdx.x & 63) == 0) {
    lds8[wave] = cnt;
    lds8[kGroupTiles + wave] = bad ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0, nbad = 0;
#pragma unroll
    for (int w = 0; w < kGroupTiles; ++w) {
      acc += lds8[w];
      nbad += lds8[kGroupTiles + w];
    }
    counts[r.tile0 + (int)r.grp0 + nt + gr.y / kGroupTiles] = acc;
    gsum[g] = acc;
    if (gbad) gbad[g] = nbad ? 2 : 0;
  }
}

__global__ __launch_bounds__(256) void json_count_kernel(JsonRecord* recs, const int* tile_rec,
                                                         int ntiles, const uint8_t* bytes,
                                                         int* counts, const int* d_ntiles,
                                                         int* status) {
  const int t = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (d_ntiles) ntiles = min(ntiles, *d_ntiles);
  if (t >= ntiles) return;  // (no workgroup barriers in this kernel)
  count_tile(recs, tile_rec, t, bytes, counts, status);
}

// crc::crc_windows over a packed span: a lane's 64-byte piece [wa, wa + 64) is assembled from
// the (at most five) 16-byte-aligned chunks covering it, expanded in registers, shifted into place
// (wa % 16 is the same on every lane of a window: pieces are 64 bytes apart, ending at the
// window's end) and folded as sixteen 32-bit words. Bytes before the window start are zeroed:
// with a zero initial register, leading zero bytes leave the raw CRC unchanged.
__device__ __forceinline__ void crc_windows_packed(const PackedText& pt, const CrcChunk* chunks,
                                                   int n, const uint32_t* T, uint32_t* out,
                                                   int block, int nblocks) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c = block * crc::kCrcWaves + wave; c < n; c += nblocks * crc::kCrcWaves) {
    const CrcChunk ch = chunks[c];
    const int64_t cs = ch.end - ch.len;
    const int64_t wa = ch.end - (int64_t)64 * (64 - lane);  // this lane's piece [wa, wa + 64)
    const int64_t hi = wa + 64;
    uint32_t crc = 0;
    if (hi > cs) {
      const int64_t b16 = wa & ~(int64_t)15;
      uint32_t w[20];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int64_t p = b16 + 16 * j;
        const uint4 v = (p < hi && p + 16 > cs) ? expand16(pt, p) : make_uint4(0, 0, 0, 0);
        w[4 * j] = v.x;
        w[4 * j + 1] = v.y;
        w[4 * j + 2] = v.z;
        w[4 * j + 3] = v.w;
      }
      const uint32_t sh = (uint32_t)(wa & 3);
      uint32_t x[16];
      switch ((int)((wa & 15) >> 2)) {  // (wave-uniform)
#define GALE_ALIGN_WORDS(D)                                                       \
  _Pragma("unroll") for (int t = 0; t < 16; ++t) x[t] =                           \
      __builtin_amdgcn_alignbyte(w[t + (D) + 1], w[t + (D)], sh);
        case 0: GALE_ALIGN_WORDS(0) break;
        case 1: GALE_ALIGN_WORDS(1) break;
        case 2: GALE_ALIGN_WORDS(2) break;
        default: GALE_ALIGN_WORDS(3) break;
#undef GALE_ALIGN_WORDS
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int64_t at = wa + 4 * t;  // word t = bytes [at, at + 4)
        uint32_t v = x[t];
        if (at + 4 <= cs) v = 0;
        else if (at < cs) v &= 0xffffffffu << (8 * (uint32_t)(cs - at));
        crc = crc::crc_word(T, crc, v);
      }
    }
    crc = crc::gf2_mulmod(crc, T[1024 + lane]);  // over the 64 * (63 - lane) bytes that follow
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) crc ^= __shfl_xor(crc, o, 64);
    if (lane == 0) out[c] = crc;
  }
}

// The ingest pass of a fetch buffer in one launch: CRC window workgroups first (they stage the
// CRC tables in LDS behind one barrier), then one workgroup per tile group (the branches are
// uniform per workgroup).
static_assert(kGroupTiles == kWaves, "one tile group per counting workgroup");
// PACKED: the buffer's text is the nibble-packed stream pt (the fetch body crossed the link
// packed); CRC windows and counting waves expand it in registers, and the counting waves store
// the record text into `bytes` for the parse - the separate text_unpack pass is folded in.
template <bool PACKED>
__global__ __launch_bounds__(256) void ingest_crc_count_kernel(
    uint8_t* bytes, PackedText pt, const CrcChunk* chunks, int nchunks, const uint32_t* tables,
    uint32_t* crc_out, int crc_blocks, JsonRecord* recs, const int2* groups, int ngroups,
    int* counts, int* gsum, int* gbad) {
  __shared__ uint32_t T[crc::kTableWords];
  if ((int)blockIdx.x < crc_blocks) {
    crc::crc_stage_tables(tables, T);
    if (PACKED)
      crc_windows_packed(pt, chunks, nchunks, T, crc_out, blockIdx.x, crc_blocks);
    else
      crc::crc_windows(bytes, chunks, nchunks, T, crc_out, blockIdx.x, crc_blocks);
    return;
  }
  const int g = (int)blockIdx.x - crc_blocks;
  if (g >= ngroups) return;
  count_group<PACKED>(recs, groups, g, bytes, pt, counts, gsum, gbad, reinterpret_cast<int*>(T));
}

__global__ __launch_bounds__(256) void json_parse_kernel(JsonRecord* recs, const int* tile_rec,
                                                         int ntiles, const uint8_t* bytes, int H,
                                                         int W, int C, const int* counts,
                                                         float* out, const int* d_ntiles,
                                                         int* status, int* tile_bad) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_text[kWaves][kText];
  __shared__ uint16_t lds_tok[kWaves][kMaxTok];
  __shared__ uint32_t lds_cm[kWaves][kTile / 16 + 1];  // packed masks of the tile's chunks + 1
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = blockIdx.x * kWaves + wave;
  if (d_ntiles) ntiles = min(ntiles, *d_ntiles);
  if (t >= ntiles) return;  // (waves only share LDS regions of their own: no barriers)
  uint8_t* text = lds_text[wave];
  uint16_t* tok = lds_tok[wave];
  uint32_t* cmk = lds_cm[wave];
  const int ri = tile_rec[t];
  const JsonRecord r = recs[ri];
  const int64_t abeg = r.off & ~(int64_t)15;
  const uint8_t* rb = bytes + abeg;
  const int beg = (int)(r.off - abeg), end = beg + r.len;
  const int aend = (end + 15) & ~15;
  const int per_image = H * W * C;
  int expected = r.images * per_image;
  if (r.images < 0) {
    // parse at ingest (has_cnt; the host has not read the counts yet): the record's image count
    // from its group sums in the count block. A total that is not a whole number of images, or
    // more images than the record's text can hold (>= 2 bytes per number: the arena reserves
    // len / (2 * per_image) slots for it), expects nothing: no element is stored and the last
    // tile reports the count mismatch.
    const int* rc = reinterpret_cast<const int*>(bytes + r.cnt_off);
    const int nt = record_tiles(r);
    const int ng = (nt + kGroupTiles - 1) / kGroupTiles;
    int s = 0;
    for (int k = lane; k < ng; k += 64) s += rc[nt + k];
    const int tot = wave_sum_i(s);
    expected = (tot % per_image == 0 && tot / per_image <= r.len / (2 * per_image)) ? tot : 0;
  }
  const int tl = t - r.tile0;
  const int t0 = tl * kTile;
  const bool last_tile = t0 + kTile >= end;

  // stage [t0 - halo, t0 + tile + halo) clipped to the record's 16-byte-aligned extent
  Text tx;
  tx.g = rb;
  tx.l = text;
  tx.lbase = t0 - kHalo;
  tx.lo = max(t0 - kHalo, 0);
  tx.hi = min(t0 + kTile + kHalo, aend);
  for (int q = tx.lo + 16 * lane; q < tx.hi; q += 16 * 64)
    *reinterpret_cast<uint4*>(text + (q - tx.lbase)) = *reinterpret_cast<const uint4*>(rb + q);

  // first element index of this tile: the token counts of the record's earlier tiles
  int part = 0;
  if (r.has_cnt) {  // counted by the ingest pass, left next to the fetch buffer's device mirror:
    // the sums of the whole tile groups before this tile, then its group's earlier tiles
    const int* rc = reinterpret_cast<const int*>(bytes + r.cnt_off);
    const int* gs = rc + record_tiles(r);
    const int gi = tl / kGroupTiles;
    for (int k = lane; k < gi; k += 64) part += gs[k];
    if (lane < tl - gi * kGroupTiles) part += rc[gi * kGroupTiles + lane];
  } else {
    for (int k = r.tile0 + lane; k < t; k += 64) part += counts[k];
  }
  const int base = wave_sum_i(part);
  wave_lds_sync();

  // token starts of this lane's 64 bytes, then a wave prefix sum -> local token indices
  const int o = t0 + kLaneBytes * lane;
  uint4 v[kChunks];
#pragma unroll
  for (int i = 0; i < kChunks; ++i)
    v[i] = (o + 16 * i < end) ? *reinterpret_cast<const uint4*>(text + (o + 16 * i - tx.lbase))
                              : make_uint4(0, 0, 0, 0);
  const bool pd = (o - 1 < beg) || is_delim(text[o - 1 - tx.lbase]);
  uint32_t st[kChunks], cm[kChunks];
  bool bad_ignored;
  token_starts(v, o, beg, end, pd, st, cm, &bad_ignored);
#pragma unroll
  for (int i = 0; i < kChunks; ++i) cmk[kChunks * lane + i] = cm[i];
  if (lane == 63) {  // the chunk after the tile (a window of the tile's last tokens reaches it)
    const int p = t0 + kTile;
    const uint4 h = p < end ? *reinterpret_cast<const uint4*>(text + (p - tx.lbase))
                            : make_uint4(0, 0, 0, 0);
    cmk[kTile / 16] = chunk_masks(classify16(h.x, h.y, h.z, h.w), p, beg, end);
  }
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < kChunks; ++i) cnt += __builtin_popcount(st[i]);
  int inc = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(inc, d, 64);
    if (lane >= d) inc += u;
  }
  const int ntok = __shfl(inc, 63, 64);
  int li = inc - cnt;
#pragma unroll
  for (int i = 0; i < kChunks; ++i) {
    uint32_t s = st[i];
    while (s) {
      const int j = __builtin_ctz(s);
      s &= s - 1;
      tok[li++] = (uint16_t)(o + 16 * i + j - tx.lbase);
    }
  }
  wave_lds_sync();

  // parse: lane handles tokens lane, lane + 64, ... (consecutive lanes -> consecutive elements)
  Dims dims;
  dims.C = (uint32_t)C; dims.W = (uint32_t)W; dims.H = (uint32_t)H;
  dims.rC = 1.0 / C; dims.rW = 1.0 / W; dims.rH = 1.0 / H;
  float* dst = out + (int64_t)r.slot * per_image;
  int bad = 0;
  for (int j = lane; j < ntok; j += 64) {
    const int x = tok[j];
    const int pos = x + tx.lbase;
    const int idx = base + j;
    float val;
    int len = 0;
    bool ok;
    const int ci = (pos - t0) >> 4;
    if (parse_window(text, x, cmk[ci], cmk[ci + 1], pos & 15, &val)) {
      ok = true;
      len = -1;  // only the last element needs its length (tail check)
    } else {
      ok = false;
      val = parse_number(tx, pos, end, &ok, &len);
    }
    if (!ok) {
      bad = max(bad, 2);
    } else {
      const int k = idx > 0 ? wraps((uint32_t)idx, dims) : 0;
      const bool fast_gap = idx > 0 && pos - 8 >= tx.lo && pos - (2 * k + 2) >= beg &&
                            gap_window(text, x, k);
      if (!fast_gap && !gap_ok(tx, beg, pos, (uint32_t)idx, k)) {
        bad = 3;
      } else if (idx == expected - 1) {
        if (len < 0) parse_number(tx, pos, end, &ok, &len);
        if (!tail_ok(tx, pos + len, end)) bad = 3;
      }
    }
    if (idx < expected) dst[idx] = val;
  }
  if (last_tile && lane == 0 && base + ntok != expected) bad = max(bad, 1);
  if (tile_bad) {
    // the tile's verdict by a plain store (host-mapped results: no atomics over the link)
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) bad = max(bad, __shfl_xor(bad, d, 64));
    if (lane == 0) tile_bad[t] = bad;
  } else if (bad) {
    atomicMax(status ? &status[ri] : &recs[ri].status, bad);
  }
}

}  // namespace



int json_tile_count(int64_t off, int32_t len) {
  if (len <= 0) return 0;
  const int64_t abeg = off & ~(int64_t)15;
  return (int)((off + len - abeg + kJsonTileBytes - 1) / kJsonTileBytes);
}

hipError_t ingest_crc_count(const uint8_t* bytes, const CrcChunk* chunks, int nchunks,
                            const uint32_t* tables, uint32_t* crc_out, int nrec, int ngroups,
                            JsonRecord* recs, const int2* groups, int* counts, int* gsum,
                            int* gbad, hipStream_t stream, const uint8_t* packed,
                            const uint32_t* tab, uint8_t* text_out) {
  if (nrec <= 0) ngroups = 0;
  int crc_blocks = (nchunks + crc::kCrcWaves - 1) / crc::kCrcWaves;
  if (crc_blocks > 1024) crc_blocks = 1024;  // (windows loop: the table load is amortised)
  if (crc_blocks + ngroups == 0) return hipSuccess;
  if (packed) {
    if (!tab || !text_out || (reinterpret_cast<uintptr_t>(packed) & 7) ||
        (reinterpret_cast<uintptr_t>(text_out) & 15))
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(ingest_crc_count_kernel<true>, dim3(crc_blocks + ngroups), dim3(256), 0,
                       stream, text_out, PackedText{packed, tab}, chunks, nchunks, tables,
                       crc_out, crc_blocks, recs, groups, ngroups, counts, gsum, gbad);
  } else {
    hipLaunchKernelGGL(ingest_crc_count_kernel<false>, dim3(crc_blocks + ngroups), dim3(256), 0,
                       stream, const_cast<uint8_t*>(bytes), PackedText{nullptr, nullptr}, chunks,
                       nchunks, tables, crc_out, crc_blocks, recs, groups, ngroups, counts, gsum,
                       gbad);
  }
  return hipGetLastError();
}

hipError_t json_parse_instances(int nrec, int ntiles, JsonRecord* recs, const int* tile_rec,
                                const uint8_t* bytes, int H, int W, int C, int* tile_counts,
                                float* out, hipStream_t stream, bool count_pass,
                                const int* d_ntiles, int* status, int* tile_bad) {
  if (nrec <= 0 || ntiles <= 0) return hipSuccess;
  if (H <= 0 || W <= 0 || C <= 0) return hipErrorInvalidValue;
  if (tile_bad && count_pass) return hipErrorInvalidValue;  // (per-tile verdicts: counted records)
  const int blocks = (ntiles + kWaves - 1) / kWaves;
  if (count_pass)
    hipLaunchKernelGGL(json_count_kernel, dim3(blocks), dim3(64 * kWaves), 0, stream, recs,
                       tile_rec, ntiles, bytes, tile_counts, d_ntiles, status);
  hipLaunchKernelGGL(json_parse_kernel, dim3(blocks), dim3(64 * kWaves), 0, stream, recs,
                     tile_rec, ntiles, bytes, H, W, C, tile_counts, out, d_ntiles, status,
                     tile_bad);
  return hipGetLastError();
}

}  // namespace gale
