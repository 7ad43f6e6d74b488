// Kafka wire primitives: CRC32C and the RecordBatch v2 codec (see wire.h).
#include "wire.h"

#include <stdlib.h>

#include <immintrin.h>
#include <nmmintrin.h>

namespace gale {
namespace kafka {

namespace {

// CRC32C with three independent crc32q streams (the instruction has 3-cycle latency and 1-cycle
// throughput, so one serial chain runs at a third of the unit's rate). Partial CRCs are joined
// with crc(A|B) = crc(A) * x^(8|B|) mod P  ^  crc(B) (raw, un-inverted states): the CRC register
// is a polynomial over GF(2) and appending k zero bits multiplies it by x^k modulo P.
constexpr uint32_t kPoly = 0x82f63b78u;  // CRC-32C polynomial, reflected
constexpr size_t kLong = 8192, kShort = 256;

// a * b mod P in the reflected domain (bit 31 = coefficient of x^0): sum of b * x^i over the set
// bits i of a, b advancing by one x per step (one zero bit through the CRC register)
uint32_t poly_mulmod(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 0; i < 32 && a; ++i) {
    const uint32_t bit = 0x80000000u >> i;
    if (a & bit) {
      r ^= b;
      a &= ~bit;
    }
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return r;
}

// x^(8 * 2^k) mod P for k = 0..63 (k = 0: one byte), by repeated squaring
struct BytePowers {
  uint32_t p[64];
  BytePowers() {
    p[0] = 0x80000000u >> 8;  // x^8
    for (int k = 1; k < 64; ++k) p[k] = poly_mulmod(p[k - 1], p[k - 1]);
  }
};
const BytePowers& byte_powers() {
  static const BytePowers t;
  return t;
}

// x^(8 n) mod P
uint32_t x8n(uint64_t n) {
  const BytePowers& bp = byte_powers();
  uint32_t r = 0x80000000u;  // x^0
  for (int k = 0; n; ++k, n >>= 1)
    if (n & 1) r = poly_mulmod(r, bp.p[k]);
  return r;
}

// Fixed-length shift by table lookup: t[j][v] = (v << 8j) * x^(8 len) mod P (linear in the
// state, so four byte lookups cover a 32-bit register)
struct ShiftTable {
  uint32_t t[4][256];
  explicit ShiftTable(size_t len) {
    const uint32_t op = x8n(len);
    for (uint32_t v = 0; v < 256; ++v)
      for (int j = 0; j < 4; ++j) t[j][v] = poly_mulmod(v << (8 * j), op);
  }
  uint32_t shift(uint32_t crc) const {
    return t[0][crc & 0xff] ^ t[1][(crc >> 8) & 0xff] ^ t[2][(crc >> 16) & 0xff] ^ t[3][crc >> 24];
  }
};

const ShiftTable& long_table() {
  static const ShiftTable t(kLong);
  return t;
}
const ShiftTable& short_table() {
  static const ShiftTable t(kShort);
  return t;
}

inline uint64_t ld64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

// three streams over consecutive blocks of `blk` bytes, combined with `tab`
inline const uint8_t* crc3(const uint8_t* p, size_t& n, uint64_t& c0, size_t blk,
                           const ShiftTable& tab) {
  while (n >= 3 * blk) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t* end = p + blk;
    do {
      c0 = _mm_crc32_u64(c0, ld64(p));
      c1 = _mm_crc32_u64(c1, ld64(p + blk));
      c2 = _mm_crc32_u64(c2, ld64(p + 2 * blk));
      p += 8;
    } while (p < end);
    c0 = tab.shift((uint32_t)c0) ^ (uint32_t)c1;
    c0 = tab.shift((uint32_t)c0) ^ (uint32_t)c2;
    p += 2 * blk;
    n -= 3 * blk;
  }
  return p;
}

// CRC32C by carry-less-multiply folding on 512-bit registers (VPCLMULQDQ + AVX-512, e.g. Zen 4/5
// hosts of MI355X nodes): four zmm accumulators fold 256 bytes per iteration, ~4x the crc32q
// rate. Reflected-domain folding of a 128-bit lane R = [lo, hi] over L bits is
//   R' = clmul(lo, reflect32(x^(64+L-1) mod P) << 32) ^ clmul(hi, reflect32(x^(L-1) mod P) << 32)
// (P = CRC-32C); the folded last 16 bytes are finished with two crc32q from state 0 (the initial
// state is XORed into the first 4 bytes, which is exactly what crc32q does with its state).
// Constants derived and checked bit-exactly against the bytewise definition offline.
constexpr uint64_t kF2048a = 0xe9a5d8be00000000ull, kF2048b = 0x1426a81500000000ull;
constexpr uint64_t kF512a = 0x1c19243b00000000ull, kF512b = 0x75bba45b00000000ull;
constexpr uint64_t kF128a = 0x3743f7bd00000000ull, kF128b = 0x3171d43000000000ull;

__attribute__((target("avx512f,avx512vl,vpclmulqdq,pclmul,sse4.2"))) inline __m512i
fold512(__m512i x, __m512i k, __m512i next) {
  return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00),
                                   _mm512_clmulepi64_epi128(x, k, 0x11), next, 0x96);
}

__attribute__((target("avx512f,avx512vl,vpclmulqdq,pclmul,sse4.2"))) inline __m128i
fold128(__m128i a, __m128i k, __m128i next) {
  return _mm_ternarylogic_epi64(_mm_clmulepi64_si128(a, k, 0x00), _mm_clmulepi64_si128(a, k, 0x11),
                                next, 0x96);
}

// Consumes every whole 64-byte block of [p, p+n) (n >= 256); returns the raw crc32q state.
__attribute__((target("avx512f,avx512vl,vpclmulqdq,pclmul,sse4.2"))) uint32_t
crc32c_vpclmul(const uint8_t*& p, size_t& n, uint32_t state) {
  const __m512i k2048 = _mm512_set_epi64(kF2048b, kF2048a, kF2048b, kF2048a, kF2048b, kF2048a,
                                         kF2048b, kF2048a);
  const __m512i k512 = _mm512_set_epi64(kF512b, kF512a, kF512b, kF512a, kF512b, kF512a, kF512b,
                                        kF512a);
  __m512i x0 = _mm512_loadu_si512(p);
  __m512i x1 = _mm512_loadu_si512(p + 64);
  __m512i x2 = _mm512_loadu_si512(p + 128);
  __m512i x3 = _mm512_loadu_si512(p + 192);
  x0 = _mm512_xor_si512(x0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)state)));
  p += 256;
  n -= 256;
  while (n >= 256) {
    x0 = fold512(x0, k2048, _mm512_loadu_si512(p));
    x1 = fold512(x1, k2048, _mm512_loadu_si512(p + 64));
    x2 = fold512(x2, k2048, _mm512_loadu_si512(p + 128));
    x3 = fold512(x3, k2048, _mm512_loadu_si512(p + 192));
    p += 256;
    n -= 256;
  }
  x1 = fold512(x0, k512, x1);
  x2 = fold512(x1, k512, x2);
  x3 = fold512(x2, k512, x3);
  while (n >= 64) {
    x3 = fold512(x3, k512, _mm512_loadu_si512(p));
    p += 64;
    n -= 64;
  }
  const __m128i k128 = _mm_set_epi64x((long long)kF128b, (long long)kF128a);
  __m128i r = _mm512_extracti32x4_epi32(x3, 0);
  r = fold128(r, k128, _mm512_extracti32x4_epi32(x3, 1));
  r = fold128(r, k128, _mm512_extracti32x4_epi32(x3, 2));
  r = fold128(r, k128, _mm512_extracti32x4_epi32(x3, 3));
  uint64_t c = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(r));
  c = _mm_crc32_u64(c, (uint64_t)_mm_extract_epi64(r, 1));
  return (uint32_t)c;
}

bool has_vpclmul() {
  static const bool ok = __builtin_cpu_supports("avx512f") &&
                         __builtin_cpu_supports("avx512vl") &&
                         __builtin_cpu_supports("vpclmulqdq");
  return ok;
}

}  // namespace

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = ~crc & 0xffffffffu;
  if (n >= 256 && has_vpclmul()) c = crc32c_vpclmul(p, n, (uint32_t)c);
  while (n && ((uintptr_t)p & 7)) {
    c = _mm_crc32_u8((uint32_t)c, *p++);
    --n;
  }
  p = crc3(p, n, c, kLong, long_table());
  p = crc3(p, n, c, kShort, short_table());
  while (n >= 8) {
    c = _mm_crc32_u64(c, ld64(p));
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *p++);
  return ~(uint32_t)c;
}

uint32_t crc32c_shift(uint32_t raw, uint64_t nbytes) { return poly_mulmod(raw, x8n(nbytes)); }

struct CrcShift::Impl {
  ShiftTable t;
  explicit Impl(uint64_t n) : t((size_t)n) {}
};
CrcShift::CrcShift(uint64_t nbytes) : impl_(std::make_shared<Impl>(nbytes)) {}
uint32_t CrcShift::operator()(uint32_t raw) const { return impl_->t.shift(raw); }

void crc32c_device_tables(uint32_t* out) {
  // slicing-by-4 byte tables: S0[v] = raw CRC register after byte v from state 0,
  // Sk[v] = Sk-1[v] advanced by one zero byte
  uint32_t* s0 = out;
  for (uint32_t v = 0; v < 256; ++v) {
    uint32_t c = v;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
    s0[v] = c;
  }
  for (int k = 1; k < 4; ++k)
    for (uint32_t v = 0; v < 256; ++v) {
      const uint32_t prev = out[(k - 1) * 256 + v];
      out[k * 256 + v] = (prev >> 8) ^ s0[prev & 0xff];
    }
  // per-lane shift constants: x^(8 * 64 * (63 - lane)) mod P (the bytes after lane l's piece
  // of a 4 KiB window), applied on the device by a GF(2) multiply
  for (int l = 0; l < 64; ++l) out[1024 + l] = x8n((uint64_t)64 * (63 - l));
}

uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  // standard (inverted) CRCs: the inversions of A's final state and B's initial state cancel
  return crc32c_shift(crc_a, len_b) ^ crc_b;
}

uint32_t crc32c_raw(const uint8_t* p, size_t n, uint32_t raw) {
  return ~crc32c(p, n, ~raw);
}

uint32_t patch_batch_crc(uint32_t crc, const uint8_t* old_bytes, const uint8_t* new_bytes,
                         size_t n, uint64_t bytes_after) {
  // equal-length messages: crc(A) ^ crc(A') = raw(A ^ A'), and the difference is zero outside
  // the patched window, so only that window and a shift over the tail are computed
  uint8_t d[64];
  if (n > sizeof(d)) throw ProtocolError("patch window too large");
  for (size_t i = 0; i < n; ++i) d[i] = old_bytes[i] ^ new_bytes[i];
  return crc ^ crc32c_shift(crc32c_raw(d, n, 0), bytes_after);
}

namespace {

size_t uvarint_size(uint64_t v) {
  size_t s = 1;
  while (v >= 0x80) { v >>= 7; ++s; }
  return s;
}
size_t varint_size(int64_t v) { return uvarint_size(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }

}  // namespace

size_t encode_batch(Writer& w, const RecordIn* recs, size_t n, int64_t base_offset,
                    int64_t base_timestamp) {
  if (n == 0) throw ProtocolError("empty record batch");
  const size_t start = w.size();
  int64_t max_ts = base_timestamp;
  for (size_t i = 0; i < n; ++i)
    if (recs[i].timestamp > max_ts) max_ts = recs[i].timestamp;
  w.i64(base_offset);
  const size_t len_pos = w.size();
  w.i32(0);   // batchLength (patched)
  w.i32(-1);  // partitionLeaderEpoch
  w.i8(2);    // magic
  const size_t crc_pos = w.size();
  w.u32(0);   // crc (patched)
  const size_t attr_pos = w.size();
  w.i16(0);   // attributes: no compression, CreateTime, not transactional
  w.i32((int32_t)(n - 1));
  w.i64(base_timestamp);
  w.i64(max_ts);
  w.i64(-1);  // producerId
  w.i16(-1);  // producerEpoch
  w.i32(-1);  // baseSequence
  w.i32((int32_t)n);
  for (size_t i = 0; i < n; ++i) {
    const RecordIn& r = recs[i];
    const int64_t tsd = (r.timestamp < 0 ? base_timestamp : r.timestamp) - base_timestamp;
    const int32_t klen = r.key_null ? -1 : (int32_t)r.key.size();
    const int32_t vlen = r.value_null ? -1 : (int32_t)r.value.size();
    const int32_t nh = r.headers ? (int32_t)r.headers->size() : 0;
    size_t body = 1 + varint_size(tsd) + varint_size((int64_t)i) + varint_size(klen) +
                  (klen > 0 ? (size_t)klen : 0) + varint_size(vlen) + (vlen > 0 ? (size_t)vlen : 0) +
                  varint_size(nh);
    if (r.headers) {
      for (const Header& h : *r.headers) {
        const int32_t hv = h.value_null ? -1 : (int32_t)h.value.size();
        body += varint_size((int32_t)h.key.size()) + h.key.size() + varint_size(hv) +
                (hv > 0 ? (size_t)hv : 0);
      }
    }
    w.varint((int32_t)body);
    w.i8(0);
    w.varlong(tsd);
    w.varint((int32_t)i);
    w.varint(klen);
    if (klen > 0) w.raw(r.key.data(), (size_t)klen);
    w.varint(vlen);
    if (vlen > 0) w.raw(r.value.data(), (size_t)vlen);
    w.varint(nh);
    if (r.headers) {
      for (const Header& h : *r.headers) {
        w.varint((int32_t)h.key.size());
        w.raw(h.key.data(), h.key.size());
        const int32_t hv = h.value_null ? -1 : (int32_t)h.value.size();
        w.varint(hv);
        if (hv > 0) w.raw(h.value.data(), (size_t)hv);
      }
    }
  }
  const size_t end = w.size();
  w.patch_i32(len_pos, (int32_t)(end - start - 12));
  w.patch_u32(crc_pos, crc32c(reinterpret_cast<const uint8_t*>(w.buf.data()) + attr_pos,
                              end - attr_pos));
  return end - start;
}

BatchInfo peek_batch(const uint8_t* p, size_t avail, bool check_crc) {
  if (avail < (size_t)kBatchHeaderBytes) throw ProtocolError("short record batch");
  Reader r(p, avail);
  BatchInfo b;
  b.base_offset = r.i64();
  const int32_t blen = r.i32();
  if (blen < kBatchHeaderBytes - 12) throw ProtocolError("bad batchLength");
  b.length = blen + 12;
  if ((size_t)b.length > avail) throw ProtocolError("truncated record batch");
  r.i32();  // partitionLeaderEpoch
  const int8_t magic = r.i8();
  if (magic != 2) throw ProtocolError("unsupported message format (magic != 2)");
  const uint32_t crc = r.u32();
  if (check_crc) {
    const uint32_t got = crc32c(p + kBatchAttrOffset, (size_t)b.length - kBatchAttrOffset);
    if (got != crc) throw ProtocolError("record batch CRC32C mismatch");
  }
  b.attributes = r.i16();
  b.last_offset_delta = r.i32();
  b.base_timestamp = r.i64();
  b.max_timestamp = r.i64();
  r.i64();
  r.i16();
  r.i32();
  b.records = r.i32();
  if (b.records < 0) throw ProtocolError("negative record count");
  return b;
}

size_t decode_records(const uint8_t* base, size_t off, size_t len, int64_t min_offset,
                      bool check_crc, std::vector<RecordRef>& out,
                      std::vector<BatchSpan>* spans, bool honor_poison) {
  size_t added = 0;
  size_t pos = off;
  const size_t end = off + len;
  while (end - pos >= 17) {
    Reader hr(base + pos, end - pos);
    hr.i64();
    const int32_t blen = hr.i32();
    if (blen < 0 || (size_t)blen + 12 > end - pos) break;  // partial trailing batch
    const BatchInfo b = peek_batch(base + pos, end - pos, check_crc);
    if (b.attributes & 0x7) throw ProtocolError("compressed record batches are not supported");
    const bool control = (b.attributes & 0x20) != 0;
    const bool poison = honor_poison && (b.attributes & 0x4000) != 0;  // kAttrGalePoison
    const size_t first = out.size();
    if (!control) {
      Reader r(base + pos + kBatchHeaderBytes, (size_t)b.length - kBatchHeaderBytes);
      const size_t rbase = pos + kBatchHeaderBytes;
      for (int32_t k = 0; k < b.records; ++k) {
        const int32_t rlen = r.varint();
        const size_t rstart = r.pos();
        r.i8();  // attributes
        const int64_t tsd = r.varlong();
        const int32_t od = r.varint();
        RecordRef rr;
        rr.offset = b.base_offset + od;
        // LogAppendTime batches (attribute bit 3): every record carries the broker's append time
        rr.timestamp = (b.attributes & kAttrLogAppendTime) ? b.max_timestamp
                                                          : b.base_timestamp + tsd;
        rr.key_len = r.varint();
        rr.key_off = (int64_t)(rbase + r.pos());
        if (rr.key_len > 0) r.skip((size_t)rr.key_len);
        rr.value_len = r.varint();
        rr.value_off = (int64_t)(rbase + r.pos());
        if (rr.value_len > 0) r.skip((size_t)rr.value_len);
        rr.header_count = r.varint();
        rr.headers_off = (int64_t)(rbase + r.pos());
        const size_t consumed = r.pos() - rstart;
        if (rlen < 0 || consumed > (size_t)rlen) throw ProtocolError("bad record length");
        r.skip((size_t)rlen - consumed);
        rr.headers_len = (int64_t)(rbase + r.pos()) - rr.headers_off;
        rr.poison = poison;
        if (rr.offset >= min_offset) {
          out.push_back(rr);
          ++added;
        }
      }
    }
    if (spans && out.size() > first) spans->push_back({pos, (size_t)b.length, first, out.size() - first});
    pos += (size_t)b.length;
  }
  return added;
}

std::vector<Header> decode_headers(const uint8_t* base, const RecordRef& rr) {
  std::vector<Header> hs;
  Reader r(base + rr.headers_off, (size_t)rr.headers_len);
  for (int32_t i = 0; i < rr.header_count; ++i) {
    Header h;
    const int32_t kl = r.varint();
    if (kl > 0) {
      h.key.assign(reinterpret_cast<const char*>(r.ptr()), (size_t)kl);
      r.skip((size_t)kl);
    }
    const int32_t vl = r.varint();
    if (vl < 0) {
      h.value_null = true;
    } else if (vl > 0) {
      h.value.assign(reinterpret_cast<const char*>(r.ptr()), (size_t)vl);
      r.skip((size_t)vl);
    }
    hs.push_back(std::move(h));
  }
  return hs;
}

int socket_buffer_bytes() {
  static const int v = [] {
    const char* e = getenv("GALE_SOCK_BUF");
    return e && *e ? atoi(e) : (8 << 20);
  }();
  return v;
}

}  // namespace kafka
}  // namespace gale
