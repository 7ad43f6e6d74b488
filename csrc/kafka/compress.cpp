// Kafka compression codecs and record-format normalisation (see compress.h).
#include "compress.h"

#include <dlfcn.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <deque>
#include <mutex>

#include "wire.h"

namespace gale {
namespace kafka {

namespace {

inline uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint32_t rd_le(const uint8_t* p, int nb) {
  uint32_t v = 0;
  for (int i = 0; i < nb; ++i) v |= (uint32_t)p[i] << (8 * i);
  return v;
}
inline uint32_t rd_be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
inline void put_be32(std::string& s, uint32_t v) {
  const char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  s.append(b, 4);
}
inline void put_le32(std::string& s, uint32_t v) {
  const char b[4] = {(char)v, (char)(v >> 8), (char)(v >> 16), (char)(v >> 24)};
  s.append(b, 4);
}

// Back-reference copy inside `out` (overlapping copies replicate the period, as LZ77 wants).
inline void lz_copy(std::string& out, size_t off, size_t len) {
  const size_t pos = out.size();
  out.resize(pos + len);
  char* d = &out[0];
  const size_t from = pos - off;
  if (off >= len) {
    memcpy(d + pos, d + from, len);
  } else {
    for (size_t k = 0; k < len; ++k) d[pos + k] = d[from + k];
  }
}

// ---- zlib (gzip) -------------------------------------------------------------------------------

bool gzip_decompress(const uint8_t* in, size_t n, std::string& out, size_t limit,
                     std::string* err) {
  z_stream s;
  memset(&s, 0, sizeof(s));
  if (inflateInit2(&s, 15 + 32) != Z_OK) {  // +32: gzip or zlib header, detected
    if (err) *err = "inflateInit2 failed";
    return false;
  }
  s.next_in = const_cast<Bytef*>(in);
  s.avail_in = (uInt)n;
  char buf[65536];
  int rc = Z_OK;
  for (;;) {
    s.next_out = reinterpret_cast<Bytef*>(buf);
    s.avail_out = sizeof(buf);
    rc = inflate(&s, Z_NO_FLUSH);
    const size_t got = sizeof(buf) - s.avail_out;
    if (out.size() + got > limit) {
      rc = Z_BUF_ERROR;
      if (err) *err = "gzip: decompressed size over the limit";
      break;
    }
    out.append(buf, got);
    if (rc == Z_STREAM_END) {
      if (s.avail_in == 0) break;
      inflateReset(&s);  // concatenated gzip members
      continue;
    }
    if (rc != Z_OK) {
      if (err) *err = std::string("gzip: ") + (s.msg ? s.msg : "corrupt stream");
      break;
    }
    if (s.avail_in == 0 && got == 0) {
      rc = Z_DATA_ERROR;
      if (err) *err = "gzip: truncated stream";
      break;
    }
  }
  inflateEnd(&s);
  return rc == Z_STREAM_END;
}

std::string gzip_compress(const uint8_t* in, size_t n) {
  z_stream s;
  memset(&s, 0, sizeof(s));
  if (deflateInit2(&s, 6, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK)
    throw std::runtime_error("deflateInit2 failed");
  std::string out;
  out.resize(deflateBound(&s, (uLong)n) + 32);
  s.next_in = const_cast<Bytef*>(in);
  s.avail_in = (uInt)n;
  s.next_out = reinterpret_cast<Bytef*>(&out[0]);
  s.avail_out = (uInt)out.size();
  const int rc = deflate(&s, Z_FINISH);
  out.resize(out.size() - s.avail_out);
  deflateEnd(&s);
  if (rc != Z_STREAM_END) throw std::runtime_error("gzip: deflate failed");
  return out;
}

// ---- zstd through the system library (no headers in the image: the stable ABI, declared) -----

struct ZstdIn {
  const void* src;
  size_t size, pos;
};
struct ZstdOut {
  void* dst;
  size_t size, pos;
};
struct Zstd {
  void* h = nullptr;
  void* (*createDStream)() = nullptr;
  size_t (*initDStream)(void*) = nullptr;
  size_t (*decompressStream)(void*, ZstdOut*, ZstdIn*) = nullptr;
  size_t (*freeDStream)(void*) = nullptr;
  unsigned (*isError)(size_t) = nullptr;
  const char* (*errorName)(size_t) = nullptr;
  size_t (*compressBound)(size_t) = nullptr;
  size_t (*compress)(void*, size_t, const void*, size_t, int) = nullptr;
  bool ok = false;
};
const Zstd& zstd() {
  static Zstd z = [] {
    Zstd z;
    z.h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!z.h) return z;
    auto sym = [&](const char* n) { return dlsym(z.h, n); };
    z.createDStream = reinterpret_cast<void* (*)()>(sym("ZSTD_createDStream"));
    z.initDStream = reinterpret_cast<size_t (*)(void*)>(sym("ZSTD_initDStream"));
    z.decompressStream =
        reinterpret_cast<size_t (*)(void*, ZstdOut*, ZstdIn*)>(sym("ZSTD_decompressStream"));
    z.freeDStream = reinterpret_cast<size_t (*)(void*)>(sym("ZSTD_freeDStream"));
    z.isError = reinterpret_cast<unsigned (*)(size_t)>(sym("ZSTD_isError"));
    z.errorName = reinterpret_cast<const char* (*)(size_t)>(sym("ZSTD_getErrorName"));
    z.compressBound = reinterpret_cast<size_t (*)(size_t)>(sym("ZSTD_compressBound"));
    z.compress = reinterpret_cast<size_t (*)(void*, size_t, const void*, size_t, int)>(
        sym("ZSTD_compress"));
    z.ok = z.createDStream && z.initDStream && z.decompressStream && z.freeDStream &&
           z.isError && z.errorName && z.compressBound && z.compress;
    return z;
  }();
  return z;
}

bool zstd_decompress(const uint8_t* in, size_t n, std::string& out, size_t limit,
                     std::string* err) {
  const Zstd& z = zstd();
  if (!z.ok) {
    if (err) *err = "zstd: libzstd.so.1 not available";
    return false;
  }
  void* ds = z.createDStream();
  if (!ds) {
    if (err) *err = "zstd: createDStream failed";
    return false;
  }
  z.initDStream(ds);
  ZstdIn zi{in, n, 0};
  char buf[65536];
  bool ok = true;
  size_t last = 1;
  while (zi.pos < zi.size || last != 0) {
    ZstdOut zo{buf, sizeof(buf), 0};
    last = z.decompressStream(ds, &zo, &zi);
    if (z.isError(last)) {
      if (err) *err = std::string("zstd: ") + z.errorName(last);
      ok = false;
      break;
    }
    if (out.size() + zo.pos > limit) {
      if (err) *err = "zstd: decompressed size over the limit";
      ok = false;
      break;
    }
    out.append(buf, zo.pos);
    if (zi.pos >= zi.size && zo.pos == 0 && last != 0) {
      if (err) *err = "zstd: truncated frame";
      ok = false;
      break;
    }
  }
  z.freeDStream(ds);
  return ok;
}

// ---- snappy ------------------------------------------------------------------------------------

const uint8_t kXerialMagic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};

void snappy_literal(std::string& out, const uint8_t* p, size_t len) {
  while (len > 0) {
    const size_t l = std::min<size_t>(len, (size_t)1 << 24);
    const size_t m = l - 1;
    if (m < 60) {
      out.push_back((char)(m << 2));
    } else {
      const int nb = m < 256 ? 1 : m < 65536 ? 2 : 3;
      out.push_back((char)((59 + nb) << 2));
      for (int i = 0; i < nb; ++i) out.push_back((char)(m >> (8 * i)));
    }
    out.append(reinterpret_cast<const char*>(p), l);
    p += l;
    len -= l;
  }
}

void snappy_copy(std::string& out, size_t off, size_t len) {
  while (len > 0) {
    // copy-2 carries 1..64 bytes; never leave a 1-3 byte remainder that copy-1 could not hold
    size_t l = std::min<size_t>(len, 64);
    if (len > 64 && len - 64 < 4) l = len - 4;
    if (l >= 4 && l <= 11 && off < 2048) {  // copy-1: 4..11 bytes, 11-bit offset
      out.push_back((char)(1 | ((l - 4) << 2) | ((off >> 8) << 5)));
      out.push_back((char)(off & 0xff));
    } else {
      out.push_back((char)(2 | ((l - 1) << 2)));
      out.push_back((char)(off & 0xff));
      out.push_back((char)(off >> 8));
    }
    len -= l;
  }
}

// ---- lz4 ---------------------------------------------------------------------------------------

constexpr uint32_t kLz4Magic = 0x184D2204u;

bool lz4_block_decompress(const uint8_t* in, size_t n, std::string& out, size_t limit) {
  size_t ip = 0;
  for (;;) {
    if (ip >= n) return false;
    const uint8_t token = in[ip++];
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= n) return false;
        b = in[ip++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - ip || out.size() + lit > limit) return false;
    out.append(reinterpret_cast<const char*>(in + ip), lit);
    ip += lit;
    if (ip == n) return true;  // the last sequence has literals only
    if (n - ip < 2) return false;
    const size_t off = (size_t)in[ip] | (size_t)in[ip + 1] << 8;
    ip += 2;
    if (off == 0 || off > out.size()) return false;
    size_t ml = token & 15;
    if (ml == 15) {
      uint8_t b;
      do {
        if (ip >= n) return false;
        b = in[ip++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (out.size() + ml > limit) return false;
    lz_copy(out, off, ml);
  }
}

void lz4_len_ext(std::string& out, size_t v) {  // v >= 15 already subtracted by the caller
  while (v >= 255) {
    out.push_back((char)255);
    v -= 255;
  }
  out.push_back((char)v);
}

// Greedy LZ4 block compressor (4-byte hash matches within 64 KiB). Block-format rules: the last
// 5 bytes are literals and no match starts within the last 12 bytes.
std::string lz4_block_compress(const uint8_t* in, size_t n) {
  std::string out;
  out.reserve(n + n / 255 + 16);
  constexpr int kBits = 14;
  std::vector<int32_t> table((size_t)1 << kBits, -1);
  size_t anchor = 0, i = 0;
  auto emit = [&](size_t lit_end, size_t off, size_t ml) {
    const size_t lit = lit_end - anchor;
    const size_t mcode = ml - 4;
    out.push_back((char)((std::min<size_t>(lit, 15) << 4) | std::min<size_t>(mcode, 15)));
    if (lit >= 15) lz4_len_ext(out, lit - 15);
    out.append(reinterpret_cast<const char*>(in + anchor), lit);
    out.push_back((char)(off & 0xff));
    out.push_back((char)(off >> 8));
    if (mcode >= 15) lz4_len_ext(out, mcode - 15);
  };
  if (n > 12) {
    const size_t mflimit = n - 12, match_end = n - 5;
    while (i < mflimit) {
      const uint32_t v = ld32(in + i);
      const uint32_t h = (v * 2654435761u) >> (32 - kBits);
      const int32_t cand = table[h];
      table[h] = (int32_t)i;
      if (cand >= 0 && i - (size_t)cand <= 65535 && ld32(in + cand) == v) {
        size_t ml = 4;
        while (i + ml < match_end && in[cand + ml] == in[i + ml]) ++ml;
        emit(i, i - (size_t)cand, ml);
        i += ml;
        anchor = i;
      } else {
        ++i;
      }
    }
  }
  const size_t lit = n - anchor;
  out.push_back((char)(std::min<size_t>(lit, 15) << 4));
  if (lit >= 15) lz4_len_ext(out, lit - 15);
  out.append(reinterpret_cast<const char*>(in + anchor), lit);
  return out;
}

}  // namespace

uint32_t xxh32(const uint8_t* p, size_t n, uint32_t seed) {
  constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                     P5 = 374761393u;
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  const uint8_t* end = p + n;
  uint32_t h;
  if (n >= 16) {
    uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* limit = end - 16;
    do {
      v1 = rotl(v1 + ld32(p) * P2, 13) * P1;
      v2 = rotl(v2 + ld32(p + 4) * P2, 13) * P1;
      v3 = rotl(v3 + ld32(p + 8) * P2, 13) * P1;
      v4 = rotl(v4 + ld32(p + 12) * P2, 13) * P1;
      p += 16;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
  } else {
    h = seed + P5;
  }
  h += (uint32_t)n;
  while (p + 4 <= end) {
    h = rotl(h + ld32(p) * P3, 17) * P4;
    p += 4;
  }
  while (p < end) {
    h = rotl(h + (*p) * P5, 11) * P1;
    ++p;
  }
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

uint32_t crc32_ieee(const uint8_t* p, size_t n) {
  return (uint32_t)crc32(crc32(0L, Z_NULL, 0), p, (uInt)n);
}

bool snappy_decompress_raw(const uint8_t* in, size_t n, std::string& out, size_t limit) {
  size_t ip = 0;
  uint64_t ulen = 0;
  for (int s = 0;; s += 7) {
    if (ip >= n || s > 28) return false;
    const uint8_t b = in[ip++];
    ulen |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) break;
  }
  const size_t start = out.size();
  if (start + ulen > limit) return false;
  out.reserve(start + ulen);
  while (ip < n) {
    const uint8_t tag = in[ip++];
    size_t len, off;
    switch (tag & 3) {
      case 0: {
        len = tag >> 2;
        if (len >= 60) {
          const int nb = (int)len - 59;
          if (n - ip < (size_t)nb) return false;
          len = rd_le(in + ip, nb);
          ip += (size_t)nb;
        }
        len += 1;
        if (len > n - ip || out.size() - start + len > ulen) return false;
        out.append(reinterpret_cast<const char*>(in + ip), len);
        ip += len;
        continue;
      }
      case 1:
        if (ip >= n) return false;
        len = 4 + ((tag >> 2) & 7);
        off = ((size_t)(tag >> 5) << 8) | in[ip++];
        break;
      case 2:
        if (n - ip < 2) return false;
        len = 1 + (tag >> 2);
        off = rd_le(in + ip, 2);
        ip += 2;
        break;
      default:
        if (n - ip < 4) return false;
        len = 1 + (tag >> 2);
        off = rd_le(in + ip, 4);
        ip += 4;
        break;
    }
    if (off == 0 || off > out.size() - start || out.size() - start + len > ulen) return false;
    lz_copy(out, off, len);
  }
  return out.size() - start == ulen;
}

std::string snappy_compress_raw(const uint8_t* in, size_t n) {
  std::string out;
  out.reserve(n + n / 6 + 16);
  for (uint64_t v = n;; v >>= 7) {  // preamble: uncompressed length
    if (v < 0x80) {
      out.push_back((char)v);
      break;
    }
    out.push_back((char)(v | 0x80));
  }
  constexpr int kBits = 14;
  std::vector<int32_t> table((size_t)1 << kBits, -1);
  size_t lit = 0, i = 0;
  while (i + 4 <= n) {
    const uint32_t v = ld32(in + i);
    const uint32_t h = (v * 0x1e35a7bdu) >> (32 - kBits);
    const int32_t cand = table[h];
    table[h] = (int32_t)i;
    if (cand >= 0 && i - (size_t)cand <= 65535 && ld32(in + cand) == v) {
      size_t len = 4;
      while (i + len < n && in[cand + len] == in[i + len]) ++len;
      snappy_literal(out, in + lit, i - lit);
      snappy_copy(out, i - (size_t)cand, len);
      i += len;
      lit = i;
    } else {
      ++i;
    }
  }
  snappy_literal(out, in + lit, n - lit);
  return out;
}

bool lz4_decompress_frame(const uint8_t* in, size_t n, std::string& out, size_t limit) {
  size_t pos = 0;
  bool frames = false;
  while (pos < n) {
    if (n - pos < 4) return false;
    const uint32_t magic = ld32(in + pos);
    if ((magic & 0xfffffff0u) == 0x184D2A50u) {  // skippable frame
      if (n - pos < 8) return false;
      const size_t sz = ld32(in + pos + 4);
      if (sz > n - pos - 8) return false;
      pos += 8 + sz;
      continue;
    }
    if (magic != kLz4Magic || n - pos < 7) return false;
    const uint8_t flg = in[pos + 4];
    if ((flg >> 6) != 1) return false;  // frame version 01
    const bool block_ck = flg & 0x10, content_size = flg & 0x08, content_ck = flg & 0x04,
               dict = flg & 0x01;
    if (dict) return false;  // dictionaries are never used by Kafka
    // (the header checksum is not verified: Kafka's magic-0 LZ4 framing computed it over the
    // wrong bytes, KAFKA-3160, and the batch CRC already covers the frame)
    pos += 6 + (content_size ? 8 : 0) + 1;
    if (pos > n) return false;
    for (;;) {
      if (n - pos < 4) return false;
      const uint32_t bs = ld32(in + pos);
      pos += 4;
      if (bs == 0) break;  // EndMark
      const size_t sz = bs & 0x7fffffffu;
      if (sz > n - pos) return false;
      if (bs & 0x80000000u) {
        if (out.size() + sz > limit) return false;
        out.append(reinterpret_cast<const char*>(in + pos), sz);
      } else if (!lz4_block_decompress(in + pos, sz, out, limit)) {
        return false;
      }
      pos += sz + (block_ck ? 4 : 0);
      if (pos > n) return false;
    }
    if (content_ck) pos += 4;
    if (pos > n) return false;
    frames = true;
  }
  return frames;
}

std::string lz4_compress_frame(const uint8_t* in, size_t n) {
  std::string out;
  put_le32(out, kLz4Magic);
  const uint8_t desc[2] = {0x60, 0x40};  // version 01, independent blocks; 64 KiB max block
  out.append(reinterpret_cast<const char*>(desc), 2);
  out.push_back((char)((xxh32(desc, 2, 0) >> 8) & 0xff));
  for (size_t o = 0; o < n; o += 65536) {
    const size_t l = std::min<size_t>(65536, n - o);
    const std::string b = lz4_block_compress(in + o, l);
    if (b.size() < l) {
      put_le32(out, (uint32_t)b.size());
      out += b;
    } else {
      put_le32(out, (uint32_t)l | 0x80000000u);
      out.append(reinterpret_cast<const char*>(in + o), l);
    }
  }
  put_le32(out, 0);
  return out;
}

const char* codec_name(int c) {
  switch (c) {
    case CODEC_NONE: return "none";
    case CODEC_GZIP: return "gzip";
    case CODEC_SNAPPY: return "snappy";
    case CODEC_LZ4: return "lz4";
    case CODEC_ZSTD: return "zstd";
    default: return "unknown";
  }
}

int codec_from_name(const std::string& s) {
  for (int c = 0; c <= CODEC_ZSTD; ++c)
    if (s == codec_name(c)) return c;
  throw std::invalid_argument("compression must be none|gzip|snappy|lz4|zstd, got " + s);
}

bool codec_available(int c) {
  if (c == CODEC_ZSTD) return zstd().ok;
  return c >= CODEC_NONE && c <= CODEC_LZ4;
}

bool decompress(int codec, const uint8_t* in, size_t n, std::string& out, size_t limit,
                std::string* err) {
  switch (codec) {
    case CODEC_NONE:
      if (out.size() + n > limit) return false;
      out.append(reinterpret_cast<const char*>(in), n);
      return true;
    case CODEC_GZIP:
      return gzip_decompress(in, n, out, limit, err);
    case CODEC_SNAPPY: {
      bool ok = true;
      if (n >= 16 && memcmp(in, kXerialMagic, 8) == 0) {  // xerial framing (Kafka's Java client)
        size_t pos = 16;
        while (ok && pos < n) {
          if (n - pos < 4) {
            ok = false;
            break;
          }
          const size_t bl = rd_be32(in + pos);
          pos += 4;
          if (bl > n - pos) {
            ok = false;
            break;
          }
          ok = snappy_decompress_raw(in + pos, bl, out, limit);
          pos += bl;
        }
      } else {
        ok = snappy_decompress_raw(in, n, out, limit);
      }
      if (!ok && err) *err = "snappy: corrupt stream";
      return ok;
    }
    case CODEC_LZ4: {
      const bool ok = lz4_decompress_frame(in, n, out, limit);
      if (!ok && err) *err = "lz4: corrupt frame";
      return ok;
    }
    case CODEC_ZSTD:
      return zstd_decompress(in, n, out, limit, err);
    default:
      if (err) *err = "unknown compression codec " + std::to_string(codec);
      return false;
  }
}

std::string compress(int codec, const uint8_t* in, size_t n) {
  switch (codec) {
    case CODEC_NONE:
      return std::string(reinterpret_cast<const char*>(in), n);
    case CODEC_GZIP:
      return gzip_compress(in, n);
    case CODEC_SNAPPY: {  // xerial framing, 32 KiB blocks (Kafka's SnappyOutputStream)
      std::string out(reinterpret_cast<const char*>(kXerialMagic), 8);
      put_be32(out, 1);
      put_be32(out, 1);
      for (size_t o = 0; o < n || o == 0; o += 32768) {
        const std::string b = snappy_compress_raw(in + o, std::min<size_t>(32768, n - o));
        put_be32(out, (uint32_t)b.size());
        out += b;
        if (n == 0) break;
      }
      return out;
    }
    case CODEC_LZ4:
      return lz4_compress_frame(in, n);
    case CODEC_ZSTD: {
      const Zstd& z = zstd();
      if (!z.ok) throw std::runtime_error("zstd: libzstd.so.1 not available");
      std::string out(z.compressBound(n), '\0');
      const size_t r = z.compress(&out[0], out.size(), in, n, 3);
      if (z.isError(r)) throw std::runtime_error(std::string("zstd: ") + z.errorName(r));
      out.resize(r);
      return out;
    }
    default:
      throw std::invalid_argument("unknown compression codec " + std::to_string(codec));
  }
}

// ---- record-format conversion ---------------------------------------------------------------

namespace {

struct Rec {
  int64_t offset = 0, timestamp = -1;
  const uint8_t* key = nullptr;
  int32_t key_len = -1;
  const uint8_t* value = nullptr;
  int32_t value_len = -1;
};

size_t uvarint_size(uint64_t v) {
  size_t s = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++s;
  }
  return s;
}
size_t zz_size(int64_t v) { return uvarint_size(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }

// Append a plain v2 batch of `recs` (explicit offsets; headers none) with `attributes`.
void append_v2(std::string& out, const std::vector<Rec>& recs, int16_t attributes) {
  if (recs.empty()) return;
  Writer w;
  const int64_t base = recs.front().offset;
  int64_t base_ts = -1, max_ts = -1;
  for (const Rec& r : recs)
    if (r.timestamp >= 0) {
      if (base_ts < 0) base_ts = r.timestamp;
      max_ts = std::max(max_ts, r.timestamp);
    }
  w.i64(base);
  w.i32(0);   // batchLength (patched)
  w.i32(-1);  // partitionLeaderEpoch
  w.i8(2);
  w.u32(0);   // crc (patched)
  w.i16(attributes);
  w.i32((int32_t)(recs.back().offset - base));
  w.i64(base_ts);
  w.i64(max_ts);
  w.i64(-1);
  w.i16(-1);
  w.i32(-1);
  w.i32((int32_t)recs.size());
  for (const Rec& r : recs) {
    const int64_t tsd = r.timestamp >= 0 && base_ts >= 0 ? r.timestamp - base_ts : 0;
    const int64_t od = r.offset - base;
    const size_t body = 1 + zz_size(tsd) + zz_size(od) + zz_size(r.key_len) +
                        (r.key_len > 0 ? (size_t)r.key_len : 0) + zz_size(r.value_len) +
                        (r.value_len > 0 ? (size_t)r.value_len : 0) + zz_size(0);
    w.varint((int32_t)body);
    w.i8(0);
    w.varlong(tsd);
    w.varint((int32_t)od);
    w.varint(r.key_len);
    if (r.key_len > 0) w.raw(r.key, (size_t)r.key_len);
    w.varint(r.value_len);
    if (r.value_len > 0) w.raw(r.value, (size_t)r.value_len);
    w.varint(0);
  }
  w.patch_i32(8, (int32_t)(w.size() - 12));
  w.patch_u32(kBatchCrcOffset,
              crc32c(reinterpret_cast<const uint8_t*>(w.buf.data()) + kBatchAttrOffset,
                     w.size() - kBatchAttrOffset));
  out += w.buf;
}

// Poison batch: null records at [first, last] (one per offset when count matches the span, else
// one at `last`), never below min_offset.
void append_poison(std::string& out, int64_t first, int64_t last, int32_t count,
                   int64_t min_offset, NormalizeStats& st, const std::string& why) {
  std::vector<Rec> recs;
  if (last < min_offset) last = min_offset;
  if (first < min_offset) first = min_offset;
  if (count > 0 && count == last - first + 1 && count <= 1 << 20) {
    for (int64_t o = first; o <= last; ++o) {
      Rec r;
      r.offset = o;
      recs.push_back(r);
    }
  } else {
    Rec r;
    r.offset = last;
    recs.push_back(r);
  }
  ++st.poison_batches;
  st.poison_records += (int64_t)recs.size();
  st.last_error = why;
  append_v2(out, recs, kAttrGalePoison);
}

// Parse v2 records out of [p, p+n) (count records) into `recs` (pointers into p).
void parse_v2_records(const uint8_t* p, size_t n, int32_t count, int64_t base_offset,
                      int64_t base_ts, int64_t max_ts, bool log_append, std::vector<Rec>& recs) {
  Reader r(p, n);
  for (int32_t k = 0; k < count; ++k) {
    const int32_t rlen = r.varint();
    const size_t rs = r.pos();
    r.i8();
    const int64_t tsd = r.varlong();
    const int32_t od = r.varint();
    Rec x;
    x.offset = base_offset + od;
    x.timestamp = log_append ? max_ts : base_ts + tsd;
    x.key_len = r.varint();
    x.key = r.ptr();
    if (x.key_len > 0) r.skip((size_t)x.key_len);
    x.value_len = r.varint();
    x.value = r.ptr();
    if (x.value_len > 0) r.skip((size_t)x.value_len);
    const int32_t nh = r.varint();
    for (int32_t h = 0; h < nh; ++h) {
      const int32_t kl = r.varint();
      if (kl > 0) r.skip((size_t)kl);
      const int32_t vl = r.varint();
      if (vl > 0) r.skip((size_t)vl);
    }
    const size_t used = r.pos() - rs;
    if (rlen < 0 || used > (size_t)rlen) throw ProtocolError("bad record length");
    r.skip((size_t)rlen - used);
    recs.push_back(x);
  }
}

// One legacy message at p (offset, size, crc, magic, attrs, [ts], key, value): parsed into
// Rec (value = the wrapper's compressed payload when attrs & 7). Returns the entry size.
struct LegacyMsg {
  Rec rec;
  int magic = 0, codec = 0;
  bool log_append = false;
};
size_t parse_legacy(const uint8_t* p, size_t avail, bool check_crc, LegacyMsg& m) {
  Reader r(p, avail);
  m.rec.offset = r.i64();
  const int32_t size = r.i32();
  if (size < 14 || (size_t)size > avail - 12) throw ProtocolError("bad message size");
  const uint32_t crc = r.u32();
  if (check_crc && crc32_ieee(p + 16, (size_t)size - 4) != crc)
    throw ProtocolError("message CRC32 mismatch");
  m.magic = r.i8();
  if (m.magic != 0 && m.magic != 1) throw ProtocolError("bad legacy magic");
  const int8_t attrs = r.i8();
  m.codec = attrs & 7;
  m.log_append = (attrs & 8) != 0;
  m.rec.timestamp = m.magic == 1 ? r.i64() : -1;
  const auto k = r.bytes_ref();
  m.rec.key = p + k.first;
  m.rec.key_len = k.second;
  const auto v = r.bytes_ref();
  m.rec.value = p + v.first;
  m.rec.value_len = v.second;
  if (r.pos() != (size_t)size + 12) throw ProtocolError("bad message layout");
  return (size_t)size + 12;
}

// A legacy message (plain, or a compressed wrapper) -> its records (pointers into `p` or into
// `hold`, which keeps decompressed payloads alive).
void legacy_records(const uint8_t* p, size_t avail, bool check_crc, size_t limit,
                    std::deque<std::string>& hold, std::vector<Rec>& recs, size_t* used) {
  LegacyMsg m;
  *used = parse_legacy(p, avail, check_crc, m);
  if (m.codec == 0) {
    recs.push_back(m.rec);
    return;
  }
  if (m.rec.value_len < 0) throw ProtocolError("compressed wrapper without a value");
  std::string inner;
  std::string err;
  if (!decompress(m.codec, m.rec.value, (size_t)m.rec.value_len, inner, limit, &err))
    throw ProtocolError(err.empty() ? "corrupt compressed message" : err);
  hold.push_back(std::move(inner));
  const std::string& in = hold.back();
  const uint8_t* q = reinterpret_cast<const uint8_t*>(in.data());
  std::vector<Rec> inner_recs;
  for (size_t pos = 0; pos < in.size();) {
    LegacyMsg im;
    pos += parse_legacy(q + pos, in.size() - pos, check_crc, im);
    if (im.codec != 0) throw ProtocolError("nested compression");
    inner_recs.push_back(im.rec);
  }
  if (inner_recs.empty()) return;
  // magic 1: inner offsets are relative, the wrapper carries the last one's absolute offset;
  // magic 0: the broker wrote absolute inner offsets
  if (m.magic == 1) {
    const int64_t delta = m.rec.offset - inner_recs.back().offset;
    for (Rec& r : inner_recs) {
      r.offset += delta;
      if (m.log_append) r.timestamp = m.rec.timestamp;
    }
  }
  recs.insert(recs.end(), inner_recs.begin(), inner_recs.end());
}

}  // namespace

std::string normalize_records(const uint8_t* p, size_t len, int64_t min_offset, bool check_crc,
                              size_t limit, NormalizeStats& st) {
  std::string out;
  size_t pos = 0;
  std::vector<Rec> legacy_run;           // consecutive plain legacy messages -> one v2 batch
  std::deque<std::string> hold;  // (deque: elements never move, records point into them)
  // `limit` bounds the decompressed bytes of the whole call, not just of each batch: a
  // partition fetch of highly compressible batches must not grow the consumer by gigabytes.
  // Once it is spent, conversion stops and the next fetch resumes at the first batch not
  // converted; a batch that fails with budget already spent is retried there with the whole
  // budget before it can become poison.
  size_t spent = 0;
  // `out` already holds a record at or past min_offset: only then may the budget stop the
  // conversion, since the consumer advances its position from decoded records alone - a stop
  // before any of them (e.g. a compacted batch whose surviving records all lie below min_offset
  // came first) would refetch the same prefix forever. Until then a batch gets the
  // whole budget, and one that still fails becomes poison.
  bool served = false;
  auto any_at_or_past = [&](const std::vector<Rec>& v) {
    for (const Rec& r : v)
      if (r.offset >= min_offset) return true;
    return false;
  };
  auto room = [&]() -> size_t { return served ? (limit > spent ? limit - spent : 0) : limit; };
  // offset after the previous entry of this response (a failed legacy wrapper's inner records
  // are the offsets from here to the wrapper's own, its last inner record's)
  int64_t prev_end = min_offset;
  auto flush_legacy = [&] {
    std::vector<Rec> keep;
    for (const Rec& r : legacy_run)
      if (r.offset >= min_offset) keep.push_back(r);
    served |= !keep.empty();
    append_v2(out, keep, 0);
    legacy_run.clear();
    hold.clear();
  };
  while (len - pos >= 17) {
    Reader hr(p + pos, len - pos);
    const int64_t base = hr.i64();
    const int32_t size = hr.i32();
    if (size < 0 || (size_t)size > len - pos - 12) break;  // partial trailing entry
    const size_t entry = (size_t)size + 12;
    const int magic = (int8_t)p[pos + 16];
    if (magic == 2) {
      if (!legacy_run.empty()) flush_legacy();
      BatchInfo bi;
      bool have_hdr = false;
      try {
        bi = peek_batch(p + pos, len - pos, false);
        have_hdr = true;
        const bool compressed = (bi.attributes & 7) != 0;
        if (compressed || check_crc) {
          Reader cr(p + pos + kBatchCrcOffset, 4);
          if (crc32c(p + pos + kBatchAttrOffset, (size_t)bi.length - kBatchAttrOffset) != cr.u32())
            throw ProtocolError("record batch CRC32C mismatch");
        }
        if (base + bi.last_offset_delta < min_offset) {
          pos += entry;
          continue;
        }
        const bool control = (bi.attributes & 0x20) != 0;
        // (budget spent: the next fetch resumes here)
        if (compressed && !control && spent >= limit && served) break;
        if (!compressed || control) {
          // verify the records parse, then copy the batch through verbatim
          std::vector<Rec> probe;
          if (!control)
            parse_v2_records(p + pos + kBatchHeaderBytes, (size_t)bi.length - kBatchHeaderBytes,
                             bi.records, base, bi.base_timestamp, bi.max_timestamp,
                             (bi.attributes & kAttrLogAppendTime) != 0, probe);
          out.append(reinterpret_cast<const char*>(p + pos), (size_t)bi.length);
          served |= any_at_or_past(probe);
        } else {
          std::string plain;
          std::string err;
          if (!decompress(bi.attributes & 7, p + pos + kBatchHeaderBytes,
                          (size_t)bi.length - kBatchHeaderBytes, plain, room(), &err)) {
            // (maybe only the remaining budget: retried next fetch with all of it)
            if (spent > 0 && served) break;
            throw ProtocolError(err.empty() ? "corrupt compressed batch" : err);
          }
          spent += plain.size();
          std::vector<Rec> probe;
          parse_v2_records(reinterpret_cast<const uint8_t*>(plain.data()), plain.size(),
                           bi.records, base, bi.base_timestamp, bi.max_timestamp,
                           (bi.attributes & kAttrLogAppendTime) != 0, probe);
          served |= any_at_or_past(probe);
          // header verbatim (attributes without the codec), decompressed records, new length/CRC
          std::string b(reinterpret_cast<const char*>(p + pos), (size_t)kBatchHeaderBytes);
          b += plain;
          const int32_t blen = (int32_t)(b.size() - 12);
          const int16_t attrs = (int16_t)(bi.attributes & ~7);
          Writer::put_be(&b[kBatchLengthOffset], &blen, 4);
          Writer::put_be(&b[kBatchAttrOffset], &attrs, 2);
          const uint32_t crc = crc32c(reinterpret_cast<const uint8_t*>(b.data()) + kBatchAttrOffset,
                                      b.size() - kBatchAttrOffset);
          Writer::put_be(&b[kBatchCrcOffset], &crc, 4);
          out += b;
          ++st.converted_batches;
        }
      } catch (const ProtocolError& e) {
        if (have_hdr)
          append_poison(out, base, base + bi.last_offset_delta, bi.records, min_offset, st,
                        e.what());
        else
          append_poison(out, base, base, 1, min_offset, st, e.what());
        served |= base + (have_hdr ? bi.last_offset_delta : 0) >= min_offset;
      }
      prev_end = base + (have_hdr ? bi.last_offset_delta : 0) + 1;
    } else if (magic == 0 || magic == 1) {
      const int attrs = (int8_t)p[pos + 17];
      if (base < min_offset) {
        // a legacy entry's offset is its last (inner) record's: all of it lies below the
        // position, so it is skipped before any decompression
        if (!legacy_run.empty()) flush_legacy();
        prev_end = base + 1;
        pos += entry;
        continue;
      }
      if ((attrs & 7) != 0 && spent >= limit && served) break;  // (budget spent: next fetch)
      const size_t held = hold.size();
      try {
        std::vector<Rec> recs;
        size_t used = 0;
        legacy_records(p + pos, len - pos, true, room(), hold, recs, &used);
        for (size_t h = held; h < hold.size(); ++h) spent += hold[h].size();
        legacy_run.insert(legacy_run.end(), recs.begin(), recs.end());
        served |= any_at_or_past(recs);
        ++st.converted_batches;
      } catch (const ProtocolError& e) {
        // (maybe only the remaining budget)
        if (spent > 0 && (attrs & 7) != 0 && served) break;
        if (!legacy_run.empty()) flush_legacy();
        // the wrapper's offset is its LAST inner record's; the inner count is unreadable, so
        // every offset from the previous entry's end up to it becomes one poison record (for
        // a compacted log some of those offsets may not exist: poison_unknown_span counts the
        // records poisoned on that estimate)
        const int64_t first = std::max(prev_end, min_offset);
        if ((attrs & 7) != 0 && first < base) {
          const int64_t n = std::min<int64_t>(base - first + 1, 1 << 20);
          append_poison(out, base - n + 1, base, (int32_t)n, min_offset, st, e.what());
          st.poison_unknown_span += n;
        } else {
          append_poison(out, base, base, 1, min_offset, st, e.what());
        }
        served = true;  // (base >= min_offset here)
      }
      prev_end = base + 1;
    } else {
      // unreadable format: its offsets end where the next entry begins (when the response holds
      // one); otherwise one poison record at the position, which then advances by one per fetch
      if (!legacy_run.empty()) flush_legacy();
      int64_t next_base = INT64_MAX;
      if (len - pos - entry >= 8) next_base = Reader(p + pos + entry, 8).i64();
      if (next_base <= min_offset) {
        pos += entry;
        continue;
      }
      const int64_t first = std::max(base, min_offset);
      const int64_t last = next_base != INT64_MAX && next_base > first ? next_base - 1 : first;
      append_poison(out, first, last, (int32_t)std::min<int64_t>(last - first + 1, 1 << 20),
                    min_offset, st,
                    "unsupported message format (magic " + std::to_string(magic) + ")");
      served = true;
      prev_end = last + 1;
    }
    pos += entry;
  }
  if (!legacy_run.empty()) flush_legacy();
  return out;
}

std::string compress_batch(const std::string& b, int codec) {
  if (codec == CODEC_NONE) return b;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(b.data());
  const BatchInfo bi = peek_batch(p, b.size(), false);
  if (bi.attributes & 7) throw ProtocolError("batch is already compressed");
  std::string out(b.data(), (size_t)kBatchHeaderBytes);
  out += compress(codec, p + kBatchHeaderBytes, (size_t)bi.length - kBatchHeaderBytes);
  const int32_t blen = (int32_t)(out.size() - 12);
  const int16_t attrs = (int16_t)((bi.attributes & ~7) | codec);
  Writer::put_be(&out[kBatchLengthOffset], &blen, 4);
  Writer::put_be(&out[kBatchAttrOffset], &attrs, 2);
  const uint32_t crc = crc32c(reinterpret_cast<const uint8_t*>(out.data()) + kBatchAttrOffset,
                              out.size() - kBatchAttrOffset);
  Writer::put_be(&out[kBatchCrcOffset], &crc, 4);
  return out;
}

namespace {

void legacy_message(Writer& w, int magic, int attrs, int64_t offset, int64_t ts,
                    const std::string* key, const std::string* value) {
  w.i64(offset);
  const size_t size_pos = w.size();
  w.i32(0);
  const size_t crc_pos = w.size();
  w.u32(0);
  w.i8((int8_t)magic);
  w.i8((int8_t)attrs);
  if (magic == 1) w.i64(ts);
  if (key) w.bytes(*key); else w.null_bytes();
  if (value) w.bytes(*value); else w.null_bytes();
  w.patch_i32(size_pos, (int32_t)(w.size() - size_pos - 4));
  w.patch_u32(crc_pos, crc32_ieee(reinterpret_cast<const uint8_t*>(w.buf.data()) + crc_pos + 4,
                                  w.size() - crc_pos - 4));
}

}  // namespace

std::string encode_message_set(int magic, const std::vector<LegacyRecord>& recs,
                               int64_t base_offset, int codec) {
  if (magic != 0 && magic != 1) throw std::invalid_argument("legacy magic must be 0 or 1");
  if (codec == CODEC_ZSTD) throw std::invalid_argument("zstd needs message format v2");
  Writer inner;
  for (size_t i = 0; i < recs.size(); ++i) {
    const LegacyRecord& r = recs[i];
    // wrapped magic-1 messages carry relative offsets, everything else absolute ones
    const int64_t off = codec && magic == 1 ? (int64_t)i : base_offset + (int64_t)i;
    legacy_message(inner, magic, 0, off, r.timestamp, r.key_null ? nullptr : &r.key,
                   r.value_null ? nullptr : &r.value);
  }
  if (codec == CODEC_NONE) return inner.buf;
  const std::string z = compress(codec, reinterpret_cast<const uint8_t*>(inner.buf.data()),
                                 inner.size());
  Writer w;
  const int64_t ts = recs.empty() ? -1 : recs.back().timestamp;
  legacy_message(w, magic, codec, base_offset + (int64_t)recs.size() - 1, ts, nullptr, &z);
  return w.buf;
}

void message_set_offsets(const uint8_t* p, size_t len, int64_t* first, int64_t* last) {
  std::deque<std::string> hold;
  *first = -1;
  *last = -1;
  for (size_t pos = 0; pos < len;) {
    std::vector<Rec> recs;
    size_t used = 0;
    legacy_records(p + pos, len - pos, true, (size_t)1 << 30, hold, recs, &used);
    for (const Rec& r : recs) {
      if (*first < 0) *first = r.offset;
      *last = r.offset;
    }
    pos += used;
  }
  if (*first < 0) throw ProtocolError("empty message set");
}

}  // namespace kafka
}  // namespace gale
