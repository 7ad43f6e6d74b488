// Host JSON codec for the InstObj/PredObj contract (see json_codec.h).
#include "json_codec.h"

#include <algorithm>

#include <immintrin.h>
#include <math.h>
#include <string.h>

#include <charconv>

namespace gale {
namespace codec {

const char* status_name(int s) {
  switch (s) {
    case OK: return "ok";
    case BAD_ENVELOPE: return "bad_envelope";
    case UNKNOWN_KEY: return "unknown_key";
    case BAD_SHAPE: return "bad_shape";
    case EMPTY: return "empty";
    case BAD_NUMBER: return "bad_number";
    case NULL_INSTANCES: return "null_instances";
    case TOO_LARGE: return "too_large";
    case CORRUPT: return "corrupt";
    default: return "unknown";
  }
}

namespace {

inline bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

inline size_t skip_ws(const uint8_t* p, size_t i, size_t n) {
  while (i < n && is_ws(p[i])) ++i;
  return i;
}

struct Counts {
  int64_t open = 0, close = 0, quote = 0;
  int64_t first_quote = -1;
};

// One AVX-512BW pass (64 bytes per step, mask compares + popcount) where the host has it
// (Zen 4/5 hosts of MI355X nodes), else AVX2.
__attribute__((target("avx512f,avx512bw,popcnt"))) Counts count_brackets_avx512(const uint8_t* p,
                                                                                size_t n) {
  Counts c;
  size_t i = 0;
  const __m512i vo = _mm512_set1_epi8('['), vc = _mm512_set1_epi8(']'),
                vq = _mm512_set1_epi8('"');
  for (; i + 64 <= n; i += 64) {
    const __m512i v = _mm512_loadu_si512(p + i);
    c.open += __builtin_popcountll(_mm512_cmpeq_epi8_mask(v, vo));
    c.close += __builtin_popcountll(_mm512_cmpeq_epi8_mask(v, vc));
    const uint64_t q = _mm512_cmpeq_epi8_mask(v, vq);
    if (q) {
      if (c.first_quote < 0) c.first_quote = (int64_t)i + __builtin_ctzll(q);
      c.quote += __builtin_popcountll(q);
    }
  }
  for (; i < n; ++i) {
    c.open += p[i] == '[';
    c.close += p[i] == ']';
    if (p[i] == '"') {
      if (c.first_quote < 0) c.first_quote = (int64_t)i;
      ++c.quote;
    }
  }
  return c;
}

Counts count_brackets(const uint8_t* p, size_t n) {
  static const bool avx512 =
      __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  if (avx512) return count_brackets_avx512(p, n);
  Counts c;
  size_t i = 0;
  const __m256i vo = _mm256_set1_epi8('['), vc = _mm256_set1_epi8(']'),
                vq = _mm256_set1_epi8('"');
  for (; i + 32 <= n; i += 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i));
    c.open += __builtin_popcount((unsigned)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, vo)));
    c.close += __builtin_popcount((unsigned)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, vc)));
    const unsigned q = (unsigned)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, vq));
    if (q) {
      if (c.first_quote < 0) c.first_quote = (int64_t)i + __builtin_ctz(q);
      c.quote += __builtin_popcount(q);
    }
  }
  for (; i < n; ++i) {
    c.open += p[i] == '[';
    c.close += p[i] == ']';
    if (p[i] == '"') {
      if (c.first_quote < 0) c.first_quote = (int64_t)i;
      ++c.quote;
    }
  }
  return c;
}

// Strict JSON number -> float. Returns bytes consumed, 0 on a grammar error.
size_t parse_json_number(const uint8_t* p, size_t n, float* out) {
  size_t i = 0;
  if (i < n && p[i] == '-') ++i;
  if (i >= n) return 0;
  if (p[i] == '0') {
    ++i;
  } else if (p[i] >= '1' && p[i] <= '9') {
    while (i < n && p[i] >= '0' && p[i] <= '9') ++i;
  } else {
    return 0;
  }
  if (i < n && p[i] == '.') {
    ++i;
    const size_t s = i;
    while (i < n && p[i] >= '0' && p[i] <= '9') ++i;
    if (i == s) return 0;
  }
  if (i < n && (p[i] == 'e' || p[i] == 'E')) {
    ++i;
    if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
    const size_t s = i;
    while (i < n && p[i] >= '0' && p[i] <= '9') ++i;
    if (i == s) return 0;
  }
  float v = 0.f;
  auto r = std::from_chars(reinterpret_cast<const char*>(p), reinterpret_cast<const char*>(p) + i,
                           v, std::chars_format::general);
  if (r.ec == std::errc::result_out_of_range) {
    // overflow -> +-inf, underflow -> +-0 (Jackson/Java Float.parseFloat semantics)
    double d = strtod(std::string(reinterpret_cast<const char*>(p), i).c_str(), nullptr);
    v = (float)d;
  } else if (r.ec != std::errc()) {
    return 0;
  }
  *out = v;
  return i;
}

// Decimal digits (trailing zeros dropped) and exponent of a > 0: a = d1.d2d3.. x 10^e.
// precision < 0: shortest round-trip digits; otherwise `precision` digits after the first.
void sci_digits(float a, int precision, char* dig, int* nd, int* e) {
  char buf[48];
  auto r = precision < 0
               ? std::to_chars(buf, buf + sizeof(buf), a, std::chars_format::scientific)
               : std::to_chars(buf, buf + sizeof(buf), a, std::chars_format::scientific, precision);
  int n = 0;
  const char* c = buf;
  while (c < r.ptr && *c != 'e') {
    if (*c != '.') dig[n++] = *c;
    ++c;
  }
  int x = 0;
  if (c < r.ptr) {
    ++c;
    bool neg = false;
    if (*c == '-' || *c == '+') { neg = *c == '-'; ++c; }
    while (c < r.ptr) x = x * 10 + (*c++ - '0');
    if (neg) x = -x;
  }
  while (n > 1 && dig[n - 1] == '0') --n;
  *nd = n;
  *e = x;
}

}  // namespace

Scan scan_envelope(const uint8_t* p, size_t full_n, size_t head_limit, size_t tail_limit) {
  Scan s;
  // forward scans stay inside the head window, the backward scan inside the tail window
  const size_t n = std::min(full_n, head_limit);
  size_t i = skip_ws(p, 0, n);
  if (i >= n || p[i] != '{') { s.status = BAD_ENVELOPE; return s; }
  i = skip_ws(p, i + 1, n);
  if (i < n && p[i] == '}') { s.status = NULL_INSTANCES; return s; }  // {} -> instances unset
  if (i >= n || p[i] != '"') { s.status = BAD_ENVELOPE; return s; }
  static const char kKey[] = "instances";
  const size_t ks = i + 1;
  size_t ke = ks;
  while (ke < n && p[ke] != '"') {
    if (p[ke] == '\\') ++ke;
    ++ke;
  }
  if (ke >= n) { s.status = BAD_ENVELOPE; return s; }
  if (ke - ks != sizeof(kKey) - 1 || memcmp(p + ks, kKey, sizeof(kKey) - 1) != 0) {
    s.status = UNKNOWN_KEY;
    return s;
  }
  i = skip_ws(p, ke + 1, n);
  if (i >= n || p[i] != ':') { s.status = BAD_ENVELOPE; return s; }
  i = skip_ws(p, i + 1, n);
  if (i + 4 <= n && memcmp(p + i, "null", 4) == 0) {
    size_t j = skip_ws(p, i + 4, n);
    s.status = (j < n && p[j] == '}') ? NULL_INSTANCES : (j < n && p[j] == ',' ? UNKNOWN_KEY
                                                                              : BAD_ENVELOPE);
    return s;
  }
  if (i >= n || p[i] != '[') { s.status = BAD_ENVELOPE; return s; }
  const size_t beg = i;
  // trailing "] ws } ws"
  const size_t lo = std::max(beg, full_n > tail_limit ? full_n - tail_limit : (size_t)0);
  size_t j = full_n;
  while (j > lo && is_ws(p[j - 1])) --j;
  if (j == lo || p[j - 1] != '}') { s.status = BAD_ENVELOPE; return s; }
  --j;
  while (j > lo && is_ws(p[j - 1])) --j;
  if (j == lo || p[j - 1] != ']') {
    s.status = (j > beg) ? UNKNOWN_KEY : BAD_ENVELOPE;  // e.g. {"instances":[..],"k":1}
    return s;
  }
  s.arr_off = (int64_t)beg;
  s.arr_len = (int64_t)(j - beg);  // up to and including the closing ']'
  return s;
}

bool split_instances(const uint8_t* arr, size_t len,
                     std::vector<std::pair<uint32_t, uint32_t>>& spans) {
  spans.clear();
  if (len < 2 || arr[0] != '[' || arr[len - 1] != ']') return false;
  int depth = 0;
  uint32_t start = 0;
  for (size_t i = 0; i < len; ++i) {
    const uint8_t c = arr[i];
    if (c == '[') {
      if (++depth == 2) start = (uint32_t)i;
    } else if (c == ']') {
      if (depth == 2) spans.emplace_back(start, (uint32_t)(i + 1));
      if (--depth < 0) return false;
      if (depth == 0 && i != len - 1) return false;
    }
  }
  return depth == 0;
}

Scan scan_instances(const uint8_t* p, size_t n, int H, int W, int C) {
  (void)C;
  Scan s = scan_envelope(p, n);
  if (s.status != OK) return s;
  const size_t beg = (size_t)s.arr_off;
  const size_t end = beg + (size_t)s.arr_len;  // one past the closing ']'
  s.arr_off = s.arr_len = 0;
  const Counts c = count_brackets(p + beg, end - beg);
  if (c.quote > 0) {
    // a string inside the region: another key ("k": ...) or a non-number element
    size_t q = (size_t)(beg + c.first_quote) + 1;
    while (q < end && p[q] != '"') {
      if (p[q] == '\\') ++q;
      ++q;
    }
    q = skip_ws(p, q + 1, end);
    s.status = (q < end && p[q] == ':') ? UNKNOWN_KEY : BAD_NUMBER;
    return s;
  }
  if (c.open != c.close) { s.status = BAD_ENVELOPE; return s; }
  const int64_t per = 1 + (int64_t)H + (int64_t)H * W;
  if ((c.open - 1) % per != 0) { s.status = BAD_SHAPE; return s; }
  const int64_t N = (c.open - 1) / per;
  if (N == 0) { s.status = c.open == 1 ? EMPTY : BAD_SHAPE; return s; }
  if (N > (1 << 30)) { s.status = TOO_LARGE; return s; }
  s.arr_off = (int64_t)beg;
  s.arr_len = (int64_t)(end - beg);
  s.images = (int)N;
  return s;
}

int parse_instances_host(const uint8_t* p, size_t n, int H, int W, int C, float* out,
                         int max_images, int* images) {
  *images = 0;
  Scan s = scan_instances(p, n, H, W, C);
  if (s.status != OK) return s.status;
  if (max_images >= 0 && s.images > max_images) return TOO_LARGE;
  const uint8_t* q = p + s.arr_off;
  const size_t m = (size_t)s.arr_len;
  size_t i = 1;  // past the outer '['
  int64_t idx = 0;
  int img = 0;
  auto expect = [&](uint8_t ch) -> bool {
    i = skip_ws(q, i, m);
    if (i < m && q[i] == ch) { ++i; return true; }
    return false;
  };
  for (;;) {
    if (!expect('[')) return BAD_SHAPE;
    for (int h = 0; h < H; ++h) {
      if (h && !expect(',')) return BAD_SHAPE;
      if (!expect('[')) return BAD_SHAPE;
      for (int w = 0; w < W; ++w) {
        if (w && !expect(',')) return BAD_SHAPE;
        if (!expect('[')) return BAD_SHAPE;
        for (int c = 0; c < C; ++c) {
          if (c && !expect(',')) return BAD_SHAPE;
          i = skip_ws(q, i, m);
          float v;
          const size_t used = parse_json_number(q + i, m - i, &v);
          if (!used) return (i < m && (q[i] == '[' || q[i] == ']')) ? BAD_SHAPE : BAD_NUMBER;
          if (out) out[idx] = v;
          ++idx;
          i += used;
        }
        if (!expect(']')) return BAD_SHAPE;
      }
      if (!expect(']')) return BAD_SHAPE;
    }
    if (!expect(']')) return BAD_SHAPE;
    ++img;
    i = skip_ws(q, i, m);
    if (i < m && q[i] == ',') { ++i; continue; }
    if (i < m && q[i] == ']') { ++i; break; }
    return BAD_SHAPE;
  }
  if (skip_ws(q, i, m) != m) return BAD_SHAPE;
  if (img != s.images) return BAD_SHAPE;
  *images = img;
  return OK;
}

int format_float_java(float v, char* out) {
  char* o = out;
  if (isnan(v)) { memcpy(o, "NaN", 3); return 3; }
  if (signbit(v)) *o++ = '-';
  const float a = fabsf(v);
  if (isinf(a)) { memcpy(o, "Infinity", 8); return (int)(o - out) + 8; }
  if (a == 0.f) { memcpy(o, "0.0", 3); return (int)(o - out) + 3; }
  // shortest round-trip digits (std::to_chars, Ryu); JDK 19+ spec: when the shortest decimal
  // has one digit, take the decimal of length 1 or 2 closest to the value instead
  // (Float.MIN_VALUE -> "1.4E-45", not "1.0E-45"), i.e. the correctly rounded 2-digit form.
  char dig[16];
  int nd = 0, e = 0;
  sci_digits(a, -1, dig, &nd, &e);
  if (nd == 1) sci_digits(a, 1, dig, &nd, &e);
  const int dec_exp = e + 1;  // value = 0.d1d2.. x 10^dec_exp (Java FloatingDecimal decExponent)
  if (dec_exp > 0 && dec_exp < 8) {
    if (nd <= dec_exp) {
      memcpy(o, dig, nd); o += nd;
      for (int k = nd; k < dec_exp; ++k) *o++ = '0';
      *o++ = '.'; *o++ = '0';
    } else {
      memcpy(o, dig, dec_exp); o += dec_exp;
      *o++ = '.';
      memcpy(o, dig + dec_exp, nd - dec_exp); o += nd - dec_exp;
    }
  } else if (dec_exp <= 0 && dec_exp > -3) {
    *o++ = '0'; *o++ = '.';
    for (int k = 0; k < -dec_exp; ++k) *o++ = '0';
    memcpy(o, dig, nd); o += nd;
  } else {
    *o++ = dig[0];
    *o++ = '.';
    if (nd > 1) { memcpy(o, dig + 1, nd - 1); o += nd - 1; }
    else *o++ = '0';
    *o++ = 'E';
    auto r2 = std::to_chars(o, o + 8, e);
    o = r2.ptr;
  }
  return (int)(o - out);
}

void encode_predictions(const float* probs, int n, int classes, bool json_string,
                        std::string& out, bool java8) {
  out.clear();
  out.reserve((size_t)n * classes * 14 + 32);
  const char* q = json_string ? "\\\"" : "\"";
  if (json_string) out.push_back('"');
  out.push_back('{');
  out.append(q);
  out.append("predictions");
  out.append(q);
  out.append(":[");
  char buf[32];
  for (int i = 0; i < n; ++i) {
    if (i) out.push_back(',');
    out.push_back('[');
    for (int k = 0; k < classes; ++k) {
      if (k) out.push_back(',');
      const float v = probs[(size_t)i * classes + k];
      out.append(buf, java8 ? format_float_java8(v, buf) : format_float_java(v, buf));
    }
    out.push_back(']');
  }
  out.append("]}");
  if (json_string) out.push_back('"');
}

void encode_predictions_text(const uint8_t* text16, int n, int classes, bool json_string,
                             std::string& out) {
  out.clear();
  out.reserve((size_t)n * classes * 12 + 32);
  const char* q = json_string ? "\\\"" : "\"";
  if (json_string) out.push_back('"');
  out.push_back('{');
  out.append(q);
  out.append("predictions");
  out.append(q);
  out.append(":[");
  for (int i = 0; i < n; ++i) {
    if (i) out.push_back(',');
    out.push_back('[');
    for (int k = 0; k < classes; ++k) {
      if (k) out.push_back(',');
      const uint8_t* t = text16 + ((size_t)i * classes + k) * 16;
      out.append(reinterpret_cast<const char*>(t), t[15]);
    }
    out.push_back(']');
  }
  out.append("]}");
  if (json_string) out.push_back('"');
}

void encode_instances(const float* x, int n, int H, int W, int C, std::string& out) {
  out.clear();
  out.reserve((size_t)n * H * W * C * 12 + 32);
  out.append("{\"instances\":[");
  char buf[32];
  size_t i = 0;
  for (int a = 0; a < n; ++a) {
    if (a) out.push_back(',');
    out.push_back('[');
    for (int h = 0; h < H; ++h) {
      if (h) out.push_back(',');
      out.push_back('[');
      for (int w = 0; w < W; ++w) {
        if (w) out.push_back(',');
        out.push_back('[');
        for (int c = 0; c < C; ++c) {
          if (c) out.push_back(',');
          out.append(buf, format_float_java(x[i++], buf));
        }
        out.push_back(']');
      }
      out.push_back(']');
    }
    out.push_back(']');
  }
  out.append("]}");
}

void encode_error(int status, const char* detail, bool json_string, std::string& out) {
  out.clear();
  const char* q = json_string ? "\\\"" : "\"";
  if (json_string) out.push_back('"');
  out.push_back('{');
  out += q; out += "error"; out += q; out += ':'; out += q; out += status_name(status); out += q;
  if (detail && *detail) {
    out += ','; out += q; out += "detail"; out += q; out += ':'; out += q;
    for (const char* c = detail; *c; ++c) {
      if (*c == '"' || *c == '\\') out += json_string ? "\\\\\\" : "\\";
      if ((unsigned char)*c >= 0x20) out += *c;
    }
    out += q;
  }
  out.push_back('}');
  if (json_string) out.push_back('"');
}

}  // namespace codec
}  // namespace gale
