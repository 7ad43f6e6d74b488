// GPU decoder for the InstObj JSON contract ({"instances": float[N][H][W][C]},
// /root/reference/src/main/java/dke/model/data/InstObj.java:8).
//
// The reference decodes every record with Jackson on a CPU worker thread
// (InferenceBolt.java:76-77) and then copies the nested float arrays into a native tensor
// (Tensor.create, :80). At ~35 KB of text per CIFAR image that float parsing is the dominant host
// cost of the whole pipeline, so gale moves it to the GPU. The host only validates
// the envelope and counts '[' to get N (codec::scan_instances, AVX2) and stages the raw bytes of
// the instances array; this kernel
//   * finds every number token with a block-wide prefix sum over 16-byte lane chunks,
//   * parses it with the strict JSON number grammar straight into the fp32 NHWC batch tensor,
//   * checks that the delimiters in front of token i are exactly what a rectangular
//     [N][H][W][C] array requires ("," inside a pixel, "],[" between pixels, "]],[[" between
//     rows, "]]],[[[" between images, "[[[[" before the first and "]]]]" after the last) and that
//     the token count is N*H*W*C, so ragged or wrong-rank input is rejected like Jackson would.
//
// One 256-thread workgroup per record, 4 KiB of text per tile. Each record's bytes start 16-byte
// aligned; the buffer must be readable 16 bytes past the last record.
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

__device__ __forceinline__ bool is_ws(unsigned c) {
  return c == ' ' || c == '\n' || c == '\r' || c == '\t';
}
__device__ __forceinline__ bool is_delim(unsigned c) {
  return c == '[' || c == ']' || c == ',' || is_ws(c);
}

__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Strict JSON number -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)? ending at a delimiter.
// *len receives the token length.
__device__ float parse_number(const uint8_t* s, int64_t n, bool* ok, int* len) {
  int64_t i = 0;
  bool neg = false;
  if (i < n && s[i] == '-') { neg = true; ++i; }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool good = true;
  if (i >= n) {
    good = false;
  } else if (s[i] == '0') {
    ++i;
    if (i < n && s[i] >= '0' && s[i] <= '9') good = false;  // leading zero
  } else if (s[i] >= '1' && s[i] <= '9') {
    while (i < n && s[i] >= '0' && s[i] <= '9') {
      if (digits < 19) { mant = mant * 10 + (s[i] - '0'); ++digits; }
      else ++exp10;
      ++i;
    }
  } else {
    good = false;
  }
  if (good && i < n && s[i] == '.') {
    ++i;
    int fd = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') {
      if (digits < 19) {
        if (mant != 0 || s[i] != '0') ++digits;
        mant = mant * 10 + (s[i] - '0');
        --exp10;
      }
      ++fd;
      ++i;
    }
    if (fd == 0) good = false;
  }
  if (good && i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { eneg = s[i] == '-'; ++i; }
    int e = 0, ed = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') {
      if (e < 100000) e = e * 10 + (s[i] - '0');
      ++ed;
      ++i;
    }
    if (ed == 0) good = false;
    exp10 += eneg ? -e : e;
  }
  while (i < n && !is_delim(s[i])) { good = false; ++i; }  // trailing garbage in the token
  *ok = good;
  *len = (int)i;
  if (!good) return 0.f;
  double v = (double)mant;
  if (mant == 0) v = 0.0;
  else if (exp10 >= 0 && exp10 <= 22) v *= kPow10[exp10];
  else if (exp10 < 0 && exp10 >= -22) v /= kPow10[-exp10];
  else v *= pow(10.0, (double)exp10);
  return (float)(neg ? -v : v);
}

// Delimiters in front of token `idx` (scanning back from pos-1). Between tokens the text must be
// ws* (']' ws*)^k ',' ws* ('[' ws*)^k with k = number of trailing dimensions that wrap.
__device__ bool gap_ok(const uint8_t* s, int64_t beg, int64_t pos, int64_t idx, int C, int W,
                       int H) {
  int k = 0;
  if (idx > 0) {
    if (idx % C) k = 0;
    else if ((idx / C) % W) k = 1;
    else if ((idx / ((int64_t)C * W)) % H) k = 2;
    else k = 3;
  }
  int opens = 0, closes = 0, commas = 0;
  int64_t q = pos - 1;
  for (; q >= beg; --q) {
    const unsigned c = s[q];
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
__device__ bool tail_ok(const uint8_t* s, int64_t pos, int64_t end) {
  int closes = 0;
  for (int64_t q = pos; q < end; ++q) {
    const unsigned c = s[q];
    if (is_ws(c)) continue;
    if (c != ']') return false;
    ++closes;
  }
  return closes == 4;
}

__global__ __launch_bounds__(256) void json_parse_kernel(JsonRecord* recs, int nrec,
                                                         const uint8_t* bytes, int H, int W,
                                                         int C, float* out) {
  __shared__ int wave_tot[4];
  __shared__ int bad;
  if ((int)blockIdx.x >= nrec) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const JsonRecord r = recs[blockIdx.x];
  if (r.images <= 0 || r.len <= 0) return;
  const int per_image = H * W * C;
  const int64_t beg = r.off, end = r.off + r.len;
  const int64_t expected = (int64_t)r.images * per_image;
  float* dst = out + (int64_t)r.slot * per_image;
  if (tid == 0) bad = 0;
  __syncthreads();
  int64_t base_idx = 0;
  for (int64_t t0 = beg & ~(int64_t)15; t0 < end; t0 += 4096) {
    const int64_t p0 = t0 + 16 * tid;
    uint4 raw = make_uint4(0, 0, 0, 0);
    if (p0 < end) raw = *reinterpret_cast<const uint4*>(bytes + p0);
    const uint32_t wd[4] = {raw.x, raw.y, raw.z, raw.w};
    unsigned prev = (p0 > beg && p0 - 1 < end) ? bytes[p0 - 1] : '[';
    unsigned mask = 0;
    bool badchar = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const unsigned c = (wd[j >> 2] >> (8 * (j & 3))) & 0xff;
      const int64_t pos = p0 + j;
      if (pos >= beg && pos < end) {
        if (!is_delim(c)) {
          const bool numch = (c >= '0' && c <= '9') || c == '-' || c == '+' || c == '.' ||
                             c == 'e' || c == 'E';
          badchar |= !numch;
          if (is_delim(prev)) mask |= 1u << j;
        }
        prev = c;
      }
    }
    if (badchar) bad = 2;
    // block exclusive scan of token counts
    const int cnt = __popc(mask);
    int inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wave_tot[wave] = inc;
    __syncthreads();
    int wbase = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (w < wave) wbase += wave_tot[w];
      total += wave_tot[w];
    }
    int64_t idx = base_idx + wbase + inc - cnt;
    while (mask) {
      const int j = __ffs(mask) - 1;
      mask &= mask - 1;
      const int64_t pos = p0 + j;
      bool ok = true;
      int len = 0;
      const float v = parse_number(bytes + pos, end - pos, &ok, &len);
      if (!ok) bad = 2;
      else if (!gap_ok(bytes, beg, pos, idx, C, W, H)) bad = 3;
      else if (idx == expected - 1 && !tail_ok(bytes, pos + len, end)) bad = 3;
      if (idx < expected) dst[idx] = v;
      ++idx;
    }
    base_idx += total;
    __syncthreads();  // wave_tot reuse
  }
  __syncthreads();
  if (tid == 0) recs[blockIdx.x].status = bad ? bad : (base_idx != expected ? 1 : 0);
}

}  // namespace

hipError_t json_parse_instances(int nrec, const JsonRecord* recs, const uint8_t* bytes, int H,
                                int W, int C, float* out, hipStream_t stream) {
  if (nrec <= 0) return hipSuccess;
  if (H <= 0 || W <= 0 || C <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(json_parse_kernel, dim3(nrec), dim3(256), 0, stream,
                     const_cast<JsonRecord*>(recs), nrec, bytes, H, W, C, out);
  return hipGetLastError();
}

}  // namespace gale
