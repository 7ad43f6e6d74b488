// GPU tokenizer for the InstObj JSON contract ({"instances": float[N][H][W][C]},
// /root/reference/src/main/java/dke/model/data/InstObj.java:8).
//
// The reference decodes every record with Jackson on a CPU worker thread
// (InferenceBolt.java:76-77) and then copies the nested float arrays into a native tensor
// (Tensor.create, :80). At ~35 KB of text per CIFAR image that float parsing is the dominant host
// cost of the whole pipeline, so gale moves it to the GPU: the host validates the
// bracket/comma structure (cheap, SIMD) and stages the raw bytes; this kernel finds every number
// token with a block-wide prefix sum, parses it with the strict JSON number grammar and writes it
// straight into the fp32 NHWC input tensor of the micro-batch.
//
// One 256-thread workgroup per record; 4 KiB of text per tile (16 B per lane, aligned loads).
// The staged byte buffer must be readable 16 bytes past every record end.
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

__device__ __forceinline__ bool is_delim(unsigned c) {
  return c == '[' || c == ']' || c == ',' || c == ' ' || c == '\n' || c == '\r' || c == '\t';
}

__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Strict JSON number: -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?, terminated by a delimiter.
__device__ float parse_number(const uint8_t* s, int64_t end, bool* ok) {
  int64_t i = 0;
  const int64_t n = end;
  bool neg = false;
  if (i < n && s[i] == '-') { neg = true; ++i; }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool good = true;
  if (i >= n) good = false;
  else if (s[i] == '0') {
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
  if (i < n && !is_delim(s[i])) good = false;  // trailing garbage inside the token
  *ok = good;
  if (!good) return 0.f;
  double v = (double)mant;
  if (mant == 0) v = 0.0;
  else if (exp10 >= 0 && exp10 <= 22) v *= kPow10[exp10];
  else if (exp10 < 0 && exp10 >= -22) v /= kPow10[-exp10];
  else v *= pow(10.0, (double)exp10);
  return (float)(neg ? -v : v);
}

__global__ __launch_bounds__(256) void json_parse_kernel(JsonRecord* recs, const uint8_t* bytes,
                                                         int per_image, float* out) {
  __shared__ int wave_tot[4];
  __shared__ int bad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const JsonRecord r = recs[blockIdx.x];
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
        const bool d = is_delim(c);
        if (!d) {
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
      bool ok = true;
      const float v = parse_number(bytes + p0 + j, end - (p0 + j), &ok);
      if (!ok) bad = 2;
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

hipError_t json_parse_instances(int nrec, const JsonRecord* recs, const uint8_t* bytes,
                                int per_image, float* out, hipStream_t stream) {
  if (nrec <= 0) return hipSuccess;
  hipLaunchKernelGGL(json_parse_kernel, dim3(nrec), dim3(256), 0, stream,
                     const_cast<JsonRecord*>(recs), bytes, per_image, out);
  return hipGetLastError();
}

}  // namespace gale
