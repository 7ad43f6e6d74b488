// GPU decoder for the InstObj JSON contract ({"instances": float[N][H][W][C]},
// /root/reference/src/main/java/dke/model/data/InstObj.java:8).
//
// The reference decodes every record with Jackson on a CPU worker thread
// (InferenceBolt.java:76-77) and then copies the nested float arrays into a native tensor
// (Tensor.create, :80). At ~35 KB of text per CIFAR image that float parsing is the dominant host
// cost of the whole pipeline, so gale moves it to the GPU. The host only validates
// the envelope and counts '[' to get N (codec::scan_instances, AVX2) and stages the raw bytes of
// the instances array; the device then
//   * splits every record's text into 4 KiB tiles (tile t of the batch = one workgroup, so a
//     256-record CIFAR batch is ~2300 workgroups: the whole chip, not one workgroup per record),
//   * pass 1 (json_count_kernel): counts the number tokens of each tile (a token starts at a
//     non-delimiter byte that follows a delimiter) and rejects bytes outside the number alphabet,
//   * pass 2 (json_parse_kernel): the tile's first token index = sum of the counts of the
//     record's earlier tiles (block reduction), a block-wide prefix sum over 16-byte lane chunks
//     gives every token its element index, and each token is parsed with the strict JSON number
//     grammar straight into the fp32 NHWC batch tensor from an LDS copy of the tile (+ halos),
//   * checks that the delimiters in front of token i are exactly what a rectangular
//     [N][H][W][C] array requires ("," inside a pixel, "],[" between pixels, "]],[[" between
//     rows, "]]],[[[" between images, "[[[[" before the first and "]]]]" after the last) and that
//     the token count is N*H*W*C, so ragged or wrong-rank input is rejected like Jackson would.
// Per-record status is the max over the flags raised by its tiles (atomicMax): 1 count mismatch,
// 2 malformed number / element, 3 bad structure; the host zeroes it before the launch.
//
// Each record's bytes start 16-byte aligned; the buffer must be readable 16 bytes past the last
// record.
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

constexpr int kTile = kJsonTileBytes;  // bytes per workgroup tile (256 lanes x 16 B)
constexpr int kHalo = 64;              // LDS halo on each side (token tails, delimiter look-back)

__device__ __forceinline__ bool is_ws(unsigned c) {
  return c == ' ' || c == '\n' || c == '\r' || c == '\t';
}
__device__ __forceinline__ bool is_delim(unsigned c) {
  return c == '[' || c == ']' || c == ',' || is_ws(c);
}
__device__ __forceinline__ bool is_numch(unsigned c) {
  return (c >= '0' && c <= '9') || c == '-' || c == '+' || c == '.' || c == 'e' || c == 'E';
}

__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// The record text as seen by one workgroup: [lo, hi) is mirrored in LDS, anything else (a very
// long token or a very long whitespace run) falls back to global memory.
struct Text {
  const uint8_t* g;
  const uint8_t* l;
  int64_t lo, hi;
  __device__ __forceinline__ unsigned at(int64_t q) const {
    return (q >= lo && q < hi) ? (unsigned)l[q - lo] : (unsigned)g[q];
  }
};

// Token-start mask of the 16 bytes at p0 (bit j: byte p0+j starts a token); *badchar is set for a
// byte inside [beg, end) that is neither a delimiter nor in the number alphabet.
__device__ __forceinline__ unsigned token_mask(uint4 raw, unsigned prev, int64_t p0, int64_t beg,
                                               int64_t end, bool* badchar) {
  const uint32_t wd[4] = {raw.x, raw.y, raw.z, raw.w};
  unsigned mask = 0;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const unsigned c = (wd[j >> 2] >> (8 * (j & 3))) & 0xff;
    const int64_t pos = p0 + j;
    if (pos >= beg && pos < end) {
      if (!is_delim(c)) {
        bad |= !is_numch(c);
        if (is_delim(prev)) mask |= 1u << j;
      }
      prev = c;
    }
  }
  *badchar = bad;
  return mask;
}

// Strict JSON number -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)? starting at i and ending at a
// delimiter or `end`. *len receives the token length.
__device__ float parse_number(const Text& t, int64_t i0, int64_t end, bool* ok, int* len) {
  int64_t i = i0;
  bool neg = false;
  unsigned c = i < end ? t.at(i) : 0u;
  if (c == '-') { neg = true; ++i; c = i < end ? t.at(i) : 0u; }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool good = true;
  if (i >= end) {
    good = false;
  } else if (c == '0') {
    ++i;
    c = i < end ? t.at(i) : 0u;
    if (c >= '0' && c <= '9') good = false;  // leading zero
  } else if (c >= '1' && c <= '9') {
    while (c >= '0' && c <= '9') {
      if (digits < 19) { mant = mant * 10 + (c - '0'); ++digits; }
      else ++exp10;
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
  *len = (int)(i - i0);
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
__device__ bool gap_ok(const Text& t, int64_t beg, int64_t pos, uint32_t idx, uint32_t C,
                       uint32_t W, uint32_t H) {
  int k = 0;
  if (idx > 0) {  // (32-bit: a record holds < 2^32 numbers; 64-bit division is ~10x dearer)
    const uint32_t px = idx / C;
    if (idx - px * C) k = 0;
    else {
      const uint32_t row = px / W;
      if (px - row * W) k = 1;
      else if (row % H) k = 2;
      else k = 3;
    }
  }
  int opens = 0, closes = 0, commas = 0;
  int64_t q = pos - 1;
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
__device__ bool tail_ok(const Text& t, int64_t pos, int64_t end) {
  int closes = 0;
  for (int64_t q = pos; q < end; ++q) {
    const unsigned c = t.at(q);
    if (is_ws(c)) continue;
    if (c != ']') return false;
    ++closes;
  }
  return closes == 4;
}

__device__ __forceinline__ int block_sum(int v, int* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) red[wave] = v;
  __syncthreads();
  const int s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(256) void json_count_kernel(JsonRecord* recs, const int* tile_rec,
                                                         const uint8_t* bytes, int* counts) {
  __shared__ int red[4];
  const int t = blockIdx.x;
  const int ri = tile_rec[t];
  const JsonRecord r = recs[ri];
  const int64_t beg = r.off, end = r.off + r.len;
  const int64_t t0 = (beg & ~(int64_t)15) + (int64_t)(t - r.tile0) * kTile;
  const int64_t p0 = t0 + 16 * threadIdx.x;
  int cnt = 0;
  bool bad = false;
  if (p0 < end) {
    const uint4 raw = *reinterpret_cast<const uint4*>(bytes + p0);
    const unsigned prev = (p0 > beg) ? bytes[p0 - 1] : '[';
    cnt = __popc(token_mask(raw, prev, p0, beg, end, &bad));
  }
  if (bad) atomicMax(&recs[ri].status, 2);
  cnt = block_sum(cnt, red);
  if (threadIdx.x == 0) counts[t] = cnt;
}

__global__ __launch_bounds__(256) void json_parse_kernel(JsonRecord* recs, const int* tile_rec,
                                                         const uint8_t* bytes, int H, int W,
                                                         int C, const int* counts, float* out) {
  __shared__ __attribute__((aligned(16))) uint8_t text[kTile + 2 * kHalo];
  __shared__ int red[4];
  __shared__ int wave_tot[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = blockIdx.x;
  const int ri = tile_rec[t];
  const JsonRecord r = recs[ri];
  const int per_image = H * W * C;
  const int64_t beg = r.off, end = r.off + r.len;
  const int64_t abeg = beg & ~(int64_t)15;
  const int64_t expected = (int64_t)r.images * per_image;
  const int64_t t0 = abeg + (int64_t)(t - r.tile0) * kTile;
  const int ntiles = (int)((end - abeg + kTile - 1) / kTile);
  const bool last_tile = (t - r.tile0) == ntiles - 1;

  // stage [t0 - halo, t0 + tile + halo) clipped to the record's 16-byte-aligned extent
  Text tx;
  tx.g = bytes;
  tx.l = text;
  tx.lo = t0 - kHalo < abeg ? abeg : t0 - kHalo;
  const int64_t aend = (end + 15) & ~(int64_t)15;
  tx.hi = t0 + kTile + kHalo > aend ? aend : t0 + kTile + kHalo;
  for (int64_t q = tx.lo + 16 * tid; q < tx.hi; q += 16 * 256)
    *reinterpret_cast<uint4*>(text + (q - tx.lo)) = *reinterpret_cast<const uint4*>(bytes + q);

  // first token index of this tile: the counts of the record's earlier tiles
  int part = 0;
  for (int k = r.tile0 + tid; k < t; k += 256) part += counts[k];
  const int64_t base_idx = block_sum(part, red);  // (its barriers also publish the LDS text)

  const int64_t p0 = t0 + 16 * tid;
  uint4 raw = make_uint4(0, 0, 0, 0);
  unsigned mask = 0;
  bool bad_ignored;
  if (p0 < end) {
    raw = *reinterpret_cast<const uint4*>(text + (p0 - tx.lo));
    const unsigned prev = (p0 > beg) ? tx.at(p0 - 1) : '[';
    mask = token_mask(raw, prev, p0, beg, end, &bad_ignored);
  }
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
  float* dst = out + (int64_t)r.slot * per_image;
  int bad = 0;
  while (mask) {
    const int j = __ffs(mask) - 1;
    mask &= mask - 1;
    const int64_t pos = p0 + j;
    bool ok = true;
    int len = 0;
    const float v = parse_number(tx, pos, end, &ok, &len);
    if (!ok) bad = max(bad, 2);
    else if (!gap_ok(tx, beg, pos, (uint32_t)idx, (uint32_t)C, (uint32_t)W, (uint32_t)H)) bad = 3;
    else if (idx == expected - 1 && !tail_ok(tx, pos + len, end)) bad = 3;
    if (idx < expected) dst[idx] = v;
    ++idx;
  }
  if (last_tile && tid == 0 && base_idx + total != expected) bad = max(bad, 1);
  if (bad) atomicMax(&recs[ri].status, bad);
}

}  // namespace

int json_tile_count(int64_t off, int32_t len) {
  if (len <= 0) return 0;
  const int64_t abeg = off & ~(int64_t)15;
  return (int)((off + len - abeg + kJsonTileBytes - 1) / kJsonTileBytes);
}

hipError_t json_parse_instances(int nrec, int ntiles, JsonRecord* recs, const int* tile_rec,
                                const uint8_t* bytes, int H, int W, int C, int* tile_counts,
                                float* out, hipStream_t stream) {
  if (nrec <= 0 || ntiles <= 0) return hipSuccess;
  if (H <= 0 || W <= 0 || C <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(json_count_kernel, dim3(ntiles), dim3(256), 0, stream, recs, tile_rec, bytes,
                     tile_counts);
  hipLaunchKernelGGL(json_parse_kernel, dim3(ntiles), dim3(256), 0, stream, recs, tile_rec, bytes,
                     H, W, C, tile_counts, out);
  return hipGetLastError();
}

}  // namespace gale
