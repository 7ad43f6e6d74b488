// CRC32C of Kafka record-batch windows on the device (see ingest.hip): slicing-by-4 tables in
// LDS, one wave per 4 KiB window, lanes joined by GF(2) shifts. Shared by the standalone CRC
// kernel (ingest.hip) and the fused ingest kernel (json_parse.hip).
#pragma once
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace crc {

constexpr int kCrcWaves = 4;
constexpr int kTableWords = 1024 + 64;
constexpr uint32_t kPoly = 0x82f63b78u;  // CRC-32C, reflected

__device__ __forceinline__ uint32_t crc_byte(const uint32_t* T, uint32_t c, uint32_t b) {
  return (c >> 8) ^ T[(c ^ b) & 0xffu];
}

__device__ __forceinline__ uint32_t crc_word(const uint32_t* T, uint32_t c, uint32_t w) {
  const uint32_t x = c ^ w;  // byte 0 (first in the stream) is advanced the most
  return T[768 + (x & 0xffu)] ^ T[512 + ((x >> 8) & 0xffu)] ^ T[256 + ((x >> 16) & 0xffu)] ^
         T[x >> 24];
}

// a * b mod P, reflected domain (bit 31 = x^0): the host's poly_mulmod (csrc/kafka/wire.cpp)
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    r ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return r;
}

// The windows of workgroup `block` of `nblocks` (T: the tables, already staged in LDS).
__device__ __forceinline__ void crc_windows(const uint8_t* bytes, const CrcChunk* chunks, int n,
                                            const uint32_t* T, uint32_t* out, int block,
                                            int nblocks) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c = block * kCrcWaves + wave; c < n; c += nblocks * kCrcWaves) {
    const CrcChunk ch = chunks[c];
    const int64_t cs = ch.end - ch.len;
    const int64_t wa = ch.end - (int64_t)64 * (64 - lane);  // this lane's piece [wa, wa + 64)
    const int64_t hi = wa + 64;
    int64_t q = wa > cs ? wa : cs;
    uint32_t crc = 0;
    if (q < hi) {
      while (q < hi && (q & 3)) crc = crc_byte(T, crc, bytes[q++]);
      for (; q + 4 <= hi; q += 4) crc = crc_word(T, crc, *reinterpret_cast<const uint32_t*>(bytes + q));
      while (q < hi) crc = crc_byte(T, crc, bytes[q++]);
    }
    crc = gf2_mulmod(crc, T[1024 + lane]);  // over the 64 * (63 - lane) bytes that follow
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) crc ^= __shfl_xor(crc, o, 64);
    if (lane == 0) out[c] = crc;
  }
}

__device__ __forceinline__ void crc_stage_tables(const uint32_t* tables, uint32_t* T) {
  for (int i = threadIdx.x; i < kTableWords; i += blockDim.x) T[i] = tables[i];
  __syncthreads();
}

}  // namespace crc
}  // namespace gale
