// GPU CRC32C of Kafka record batches (the consumer's check.crcs) for the
// device-side ingest pass (csrc/runtime/gpu_ingest.cpp).
//
// The reference's KafkaSpout validates every fetched batch on a JVM thread (storm-kafka /
// kafka-clients, MainTopology.java:53,95-106). gale's host did it with VPCLMULQDQ folding at
// ~1.4 cores per MI355X of JSON; here the fetch buffer is DMA'd to the GPU once (the JSON parser
// then reads it from there) and the GPU folds it: one wave per 4 KiB window, 64 contiguous bytes
// per lane through slicing-by-4 tables in LDS, then each lane's register is advanced over the
// bytes that follow its piece by ONE GF(2) multiply with its constant x^(8*64*(63-lane)) mod P
// (a 32-step shift-and-xor: no per-level shift tables, so a workgroup stages 4.25 KB of tables
// instead of 28 KB) and the wave XOR-reduces (CRCs are linear: crc(A ++ B) =
// crc(A) * x^(8|B|) ^ crc(B) for raw registers). Leading zero
// bytes do not change a raw CRC, so a window shorter than 4 KiB simply leaves its first lanes
// empty. Misaligned ends are folded byte by byte; everything else uses aligned dword loads.
#include "common.cuh"
#include "crc32c.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

__global__ __launch_bounds__(256) void crc32c_chunks_kernel(const uint8_t* bytes,
                                                            const CrcChunk* chunks, int n,
                                                            const uint32_t* tables,
                                                            uint32_t* out) {
  __shared__ uint32_t T[crc::kTableWords];
  crc::crc_stage_tables(tables, T);
  crc::crc_windows(bytes, chunks, n, T, out, blockIdx.x, gridDim.x);
}

// Nibble-transport expansion (csrc/codec/text_pack.h): one thread per 16 output bytes, so a
// 64-byte block is four lanes and a 2 KiB group two quarter-waves. A lane finds its block's
// source from the group's base offset plus the popcount of the packed blocks before it (packed
// blocks are 32 bytes, raw 64): one 8-byte load becomes 16 characters (one 16-byte store), or a
// raw piece is copied. Only a raw final partial block stores bytewise. The volume is the fetched
// text (~54 GB/s at the link's pace): a few us per fetch against 8 TB/s of HBM.
__global__ __launch_bounds__(256) void text_unpack_kernel(const uint8_t* __restrict__ packed,
                                                          const uint32_t* __restrict__ tab,
                                                          int64_t n, uint8_t* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t o = q * 16;
  if (o >= n) return;
  const int64_t b = q >> 2;
  const int sub = (int)(q & 3);
  const int64_t g = b >> 5;
  const int k = (int)(b & 31);
  const uint32_t base = tab[2 * g], mask = tab[2 * g + 1];
  const int np = __popc(mask & ((1u << k) - 1u));
  const int64_t src = (int64_t)base + np * 32 + (k - np) * 64;
  if ((mask >> k) & 1u) {
    const uint64_t w = *reinterpret_cast<const uint64_t*>(packed + src + sub * 8);
    uint32_t c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t nib = (uint32_t)(w >> (16 * i + 4 * j)) & 15u;
        // codes 10..15 -> "[],-.E"
        const uint32_t ch = nib < 10 ? 0x30u + nib
                                     : (uint32_t)(0x452E2D2C5D5Bull >> ((nib - 10) * 8)) & 0xffu;
        v |= ch << (8 * j);
      }
      c[i] = v;
    }
    *reinterpret_cast<uint4*>(out + o) = make_uint4(c[0], c[1], c[2], c[3]);
  } else if (o + 16 <= n) {
    *reinterpret_cast<uint4*>(out + o) =
        *reinterpret_cast<const uint4*>(packed + src + sub * 16);
  } else {
    for (int64_t j = 0; o + j < n; ++j) out[o + j] = packed[src + sub * 16 + j];
  }
}

}  // namespace

hipError_t text_unpack(const uint8_t* packed, const uint32_t* tab, int64_t n, uint8_t* out,
                       hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t pieces = (n + 15) / 16;
  hipLaunchKernelGGL(text_unpack_kernel, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0,
                     stream, packed, tab, n, out);
  return hipGetLastError();
}

hipError_t crc32c_chunks(const uint8_t* bytes, const CrcChunk* chunks, int n,
                         const uint32_t* tables, uint32_t* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int blocks = (n + crc::kCrcWaves - 1) / crc::kCrcWaves;
  if (blocks > 1024) blocks = 1024;  // waves loop: the 28 KB table load is amortised
  hipLaunchKernelGGL(crc32c_chunks_kernel, dim3(blocks), dim3(64 * crc::kCrcWaves), 0, stream, bytes,
                     chunks, n, tables, out);
  return hipGetLastError();
}

}  // namespace gale
