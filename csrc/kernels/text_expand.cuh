// Random access into a nibble-packed span (csrc/codec/text_pack.h) on the device: the 16 bytes
// at any 16-byte-aligned offset of the logical text, expanded in registers. Shared by
// text_unpack (ingest.hip: the whole span into device memory) and the fused GPU ingest pass
// (json_parse.hip: CRC windows and token counting read the packed stream directly, and the
// counting waves store the expanded record text the parse needs - no separate expansion pass).
#pragma once
#include "common.cuh"

namespace gale {
namespace {

struct PackedText {
  const uint8_t* packed;  // the packed stream (device memory)
  const uint32_t* tab;    // per 2 KiB group: {packed offset of its first block, packed-block mask}
};

// nibble codes 0..15 of 8 bytes -> the 16 characters "0123456789[],-.E"
__device__ __forceinline__ uint4 expand_nibbles(uint64_t w) {
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
  return make_uint4(c[0], c[1], c[2], c[3]);
}

// bytes [p, p + 16) of the logical text, p a multiple of 16 below the span length (in the span's
// final partial block the bytes past its end are unspecified)
__device__ __forceinline__ uint4 expand16(const PackedText& t, int64_t p) {
  const int64_t q = p >> 4;
  const int64_t b = q >> 2;
  const int sub = (int)(q & 3);
  const int64_t g = b >> 5;
  const int k = (int)(b & 31);
  const uint32_t base = t.tab[2 * g], mask = t.tab[2 * g + 1];
  const int np = __popc(mask & ((1u << k) - 1u));
  const int64_t src = (int64_t)base + np * 32 + (k - np) * 64;
  if ((mask >> k) & 1u) return expand_nibbles(*reinterpret_cast<const uint64_t*>(t.packed + src + sub * 8));
  return *reinterpret_cast<const uint4*>(t.packed + src + sub * 16);
}

}  // namespace
}  // namespace gale
