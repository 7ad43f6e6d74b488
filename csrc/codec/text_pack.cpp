// Nibble transport packer (text_pack.h).
#include "text_pack.h"

#include <immintrin.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>

namespace gale {
namespace codec {

const char kPackAlphabet[17] = "0123456789[],-.E";

namespace {

// byte -> code (0..15), 0x80 outside the alphabet
std::array<uint8_t, 256> make_lut() {
  std::array<uint8_t, 256> t;
  t.fill(0x80);
  for (int c = 0; c < 16; ++c) t[(uint8_t)kPackAlphabet[c]] = (uint8_t)c;
  return t;
}
const std::array<uint8_t, 256> kLut = make_lut();

// block b is packed (32 bytes at st.out) or raw (64 bytes); group bookkeeping around it
inline void open_block(uint32_t* tab, PackState& st) {
  if (st.block % kPackGroupBlocks == 0) {
    tab[2 * (st.block / kPackGroupBlocks)] = (uint32_t)st.out;
    st.mask = 0;
  }
}
inline void close_block(uint32_t* tab, PackState& st, bool packed) {
  st.mask |= (uint32_t)packed << (st.block % kPackGroupBlocks);
  st.out += packed ? kPackBlock / 2 : kPackBlock;
  if (++st.block % kPackGroupBlocks == 0)
    tab[2 * (st.block / kPackGroupBlocks - 1) + 1] = st.mask;
}

void pack_scalar(const uint8_t* src, size_t upto, uint8_t* dst, uint32_t* tab, PackState& st,
                 size_t src_base) {
  for (; st.block < upto;) {
    open_block(tab, st);
    const uint8_t* s = src + (st.block * kPackBlock - src_base);
    uint8_t bad = 0;
    for (int i = 0; i < kPackBlock; ++i) bad |= kLut[s[i]];
    const bool packed = !(bad & 0x80);
    if (packed) {
      for (int j = 0; j < kPackBlock / 2; ++j)
        dst[st.out + j] = (uint8_t)(kLut[s[2 * j]] | (kLut[s[2 * j + 1]] << 4));
    } else {
      memcpy(dst + st.out, s, kPackBlock);
    }
    close_block(tab, st, packed);
  }
}

// 64 bytes per step: one two-table byte permute maps ASCII (low 7 bits) to codes, a sign-bit mask
// of (code | byte) rejects the block, a multiply-add of byte pairs by (1, 16) forms the packed
// bytes in 16-bit lanes and a word -> byte narrowing stores them. The group's block mask and the
// output offset stay in registers (one table store per 2 KiB).
// Stores: the packed stream goes to pinned memory that only the GPU's DMA reads next, so it is
// written with non-temporal stores (NT = true): full 64-byte lines leave through the write-
// combining buffers without a read-for-ownership of each destination line and without evicting
// the L2-resident receive window (two 32-byte halves of a line are written back to back: a
// packed block is 32 bytes, a raw one two 32-byte halves, every block 32-byte aligned).
template <bool NT>
__attribute__((target("avx512f,avx512bw,avx512vbmi"), always_inline)) inline void store32(
    uint8_t* p, __m256i v) {
  if (NT)
    _mm256_stream_si256(reinterpret_cast<__m256i*>(p), v);
  else
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(p), v);
}

template <bool NT>
__attribute__((target("avx512f,avx512bw,avx512vbmi"))) void pack_avx512(const uint8_t* src,
                                                                        size_t upto, uint8_t* dst,
                                                                        uint32_t* tab,
                                                                        PackState& st,
                                                                        size_t src_base) {
  const __m512i t0 = _mm512_loadu_si512(kLut.data());
  const __m512i t1 = _mm512_loadu_si512(kLut.data() + 64);
  const __m512i pair = _mm512_set1_epi16(0x1001);  // bytes (1, 16)
  size_t b = st.block, o = st.out;
  uint32_t mask = st.mask;
  while (b < upto) {
    const size_t g = b / kPackGroupBlocks;
    if (b % kPackGroupBlocks == 0) {
      tab[2 * g] = (uint32_t)o;
      mask = 0;
    }
    const size_t gend = std::min(upto, (g + 1) * kPackGroupBlocks);
    const uint8_t* s = src + (b * kPackBlock - src_base);
    for (; b < gend; ++b, s += kPackBlock) {
      const __m512i v = _mm512_loadu_si512(s);
      const __m512i c = _mm512_permutex2var_epi8(t0, v, t1);
      if (__builtin_expect(_mm512_movepi8_mask(_mm512_or_si512(c, v)) == 0, 1)) {
        const __m512i w = _mm512_maddubs_epi16(c, pair);
        store32<NT>(dst + o, _mm512_cvtepi16_epi8(w));
        mask |= 1u << (b % kPackGroupBlocks);
        o += kPackBlock / 2;
      } else {
        store32<NT>(dst + o, _mm512_castsi512_si256(v));
        store32<NT>(dst + o + 32, _mm512_extracti64x4_epi64(v, 1));
        o += kPackBlock;
      }
    }
    if (b % kPackGroupBlocks == 0) tab[2 * g + 1] = mask;
  }
  st.block = b;
  st.out = o;
  st.mask = mask;
}

std::atomic<bool> g_pack_nt{true};

}  // namespace

void set_pack_stream_stores(bool on) { g_pack_nt = on; }
bool pack_stream_stores() { return g_pack_nt.load(std::memory_order_relaxed); }

namespace {

__attribute__((target("sse2"))) inline void store_fence() { _mm_sfence(); }

}  // namespace

bool text_pack_fast() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                         __builtin_cpu_supports("avx512vbmi");
  return ok;
}

void text_pack_blocks(const uint8_t* src, size_t upto, uint8_t* dst, uint32_t* tab,
                      PackState& st, size_t src_base) {
  if (upto <= st.block) return;
  if (!text_pack_fast()) {
    pack_scalar(src, upto, dst, tab, st, src_base);
  } else if ((reinterpret_cast<uintptr_t>(dst) & 31) == 0 && pack_stream_stores()) {
    pack_avx512<true>(src, upto, dst, tab, st, src_base);
  } else {
    pack_avx512<false>(src, upto, dst, tab, st, src_base);
  }
}

size_t text_pack_finish(const uint8_t* src, size_t n, uint8_t* dst, uint32_t* tab, PackState& st,
                        size_t src_base) {
  const size_t full = n / kPackBlock;
  text_pack_blocks(src, full, dst, tab, st, src_base);
  const size_t r = n - full * kPackBlock;
  if (r) {  // the partial tail block: raw
    open_block(tab, st);
    memcpy(dst + st.out, src + (full * kPackBlock - src_base), r);
    st.out += r;
    st.mask &= ~(1u << (full % kPackGroupBlocks));
  }
  if (st.block % kPackGroupBlocks != 0 || r)  // an open group: its mask
    tab[2 * (full / kPackGroupBlocks) + 1] = st.mask;
  store_fence();  // the streamed stores are globally visible before the stream is handed on
  return st.out;
}

size_t text_pack(const uint8_t* src, size_t n, uint8_t* dst, uint32_t* tab, bool force_scalar) {
  PackState st;
  if (force_scalar) {
    pack_scalar(src, n / kPackBlock, dst, tab, st, 0);
    st.block = n / kPackBlock;  // (text_pack_finish sees every full block done)
  }
  return text_pack_finish(src, n, dst, tab, st);
}

void text_unpack_host(const uint8_t* packed, const uint32_t* tab, size_t n, uint8_t* out) {
  const size_t nb = (n + kPackBlock - 1) / kPackBlock;
  for (size_t b = 0; b < nb; ++b) {
    const size_t g = b / kPackGroupBlocks, k = b % kPackGroupBlocks;
    const uint32_t mask = tab[2 * g + 1];
    const uint32_t below = mask & ((1u << k) - 1u);
    const size_t np = (size_t)__builtin_popcount(below);
    const size_t src = tab[2 * g] + np * (kPackBlock / 2) + (k - np) * kPackBlock;
    const size_t len = b + 1 < nb || n % kPackBlock == 0 ? kPackBlock : n % kPackBlock;
    uint8_t* d = out + b * kPackBlock;
    if (mask >> k & 1u) {
      for (size_t j = 0; j < len; ++j)
        d[j] = (uint8_t)kPackAlphabet[(packed[src + j / 2] >> (4 * (j & 1))) & 15];
    } else {
      memcpy(d, packed + src, len);
    }
  }
}

}  // namespace codec
}  // namespace gale
