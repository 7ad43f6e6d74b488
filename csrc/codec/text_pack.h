// Nibble transport for JSON number text across the host -> GPU link.
//
// The InstObj records the reference's spout reads are Jackson text (float[][][][] written with
// Java Float.toString): after the 13-byte envelope, every byte is one of 16 characters
//     0 1 2 3 4 5 6 7 8 9 [ ] , - . E
// so a 4-bit code carries it losslessly. On one MI355X the headline path is bound by the PCIe
// link (the fetched text crosses it once, 54 of ~55.5 GB/s measured pinned H2D at 1.56 M img/s,
// profiles/archive/r3_bench_session2_start.jsonl); packing the text 2:1 on the host before the DMA and
// expanding it on the device (text_unpack in csrc/kernels/ingest.hip) halves the link bytes at
// the price of one more host pass (opt-in, see csrc/runtime/pack_tap.h for the measured trade). The
// device then holds the exact fetched bytes again: the batch CRC32Cs are checked over the
// expanded text, so a packing error cannot pass silently.
//
// Format of a packed span of n logical bytes:
//   * 64-byte blocks; a block whose 64 bytes are all in the alphabet is stored as 32 bytes (code
//     of byte 2j in the low nibble of byte j, byte 2j+1 in the high nibble), any other block as
//     its 64 raw bytes. A final partial block (n % 64 bytes) is always raw.
//   * groups of 32 blocks (2 KiB of text): tab[2g] = byte offset of group g's first block in
//     the packed stream, tab[2g + 1] = bit b set <=> block b of the group is packed.
// Every block starts at a multiple of 32 bytes of the packed stream (16-byte aligned stores and
// loads on the device). Record framing, headers and keys fall into the (rare) raw blocks, so no
// record structure is needed on the packing side: it is a pass over the fetch buffer.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace gale {
namespace codec {

constexpr int kPackBlock = 64;
constexpr int kPackGroupBlocks = 32;
constexpr int kPackGroupBytes = kPackBlock * kPackGroupBlocks;

inline size_t pack_groups(size_t n) { return (n + kPackGroupBytes - 1) / kPackGroupBytes; }
// worst case (no block packs): the raw bytes
inline size_t pack_bound(size_t n) { return n; }

// code -> character
extern const char kPackAlphabet[17];

// In-place layout used by the fetch path (the packed copy lives in the same pinned chunk as the
// n-byte body it was made from, so the device mirror of that chunk doubles as its landing zone):
//   [0, n) body | [pack_offset(n), +n) packed stream | [tab_offset(n), +8 * pack_groups(n)) tab
inline size_t pack_offset(size_t n) { return (n + 63) & ~(size_t)63; }
inline size_t tab_offset(size_t n) { return 2 * pack_offset(n); }
inline size_t pack_layout_bytes(size_t n) { return tab_offset(n) + 8 * pack_groups(n); }

// Resumable packing (e.g. chunk by chunk while a socket receive fills the buffer): blocks are
// numbered from src; text_pack_blocks packs whole blocks [st.block, upto) and text_pack_finish
// packs the remaining blocks and the partial tail of an n-byte span and returns the packed size.
struct PackState {
  size_t block = 0;   // next block to pack
  size_t out = 0;     // packed bytes written so far
  uint32_t mask = 0;  // packed-block bits of the open group
};
// src_base: the span offset src points at (src holds bytes [src_base, ...) of the span: a
// receive window sliding over it); blocks before src_base must already be packed.
void text_pack_blocks(const uint8_t* src, size_t upto, uint8_t* dst, uint32_t* tab,
                      PackState& st, size_t src_base = 0);
size_t text_pack_finish(const uint8_t* src, size_t n, uint8_t* dst, uint32_t* tab, PackState& st,
                        size_t src_base = 0);

// True when the host has the vector path (AVX-512 VBMI byte permutes); the scalar path is exact
// but ~10x slower, so the engine only packs by default when this holds.
bool text_pack_fast();

// Non-temporal stores for the packed stream (default on; a 32-byte-aligned destination): the
// pinned chunk is read next by the GPU's DMA, not by this core. Process-wide switch for A/B.
void set_pack_stream_stores(bool on);
bool pack_stream_stores();

// Packs src[0, n) into dst (>= pack_bound(n) bytes) and tab (2 * pack_groups(n) words).
// Returns the packed size. force_scalar selects the reference path (tests).
size_t text_pack(const uint8_t* src, size_t n, uint8_t* dst, uint32_t* tab,
                 bool force_scalar = false);

// Host reference of the device expansion (tests).
void text_unpack_host(const uint8_t* packed, const uint32_t* tab, size_t n, uint8_t* out);

}  // namespace codec
}  // namespace gale
