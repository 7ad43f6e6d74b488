// PackTap: a source's kafka::RecvTap that nibble-packs each fetch body (csrc/codec/text_pack.h)
// while the socket receive fills its pinned chunk (receive calls of <= 256 KiB, packed right
// after they land); the packed stream and its group table go after the
// body in the same chunk (pack_offset / tab_offset), whose device mirror is also where the GPU
// ingest lands and expands them (gpu_ingest.cpp). Bodies that do not fit twice into a chunk, or
// that went to heap memory, stay unpacked (tap_result -1).
//
// Off by default (EngineConfig::text_pack): it halves the PCIe bytes, but on the bench's 16-CPU
// share, which also runs the embedded broker, the extra pass makes the pipeline CPU-bound
// (1.21-1.26 vs 1.55 M img/s, profiles/archive/r3_nibble_transport_ab.txt). It is for hosts with cores
// to spare behind a link-bound GPU (a remote Kafka cluster leaves ~10 of 16 cores idle).
#pragma once
#include <string.h>

#include <atomic>
#include <functional>
#include <memory>
#include <vector>

#include "../codec/text_pack.h"
#include "../kafka/client.h"
#include "../kafka/fetch_framing.h"
#include "pinned_pool.h"

namespace gale {

class PackTap : public kafka::RecvTap {
 public:
  // bodies below min_bytes are not worth a device expansion launch
  explicit PackTap(std::shared_ptr<PinnedPool> pool, size_t min_bytes = 64 << 10)
      : pool_(std::move(pool)), min_bytes_(min_bytes) {}
  bool begin(uint8_t* buf, size_t n) override {
    buf_ = nullptr;
    st_ = codec::PackState();
    if (n < min_bytes_ || codec::pack_layout_bytes(n) + 64 > pool_->chunk_bytes() ||
        !pool_->owns(buf))
      return false;
    buf_ = buf;
    n_ = n;
    return false;  // (the body is received into buf as usual and packed behind it)
  }
  void progress(size_t done) override {
    if (buf_)
      codec::text_pack_blocks(buf_, done / codec::kPackBlock, buf_ + codec::pack_offset(n_), tab(),
                              st_);
  }
  int64_t finish() override {
    if (!buf_) return -1;
    const size_t link = codec::text_pack_finish(buf_, n_, buf_ + codec::pack_offset(n_), tab(), st_);
    buf_ = nullptr;
    return (int64_t)link;
  }

 private:
  uint32_t* tab() { return reinterpret_cast<uint32_t*>(buf_ + codec::tab_offset(n_)); }
  std::shared_ptr<PinnedPool> pool_;
  size_t min_bytes_;
  uint8_t* buf_ = nullptr;
  size_t n_ = 0;
  codec::PackState st_;
};

// BouncePackTap: the bounce receive. The fetch body is received piece by piece into a small
// per-source window (256 KiB: it stays in the core's L2) instead of into the pinned chunk, and
// from there
//   * nibble-packed into the chunk's packed region (pack_offset / tab_offset, as PackTap), and
//   * its Kafka framing and the two ends of every record value copied into the chunk at their
//     own offsets (kafka::FramingWalker) - the host decoders read nothing else.
// The JSON text itself is never written to host memory in full: per CIFAR image the pinned
// write and the DMA read both halve (17.4 instead of 34.8 KB) and the receive copy lands in
// cache. The device expands the packed stream into its mirror of the chunk before the CRC /
// count / parse passes (gpu_ingest.cpp), which then see the exact fetched bytes. A host path
// that needs the text (an ingest failure, the consumer's format normalisation, an oversized
// record's split) calls restore() first, which expands the packed stream in place.
class BouncePackTap : public kafka::RecvTap {
 public:
  BouncePackTap(size_t chunk_bytes, std::function<bool(const uint8_t*)> owns,
                size_t min_bytes = 64 << 10, size_t window = 256 << 10)
      : chunk_(chunk_bytes), owns_(std::move(owns)), min_bytes_(min_bytes),
        win_(window + 2 * codec::kPackBlock) {}
  bool begin(uint8_t* buf, size_t n) override {
    active_ = false;
    last_sparse_ = false;
    if (n < min_bytes_ || codec::pack_layout_bytes(n) + 64 > chunk_ || !owns_(buf)) return false;
    active_ = true;
    buf_ = buf;
    n_ = n;
    st_ = codec::PackState();
    base_ = fill_ = 0;
    walker_.reset(buf, n);
    return true;
  }
  uint8_t* window(size_t* room) override {
    *room = win_.size() - codec::kPackBlock - fill_;
    return win_.data() + fill_;
  }
  void received(size_t bytes) override {
    fill_ += bytes;
    const size_t avail = base_ + fill_;
    walker_.feed(win_.data(), base_, avail);
    const size_t full = avail / codec::kPackBlock;
    codec::text_pack_blocks(win_.data(), full, buf_ + codec::pack_offset(n_), tab(), st_, base_);
    const size_t keep_from = full * codec::kPackBlock;  // the partial block stays in the window
    const size_t keep = avail - keep_from;
    if (keep && keep_from > base_) memmove(win_.data(), win_.data() + (keep_from - base_), keep);
    base_ = keep_from;
    fill_ = keep;
  }
  void progress(size_t) override {}
  int64_t finish() override {
    if (!active_) return -1;
    active_ = false;
    const size_t link =
        codec::text_pack_finish(win_.data(), n_, buf_ + codec::pack_offset(n_), tab(), st_, base_);
    skipped_ += (int64_t)walker_.skipped();
    last_sparse_ = true;
    return (int64_t)link;
  }
  bool sparse() const override { return last_sparse_; }
  void restore(const std::shared_ptr<uint8_t>& buf, size_t n) override {
    uint8_t* b = buf.get();
    codec::text_unpack_host(b + codec::pack_offset(n),
                            reinterpret_cast<const uint32_t*>(b + codec::tab_offset(n)), n, b);
    ++restores_;
  }
  int64_t skipped_bytes() const { return skipped_; }  // value bytes never written on the host
  int64_t restores() const { return restores_.load(); }

 private:
  uint32_t* tab() { return reinterpret_cast<uint32_t*>(buf_ + codec::tab_offset(n_)); }
  size_t chunk_;
  std::function<bool(const uint8_t*)> owns_;
  size_t min_bytes_;
  std::vector<uint8_t> win_;
  bool active_ = false, last_sparse_ = false;
  uint8_t* buf_ = nullptr;
  size_t n_ = 0, base_ = 0, fill_ = 0;
  codec::PackState st_;
  kafka::FramingWalker walker_;
  int64_t skipped_ = 0;
  std::atomic<int64_t> restores_{0};  // (restore() runs on decode threads)
};

}  // namespace gale
