// PackTap: a source's kafka::RecvTap that nibble-packs each fetch body (csrc/codec/text_pack.h)
// while the socket receive fills its pinned chunk (receive calls of <= 256 KiB, packed right
// after they land); the packed stream and its group table go after the
// body in the same chunk (pack_offset / tab_offset), whose device mirror is also where the GPU
// ingest lands and expands them (gpu_ingest.cpp). Bodies that do not fit twice into a chunk, or
// that went to heap memory, stay unpacked (tap_result -1).
//
// Off by default (EngineConfig::text_pack): it halves the PCIe bytes, but on the bench's 16-CPU
// share, which also runs the embedded broker, the extra pass makes the pipeline CPU-bound
// (1.21-1.26 vs 1.55 M img/s, profiles/r3_nibble_transport_ab.txt). It is for hosts with cores
// to spare behind a link-bound GPU (a remote Kafka cluster leaves ~10 of 16 cores idle).
#pragma once
#include <memory>

#include "../codec/text_pack.h"
#include "../kafka/client.h"
#include "pinned_pool.h"

namespace gale {

class PackTap : public kafka::RecvTap {
 public:
  // bodies below min_bytes are not worth a device expansion launch
  explicit PackTap(std::shared_ptr<PinnedPool> pool, size_t min_bytes = 64 << 10)
      : pool_(std::move(pool)), min_bytes_(min_bytes) {}
  void begin(uint8_t* buf, size_t n) override {
    buf_ = nullptr;
    st_ = codec::PackState();
    if (n < min_bytes_ || codec::pack_layout_bytes(n) + 64 > pool_->chunk_bytes() ||
        !pool_->owns(buf))
      return;
    buf_ = buf;
    n_ = n;
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

}  // namespace gale
