// Pool of pinned (page-locked) host buffers for Kafka fetch responses.
//
// The engine's consumers receive Fetch response bodies straight into these buffers, so the
// GPU replica can DMA the JSON text of a micro-batch to the device with hipMemcpyAsync without
// first copying it into a staging buffer (the reference copies every tuple's float arrays into a
// fresh native Tensor instead, InferenceBolt.java:80). Buffers are recycled through the pool
// when the last record referencing them is released; requests larger than a chunk or beyond the
// pool's byte budget fall back to ordinary heap memory (the replica then stages them).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

namespace gale {

class PinnedPool {
 public:
  PinnedPool(size_t chunk_bytes, size_t max_bytes);
  ~PinnedPool();
  PinnedPool(const PinnedPool&) = delete;
  PinnedPool& operator=(const PinnedPool&) = delete;

  // A buffer of at least n bytes (+64 slack). *pinned tells whether it is page-locked.
  std::shared_ptr<uint8_t> alloc(size_t n, bool* pinned);
  size_t chunk_bytes() const { return chunk_; }
  bool owns(const uint8_t* p) const;  // p is the base of one of this pool's pinned chunks
  size_t pinned_bytes() const;
  // heap fallbacks: requests larger than a chunk / requests past the budget with no chunk free
  struct Stats {
    int64_t chunks = 0, in_use_max = 0, heap_too_large = 0, heap_budget = 0, no_mirror = 0;
    int64_t waits = 0, wait_us = 0;
  };
  Stats stats() const;
  // Device mirrors (GPU ingest, ingest.h): every pinned chunk gets a buffer on `device` holding
  // the chunk's bytes at the same offsets, plus `extra` bytes behind them (from offset
  // mirror_extra_offset(): the image arena the GPU ingest parses the chunk's records into). Set
  // before the first alloc. mirror(base) -> nullptr when base is not a pinned chunk of this pool
  // (or mirrors are off).
  void set_mirror_device(int device, size_t extra = 0);
  size_t mirror_extra_offset() const { return (chunk_ + 255) & ~(size_t)255; }
  size_t mirror_extra() const;
  // Backpressure: with the budget spent and no chunk free, alloc waits up to `ms` for one to be
  // released before it falls back to the heap (0 = fall back at once).
  void set_wait_ms(int ms);
  uint8_t* mirror(const uint8_t* base) const;

 private:
  struct State;
  std::shared_ptr<State> st_;
  size_t chunk_;
};

}  // namespace gale
