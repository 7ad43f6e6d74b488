// Pinned fetch-buffer pool (see pinned_pool.h).
#include "pinned_pool.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <unordered_map>

#include "../kafka/client.h"

namespace gale {

struct PinnedPool::State {
  std::mutex mu;
  std::condition_variable freed;
  int wait_ms = 0;
  int64_t waits = 0, wait_us = 0;
  std::vector<uint8_t*> free;
  std::vector<uint8_t*> all;
  std::unordered_map<const uint8_t*, uint8_t*> mirrors;  // pinned chunk -> device mirror
  int mirror_device = -1;
  size_t mirror_extra = 0;
  size_t chunk = 0, max_bytes = 0;
  bool closed = false;
  int64_t in_use = 0, in_use_max = 0, heap_too_large = 0, heap_budget = 0, no_mirror = 0;
  ~State() {
    for (uint8_t* p : all) hipHostFree(p);
    if (mirror_device >= 0 && hipSetDevice(mirror_device) == hipSuccess)
      for (auto& kv : mirrors) hipFree(kv.second);
  }
};

void PinnedPool::set_wait_ms(int ms) {
  std::lock_guard<std::mutex> lk(st_->mu);
  st_->wait_ms = ms;
}

void PinnedPool::set_mirror_device(int device, size_t extra) {
  std::lock_guard<std::mutex> lk(st_->mu);
  st_->mirror_device = device;
  st_->mirror_extra = extra;
}

size_t PinnedPool::mirror_extra() const {
  std::lock_guard<std::mutex> lk(st_->mu);
  return st_->mirror_extra;
}

uint8_t* PinnedPool::mirror(const uint8_t* base) const {
  std::lock_guard<std::mutex> lk(st_->mu);
  auto it = st_->mirrors.find(base);
  return it == st_->mirrors.end() ? nullptr : it->second;
}

PinnedPool::PinnedPool(size_t chunk_bytes, size_t max_bytes)
    : st_(std::make_shared<State>()), chunk_(chunk_bytes) {
  st_->chunk = chunk_bytes;
  st_->max_bytes = max_bytes;
}

PinnedPool::~PinnedPool() {
  std::lock_guard<std::mutex> lk(st_->mu);
  st_->closed = true;  // outstanding buffers keep State alive and are freed with it
  st_->freed.notify_all();
}

PinnedPool::Stats PinnedPool::stats() const {
  std::lock_guard<std::mutex> lk(st_->mu);
  Stats s;
  s.chunks = (int64_t)st_->all.size();
  s.in_use_max = st_->in_use_max;
  s.heap_too_large = st_->heap_too_large;
  s.heap_budget = st_->heap_budget;
  s.no_mirror = st_->no_mirror;
  s.waits = st_->waits;
  s.wait_us = st_->wait_us;
  return s;
}

size_t PinnedPool::pinned_bytes() const {
  std::lock_guard<std::mutex> lk(st_->mu);
  return st_->all.size() * st_->chunk;
}

bool PinnedPool::owns(const uint8_t* p) const {
  std::lock_guard<std::mutex> lk(st_->mu);
  for (const uint8_t* q : st_->all)
    if (q == p) return true;
  return false;
}

std::shared_ptr<uint8_t> PinnedPool::alloc(size_t n, bool* pinned) {
  if (n + 64 <= chunk_) {
    uint8_t* p = nullptr;
    {
      std::unique_lock<std::mutex> lk(st_->mu);
      if (st_->free.empty() && (st_->all.size() + 1) * st_->chunk > st_->max_bytes &&
          st_->wait_ms > 0 && !st_->closed) {
        // budget spent: wait for a release rather than stage this fetch through the heap (a
        // heap buffer takes the host decode path, which is slower and so holds records, and
        // with them chunks, longer - the pool would not recover)
        const auto t0 = std::chrono::steady_clock::now();
        ++st_->waits;
        st_->freed.wait_for(lk, std::chrono::milliseconds(st_->wait_ms),
                            [&] { return !st_->free.empty() || st_->closed; });
        st_->wait_us += std::chrono::duration_cast<std::chrono::microseconds>(
                            std::chrono::steady_clock::now() - t0)
                            .count();
      }
      if (!st_->free.empty()) {
        p = st_->free.back();
        st_->free.pop_back();
      } else if ((st_->all.size() + 1) * st_->chunk <= st_->max_bytes) {
        // portable + mapped: a DMA source for every GPU of the process, and directly readable
        // by kernels at the same address (the GPU ingest expands the packed text from here)
        if (hipHostMalloc(reinterpret_cast<void**>(&p), st_->chunk,
                          hipHostMallocPortable | hipHostMallocMapped) == hipSuccess) {
          st_->all.push_back(p);
          uint8_t* d = nullptr;
          void* dp = nullptr;
          const bool same = hipHostGetDevicePointer(&dp, p, 0) == hipSuccess && dp == p;
          if (st_->mirror_device >= 0 && same &&
              hipSetDevice(st_->mirror_device) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&d),
                        st_->mirror_extra ? mirror_extra_offset() + st_->mirror_extra
                                          : st_->chunk) == hipSuccess)
            st_->mirrors[p] = d;  // (no mirror: this chunk's records take the host path)
          else if (st_->mirror_device >= 0)
            ++st_->no_mirror;
        } else {
          p = nullptr;
        }
      }
      if (p) {
        st_->in_use_max = std::max(st_->in_use_max, ++st_->in_use);
      } else {
        ++st_->heap_budget;
      }
    }
    if (p) {
      *pinned = true;
      std::shared_ptr<State> st = st_;
      return std::shared_ptr<uint8_t>(p, [st](uint8_t* q) {
        {
          std::lock_guard<std::mutex> lk(st->mu);
          st->free.push_back(q);
          --st->in_use;
        }
        st->freed.notify_one();
      });
    }
  } else {
    std::lock_guard<std::mutex> lk(st_->mu);
    ++st_->heap_too_large;
  }
  *pinned = false;
  return kafka::heap_alloc(n);
}

}  // namespace gale
