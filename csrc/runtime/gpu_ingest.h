// GpuIngest: the HIP implementation of Ingest (see ingest.h). Kept out of engine.cpp so the
// sanitizer build of the host pipeline links no GPU kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "gale/kernels.h"
#include "ingest.h"

namespace gale {

class GpuIngest : public Ingest {
 public:
  // lanes: decode threads that may call run() concurrently; poll_us: sleep between completion
  // polls (0 = hipEventSynchronize)
  GpuIngest(int device, int lanes, int poll_us);
  ~GpuIngest() override;
  int device() const override { return device_; }
  void run(int lane, const kafka::Fetched& f, uint8_t* dev, size_t dev_cap, bool check_crcs,
           int H, int W, int C, IngestIO& io, float* arena = nullptr,
           size_t arena_bytes = 0) override;
  void link_bytes(int64_t& text, int64_t& link) const override {
    text = text_bytes_.load();
    link = link_bytes_.load();
  }
  Timing timing() const override {
    Timing t;
    t.runs = runs_.load();
    t.prep_ns = prep_ns_.load();
    t.plan_ns = plan_ns_.load();
    t.wait_ns = wait_ns_.load();
    t.post_ns = post_ns_.load();
    t.dev_runs = dev_runs_.load();
    t.dev_copy_ns = dev_copy_ns_.load();
    t.dev_count_ns = dev_count_ns_.load();
    t.dev_parse_ns = dev_parse_ns_.load();
    t.dev_wait_ns = dev_wait_ns_.load();
    t.plan_in_chunk = plan_in_chunk_.load();
    return t;
  }

 private:
  struct Lane {
    std::mutex mu;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    // one host-mapped pinned buffer and a device image of its plan part:
    //   [pack tab u32 x 2 per 2 KiB group][CrcChunk x nc][int2 group x ng][JsonRecord x nr]
    //   [parse JsonRecord x np][parse tile -> record i32 x npt]
    //   [group sum i32 x ng][crc u32 x nc][group verdict i32 x ng][parse tile verdict i32 x npt]
    // the host writes the plan, ONE H2D copies it (up to the group sums) into d_io, and
    // ingest_crc_count stores the results (group sums and verdicts, window CRCs) straight into
    // the host buffer: no D2H copy
    uint8_t* h_io = nullptr;
    uint8_t* d_io = nullptr;
    size_t io_cap = 0;
    int* d_counts = nullptr;  // per-tile token counts (scratch)
    size_t counts_cap = 0;
    hipEvent_t tev[4] = {nullptr, nullptr, nullptr, nullptr};  // sampled device timing
    int64_t nrun = 0;
  };
  void grow(Lane& L, size_t io_bytes, size_t tiles);
  void wait(Lane& L);
  int device_, poll_us_;
  std::atomic<int64_t> text_bytes_{0}, link_bytes_{0};
  std::atomic<int64_t> runs_{0}, prep_ns_{0}, plan_ns_{0}, wait_ns_{0}, post_ns_{0};
  std::atomic<int64_t> dev_runs_{0}, dev_copy_ns_{0}, dev_count_ns_{0}, dev_parse_ns_{0},
      dev_wait_ns_{0};
  int dev_every_ = 0;  // GALE_INGEST_DEV_TIMING
  bool plan_separate_ = false;  // GALE_INGEST_PLAN_SEPARATE
  std::atomic<int64_t> plan_in_chunk_{0};
  uint32_t* d_tables_ = nullptr;
  std::vector<std::unique_ptr<Lane>> lanes_;
  kafka::CrcShift shift_chunk_;
};

}  // namespace gale
