// Inference replicas driven by the serving engine.
//
// A replica is the InferenceBolt's model + session (InferenceBolt.java:43-62) and its per-tuple
// execute (:70-99), generalised to micro-batches: the engine hands it a Batch of Kafka records
// (already envelope-validated by codec::scan_instances), the replica turns their JSON text into
// softmax rows. Replicas are asynchronous with a fixed depth so that host staging of batch k+1
// overlaps device work on batch k:
//   submit(b)  — enqueue (returns immediately for the GPU replica)
//   wait(b)    — block until b's outputs and per-record statuses are on the host
#pragma once
#include <stdint.h>

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "gale/executor.h"
#include "gale/kernels.h"

namespace gale {

struct InRecord;
// A record with more images than one micro-batch holds (InstObj N > max_batch): it is served as
// consecutive fragments of <= max_batch images, each a record of its own in the batcher, and the
// prediction rows are joined back into ONE {"predictions": [...]} record for the input offset.
struct SplitRecord;

struct InRecord {
  std::shared_ptr<uint8_t> buf;  // keeps the fetch buffer alive
  const uint8_t* value = nullptr;
  int32_t len = -1;              // -1 = null value
  const uint8_t* key = nullptr;  // record key (inside buf), key_len -1 = null
  int32_t key_len = -1;
  int32_t partition = -1;
  int64_t offset = -1;
  int64_t timestamp_ms = -1;     // Kafka record CreateTime
  int64_t t_fetch_ns = 0;        // host receive time
  int64_t t_take_ns = 0, t_done_ns = 0;  // its batch's dispatch / device-done time (sink metas)
  int64_t t_ready_ns = 0;                // decoded / ingested: handed to the batcher
  int64_t arr_off = 0, arr_len = 0;  // instances array inside the value (scan result)
  int32_t images = 0;
  int32_t status = 0;            // codec::Status (scan, then device parse)
  int32_t source = 0;
  bool pinned = false;           // buf is page-locked: the GPU replica DMAs straight from it
  // GPU ingest (ingest.h): the value's bytes are already in device memory, in the mirror of
  // the fetch pool of locality slot dev_locality (its key: the device, or the split slot)
  const uint8_t* dev_value = nullptr;
  int32_t dev_locality = -1;
  // its per-tile token counts, left on the device by the ingest pass (null: none)
  const uint8_t* dev_counts = nullptr;
  // its images, already parsed by the ingest pass: fp32 [H][W][C] each, contiguous, in the
  // fetch's device image arena (null: the replica parses the text)
  const float* dev_image = nullptr;
  const float* dev_arena = nullptr;  // the arena dev_image lies in (its fetch's)
  // fragment `split_index` of an oversized record (null for ordinary records)
  std::shared_ptr<SplitRecord> split;
  int32_t split_index = -1;
};

struct Batch {
  std::vector<InRecord> recs;
  int images = 0;
  int slot = 0;
  const float* probs = nullptr;  // [images, classes] after wait()
  // [images, classes] Java Float.toString slots (kFloatTextSlot bytes each) when the replica
  // formats on the device (GpuReplica gpu_encode), else null: the engine formats `probs`
  const uint8_t* pred_text = nullptr;
  std::vector<int32_t> dev_status;  // per-record codec::Status found by the replica's parser
  int64_t t_take_ns = 0, t_submit_ns = 0, t_done_ns = 0;
  bool step_graph = false;  // (GpuReplica) submitted as one replay of the slot's step graph
};

class Replica {
 public:
  virtual ~Replica() = default;
  virtual std::string name() const = 0;
  virtual int max_images() const = 0;
  virtual int depth() const = 0;  // batches that may be in flight
  virtual void submit(Batch& b) = 0;
  virtual void wait(Batch& b) = 0;
  virtual int device() const { return -1; }
  // locality slot key: replicas with the same key share a batcher and fetch-buffer pool (the
  // device for GPU replicas; stub replicas take a tag so the scheme is testable on CPU)
  virtual int locality() const { return device(); }
  // Supervisor restart after submit/wait threw (its in-flight batches were already re-queued):
  // bring the replica back to an idle, usable state or throw if it cannot be.
  virtual void recover() {}
  // records whose text this replica parsed from device memory already holding it (GPU ingest
  // mirror of its own locality slot) vs. copied over the host link (pinned or staged)
  virtual int64_t resident_records() const { return 0; }
  virtual int64_t host_records() const { return 0; }
  // batches run as ONE captured step graph (parse + forward + format + status) / with a
  // graph-captured forward only (the rest launched directly)
  virtual int64_t graph_step_batches() const { return 0; }
  virtual int64_t graph_forward_batches() const { return 0; }
  // records whose images the GPU ingest had parsed (the step ran only the forward for them)
  virtual int64_t preparsed_records() const { return 0; }
  // batches whose step was the forward alone with its inputs in the kernel arguments
  virtual int64_t table_batches() const { return 0; }
};

// CPU stub (SURVEY.md §4 "stub replica for plumbing tests on GPU-less hosts"): parses on the
// host and computes a fixed deterministic classifier, logits[k] = (k+1) * mean(x[..., k % C]),
// followed by softmax. An optional per-batch delay emulates device time.
class StubReplica : public Replica {
 public:
  StubReplica(int H, int W, int C, int classes, int max_images, int delay_us, bool compute = true,
              int locality = -1);
  std::string name() const override { return "stub"; }
  int locality() const override { return locality_; }
  int max_images() const override { return max_images_; }
  int depth() const override { return 1; }
  void submit(Batch& b) override;
  void wait(Batch& b) override;

 private:
  int H_, W_, C_, classes_, max_images_, delay_us_;
  bool compute_;
  int locality_ = -1;  // false: a "null" replica (uniform softmax, no parsing) to measure host paths
  std::vector<float> x_, probs_;
};

// One model replica on one GPU: staged JSON bytes -> GPU JSON parser -> hipGraph forward ->
// softmax rows, all on the replica's own stream. `slots` I/O buffer sets pipeline host staging
// with device work (the executor's per-slot graphs, csrc/runtime/executor.cpp).
class GpuReplica : public Replica {
 public:
  // wait_poll_us > 0: wait() first sleeps until ~85 % of the batch's expected submit -> done
  // time (a running average of the replica's recent batches), then polls the completion event
  // every wait_poll_us (the worker thread costs ~no CPU while the GPU works, and polls only
  // around the expected completion); 0: hipEventSynchronize (the HIP runtime busy-waits, lowest
  // wake-up latency, one core per waiting replica); < 0: blocking-sync completion events (the
  // thread sleeps on the device interrupt)
  // gpu_encode: the softmax rows are also formatted as prediction text on the device
  // locality: the replica's locality slot key (-1 = its device). Records ingested by another
  // slot - a steal - are not resident for this replica even on the same device: their text is
  // DMA'd from the host-pinned fetch buffer, as it would be across GPUs (--locality-split
  // exercises the multi-GPU dispatch on one device)
  // step_graph: with use_graph and a whole-network plan (Executor::device_batch_ok), each batch
  // is ONE hipGraphLaunch of the slot's captured step: JSON parse -> forward -> prediction text +
  // parse verdicts, the kernels reading the batch's record / tile / image counts and records from
  // the host-mapped metadata (no copy nodes; without gpu_encode: metadata H2D -> parse -> forward
  // -> probabilities D2H -> status D2H), so one graph per slot serves every batch size
  // high_priority: the replica's stream at the device's highest stream priority, so its step
  // kernels are dispatched ahead of the GPU ingest's when both wait for CUs
  GpuReplica(std::shared_ptr<Executor> exec, int H, int W, int C, int classes, bool use_graph,
             int wait_poll_us = 0, bool gpu_encode = false, int locality = -1,
             bool step_graph = true, bool high_priority = false, bool step_direct = false);
  ~GpuReplica() override;
  std::string name() const override;
  int max_images() const override { return exec_->max_batch(); }
  int depth() const override { return exec_->slots(); }
  int device() const override { return exec_->device(); }
  int locality() const override { return locality_ >= 0 ? locality_ : exec_->device(); }
  void submit(Batch& b) override;
  void wait(Batch& b) override;
  void recover() override;
  int64_t resident_records() const override { return resident_; }
  int64_t host_records() const override { return host_; }
  int64_t graph_step_batches() const override { return step_batches_; }
  int64_t graph_forward_batches() const override { return fwd_graph_batches_; }
  int64_t preparsed_records() const override { return preparsed_; }
  int64_t table_batches() const override { return table_batches_; }
  bool step_graph() const { return step_graph_; }

 private:
  static constexpr size_t kMetaHdr = 64;  // [nrec, ntiles, images, ...] ahead of the records
  struct Slot {
    uint8_t* h_bytes = nullptr;  // pinned staging for records that arrived in pageable memory
    uint8_t* d_bytes = nullptr;  // device copy of the batch's JSON text
    size_t h_cap = 0, d_cap = 0;
    int32_t* h_hdr = nullptr;      // metadata header (pinned) and its device mirror:
    int32_t* d_hdr = nullptr;      // [kMetaHdr][records][tile map], one allocation each
    JsonRecord* h_recs = nullptr;  // [max_batch records][tile -> record map] (pinned)
    JsonRecord* d_recs = nullptr;  // device mirror
    hipGraphExec_t step[2] = {nullptr, nullptr};  // captured steps (without / with count pass)
    int* h_tile_rec = nullptr;
    int* d_tile_rec = nullptr;
    int* d_tiles = nullptr;      // per-tile token counts (parser scratch)
    int tiles_cap = 0;
    float* h_out = nullptr;      // pinned softmax rows
    uint8_t* h_text = nullptr;   // pinned, device-mapped prediction text slots (gpu_encode)
    // copy-free step graph (gpu_encode): the kernels read the metadata from h_hdr (host-mapped)
    // and raise verdicts in d_status; the format node hands them to h_status (host-mapped)
    int* d_status = nullptr;
    int* h_status = nullptr;
    // input pointer table (ptr_input_): per batch image, its fp32 input on the device (the
    // ingest arena, or the slot's input buffer for records parsed in the step), in the metadata
    // allocation behind the records
    const float** h_xs = nullptr;
    const float** d_xs = nullptr;
    // per batch record: its index among the records the step parses (-1: parsed at ingest)
    std::vector<int> parse_idx;
    hipEvent_t done = nullptr;
    int64_t t_submit_ns = 0;
  };
  void ensure_host(Slot& s, size_t bytes);
  void ensure_device(Slot& s, size_t bytes);
  void ensure_tiles(Slot& s, int ntiles, int keep);
  void drop_steps(Slot& s);  // (buffers moved: the captured steps point at the old ones)
  hipGraphExec_t step_for(Slot& s, int slot, bool count_pass);
  hipError_t enqueue_step(Slot& s, int slot, bool count_pass, hipStream_t st, bool parse = true,
                          bool xs = false);
  template <typename Pre>
  bool try_table_step(Batch& b, Slot& s, int slot, const Pre& preparsed);
  size_t meta_rec_bytes() const;  // records + input pointer table of the metadata allocation
  static void* mapped_alloc(size_t bytes, const char* what);
  std::shared_ptr<Executor> exec_;
  int H_, W_, C_, classes_;
  bool use_graph_;
  int wait_poll_us_ = 0;
  bool gpu_encode_ = false;
  // H2D of the batch's metadata (and of any text not already resident) + parse + forward + D2H,
  // in order on ONE stream: with GPU ingest the text is resident, so a separate copy stream
  // bought no overlap, and its cross-stream wait (hipStreamWaitEvent) was where rocprofv3's
  // kernel tracing crashed under the default 6-replica concurrency; overlap comes from the
  // replicas' streams running side by side
  hipStream_t stream_ = nullptr;
  std::vector<Slot> slots_;
  int next_slot_ = 0;
  int locality_ = -1;
  std::atomic<int64_t> resident_{0}, host_{0};
  std::atomic<int64_t> step_batches_{0}, fwd_graph_batches_{0};
  bool step_graph_ = false;
  bool step_direct_ = false;  // the kernels-only step launched directly, not as a graph replay
  // batches whose records the GPU ingest already parsed (InRecord::dev_image) run the forward
  // only, reading each image through the slot's input pointer table (direct-launch step of a
  // whole-network plan with the epilogue outputs); records without parse as before
  bool ptr_input_ = false;
  std::atomic<int64_t> preparsed_{0};
  std::atomic<int64_t> table_batches_{0};  // batches launched with a kernel-argument input table
  int64_t expect_ns_ = 0;  // running average of submit -> done (adaptive sleep-poll)
};

}  // namespace gale
