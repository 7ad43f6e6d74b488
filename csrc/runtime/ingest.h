// Device-side ingest of Kafka fetch buffers (SURVEY.md §7.5 hard part 1: host throughput).
//
// The host path verifies every record batch's CRC32C and scans every record's JSON envelope to
// count its images before micro-batching: ~35 KB of host reads per CIFAR image on top of the
// socket receive. With an Ingest attached, a pinned fetch buffer is instead DMA'd once to its
// device mirror (PinnedPool::mirror) and the GPU computes the batch CRCs and the per-record
// element counts in one launch (ingest_crc_count, csrc/kernels/json_parse.hip). The host reads only Kafka framing
// and a bounded prefix/suffix of each record (codec::scan_envelope); the GPU replica later parses
// the records straight from the device mirror, so the JSON text crosses PCIe once and is never
// read by a host core.
#pragma once
#include <stdint.h>

#include <vector>

#include "../kafka/client.h"

namespace gale {

struct IngestIO {
  // in: per record (index into Fetched::records) the envelope check result (codec::Status,
  // array extent relative to the record value); out: image count, status raised by the GPU
  std::vector<int32_t> status;
  std::vector<int64_t> arr_off, arr_len;
  std::vector<int32_t> images;
  // out: per record, where the device left its per-tile token counts (offset from the device
  // mirror's base; -1: not kept) - the replica's parse then skips its own counting pass
  std::vector<int64_t> cnt_off;
  // out: per Fetched::batches entry, false when its CRC32C did not match (check_crcs)
  std::vector<char> batch_ok;
  // out (run() with an image arena): per record, its first image already parsed into the arena
  // as fp32 [H][W][C] (device pointer; its images follow contiguously), null: not parsed
  std::vector<const float*> img;
};

class Ingest {
 public:
  virtual ~Ingest() = default;
  virtual int device() const = 0;
  // lane: the calling decode thread (each lane owns its stream and staging buffers).
  // dev: device mirror of f.buf (same offsets), dev_cap bytes. Throws on a device error.
  // arena (optional, device memory, arena_bytes): the fetch's records are also parsed into it
  // (io.img), right behind the counting launch - the batch step then runs the forward only.
  // Record r's images take the arena slots from ceil(o / S) on, o = its instances array's
  // offset in the fetch body and S = 2 * H * W * C (a number and its separator take >= 2 bytes,
  // so the records' slot ranges never overlap and slots < f.size / S + 1).
  virtual void run(int lane, const kafka::Fetched& f, uint8_t* dev, size_t dev_cap,
                   bool check_crcs, int H, int W, int C, IngestIO& io, float* arena = nullptr,
                   size_t arena_bytes = 0) = 0;
  // fetched text bytes staged so far, and the bytes that crossed the host link for them (less
  // when the text is nibble-packed, csrc/codec/text_pack.h)
  virtual void link_bytes(int64_t& text, int64_t& link) const { text = link = 0; }
  // per run(): host work before the device (plan), the wait for the device, host work after
  // (verdicts), summed in ns over `runs` calls
  // dev_*: a sample of the runs (GALE_INGEST_DEV_TIMING=N: every N-th run of a lane) timed on
  // the device with events - the H2D copies, the count pass, the parse - and the host wait of
  // the same runs, so (host wait - device spans) is queueing behind other streams + completion
  struct Timing {
    int64_t runs = 0, prep_ns = 0, wait_ns = 0, post_ns = 0;
    int64_t plan_ns = 0;  // the part of prep_ns before the first HIP call (the rest: HIP API)
    int64_t dev_runs = 0, dev_copy_ns = 0, dev_count_ns = 0, dev_parse_ns = 0, dev_wait_ns = 0;
    int64_t plan_in_chunk = 0;  // runs whose plan rode the text's DMA (one copy, not two)
  };
  virtual Timing timing() const { return Timing(); }
};

}  // namespace gale
