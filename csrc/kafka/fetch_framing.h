// Sparse host copy of a streamed Fetch v4 response body (the bounce receive of
// csrc/runtime/pack_tap.h).
//
// The GPU ingest path never needs a host copy of the JSON text: the text crosses the link packed
// and is expanded, CRC-checked, counted and parsed on the device. The host only reads Kafka
// framing (response / partition headers, batch headers, record headers, keys, headers) and the
// two ends of each record value (the {"instances": ... } envelope check). FramingWalker sees the
// body as it streams through a small receive window and copies exactly that into the body's
// buffer at the same offsets: every byte except the interior of large record values. The
// decoders that later run on the buffer (decode_fetch_response, decode_records,
// codec::scan_envelope with its head / tail limits) read nothing else.
//
// Structure it follows: throttle, topics [name, partitions [index, error, high watermark, last
// stable offset, aborted transactions, records]], records = RecordBatch v2 [61-byte header,
// records [length, attributes, timestamp delta, offset delta, key, value, headers]]. Anything
// else inside a records region - compressed or control batches, older message formats, a
// partial trailing batch, malformed framing - is copied whole (the consumer's normalisation or
// error handling then reads it as it would a plain body).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace gale {
namespace kafka {

class FramingWalker {
 public:
  // value bytes kept at the front / back of a record value (the envelope check reads nothing
  // beyond them, codec::scan_envelope limits)
  static constexpr size_t kHead = 256, kTail = 64;

  void reset(uint8_t* dst, size_t n);
  // Body bytes [0, avail) have arrived; src points at body offset 0 (only [from, avail) of it is
  // readable: from = the lowest offset still held by the caller's window, <= copied()).
  void feed(const uint8_t* src, size_t from, size_t avail);
  size_t copied() const { return copy_; }
  size_t skipped() const { return skipped_; }  // value interior bytes not copied
  bool done() const { return copy_ >= n_; }

 private:
  enum State { RESP, TOPIC, PART, REGION, BATCH, RECORD, TAIL };
  // one parse step over dst_[0, limit): 0 = progressed; otherwise the body offset it needs
  // available (> limit) to progress
  size_t step(size_t limit);
  uint8_t* dst_ = nullptr;
  size_t n_ = 0;
  size_t copy_ = 0;     // bytes [0, copy_) handled (copied or skipped)
  size_t skipped_ = 0;
  size_t ilo_ = 0, ihi_ = 0;  // pending value interior [ilo_, ihi_), ilo_ < ihi_ when set
  State st_ = RESP;
  size_t pos_ = 0;            // parser position
  int32_t topics_left_ = 0, parts_left_ = 0, recs_left_ = 0;
  size_t region_end_ = 0, batch_end_ = 0;
};

}  // namespace kafka
}  // namespace gale
