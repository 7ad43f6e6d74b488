// Kafka wire-protocol primitives: big-endian framing, zig-zag varints, CRC32C and the
// RecordBatch v2 ("magic 2") codec.
//
// The reference reaches Kafka through storm-kafka's KafkaSpout (consume, MainTopology.java:53,
// 95-106) and kafka-clients 0.11's KafkaProducer (produce, KafkaBolt.java:111-113, 144). Neither
// library exists in this image and the GPU boxes have no network, so gale speaks the protocol
// itself: this header is the shared codec of the in-repo client
// (csrc/kafka/client.cpp) and the embedded broker (csrc/kafka/broker.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace gale {
namespace kafka {

struct ProtocolError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// CRC32C (Castagnoli) with the SSE4.2 crc32 instruction (VPCLMULQDQ folding when available).
uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc = 0);
// Raw (un-inverted) CRC register arithmetic: crc32c_raw continues a raw state over p[0..n);
// crc32c_shift appends nbytes zero bytes to a raw state (multiplication by x^(8 nbytes) mod P).
uint32_t crc32c_raw(const uint8_t* p, size_t n, uint32_t raw);
uint32_t crc32c_shift(uint32_t raw, uint64_t nbytes);
// Fixed-length shift of a raw CRC register by table lookup (4 loads).
class CrcShift {
 public:
  explicit CrcShift(uint64_t nbytes);
  uint32_t operator()(uint32_t raw) const;

 private:
  struct Impl;
  std::shared_ptr<Impl> impl_;
};
// Tables of the GPU CRC32C kernel (csrc/kernels/ingest.hip), kCrcDeviceTableWords words:
// [0, 1024) slicing-by-4 byte tables, [1024, 1088) per-lane shift constants
// x^(8 * 64 * (63 - lane)) mod P (reflected).
constexpr int kCrcDeviceTableWords = 1024 + 64;
void crc32c_device_tables(uint32_t* out);
// crc32c(A ++ B) from crc32c(A), crc32c(B) and |B|.
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
// CRC of a message after bytes [k, k+n) changed from old_bytes to new_bytes, with bytes_after
// bytes following the window (n <= 64): O(log length), the message itself is not re-read.
uint32_t patch_batch_crc(uint32_t crc, const uint8_t* old_bytes, const uint8_t* new_bytes,
                         size_t n, uint64_t bytes_after);

class Writer {
 public:
  std::string buf;
  void reserve(size_t n) { buf.reserve(n); }
  size_t size() const { return buf.size(); }
  void i8(int8_t v) { buf.push_back((char)v); }
  void i16(int16_t v) { be(&v, 2); }
  void i32(int32_t v) { be(&v, 4); }
  void u32(uint32_t v) { be(&v, 4); }
  void i64(int64_t v) { be(&v, 8); }
  void raw(const void* p, size_t n) { buf.append(static_cast<const char*>(p), n); }
  void str(std::string_view s) {
    i16((int16_t)s.size());
    raw(s.data(), s.size());
  }
  void nstr(const std::string* s) {  // nullable string
    if (!s) { i16(-1); return; }
    str(*s);
  }
  void null_str() { i16(-1); }
  void bytes(std::string_view s) {
    i32((int32_t)s.size());
    raw(s.data(), s.size());
  }
  void null_bytes() { i32(-1); }
  void array_len(int32_t n) { i32(n); }
  void varint(int32_t v) { uvarint(((uint32_t)v << 1) ^ (uint32_t)(v >> 31)); }
  void varlong(int64_t v) { uvarint(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
  void uvarint(uint64_t v) {
    while (v >= 0x80) {
      buf.push_back((char)(v | 0x80));
      v >>= 7;
    }
    buf.push_back((char)v);
  }
  void patch_i32(size_t pos, int32_t v) { put_be(&buf[pos], &v, 4); }
  void patch_u32(size_t pos, uint32_t v) { put_be(&buf[pos], &v, 4); }
  static void put_be(char* dst, const void* v, int n) {
    const uint8_t* s = static_cast<const uint8_t*>(v);
    for (int i = 0; i < n; ++i) dst[i] = (char)s[n - 1 - i];
  }

 private:
  void be(const void* v, int n) {
    char t[8];
    put_be(t, v, n);
    buf.append(t, n);
  }
};

class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  Reader(std::string_view s) : p_(reinterpret_cast<const uint8_t*>(s.data())), n_(s.size()) {}
  size_t pos() const { return i_; }
  size_t remaining() const { return n_ - i_; }
  const uint8_t* ptr() const { return p_ + i_; }
  const uint8_t* base() const { return p_; }
  void skip(size_t k) { need(k); i_ += k; }
  int8_t i8() { need(1); return (int8_t)p_[i_++]; }
  int16_t i16() { return (int16_t)get(2); }
  int32_t i32() { return (int32_t)get(4); }
  uint32_t u32() { return (uint32_t)get(4); }
  int64_t i64() { return (int64_t)get(8); }
  std::string str() {
    const int16_t l = i16();
    if (l < 0) return std::string();
    need((size_t)l);
    std::string s(reinterpret_cast<const char*>(p_ + i_), (size_t)l);
    i_ += (size_t)l;
    return s;
  }
  bool nstr(std::string* out) {  // false if null
    const int16_t l = i16();
    if (l < 0) { out->clear(); return false; }
    need((size_t)l);
    out->assign(reinterpret_cast<const char*>(p_ + i_), (size_t)l);
    i_ += (size_t)l;
    return true;
  }
  // nullable bytes -> (offset into base, length); length -1 = null
  std::pair<size_t, int32_t> bytes_ref() {
    const int32_t l = i32();
    if (l < 0) return {i_, -1};
    need((size_t)l);
    const size_t at = i_;
    i_ += (size_t)l;
    return {at, l};
  }
  int32_t array_len() { return i32(); }
  uint64_t uvarint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      need(1);
      const uint8_t b = p_[i_++];
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    throw ProtocolError("varint too long");
  }
  int32_t varint() {
    const uint32_t u = (uint32_t)uvarint();
    return (int32_t)((u >> 1) ^ (~(u & 1) + 1));
  }
  int64_t varlong() {
    const uint64_t u = uvarint();
    return (int64_t)((u >> 1) ^ (~(u & 1) + 1));
  }

 private:
  void need(size_t k) const {
    if (n_ - i_ < k) throw ProtocolError("truncated Kafka message");
  }
  uint64_t get(int k) {
    need((size_t)k);
    uint64_t v = 0;
    for (int j = 0; j < k; ++j) v = (v << 8) | p_[i_ + j];
    i_ += (size_t)k;
    return v;
  }
  const uint8_t* p_;
  size_t n_;
  size_t i_ = 0;
};

// ---- RecordBatch v2 --------------------------------------------------------------------------

constexpr int kBatchHeaderBytes = 61;      // baseOffset .. recordCount
constexpr int kBatchCrcOffset = 17;        // crc field
constexpr int kBatchAttrOffset = 21;       // CRC covers attributes .. end
constexpr int kBatchLengthOffset = 8;
constexpr int kBatchMaxTsOffset = 35;      // maxTimestamp
constexpr int16_t kAttrLogAppendTime = 0x08;  // timestamp type bit of the batch attributes

struct Header {
  std::string key;
  std::string value;
  bool value_null = false;
};

// A record to encode. Null key/value are expressed with the *_null flags.
struct RecordIn {
  std::string_view key;
  bool key_null = true;
  std::string_view value;
  bool value_null = false;
  int64_t timestamp = -1;  // -1: use the batch base timestamp
  const std::vector<Header>* headers = nullptr;
};

// Append one RecordBatch v2 (uncompressed, no producer id) to w. Returns the batch size.
size_t encode_batch(Writer& w, const RecordIn* recs, size_t n, int64_t base_offset,
                    int64_t base_timestamp);

// A decoded record, pointing into the buffer it was decoded from.
struct RecordRef {
  int32_t partition = -1;  // filled by the consumer
  int64_t offset = 0;
  int64_t timestamp = 0;
  int64_t key_off = 0;   // offsets relative to the decoded buffer's base
  int32_t key_len = -1;  // -1 = null
  int64_t value_off = 0;
  int32_t value_len = -1;
  int32_t header_count = 0;
  int64_t headers_off = 0;  // raw header bytes (decode with decode_headers)
  int64_t headers_len = 0;
  // a marker for a record the consumer could not decode (compress.h poison batches): the value
  // is null and the engine applies --on-error with status CORRUPT
  bool poison = false;
};

struct BatchInfo {
  int64_t base_offset = 0;
  int32_t length = 0;       // full batch size in bytes (incl. baseOffset/batchLength)
  int32_t records = 0;
  int64_t base_timestamp = 0;
  int64_t max_timestamp = 0;
  int16_t attributes = 0;
  int32_t last_offset_delta = 0;
};

// Parse the fixed header of the batch at r.ptr(); validates magic (and CRC when check_crc).
// Does not consume. Throws ProtocolError on malformed input.
BatchInfo peek_batch(const uint8_t* p, size_t avail, bool check_crc);

// Decode every record of a records blob [base+off, base+off+len) (a Fetch response's records
// field). Records with offset < min_offset are skipped (a fetch may start mid-batch). A trailing
// partial batch (allowed by the protocol) is ignored. Returns the number of records appended.
// A record batch inside a decoded buffer and the records it contributed to `out`
// (lets a caller defer CRC validation to other threads).
struct BatchSpan {
  size_t off = 0, len = 0;
  size_t first_rec = 0, nrec = 0;
};
// Throws ProtocolError on anything but plain v2 batches (compressed / legacy formats, CRC
// mismatches, malformed records): the consumer then normalises the blob (compress.h) and decodes
// that with honor_poison, which marks the records of poison batches.
size_t decode_records(const uint8_t* base, size_t off, size_t len, int64_t min_offset,
                      bool check_crc, std::vector<RecordRef>& out,
                      std::vector<BatchSpan>* spans = nullptr, bool honor_poison = false);

std::vector<Header> decode_headers(const uint8_t* base, const RecordRef& r);

// SO_SNDBUF / SO_RCVBUF for broker and client sockets: GALE_SOCK_BUF bytes (read once; default
// 8 MiB). 0 leaves the kernel's buffer autotuning on (an explicit size turns it off and is
// clamped to net.core.{w,r}mem_max).
int socket_buffer_bytes();

}  // namespace kafka
}  // namespace gale
