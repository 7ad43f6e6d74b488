// Kafka record compression codecs and message-format conversion.
//
// The reference consumes through storm-kafka 1.2.3 on kafka-clients 0.11 (pom.xml:40-43,56-58,
// 76-77; MainTopology.java:95-106). That stack reads what any ordinary producer writes into a
// topic: RecordBatch v2 with gzip / snappy / lz4 compressed record sections, and the older
// message sets (magic 0 / 1, plain or wrapped in a compressed message). gale's fetch path is
// built around plain v2 batches whose record values point straight into the (pinned, device-
// mirrored) fetch buffer, so anything else is NORMALISED once on the consumer thread: each batch
// that is compressed or in an older format is rewritten as a plain v2 batch (same offsets,
// timestamps, keys, values and headers; fresh CRC32C) and the rest of the pipeline - deferred
// CRC checks, GPU ingest, the JSON parser - sees only the format it already handles.
//
// A batch that cannot be decoded (unknown codec, corrupt compressed data, CRC mismatch, unknown
// magic, a malformed record) never stalls the source: it becomes a POISON batch of null records
// covering its offsets (one per record when the batch header says so, else one), which the
// engine routes through --on-error per record (status CORRUPT) and counts.
//
// Codecs: gzip through zlib (the image's libz); snappy (raw and Kafka's xerial framing) and lz4
// (the LZ4 frame format Kafka uses since message format v1) are decoded and encoded by the
// hand-written block codecs in compress.cpp; zstd (Kafka 2.1+, beyond the reference's 0.11)
// through the system libzstd loaded at run time, when present.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace gale {
namespace kafka {

enum Codec : int { CODEC_NONE = 0, CODEC_GZIP = 1, CODEC_SNAPPY = 2, CODEC_LZ4 = 3, CODEC_ZSTD = 4 };

const char* codec_name(int codec);
int codec_from_name(const std::string& name);  // "none|gzip|snappy|lz4|zstd"; throws otherwise
bool codec_available(int codec);               // zstd: libzstd.so.1 could be loaded

// Decompress `n` bytes, appending to `out` (at most `limit` bytes in total in `out`).
// false (with *err) on corrupt input, an unknown / unavailable codec, or an output over limit.
bool decompress(int codec, const uint8_t* in, size_t n, std::string& out, size_t limit,
                std::string* err);
// Compress (producer side and test fixtures). Throws on an unavailable codec.
std::string compress(int codec, const uint8_t* in, size_t n);

// Individual codecs (exposed for golden-byte tests)
bool snappy_decompress_raw(const uint8_t* in, size_t n, std::string& out, size_t limit);
std::string snappy_compress_raw(const uint8_t* in, size_t n);
bool lz4_decompress_frame(const uint8_t* in, size_t n, std::string& out, size_t limit);
std::string lz4_compress_frame(const uint8_t* in, size_t n);
uint32_t xxh32(const uint8_t* p, size_t n, uint32_t seed);
uint32_t crc32_ieee(const uint8_t* p, size_t n);  // legacy message CRC (zlib crc32)

// ---- record-format conversion ---------------------------------------------------------------

// gale-private attribute bit on a synthesised batch: its records are poison markers (null
// values standing for records that could not be decoded). Only honoured inside regions the
// consumer normalised itself (decode_records(..., honor_poison=true)).
constexpr int16_t kAttrGalePoison = 0x4000;

struct NormalizeStats {
  int64_t converted_batches = 0;  // compressed v2 batches and legacy messages rewritten
  int64_t poison_batches = 0;
  int64_t poison_records = 0;
  // poison records of failed compressed legacy wrappers, whose inner record count cannot be
  // read: the offsets from the previous entry's end to the wrapper's (its last inner record's)
  int64_t poison_unknown_span = 0;
  std::string last_error;
};

// Rewrite a records blob (a Fetch response's records field) as plain v2 batches (see above).
// Batches wholly below min_offset are dropped. Original CRCs of converted batches are always
// verified (their bytes do not survive the conversion); plain v2 batches are copied verbatim
// (CRC left to the caller's deferred check unless check_crc). limit bounds the decompressed bytes
// of the whole call: once spent, the blob ends before the next compressed batch (the caller's
// next fetch resumes there).
std::string normalize_records(const uint8_t* p, size_t len, int64_t min_offset, bool check_crc,
                              size_t limit, NormalizeStats& st);

// A plain v2 batch -> the same batch with its record section compressed (producer
// compression.type). Returns the input unchanged for CODEC_NONE.
std::string compress_batch(const std::string& plain_batch, int codec);

// A legacy message set (magic 0 or 1) of `n` records at offsets base_offset.., optionally wrapped
// in one compressed message (test fixtures; the embedded broker's old message format).
struct LegacyRecord {
  std::string key, value;
  bool key_null = true, value_null = false;
  int64_t timestamp = -1;
};
std::string encode_message_set(int magic, const std::vector<LegacyRecord>& recs,
                               int64_t base_offset, int codec);
// First and last offset of a legacy message set (throws ProtocolError when malformed).
void message_set_offsets(const uint8_t* p, size_t len, int64_t* first, int64_t* last);

}  // namespace kafka
}  // namespace gale
