// Host side of the InstObj / PredObj JSON contract.
//
// Input  (InstObj, /root/reference/src/main/java/dke/model/data/InstObj.java:8):
//     {"instances": float[N][H][W][C]}
// Output (PredObj, /root/reference/src/main/java/dke/model/data/PredObj.java:9):
//     {"predictions": float[N][classes]}
//
// The reference decodes with Jackson on the bolt thread (InferenceBolt.java:76) and re-encodes
// with a fresh ObjectMapper per tuple (:90-91). gale splits decoding in two:
//   * scan_instances() — a cheap AVX2 pass on the consumer thread: validates the envelope
//     (exactly one key, "instances", like Jackson's FAIL_ON_UNKNOWN_PROPERTIES) and derives N
//     from the '[' count of a rank-4 rectangular array (1 + N + N*H + N*H*W opening brackets);
//   * the float parsing and the full per-token structural check run on the GPU
//     (csrc/kernels/json_parse.hip), reading the staged bytes straight from pinned memory.
// parse_instances_host() is the complete host decoder (CPU stub replica, tests, diagnostics).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <cstdint>

#include <string>
#include <utility>
#include <vector>

namespace gale {
namespace codec {

enum Status : int {
  OK = 0,
  BAD_ENVELOPE = 1,   // not {"instances": [...]} (syntax error, not an object, no array)
  UNKNOWN_KEY = 2,    // a top-level key other than "instances" (Jackson FAIL_ON_UNKNOWN_PROPERTIES)
  BAD_SHAPE = 3,      // not rank 4, ragged, or per-image shape != model H x W x C
  EMPTY = 4,          // zero images
  BAD_NUMBER = 5,     // malformed JSON number / non-number element
  NULL_INSTANCES = 6, // "instances": null
  TOO_LARGE = 7,      // more images than the caller allows
  CORRUPT = 8,        // the Kafka batch holding the record could not be decoded (unknown codec,
                      // corrupt compressed data, CRC mismatch; kafka/compress.h poison records)
};
constexpr int kStatusCount = 9;

const char* status_name(int s);

struct Scan {
  int status = OK;
  int64_t arr_off = 0;  // byte offset of the outer '[' of the instances array
  int64_t arr_len = 0;  // bytes up to and including the matching ']'
  int images = 0;       // N
};

// Bounded envelope check: the {"instances": ... } prefix and the "] }" suffix only (reads a
// few bytes at each end; the array's interior, its image count and any key hidden inside it are
// left to the device ingest / parser). images stays 0.
// head_limit / tail_limit: only the first / last that many bytes of the value are read (a sparse
// host copy holds nothing else, kafka/fetch_framing.h); an envelope reaching beyond them is
// rejected as BAD_ENVELOPE (documented limit: <= ~200 bytes of whitespace around it).
Scan scan_envelope(const uint8_t* p, size_t n, size_t head_limit = SIZE_MAX,
                   size_t tail_limit = SIZE_MAX);

// Envelope validation + image count (the per-number work is left to the GPU parser).
Scan scan_instances(const uint8_t* p, size_t n, int H, int W, int C);

// Byte spans [begin, end) of the top-level elements (the images) of the instances array
// `arr[0..len)` (its outer '[' ... ']'), for splitting a record with more images than one
// micro-batch holds. false when the bracket structure is broken.
bool split_instances(const uint8_t* arr, size_t len,
                     std::vector<std::pair<uint32_t, uint32_t>>& spans);

// Full host decoder: validates structure and parses every number into out[N*H*W*C].
// Returns the status; *images receives N. out may be null to validate only.
int parse_instances_host(const uint8_t* p, size_t n, int H, int W, int C, float* out,
                         int max_images, int* images);

// Java Float.toString formatting (what Jackson emits for float[]): shortest digits
// that round-trip, decimal for 1e-3 <= |v| < 1e7 ("0.125", "3.0"), else "1.0E-5". Returns length.
int format_float_java(float v, char* out);
// Java 8 Float.toString (FloatingDecimal's free-format digit loop, csrc/codec/java8_float.cpp):
// the reference's runtime; it sometimes prints more digits than the shortest form. Parity with
// a real Java 8 is unpinned (no JVM here).
int format_float_java8(float v, char* out);

// {"predictions":[[p00,p01,...],[p10,...]]} (Jackson compact). json_string=true wraps the
// document in a JSON string literal, which is what spring-kafka's JsonSerializer does to the
// already-serialized String value (MainTopology.java:115).
// java8: Java 8 Float.toString digits (format_float_java8) instead of the JDK 19 rule
void encode_predictions(const float* probs, int n, int classes, bool json_string,
                        std::string& out, bool java8 = false);
// Same output from pre-formatted values: text16 holds n * classes 16-byte slots (characters,
// length in byte 15; format_floats_java in csrc/kernels/format.hip).
void encode_predictions_text(const uint8_t* text16, int n, int classes, bool json_string,
                             std::string& out);

// {"instances":[[[[x,...]]]]} with Java Float.toString numbers: the load generator's encoder
// (the reference's producers are external; this is the shape README.md:22-27 documents).
void encode_instances(const float* x, int n, int H, int W, int C, std::string& out);

// {"error":"<status>","detail":"..."} record used by --on-error error-json.
void encode_error(int status, const char* detail, bool json_string, std::string& out);

}  // namespace codec
}  // namespace gale
