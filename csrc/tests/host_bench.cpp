// Host codec micro-benchmark: CRC32C (Kafka record-batch checksum) and the InstObj envelope scan
// over synthetic CIFAR-shaped records, single thread. Reports GB/s per core for each pass.
//
// usage: host_bench [iterations=200]
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <random>
#include <string>
#include <vector>

#include "../codec/json_codec.h"
#include "../kafka/wire.h"

using namespace gale;

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  std::vector<std::string> recs(64);
  size_t total = 0;
  for (auto& r : recs) {
    std::vector<float> x(32 * 32 * 3);
    for (float& v : x) v = u(rng);
    codec::encode_instances(x.data(), 1, 32, 32, 3, r);
    total += r.size();
  }
  std::string blob;
  for (auto& r : recs) blob += r;
  uint32_t acc = 0;
  double t0 = now();
  for (int i = 0; i < iters; ++i)
    acc ^= kafka::crc32c(reinterpret_cast<const uint8_t*>(blob.data()), blob.size());
  double t1 = now();
  int64_t imgs = 0;
  for (int i = 0; i < iters; ++i)
    for (auto& r : recs)
      imgs += codec::scan_instances(reinterpret_cast<const uint8_t*>(r.data()), r.size(), 32, 32,
                                    3).images;
  double t2 = now();
  const double gb = (double)total * iters / 1e9;
  printf("{\"record_bytes\": %.0f, \"crc32c_GBps\": %.2f, \"scan_GBps\": %.2f, \"chk\": %u, "
         "\"imgs\": %lld}\n",
         (double)total / recs.size(), gb / (t1 - t0), gb / (t2 - t1), acc, (long long)imgs);
  return 0;
}
