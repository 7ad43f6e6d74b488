// Lock-free latency histograms and counters for the serving engine.
//
// The reference's only observability is Storm UI (per-component execute latency / capacity,
// E4) and the KafkaSpout offset metrics (E1). gale records per-stage latencies (queue wait,
// device time, end-to-end from fetch to produce-ack and from the record's CreateTime) in
// log-linear histograms (8 sub-buckets per power of two: <= 12.5 % relative error), plus
// throughput / error counters, exported as a dict to the Python reporter (gale/metrics.py).
#pragma once
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <vector>

namespace gale {

inline int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
inline int64_t wall_ms_now() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

class Histogram {
 public:
  static constexpr int kBuckets = 16 + 44 * 8;
  Histogram() { reset(); }
  void reset() {
    for (auto& b : b_) b.store(0, std::memory_order_relaxed);
    count_.store(0);
    sum_.store(0);
    max_.store(0);
  }
  void add(int64_t v) {
    if (v < 0) v = 0;
    b_[bucket(v)].fetch_add(1, std::memory_order_relaxed);
    count_.fetch_add(1, std::memory_order_relaxed);
    sum_.fetch_add(v, std::memory_order_relaxed);
    int64_t m = max_.load(std::memory_order_relaxed);
    while (v > m && !max_.compare_exchange_weak(m, v, std::memory_order_relaxed)) {
    }
  }
  int64_t count() const { return count_.load(); }
  double mean() const {
    const int64_t c = count_.load();
    return c ? (double)sum_.load() / (double)c : 0.0;
  }
  int64_t max() const { return max_.load(); }
  // value at quantile q (bucket midpoint)
  double quantile(double q) const {
    const int64_t c = count_.load();
    if (!c) return 0.0;
    const int64_t target = (int64_t)(q * (double)(c - 1)) + 1;
    int64_t acc = 0;
    for (int i = 0; i < kBuckets; ++i) {
      acc += b_[i].load(std::memory_order_relaxed);
      if (acc >= target) {
        const double m = mid(i), mx = (double)max_.load();
        return m < mx ? m : mx;
      }
    }
    return (double)max_.load();
  }

 private:
  static int bucket(int64_t v) {
    if (v < 16) return (int)v;
    const int e = 63 - __builtin_clzll((uint64_t)v);
    const int m = (int)((v >> (e - 3)) & 7);
    const int b = 16 + (e - 4) * 8 + m;
    return b < kBuckets ? b : kBuckets - 1;
  }
  static double mid(int b) {
    if (b < 16) return (double)b;
    const int e = (b - 16) / 8 + 4, m = (b - 16) % 8;
    const double lo = (double)((8 + m) * (1ll << (e - 3)));
    return lo + (double)(1ll << (e - 3)) * 0.5;
  }
  std::atomic<int64_t> b_[kBuckets];
  std::atomic<int64_t> count_, sum_, max_;
};

}  // namespace gale
