// Lock-free latency histograms and counters for the serving engine.
//
// The reference's only observability is Storm UI (per-component execute latency / capacity,
// E4) and the KafkaSpout offset metrics (E1). gale records per-stage latencies (queue wait,
// device time, end-to-end from fetch to produce-ack and from the record's CreateTime) in
// log-linear histograms (32 sub-buckets per power of two: <= 3.1 % bucket width, quantiles
// interpolated inside the bucket), plus
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
  static constexpr int kSub = 32;  // sub-buckets per power of two (values < kSub are exact)
  static constexpr int kBuckets = kSub + (64 - 5) * kSub;
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
  // value at quantile q: the rank's position inside its bucket, linearly interpolated
  double quantile(double q) const {
    const int64_t c = count_.load();
    if (!c) return 0.0;
    const int64_t target = (int64_t)(q * (double)(c - 1)) + 1;
    int64_t acc = 0;
    for (int i = 0; i < kBuckets; ++i) {
      const int64_t n = b_[i].load(std::memory_order_relaxed);
      if (acc + n >= target) {
        double lo, w;
        range(i, lo, w);
        const double v = w <= 1.0 ? lo : lo + w * ((double)(target - acc) - 0.5) / (double)n;
        const double mx = (double)max_.load();
        return v < mx ? v : mx;
      }
      acc += n;
    }
    return (double)max_.load();
  }

 private:
  static int bucket(int64_t v) {
    if (v < kSub) return (int)v;
    const int e = 63 - __builtin_clzll((uint64_t)v);  // >= 5
    const int m = (int)((v >> (e - 5)) & (kSub - 1));
    const int b = kSub + (e - 5) * kSub + m;
    return b < kBuckets ? b : kBuckets - 1;
  }
  // bucket b covers [lo, lo + w)
  static void range(int b, double& lo, double& w) {
    if (b < kSub) {
      lo = (double)b;
      w = 1.0;
      return;
    }
    const int e = (b - kSub) / kSub + 5, m = (b - kSub) % kSub;
    w = (double)(1ll << (e - 5));
    lo = (double)(kSub + m) * w;
  }
  std::atomic<int64_t> b_[kBuckets];
  std::atomic<int64_t> count_, sum_, max_;
};

}  // namespace gale
