// DRAM antagonist for the N = 8 host projection (profiles/r5_host_budget.txt
// §4): on the one-GPU box, run next to bench.py and add the DRAM traffic that the other ranks of
// a socket would add, or - the control - burn the same CPU time with no memory traffic.
//
//   dram_antagonist --mode stream|burn --threads T --seconds S [--cpus LIST] [--buffer-mb M]
//                   [--report FILE]
//
// stream: every thread copies its own buffer (M MiB, far beyond the L3) onto a second one with
//   AVX2 loads and non-temporal stores - a read stream plus a write stream that bypasses the
//   caches, like the engine's receive copy + packed-stream stores. Each thread runs flat out
//   (one core), so T sets the level of extra DRAM traffic; the achieved GB/s (bytes read +
//   bytes written) is reported once a second.
// burn: every thread spins on register arithmetic: the same CPU time as `stream` with the same
//   T, no memory traffic (the control that separates CPU contention from DRAM contention).
// Threads are pinned to --cpus (round robin; the GPU's NUMA node in practice) and first-touch
// their buffers there, so the traffic lands on that socket's memory controllers.
// Reports JSON lines {"t": s, "gbs": x, "threads": T, "mode": m} to --report (default stdout).
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

static std::atomic<bool> g_stop{false};
static std::atomic<uint64_t> g_bytes{0};

static double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void on_signal(int) { g_stop = true; }

static std::vector<int> parse_cpus(const std::string& s) {
  std::vector<int> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string part = s.substr(i, j - i);
    const size_t d = part.find('-');
    if (!part.empty()) {
      if (d == std::string::npos) {
        out.push_back(atoi(part.c_str()));
      } else {
        const int a = atoi(part.substr(0, d).c_str()), b = atoi(part.substr(d + 1).c_str());
        for (int c = a; c <= b; ++c) out.push_back(c);
      }
    }
    i = j + 1;
  }
  return out;
}

static void pin(int cpu) {
  if (cpu < 0) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  sched_setaffinity(0, sizeof(set), &set);
}

static void stream_thread(int cpu, size_t bytes) {
  pin(cpu);
  uint8_t* src = static_cast<uint8_t*>(aligned_alloc(64, bytes));
  uint8_t* dst = static_cast<uint8_t*>(aligned_alloc(64, bytes));
  if (!src || !dst) {
    fprintf(stderr, "dram_antagonist: allocation of 2 x %zu bytes failed\n", bytes);
    return;
  }
  memset(src, 1, bytes);  // first touch on this thread's CPU
  memset(dst, 2, bytes);
  const size_t step = 1 << 20;
  while (!g_stop.load(std::memory_order_relaxed)) {
    for (size_t off = 0; off + step <= bytes && !g_stop.load(std::memory_order_relaxed);
         off += step) {
      const __m256i* s = reinterpret_cast<const __m256i*>(src + off);
      __m256i* d = reinterpret_cast<__m256i*>(dst + off);
      for (size_t k = 0; k < step / 32; k += 4) {
        const __m256i a = _mm256_load_si256(s + k), b = _mm256_load_si256(s + k + 1);
        const __m256i c = _mm256_load_si256(s + k + 2), e = _mm256_load_si256(s + k + 3);
        _mm256_stream_si256(d + k, a);
        _mm256_stream_si256(d + k + 1, b);
        _mm256_stream_si256(d + k + 2, c);
        _mm256_stream_si256(d + k + 3, e);
      }
      g_bytes.fetch_add(2 * step, std::memory_order_relaxed);
    }
    _mm_sfence();
  }
  free(src);
  free(dst);
}

static void burn_thread(int cpu) {
  pin(cpu);
  uint64_t x = 0x9e3779b97f4a7c15ull + (uint64_t)cpu, acc = 0;
  while (!g_stop.load(std::memory_order_relaxed)) {
    for (int i = 0; i < 1 << 16; ++i) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      acc += x;
    }
  }
  if (acc == 42) fprintf(stderr, "!");  // (keeps the loop)
}

int main(int argc, char** argv) {
  std::string mode = "stream", cpus, report;
  int threads = 1;
  double seconds = 60;
  size_t buffer_mb = 512;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i], v = argv[i + 1];
    if (k == "--mode") mode = v;
    else if (k == "--threads") threads = atoi(v.c_str());
    else if (k == "--seconds") seconds = atof(v.c_str());
    else if (k == "--cpus") cpus = v;
    else if (k == "--buffer-mb") buffer_mb = (size_t)atol(v.c_str());
    else if (k == "--report") report = v;
    else {
      fprintf(stderr, "dram_antagonist: unknown option %s\n", k.c_str());
      return 2;
    }
  }
  if ((mode != "stream" && mode != "burn") || threads < 0) {
    fprintf(stderr, "dram_antagonist: --mode stream|burn, --threads >= 0\n");
    return 2;
  }
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  FILE* out = report.empty() ? stdout : fopen(report.c_str(), "w");
  if (!out) {
    perror("dram_antagonist: report");
    return 2;
  }
  const std::vector<int> cl = parse_cpus(cpus);
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    const int cpu = cl.empty() ? -1 : cl[(size_t)t % cl.size()];
    if (mode == "stream") ts.emplace_back(stream_thread, cpu, buffer_mb << 20);
    else ts.emplace_back(burn_thread, cpu);
  }
  const double t0 = now_s();
  double tl = t0;
  uint64_t bl = 0;
  while (!g_stop && now_s() - t0 < seconds) {
    struct timespec ts100 = {0, 100 * 1000 * 1000};
    nanosleep(&ts100, nullptr);
    const double t = now_s();
    if (t - tl >= 1.0) {
      const uint64_t b = g_bytes.load();
      fprintf(out, "{\"t\": %.2f, \"gbs\": %.2f, \"threads\": %d, \"mode\": \"%s\"}\n", t - t0,
              (double)(b - bl) / (t - tl) / 1e9, threads, mode.c_str());
      fflush(out);
      tl = t;
      bl = b;
    }
  }
  g_stop = true;
  for (auto& t : ts) t.join();
  if (out != stdout) fclose(out);
  return 0;
}
