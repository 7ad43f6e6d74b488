// Host-pipeline stress driver for the sanitizer builds ("a C++ build with
// -fsanitize=thread / address for host queues, run in CI on CPU").
//
// Runs the whole serving engine with CPU stub replicas against the embedded Kafka broker, so
// every host thread of the topology is live at once: consumer (source) threads, CRC32C/scan
// decode workers, the micro-batcher, replica workers, the watchdog, async producers (sink) and
// the broker's connection threads. Scenarios:
//   1. clean run: N records over 4 partitions, 3 replicas -> exactly N outputs, offsets committed
//   2. faults:   a replica crash (its in-flight batches re-queue to the survivors), injected
//                parse errors and producer failures -> every record still accounted for
//   3. stop while busy: Engine::stop() with records still queued (drain + commit path)
// The reference's only concurrency primitive is `synchronized (collector)` in the producer
// callback (KafkaBolt.java:129-143); gale's queues and callbacks are what this exercises.
//
// usage: engine_stress [records=4000]; exit code 0 = all checks passed.
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <string>
#include <vector>

#include "../codec/json_codec.h"
#include "../kafka/broker.h"
#include "../runtime/engine.h"

using namespace gale;

namespace {

int failures = 0;
#define CHECK(cond, ...)                            \
  do {                                              \
    if (!(cond)) {                                  \
      fprintf(stderr, "CHECK failed: %s: ", #cond); \
      fprintf(stderr, __VA_ARGS__);                 \
      fprintf(stderr, "\n");                        \
      ++failures;                                   \
    }                                               \
  } while (0)

constexpr int H = 4, W = 4, C = 3, CLASSES = 10;

void preload(kafka::Broker& b, const std::string& topic, int parts, int n, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  std::vector<std::string> vals;
  for (int i = 0; i < n; ++i) {
    const int imgs = 1 + (int)(rng() % 3);
    std::vector<float> x((size_t)imgs * H * W * C);
    for (float& v : x) v = u(rng);
    std::string s;
    codec::encode_instances(x.data(), imgs, H, W, C, s);
    vals.push_back(std::move(s));
  }
  for (int p = 0; p < parts; ++p) {
    std::vector<kafka::RecordIn> recs;
    for (int i = p; i < n; i += parts) {
      kafka::RecordIn r;
      r.value = vals[(size_t)i];
      recs.push_back(r);
      if (recs.size() == 50) {
        b.append(topic, p, recs);
        recs.clear();
      }
    }
    if (!recs.empty()) b.append(topic, p, recs);
  }
}

int64_t count_out(kafka::Broker& b, const std::string& topic) {
  int64_t n = 0;
  for (int p = 0; p < b.partitions(topic); ++p) n += b.log_end(topic, p) - b.log_start(topic, p);
  return n;
}

EngineConfig base_cfg(int port, const std::string& in, const std::string& out) {
  EngineConfig c;
  c.bootstrap = "127.0.0.1:" + std::to_string(port);
  c.input_topic = in;
  c.output_topic = out;
  c.group_id = "stress";
  c.start_offset = "earliest";
  c.source_parallelism = 2;
  c.decode_threads = 2;
  c.sink_parallelism = 2;
  c.H = H; c.W = W; c.C = C; c.classes = CLASSES;
  c.max_batch = 32;
  c.max_wait_us = 300;
  c.queue_depth = 256;
  c.commit_interval_ms = 50;
  c.fetch_max_wait_ms = 5;
  return c;
}

void add_stubs(Engine& e, int n, int delay_us) {
  for (int i = 0; i < n; ++i)
    e.add_replica(std::make_shared<StubReplica>(H, W, C, CLASSES, 32, delay_us, true));
}

}  // namespace

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4000;
  kafka::BrokerConfig bc;
  kafka::Broker broker(bc);
  broker.start();
  broker.create_topic("in", 4);
  broker.create_topic("out", 2);
  broker.create_topic("out2", 2);
  broker.create_topic("out3", 1);
  preload(broker, "in", 4, n, 7);

  {  // 1. clean run
    EngineConfig c = base_cfg(broker.port(), "in", "out");
    c.max_records = n;
    Engine e(c);
    add_stubs(e, 3, 0);
    e.start();
    const bool done = e.wait(120000);
    e.stop();
    CHECK(done, "clean run timed out at %lld/%d", (long long)e.completed(), n);
    CHECK(e.completed() == n, "completed %lld != %d", (long long)e.completed(), n);
    CHECK(count_out(broker, "out") == n, "out records %lld != %d",
          (long long)count_out(broker, "out"), n);
    int64_t committed = 0;
    for (int p = 0; p < 4; ++p) committed += broker.committed("stress", "in", p);
    CHECK(committed == n, "committed %lld != %d", (long long)committed, n);
    fprintf(stderr, "[stress] clean run: %lld records OK\n", (long long)e.completed());
  }
  {  // 2. faults: replica crash + parse errors + producer failures (on_error=error-json)
    EngineConfig c = base_cfg(broker.port(), "in", "out2");
    c.group_id = "stress-faults";
    c.max_records = n;
    c.on_error = "error-json";
    c.fault = "replica_crash@5,parse_error@0.02,producer_fail@0.01";
    Engine e(c);
    add_stubs(e, 3, 50);
    e.start();
    const bool done = e.wait(120000);
    e.stop();
    const auto st = e.stats();
    CHECK(done, "fault run timed out at %lld/%d", (long long)e.completed(), n);
    CHECK(st.at("replica_failures") == 1, "replica_failures %g", st.at("replica_failures"));
    CHECK(st.at("errors") > 0, "no injected parse errors surfaced");
    fprintf(stderr, "[stress] fault run: completed %lld, requeued %g, errors %g, produce "
            "failures %g\n", (long long)e.completed(), st.at("requeued"), st.at("errors"),
            st.at("produce_failures"));
  }
  {  // 3. stop while records are still queued
    EngineConfig c = base_cfg(broker.port(), "in", "out3");
    c.group_id = "stress-stop";
    Engine e(c);
    add_stubs(e, 2, 2000);
    e.start();
    while (e.completed() < 64) std::this_thread::sleep_for(std::chrono::milliseconds(2));
    e.stop();
    CHECK(!e.running(), "engine still running after stop()");
    fprintf(stderr, "[stress] stop-while-busy: completed %lld before stop\n",
            (long long)e.completed());
  }
  broker.stop();
  if (failures) {
    fprintf(stderr, "[stress] %d check(s) FAILED\n", failures);
    return 1;
  }
  fprintf(stderr, "[stress] all checks passed\n");
  return 0;
}
