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
//   4. bounce receive: four consumer threads at once receive through the bounce tap
//      (runtime/pack_tap.h: L2 window, framing walker, nibble packing) over plain, lz4- and
//      gzip-compressed and legacy magic-1 batches; every value restored from the packed stream
//      equals what was appended
// The reference's only concurrency primitive is `synchronized (collector)` in the producer
// callback (KafkaBolt.java:129-143); gale's queues and callbacks are what this exercises.
//
// usage: engine_stress [records=4000]; exit code 0 = all checks passed.
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <string>
#include <vector>

#include <thread>

#include "../codec/json_codec.h"
#include "../codec/text_pack.h"
#include "../kafka/broker.h"
#include "../kafka/client.h"
#include "../kafka/compress.h"
#include "../runtime/engine.h"
#include "../runtime/pack_tap.h"

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

// Scenario 4: the values appended to partition p of `topic`, by offset.
std::vector<std::vector<std::string>> preload_formats(kafka::Broker& b, const std::string& topic,
                                                      int parts, int per_part, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  std::vector<std::vector<std::string>> vals((size_t)parts);
  for (int p = 0; p < parts; ++p) {
    int k = 0;
    while (k < per_part) {
      const int n = std::min(per_part - k, 5 + (int)(rng() % 20));
      std::vector<std::string> v;
      for (int i = 0; i < n; ++i) {
        const int imgs = 1 + (int)(rng() % 2);
        std::vector<float> x((size_t)imgs * 32 * 32 * 3);  // ~35 KB of text per image
        for (float& f : x) f = u(rng);
        std::string sv;
        codec::encode_instances(x.data(), imgs, 32, 32, 3, sv);
        v.push_back(std::move(sv));
      }
      // plain, lz4, gzip, legacy magic 1 (partition 0 plain only: sparse fetches throughout)
      const int kind = p == 0 ? 0 : (int)(rng() % 4);
      if (kind == 3) {
        std::vector<kafka::LegacyRecord> lr(v.size());
        for (size_t i = 0; i < v.size(); ++i) {
          lr[i].value = v[i];
          lr[i].timestamp = 1000 + (int64_t)i;
        }
        b.append_legacy(topic, p, 1, lr, kafka::CODEC_NONE);
      } else {
        std::vector<kafka::RecordIn> recs(v.size());
        for (size_t i = 0; i < v.size(); ++i) recs[i].value = v[i];
        kafka::Writer w;
        kafka::encode_batch(w, recs.data(), recs.size(), 0, 1000);
        const int codec = kind == 1 ? kafka::CODEC_LZ4 : kind == 2 ? kafka::CODEC_GZIP
                                                                   : kafka::CODEC_NONE;
        b.append_shared(topic, p,
                        std::make_shared<const std::string>(kafka::compress_batch(w.buf, codec)));
      }
      for (auto& sv : v) vals[(size_t)p].push_back(std::move(sv));
      k += n;
    }
  }
  return vals;
}

void consume_bounce(int port, const std::string& topic, int p,
                    const std::vector<std::string>& want, int* bad, int64_t* sparse) {
  kafka::ConsumerConfig cc;
  cc.bootstrap = "127.0.0.1:" + std::to_string(port);
  cc.max_wait_ms = 20;
  cc.fetch_max_bytes = 1 << 20;
  cc.partition_max_bytes = 600 << 10;
  cc.check_crcs = false;  // (the host copy of a bounce-received body is sparse)
  const size_t chunk = codec::pack_layout_bytes((size_t)cc.fetch_max_bytes + (1 << 20)) + 4096;
  kafka::Consumer cons(cc, [chunk](size_t n) { return kafka::heap_alloc(std::max(n, chunk)); });
  cons.set_recv_tap(std::make_shared<BouncePackTap>(
      chunk, [](const uint8_t*) { return true; }, 1, (size_t)(8 + 8 * p) << 10));
  cons.assign(topic, {p});
  cons.seek_to("earliest");
  size_t got = 0;
  for (int round = 0; round < 4000 && got < want.size(); ++round) {
    for (kafka::Fetched& f : cons.poll()) {
      if (f.sparse) ++*sparse;
      f.restore();
      for (const kafka::RecordRef& r : f.records) {
        const std::string v(reinterpret_cast<const char*>(f.buf.get()) + r.value_off,
                            r.value_len > 0 ? (size_t)r.value_len : 0);
        if (r.offset < 0 || (size_t)r.offset >= want.size() || r.poison ||
            v != want[(size_t)r.offset])
          ++*bad;
        ++got;
      }
    }
  }
  if (got != want.size()) ++*bad;
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
  if (codec::text_pack_fast()) {  // 4. bounce receive over plain / compressed / legacy batches
    const int parts = 4;
    broker.create_topic("bounce", parts);
    const auto want = preload_formats(broker, "bounce", parts, std::max(40, n / 40), 11);
    std::vector<int> bad((size_t)parts, 0);
    std::vector<int64_t> sparse((size_t)parts, 0);
    std::vector<std::thread> ts;
    for (int p = 0; p < parts; ++p)
      ts.emplace_back(consume_bounce, broker.port(), "bounce", p, std::cref(want[(size_t)p]),
                      &bad[(size_t)p], &sparse[(size_t)p]);
    for (auto& t : ts) t.join();
    int64_t nbad = 0, nsparse = 0;
    for (int p = 0; p < parts; ++p) {
      nbad += bad[(size_t)p];
      nsparse += sparse[(size_t)p];
    }
    CHECK(nbad == 0, "%lld bounce-received values differ from what was appended",
          (long long)nbad);
    CHECK(nsparse > 0, "no fetch was received sparse");
    fprintf(stderr, "[stress] bounce receive: %lld sparse fetches, values OK\n",
            (long long)nsparse);
  }
  broker.stop();
  if (failures) {
    fprintf(stderr, "[stress] %d check(s) FAILED\n", failures);
    return 1;
  }
  fprintf(stderr, "[stress] all checks passed\n");
  return 0;
}
