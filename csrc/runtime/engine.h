// The gale serving engine: Kafka source -> micro-batcher -> model replicas -> Kafka sink.
//
// This is the whole Storm topology of the reference (MainTopology.java:52-92) collapsed into one
// process per GPU with native threads and bounded in-memory queues instead of Storm executors,
// Netty/Kryo tuple transport and ackers:
//
//   source threads  (KafkaSpout x KAFKA_SPOUT_PARAL, MainTopology.java:26,61)
//      Consumer.poll -> codec::scan_instances (envelope check + image count, AVX2)
//      -> Batcher (bounded: backpressure to the consumer)
//   replica workers (InferenceBolt x INFERENCE_BOLT_PARAL, :27,62; shuffle grouping :62 -> pull)
//      Batcher.take: continuous micro-batching (max_batch images or max_wait_us since the oldest
//      record; an idle replica pulls first, which is least-loaded dispatch) -> Replica.submit /
//      wait (depth-deep pipelining) -> encode {"predictions": ...} per record
//   sink            (KafkaBolt x KAFKA_BOLT_PARAL, :28,63)
//      Producer.send async | sync | fire-and-forget (KafkaBolt.java:129-155), acks (:113)
//
// Delivery: offsets of a partition are committed up to the first record whose output has not
// been acknowledged. delivery = "at-most-once" (the reference, SURVEY.md §3.4: KafkaBolt fails
// an unanchored tuple and nothing replays it, KafkaBolt.java:133-137,160-162) completes a record
// whose produce failed, so the commit moves past it. delivery = "at-least-once" never does: the
// producer retries it (producer_retries, retry_backoff_ms, delivery_timeout_ms) and when the
// retries are spent the record stays pending - the commit cannot pass it - and the engine reports
// delivery_failed, on which the rank exits non-zero and is respawned from the committed offsets
// (gale/topology.py, gale/supervisor.py).
// Failure handling: a replica that throws or exceeds the watchdog deadline is
// marked dead and its in-flight batches are re-queued to the surviving replicas; malformed input
// follows on_error = null (reference: a null record, InferenceBolt.java:92-99) | error-json |
// drop.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <utility>
#include <thread>
#include <vector>

#include "../kafka/client.h"
#include "ingest.h"
#include "metrics.h"
#include "pinned_pool.h"
#include "replica.h"

namespace gale {

struct EngineConfig {
  // source (R4, E1)
  std::string bootstrap = "127.0.0.1:9092";
  std::string input_topic, output_topic;
  int output_partition = -1;       // -1: the producer's partitioner; >= 0: this partition
  int64_t producer_buffer_bytes = 32ll << 20;  // per sink producer (Kafka buffer.memory)
  int64_t producer_request_bytes = 1 << 20;    // per produce request (Kafka max.request.size)
  std::string group_id;            // offsets committed under this group (empty: no commits)
  std::string client_id = "gale";
  std::vector<int> partitions;     // empty = every partition of input_topic
  int source_parallelism = 2;      // KAFKA_SPOUT_PARAL (MainTopology.java:26)
  std::string start_offset = "latest";  // latest | earliest | committed
  // where start_offset=committed (and group-managed partitions) start when the group has no
  // committed offset for a partition (Kafka auto.offset.reset): latest | earliest
  std::string auto_offset_reset = "latest";
  int fetch_max_wait_ms = 20;
  int fetch_min_bytes = 1;         // Kafka fetch.min.bytes: a long-poll returns once this much
                                   // is available (or fetch_max_wait_ms passed)
  int fetch_max_bytes = 16 << 20;
  int partition_max_bytes = 8 << 20;
  bool check_crcs = true;
  int decode_threads = 2;          // CRC32C + envelope scan workers (0 = on the source thread)
  int64_t pinned_fetch_bytes = 4ll << 30;  // pinned fetch-buffer budget (GPU replicas only)
  // GPU ingest: sources nibble-pack fetch bodies while receiving them (pack_tap.h) and the text
  // crosses the host link packed (csrc/codec/text_pack.h)
  bool text_pack = false;
  // with text_pack: receive each fetch body through a cache-resident window and keep only its
  // packed text + a sparse framing copy in the pinned chunk (BouncePackTap, pack_tap.h); false:
  // the body lands in the chunk whole and is packed behind it (PackTap)
  bool text_pack_bounce = true;
  // GPU ingest also parses each fetch's records into an fp32 image arena behind its device
  // mirror (Ingest::run arena): the replicas' batch step then runs the forward only, reading
  // the images through a pointer table (whole-network plans; others ignore the arena)
  bool ingest_parse = false;
  int text_pack_window_kb = 256;   // the bounce receive window per source (L2 resident)
  // consumers' receive low-water mark (kafka::ClientConfig::recv_lowat), bytes; 0 = off,
  // < 0 = auto (the bounce window when the bounce receive is on, else off)
  int recv_lowat = -1;
  int commit_interval_ms = 2000;   // storm-kafka's ZK commit period
  // consumer-group membership (elastic DP, kafka::GroupMember): the input partitions are shared
  // by every engine of group_id; a member that dies or leaves has its partitions moved to the
  // survivors, which resume them from the committed offsets (at-least-once across the move)
  bool group_membership = false;
  int session_timeout_ms = 6000;
  int rebalance_timeout_ms = 8000;
  int heartbeat_interval_ms = 500;
  std::string assignor = "range";  // range | roundrobin | load-aware
  // load-aware assignor: every member reports its serving capacity (full micro-batches per busy
  // replica second, in images/s) and owned partitions in JoinGroup; a member whose own lag stays above
  // lag_rebalance_records and keeps growing for a second triggers a rebalance (at most once
  // per rebalance_cooldown_ms), so a slow GPU sheds partitions to faster ones
  int lag_rebalance_records = 0;   // 0 = 8 x max_batch x replicas
  int rebalance_cooldown_ms = 10000;
  // NUMA placement: device -> CPUs for the threads serving it (replica workers, the sources of
  // its locality slot); empty = no pinning
  std::map<int, std::vector<int>> device_cpus;
  // sink (R5, R9, E7-E9)
  int sink_parallelism = 2;        // KAFKA_BOLT_PARAL (MainTopology.java:28)
  int acks = 1;                    // MainTopology.java:113
  std::string sink_mode = "async"; // async | sync | fire-and-forget (KafkaBolt.java:186-197)
  std::string delivery = "at-most-once";  // at-most-once | at-least-once (header comment)
  int producer_retries = 0;        // kafka-clients retries (0.11 default 0)
  int retry_backoff_ms = 100;      // retry.backoff.ms
  int delivery_timeout_ms = 120000;  // delivery.timeout.ms: bound on a record's retries
  int linger_ms = 0;
  int batch_size = 1 << 20;
  std::string compression = "none";  // sink compression.type (kafka/compress.h codecs)
  std::string value_format = "json";  // json | json-string (spring JsonSerializer, E8)
  // prediction digits: "jdk19" (shortest, also on the GPU) | "java8" (the reference runtime's
  // Float.toString, host-formatted; codec::format_float_java8)
  std::string float_format = "jdk19";
  bool type_id_header = false;     // __TypeId__: java.lang.String header (E8)
  std::string on_error = "null";   // null | error-json | drop
  // output record key: "none" = unkeyed (the reference, E9: FieldNameBasedTupleToKafkaMapper
  // finds no "key" field) | "input" = the input record's key (request/response correlation)
  std::string output_key = "none";
  // model I/O contract (InstObj [N][H][W][C] -> PredObj [N][classes])
  int H = 32, W = 32, C = 3, classes = 10;
  // batching (P7)
  int max_batch = 256;             // images per micro-batch (<= every replica's max)
  int max_wait_us = 2000;          // latency bound on batch formation
  // latency-SLO mode (BASELINE config 5): > 0 = a controller adapts the effective batch size and
  // wait bound every 100 ms from the window's end-to-end p99 (AIMD, Clipper-style adaptive
  // batching): back off while p99 exceeds the target, grow while well under it; when p99 is
  // over the target because records queue up (offered load above capacity) it grows the batch
  // instead, since only larger batches add capacity
  double slo_p99_ms = 0;
  int queue_depth = 8192;          // records buffered between source and replicas
  // robustness
  int watchdog_ms = 30000;         // a batch longer than this on a replica marks it dead
  // supervisor (E4: Storm supervisors restart dead workers): a replica whose submit/wait threw is
  // recovered (Replica::recover) after restart_backoff_ms and rejoins, at most max_restarts
  // times; a replica the watchdog killed (hung device) is never restarted
  int max_restarts = 0;
  int restart_backoff_ms = 500;
  std::string fault;               // "replica_crash@N,parse_error@P,producer_fail@P"
  bool trace = false;              // roctx ranges around pipeline stages (also GALE_ROCTX=1)
  int64_t max_records = -1;        // stop once this many records are completed (bench/tests)
  uint64_t seed = 0;
};

// One acknowledged output (ack log): input record (partition, offset), the monotonic time its
// prediction was acknowledged by the sink (CLOCK_MONOTONIC ns, the clock of mono_ns()) and the
// times it passed the earlier stages: fetch response received, batch dispatched to a replica,
// device work done (prediction handed to the producer right after).
struct AckSample {
  int32_t partition;
  int64_t offset;
  int64_t t_ns;
  int64_t t_fetch_ns, t_take_ns, t_done_ns;
  int64_t t_ready_ns;  // decode / GPU ingest done: pushed to the batcher
};

struct ReplicaStats {
  std::string name;
  int device = -1;
  bool alive = true;
  int64_t batches = 0, images = 0, records = 0;
  int restarts = 0;
  int slot = 0;                                 // locality slot
  int64_t resident_records = 0, host_records = 0;  // parsed from the slot's device mirror / host
};

// Per-partition offsets, the storm-kafka `kafkaOffset` spout metric: log end
// (high watermark), next offset to fetch (emitted), first offset not yet acknowledged downstream
// (completed / commit position) and the lag behind the log end.
struct PartitionOffsets {
  int partition = -1;
  int64_t high_watermark = -1, fetched = -1, committed = -1;
  int64_t lag = 0;        // high_watermark - committed
  int64_t fetch_lag = 0;  // high_watermark - fetched
};

// Offsets fetched but not yet acknowledged downstream, per partition: a sliding window over
// the offsets (one byte per offset from the oldest pending one), so registering a fetched
// record and completing it are O(1) instead of a tree insert / erase per record. The window
// spans at most kMaxSpan offsets: an offset further away (a forward seek past records still
// pending, a record that is never acknowledged while the log moves on) goes to a sparse set,
// and the window re-bases onto the set once it drains - the span, and the memory, stay bounded.
struct OffsetWindow {
  static constexpr int64_t kMaxSpan = 1 << 22;
  int64_t base = 0;          // offset of st[0]
  std::deque<uint8_t> st;    // 1 = pending; the front is pending whenever npending > 0
  int64_t npending = 0;
  std::set<int64_t> sparse;  // pending offsets outside the window
  void add(int64_t off) {
    if (npending == 0 && sparse.empty()) {
      st.clear();
      base = off;
    }
    if (off < base) {
      if (base - off > kMaxSpan || (int64_t)st.size() + (base - off) > kMaxSpan) {
        sparse.insert(off);
        return;
      }
      st.insert(st.begin(), (size_t)(base - off), 0);  // (a seek back re-fetched them)
      base = off;
    }
    if (off - base >= kMaxSpan) {
      sparse.insert(off);
      return;
    }
    const size_t i = (size_t)(off - base);
    if (i >= st.size()) st.resize(i + 1, 0);
    if (!st[i]) {
      st[i] = 1;
      ++npending;
    }
  }
  void done(int64_t off) {
    if (off < base || (size_t)(off - base) >= st.size()) {
      sparse.erase(off);
    } else {
      uint8_t& f = st[(size_t)(off - base)];
      if (!f) {
        // not pending in the window: it may be a sparse offset that the window grew over
        // after it was set aside (add() past kMaxSpan while base was stalled, then base moved)
        sparse.erase(off);
      } else {
        f = 0;
        --npending;
        while (!st.empty() && st.front() == 0) {
          st.pop_front();
          ++base;
        }
      }
    }
    if (npending == 0 && !sparse.empty()) {  // re-base the window onto the sparse offsets
      st.clear();
      base = *sparse.begin();
      while (!sparse.empty() && *sparse.begin() - base < kMaxSpan) {
        const int64_t o = *sparse.begin();
        sparse.erase(sparse.begin());
        const size_t i = (size_t)(o - base);
        if (i >= st.size()) st.resize(i + 1, 0);
        st[i] = 1;
        ++npending;
      }
    }
  }
  bool empty() const { return npending == 0 && sparse.empty(); }
  int64_t first() const {  // the oldest pending offset (when !empty())
    if (npending == 0) return *sparse.begin();
    return sparse.empty() ? base : std::min(base, *sparse.begin());
  }
};

class Engine {
 public:
  explicit Engine(EngineConfig cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  void add_replica(std::shared_ptr<Replica> r);
  // Device-side ingest of pinned fetch buffers (CRC32C + image counts on the GPU, ingest.h);
  // set before start(). Records whose buffer has no device mirror take the host path.
  void set_ingest(std::shared_ptr<Ingest> ing);
  void start();
  // Graceful stop: sources stop fetching, queued records drain through the replicas, the sink
  // is flushed and offsets are committed.
  void stop();
  // Block until max_records completed, stop() was called, or timeout (ms; <0 = forever).
  // Returns true when the record target was reached.
  bool wait(int64_t timeout_ms);
  // Block (without stopping anything) until at least n records completed; false on timeout or
  // when the engine stopped first.
  bool wait_completed(int64_t n, int64_t timeout_ms);
  // CLOCK_MONOTONIC ns of the completion that reached the last wait_completed target (0 = it
  // was reached before the wait started): the waiting thread's own wake-up can run late on a
  // busy host, so step times taken from it alias into an alternating fast/slow pattern
  std::pair<int64_t, int64_t> last_wait() const {  // (ns, records completed by then)
    std::lock_guard<std::mutex> lk(done_mu_);
    return {last_wait_ns_, last_wait_c_};
  }
  bool running() const { return running_; }
  int64_t completed() const { return completed_.load(); }

  // counters and latency quantiles for the metrics reporter
  std::map<std::string, double> stats() const;
  std::vector<ReplicaStats> replica_stats() const;
  std::vector<PartitionOffsets> partition_offsets() const;
  void reset_stats();
  // Record-level latency probe: while on, every acknowledged record is logged (bounded at
  // `capacity` samples); switching it on clears the log. The benchmark joins the log with its
  // producer's append times for the append -> produce-ack latency at microsecond resolution.
  void set_ack_log(bool on, size_t capacity = 8u << 20);
  std::vector<AckSample> take_ack_log();
  const EngineConfig& config() const { return cfg_; }

 private:
  struct ReplicaSlot;
  class Batcher;
  struct FetchItem {
    kafka::Fetched f;
    int source = 0;
    int slot = 0;  // locality slot of the source (its batcher, pool and ingest device)
    int64_t t_fetch_ns = 0;
    bool pinned = false;
  };

  struct SourceCtl {  // a source thread's (group-managed) partition assignment
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int> parts;
    uint64_t epoch = 0, acked = 0;
    int32_t generation = -1;
    std::string member;
  };
  void source_loop(int idx);
  void group_loop();
  bool distribute(const std::vector<int>& parts, int32_t generation, const std::string& member,
                  int timeout_ms);
  bool drain_pending(const std::vector<int>& parts, int timeout_ms);
  void decode_loop(int idx);
  void decode_fetch(FetchItem& it, std::vector<InRecord>& good, int lane);
  bool ingest_fetch(FetchItem& it, std::vector<InRecord>& good, int lane);
  void worker_loop(ReplicaSlot* rs);
  void serve(ReplicaSlot* rs);  // one replica life: returns once it dies or the engine drains
  void watchdog_loop();
  void slo_step();
  void finish_batch(ReplicaSlot* rs, Batch& b);
  void emit(InRecord& r, std::string value, bool null_value, kafka::Producer* prod);
  // an oversized record -> fragments of <= max_batch images appended to `good` (false: the
  // array could not be split; the record keeps its status for the error policy)
  bool split_record(InRecord& r, std::vector<InRecord>& good);
  void fragment_done(const InRecord& frag, std::string rows, int status, kafka::Producer* prod);
  void emit_error(InRecord& r, int status, kafka::Producer* prod);
  void complete_record(const InRecord& r, bool ok);
  void complete_records(const std::vector<InRecord>& rs, bool ok);
  // at-least-once: outputs that were never acknowledged stay pending (their offsets are never
  // committed); the first one is logged and delivery_failed is raised
  void undelivered(const std::vector<InRecord>& rs);
  void commit(kafka::Consumer& c, const std::vector<int>& parts);
  kafka::Producer* producer_for(int i);
  bool fault_hit(double p);

  EngineConfig cfg_;
  std::vector<std::shared_ptr<ReplicaSlot>> replicas_;
  std::vector<std::unique_ptr<Batcher>> batchers_;  // one per locality slot
  std::vector<int> slot_key_;                         // slot -> locality key of its replicas
  std::vector<int> slot_dev_;                         // slot -> replica device (-1: CPU)
  std::vector<std::unique_ptr<kafka::Producer>> producers_;
  std::vector<std::thread> sources_, workers_, decoders_;
  std::vector<std::unique_ptr<SourceCtl>> src_ctl_;
  std::thread group_thread_;
  std::atomic<bool> group_stop_{false};
  std::atomic<int64_t> rebalances_{0};
  std::atomic<int> assigned_partitions_{0}, generation_{-1};
  std::vector<std::shared_ptr<PinnedPool>> pools_;    // per locality slot (null: heap)
  std::map<int, std::shared_ptr<Ingest>> ingests_;    // device -> GPU ingest
  Ingest* ingest_for(int slot);
  void pin_thread(int device);
  std::atomic<int64_t> steals_{0};
  std::atomic<bool> ingest_failed_{false};
  std::atomic<int64_t> ingested_records_{0}, ingest_ns_{0};
  std::atomic<int64_t> ingest_parsed_{0};  // records whose images the ingest pass parsed
  std::mutex dec_mu_;
  std::condition_variable dec_cv_, dec_space_cv_;
  std::deque<FetchItem> dec_q_;
  bool dec_closed_ = false;
  std::thread watchdog_;
  std::atomic<bool> running_{false}, stopping_{false}, sources_done_{false},
      workers_done_{false};
  std::atomic<int> sources_active_{0};

  std::mutex pend_mu_;
  std::map<int, OffsetWindow> pending_;  // partition -> fetched, unacknowledged offsets
  std::map<int, int64_t> next_fetch_;              // partition -> next offset to fetch
  std::map<int, int64_t> high_watermark_;          // partition -> log end (last fetch response)

  mutable std::mutex done_mu_;
  int64_t hit_target_ = 0, hit_ns_ = 0, hit_c_ = 0, last_wait_ns_ = 0, last_wait_c_ = 0;
  void note_completed(int64_t c, int64_t now);
  std::condition_variable done_cv_;
  std::atomic<int64_t> completed_{0};
  std::atomic<int64_t> wait_target_{0};

  // fault injection
  int64_t crash_at_batch_ = -1;
  double parse_error_p_ = 0, producer_fail_p_ = 0;  // (producer_fail: the sink producers')
  std::atomic<int64_t> undelivered_{0};
  mutable std::mutex prod_mu_;  // producers_ against stats() (stop() clears it)
  int64_t prod_retried_ = 0, prod_req_failed_ = 0;  // of producers already closed
  std::atomic<bool> delivery_failed_{false};
  std::atomic<int64_t> batches_total_{0};
  std::mutex rng_mu_;
  std::mt19937_64 rng_;

  // metrics
  std::atomic<int64_t> records_in_{0}, images_in_{0}, records_out_{0}, images_out_{0};
  std::atomic<int64_t> bytes_in_{0}, errors_{0}, produce_failures_{0}, dropped_{0};
  std::atomic<int64_t> requeued_{0}, replica_failures_{0}, replica_restarts_{0}, commits_{0};
  std::atomic<int64_t> err_by_status_[16] = {};
  std::atomic<int64_t> converted_batches_{0}, poison_batches_{0}, poison_records_{0};
  std::atomic<int64_t> poison_unknown_span_{0};  // legacy wrapper poison on an estimated span
  std::atomic<int64_t> split_records_{0}, split_fragments_{0};
  std::atomic<int64_t> sparse_fetches_{0}, restored_fetches_{0};  // bounce receive (pack_tap.h)
  Histogram h_queue_us_, h_device_us_, h_engine_e2e_us_, h_record_e2e_ms_, h_batch_images_;
  Histogram h_slo_win_us_;  // e2e latency of the SLO controller's current window
  Histogram h_slo_batch_;   // batch sizes (images) of the SLO controller's current window
  std::atomic<int> eff_batch_{0};
  std::atomic<int64_t> eff_wait_ns_{0};
  std::atomic<int64_t> slo_adjustments_{0};
  // thread time per pipeline stage (summed over threads): where the host spends its cycles
  std::atomic<int64_t> ns_poll_{0}, ns_decode_{0}, ns_take_{0}, ns_submit_{0}, ns_wait_{0},
      ns_finish_{0};
  std::atomic<int64_t> ns_handoff_{0};  // sources blocked on a full decode queue (backpressure)
  std::atomic<int64_t> ns_lane_wait_{0};  // GPU-ingested fetches: received -> a lane took it
  int64_t replica_busy_ns() const;  // summed over replicas, up to now
  std::atomic<double> capacity_rps_{0.0};   // load-aware: measured capacity (images/s)
  std::atomic<int64_t> lag_rebalances_{0};  // rebalances this member triggered on its lag
  std::atomic<int64_t> lag_rebalances_skipped_{0};  // lag over the bound, but group-wide
  std::atomic<int64_t> t_first_ns_{0}, t_last_ns_{0};
  std::atomic<bool> ack_log_on_{false};
  std::mutex ack_mu_;
  // fixed-size blocks, never reallocated: a growing vector copied hundreds of MB under ack_mu_
  // mid-window (at 4 M samples) and stalled every produce callback for ~50 ms - the LeNet-5
  // "sink tail" of round 3 was that measurement artifact
  static constexpr size_t kAckBlock = 1 << 16;
  std::vector<std::unique_ptr<AckSample[]>> ack_blocks_;
  size_t ack_n_ = 0;
  size_t ack_cap_ = 0;
  void ack_push(const AckSample& a);  // under ack_mu_
};

}  // namespace gale
