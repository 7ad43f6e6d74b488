// Embedded Kafka-protocol broker.
//
// Plays the role that an embedded Kafka / Storm LocalCluster plays for the reference's topology
// ("an embedded in-process Kafka-protocol broker"): tests, benchmarks and the
// GPU boxes (which have no network) get real Kafka topics on 127.0.0.1 that any Kafka-protocol
// client can talk to, with the reference's external contract unchanged (INPUT_TOPIC records in,
// OUTPUT_TOPIC records out, MainTopology.java:36-38).
//
// * One thread per client connection (blocking I/O, so concurrent consumers are served in
//   parallel); in-memory partition logs of RecordBatch v2 segments with byte-based retention;
//   zero-copy Fetch responses (writev straight from the stored batches).
// * Long-poll Fetch (max_wait_ms / min_bytes), acks 0/1/-1 Produce, ListOffsets, consumer-group
//   offset storage (FindCoordinator / OffsetCommit / OffsetFetch), group membership (JoinGroup /
//   SyncGroup / Heartbeat / LeaveGroup, group_coordinator.h), CreateTopics, ApiVersions.
// * Multi-broker clusters: set_cluster() makes partition p of every topic led by node
//   nodes[p % n]; Metadata advertises the whole cluster (one broker per GPU rank in bench.py).
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "group_coordinator.h"
#include "protocol.h"
#include "compress.h"
#include "wire.h"

namespace gale {
namespace kafka {

struct BrokerConfig {
  std::string host = "127.0.0.1";
  int port = 0;                       // 0 = ephemeral
  int node_id = 0;
  int default_partitions = 1;         // num.partitions for auto-created topics
  bool auto_create_topics = true;
  int64_t max_message_bytes = 64ll << 20;  // message.max.bytes (per record batch)
  int64_t retention_bytes = 4ll << 30;     // per partition; oldest segments dropped beyond it
  bool check_crcs = true;             // validate produced batches
  // Fetch responses send stored record batches without a user->kernel copy (vmsplice the
  // immutable batch pages into a pipe, splice the pipe into the socket), as a Kafka broker's
  // sendfile() from the page cache does. Small/owned pieces (headers) are written normally.
  // Off by default here; bench.py turns it on (profiles/archive/r3_broker_zero_copy_default.jsonl):
  // with 11 loopback connections the transport costs 0.161 core-s per GB spliced against 0.206
  // copied, sender and receiver together (profiles/r5_llc_pair.jsonl).
  bool zero_copy = false;
  // log.message.timestamp.type=LogAppendTime: every appended batch is stamped with the broker's
  // wall clock (attributes timestamp-type bit + maxTimestamp, CRC patched in O(log n) without
  // re-reading the batch); consumers then see the append time as each record's timestamp, which
  // makes record-timestamp end-to-end latency exact even for pre-encoded (bench) batches.
  bool log_append_time = false;
  std::string cluster_id = "gale-embedded";
};

struct BrokerStats {
  int64_t requests = 0, produce_requests = 0, fetch_requests = 0;
  int64_t bytes_in = 0, bytes_out = 0, records_in = 0, connections = 0;
  int64_t bytes_spliced = 0;  // part of bytes_out sent zero-copy
};

// Latency-tail probes of the serving path, since the last take_probes(): the worst and the
// number of > 1 ms cases of (a) a parked fetch's wake-up: append signalled -> response built,
// (b) writing one response to the socket, (c) an append waiting for the log lock.
struct BrokerProbes {
  int64_t wake_max_us = 0, wake_slow = 0, flush_max_us = 0, flush_slow = 0;
  int64_t lock_max_us = 0, lock_slow = 0;
};

class Broker {
 public:
  explicit Broker(BrokerConfig cfg);
  ~Broker();
  Broker(const Broker&) = delete;
  Broker& operator=(const Broker&) = delete;

  void start();
  void stop();
  int port() const { return port_; }
  int node_id() const { return cfg_.node_id; }
  const BrokerConfig& config() const { return cfg_; }

  void set_cluster(const std::vector<BrokerNode>& nodes);
  std::vector<BrokerNode> cluster() const;
  bool leads(int partition) const;

  // Returns false if the topic already existed (partition count unchanged).
  bool create_topic(const std::string& topic, int partitions);
  std::vector<std::string> topics() const;
  int partitions(const std::string& topic) const;  // -1 if unknown

  // Local (in-process) producer: appends one batch; returns its base offset.
  int64_t append(const std::string& topic, int partition, const std::vector<RecordIn>& recs);
  // Append a pre-encoded batch shared by reference (bench preloading of repeated payloads).
  // Old message format (log.message.format.version < 0.11): `recs` appended as ONE legacy
  // message set of magic 0 or 1, wrapped in a `codec`-compressed message when codec != 0. The
  // bytes are stored and served as such (consumers must read the old format). Returns the first
  // offset.
  int64_t append_legacy(const std::string& topic, int partition, int magic,
                        const std::vector<LegacyRecord>& recs, int codec);
  int64_t append_shared(const std::string& topic, int partition,
                        std::shared_ptr<const std::string> batch);
  int64_t log_start(const std::string& topic, int partition) const;
  int64_t log_end(const std::string& topic, int partition) const;
  // Concatenated batches (base offsets patched) covering [offset, ...) up to ~max_bytes.
  std::string read_raw(const std::string& topic, int partition, int64_t offset,
                       int64_t max_bytes) const;
  int64_t committed(const std::string& group, const std::string& topic, int partition) const;
  BrokerStats stats() const;
  BrokerProbes take_probes();
  GroupInfo describe_group(const std::string& group) { return coord_.describe(group); }
  // Fault injection (tests): the next `n` partition appends of Produce requests to `topic` are
  // rejected with `error` (nothing is appended) - a broker that truly refuses produces, e.g.
  // NOT_LEADER_FOR_PARTITION during a leader move. n = 0 clears it.
  void fail_produce(const std::string& topic, int64_t n, int16_t error);

 public:
  struct Chunk;  // one piece of a response (owned bytes or a zero-copy slice of a stored batch)

 private:
  struct Segment {
    int64_t base;
    int64_t next;  // base + lastOffsetDelta + 1
    int64_t max_ts;
    std::shared_ptr<const std::string> bytes;
    // LogAppendTime: bytes [kBatchAttrOffset, kBatchMaxTsOffset + 8) and the CRC as sent
    bool stamped = false;
    uint32_t crc = 0;
    uint8_t hdr[22] = {};
    // a legacy message set (magic 0/1, kafka/compress.h): served verbatim, offsets included
    bool legacy = false;
  };
  struct PartitionLog {
    std::vector<Segment> segs;
    size_t first = 0;  // index of the first retained segment
    int64_t start = 0, end = 0;
    int64_t bytes = 0;
  };
  struct Conn;

  void accept_loop();
  void serve(int fd);
  void wake(const std::string& topic, int partition);
  void wake_all();
  bool handle_request(Conn& c, const uint8_t* p, size_t n);
  bool try_fetch(Conn& c, bool final_attempt);
  bool flush(Conn& c);
  // 1 sent, 0 splice unusable, -1 connection error
  int splice_chunk(Conn& c, const Chunk& f, bool more);
  int64_t append_locked(PartitionLog& log, std::shared_ptr<const std::string> batch, bool legacy,
                        const BatchInfo& bi);
  PartitionLog* find_log(const std::string& topic, int partition);
  const PartitionLog* find_log(const std::string& topic, int partition) const;
  BrokerNode self_node() const;
  int32_t leader_of(int partition) const;

  BrokerConfig cfg_;
  int listen_fd_ = -1;
  int port_ = 0;
  std::thread thread_;  // acceptor
  std::mutex conn_mu_;
  std::vector<std::thread> conn_threads_;
  std::deque<std::pair<int64_t, std::shared_ptr<const std::string>>> spliced_grave_;
  std::vector<int> conn_fds_;
  // long-poll wakeups: a parked Fetch registers a waiter on each partition it asks for; an
  // append to a partition wakes only the fetches waiting on it (a wake-everyone scheme woke
  // every consumer connection per appended batch: 12 x ~19k wakeups/s at 1.2 M img/s offered)
  struct Waiter {
    std::mutex m;
    std::condition_variable cv;
    bool flag = false;
    int64_t t_wake_ns = 0;  // when the flag was first set (probe)
  };
  struct Probe {
    std::atomic<int64_t> max_ns{0}, slow{0};
    void add(int64_t ns) {
      int64_t m = max_ns.load(std::memory_order_relaxed);
      while (ns > m && !max_ns.compare_exchange_weak(m, ns, std::memory_order_relaxed)) {
      }
      if (ns > 1000000) slow.fetch_add(1, std::memory_order_relaxed);
    }
  };
  Probe probe_wake_, probe_flush_, probe_lock_;
  std::mutex append_mu_;  // waiters_
  std::map<std::pair<std::string, int>, std::vector<Waiter*>> waiters_;
  std::atomic<bool> running_{false};
  mutable std::mutex mu_;  // topics_, offsets_, cluster_, stats_
  std::map<std::string, std::vector<PartitionLog>> topics_;
  std::map<std::string, int64_t> offsets_;  // "group\0topic\0partition" -> offset
  std::map<std::string, std::pair<int64_t, int16_t>> produce_faults_;  // topic -> (left, error)
  std::vector<BrokerNode> cluster_;
  BrokerStats stats_;
  GroupCoordinator coord_;
};

}  // namespace kafka
}  // namespace gale
