// Kafka-protocol client: cluster metadata, producer and consumer.
//
// Replaces the two Kafka libraries of the reference:
//   * Consumer  <- storm-kafka KafkaSpout (E1): partition discovery via Metadata, start position
//     latest / earliest / committed (ListOffsets / OffsetFetch; the reference hard-wires
//     LatestTime + ignoreZkOffsets, MainTopology.java:101-103), long-poll Fetch, offset commits
//     (the spout's periodic ZK commits, X3), lag metrics (the spout's kafkaOffset metric).
//   * Producer  <- kafka-clients 0.11 KafkaProducer (E7, KafkaBolt.java:111-113,144): async send
//     with per-record callbacks on the sender thread, acks 0/1/-1 (MainTopology.java:113),
//     batch.size / linger.ms accumulation per partition, pipelined in-flight requests, the
//     DefaultPartitioner (murmur2 for keyed records, round-robin for null keys, E7/E9).
// Fetch response bodies are received straight into caller-provided buffers (pinned host memory in
// the serving engine), so record values are staged for the GPU without another copy.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "protocol.h"
#include "wire.h"

namespace gale {
namespace kafka {

struct KafkaError : std::runtime_error {
  int code;
  KafkaError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct ClientConfig {
  std::string bootstrap = "127.0.0.1:9092";  // host:port[,host:port...]
  std::string client_id = "gale";
  int request_timeout_ms = 30000;
  int connect_timeout_ms = 10000;
  // > 0: each receive waits (poll) until min(this, bytes still wanted) bytes are queued
  // (SO_RCVLOWAT, set per call so the last piece of a response never waits for more), then
  // takes them without blocking: one wake-up per ~this many bytes of a large response instead of
  // one per arriving segment. (A blocking recv cannot be used with it: after a partial copy the
  // kernel compares only the still-unread bytes with the mark, and the reader sleeps on.)
  int recv_lowat = 0;
};

// Response buffers: the body of a response frame (after the 4-byte size) is received into
// memory obtained from this allocator. The shared_ptr's deleter returns it to its pool.
using BufferAlloc = std::function<std::shared_ptr<uint8_t>(size_t bytes)>;
std::shared_ptr<uint8_t> heap_alloc(size_t bytes);

// Observes a response body while it is received (e.g. to transform the bytes while they are
// cache-hot). begin(buf, n) before the first byte; progress(done) after every receive call
// (bytes [0, done) are in place; one call receives at most chunk_bytes()); finish() after the
// last one, its value is kept in Fetched::tap_result.
//
// Bounce mode: a tap whose begin() returns true takes the body over - it is received piece by
// piece into the tap's own (cache-resident) window (window(&room) -> receive -> received(bytes))
// and buf gets only what the tap writes into it; finish() then says what buf holds.
class RecvTap {
 public:
  virtual ~RecvTap() = default;
  virtual bool begin(uint8_t* buf, size_t n) = 0;  // true: bounce mode for this body
  virtual void progress(size_t done) = 0;
  virtual int64_t finish() = 0;
  virtual size_t chunk_bytes() const { return 256 << 10; }
  virtual uint8_t* window(size_t* room) {
    *room = 0;
    return nullptr;
  }
  virtual void received(size_t bytes) { (void)bytes; }
  // the last body was kept sparse (bounce mode: framing only on the host, text packed)
  virtual bool sparse() const { return false; }
  // a sparse body -> its full bytes in place (host fallback paths; buf, n as in begin)
  virtual void restore(const std::shared_ptr<uint8_t>& buf, size_t n) {
    (void)buf;
    (void)n;
  }
};

class Connection {
 public:
  Connection(const std::string& host, int port, const ClientConfig& cfg);
  ~Connection();
  Connection(const Connection&) = delete;
  Connection& operator=(const Connection&) = delete;

  int32_t send(ApiKey key, const Writer& body);  // returns the correlation id
  // Receive the response for `corr` (responses arrive in request order on one connection).
  // The returned buffer starts AFTER the correlation id.
  std::shared_ptr<uint8_t> recv(int32_t corr, size_t* size, const BufferAlloc& alloc,
                                RecvTap* tap = nullptr, int64_t* tap_result = nullptr);
  std::string request(ApiKey key, const Writer& body);  // send + recv into a string
  const std::string& host() const { return host_; }
  int port() const { return port_; }

 private:
  void send_all(const char* p, size_t n);
  void recv_all(uint8_t* p, size_t n, RecvTap* tap = nullptr);
  int fd_ = -1;
  int lowat_cap_ = 0, lowat_cur_ = 1, timeout_ms_ = 30000;
  std::string host_;
  int port_;
  int32_t next_corr_ = 1;
  std::string client_id_;
};

// Metadata cache + per-node connections (one Cluster per client thread; not thread-safe).
class Cluster {
 public:
  explicit Cluster(ClientConfig cfg);
  const ClientConfig& config() const { return cfg_; }
  // Refresh metadata for `topics` (auto-creating them when the broker allows).
  void refresh(const std::vector<std::string>& topics, bool auto_create = true);
  int partitions(const std::string& topic);  // refreshes when unknown; -1 if absent
  int32_t leader(const std::string& topic, int partition);
  Connection& node(int32_t node_id);
  Connection& any();
  Connection& coordinator(const std::string& group);
  std::vector<BrokerNode> brokers() const;
  void invalidate() { topics_.clear(); }
  // Close a node's connection (after a failed/timed-out exchange left it mid-response); the
  // next node() call reconnects.
  void drop(int32_t node_id) { conns_.erase(node_id); }

 private:
  void check_versions(Connection& c);
  ClientConfig cfg_;
  std::map<int32_t, BrokerNode> nodes_;
  std::map<int32_t, std::unique_ptr<Connection>> conns_;
  std::unique_ptr<Connection> bootstrap_;
  std::map<std::string, std::vector<int32_t>> topics_;  // topic -> leader per partition
  std::map<std::string, int32_t> coordinators_;
};

// Java Kafka's murmur2 (Utils.murmur2), for keyed-record partitioning compatibility.
int32_t murmur2(const uint8_t* data, size_t n);

struct ProducerConfig : ClientConfig {
  int acks = 1;                    // MainTopology.java:113
  int linger_ms = 0;               // kafka-clients 0.11 default
  int batch_size = 16384;          // kafka-clients 0.11 default (bytes per partition batch)
  int max_request_size = 64 << 20;
  int max_in_flight = 5;
  int64_t buffer_memory = 1ll << 30;  // send() blocks while more than this is unsent
  int compression = 0;  // compression.type (compress.h Codec; kafka-clients default none)
  // kafka-clients `retries` / `retry.backoff.ms` / `delivery.timeout.ms`: a request that failed
  // with a retriable error (protocol.h error_retriable: leader moved, timeout, connection lost)
  // is sent again after the backoff, at most `retries` times and while the record is younger
  // than the delivery timeout; only then does its callback see the error. As in kafka-clients,
  // a retried batch can land behind batches of the same partition that were sent after it
  // while it waited (max_in_flight > 1).
  int retries = 0;
  int retry_backoff_ms = 100;
  int delivery_timeout_ms = 120000;
  // fault injection (tests, GALE_FAULT producer_fail@P): each produce request is dropped before
  // it is sent with probability fail_p and completes with NETWORK_EXCEPTION (then retried)
  double fail_p = 0;
  uint64_t fail_seed = 0;
};

struct SendResult {
  int16_t error = 0;
  int32_t partition = -1;
  int64_t offset = -1;
};
using SendCallback = std::function<void(const SendResult&)>;

// Several records for one partition sent (and acknowledged) as a unit: the serving engine hands
// each micro-batch's predictions over in one call instead of one send() per record. Record i's
// value is values[off[i], off[i + 1]) (null when null_value[i] is set); keys likewise from
// keys / koff / key_null (koff empty = every key null); every record carries `headers`.
struct RecordGroup {
  std::string values;
  std::vector<uint32_t> off;        // n + 1 boundaries
  std::vector<uint8_t> null_value;  // n flags, or empty (no null values)
  std::string keys;
  std::vector<uint32_t> koff;       // n + 1 boundaries, or empty (all keys null)
  std::vector<uint8_t> key_null;    // n flags (with koff)
  std::vector<Header> headers;
  int64_t ts = -1;
  size_t size() const { return off.empty() ? 0 : off.size() - 1; }
};
// (error, partition, offset of the group's first record, records): once per group
using GroupCallback = std::function<void(int16_t, int32_t, int64_t, size_t)>;

struct ProducerStats {
  int64_t records_sent = 0, records_acked = 0, records_failed = 0, requests = 0, bytes = 0;
  int64_t records_retried = 0, requests_failed = 0;  // re-sent records; requests that failed
};

class Producer {
 public:
  explicit Producer(ProducerConfig cfg);
  ~Producer();
  Producer(const Producer&) = delete;
  Producer& operator=(const Producer&) = delete;

  // Asynchronous send. partition < 0 selects the partitioner. value_null sends a null record
  // (tombstone) - what the reference's JsonSerializer does for a failed tuple.
  void send(const std::string& topic, int partition, const std::string* key, std::string value,
            bool value_null, std::vector<Header> headers, int64_t timestamp, SendCallback cb);
  // A group of records to one partition (partition < 0: the partitioner picks one for the
  // whole group), acknowledged together; the records stay in order and in one batch.
  void send_group(const std::string& topic, int partition, RecordGroup g, GroupCallback cb);
  void flush();  // blocks until every record sent so far is acked or failed
  void close();
  int partitions_for(const std::string& topic);
  ProducerStats stats() const;

 private:
  struct Pending {
    std::string key;
    bool key_null = true;
    std::string value;
    bool value_null = false;
    std::vector<Header> headers;
    int64_t ts = -1;
    SendCallback cb;
    std::unique_ptr<RecordGroup> group;  // set: this entry is a whole group of records
    GroupCallback gcb;
    int attempts = 0;    // sends that failed with a retriable error so far
    int64_t enq_ms = 0;  // when it was handed to send() / send_group() (delivery timeout)
    size_t records() const { return group ? group->size() : 1; }
  };
  struct PartBatch {
    std::vector<Pending> recs;
    size_t bytes = 0;
    int64_t first_ms = 0;
  };
  struct InFlight {
    int32_t corr;
    int32_t node;
    std::vector<std::pair<std::pair<std::string, int>, std::vector<Pending>>> batches;
  };
  struct Retry {  // a failed chunk waiting for its backoff (sender thread only)
    std::pair<std::string, int> tp;
    std::vector<Pending> recs;
    int64_t due_ms;
  };
  void run();
  int choose_partition(const std::string& topic, const std::string* key);

  ProducerConfig cfg_;
  Cluster cluster_;  // sender thread only
  Cluster meta_;     // partition counts for send(), under mu_
  mutable std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::map<std::pair<std::string, int>, PartBatch> acc_;
  std::map<std::string, int> nparts_;
  int64_t unsent_bytes_ = 0;
  int64_t outstanding_ = 0;
  bool flush_req_ = false, closing_ = false;
  uint32_t rr_ = 0;
  std::thread thread_;
  ProducerStats stats_;
  std::deque<Retry> retry_;  // sender thread only
  uint64_t fault_state_;     // fail_p's generator (sender thread only)
};

struct ConsumerConfig : ClientConfig {
  std::string group_id;            // empty: no offset commits
  int max_wait_ms = 100;           // fetch long-poll
  int min_bytes = 1;
  int fetch_max_bytes = 64 << 20;
  int partition_max_bytes = 16 << 20;
  bool check_crcs = true;
  std::string auto_offset_reset = "latest";  // on OFFSET_OUT_OF_RANGE / no committed offset
  // keep the next fetch of every leader in flight while the application processes the previous
  // response (the Java consumer's fetcher does the same): the broker's send overlaps our work
  bool prefetch = true;
  // bound on one decompressed batch (compressed batches / legacy wrappers, compress.h)
  size_t max_decompressed_bytes = (size_t)256 << 20;
};

// One fetch round: records point into `buf` (the response body).
struct Fetched {
  std::shared_ptr<uint8_t> buf;
  size_t size = 0;
  std::vector<RecordRef> records;
  std::vector<BatchSpan> batches;  // record batches (for deferred CRC checks)
  bool crc_checked = false;
  int64_t tap_result = -1;  // the consumer's RecvTap::finish() for this body (-1: no tap)
  // the host copy of the body holds Kafka framing and the ends of each value only (bounce
  // receive, csrc/runtime/pack_tap.h): the full text is the packed stream in the same buffer.
  // restore() rebuilds it in place for the host paths.
  bool sparse = false;
  std::shared_ptr<RecvTap> restorer;
  void restore() {
    if (!sparse) return;
    restorer->restore(buf, size);
    sparse = false;
  }
};

class Consumer {
 public:
  Consumer(ConsumerConfig cfg, BufferAlloc alloc = heap_alloc);
  void assign(const std::string& topic, const std::vector<int>& partitions);
  const std::vector<int>& assignment() const { return parts_; }
  const std::string& topic() const { return topic_; }
  // "latest" | "earliest" | "committed" (committed falls back to auto_offset_reset)
  void seek_to(const std::string& where);
  void seek(int partition, int64_t offset);
  int64_t position(int partition) const;
  // One fetch round over all assigned partitions (grouped by leader). Empty when nothing arrived
  // within max_wait_ms. With prefetch the next round is already requested when this returns.
  std::vector<Fetched> poll();
  void commit(const std::map<int, int64_t>& offsets);  // next offset to read, per partition
  // group-managed consumers commit under their generation (fenced by the coordinator)
  void set_generation(int32_t generation, const std::string& member_id) {
    generation_ = generation;
    member_id_ = member_id;
  }
  int64_t committed(int partition);
  std::map<int, int64_t> high_watermarks() const { return hw_; }
  Cluster& cluster() { return cluster_; }
  // record-format conversion counters (compress.h): batches rewritten from a compressed or
  // legacy format, undecodable batches skipped as poison records
  int64_t converted_batches() const { return converted_batches_; }
  int64_t poison_batches() const { return poison_batches_; }
  int64_t poison_records() const { return poison_records_; }
  int64_t poison_unknown_span() const { return poison_unknown_span_; }
  // fetch response bodies are shown to this tap while they are received
  void set_recv_tap(std::shared_ptr<RecvTap> tap) { tap_ = std::move(tap); }

 private:
  int64_t list_offset(int partition, int64_t ts);
  struct InFlight {
    int32_t node, corr;
    std::map<int, int64_t> from;  // partition -> offset the fetch was issued at
  };
  void send_fetches();
  // receive every in-flight response; records at a position that moved meanwhile are dropped
  void collect(std::vector<Fetched>& out);
  void drain();  // collect into ready_ (before any other request on a fetch connection)
  ConsumerConfig cfg_;
  BufferAlloc alloc_;
  std::shared_ptr<RecvTap> tap_;
  Cluster cluster_;
  std::string topic_;
  std::vector<int> parts_;
  std::map<int, int64_t> pos_, hw_;
  std::vector<InFlight> inflight_;
  std::vector<Fetched> ready_;  // drained responses not yet returned by poll()
  int32_t generation_ = -1;
  std::string member_id_;
  std::atomic<int64_t> converted_batches_{0}, poison_batches_{0}, poison_records_{0};
  std::atomic<int64_t> poison_unknown_span_{0};
  int poison_logged_ = 0;
};

// Consumer-group membership (Kafka's eager rebalance protocol): JoinGroup -> (leader computes
// the assignment with the chosen assignor) -> SyncGroup -> periodic Heartbeat; LeaveGroup on
// close. The elastic replacement of the reference's static spout/partition split (E1, E4): a
// member that dies stops heartbeating, the coordinator rebalances and the survivors adopt its
// partitions. One topic per group (the engine's input topic).
struct GroupConfig : ClientConfig {
  std::string group_id;
  std::string topic;
  int session_timeout_ms = 6000;
  int rebalance_timeout_ms = 8000;
  std::string assignor = "range";  // range | roundrobin | load-aware
};

// What a member tells the leader in its subscription's user_data under the load-aware assignor:
// its measured serving capacity (records/s; <= 0 = not measured yet) and the partitions it owns
// now (the assignment keeps them where the quotas allow, like Kafka's sticky assignor).
struct MemberLoad {
  double capacity = 0;
  std::vector<int32_t> owned;
};
std::string encode_member_load(const MemberLoad& m);
MemberLoad decode_member_load(const std::string& b);  // empty/garbled -> capacity 0

class GroupMember {
 public:
  explicit GroupMember(GroupConfig cfg);
  ~GroupMember();
  GroupMember(const GroupMember&) = delete;
  GroupMember& operator=(const GroupMember&) = delete;
  // (Re)join: blocks through the rebalance; returns this member's partitions of cfg.topic.
  std::vector<int> join();
  // false: the group is rebalancing or this member was fenced -> revoke, then join() again
  bool heartbeat();
  void leave();
  int32_t generation() const { return generation_; }
  const std::string& member_id() const { return member_id_; }
  bool is_leader() const { return leader_; }
  // The assignors, exposed for tests: member -> partitions of one topic with n partitions
  static std::map<std::string, std::vector<int>> assign(const std::string& assignor,
                                                        std::vector<std::string> members, int n);
  // Load-aware assignor (Storm's LoadAwareShuffleGrouping at partition granularity): quotas
  // proportional to the members' capacities c_i, apportioned so the largest partitions / c_i
  // is minimal (members that have not measured a capacity count as the mean of those that
  // have), filled first from the partitions each member owns now, then from the unowned ones.
  // A member whose capacity is far below the others' can get zero partitions.
  static std::map<std::string, std::vector<int>> assign_load_aware(
      std::vector<std::string> members, const std::map<std::string, MemberLoad>& load, int n);
  // user_data sent with the next JoinGroup (load-aware: encode_member_load)
  void set_user_data(std::string d) { user_data_ = std::move(d); }
  // load-aware: this member's share of the group's capacity as the leader weighed it for the
  // current assignment (carried in the assignment's user_data; -1 = unknown / other assignor)
  double capacity_share() const { return capacity_share_; }
  // per-partition lag of the group on its topic (log end - committed offset; partitions with
  // no commit yet count from the log start): what decides whether a rebalance can help
  std::map<int, int64_t> partition_lags();

 private:
  GroupConfig cfg_;
  Cluster cluster_;
  std::string member_id_;
  std::string user_data_;
  int32_t generation_ = -1;
  bool leader_ = false;
  double capacity_share_ = -1;
};

}  // namespace kafka
}  // namespace gale
