// Kafka-protocol client: connections, metadata, producer, consumer (see client.h).
#include "client.h"
#include "gale/llc_pair.h"
#include "gale/thread_name.h"

#include "compress.h"

#include <arpa/inet.h>
#include <stdio.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <sstream>

namespace gale {
namespace kafka {

namespace {

int64_t wall_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}
int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::vector<std::pair<std::string, int>> parse_bootstrap(const std::string& s) {
  std::vector<std::pair<std::string, int>> out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, ',')) {
    while (!item.empty() && isspace((unsigned char)item.back())) item.pop_back();
    while (!item.empty() && isspace((unsigned char)item.front())) item.erase(0, 1);
    if (item.empty()) continue;
    const size_t c = item.rfind(':');
    if (c == std::string::npos) {
      out.push_back({item, 9092});
    } else {
      out.push_back({item.substr(0, c), std::stoi(item.substr(c + 1))});
    }
  }
  if (out.empty()) throw std::invalid_argument("empty bootstrap server list");
  return out;
}

}  // namespace

std::shared_ptr<uint8_t> heap_alloc(size_t bytes) {
  return std::shared_ptr<uint8_t>(new uint8_t[bytes + 64], std::default_delete<uint8_t[]>());
}

// ---------------------------------------------------------------------------------------------
// Connection
// ---------------------------------------------------------------------------------------------

Connection::Connection(const std::string& host, int port, const ClientConfig& cfg)
    : lowat_cap_(std::max(0, cfg.recv_lowat)), timeout_ms_(cfg.request_timeout_ms), host_(host),
      port_(port),
      client_id_(cfg.client_id) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw KafkaError(-1, "cannot resolve " + host);
  fd_ = socket(AF_INET, SOCK_STREAM, 0);
  fcntl(fd_, F_SETFL, fcntl(fd_, F_GETFL) | O_NONBLOCK);
  int rc = connect(fd_, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc != 0 && errno != EINPROGRESS) {
    close(fd_);
    throw KafkaError(-1, "connect to " + host + ":" + ps + " failed: " + strerror(errno));
  }
  if (rc != 0) {
    pollfd p{fd_, POLLOUT, 0};
    int err = 0;
    socklen_t el = sizeof(err);
    if (poll(&p, 1, cfg.connect_timeout_ms) != 1 ||
        getsockopt(fd_, SOL_SOCKET, SO_ERROR, &err, &el) != 0 || err != 0) {
      close(fd_);
      throw KafkaError(-1, "connect to " + host + ":" + ps + " failed: " +
                               (err ? strerror(err) : "timeout"));
    }
  }
  fcntl(fd_, F_SETFL, fcntl(fd_, F_GETFL) & ~O_NONBLOCK);
  int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  const int sz = socket_buffer_bytes();
  if (sz > 0) setsockopt(fd_, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
  if (sz > 0) setsockopt(fd_, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
  timeval tv{cfg.request_timeout_ms / 1000, (cfg.request_timeout_ms % 1000) * 1000};
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  // an in-process broker pins the thread serving this connection to the reader's L3 domain
  sockaddr_in la{};
  socklen_t ll = sizeof(la);
  if (getsockname(fd_, reinterpret_cast<sockaddr*>(&la), &ll) == 0)
    llc::register_local_port(ntohs(la.sin_port));
}

Connection::~Connection() {
  if (fd_ >= 0) close(fd_);
}

void Connection::send_all(const char* p, size_t n) {
  while (n) {
    const ssize_t w = ::send(fd_, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw KafkaError(-1, std::string("send failed: ") + strerror(errno));
    }
    p += w;
    n -= (size_t)w;
  }
}

void Connection::recv_all(uint8_t* p, size_t n, RecvTap* tap) {
  const uint8_t* base = p;
  const size_t cap = tap ? std::max<size_t>(4096, tap->chunk_bytes()) : n;
  while (n) {
    const size_t want = std::min(n, cap);
    int flags = 0;
    if (lowat_cap_ > 0) {
      const int lw = (int)std::min<size_t>(want, (size_t)lowat_cap_);
      if (lw != lowat_cur_ && setsockopt(fd_, SOL_SOCKET, SO_RCVLOWAT, &lw, sizeof(lw)) == 0)
        lowat_cur_ = lw;
      pollfd pf{fd_, POLLIN, 0};
      const int pr = ::poll(&pf, 1, timeout_ms_);
      if (pr == 0) throw KafkaError(REQUEST_TIMED_OUT, "request timed out on " + host_);
      if (pr < 0) {
        if (errno == EINTR) continue;
        throw KafkaError(-1, std::string("poll failed: ") + strerror(errno));
      }
      flags = MSG_DONTWAIT;
    }
    const ssize_t r = ::recv(fd_, p, want, flags);
    if (r == 0) throw KafkaError(-1, "connection closed by broker " + host_);
    if (r < 0) {
      if (errno == EINTR) continue;
      if (flags && (errno == EAGAIN || errno == EWOULDBLOCK)) continue;  // (raced the mark)
      if (errno == EAGAIN || errno == EWOULDBLOCK)
        throw KafkaError(REQUEST_TIMED_OUT, "request timed out on " + host_);
      throw KafkaError(-1, std::string("recv failed: ") + strerror(errno));
    }
    p += r;
    n -= (size_t)r;
    if (tap) tap->progress((size_t)(p - base));
  }
}

int32_t Connection::send(ApiKey key, const Writer& body) {
  Writer w;
  w.reserve(body.size() + 64);
  w.i32(0);
  RequestHeader h;
  h.api_key = key;
  h.api_version = kVersion(key);
  h.correlation_id = next_corr_++;
  h.client_id = client_id_;
  encode_request_header(w, h);
  w.raw(body.buf.data(), body.buf.size());
  w.patch_i32(0, (int32_t)(w.size() - 4));
  send_all(w.buf.data(), w.buf.size());
  return h.correlation_id;
}

std::shared_ptr<uint8_t> Connection::recv(int32_t corr, size_t* size, const BufferAlloc& alloc,
                                          RecvTap* tap, int64_t* tap_result) {
  uint8_t hdr[8];
  recv_all(hdr, 8);
  Reader r(hdr, 8);
  const int32_t sz = r.i32();
  const int32_t got = r.i32();
  if (sz < 4) throw KafkaError(-1, "bad response size");
  if (got != corr)
    throw KafkaError(-1, "correlation id mismatch (" + std::to_string(got) + " != " +
                             std::to_string(corr) + ")");
  const size_t n = (size_t)sz - 4;
  std::shared_ptr<uint8_t> buf = alloc(n);
  const bool bounce = tap && tap->begin(buf.get(), n);
  if (bounce) {
    // the tap's window takes the bytes; the tap writes what it keeps into buf
    size_t left = n;
    while (left) {
      size_t room = 0;
      uint8_t* w = tap->window(&room);
      if (!w || room == 0) throw KafkaError(-1, "receive tap without a window");
      const size_t want = std::min(left, room);
      recv_all(w, want, nullptr);
      tap->received(want);
      left -= want;
    }
  } else {
    recv_all(buf.get(), n, tap);
  }
  if (tap && tap_result) *tap_result = tap->finish();
  *size = n;
  return buf;
}

std::string Connection::request(ApiKey key, const Writer& body) {
  const int32_t corr = send(key, body);
  size_t n = 0;
  auto buf = recv(corr, &n, heap_alloc);
  return std::string(reinterpret_cast<const char*>(buf.get()), n);
}

// ---------------------------------------------------------------------------------------------
// Cluster
// ---------------------------------------------------------------------------------------------

Cluster::Cluster(ClientConfig cfg) : cfg_(std::move(cfg)) {}

void Cluster::check_versions(Connection& c) {
  Writer w;
  const std::string resp = c.request(API_VERSIONS, w);
  Reader r(resp);
  const ApiVersionsResponse av = decode_api_versions_response(r);
  if (av.error != NONE) throw KafkaError(av.error, "ApiVersions failed");
  for (ApiKey k : {PRODUCE, FETCH, LIST_OFFSETS, METADATA, OFFSET_COMMIT, OFFSET_FETCH,
                   FIND_COORDINATOR}) {
    bool ok = false;
    for (const auto& a : av.apis)
      if (a.key == k && a.min_version <= kVersion(k) && kVersion(k) <= a.max_version) ok = true;
    if (!ok)
      throw KafkaError(UNSUPPORTED_VERSION, "broker " + c.host() + " does not support api " +
                                                std::to_string(k) + " v" +
                                                std::to_string(kVersion(k)));
  }
}

Connection& Cluster::any() {
  if (!conns_.empty()) return *conns_.begin()->second;
  if (bootstrap_) return *bootstrap_;
  std::string errs;
  for (auto& hp : parse_bootstrap(cfg_.bootstrap)) {
    try {
      auto c = std::make_unique<Connection>(hp.first, hp.second, cfg_);
      check_versions(*c);
      bootstrap_ = std::move(c);
      return *bootstrap_;
    } catch (const KafkaError& e) {
      errs += std::string(e.what()) + "; ";
    }
  }
  throw KafkaError(-1, "no bootstrap broker reachable: " + errs);
}

void Cluster::refresh(const std::vector<std::string>& topics, bool auto_create) {
  for (int attempt = 0;; ++attempt) {
    MetadataRequest req;
    req.topics = topics;
    req.allow_auto_topic_creation = auto_create;
    Writer w;
    encode_metadata_request(w, req);
    const std::string resp = any().request(METADATA, w);
    Reader r(resp);
    const MetadataResponse m = decode_metadata_response(r);
    for (const BrokerNode& b : m.brokers) nodes_[b.node_id] = b;
    bool retry = false;
    for (const TopicMetadata& t : m.topics) {
      if (t.error == LEADER_NOT_AVAILABLE) {
        retry = true;
        continue;
      }
      if (t.error != NONE) {
        topics_.erase(t.name);
        continue;
      }
      std::vector<int32_t> leaders(t.partitions.size(), -1);
      for (const PartitionMetadata& p : t.partitions)
        if ((size_t)p.index < leaders.size()) leaders[(size_t)p.index] = p.leader;
      topics_[t.name] = leaders;
    }
    if (!retry || attempt >= 20) return;
    usleep(50000);
  }
}

int Cluster::partitions(const std::string& topic) {
  auto it = topics_.find(topic);
  if (it == topics_.end()) {
    refresh({topic});
    it = topics_.find(topic);
    if (it == topics_.end()) return -1;
  }
  return (int)it->second.size();
}

int32_t Cluster::leader(const std::string& topic, int partition) {
  if (partitions(topic) <= partition) throw KafkaError(UNKNOWN_TOPIC_OR_PARTITION, topic);
  const int32_t l = topics_[topic][(size_t)partition];
  if (l < 0) throw KafkaError(LEADER_NOT_AVAILABLE, topic);
  return l;
}

Connection& Cluster::node(int32_t node_id) {
  auto it = conns_.find(node_id);
  if (it != conns_.end()) return *it->second;
  auto nit = nodes_.find(node_id);
  if (nit == nodes_.end()) throw KafkaError(-1, "unknown broker node " + std::to_string(node_id));
  auto c = std::make_unique<Connection>(nit->second.host, nit->second.port, cfg_);
  check_versions(*c);
  Connection& ref = *c;
  conns_[node_id] = std::move(c);
  return ref;
}

Connection& Cluster::coordinator(const std::string& group) {
  auto it = coordinators_.find(group);
  if (it == coordinators_.end()) {
    FindCoordinatorRequest req;
    req.key = group;
    Writer w;
    encode_find_coordinator_request(w, req);
    const std::string resp = any().request(FIND_COORDINATOR, w);
    Reader r(resp);
    const FindCoordinatorResponse m = decode_find_coordinator_response(r);
    if (m.error != NONE) throw KafkaError(m.error, "FindCoordinator: " + std::string(error_name(m.error)));
    nodes_[m.node.node_id] = m.node;
    it = coordinators_.emplace(group, m.node.node_id).first;
  }
  return node(it->second);
}

std::vector<BrokerNode> Cluster::brokers() const {
  std::vector<BrokerNode> v;
  for (auto& kv : nodes_) v.push_back(kv.second);
  return v;
}

// ---------------------------------------------------------------------------------------------
// Producer
// ---------------------------------------------------------------------------------------------

int32_t murmur2(const uint8_t* data, size_t n) {
  const uint32_t m = 0x5bd1e995;
  const int r = 24;
  uint32_t h = 0x9747b28cu ^ (uint32_t)n;
  const size_t n4 = n / 4;
  for (size_t i = 0; i < n4; ++i) {
    uint32_t k = (uint32_t)data[4 * i] | ((uint32_t)data[4 * i + 1] << 8) |
                 ((uint32_t)data[4 * i + 2] << 16) | ((uint32_t)data[4 * i + 3] << 24);
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
  }
  const size_t t = n & ~(size_t)3;
  switch (n % 4) {
    case 3: h ^= (uint32_t)data[t + 2] << 16; [[fallthrough]];
    case 2: h ^= (uint32_t)data[t + 1] << 8; [[fallthrough]];
    case 1: h ^= (uint32_t)data[t]; h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

Producer::Producer(ProducerConfig cfg)
    : cfg_(std::move(cfg)), cluster_(cfg_), meta_(cfg_),
      fault_state_(cfg_.fail_seed * 0x9e3779b97f4a7c15ull + 1) {
  if (cfg_.acks != 0 && cfg_.acks != 1 && cfg_.acks != -1)
    throw std::invalid_argument("acks must be 0, 1 or -1");
  if (cfg_.retries < 0 || cfg_.retry_backoff_ms < 0 || cfg_.delivery_timeout_ms <= 0)
    throw std::invalid_argument("retries / retry_backoff_ms must be >= 0, delivery_timeout_ms > 0");
  thread_ = std::thread([this] {
    name_thread("gl-sink");
    run();
  });
}

Producer::~Producer() {
  try {
    close();
  } catch (...) {
  }
}

int Producer::partitions_for(const std::string& topic) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = nparts_.find(topic);
  if (it != nparts_.end()) return it->second;
  const int n = meta_.partitions(topic);
  if (n > 0) nparts_[topic] = n;
  return n;
}

int Producer::choose_partition(const std::string& topic, const std::string* key) {  // mu_ held
  auto it = nparts_.find(topic);
  int n;
  if (it == nparts_.end()) {
    n = meta_.partitions(topic);
    if (n <= 0) throw KafkaError(UNKNOWN_TOPIC_OR_PARTITION, "unknown topic " + topic);
    nparts_[topic] = n;
  } else {
    n = it->second;
  }
  if (key)
    return (int)((uint32_t)murmur2(reinterpret_cast<const uint8_t*>(key->data()), key->size()) &
                 0x7fffffffu) % n;
  return (int)((rr_++ & 0x7fffffffu) % (uint32_t)n);
}

// Upper bound of one record's encoded size in a RecordBatch v2: the varint fields (length,
// attributes, timestamp / offset deltas, key / value lengths, header count) take at most 36
// bytes, each header at most 10 more besides its key and value. Chunks are cut on this bound so
// an encoded batch never exceeds max_request_size (headers such as __TypeId__ included).
static size_t record_bound(const std::string& key, const std::string& value,
                           const std::vector<Header>& headers) {
  size_t n = key.size() + value.size() + 36;
  for (const Header& h : headers) n += h.key.size() + h.value.size() + 10;
  return n;
}

// request bytes outside the records: request header, topic / partition framing and the
// 61-byte RecordBatch header
static constexpr size_t kRequestOverhead = 1024;

void Producer::send(const std::string& topic, int partition, const std::string* key,
                    std::string value, bool value_null, std::vector<Header> headers,
                    int64_t timestamp, SendCallback cb) {
  std::unique_lock<std::mutex> lk(mu_);
  if (closing_) throw std::runtime_error("producer is closed");
  if (partition < 0) partition = choose_partition(topic, key);
  done_cv_.wait(lk, [&] { return unsent_bytes_ < cfg_.buffer_memory || closing_; });
  Pending p;
  if (key) {
    p.key = *key;
    p.key_null = false;
  }
  p.value = std::move(value);
  p.value_null = value_null;
  p.headers = std::move(headers);
  p.ts = timestamp >= 0 ? timestamp : wall_ms();
  p.cb = std::move(cb);
  p.enq_ms = mono_ms();
  const size_t sz = record_bound(p.key, p.value, p.headers);
  PartBatch& b = acc_[{topic, partition}];
  if (b.recs.empty()) b.first_ms = mono_ms();
  b.bytes += sz;
  b.recs.push_back(std::move(p));
  unsent_bytes_ += (int64_t)sz;
  ++outstanding_;
  ++stats_.records_sent;
  if (b.bytes >= (size_t)cfg_.batch_size || cfg_.linger_ms <= 0) cv_.notify_one();
}

void Producer::send_group(const std::string& topic, int partition, RecordGroup g,
                          GroupCallback cb) {
  const size_t n = g.size();
  if (n == 0) return;
  if (partition < 0) {
    // the partitioner's choice is per record (kafka-clients 0.11: round-robin for null keys,
    // murmur2 of the key otherwise): split into one sub-group per partition, acknowledged
    // together once every sub-group is
    std::vector<int> part(n);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (closing_) throw std::runtime_error("producer is closed");
      for (size_t i = 0; i < n; ++i) {
        std::string key;
        const bool keyed = !g.koff.empty() && !g.key_null[i];
        if (keyed) key.assign(g.keys, g.koff[i], g.koff[i + 1] - g.koff[i]);
        part[i] = choose_partition(topic, keyed ? &key : nullptr);
      }
    }
    std::map<int, RecordGroup> subs;
    for (size_t i = 0; i < n; ++i) {
      RecordGroup& s = subs[part[i]];
      if (s.off.empty()) {
        s.off.push_back(0);
        if (!g.koff.empty()) s.koff.push_back(0);
        s.headers = g.headers;
        s.ts = g.ts;
      }
      s.values.append(g.values, g.off[i], g.off[i + 1] - g.off[i]);
      s.off.push_back((uint32_t)s.values.size());
      if (!g.null_value.empty()) {
        if (s.null_value.empty()) s.null_value.assign(s.off.size() - 2, 0);
        s.null_value.push_back(g.null_value[i]);
      } else if (!s.null_value.empty()) {
        s.null_value.push_back(0);
      }
      if (!g.koff.empty()) {
        s.keys.append(g.keys, g.koff[i], g.koff[i + 1] - g.koff[i]);
        s.koff.push_back((uint32_t)s.keys.size());
        s.key_null.push_back(g.key_null[i]);
      }
    }
    if (subs.size() > 1) {
      struct Join {
        std::mutex mu;
        size_t left;
        int16_t err = 0;
        GroupCallback cb;
      };
      auto j = std::make_shared<Join>();
      j->left = subs.size();
      j->cb = std::move(cb);
      for (auto& kv : subs)
        send_group(topic, kv.first, std::move(kv.second),
                   [j, n](int16_t err, int32_t, int64_t, size_t) {
                     bool last;
                     int16_t e;
                     {
                       std::lock_guard<std::mutex> lk(j->mu);
                       if (err && !j->err) j->err = err;
                       last = --j->left == 0;
                       e = j->err;
                     }
                     if (last && j->cb) j->cb(e, -1, -1, n);
                   });
      return;
    }
    partition = subs.begin()->first;
    g = std::move(subs.begin()->second);
  }
  size_t sz = 0;
  for (size_t i = 0; i < n; ++i) {
    sz += (size_t)(g.off[i + 1] - g.off[i]) + 36;
    if (!g.koff.empty()) sz += (size_t)(g.koff[i + 1] - g.koff[i]);
    for (const Header& h : g.headers) sz += h.key.size() + h.value.size() + 10;
  }
  std::unique_lock<std::mutex> lk(mu_);
  if (closing_) throw std::runtime_error("producer is closed");
  done_cv_.wait(lk, [&] { return unsent_bytes_ < cfg_.buffer_memory || closing_; });
  Pending p;
  p.ts = g.ts >= 0 ? g.ts : wall_ms();
  p.group = std::make_unique<RecordGroup>(std::move(g));
  p.gcb = std::move(cb);
  p.enq_ms = mono_ms();
  PartBatch& b = acc_[{topic, partition}];
  if (b.recs.empty()) b.first_ms = mono_ms();
  b.bytes += sz;
  b.recs.push_back(std::move(p));
  unsent_bytes_ += (int64_t)sz;
  outstanding_ += (int64_t)n;
  stats_.records_sent += (int64_t)n;
  if (b.bytes >= (size_t)cfg_.batch_size || cfg_.linger_ms <= 0) cv_.notify_one();
}

// bytes an entry was charged to unsent_bytes_ (and to its chunk)
static size_t pending_bound(const std::string& key, const std::string& value,
                            const std::vector<Header>& headers, const RecordGroup* g) {
  if (!g) return record_bound(key, value, headers);
  size_t sz = 0;
  const size_t n = g->size();
  for (size_t i = 0; i < n; ++i) {
    sz += (size_t)(g->off[i + 1] - g->off[i]) + 36;
    if (!g->koff.empty()) sz += (size_t)(g->koff[i + 1] - g->koff[i]);
    for (const Header& h : g->headers) sz += h.key.size() + h.value.size() + 10;
  }
  return sz;
}

void Producer::flush() {
  std::unique_lock<std::mutex> lk(mu_);
  flush_req_ = true;
  cv_.notify_one();
  done_cv_.wait(lk, [&] { return outstanding_ == 0; });
  flush_req_ = false;
}

void Producer::close() {
  {
    std::unique_lock<std::mutex> lk(mu_);
    if (closing_ && !thread_.joinable()) return;
  }
  flush();
  {
    std::lock_guard<std::mutex> lk(mu_);
    closing_ = true;
  }
  cv_.notify_all();
  done_cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

ProducerStats Producer::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

void Producer::run() {
  std::deque<InFlight> inflight;
  using TP = std::pair<std::string, int>;
  // a request's outcome for one partition's chunk: retriable failures of records that still have
  // attempts and time left wait in retry_ for their backoff; everything else is final
  auto complete = [&](const TP& tp, std::vector<Pending>& recs, int16_t err, int64_t base) {
    if (err != NONE && error_retriable(err) && cfg_.retries > 0) {
      const int64_t now = mono_ms();
      std::vector<Pending> again, last;
      int64_t n_again = 0;
      for (auto& p : recs) {
        if (p.attempts < cfg_.retries && now - p.enq_ms < cfg_.delivery_timeout_ms) {
          ++p.attempts;
          n_again += (int64_t)p.records();
          again.push_back(std::move(p));
        } else {
          last.push_back(std::move(p));
        }
      }
      if (!again.empty()) {
        retry_.push_back(Retry{tp, std::move(again), now + cfg_.retry_backoff_ms});
        std::lock_guard<std::mutex> lk(mu_);
        stats_.records_retried += n_again;
        ++stats_.requests_failed;
      }
      if (last.empty()) return;
      recs = std::move(last);
    }
    int64_t idx = 0;
    for (size_t i = 0; i < recs.size(); ++i) {
      const int64_t off = (err == NONE && base >= 0) ? base + idx : -1;
      if (recs[i].group) {
        if (recs[i].gcb) {
          try {
            recs[i].gcb(err, tp.second, off, recs[i].group->size());
          } catch (...) {
          }
        }
      } else if (recs[i].cb) {
        SendResult r;
        r.error = err;
        r.partition = tp.second;
        r.offset = off;
        try {
          recs[i].cb(r);
        } catch (...) {
        }
      }
      idx += (int64_t)recs[i].records();
    }
    std::lock_guard<std::mutex> lk(mu_);
    outstanding_ -= idx;
    if (err == NONE) stats_.records_acked += idx;
    else stats_.records_failed += idx;
    done_cv_.notify_all();
  };
  // a node's connection broke (or is mid-response): every request still in flight on it is
  // lost with it; the next request to the node reconnects
  auto lose_node = [&](int32_t node) {
    for (auto it = inflight.begin(); it != inflight.end();) {
      if (it->node == node) {
        for (auto& b : it->batches) complete(b.first, b.second, NETWORK_EXCEPTION, -1);
        it = inflight.erase(it);
      } else {
        ++it;
      }
    }
    cluster_.drop(node);
    cluster_.invalidate();
  };
  auto read_one = [&]() {
    InFlight f = std::move(inflight.front());
    inflight.pop_front();
    size_t n = 0;
    std::shared_ptr<uint8_t> buf;
    try {
      buf = cluster_.node(f.node).recv(f.corr, &n, heap_alloc);
    } catch (const std::exception&) {
      for (auto& b : f.batches) complete(b.first, b.second, REQUEST_TIMED_OUT, -1);
      lose_node(f.node);
      return;
    }
    Reader r(buf.get(), n);
    const ProduceResponse resp = decode_produce_response(r);
    for (auto& b : f.batches) {
      int16_t err = UNKNOWN_SERVER_ERROR;
      int64_t base = -1;
      for (const auto& t : resp.topics)
        if (t.name == b.first.first)
          for (const auto& p : t.partitions)
            if (p.index == b.first.second) {
              err = p.error;
              base = p.base_offset;
            }
      if (err != NONE) cluster_.invalidate();
      complete(b.first, b.second, err, base);
    }
  };

  for (;;) {
    std::vector<std::pair<std::pair<std::string, int>, std::vector<Pending>>> ready;
    bool stop = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      for (;;) {
        const int64_t now = mono_ms();
        int64_t next = INT64_MAX;
        // retries whose backoff ended go first (ahead of newer records of their partition)
        for (auto it = retry_.begin(); it != retry_.end();) {
          if (it->due_ms <= now) {
            ready.push_back({it->tp, std::move(it->recs)});
            it = retry_.erase(it);
          } else {
            next = std::min(next, it->due_ms);
            ++it;
          }
        }
        for (auto it = acc_.begin(); it != acc_.end();) {
          PartBatch& b = it->second;
          if (b.recs.empty()) {
            it = acc_.erase(it);
            continue;
          }
          if (flush_req_ || closing_ || b.bytes >= (size_t)cfg_.batch_size ||
              now - b.first_ms >= cfg_.linger_ms) {
            // drained as batches of at most max_request_size (at least one record each): what
            // accumulated behind a busy sender leaves in request-sized batches, so a request
            // (and the bytes awaiting acks, max_in_flight of them) stays bounded instead of
            // growing with the backlog (one 30 MB batch per request was 0.5-1 s of ack latency
            // at saturation, profiles/archive/r2_producer_request_ab.txt)
            size_t total = 0;
            std::vector<Pending> chunk;
            size_t cbytes = 0;
            const size_t cap = (size_t)cfg_.max_request_size > 2 * kRequestOverhead
                                   ? (size_t)cfg_.max_request_size - kRequestOverhead
                                   : (size_t)cfg_.max_request_size / 2;
            for (auto& p : b.recs) {
              const size_t sz = pending_bound(p.key, p.value, p.headers, p.group.get());
              if (!chunk.empty() && cbytes + sz > cap) {
                ready.push_back({it->first, std::move(chunk)});
                chunk.clear();
                cbytes = 0;
              }
              chunk.push_back(std::move(p));
              cbytes += sz;
              total += sz;
            }
            if (!chunk.empty()) ready.push_back({it->first, std::move(chunk)});
            unsent_bytes_ -= (int64_t)total;
            it = acc_.erase(it);
          } else {
            next = std::min(next, b.first_ms + cfg_.linger_ms);
            ++it;
          }
        }
        if (!ready.empty()) {
          done_cv_.notify_all();
          break;
        }
        if (!inflight.empty()) break;
        if (closing_ && retry_.empty()) {
          stop = true;
          break;
        }
        if (next == INT64_MAX) cv_.wait(lk);
        else cv_.wait_for(lk, std::chrono::milliseconds(std::max<int64_t>(1, next - now)));
      }
    }
    if (stop) return;
    // group by leader and send (one request per node, split at max_request_size)
    std::map<int32_t, std::vector<size_t>> by_node;
    for (size_t i = 0; i < ready.size(); ++i) {
      try {
        by_node[cluster_.leader(ready[i].first.first, ready[i].first.second)].push_back(i);
      } catch (const KafkaError& e) {
        complete(ready[i].first, ready[i].second, (int16_t)e.code, -1);
        cluster_.invalidate();
      }
    }
    for (auto& kv : by_node) {
      size_t k = 0;
      while (k < kv.second.size()) {
        ProduceRequest req;
        req.acks = (int16_t)cfg_.acks;
        req.timeout_ms = cfg_.request_timeout_ms;
        InFlight f;
        f.node = kv.first;
        size_t bytes = 0;
        for (; k < kv.second.size(); ++k) {
          auto& item = ready[kv.second[k]];
          // one batch per partition per request (consecutive chunks of one partition's backlog
          // go in separate requests, in order)
          bool dup = false;
          for (const auto& fb : f.batches) dup |= fb.first == item.first;
          if (dup) break;
          std::vector<RecordIn> ins;
          ins.reserve(item.second.size());
          for (size_t j = 0; j < item.second.size(); ++j) {
            const Pending& p = item.second[j];
            if (p.group) {
              const RecordGroup& g = *p.group;
              for (size_t i = 0; i < g.size(); ++i) {
                RecordIn r;
                r.value = std::string_view(g.values).substr(g.off[i], g.off[i + 1] - g.off[i]);
                r.value_null = !g.null_value.empty() && g.null_value[i];
                if (!g.koff.empty() && !g.key_null[i]) {
                  r.key = std::string_view(g.keys).substr(g.koff[i], g.koff[i + 1] - g.koff[i]);
                  r.key_null = false;
                }
                r.timestamp = p.ts;
                r.headers = g.headers.empty() ? nullptr : &g.headers;
                ins.push_back(r);
              }
              continue;
            }
            RecordIn r;
            r.key = p.key;
            r.key_null = p.key_null;
            r.value = p.value;
            r.value_null = p.value_null;
            r.timestamp = p.ts;
            r.headers = p.headers.empty() ? nullptr : &p.headers;
            ins.push_back(r);
          }
          Writer bw;
          encode_batch(bw, ins.data(), ins.size(), 0, item.second.front().ts);
          if (cfg_.compression != CODEC_NONE) bw.buf = compress_batch(bw.buf, cfg_.compression);
          if (bytes && bytes + bw.size() > (size_t)cfg_.max_request_size) break;
          bytes += bw.size();
          ProduceTopic* pt = nullptr;
          for (auto& t : req.topics)
            if (t.name == item.first.first) pt = &t;
          if (!pt) {
            req.topics.push_back(ProduceTopic{item.first.first, {}});
            pt = &req.topics.back();
          }
          ProducePartition pp;
          pp.index = item.first.second;
          pp.records = std::move(bw.buf);
          pt->partitions.push_back(std::move(pp));
          f.batches.push_back({item.first, std::move(item.second)});
        }
        Writer w;
        encode_produce_request(w, req);
        if (cfg_.fail_p > 0) {  // injected loss of the request (never reaches the broker)
          fault_state_ ^= fault_state_ << 13;
          fault_state_ ^= fault_state_ >> 7;
          fault_state_ ^= fault_state_ << 17;
          if ((double)(fault_state_ >> 11) * 0x1.0p-53 < cfg_.fail_p) {
            for (auto& b : f.batches) complete(b.first, b.second, NETWORK_EXCEPTION, -1);
            continue;
          }
        }
        try {
          Connection& c = cluster_.node(kv.first);
          f.corr = c.send(PRODUCE, w);
          {
            std::lock_guard<std::mutex> lk(mu_);
            ++stats_.requests;
            stats_.bytes += (int64_t)w.size();
          }
        } catch (const std::exception&) {
          for (auto& b : f.batches) complete(b.first, b.second, NETWORK_EXCEPTION, -1);
          lose_node(kv.first);
          continue;
        }
        if (cfg_.acks == 0) {
          for (auto& b : f.batches) complete(b.first, b.second, NONE, -1);
        } else {
          inflight.push_back(std::move(f));
          if ((int)inflight.size() >= cfg_.max_in_flight) read_one();
        }
      }
    }
    // read responses when there is nothing new to send
    bool more;
    {
      std::lock_guard<std::mutex> lk(mu_);
      more = false;
      for (auto& kv : acc_)
        if (!kv.second.recs.empty() &&
            (flush_req_ || closing_ || kv.second.bytes >= (size_t)cfg_.batch_size ||
             cfg_.linger_ms <= 0))
          more = true;
    }
    if (!more) {
      while (!inflight.empty()) read_one();
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Consumer
// ---------------------------------------------------------------------------------------------

Consumer::Consumer(ConsumerConfig cfg, BufferAlloc alloc)
    : cfg_(std::move(cfg)), alloc_(std::move(alloc)), cluster_(cfg_) {}

void Consumer::assign(const std::string& topic, const std::vector<int>& partitions) {
  drain();
  ready_.clear();
  topic_ = topic;
  const int n = cluster_.partitions(topic);
  if (n < 0) throw KafkaError(UNKNOWN_TOPIC_OR_PARTITION, "unknown topic " + topic);
  parts_.clear();
  if (partitions.empty()) {
    for (int p = 0; p < n; ++p) parts_.push_back(p);
  } else {
    for (int p : partitions) {
      if (p < 0 || p >= n)
        throw KafkaError(UNKNOWN_TOPIC_OR_PARTITION,
                         "partition " + std::to_string(p) + " not in " + topic);
      parts_.push_back(p);
    }
  }
  pos_.clear();
}

int64_t Consumer::list_offset(int partition, int64_t ts) {
  ListOffsetsRequest req;
  req.topics.push_back({topic_, {{partition, ts}}});
  Writer w;
  encode_list_offsets_request(w, req);
  const std::string resp = cluster_.node(cluster_.leader(topic_, partition)).request(LIST_OFFSETS, w);
  Reader r(resp);
  const ListOffsetsResponse m = decode_list_offsets_response(r);
  for (auto& t : m.topics)
    for (auto& p : t.partitions)
      if (p.index == partition) {
        if (p.error != NONE) throw KafkaError(p.error, "ListOffsets: " + std::string(error_name(p.error)));
        return p.offset;
      }
  throw KafkaError(-1, "ListOffsets: partition missing from response");
}

void Consumer::seek(int partition, int64_t offset) {
  drain();
  ready_.clear();  // nothing fetched before a seek may be returned after it
  pos_[partition] = offset;
}

int64_t Consumer::position(int partition) const {
  auto it = pos_.find(partition);
  return it == pos_.end() ? -1 : it->second;
}

void Consumer::seek_to(const std::string& where) {
  drain();
  ready_.clear();
  for (int p : parts_) {
    if (where == "latest") {
      pos_[p] = list_offset(p, kLatest);
    } else if (where == "earliest") {
      pos_[p] = list_offset(p, kEarliest);
    } else if (where == "committed") {
      const int64_t c = cfg_.group_id.empty() ? -1 : committed(p);
      pos_[p] = c >= 0 ? c : list_offset(p, cfg_.auto_offset_reset == "earliest" ? kEarliest : kLatest);
    } else {
      throw std::invalid_argument("seek_to: expected latest|earliest|committed, got " + where);
    }
  }
}

void Consumer::send_fetches() {
  std::map<int32_t, std::vector<int>> by_leader;
  for (int p : parts_) {
    try {
      by_leader[cluster_.leader(topic_, p)].push_back(p);
    } catch (const KafkaError&) {
      cluster_.invalidate();
    }
  }
  // issue every leader's fetch first (long polls run concurrently), then collect
  for (auto& kv : by_leader) {
    FetchRequest req;
    req.max_wait_ms = cfg_.max_wait_ms;
    req.min_bytes = cfg_.min_bytes;
    req.max_bytes = cfg_.fetch_max_bytes;
    FetchTopic ft;
    ft.name = topic_;
    InFlight inf;
    inf.node = kv.first;
    for (int p : kv.second) {
      ft.partitions.push_back({p, pos_[p], cfg_.partition_max_bytes});
      inf.from[p] = pos_[p];
    }
    req.topics.push_back(std::move(ft));
    Writer w;
    encode_fetch_request(w, req);
    inf.corr = cluster_.node(kv.first).send(FETCH, w);
    inflight_.push_back(std::move(inf));
  }
}

void Consumer::collect(std::vector<Fetched>& out) {
  std::vector<InFlight> infs;
  infs.swap(inflight_);
  bool stale = false;
  for (size_t i = 0; i < infs.size(); ++i) {
    const InFlight& inf = infs[i];
    Fetched f;
    f.crc_checked = cfg_.check_crcs;
    try {
      f.buf = cluster_.node(inf.node).recv(inf.corr, &f.size, alloc_, tap_.get(), &f.tap_result);
      if (tap_ && tap_->sparse()) {
        f.sparse = true;
        f.restorer = tap_;
      }
    } catch (...) {
      // these connections are mid-response: reconnect them, forget their in-flight fetches
      for (size_t j = i; j < infs.size(); ++j) cluster_.drop(infs[j].node);
      cluster_.invalidate();
      throw;
    }
    Reader r(f.buf.get(), f.size);
    const FetchResponse m = decode_fetch_response(r);
    // partitions whose records are not plain v2 batches: normalised copies (compress.h),
    // appended behind the response body once every partition was looked at
    struct Conv {
      int partition;
      std::string blob;
    };
    std::vector<Conv> convs;
    for (auto& t : m.topics)
      for (auto& p : t.partitions) {
        auto it = inf.from.find(p.index);
        if (it == inf.from.end() || pos_[p.index] != it->second) continue;  // seeked meanwhile
        if (p.error == OFFSET_OUT_OF_RANGE) {
          pos_[p.index] = list_offset(p.index, cfg_.auto_offset_reset == "earliest" ? kEarliest : kLatest);
          continue;
        }
        if (p.error != NONE) {
          stale = true;
          continue;
        }
        hw_[p.index] = p.high_watermark;
        if (p.records_len <= 0) continue;
        const size_t before = f.records.size(), bbefore = f.batches.size();
        try {
          decode_records(f.buf.get(), p.records_off, (size_t)p.records_len, pos_[p.index],
                         cfg_.check_crcs, f.records, &f.batches);
        } catch (const ProtocolError&) {
          // compressed / legacy / corrupt: never thrown out of poll (that would retry the same
          // position forever); the partition's records are rewritten as plain v2 batches, with
          // undecodable batches as poison records that advance the position
          f.records.resize(before);
          f.batches.resize(bbefore);
          f.restore();  // (the rewrite copies values: they must be whole on the host)
          NormalizeStats ns;
          std::string blob = normalize_records(f.buf.get() + p.records_off, (size_t)p.records_len,
                                               pos_[p.index], cfg_.check_crcs,
                                               cfg_.max_decompressed_bytes, ns);
          converted_batches_ += ns.converted_batches;
          poison_batches_ += ns.poison_batches;
          poison_records_ += ns.poison_records;
          poison_unknown_span_ += ns.poison_unknown_span;
          if (ns.poison_batches && poison_logged_ < 16) {
            ++poison_logged_;
            fprintf(stderr, "[gale consumer] %s-%d: %lld undecodable batch(es) from offset %lld "
                    "skipped as %lld poison record(s): %s\n", topic_.c_str(), p.index,
                    (long long)ns.poison_batches, (long long)pos_[p.index],
                    (long long)ns.poison_records, ns.last_error.c_str());
          }
          if (!blob.empty()) convs.push_back({p.index, std::move(blob)});
          continue;
        }
        for (size_t k = before; k < f.records.size(); ++k) f.records[k].partition = p.index;
        if (f.records.size() > before) pos_[p.index] = f.records.back().offset + 1;
      }
    if (!convs.empty()) {
      // one buffer: [response body][normalised blobs], so every record still points into ONE
      // buffer (pinned when the pool's chunk fits it; the device-side packed copy of the body,
      // if any, does not describe the new buffer)
      size_t total = (f.size + 15) & ~(size_t)15;
      for (const Conv& c : convs) total += (c.blob.size() + 15) & ~(size_t)15;
      std::shared_ptr<uint8_t> nb = alloc_(total);
      memcpy(nb.get(), f.buf.get(), f.size);
      size_t at = (f.size + 15) & ~(size_t)15;
      f.buf = nb;
      f.tap_result = -1;
      f.sparse = false;
      for (const Conv& c : convs) {
        memcpy(nb.get() + at, c.blob.data(), c.blob.size());
        const size_t before = f.records.size();
        decode_records(nb.get(), at, c.blob.size(), pos_[c.partition], false, f.records,
                       &f.batches, /*honor_poison=*/true);
        for (size_t k = before; k < f.records.size(); ++k) f.records[k].partition = c.partition;
        if (f.records.size() > before) pos_[c.partition] = f.records.back().offset + 1;
        at += (c.blob.size() + 15) & ~(size_t)15;
      }
      f.size = at;
    }
    if (!f.records.empty()) out.push_back(std::move(f));
  }
  if (stale) cluster_.invalidate();
}

void Consumer::drain() {
  if (!inflight_.empty()) collect(ready_);
}

std::vector<Fetched> Consumer::poll() {
  std::vector<Fetched> out;
  out.swap(ready_);
  if (!out.empty()) {  // responses drained by an earlier commit
    if (cfg_.prefetch && inflight_.empty()) send_fetches();
    return out;
  }
  for (int p : parts_)
    if (!pos_.count(p)) pos_[p] = list_offset(p, cfg_.auto_offset_reset == "earliest" ? kEarliest : kLatest);
  if (inflight_.empty()) send_fetches();
  collect(out);
  if (cfg_.prefetch) send_fetches();
  return out;
}

void Consumer::commit(const std::map<int, int64_t>& offsets) {
  if (cfg_.group_id.empty()) throw std::invalid_argument("commit needs a group_id");
  if (offsets.empty()) return;
  drain();  // the coordinator may share a connection with an in-flight fetch
  OffsetCommitRequest req;
  req.group_id = cfg_.group_id;
  req.generation_id = generation_;
  req.member_id = member_id_;
  CommitTopic t;
  t.name = topic_;
  for (auto& kv : offsets) {
    CommitPartition cp;
    cp.index = kv.first;
    cp.offset = kv.second;
    t.partitions.push_back(cp);
  }
  req.topics.push_back(std::move(t));
  Writer w;
  encode_offset_commit_request(w, req);
  const std::string resp = cluster_.coordinator(cfg_.group_id).request(OFFSET_COMMIT, w);
  Reader r(resp);
  for (auto& ct : decode_offset_commit_response(r))
    for (auto& cp : ct.partitions)
      if (cp.error != NONE)
        throw KafkaError(cp.error, std::string("OffsetCommit failed: ") + error_name(cp.error));
}

// ---------------------------------------------------------------------------------------------
// GroupMember
// ---------------------------------------------------------------------------------------------

std::string encode_member_load(const MemberLoad& m) {
  Writer w;
  w.i16(1);  // version
  w.i64((int64_t)(m.capacity * 1000.0));  // milli-records/s
  w.array_len((int32_t)m.owned.size());
  for (int32_t p : m.owned) w.i32(p);
  return w.buf;
}

MemberLoad decode_member_load(const std::string& b) {
  MemberLoad m;
  if (b.size() < 14) return m;
  try {
    Reader r(b);
    if (r.i16() < 1) return m;
    m.capacity = (double)r.i64() / 1000.0;
    const int32_t n = r.i32();
    for (int32_t i = 0; i < n && r.remaining() >= 4; ++i) m.owned.push_back(r.i32());
  } catch (const ProtocolError&) {
    m = MemberLoad();
  }
  return m;
}

std::map<std::string, std::vector<int>> GroupMember::assign_load_aware(
    std::vector<std::string> members, const std::map<std::string, MemberLoad>& load, int n) {
  std::sort(members.begin(), members.end());
  std::map<std::string, std::vector<int>> out;
  for (const auto& m : members) out[m];
  if (members.empty() || n <= 0) return out;
  const size_t k = members.size();
  std::vector<double> cap(k, 0.0);
  double known = 0;
  int nknown = 0;
  for (size_t i = 0; i < k; ++i) {
    auto it = load.find(members[i]);
    if (it != load.end() && it->second.capacity > 0) {
      cap[i] = it->second.capacity;
      known += cap[i];
      ++nknown;
    }
  }
  const double fill = nknown ? known / nknown : 1.0;
  double total = 0;
  for (double& c : cap) {
    if (c <= 0) c = fill;
    total += c;
  }
  // quotas: partitions one at a time to the member whose utilisation (partitions per unit of
  // capacity) stays lowest after taking it (D'Hondt / Jefferson apportionment): this minimises
  // the most loaded member's partitions / capacity, so a slow member is never rounded up past
  // what it can serve while faster members have room (ties: the faster, then the first member)
  std::vector<int> quota(k, 0);
  for (int p = 0; p < n; ++p) {
    size_t best = 0;
    for (size_t i = 1; i < k; ++i) {
      const double a = (quota[i] + 1) / cap[i], b = (quota[best] + 1) / cap[best];
      if (a < b - 1e-12 || (std::abs(a - b) <= 1e-12 && cap[i] > cap[best])) best = i;
    }
    ++quota[best];
  }
  // sticky fill: current owners keep partitions up to their quota
  std::vector<int> owner(n, -1), count(k, 0);
  for (size_t i = 0; i < k; ++i) {
    auto it = load.find(members[i]);
    if (it == load.end()) continue;
    std::vector<int32_t> own = it->second.owned;
    std::sort(own.begin(), own.end());
    for (int32_t p : own)
      if (p >= 0 && p < n && owner[p] < 0 && count[i] < quota[i]) {
        owner[p] = (int)i;
        ++count[i];
      }
  }
  for (int p = 0; p < n; ++p) {
    if (owner[p] >= 0) continue;
    size_t best = 0;
    for (size_t i = 1; i < k; ++i)
      if (quota[i] - count[i] > quota[best] - count[best]) best = i;
    owner[p] = (int)best;
    ++count[best];
  }
  for (int p = 0; p < n; ++p) out[members[(size_t)owner[p]]].push_back(p);
  return out;
}

GroupMember::GroupMember(GroupConfig cfg) : cfg_(std::move(cfg)), cluster_(cfg_) {
  if (cfg_.group_id.empty() || cfg_.topic.empty())
    throw std::invalid_argument("GroupMember needs a group_id and a topic");
  if (cfg_.assignor != "range" && cfg_.assignor != "roundrobin" &&
      cfg_.assignor != "load-aware")
    throw std::invalid_argument("assignor must be range|roundrobin|load-aware");
  // JoinGroup blocks for up to the rebalance timeout: the socket timeout must outlast it
  ClientConfig cc = cfg_;
  cc.request_timeout_ms = std::max(cfg_.request_timeout_ms, cfg_.rebalance_timeout_ms + 5000);
  cluster_ = Cluster(cc);
}

GroupMember::~GroupMember() {
  try {
    leave();
  } catch (...) {
  }
}

std::map<std::string, std::vector<int>> GroupMember::assign(const std::string& assignor,
                                                            std::vector<std::string> members,
                                                            int n) {
  std::sort(members.begin(), members.end());
  std::map<std::string, std::vector<int>> out;
  for (const auto& m : members) out[m];
  if (members.empty()) return out;
  const int k = (int)members.size();
  if (assignor == "roundrobin") {
    for (int p = 0; p < n; ++p) out[members[(size_t)(p % k)]].push_back(p);
  } else {  // range: contiguous blocks, the first n % k members take one extra
    int p = 0;
    for (int i = 0; i < k; ++i) {
      const int cnt = n / k + (i < n % k ? 1 : 0);
      for (int j = 0; j < cnt; ++j) out[members[(size_t)i]].push_back(p++);
    }
  }
  return out;
}

std::vector<int> GroupMember::join() {
  for (int attempt = 0;; ++attempt) {
    if (attempt > 50) throw KafkaError(REBALANCE_IN_PROGRESS, "group join did not converge");
    JoinGroupRequest jr;
    jr.group_id = cfg_.group_id;
    jr.session_timeout_ms = cfg_.session_timeout_ms;
    jr.rebalance_timeout_ms = cfg_.rebalance_timeout_ms;
    jr.member_id = member_id_;
    ConsumerSubscription sub;
    sub.topics = {cfg_.topic};
    sub.user_data = user_data_;
    jr.protocols.push_back({cfg_.assignor, encode_subscription(sub)});
    Writer w;
    encode_join_group_request(w, jr);
    JoinGroupResponse resp;
    try {
      const std::string raw = cluster_.coordinator(cfg_.group_id).request(JOIN_GROUP, w);
      Reader r(raw);
      resp = decode_join_group_response(r);
    } catch (const KafkaError& e) {
      if (e.code != -1 && e.code != REQUEST_TIMED_OUT) throw;
      cluster_ = Cluster(cluster_.config());  // reconnect (the exchange may be half done)
      usleep(100000);
      continue;
    }
    if (resp.error == UNKNOWN_MEMBER_ID) {
      member_id_.clear();  // fenced: rejoin as a new member
      continue;
    }
    if (resp.error == REBALANCE_IN_PROGRESS) continue;
    if (resp.error != NONE)
      throw KafkaError(resp.error, std::string("JoinGroup: ") + error_name(resp.error));
    member_id_ = resp.member_id;
    generation_ = resp.generation_id;
    leader_ = resp.leader_id == resp.member_id;
    SyncGroupRequest sr;
    sr.group_id = cfg_.group_id;
    sr.generation_id = generation_;
    sr.member_id = member_id_;
    if (leader_) {
      std::vector<std::string> subscribed;
      std::map<std::string, MemberLoad> loads;
      for (const GroupMemberMeta& m : resp.members) {
        const ConsumerSubscription s = decode_subscription(m.metadata);
        if (std::find(s.topics.begin(), s.topics.end(), cfg_.topic) != s.topics.end()) {
          subscribed.push_back(m.member_id);
          loads[m.member_id] = decode_member_load(s.user_data);
        }
      }
      cluster_.invalidate();  // the partition count may have grown
      const int n = std::max(0, cluster_.partitions(cfg_.topic));
      const bool la = resp.protocol == "load-aware";
      // load-aware: every member learns its capacity share (unmeasured members count as the
      // mean of the measured ones, as in the assignor), so it can tell whether its lag is out
      // of proportion - only then can a new assignment help
      std::map<std::string, double> share;
      if (la) {
        double known = 0, total = 0;
        int nknown = 0;
        for (const auto& m : subscribed)
          if (loads[m].capacity > 0) {
            known += loads[m].capacity;
            ++nknown;
          }
        const double fill = nknown ? known / nknown : 1.0;
        for (const auto& m : subscribed) total += loads[m].capacity > 0 ? loads[m].capacity : fill;
        for (const auto& m : subscribed)
          share[m] = (loads[m].capacity > 0 ? loads[m].capacity : fill) / std::max(total, 1e-9);
      }
      for (auto& kv : la ? assign_load_aware(subscribed, loads, n)
                         : assign(resp.protocol, subscribed, n)) {
        ConsumerAssignment a;
        a.partitions.push_back({cfg_.topic, std::vector<int32_t>(kv.second.begin(),
                                                                 kv.second.end())});
        if (la) {
          Writer u;
          u.i16(1);  // version
          u.i64((int64_t)(share[kv.first] * 1e9));
          a.user_data = u.buf;
        }
        sr.assignments.push_back({kv.first, encode_assignment(a)});
      }
      for (const GroupMemberMeta& m : resp.members)  // members not on this topic: nothing
        if (std::find(subscribed.begin(), subscribed.end(), m.member_id) == subscribed.end())
          sr.assignments.push_back({m.member_id, encode_assignment(ConsumerAssignment())});
    }
    Writer w2;
    encode_sync_group_request(w2, sr);
    SyncGroupResponse sresp;
    try {
      const std::string raw = cluster_.coordinator(cfg_.group_id).request(SYNC_GROUP, w2);
      Reader r(raw);
      sresp = decode_sync_group_response(r);
    } catch (const KafkaError& e) {
      if (e.code != -1 && e.code != REQUEST_TIMED_OUT) throw;
      cluster_ = Cluster(cluster_.config());
      continue;
    }
    if (sresp.error == UNKNOWN_MEMBER_ID) {
      member_id_.clear();
      continue;
    }
    if (sresp.error == REBALANCE_IN_PROGRESS || sresp.error == ILLEGAL_GENERATION) continue;
    if (sresp.error != NONE)
      throw KafkaError(sresp.error, std::string("SyncGroup: ") + error_name(sresp.error));
    std::vector<int> mine;
    const ConsumerAssignment asg = decode_assignment(sresp.assignment);
    for (const auto& tp : asg.partitions)
      if (tp.first == cfg_.topic) mine.insert(mine.end(), tp.second.begin(), tp.second.end());
    std::sort(mine.begin(), mine.end());
    capacity_share_ = -1;
    if (asg.user_data.size() >= 10) {
      Reader u(asg.user_data);
      if (u.i16() == 1) capacity_share_ = (double)u.i64() * 1e-9;
    }
    return mine;
  }
}

std::map<int, int64_t> GroupMember::partition_lags() {
  std::map<int, int64_t> lag;
  const int n = cluster_.partitions(cfg_.topic);
  if (n <= 0) return lag;
  // committed offsets (one OffsetFetch to the coordinator)
  OffsetFetchRequest fr;
  fr.group_id = cfg_.group_id;
  CommitTopic ct;
  ct.name = cfg_.topic;
  for (int p = 0; p < n; ++p) {
    CommitPartition cp;
    cp.index = p;
    ct.partitions.push_back(cp);
  }
  fr.topics.push_back(std::move(ct));
  Writer w;
  encode_offset_fetch_request(w, fr);
  std::map<int, int64_t> committed;
  {
    const std::string resp = cluster_.coordinator(cfg_.group_id).request(OFFSET_FETCH, w);
    Reader r(resp);
    for (auto& t : decode_offset_fetch_response(r))
      for (auto& p : t.partitions) committed[p.index] = p.offset;
  }
  // log ends and starts (ListOffsets per partition leader)
  std::map<int32_t, std::vector<int>> by_leader;
  for (int p = 0; p < n; ++p) by_leader[cluster_.leader(cfg_.topic, p)].push_back(p);
  std::map<int, int64_t> end, start;
  for (auto& kv : by_leader) {
    for (int64_t ts : {kLatest, kEarliest}) {
      ListOffsetsRequest lr;
      ListOffsetsTopic lt;
      lt.name = cfg_.topic;
      for (int p : kv.second) lt.partitions.push_back({p, ts});
      lr.topics.push_back(std::move(lt));
      Writer lw;
      encode_list_offsets_request(lw, lr);
      const std::string resp = cluster_.node(kv.first).request(LIST_OFFSETS, lw);
      Reader r(resp);
      for (auto& t : decode_list_offsets_response(r).topics)
        for (auto& p : t.partitions)
          if (p.error == NONE) (ts == kLatest ? end : start)[p.index] = p.offset;
    }
  }
  for (int p = 0; p < n; ++p) {
    auto e = end.find(p);
    if (e == end.end()) continue;
    auto c = committed.find(p);
    const int64_t from = c != committed.end() && c->second >= 0 ? c->second : start[p];
    lag[p] = std::max<int64_t>(0, e->second - from);
  }
  return lag;
}

bool GroupMember::heartbeat() {
  if (member_id_.empty()) return false;
  HeartbeatRequest hr;
  hr.group_id = cfg_.group_id;
  hr.generation_id = generation_;
  hr.member_id = member_id_;
  Writer w;
  encode_heartbeat_request(w, hr);
  int16_t err;
  try {
    const std::string raw = cluster_.coordinator(cfg_.group_id).request(HEARTBEAT, w);
    Reader r(raw);
    err = decode_group_error_response(r);
  } catch (const KafkaError& e) {
    if (e.code != -1 && e.code != REQUEST_TIMED_OUT) throw;
    cluster_ = Cluster(cluster_.config());
    return true;  // transient: the session outlives one missed heartbeat
  }
  if (err == UNKNOWN_MEMBER_ID) member_id_.clear();
  if (err == NONE) return true;
  if (err == REBALANCE_IN_PROGRESS || err == ILLEGAL_GENERATION || err == UNKNOWN_MEMBER_ID)
    return false;
  throw KafkaError(err, std::string("Heartbeat: ") + error_name(err));
}

void GroupMember::leave() {
  if (member_id_.empty()) return;
  LeaveGroupRequest lr;
  lr.group_id = cfg_.group_id;
  lr.member_id = member_id_;
  member_id_.clear();
  generation_ = -1;
  Writer w;
  encode_leave_group_request(w, lr);
  cluster_.coordinator(cfg_.group_id).request(LEAVE_GROUP, w);
}

int64_t Consumer::committed(int partition) {
  drain();
  OffsetFetchRequest req;
  req.group_id = cfg_.group_id;
  CommitTopic t;
  t.name = topic_;
  CommitPartition cp;
  cp.index = partition;
  t.partitions.push_back(cp);
  req.topics.push_back(std::move(t));
  Writer w;
  encode_offset_fetch_request(w, req);
  const std::string resp = cluster_.coordinator(cfg_.group_id).request(OFFSET_FETCH, w);
  Reader r(resp);
  for (auto& ct : decode_offset_fetch_response(r))
    for (auto& p : ct.partitions)
      if (p.index == partition) return p.offset;
  return -1;
}

}  // namespace kafka
}  // namespace gale
