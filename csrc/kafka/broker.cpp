// Embedded Kafka-protocol broker (see broker.h).
#include "broker.h"
#include "gale/llc_pair.h"
#include "gale/thread_name.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <stdexcept>

namespace gale {
namespace kafka {

namespace {

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int64_t wall_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

bool valid_topic(const std::string& t) {
  if (t.empty() || t.size() > 249 || t == "." || t == "..") return false;
  for (char c : t)
    if (!(isalnum((unsigned char)c) || c == '.' || c == '_' || c == '-')) return false;
  return true;
}

void set_sock_opts(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  const int sz = socket_buffer_bytes();
  if (sz > 0) setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
  if (sz > 0) setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
}

std::string offset_key(const std::string& g, const std::string& t, int p) {
  std::string k = g;
  k.push_back('\0');
  k += t;
  k.push_back('\0');
  k += std::to_string(p);
  return k;
}

}  // namespace

struct Broker::Chunk {
  std::string own;
  std::shared_ptr<const std::string> shared;
  size_t off = 0, len = 0;
  const char* data() const { return (shared ? shared->data() : own.data()) + off; }
};

struct Broker::Conn {
  int fd = -1;
  std::deque<Chunk> out;
  // zero-copy sends: the pipe, and references to recently spliced batches. The socket (and the
  // peer's receive queue) may still reference their pages after splice() returns, so the last
  // kSpliceKeepBytes sent stay alive here (more than both socket buffers can hold).
  int pipe_rd = -1, pipe_wr = -1;
  size_t pipe_cap = 0;
  bool splice_ok = true;
  std::deque<std::shared_ptr<const std::string>> spliced;
  std::deque<size_t> spliced_len;
  size_t spliced_bytes = 0;
  ~Conn() {
    if (pipe_rd >= 0) close(pipe_rd);
    if (pipe_wr >= 0) close(pipe_wr);
  }
  bool parked = false;
  FetchRequest fetch;
  int32_t fetch_corr = 0;
  int64_t deadline = 0;
};

// Response under construction: owned bytes interleaved with zero-copy references.
struct ResponseBuilder {
  Writer w;
  size_t total = 0;
  std::vector<Broker::Chunk> chunks;
  void cut() {
    if (w.buf.empty()) return;
    Broker::Chunk c;
    c.own = std::move(w.buf);
    c.len = c.own.size();
    total += c.len;
    chunks.push_back(std::move(c));
    w.buf = std::string();
  }
  void shared(std::shared_ptr<const std::string> s, size_t off, size_t len) {
    cut();
    Broker::Chunk c;
    c.shared = std::move(s);
    c.off = off;
    c.len = len;
    total += len;
    chunks.push_back(std::move(c));
  }
  void finish() {
    cut();
    // frame size excludes the 4-byte size field at the front of chunk 0
    const int32_t sz = (int32_t)(total - 4);
    Writer::put_be(&chunks[0].own[0], &sz, 4);
  }
};

Broker::Broker(BrokerConfig cfg) : cfg_(std::move(cfg)) {}

Broker::~Broker() { stop(); }

BrokerNode Broker::self_node() const {
  BrokerNode n;
  n.node_id = cfg_.node_id;
  n.host = cfg_.host;
  n.port = port_;
  return n;
}

void Broker::set_cluster(const std::vector<BrokerNode>& nodes) {
  std::lock_guard<std::mutex> lk(mu_);
  cluster_ = nodes;
}

std::vector<BrokerNode> Broker::cluster() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (cluster_.empty()) return {self_node()};
  return cluster_;
}

int32_t Broker::leader_of(int partition) const {  // mu_ held
  if (cluster_.empty()) return cfg_.node_id;
  return cluster_[(size_t)partition % cluster_.size()].node_id;
}

bool Broker::leads(int partition) const {
  std::lock_guard<std::mutex> lk(mu_);
  return leader_of(partition) == cfg_.node_id;
}

void Broker::start() {
  if (running_) return;
  listen_fd_ = socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("broker: socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)cfg_.port);
  if (inet_pton(AF_INET, cfg_.host.c_str(), &a.sin_addr) != 1)
    throw std::runtime_error("broker: bad host " + cfg_.host);
  if (bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    close(listen_fd_);
    listen_fd_ = -1;
    throw std::runtime_error("broker: bind failed on " + cfg_.host + ":" +
                             std::to_string(cfg_.port) + ": " + strerror(errno));
  }
  listen(listen_fd_, 128);
  socklen_t len = sizeof(a);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&a), &len);
  port_ = ntohs(a.sin_port);
  running_ = true;
  thread_ = std::thread([this] {
    name_thread("gl-brk-acc");
    // writev() / splice() to a socket whose peer has gone raise SIGPIPE, which would kill an
    // embedding process that does not ignore it (Python does, a C++ host need not): block it in
    // the accept thread, whose mask the connection threads inherit, so the calls just fail
    // with EPIPE and the connection closes
    sigset_t pipe_set;
    sigemptyset(&pipe_set);
    sigaddset(&pipe_set, SIGPIPE);
    pthread_sigmask(SIG_BLOCK, &pipe_set, nullptr);
    accept_loop();
  });
}

void Broker::stop() {
  if (!running_.exchange(false)) return;
  coord_.shutdown();  // wakes connection threads blocked in JoinGroup / SyncGroup
  shutdown(listen_fd_, SHUT_RDWR);  // unblocks accept()
  if (thread_.joinable()) thread_.join();
  close(listen_fd_);
  listen_fd_ = -1;
  {
    std::lock_guard<std::mutex> lk(conn_mu_);
    for (int fd : conn_fds_) shutdown(fd, SHUT_RDWR);  // unblocks recv()/writev()
  }
  wake_all();
  for (auto& t : conn_threads_) t.join();
  conn_threads_.clear();
  conn_fds_.clear();
}

// Signals new data on (topic, partition) to the long-polling fetches waiting on it.
void Broker::wake(const std::string& topic, int partition) {
  std::lock_guard<std::mutex> lk(append_mu_);
  auto it = waiters_.find({topic, partition});
  if (it == waiters_.end()) return;
  const int64_t t = now_ns();
  for (Waiter* w : it->second) {
    {
      std::lock_guard<std::mutex> wl(w->m);
      if (!w->flag) w->t_wake_ns = t;
      w->flag = true;
    }
    w->cv.notify_one();
  }
}

void Broker::wake_all() {
  std::lock_guard<std::mutex> lk(append_mu_);
  for (auto& kv : waiters_)
    for (Waiter* w : kv.second) {
      {
        std::lock_guard<std::mutex> wl(w->m);
        w->flag = true;
      }
      w->cv.notify_one();
    }
}

bool Broker::create_topic(const std::string& topic, int partitions) {
  if (!valid_topic(topic)) throw std::invalid_argument("invalid topic name: " + topic);
  if (partitions <= 0) throw std::invalid_argument("partitions must be > 0");
  std::lock_guard<std::mutex> lk(mu_);
  if (topics_.count(topic)) return false;
  topics_[topic].resize((size_t)partitions);
  return true;
}

std::vector<std::string> Broker::topics() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> v;
  for (auto& kv : topics_) v.push_back(kv.first);
  return v;
}

int Broker::partitions(const std::string& topic) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = topics_.find(topic);
  return it == topics_.end() ? -1 : (int)it->second.size();
}

Broker::PartitionLog* Broker::find_log(const std::string& topic, int partition) {
  auto it = topics_.find(topic);
  if (it == topics_.end() || partition < 0 || (size_t)partition >= it->second.size())
    return nullptr;
  return &it->second[(size_t)partition];
}

const Broker::PartitionLog* Broker::find_log(const std::string& topic, int partition) const {
  auto it = topics_.find(topic);
  if (it == topics_.end() || partition < 0 || (size_t)partition >= it->second.size())
    return nullptr;
  return &it->second[(size_t)partition];
}

int64_t Broker::append_locked(PartitionLog& log, std::shared_ptr<const std::string> batch,
                              bool legacy, const BatchInfo& bi) {
  Segment s;
  s.base = log.end;
  s.next = log.end + bi.last_offset_delta + 1;
  s.max_ts = bi.max_timestamp;
  s.bytes = std::move(batch);
  s.legacy = legacy;
  if (cfg_.log_append_time && !legacy) {
    // the stored bytes may be shared (preloaded by reference): the stamp lives in the segment
    const uint8_t* b = reinterpret_cast<const uint8_t*>(s.bytes->data());
    const size_t n = kBatchMaxTsOffset + 8 - kBatchAttrOffset;
    static_assert(kBatchMaxTsOffset + 8 - kBatchAttrOffset == sizeof(s.hdr), "header window");
    memcpy(s.hdr, b + kBatchAttrOffset, n);
    const int16_t attrs = (int16_t)(bi.attributes | kAttrLogAppendTime);
    const int64_t now = wall_ms();
    Writer::put_be(reinterpret_cast<char*>(s.hdr), &attrs, 2);
    Writer::put_be(reinterpret_cast<char*>(s.hdr) + (kBatchMaxTsOffset - kBatchAttrOffset), &now,
                   8);
    Reader cr(b + kBatchCrcOffset, 4);
    s.crc = patch_batch_crc(cr.u32(), b + kBatchAttrOffset, s.hdr, n,
                            s.bytes->size() - (size_t)(kBatchMaxTsOffset + 8));
    s.max_ts = now;
    s.stamped = true;
  }
  log.bytes += (int64_t)s.bytes->size();
  log.end = s.next;
  log.segs.push_back(std::move(s));
  stats_.records_in += bi.records;
  // byte retention: drop the oldest segments (never the newest)
  while (log.bytes > cfg_.retention_bytes && log.first + 1 < log.segs.size()) {
    log.bytes -= (int64_t)log.segs[log.first].bytes->size();
    log.segs[log.first].bytes.reset();
    ++log.first;
    log.start = log.segs[log.first].base;
  }
  if (log.first > 4096 && log.first * 2 > log.segs.size()) {
    log.segs.erase(log.segs.begin(), log.segs.begin() + (long)log.first);
    log.first = 0;
  }
  return s.next - (bi.last_offset_delta + 1);
}

int64_t Broker::append(const std::string& topic, int partition, const std::vector<RecordIn>& recs) {
  if (recs.empty()) return log_end(topic, partition);
  Writer w;
  encode_batch(w, recs.data(), recs.size(), 0, wall_ms());
  auto bytes = std::make_shared<const std::string>(std::move(w.buf));
  const BatchInfo bi =
      peek_batch(reinterpret_cast<const uint8_t*>(bytes->data()), bytes->size(), false);
  int64_t base;
  {
    std::lock_guard<std::mutex> lk(mu_);
    PartitionLog* log = find_log(topic, partition);
    if (!log) throw std::invalid_argument("unknown topic/partition " + topic);
    base = append_locked(*log, std::move(bytes), false, bi);
  }
  wake(topic, partition);
  return base;
}

int64_t Broker::append_legacy(const std::string& topic, int partition, int magic,
                              const std::vector<LegacyRecord>& recs, int codec) {
  if (recs.empty()) return log_end(topic, partition);
  int64_t base;
  {
    std::lock_guard<std::mutex> lk(mu_);
    PartitionLog* log = find_log(topic, partition);
    if (!log) throw std::invalid_argument("unknown topic/partition " + topic);
    base = log->end;
    auto bytes = std::make_shared<const std::string>(encode_message_set(magic, recs, base, codec));
    BatchInfo bi;
    bi.base_offset = base;
    bi.records = (int32_t)recs.size();
    bi.last_offset_delta = (int32_t)recs.size() - 1;
    bi.max_timestamp = recs.back().timestamp;
    append_locked(*log, std::move(bytes), true, bi);
  }
  wake(topic, partition);
  return base;
}

int64_t Broker::append_shared(const std::string& topic, int partition,
                              std::shared_ptr<const std::string> batch) {
  const BatchInfo bi =
      peek_batch(reinterpret_cast<const uint8_t*>(batch->data()), batch->size(), false);
  int64_t base;
  {
    const int64_t t0 = now_ns();
    std::lock_guard<std::mutex> lk(mu_);
    probe_lock_.add(now_ns() - t0);
    PartitionLog* log = find_log(topic, partition);
    if (!log) throw std::invalid_argument("unknown topic/partition " + topic);
    base = append_locked(*log, std::move(batch), false, bi);
  }
  wake(topic, partition);
  return base;
}

BrokerProbes Broker::take_probes() {
  BrokerProbes p;
  p.wake_max_us = probe_wake_.max_ns.exchange(0) / 1000;
  p.wake_slow = probe_wake_.slow.exchange(0);
  p.flush_max_us = probe_flush_.max_ns.exchange(0) / 1000;
  p.flush_slow = probe_flush_.slow.exchange(0);
  p.lock_max_us = probe_lock_.max_ns.exchange(0) / 1000;
  p.lock_slow = probe_lock_.slow.exchange(0);
  return p;
}

int64_t Broker::log_start(const std::string& topic, int partition) const {
  std::lock_guard<std::mutex> lk(mu_);
  const PartitionLog* log = find_log(topic, partition);
  return log ? log->start : -1;
}

int64_t Broker::log_end(const std::string& topic, int partition) const {
  std::lock_guard<std::mutex> lk(mu_);
  const PartitionLog* log = find_log(topic, partition);
  return log ? log->end : -1;
}

int64_t Broker::committed(const std::string& group, const std::string& topic, int partition) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = offsets_.find(offset_key(group, topic, partition));
  return it == offsets_.end() ? -1 : it->second;
}

void Broker::fail_produce(const std::string& topic, int64_t n, int16_t error) {
  std::lock_guard<std::mutex> lk(mu_);
  if (n <= 0) produce_faults_.erase(topic);
  else produce_faults_[topic] = {n, error};
}

BrokerStats Broker::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

std::string Broker::read_raw(const std::string& topic, int partition, int64_t offset,
                             int64_t max_bytes) const {
  std::lock_guard<std::mutex> lk(mu_);
  const PartitionLog* log = find_log(topic, partition);
  std::string out;
  if (!log) return out;
  for (size_t i = log->first; i < log->segs.size(); ++i) {
    const Segment& s = log->segs[i];
    if (s.next <= offset) continue;
    if (!out.empty() && (int64_t)(out.size() + s.bytes->size()) > max_bytes) break;
    const size_t at = out.size();
    out += *s.bytes;
    if (s.legacy) continue;  // (offsets inside, as written)
    Writer::put_be(&out[at], &s.base, 8);
    if (s.stamped) {
      Writer::put_be(&out[at + kBatchCrcOffset], &s.crc, 4);
      memcpy(&out[at + kBatchAttrOffset], s.hdr, sizeof(s.hdr));
    }
  }
  return out;
}

// ------------------------------------------------------------------------------------------
// I/O loop
// ------------------------------------------------------------------------------------------

void Broker::accept_loop() {
  while (running_) {
    const int fd = accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) {
      if (errno == EINTR) continue;
      if (!running_) return;
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      continue;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    const int sz = socket_buffer_bytes();
    if (sz > 0) setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
    if (sz > 0) setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
    std::lock_guard<std::mutex> lk(conn_mu_);
    if (!running_) {
      close(fd);
      return;
    }
    conn_fds_.push_back(fd);
    conn_threads_.emplace_back([this, fd] {
      name_thread("gl-brk-conn");
      serve(fd);
    });
    std::lock_guard<std::mutex> lk2(mu_);
    ++stats_.connections;
  }
}

namespace {
bool read_exact(int fd, char* p, size_t n) {
  while (n) {
    const ssize_t r = recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}
}  // namespace

// One thread per client connection: blocking reads, requests answered in order, long-poll
// Fetch waits on its partitions' appends (so concurrent consumers are served by concurrent
// threads).
void Broker::serve(int fd) {
  Conn c;
  c.fd = fd;
  std::string frame;
  // L3 pairing with an in-process reader (gale/llc_pair.h): its registration may follow our
  // accept, so look again before each of the first requests
  int peer_port = -1, pair_tries = llc::enabled() ? 64 : 0;
  {
    sockaddr_in pa{};
    socklen_t pl = sizeof(pa);
    if (getpeername(fd, reinterpret_cast<sockaddr*>(&pa), &pl) == 0) peer_port = ntohs(pa.sin_port);
  }
  while (running_) {
    char hdr[4];
    if (!read_exact(fd, hdr, 4)) break;
    if (pair_tries > 0) pair_tries = llc::pin_self_for_peer(peer_port) ? 0 : pair_tries - 1;
    Reader hr(reinterpret_cast<const uint8_t*>(hdr), 4);
    const int32_t sz = hr.i32();
    if (sz < 0 || sz > (int32_t)std::min<int64_t>(cfg_.max_message_bytes + (16 << 20), 1 << 30))
      break;
    frame.resize((size_t)sz);
    if (!read_exact(fd, &frame[0], (size_t)sz)) break;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.bytes_in += 4 + sz;
    }
    bool ok;
    try {
      ok = handle_request(c, reinterpret_cast<const uint8_t*>(frame.data()), frame.size());
    } catch (const ProtocolError&) {
      ok = false;
    }
    if (!ok) break;
    const bool fetch = c.parked;
    if (c.parked) {
      // register on every requested partition before the first attempt, so an append between
      // an attempt and the wait sets the flag and is not missed
      Waiter w;
      std::vector<std::pair<std::string, int>> keys;
      for (const FetchTopic& t : c.fetch.topics)
        for (const FetchPartition& fp : t.partitions) keys.emplace_back(t.name, fp.index);
      {
        std::lock_guard<std::mutex> lk(append_mu_);
        for (auto& k : keys) waiters_[k].push_back(&w);
      }
      // unregistered on every exit path (a throwing try_fetch included): wake() must never see
      // a pointer to this stack frame after it is gone
      struct Unregister {
        Broker* b;
        Waiter* w;
        const std::vector<std::pair<std::string, int>>& keys;
        ~Unregister() {
          std::lock_guard<std::mutex> lk(b->append_mu_);
          for (auto& k : keys) {
            auto it = b->waiters_.find(k);
            if (it == b->waiters_.end()) continue;
            auto& v = it->second;
            v.erase(std::remove(v.begin(), v.end(), w), v.end());
            if (v.empty()) b->waiters_.erase(it);
          }
        }
      } unregister{this, &w, keys};
      bool final_attempt = c.fetch.max_wait_ms <= 0;
      int64_t t_wake = 0;
      for (;;) {
        {
          std::lock_guard<std::mutex> wl(w.m);
          w.flag = false;
        }
        if (try_fetch(c, final_attempt)) {
          if (t_wake) probe_wake_.add(now_ns() - t_wake);
          break;
        }
        std::unique_lock<std::mutex> wl(w.m);
        w.cv.wait_until(
            wl, std::chrono::steady_clock::time_point(std::chrono::milliseconds(c.deadline)),
            [&] { return w.flag || !running_; });
        t_wake = w.flag ? w.t_wake_ns : 0;
        final_attempt = now_ms() >= c.deadline || !running_;
      }
    }
    const int64_t t0 = fetch ? now_ns() : 0;
    if (!flush(c)) break;
    if (fetch) probe_flush_.add(now_ns() - t0);
  }
  close(fd);
  if (!c.spliced.empty()) {
    // data queued toward a peer that has not read it may still reference these pages: keep
    // them for a grace period after the connection is gone
    const int64_t now = now_ms();
    std::lock_guard<std::mutex> lk(conn_mu_);
    while (!spliced_grave_.empty() && now - spliced_grave_.front().first > 30000)
      spliced_grave_.pop_front();
    for (auto& p : c.spliced) spliced_grave_.emplace_back(now, std::move(p));
  }
  std::lock_guard<std::mutex> lk(conn_mu_);
  conn_fds_.erase(std::remove(conn_fds_.begin(), conn_fds_.end(), fd), conn_fds_.end());
}

namespace {
constexpr size_t kSpliceMinBytes = 64 << 10;    // smaller stored slices are just written
constexpr size_t kSpliceKeepBytes = 96ull << 20;
constexpr size_t kWriteBurstBytes = 1 << 20;
}  // namespace

// more: bytes of this connection's queue follow the chunk. SPLICE_F_MORE (MSG_MORE) lets TCP hold
// a sub-MSS tail segment for the data that follows; on the LAST piece of a response nothing
// follows, and a held tail is only released by a later ACK - with nothing else in flight that
// stalls the fetch response for up to a TCP timer (the 100-200 ms latency tails of zero-copy
// fetches), so the final piece is spliced without it.
int Broker::splice_chunk(Conn& c, const Chunk& f, bool more) {
  if (c.pipe_wr < 0) {
    int fds[2];
    if (pipe2(fds, O_CLOEXEC) != 0) return 0;
    c.pipe_rd = fds[0];
    c.pipe_wr = fds[1];
    const int want = 1 << 20;  // (the unprivileged default pipe-max-size)
    const int got = fcntl(c.pipe_wr, F_SETPIPE_SZ, want);
    c.pipe_cap = got > 0 ? (size_t)got : (size_t)(64 << 10);
  }
  const char* p = f.data();
  size_t left = f.len;
  bool first = true;
  while (left) {
    iovec iv{const_cast<char*>(p), std::min(left, c.pipe_cap)};
    const ssize_t n = vmsplice(c.pipe_wr, &iv, 1, 0);
    if (n < 0) {
      if (errno == EINTR) continue;
      return first ? 0 : -1;  // unusable before any byte moved: fall back to write
    }
    first = false;
    size_t m = (size_t)n;
    const unsigned fl = SPLICE_F_MOVE | (more || (size_t)n < left ? SPLICE_F_MORE : 0u);
    while (m) {
      const ssize_t w = splice(c.pipe_rd, nullptr, c.fd, nullptr, m, fl);
      if (w < 0) {
        if (errno == EINTR) continue;
        return -1;
      }
      if (w == 0) return -1;
      m -= (size_t)w;
    }
    p += n;
    left -= (size_t)n;
  }
  c.spliced.push_back(f.shared);
  c.spliced_len.push_back(f.len);
  c.spliced_bytes += f.len;
  while (c.spliced.size() > 1 && c.spliced_bytes - c.spliced_len.front() >= kSpliceKeepBytes) {
    c.spliced_bytes -= c.spliced_len.front();
    c.spliced.pop_front();
    c.spliced_len.pop_front();
  }
  return 1;
}

bool Broker::flush(Conn& c) {
  while (!c.out.empty()) {
    Chunk& head = c.out.front();
    if (cfg_.zero_copy && c.splice_ok && head.shared && head.len >= kSpliceMinBytes) {
      const int r = splice_chunk(c, head, c.out.size() > 1);
      if (r < 0) return false;
      if (r > 0) {
        std::lock_guard<std::mutex> lk(mu_);
        stats_.bytes_out += (int64_t)head.len;
        stats_.bytes_spliced += (int64_t)head.len;
        c.out.pop_front();
        continue;
      }
      c.splice_ok = false;  // not supported here: plain writes from now on
    }
    // at most kWriteBurstBytes per call (the splice path moves one pipe's worth, 1 MiB): the
    // loopback device queues a sender's segments on its CPU's backlog (netdev_max_backlog
    // packets), and a multi-MB burst overflows it whenever softirq work is deferred - every
    // drop is a retransmission, a 10-200 ms latency tail (profiles/archive/r3_tail_tcp.txt)
    iovec iov[64];
    int n = 0;
    size_t burst = 0;
    for (auto it = c.out.begin(); it != c.out.end() && n < 64 && burst < kWriteBurstBytes;
         ++it, ++n) {
      if (n > 0 && cfg_.zero_copy && c.splice_ok && it->shared && it->len >= kSpliceMinBytes)
        break;  // (the next piece goes zero-copy)
      iov[n].iov_base = const_cast<char*>(it->data());
      iov[n].iov_len = std::min(it->len, kWriteBurstBytes - burst);
      burst += iov[n].iov_len;
    }
    const ssize_t w = writev(c.fd, iov, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.bytes_out += w;
    }
    size_t left = (size_t)w;
    while (left && !c.out.empty()) {
      Chunk& f = c.out.front();
      if (left >= f.len) {
        left -= f.len;
        c.out.pop_front();
      } else {
        f.off += left;
        f.len -= left;
        left = 0;
      }
    }
  }
  return true;
}

namespace {
void frame_into(std::deque<Broker::Chunk>& out, Writer& w) {
  const int32_t sz = (int32_t)(w.buf.size() - 4);
  Writer::put_be(&w.buf[0], &sz, 4);
  Broker::Chunk c;
  c.own = std::move(w.buf);
  c.len = c.own.size();
  out.push_back(std::move(c));
}
}  // namespace

bool Broker::handle_request(Conn& c, const uint8_t* p, size_t n) {
  Reader r(p, n);
  const RequestHeader h = decode_request_header(r);
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++stats_.requests;
  }
  Writer w;
  w.i32(0);
  w.i32(h.correlation_id);
  const ApiKey key = (ApiKey)h.api_key;
  if (key == API_VERSIONS) {
    ApiVersionsResponse resp;
    resp.error = h.api_version == 0 ? NONE : UNSUPPORTED_VERSION;
    for (ApiKey k : {PRODUCE, FETCH, LIST_OFFSETS, METADATA, OFFSET_COMMIT, OFFSET_FETCH,
                     FIND_COORDINATOR, JOIN_GROUP, HEARTBEAT, LEAVE_GROUP, SYNC_GROUP,
                     API_VERSIONS, CREATE_TOPICS})
      resp.apis.push_back({(int16_t)k, kVersion(k), kVersion(k)});
    encode_api_versions_response(w, resp);
    frame_into(c.out, w);
    return true;
  }
  if (kVersion(key) < 0 || h.api_version != kVersion(key)) return false;  // unsupported: close

  switch (key) {
    case METADATA: {
      const MetadataRequest req = decode_metadata_request(r);
      MetadataResponse resp;
      std::lock_guard<std::mutex> lk(mu_);
      resp.brokers = cluster_.empty() ? std::vector<BrokerNode>{self_node()} : cluster_;
      resp.cluster_id = cfg_.cluster_id;
      resp.controller_id = resp.brokers[0].node_id;
      std::vector<std::string> names;
      if (req.all_topics) {
        for (auto& kv : topics_) names.push_back(kv.first);
      } else {
        names = req.topics;
      }
      for (const std::string& t : names) {
        TopicMetadata tm;
        tm.name = t;
        auto it = topics_.find(t);
        if (it == topics_.end()) {
          if (!valid_topic(t)) {
            tm.error = INVALID_TOPIC_EXCEPTION;
          } else if (cfg_.auto_create_topics && req.allow_auto_topic_creation) {
            topics_[t].resize((size_t)cfg_.default_partitions);
            it = topics_.find(t);
          } else {
            tm.error = UNKNOWN_TOPIC_OR_PARTITION;
          }
        }
        if (it != topics_.end()) {
          for (size_t pi = 0; pi < it->second.size(); ++pi) {
            PartitionMetadata pm;
            pm.index = (int32_t)pi;
            pm.leader = leader_of((int)pi);
            pm.replicas = {pm.leader};
            pm.isr = {pm.leader};
            tm.partitions.push_back(pm);
          }
        }
        resp.topics.push_back(std::move(tm));
      }
      encode_metadata_response(w, resp);
      break;
    }
    case PRODUCE: {
      const ProduceRequest req = decode_produce_request(r);
      ProduceResponse resp;
      const int16_t ack_err = (req.acks == 0 || req.acks == 1 || req.acks == -1)
                                  ? (int16_t)NONE : (int16_t)INVALID_REQUIRED_ACKS;
      {
        std::lock_guard<std::mutex> lk(mu_);
        ++stats_.produce_requests;
        for (const ProduceTopic& t : req.topics) {
          ProduceTopicResponse tr;
          tr.name = t.name;
          for (const ProducePartition& pp : t.partitions) {
            ProducePartitionResponse pr;
            pr.index = pp.index;
            PartitionLog* log = find_log(t.name, pp.index);
            auto fault = produce_faults_.find(t.name);
            if (ack_err) {
              pr.error = ack_err;
            } else if (fault != produce_faults_.end() && fault->second.first > 0) {
              pr.error = fault->second.second;
              if (--fault->second.first == 0) produce_faults_.erase(fault);
            } else if (!log) {
              pr.error = UNKNOWN_TOPIC_OR_PARTITION;
            } else if (leader_of(pp.index) != cfg_.node_id) {
              pr.error = NOT_LEADER_FOR_PARTITION;
            } else if (pp.records_len <= 0) {
              pr.error = CORRUPT_MESSAGE;
            } else {
              // validate every batch first: a partition's append is all-or-nothing
              std::vector<std::pair<size_t, BatchInfo>> bs;
              size_t pos = 0;
              const uint8_t* blob = p + pp.records_off;
              try {
                while (pos < (size_t)pp.records_len) {
                  const BatchInfo bi =
                      peek_batch(blob + pos, (size_t)pp.records_len - pos, cfg_.check_crcs);
                  if (bi.length > cfg_.max_message_bytes) {
                    pr.error = MESSAGE_TOO_LARGE;
                    break;
                  }
                  bs.push_back({pos, bi});
                  pos += (size_t)bi.length;
                }
              } catch (const ProtocolError&) {
                pr.error = CORRUPT_MESSAGE;
              }
              if (pr.error == NONE) {
                for (size_t k = 0; k < bs.size(); ++k) {
                  auto copy = std::make_shared<std::string>(
                      reinterpret_cast<const char*>(blob + bs[k].first), (size_t)bs[k].second.length);
                  const int64_t base = log->end;
                  Writer::put_be(&(*copy)[0], &base, 8);
                  append_locked(*log, std::move(copy), false, bs[k].second);
                  if (k == 0) pr.base_offset = base;
                }
              }
            }
            tr.partitions.push_back(pr);
          }
          resp.topics.push_back(std::move(tr));
        }
      }
      for (const ProduceTopic& t : req.topics)
        for (const ProducePartition& pp : t.partitions) wake(t.name, pp.index);
      if (req.acks == 0) return true;  // Kafka sends no response for acks=0
      encode_produce_response(w, resp);
      break;
    }
    case FETCH: {
      c.fetch = decode_fetch_request(r);
      c.fetch_corr = h.correlation_id;
      c.parked = true;
      c.deadline = now_ms() + std::max(0, c.fetch.max_wait_ms);
      {
        std::lock_guard<std::mutex> lk(mu_);
        ++stats_.fetch_requests;
      }
      return true;  // serve() completes it (long poll)
    }
    case LIST_OFFSETS: {
      const ListOffsetsRequest req = decode_list_offsets_request(r);
      ListOffsetsResponse resp;
      std::lock_guard<std::mutex> lk(mu_);
      for (const ListOffsetsTopic& t : req.topics) {
        ListOffsetsTopicResponse tr;
        tr.name = t.name;
        for (const ListOffsetsPartition& lp : t.partitions) {
          ListOffsetsPartitionResponse pr;
          pr.index = lp.index;
          const PartitionLog* log = find_log(t.name, lp.index);
          if (!log) {
            pr.error = UNKNOWN_TOPIC_OR_PARTITION;
          } else if (leader_of(lp.index) != cfg_.node_id) {
            pr.error = NOT_LEADER_FOR_PARTITION;
          } else if (lp.timestamp == kLatest) {
            pr.offset = log->end;
          } else if (lp.timestamp == kEarliest) {
            pr.offset = log->start;
          } else {
            pr.offset = log->end;
            for (size_t i = log->first; i < log->segs.size(); ++i) {
              if (log->segs[i].max_ts >= lp.timestamp) {
                pr.offset = log->segs[i].base;
                pr.timestamp = log->segs[i].max_ts;
                break;
              }
            }
          }
          tr.partitions.push_back(pr);
        }
        resp.topics.push_back(std::move(tr));
      }
      encode_list_offsets_response(w, resp);
      break;
    }
    case FIND_COORDINATOR: {
      const FindCoordinatorRequest req = decode_find_coordinator_request(r);
      FindCoordinatorResponse resp;
      std::lock_guard<std::mutex> lk(mu_);
      if (cluster_.empty()) {
        resp.node = self_node();
      } else {
        resp.node = cluster_[std::hash<std::string>()(req.key) % cluster_.size()];
      }
      encode_find_coordinator_response(w, resp);
      break;
    }
    case OFFSET_COMMIT: {
      OffsetCommitRequest req = decode_offset_commit_request(r);
      // a member fenced out of its generation (its partitions moved on) must not overwrite the
      // new owner's progress
      const int16_t fence = coord_.check_commit(req.group_id, req.generation_id, req.member_id);
      std::lock_guard<std::mutex> lk(mu_);
      for (CommitTopic& t : req.topics)
        for (CommitPartition& cp : t.partitions) {
          if (fence == NONE) offsets_[offset_key(req.group_id, t.name, cp.index)] = cp.offset;
          cp.error = fence;
        }
      encode_offset_commit_response(w, req.topics);
      break;
    }
    case JOIN_GROUP: {
      const JoinGroupRequest req = decode_join_group_request(r);
      encode_join_group_response(w, coord_.join(req, h.client_id));
      break;
    }
    case SYNC_GROUP: {
      const SyncGroupRequest req = decode_sync_group_request(r);
      encode_sync_group_response(w, coord_.sync(req));
      break;
    }
    case HEARTBEAT: {
      const HeartbeatRequest req = decode_heartbeat_request(r);
      encode_group_error_response(w, coord_.heartbeat(req));
      break;
    }
    case LEAVE_GROUP: {
      const LeaveGroupRequest req = decode_leave_group_request(r);
      encode_group_error_response(w, coord_.leave(req));
      break;
    }
    case OFFSET_FETCH: {
      OffsetFetchRequest req = decode_offset_fetch_request(r);
      std::lock_guard<std::mutex> lk(mu_);
      for (CommitTopic& t : req.topics)
        for (CommitPartition& cp : t.partitions) {
          auto it = offsets_.find(offset_key(req.group_id, t.name, cp.index));
          cp.offset = it == offsets_.end() ? -1 : it->second;
          cp.error = NONE;
        }
      encode_offset_fetch_response(w, req.topics);
      break;
    }
    case CREATE_TOPICS: {
      CreateTopicsRequest req = decode_create_topics_request(r);
      std::lock_guard<std::mutex> lk(mu_);
      for (CreateTopic& t : req.topics) {
        if (!valid_topic(t.name)) {
          t.error = INVALID_TOPIC_EXCEPTION;
        } else if (t.partitions <= 0 && t.partitions != -1) {
          t.error = INVALID_PARTITIONS;
        } else if (topics_.count(t.name)) {
          t.error = TOPIC_ALREADY_EXISTS;
        } else if (!req.validate_only) {
          topics_[t.name].resize((size_t)(t.partitions == -1 ? cfg_.default_partitions
                                                             : t.partitions));
        }
      }
      encode_create_topics_response(w, req.topics);
      break;
    }
    default:
      return false;
  }
  frame_into(c.out, w);
  return true;
}

bool Broker::try_fetch(Conn& c, bool final_attempt) {
  const FetchRequest& req = c.fetch;
  ResponseBuilder rb;
  rb.w.i32(0);
  rb.w.i32(c.fetch_corr);
  rb.w.i32(0);  // throttle
  int64_t data_bytes = 0;
  bool any_error = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    int64_t budget = req.max_bytes > 0 ? req.max_bytes : INT64_MAX;
    bool first_data = true;
    rb.w.array_len((int32_t)req.topics.size());
    for (const FetchTopic& t : req.topics) {
      rb.w.str(t.name);
      rb.w.array_len((int32_t)t.partitions.size());
      for (const FetchPartition& fp : t.partitions) {
        const PartitionLog* log = find_log(t.name, fp.index);
        int16_t err = NONE;
        if (!log) err = UNKNOWN_TOPIC_OR_PARTITION;
        else if (leader_of(fp.index) != cfg_.node_id) err = NOT_LEADER_FOR_PARTITION;
        else if (fp.fetch_offset < log->start || fp.fetch_offset > log->end)
          err = OFFSET_OUT_OF_RANGE;
        rb.w.i32(fp.index);
        rb.w.i16(err);
        rb.w.i64(log ? log->end : -1);
        rb.w.i64(log ? log->end : -1);
        rb.w.array_len(-1);  // aborted transactions: null
        if (err != NONE) {
          any_error = true;
          rb.w.i32(-1);
          continue;
        }
        // segments covering [fetch_offset, end)
        std::vector<const Segment*> sel;
        int64_t pbytes = 0;
        auto it = std::upper_bound(
            log->segs.begin() + (long)log->first, log->segs.end(), fp.fetch_offset,
            [](int64_t off, const Segment& s) { return off < s.base; });
        if (it != log->segs.begin() + (long)log->first) --it;
        for (; it != log->segs.end(); ++it) {
          if (it->next <= fp.fetch_offset) continue;
          const int64_t sz = (int64_t)it->bytes->size();
          const bool forced = first_data && sel.empty();  // KIP-74: first batch always fits
          if (!forced && (pbytes + sz > fp.max_bytes || sz > budget)) break;
          sel.push_back(&*it);
          pbytes += sz;
          budget -= sz;
          if (budget <= 0) break;
        }
        if (!sel.empty()) first_data = false;
        rb.w.i32((int32_t)pbytes);
        for (const Segment* s : sel) {
          if (s->legacy) {  // legacy message set: its own offsets, verbatim
            rb.shared(s->bytes, 0, s->bytes->size());
            continue;
          }
          rb.w.i64(s->base);
          if (s->stamped) {  // batchLength, leaderEpoch, magic | crc | attrs .. maxTimestamp
            rb.w.raw(s->bytes->data() + kBatchLengthOffset, kBatchCrcOffset - kBatchLengthOffset);
            rb.w.u32(s->crc);
            rb.w.raw(s->hdr, sizeof(s->hdr));
            rb.shared(s->bytes, kBatchMaxTsOffset + 8, s->bytes->size() - (kBatchMaxTsOffset + 8));
          } else {
            rb.shared(s->bytes, 8, s->bytes->size() - 8);
          }
        }
        data_bytes += pbytes;
      }
    }
  }
  if (!final_attempt && !any_error && data_bytes < std::max(1, req.min_bytes)) return false;
  rb.finish();
  for (auto& ch : rb.chunks) c.out.push_back(std::move(ch));
  c.parked = false;
  return true;
}

}  // namespace kafka
}  // namespace gale
