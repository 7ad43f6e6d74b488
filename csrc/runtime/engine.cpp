// The gale serving engine (see engine.h).
#include "engine.h"
#include "gale/llc_pair.h"
#include "gale/thread_name.h"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <sys/prctl.h>

#include <algorithm>
#include <sstream>

#include "../codec/json_codec.h"
#include "../kafka/compress.h"
#include "pack_tap.h"
#include "../kafka/fetch_framing.h"
#include "trace.h"

namespace gale {

// ---------------------------------------------------------------------------------------------
// Batcher: bounded record queue + continuous micro-batch formation
// ---------------------------------------------------------------------------------------------

class Engine::Batcher {
 public:
  explicit Batcher(size_t cap) : cap_(cap) {}

  // Blocks while the queue is full (backpressure to the Kafka consumer). False once closed.
  bool push_many(std::vector<InRecord>& recs, const std::atomic<bool>& stop) {
    size_t i = 0;
    const int64_t now = mono_ns();  // ready for batching (decode / ingest done)
    for (InRecord& r : recs) r.t_ready_ns = now;
    std::unique_lock<std::mutex> lk(mu_);
    while (i < recs.size()) {
      while (q_.size() >= cap_ && !closed_ && !stop)
        cv_space_.wait_for(lk, std::chrono::milliseconds(20));
      if (closed_ || (stop && q_.size() >= cap_)) return false;
      while (i < recs.size() && q_.size() < cap_) {
        images_ += recs[i].images;
        q_.push_back(std::move(recs[i++]));
      }
      cv_items_.notify_all();
    }
    return true;
  }

  void requeue(std::vector<InRecord>&& recs) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = recs.rbegin(); it != recs.rend(); ++it) {
      images_ += it->images;
      q_.push_front(std::move(*it));
    }
    cv_items_.notify_all();
  }

  // Continuous batching: a full batch (max_images) is taken at once; a partial one when its
  // oldest record has waited max_wait_ns, or immediately once the queue is closed (drain).
  // With a batch already in flight on the caller's replica, a partial batch is not taken early
  // (returns true with `out` empty) so the device work accumulates a fuller next batch.
  // idle_ns > 0: also return (true, empty) when the queue stayed empty that long (the caller
  // may then steal from another locality's queue).
  bool take(int max_images, int64_t max_wait_ns, bool have_inflight, std::vector<InRecord>& out,
            int& images, int64_t idle_ns = 0) {
    out.clear();
    images = 0;
    std::unique_lock<std::mutex> lk(mu_);
    const int64_t t_idle = idle_ns > 0 ? mono_ns() + idle_ns : 0;
    for (;;) {
      if (q_.empty()) {
        if (closed_) return false;
        if (have_inflight) return true;
        if (t_idle && mono_ns() >= t_idle) return true;
        cv_items_.wait_for(lk, std::chrono::nanoseconds(t_idle ? std::max<int64_t>(
                                   t_idle - mono_ns(), 1000) : 20000000));
        continue;
      }
      const int64_t deadline = q_.front().t_fetch_ns + max_wait_ns;
      const int64_t now = mono_ns();
      if (images_ >= max_images || now >= deadline || closed_) {
        while (!q_.empty() && (images == 0 || images + q_.front().images <= max_images)) {
          images += q_.front().images;
          images_ -= q_.front().images;
          out.push_back(std::move(q_.front()));
          q_.pop_front();
        }
        cv_space_.notify_all();
        return true;
      }
      if (have_inflight) return true;
      cv_items_.wait_for(lk, std::chrono::nanoseconds(std::max<int64_t>(deadline - now, 1000)));
    }
  }

  // Non-blocking: whatever is queued now, up to max_images (work stealing by an idle replica
  // of another locality).
  bool try_take(int max_images, std::vector<InRecord>& out, int& images) {
    out.clear();
    images = 0;
    std::lock_guard<std::mutex> lk(mu_);
    while (!q_.empty() && (images == 0 || images + q_.front().images <= max_images)) {
      images += q_.front().images;
      images_ -= q_.front().images;
      out.push_back(std::move(q_.front()));
      q_.pop_front();
    }
    if (!out.empty()) cv_space_.notify_all();
    return !out.empty();
  }
  int64_t queued_images() {
    std::lock_guard<std::mutex> lk(mu_);
    return images_;
  }

  void close() {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    cv_items_.notify_all();
    cv_space_.notify_all();
  }
  size_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_items_, cv_space_;
  std::deque<InRecord> q_;
  int64_t images_ = 0;
  size_t cap_;
  bool closed_ = false;
};

struct Engine::ReplicaSlot {
  std::shared_ptr<Replica> rep;
  int index = 0;
  int slot = 0;  // locality slot (its device's batcher / fetch pool)
  std::atomic<bool> alive{true};
  std::atomic<bool> watchdog_killed{false};
  std::atomic<bool> restarting{false};  // failed, supervisor recovery pending
  std::atomic<int> restarts{0};
  std::mutex mu;  // inflight
  std::deque<std::shared_ptr<Batch>> inflight;
  std::atomic<int64_t> batches{0}, images{0}, records{0};
  // time with at least one batch in flight (the load-aware assignor's capacity estimate)
  std::atomic<int64_t> busy_ns{0}, busy_since{0};
};

struct SplitRecord {
  InRecord parent;   // the input record (its fetch buffer released; the key copied below)
  std::string key;
  int parts = 0;
  std::mutex mu;
  std::vector<std::string> rows;  // per fragment: its prediction rows "[..],[..]"
  int done = 0;
  int status = codec::OK;         // the first failing fragment's status
};

// ---------------------------------------------------------------------------------------------

Engine::Engine(EngineConfig cfg) : cfg_(std::move(cfg)), rng_(cfg_.seed) {
  if (cfg_.trace) trace::set_enabled(true);
  if (cfg_.input_topic.empty() || cfg_.output_topic.empty())
    throw std::invalid_argument("engine: input and output topics are required");
  if (cfg_.sink_mode != "async" && cfg_.sink_mode != "sync" && cfg_.sink_mode != "fire-and-forget")
    throw std::invalid_argument("engine: sink_mode must be async|sync|fire-and-forget");
  if (cfg_.on_error != "null" && cfg_.on_error != "error-json" && cfg_.on_error != "drop")
    throw std::invalid_argument("engine: on_error must be null|error-json|drop");
  if (cfg_.value_format != "json" && cfg_.value_format != "json-string")
    throw std::invalid_argument("engine: value_format must be json|json-string");
  if (cfg_.output_key != "none" && cfg_.output_key != "input")
    throw std::invalid_argument("engine: output_key must be none|input");
  if (cfg_.delivery != "at-most-once" && cfg_.delivery != "at-least-once")
    throw std::invalid_argument("engine: delivery must be at-most-once|at-least-once");
  if (cfg_.auto_offset_reset != "latest" && cfg_.auto_offset_reset != "earliest")
    throw std::invalid_argument("engine: auto_offset_reset must be latest|earliest");
  if (cfg_.delivery == "at-least-once" && cfg_.sink_mode == "fire-and-forget")
    throw std::invalid_argument("engine: at-least-once delivery needs acknowledged sends "
                                "(sink_mode async or sync)");
  if (cfg_.max_batch <= 0 || cfg_.source_parallelism <= 0 || cfg_.sink_parallelism <= 0)
    throw std::invalid_argument("engine: max_batch / parallelism must be positive");
  // fault injection spec: comma separated kind@value
  std::stringstream ss(cfg_.fault);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    const size_t at = item.find('@');
    if (at == std::string::npos) throw std::invalid_argument("engine: bad fault spec " + item);
    const std::string kind = item.substr(0, at), val = item.substr(at + 1);
    if (kind == "replica_crash") crash_at_batch_ = std::stoll(val);
    else if (kind == "parse_error") parse_error_p_ = std::stod(val);
    else if (kind == "producer_fail") producer_fail_p_ = std::stod(val);
    else throw std::invalid_argument("engine: unknown fault kind " + kind);
  }
  eff_batch_ = cfg_.max_batch;
  eff_wait_ns_ = (int64_t)cfg_.max_wait_us * 1000;
  if (cfg_.slo_p99_ms > 0)  // start with a quarter of the budget for batch formation
    eff_wait_ns_ = std::min<int64_t>(eff_wait_ns_, (int64_t)(cfg_.slo_p99_ms * 0.25e6));
}

Engine::~Engine() {
  try {
    stop();
  } catch (...) {
  }
}

void Engine::add_replica(std::shared_ptr<Replica> r) {
  if (running_) throw std::logic_error("engine: add_replica after start");
  if (r->max_images() < cfg_.max_batch)
    throw std::invalid_argument("engine: replica " + r->name() + " max batch " +
                                std::to_string(r->max_images()) + " < engine max_batch " +
                                std::to_string(cfg_.max_batch));
  auto s = std::make_shared<ReplicaSlot>();
  s->rep = std::move(r);
  s->index = (int)replicas_.size();
  replicas_.push_back(std::move(s));
}

void Engine::set_ingest(std::shared_ptr<Ingest> ing) {
  if (running_) throw std::logic_error("engine: set_ingest after start");
  ingests_[ing->device()] = std::move(ing);
}

Ingest* Engine::ingest_for(int slot) {
  auto it = ingests_.find(slot_dev_[(size_t)slot]);
  return it == ingests_.end() ? nullptr : it->second.get();
}

void Engine::pin_thread(int device) {
  auto it = cfg_.device_cpus.find(device);
  if (it == cfg_.device_cpus.end() || it->second.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : it->second)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  sched_setaffinity(0, sizeof(set), &set);  // (best effort: a failure leaves it unpinned)
}

kafka::Producer* Engine::producer_for(int i) {
  return producers_[(size_t)i % producers_.size()].get();
}

bool Engine::fault_hit(double p) {
  if (p <= 0) return false;
  std::lock_guard<std::mutex> lk(rng_mu_);
  return std::uniform_real_distribution<double>(0, 1)(rng_) < p;
}

void Engine::start() {
  if (running_) return;
  if (replicas_.empty()) throw std::logic_error("engine: no replicas");
  for (int i = 0; i < cfg_.sink_parallelism; ++i) {
    kafka::ProducerConfig pc;
    pc.bootstrap = cfg_.bootstrap;
    pc.client_id = cfg_.client_id + "-sink-" + std::to_string(i);
    pc.acks = cfg_.acks;
    pc.linger_ms = cfg_.linger_ms;
    pc.batch_size = cfg_.batch_size;
    pc.buffer_memory = cfg_.producer_buffer_bytes;
    pc.max_request_size = (int)cfg_.producer_request_bytes;
    pc.compression = kafka::codec_from_name(cfg_.compression);
    pc.retries = cfg_.producer_retries;
    pc.retry_backoff_ms = cfg_.retry_backoff_ms;
    pc.delivery_timeout_ms = cfg_.delivery_timeout_ms;
    pc.fail_p = producer_fail_p_;
    pc.fail_seed = cfg_.seed + (uint64_t)i + 1;
    auto prod = std::make_unique<kafka::Producer>(pc);
    std::lock_guard<std::mutex> lk(prod_mu_);
    producers_.push_back(std::move(prod));
  }
  // static mode: resolve the input partitions and split them over the source threads now;
  // group mode: the sources start idle and the group thread hands them the assignment
  std::vector<int> parts = cfg_.partitions;
  int ns = cfg_.source_parallelism;
  if (!cfg_.group_membership) {
    if (parts.empty()) {
      kafka::Cluster cl(kafka::ClientConfig{cfg_.bootstrap, cfg_.client_id, 30000, 10000});
      const int n = cl.partitions(cfg_.input_topic);
      if (n <= 0) throw kafka::KafkaError(kafka::UNKNOWN_TOPIC_OR_PARTITION,
                                          "input topic " + cfg_.input_topic + " not found");
      for (int p = 0; p < n; ++p) parts.push_back(p);
    }
    ns = std::min<int>(cfg_.source_parallelism, (int)parts.size());
  } else if (cfg_.group_id.empty()) {
    throw std::invalid_argument("engine: group_membership needs a group_id");
  }
  src_ctl_.clear();
  for (int i = 0; i < ns; ++i) src_ctl_.push_back(std::make_unique<SourceCtl>());
  if (!cfg_.group_membership) {
    for (size_t i = 0; i < parts.size(); ++i) src_ctl_[i % (size_t)ns]->parts.push_back(parts[i]);
    for (auto& c : src_ctl_) c->epoch = 1;
  }
  // locality slots: one per distinct replica device (first-seen order). Each has its own
  // batcher, pinned fetch pool (mirrored on its device for GPU ingest) and sources; replicas
  // serve their own slot first and steal from the most loaded other slot when idle (the
  // locality-preferring, load-aware dispatch of Storm's LoadAwareShuffleGrouping)
  slot_key_.clear();
  slot_dev_.clear();
  for (auto& rs : replicas_) {
    const int key = rs->rep->locality();
    auto it = std::find(slot_key_.begin(), slot_key_.end(), key);
    rs->slot = (int)(it - slot_key_.begin());
    if (it == slot_key_.end()) {
      slot_key_.push_back(key);
      slot_dev_.push_back(rs->rep->device() >= 0 ? rs->rep->device() : key);
    }
  }
  const size_t nslots = slot_key_.size();
  batchers_.clear();
  for (size_t i = 0; i < nslots; ++i)
    batchers_.push_back(std::make_unique<Batcher>(
        (size_t)std::max(1, cfg_.queue_depth / (int)nslots)));
  pools_.assign(nslots, nullptr);
  for (size_t i = 0; i < nslots; ++i) {
    bool gpu = false;
    for (auto& rs : replicas_) gpu |= rs->slot == (int)i && rs->rep->device() >= 0;
    if (!gpu || cfg_.pinned_fetch_bytes <= 0) continue;
    // packed fetch bodies (pack_tap.h) keep their packed copy in the same chunk
    const size_t body = (size_t)cfg_.fetch_max_bytes + (1 << 20);
    const bool pack = cfg_.text_pack && ingest_for((int)i);
    // a packed chunk holds the body's layout twice over (text region + packed stream): the same
    // number of fetches in flight needs twice the budget - with the round-3 budget ResNet-50's
    // 1.7 MB records ran the pool dry and 77 % of them fell back to heap buffers (host staging,
    // 21.6 vs 31.3 k img/s, profiles/archive/r4_ab_resnet50_lenet_sink.jsonl)
    const size_t budget = (size_t)cfg_.pinned_fetch_bytes * (pack ? 2 : 1) / nslots;
    pools_[i] = std::make_shared<PinnedPool>(pack ? codec::pack_layout_bytes(body) + 4096 : body,
                                             budget);
    if (ingest_for((int)i)) {
      // the image arena behind each mirror (ingest_parse): one fp32 image per 2 * H * W * C
      // bytes of fetch body, the most images a body of that size can hold
      const size_t per = (size_t)cfg_.H * cfg_.W * cfg_.C;
      const size_t arena = cfg_.ingest_parse && per ? (body / (2 * per) + 2) * per * 4 : 0;
      pools_[i]->set_mirror_device(slot_dev_[i], arena);
    }
    pools_[i]->set_wait_ms(200);
  }
  running_ = true;
  stopping_ = false;
  workers_done_ = false;
  sources_done_ = false;
  sources_active_ = ns;
  dec_closed_ = false;
  for (int i = 0; i < cfg_.decode_threads; ++i)
    decoders_.emplace_back([this, i] {
      name_thread("gl-dec", i);
      // 1 us timer slack: the GPU ingest sleep-polls its fetch's completion every 20 us, and
      // the default 50 us slack stretched each sleep to ~70 us (the ingest stage is the largest
      // device-side part of a record's latency)
      prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
      decode_loop(i);
    });
  for (auto& rs : replicas_)
    workers_.emplace_back([this, rs] {
      name_thread("gl-rep", rs->index);
      pin_thread(rs->rep->device());
      prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1 us: sleep-polling GPU waits stay tight
      worker_loop(rs.get());
    });
  for (int i = 0; i < ns; ++i)
    sources_.emplace_back([this, i] {
      name_thread("gl-src", i);
      pin_thread(slot_dev_[(size_t)i % slot_dev_.size()]);
      // one L3 domain of that set, shared with the in-process broker thread that serves this
      // source's connection (gale/llc_pair.h)
      llc::pin_self_next_domain();
      source_loop(i);
    });
  group_stop_ = false;
  if (cfg_.group_membership)
    group_thread_ = std::thread([this] {
      name_thread("gl-group");
      group_loop();
    });
  watchdog_ = std::thread([this] {
    name_thread("gl-watchdog");
    watchdog_loop();
  });
}

void Engine::stop() {
  if (!running_) return;
  stopping_ = true;
  {
    std::lock_guard<std::mutex> lk(dec_mu_);  // wake sources blocked on a full decode queue
  }
  dec_space_cv_.notify_all();
  {
    // wait for the sources to stop fetching
    std::unique_lock<std::mutex> lk(done_mu_);
    done_cv_.wait_for(lk, std::chrono::seconds(30), [&] { return sources_active_ == 0; });
  }
  {
    std::lock_guard<std::mutex> lk(dec_mu_);
    dec_closed_ = true;
  }
  dec_cv_.notify_all();
  dec_space_cv_.notify_all();
  for (auto& t : decoders_) t.join();
  decoders_.clear();
  for (auto& b : batchers_) b->close();
  for (size_t i = 0; i < workers_.size(); ++i) {
    if (replicas_[i]->alive || replicas_[i]->restarting) {
      workers_[i].join();
    } else {
      workers_[i].detach();  // may be stuck on a dead device; its batches were re-queued
    }
  }
  workers_done_ = true;  // (the watchdog polls this flag, never the vector being cleared)
  workers_.clear();
  for (auto& p : producers_) p->flush();
  sources_done_ = true;  // sources may now commit their final offsets
  done_cv_.notify_all();
  for (auto& t : sources_) t.join();
  sources_.clear();
  group_stop_ = true;  // (after the sources' final commits: then leave the group)
  if (group_thread_.joinable()) group_thread_.join();
  running_ = false;
  done_cv_.notify_all();
  if (watchdog_.joinable()) watchdog_.join();
  for (auto& p : producers_) p->close();
  {
    std::lock_guard<std::mutex> lk(prod_mu_);
    for (const auto& p : producers_) {
      const kafka::ProducerStats ps = p->stats();
      prod_retried_ += ps.records_retried;
      prod_req_failed_ += ps.requests_failed;
    }
    producers_.clear();
  }
}

bool Engine::wait(int64_t timeout_ms) {
  std::unique_lock<std::mutex> lk(done_mu_);
  auto pred = [&] {
    return !running_ || stopping_ ||
           (cfg_.max_records > 0 && completed_.load() >= cfg_.max_records);
  };
  if (timeout_ms < 0) done_cv_.wait(lk, pred);
  else done_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred);
  return cfg_.max_records > 0 && completed_.load() >= cfg_.max_records;
}

// ---------------------------------------------------------------------------------------------
// source
// ---------------------------------------------------------------------------------------------

void Engine::commit(kafka::Consumer& c, const std::vector<int>& parts) {
  if (cfg_.group_id.empty()) return;
  std::map<int, int64_t> offs;
  {
    std::lock_guard<std::mutex> lk(pend_mu_);
    for (int p : parts) {
      auto it = pending_.find(p);
      if (it != pending_.end() && !it->second.empty()) offs[p] = it->second.first();
      else if (next_fetch_.count(p)) offs[p] = next_fetch_[p];
    }
  }
  // GALE_LOG_COMMITS=1: one stderr line per commit (delivery diagnostics in the fault tests)
  static const bool log_commits = [] {
    const char* e = getenv("GALE_LOG_COMMITS");
    return e && *e && *e != '0';
  }();
  std::string what;
  if (log_commits)
    for (const auto& kv : offs)
      what += " p" + std::to_string(kv.first) + "=" + std::to_string(kv.second);
  try {
    c.commit(offs);
    ++commits_;
    if (log_commits)
      fprintf(stderr, "[gale commit] generation %d ok:%s\n", (int)generation_, what.c_str());
  } catch (const std::exception& e) {
    fprintf(stderr, "[gale source] offset commit failed (generation %d:%s): %s\n",
            (int)generation_, what.c_str(), e.what());
  }
}

int64_t Engine::replica_busy_ns() const {
  const int64_t now = mono_ns();
  int64_t t = 0;
  for (const auto& rs : replicas_) {
    const int64_t since = rs->busy_since.load();
    t += rs->busy_ns.load() + (since ? now - since : 0);
  }
  return t;
}

// Waits until no fetched record of `parts` is still in the pipeline (or timeout_ms).
bool Engine::drain_pending(const std::vector<int>& parts, int timeout_ms) {
  const int64_t until = mono_ns() + (int64_t)timeout_ms * 1000000;
  for (;;) {
    bool empty = true;
    {
      std::lock_guard<std::mutex> lk(pend_mu_);
      for (int p : parts) {
        auto it = pending_.find(p);
        empty &= it == pending_.end() || it->second.empty();
      }
    }
    if (empty) return true;
    if (mono_ns() >= until || stopping_) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
}

// Hands the sources a new partition set (group thread) and waits until each has taken it
// (committed and dropped its previous partitions). false = not every source confirmed in time.
bool Engine::distribute(const std::vector<int>& parts, int32_t generation,
                        const std::string& member, int timeout_ms) {
  const size_t ns = src_ctl_.size();
  std::vector<uint64_t> want(ns);
  for (size_t i = 0; i < ns; ++i) {
    SourceCtl& c = *src_ctl_[i];
    std::lock_guard<std::mutex> lk(c.mu);
    c.parts.clear();
    for (size_t k = i; k < parts.size(); k += ns) c.parts.push_back(parts[k]);
    c.generation = generation;
    c.member = member;
    want[i] = ++c.epoch;
  }
  const int64_t until = mono_ns() + (int64_t)timeout_ms * 1000000;
  bool ok = true;
  for (size_t i = 0; i < ns; ++i) {
    SourceCtl& c = *src_ctl_[i];
    std::unique_lock<std::mutex> lk(c.mu);
    while (c.acked < want[i] && !stopping_ && mono_ns() < until)
      c.cv.wait_for(lk, std::chrono::milliseconds(10));
    ok &= c.acked >= want[i];
  }
  return ok;
}

// Consumer-group membership (group_membership): join, give the assignment to the sources,
// heartbeat; on a rebalance revoke everything (the sources commit first), rejoin, repeat.
void Engine::group_loop() {
  kafka::GroupConfig gc;
  gc.bootstrap = cfg_.bootstrap;
  gc.client_id = cfg_.client_id + "-group";
  gc.group_id = cfg_.group_id;
  gc.topic = cfg_.input_topic;
  gc.session_timeout_ms = cfg_.session_timeout_ms;
  gc.rebalance_timeout_ms = cfg_.rebalance_timeout_ms;
  gc.assignor = cfg_.assignor;
  std::unique_ptr<kafka::GroupMember> gm;
  const bool load_aware = cfg_.assignor == "load-aware";
  const int64_t lag_bound =
      cfg_.lag_rebalance_records > 0
          ? cfg_.lag_rebalance_records
          : 8ll * cfg_.max_batch * std::max<int64_t>(1, (int64_t)replicas_.size());
  std::vector<int> owned;
  int64_t s_batches = batches_total_, s_busy = replica_busy_ns(), s_t = mono_ns();
  int64_t last_join = 0, over_since = 0, lag_at_over = 0;
  // capacity (images/s): full micro-batches per second of replica busy time, i.e. replicas x
  // max_batch / (busy time per batch), smoothed over heartbeats; only windows in which the
  // replicas were busy >= 10 % of the time count. A saturated member runs full batches, so its
  // estimate is what it serves; a lightly loaded one runs partial batches and is credited with
  // what full ones would carry (an upper bound - it has headroom)
  auto sample_capacity = [&] {
    const int64_t t = mono_ns(), nb = batches_total_, busy = replica_busy_ns();
    const double dt = (double)(t - s_t), nrep = (double)std::max<size_t>(1, replicas_.size());
    const double dbusy = (double)(busy - s_busy);
    if (dt > 0 && dbusy >= 0.1 * dt * nrep && nb > s_batches) {
      const double per_batch_s = dbusy * 1e-9 / (double)(nb - s_batches);
      const double inst = nrep * (double)cfg_.max_batch / per_batch_s;
      const double c = capacity_rps_.load();
      capacity_rps_ = c > 0 ? 0.7 * c + 0.3 * inst : inst;
    }
    s_t = t;
    s_batches = nb;
    s_busy = busy;
  };
  while (!group_stop_) {
    try {
      if (!gm) gm = std::make_unique<kafka::GroupMember>(gc);
      if (stopping_) {  // draining: keep the session alive until the final commits are done
        gm->heartbeat();
        std::this_thread::sleep_for(std::chrono::milliseconds(cfg_.heartbeat_interval_ms));
        continue;
      }
      if (load_aware) {
        sample_capacity();
        kafka::MemberLoad ml;
        ml.capacity = capacity_rps_.load();
        ml.owned.assign(owned.begin(), owned.end());
        gm->set_user_data(kafka::encode_member_load(ml));
      }
      const std::vector<int> mine = gm->join();
      owned = mine;
      last_join = mono_ns();
      over_since = 0;
      distribute(mine, gm->generation(), gm->member_id(), cfg_.rebalance_timeout_ms);
      generation_ = gm->generation();
      assigned_partitions_ = (int)mine.size();
      ++rebalances_;
      fprintf(stderr, "[gale group] %s generation %d: %zu partition(s)%s\n",
              gm->member_id().c_str(), gm->generation(), mine.size(),
              gm->is_leader() ? " (leader)" : "");
      for (;;) {
        const int64_t next = mono_ns() + (int64_t)cfg_.heartbeat_interval_ms * 1000000;
        while (!group_stop_ && !stopping_ && mono_ns() < next)
          std::this_thread::sleep_for(std::chrono::milliseconds(5));
        if (group_stop_) break;
        bool rejoin = false;
        if (load_aware && !stopping_) {
          // lag-triggered rebalance: this member cannot keep up with its partitions
          sample_capacity();
          int64_t lag = 0;
          for (const PartitionOffsets& o : partition_offsets()) lag += o.lag;
          const int64_t now = mono_ns();
          if (lag > lag_bound) {
            if (!over_since) {
              over_since = now;
              lag_at_over = lag;
            } else if (now - over_since >= 1000000000ll && lag > lag_at_over &&
                       now - last_join >= (int64_t)cfg_.rebalance_cooldown_ms * 1000000) {
              // a rebalance only helps when this member's lag is out of proportion to its
              // capacity share; when the whole group is overloaded every member's lag grows in
              // proportion, no assignment adds capacity, and an eager rebalance would only
              // stop the world. The group's lags come from the broker (log ends -
              // committed offsets), this member's share from the leader's assignment.
              const double share = gm->capacity_share();
              double frac = -1;
              if (share > 0) {
                try {
                  int64_t total = 0, own = 0;
                  for (const auto& kv : gm->partition_lags()) {
                    total += kv.second;
                    if (std::find(owned.begin(), owned.end(), kv.first) != owned.end())
                      own += kv.second;
                  }
                  if (total > 0) frac = (double)own / (double)total;
                } catch (const std::exception&) {
                }
              }
              if (frac < 0 || frac > std::min(0.95, 1.5 * share)) {
                fprintf(stderr, "[gale group] lag %lld > %lld and growing (capacity %.0f "
                        "images/s, %.0f%% of the group's lag at a %.0f%% capacity share): "
                        "triggering a load-aware rebalance\n", (long long)lag,
                        (long long)lag_bound, capacity_rps_.load(), 100 * frac, 100 * share);
                ++lag_rebalances_;
                rejoin = true;
              } else {
                ++lag_rebalances_skipped_;  // group-wide overload: re-arm, keep the assignment
                over_since = now;
                lag_at_over = lag;
              }
            }
          } else {
            over_since = 0;
          }
        }
        if (rejoin || !gm->heartbeat()) {
          if (stopping_) continue;
          // eager rebalance: every partition is revoked (drained and committed) before
          // rejoining. Revocation is a barrier: until every source confirmed, keep the session
          // alive and retry (a source that is still fetching a revoked partition would serve
          // records the next owner serves again), within 3/4 of the rebalance timeout so this
          // member still rejoins before the coordinator's deadline
          const int64_t until =
              mono_ns() + (int64_t)cfg_.rebalance_timeout_ms * 3 / 4 * 1000000;
          bool revoked = false;
          while (!revoked && !stopping_ && !group_stop_) {
            const int64_t left_ms = (until - mono_ns()) / 1000000;
            if (left_ms <= 0) break;
            revoked = distribute({}, gm->generation(), gm->member_id(),
                                 (int)std::min<int64_t>(left_ms, 500));
            if (!revoked) gm->heartbeat();
          }
          if (!revoked && !stopping_)
            fprintf(stderr, "[gale group] revocation not confirmed by every source within "
                    "%d ms: rejoining anyway\n", cfg_.rebalance_timeout_ms * 3 / 4);
          assigned_partitions_ = 0;
          break;
        }
        if (stopping_) continue;
      }
    } catch (const std::exception& e) {
      fprintf(stderr, "[gale group] %s: retrying\n", e.what());
      gm.reset();
      for (int i = 0; i < 50 && !group_stop_; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  if (gm) {
    try {
      gm->leave();
    } catch (const std::exception&) {
    }
  }
}

void Engine::source_loop(int idx) {
  SourceCtl& ctl = *src_ctl_[(size_t)idx];
  kafka::ConsumerConfig cc;
  cc.bootstrap = cfg_.bootstrap;
  cc.client_id = cfg_.client_id + "-source-" + std::to_string(idx);
  cc.group_id = cfg_.group_id;
  cc.max_wait_ms = cfg_.fetch_max_wait_ms;
  cc.min_bytes = std::max(1, cfg_.fetch_min_bytes);
  cc.fetch_max_bytes = cfg_.fetch_max_bytes;
  cc.partition_max_bytes = cfg_.partition_max_bytes;
  const int slot = idx % (int)slot_dev_.size();
  const std::shared_ptr<PinnedPool> pinned = pools_[(size_t)slot];
  const bool packing = pinned && cfg_.text_pack && ingest_for(slot);
  const bool bounce = packing && cfg_.text_pack_bounce && cfg_.decode_threads > 0;
  const size_t window = (size_t)std::max(4, cfg_.text_pack_window_kb) << 10;
  // recv_lowat < 0 (auto): with the bounce receive, wake per window of a large response instead
  // of per segment (+6 % img/s in 5 of 5 interleaved pairs, profiles/archive/r4_ab_recv_lowat.jsonl)
  cc.recv_lowat = cfg_.recv_lowat >= 0 ? cfg_.recv_lowat : bounce ? (int)window : 0;
  // with decode workers the CRC32C check moves off this thread (decode_fetch)
  cc.check_crcs = cfg_.check_crcs && cfg_.decode_threads <= 0;
  cc.auto_offset_reset = cfg_.start_offset == "earliest" ? "earliest" : cfg_.auto_offset_reset;
  Batcher& batcher = *batchers_[(size_t)slot];
  kafka::BufferAlloc alloc = kafka::heap_alloc;
  if (pinned) {
    std::shared_ptr<PinnedPool> pool = pinned;
    alloc = [pool](size_t n) {
      bool pinned = false;
      return pool->alloc(n, &pinned);
    };
  }
  std::unique_ptr<kafka::Consumer> cons;
  try {
    cons = std::make_unique<kafka::Consumer>(cc, alloc);
    if (packing) {
      // the bounce receive leaves only framing on the host: the CRC check must be the GPU's
      if (bounce) {
        std::shared_ptr<PinnedPool> pool = pinned;
        cons->set_recv_tap(std::make_shared<BouncePackTap>(
            pool->chunk_bytes(), [pool](const uint8_t* p) { return pool->owns(p); }, 64 << 10,
            window));
      } else {
        cons->set_recv_tap(std::make_shared<PackTap>(pinned));
      }
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "[gale source %d] failed to start: %s\n", idx, e.what());
  }
  std::vector<int> parts;
  uint64_t epoch = 0;
  // (re)assignment: commit and forget the old partitions, seek the new ones. Group-managed
  // partitions resume from the group's committed offsets (that is how a survivor takes over a
  // dead member's partitions); static ones from start_offset.
  auto reassign = [&]() {
    std::vector<int> want;
    int32_t gen;
    std::string member;
    uint64_t e;
    {
      std::lock_guard<std::mutex> lk(ctl.mu);
      if (ctl.epoch == epoch) return;
      want = ctl.parts;
      gen = ctl.generation;
      member = ctl.member;
      e = ctl.epoch;
    }
    if (!parts.empty()) {
      // revoked partitions: let their fetched records finish (bounded) so the commit covers
      // them and the next owner does not serve them again
      if (cfg_.group_membership) drain_pending(parts, cfg_.rebalance_timeout_ms / 4);
      commit(*cons, parts);
      std::lock_guard<std::mutex> lk(pend_mu_);
      for (int p : parts) {
        next_fetch_.erase(p);
        high_watermark_.erase(p);
        // (records still in flight complete against a missing entry, which is a no-op; a
        // partition assigned back later starts a fresh window)
        pending_.erase(p);
      }
    }
    parts = want;
    cons->set_generation(gen, member);
    if (!parts.empty()) {
      cons->assign(cfg_.input_topic, parts);
      cons->seek_to(cfg_.group_membership ? "committed" : cfg_.start_offset);
      std::lock_guard<std::mutex> lk(pend_mu_);
      for (int p : parts) next_fetch_[p] = cons->position(p);
    }
    epoch = e;
    {
      std::lock_guard<std::mutex> lk(ctl.mu);
      ctl.acked = e;
    }
    ctl.cv.notify_all();
  };
  int64_t last_commit = mono_ns();
  int64_t seen_conv = 0, seen_poison = 0, seen_poison_recs = 0, seen_unknown = 0;
  std::vector<InRecord> good;
  while (cons && !stopping_) {
    try {
      reassign();
    } catch (const std::exception& e) {
      fprintf(stderr, "[gale source %d] assignment failed: %s\n", idx, e.what());
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      continue;
    }
    if (parts.empty()) {  // idle until the group assigns this source something
      std::unique_lock<std::mutex> lk(ctl.mu);
      ctl.cv.wait_for(lk, std::chrono::milliseconds(20));
      continue;
    }
    std::vector<kafka::Fetched> fs;
    try {
      const int64_t t0 = mono_ns();
      trace::Range tr("gale:fetch");
      fs = cons->poll();
      ns_poll_ += mono_ns() - t0;
      // record-format conversion (compressed / legacy batches) and poison batches
      const int64_t cb = cons->converted_batches(), pb = cons->poison_batches(),
                    pr = cons->poison_records(), pu = cons->poison_unknown_span();
      if (cb != seen_conv || pb != seen_poison) {
        converted_batches_ += cb - seen_conv;
        poison_batches_ += pb - seen_poison;
        poison_records_ += pr - seen_poison_recs;
        poison_unknown_span_ += pu - seen_unknown;
        seen_conv = cb;
        seen_poison = pb;
        seen_poison_recs = pr;
        seen_unknown = pu;
      }
    } catch (const std::exception& e) {
      fprintf(stderr, "[gale source %d] fetch failed: %s\n", idx, e.what());
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      continue;
    }
    const int64_t now = mono_ns();
    {
      // register before anything can complete, and before the commit position moves past them
      std::lock_guard<std::mutex> lk(pend_mu_);
      for (auto& f : fs)
        for (const kafka::RecordRef& rr : f.records) pending_[rr.partition].add(rr.offset);
      for (int p : parts) next_fetch_[p] = cons->position(p);
      for (const auto& kv : cons->high_watermarks())
        if (std::find(parts.begin(), parts.end(), kv.first) != parts.end())
          high_watermark_[kv.first] = kv.second;
    }
    if (!fs.empty()) {
      int64_t z = 0;
      t_first_ns_.compare_exchange_strong(z, now);
    }
    for (auto& f : fs) {
      FetchItem it;
      if (f.sparse) ++sparse_fetches_;
      it.pinned = pinned && pinned->owns(f.buf.get());
      it.f = std::move(f);
      it.source = idx;
      it.slot = slot;
      it.t_fetch_ns = now;
      if (cfg_.decode_threads <= 0) {
        good.clear();
        decode_fetch(it, good, idx);
        // when stopping with a full queue the rest stays pending (never committed, so a
        // restart with start_offset=committed re-reads it)
        if (!good.empty()) batcher.push_many(good, stopping_);
      } else {
        const int64_t th = mono_ns();
        std::unique_lock<std::mutex> lk(dec_mu_);
        dec_space_cv_.wait(lk, [&] { return dec_q_.size() < (size_t)(4 * cfg_.decode_threads) ||
                                            stopping_; });
        ns_handoff_ += mono_ns() - th;
        if (stopping_) break;
        dec_q_.push_back(std::move(it));
        dec_cv_.notify_one();
      }
    }
    if (mono_ns() - last_commit > (int64_t)cfg_.commit_interval_ms * 1000000) {
      commit(*cons, parts);
      last_commit = mono_ns();
    }
  }
  {
    std::lock_guard<std::mutex> lk(done_mu_);
    --sources_active_;
  }
  done_cv_.notify_all();
  if (cons) {
    std::unique_lock<std::mutex> lk(done_mu_);
    done_cv_.wait_for(lk, std::chrono::seconds(60), [&] { return sources_done_.load(); });
    lk.unlock();
    if (!parts.empty()) commit(*cons, parts);
  }
}

void Engine::decode_loop(int idx) {
  std::vector<InRecord> good;
  for (;;) {
    FetchItem it;
    {
      std::unique_lock<std::mutex> lk(dec_mu_);
      dec_cv_.wait(lk, [&] { return !dec_q_.empty() || dec_closed_; });
      if (dec_q_.empty()) return;
      it = std::move(dec_q_.front());
      dec_q_.pop_front();
      dec_space_cv_.notify_one();
    }
    good.clear();
    const int64_t t0 = mono_ns();
    {
      trace::Range tr("gale:decode");
      decode_fetch(it, good, idx);
    }
    ns_decode_ += mono_ns() - t0;
    if (!good.empty()) batchers_[(size_t)it.slot]->push_many(good, stopping_);
  }
}

// GPU ingest of one pinned fetch buffer (ingest.h): bounded envelope checks on the host, batch
// CRCs and image counts on the device. False = not applicable (the caller takes the host path).
bool Engine::ingest_fetch(FetchItem& it, std::vector<InRecord>& good, int lane) {
  Ingest* ingest = ingest_for(it.slot);
  if (!ingest || !it.pinned || ingest_failed_) return false;
  kafka::Fetched& f = it.f;
  uint8_t* dev = pools_[(size_t)it.slot]->mirror(f.buf.get());
  if (!dev) return false;
  const int64_t t0 = mono_ns();
  ns_lane_wait_ += t0 - it.t_fetch_ns;  // (fetch received -> an ingest lane took it)
  const size_t n = f.records.size();
  IngestIO io;
  io.status.assign(n, codec::OK);
  io.arr_off.assign(n, 0);
  io.arr_len.assign(n, 0);
  for (size_t i = 0; i < n; ++i) {
    const kafka::RecordRef& rr = f.records[i];
    if (rr.poison) {
      io.status[i] = codec::CORRUPT;  // stands for a record of an undecodable batch
      continue;
    }
    if (rr.value_len < 0) {
      io.status[i] = codec::BAD_ENVELOPE;  // null value (Jackson would throw)
      continue;
    }
    // (a sparse host copy holds only the ends of each value: the scan stays inside them)
    const codec::Scan s =
        f.sparse ? codec::scan_envelope(f.buf.get() + rr.value_off, (size_t)rr.value_len,
                                        kafka::FramingWalker::kHead, kafka::FramingWalker::kTail)
                 : codec::scan_envelope(f.buf.get() + rr.value_off, (size_t)rr.value_len);
    io.status[i] = s.status;
    io.arr_off[i] = s.arr_off;
    io.arr_len[i] = s.arr_len;
  }
  PinnedPool& pool = *pools_[(size_t)it.slot];
  const size_t arena_bytes = pool.mirror_extra();
  float* arena =
      arena_bytes ? reinterpret_cast<float*>(dev + pool.mirror_extra_offset()) : nullptr;
  try {
    ingest->run(lane, f, dev, pool.chunk_bytes(), cfg_.check_crcs && !f.crc_checked, cfg_.H,
                cfg_.W, cfg_.C, io, arena, arena_bytes);
  } catch (const std::exception& e) {
    if (!ingest_failed_.exchange(true))
      fprintf(stderr, "[gale decode] GPU ingest failed (%s): host decode from now on\n", e.what());
    return false;
  }
  std::vector<char> corrupt(n, 0);
  for (size_t b = 0; b < f.batches.size(); ++b)
    if (!io.batch_ok[b])
      for (size_t i = 0; i < f.batches[b].nrec; ++i) corrupt[f.batches[b].first_rec + i] = 1;
  kafka::Producer* prod = producer_for(it.source);
  for (size_t i = 0; i < n; ++i) {
    const kafka::RecordRef& rr = f.records[i];
    InRecord r;
    r.buf = f.buf;
    r.pinned = true;
    r.value = rr.value_len >= 0 ? f.buf.get() + rr.value_off : nullptr;
    r.len = rr.value_len;
    r.key = rr.key_len >= 0 ? f.buf.get() + rr.key_off : nullptr;
    r.key_len = rr.key_len;
    r.partition = rr.partition;
    r.offset = rr.offset;
    r.timestamp_ms = rr.timestamp;
    r.t_fetch_ns = it.t_fetch_ns;
    r.source = it.source;
    r.dev_value = dev + rr.value_off;
    r.dev_locality = slot_key_[(size_t)it.slot];
    if (io.cnt_off[i] >= 0) r.dev_counts = dev + io.cnt_off[i];
    r.dev_image = io.img[i];
    r.dev_arena = r.dev_image ? arena : nullptr;
    if (r.dev_image) ++ingest_parsed_;
    ++records_in_;
    if (r.len >= 0) bytes_in_ += r.len;
    r.status = corrupt[i] ? (int)codec::CORRUPT : io.status[i];
    r.arr_off = io.arr_off[i];
    r.arr_len = io.arr_len[i];
    r.images = io.images[i];
    if (r.status == codec::OK && fault_hit(parse_error_p_)) r.status = codec::BAD_ENVELOPE;
    if (r.status == codec::OK && r.images > cfg_.max_batch) {
      images_in_ += r.images;
      if (f.sparse) {  // the split copies the record's text on the host: make it whole
        f.restore();
        ++restored_fetches_;
      }
      if (!split_record(r, good)) emit_error(r, codec::BAD_SHAPE, prod);
    } else if (r.status == codec::OK) {
      images_in_ += r.images;
      good.push_back(std::move(r));
    } else {
      emit_error(r, r.status, prod);
    }
  }
  ingested_records_ += (int64_t)n;
  ingest_ns_ += mono_ns() - t0;
  return true;
}

// CRC32C of every record batch (unless the consumer checked it), then the envelope scan of
// every record; malformed records go straight to the error policy.
void Engine::decode_fetch(FetchItem& it, std::vector<InRecord>& good, int lane) {
  if (ingest_fetch(it, good, lane)) return;
  kafka::Fetched& f = it.f;
  if (f.sparse) {  // the host path reads the text: expand the packed stream in place first
    f.restore();
    ++restored_fetches_;
  }
  std::vector<char> corrupt;
  // CRC32C and envelope scan fused in one pass: the batch CRC is chained record by record
  // (crc32c(b, crc32c(a)) == crc32c(a ++ b)) and each record is scanned right after its bytes
  // went through the CRC, while they are still in L1/L2, so the fetch buffer streams from
  // DRAM/L3 once instead of twice (per-socket memory bandwidth bounds the 8-GPU node)
  std::vector<codec::Scan> pre;
  std::vector<char> have_pre;
  if (cfg_.check_crcs && !f.crc_checked) {
    corrupt.assign(f.records.size(), 0);
    pre.resize(f.records.size());
    have_pre.assign(f.records.size(), 0);
    const uint8_t* base = f.buf.get();
    for (const kafka::BatchSpan& b : f.batches) {
      const uint8_t* p = base + b.off;
      kafka::Reader r(p + kafka::kBatchCrcOffset, 4);
      const uint32_t want = r.u32();
      const uint8_t* pos = p + kafka::kBatchAttrOffset;
      const uint8_t* end = p + b.len;
      uint32_t crc = 0;
      for (size_t i = b.first_rec; i < b.first_rec + b.nrec; ++i) {
        const kafka::RecordRef& rr = f.records[i];
        if (rr.value_len < 0) continue;
        const uint8_t* vend = base + rr.value_off + rr.value_len;
        if (vend > pos && vend <= end) {
          crc = kafka::crc32c(pos, (size_t)(vend - pos), crc);
          pos = vend;
        }
        pre[i] = codec::scan_instances(base + rr.value_off, (size_t)rr.value_len, cfg_.H,
                                       cfg_.W, cfg_.C);
        have_pre[i] = 1;
      }
      if (end > pos) crc = kafka::crc32c(pos, (size_t)(end - pos), crc);
      if (crc != want)
        for (size_t i = 0; i < b.nrec; ++i) corrupt[b.first_rec + i] = 1;
    }
  }
  kafka::Producer* prod = producer_for(it.source);
  for (size_t i = 0; i < f.records.size(); ++i) {
    const kafka::RecordRef& rr = f.records[i];
    InRecord r;
    r.buf = f.buf;
    r.pinned = it.pinned;
    r.value = rr.value_len >= 0 ? f.buf.get() + rr.value_off : nullptr;
    r.len = rr.value_len;
    r.key = rr.key_len >= 0 ? f.buf.get() + rr.key_off : nullptr;
    r.key_len = rr.key_len;
    r.partition = rr.partition;
    r.offset = rr.offset;
    r.timestamp_ms = rr.timestamp;
    r.t_fetch_ns = it.t_fetch_ns;
    r.source = it.source;
    ++records_in_;
    if (rr.poison) {
      r.status = codec::CORRUPT;  // a record of a batch the consumer could not decode
    } else if (!corrupt.empty() && corrupt[i]) {
      r.status = codec::CORRUPT;  // corrupt Kafka batch (CRC32C mismatch)
    } else if (r.len < 0) {
      r.status = codec::BAD_ENVELOPE;  // null value (Jackson would throw)
    } else {
      bytes_in_ += r.len;
      const codec::Scan s = !have_pre.empty() && have_pre[i]
                                ? pre[i]
                                : codec::scan_instances(r.value, (size_t)r.len, cfg_.H, cfg_.W,
                                                        cfg_.C);
      r.status = s.status;
      r.arr_off = s.arr_off;
      r.arr_len = s.arr_len;
      r.images = s.images;
      if (r.status == codec::OK && fault_hit(parse_error_p_)) r.status = codec::BAD_ENVELOPE;
    }
    if (r.status == codec::OK && r.images > cfg_.max_batch) {
      images_in_ += r.images;
      if (!split_record(r, good)) emit_error(r, codec::BAD_SHAPE, prod);
    } else if (r.status == codec::OK) {
      images_in_ += r.images;
      good.push_back(std::move(r));
    } else {
      emit_error(r, r.status, prod);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// replicas
// ---------------------------------------------------------------------------------------------

void Engine::worker_loop(ReplicaSlot* rs) {
  Replica& rep = *rs->rep;
  if (rep.device() >= 0) hipSetDevice(rep.device());
  for (;;) {
    serve(rs);
    if (!rs->restarting) return;
    // supervisor: back off (stop() interrupts), recover the replica, rejoin the pool
    const int64_t until = mono_ns() + (int64_t)cfg_.restart_backoff_ms * 1000000;
    while (!stopping_ && mono_ns() < until) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    bool ok = !stopping_;
    if (ok) {
      try {
        rep.recover();
      } catch (const std::exception& e) {
        fprintf(stderr, "[gale supervisor] replica %d (%s) recovery failed: %s\n", rs->index,
                rep.name().c_str(), e.what());
        ok = false;
      }
    }
    if (ok) {
      ++rs->restarts;
      ++replica_restarts_;
      fprintf(stderr, "[gale supervisor] replica %d (%s) restarted (%d of %d)\n", rs->index,
              rep.name().c_str(), rs->restarts.load(), cfg_.max_restarts);
      rs->alive = true;
    }
    rs->restarting = false;  // (after alive: stop() joins while either is set)
    if (!ok) return;
  }
}

void Engine::serve(ReplicaSlot* rs) {
  Replica& rep = *rs->rep;
  const size_t depth = (size_t)std::max(1, rep.depth());
  std::deque<std::shared_ptr<Batch>> mine;
  auto fail = [&](const char* what, const std::string& msg) {
    const bool restart = cfg_.max_restarts > rs->restarts && !stopping_;
    fprintf(stderr, "[gale replica %d %s] %s: %s -> replica marked dead, batches re-queued%s\n",
            rs->index, rep.name().c_str(), what, msg.c_str(),
            restart ? " (supervisor restart pending)" : "");
    std::vector<InRecord> back;
    {
      std::lock_guard<std::mutex> lk(rs->mu);
      if (rs->alive) {  // (else the watchdog killed it first: no restart on a hung device)
        if (restart) rs->restarting = true;  // before alive drops: stop() never detaches us
        rs->alive = false;
        for (auto& b : rs->inflight)
          for (const InRecord& r : b->recs) back.push_back(r);
        rs->inflight.clear();
      }
    }
    ++replica_failures_;
    requeued_ += (int64_t)back.size();
    if (!back.empty()) batchers_[(size_t)rs->slot]->requeue(std::move(back));
  };
  while (rs->alive) {
    if (mine.size() < depth) {
      auto b = std::make_shared<Batch>();
      int images = 0;
      const int64_t t_take0 = mono_ns();
      bool open;
      {
        trace::Range tr("gale:batch");
        const int maxb = eff_batch_.load(std::memory_order_relaxed);
        // (no steals with the text packed: a stolen record's host copy is sparse)
        const bool steal = batchers_.size() > 1 && !(cfg_.text_pack && !ingests_.empty());
        open = batchers_[(size_t)rs->slot]->take(maxb,
                                                 eff_wait_ns_.load(std::memory_order_relaxed),
                                                 !mine.empty(), b->recs, images,
                                                 steal ? 2000000 : 0);
        if (open && steal && b->recs.empty() && mine.empty()) {
          // idle: take from the most loaded other locality (its text then comes over PCIe
          // from the pinned host copy instead of the device mirror)
          Batcher* victim = nullptr;
          int64_t most = maxb / 2;
          for (size_t k = 0; k < batchers_.size(); ++k) {
            if ((int)k == rs->slot) continue;
            const int64_t q = batchers_[k]->queued_images();
            if (q >= most) {
              most = q;
              victim = batchers_[k].get();
            }
          }
          if (victim && victim->try_take(maxb, b->recs, images)) ++steals_;
        }
      }
      ns_take_ += mono_ns() - t_take0;
      if (!open) {
        if (mine.empty()) break;  // closed and drained
      } else if (!b->recs.empty()) {
        b->images = images;
        b->t_take_ns = mono_ns();
        for (const InRecord& r : b->recs) h_queue_us_.add((b->t_take_ns - r.t_fetch_ns) / 1000);
        const int64_t nb = ++batches_total_;
        b->t_submit_ns = mono_ns();  // before publishing: the watchdog reads it under rs->mu
        {
          std::lock_guard<std::mutex> lk(rs->mu);
          rs->inflight.push_back(b);
        }
        if (mine.empty()) rs->busy_since = b->t_submit_ns;  // (submit may do the work)
        try {
          if (crash_at_batch_ > 0 && nb == crash_at_batch_)
            throw std::runtime_error("injected replica crash (fault replica_crash@" +
                                     std::to_string(crash_at_batch_) + ")");
          {
            trace::Range tr("gale:h2d+launch");
            rep.submit(*b);
          }
          ns_submit_ += mono_ns() - b->t_submit_ns;
        } catch (const std::exception& e) {
          fail("submit", e.what());
          break;
        }
        mine.push_back(b);
        continue;
      }
    }
    if (mine.empty()) continue;
    std::shared_ptr<Batch> f = mine.front();
    const int64_t t_wait0 = mono_ns();
    try {
      trace::Range tr("gale:device-wait");
      rep.wait(*f);
    } catch (const std::exception& e) {
      fail("wait", e.what());
      break;
    }
    f->t_done_ns = mono_ns();
    ns_wait_ += f->t_done_ns - t_wait0;
    {
      std::lock_guard<std::mutex> lk(rs->mu);
      if (!rs->alive) break;  // the watchdog re-queued it already
      rs->inflight.pop_front();
    }
    mine.pop_front();
    {
      trace::Range tr("gale:encode+produce");
      finish_batch(rs, *f);
    }
    const int64_t t_fin = mono_ns();
    ns_finish_ += t_fin - f->t_done_ns;
    if (mine.empty()) {
      const int64_t since = rs->busy_since.exchange(0);
      if (since) rs->busy_ns += t_fin - since;
    }
  }
}

// One step of the latency-SLO controller (every 100 ms while slo_p99_ms > 0).
void Engine::slo_step() {
  const int64_t n = h_slo_win_us_.count();
  if (n < 16) return;  // too few completions in the window to estimate a p99
  const double p99_ms = h_slo_win_us_.quantile(0.99) * 1e-3;
  h_slo_win_us_.reset();
  const double mean_batch = h_slo_batch_.mean();
  h_slo_batch_.reset();
  const int maxb = cfg_.max_batch, minb = std::max(1, cfg_.max_batch / 32);
  const int64_t max_wait = (int64_t)cfg_.max_wait_us * 1000, min_wait = 20000;
  int b = eff_batch_.load();
  int64_t w = eff_wait_ns_.load();
  size_t queued = 0;
  for (auto& q : batchers_) queued += q->size();
  // Overload shows as records waiting anywhere - in the batchers, or still in the broker when
  // fetch/decode is the tight stage (then the batchers look empty): a latency miss under
  // overload needs capacity (bigger batches), not smaller ones. Unacknowledged records beyond
  // what the replicas hold in flight at the current batch size count as backlog.
  int64_t unacked = 0;
  for (const PartitionOffsets& o : partition_offsets()) unacked += o.lag;
  const int64_t in_flight = (int64_t)b * (int64_t)replicas_.size() * 3;
  const bool backlog =
      (int64_t)queued > (int64_t)b * (int64_t)replicas_.size() || unacked > 2 * in_flight;
  // Batches leaving (nearly) full: they form faster than the window, so the latency is set by
  // the replicas' capacity, not by batching delay - shrinking them would only cut capacity (the
  // fp8 ResNet-20 at 1.0 M img/s fell into that cycle: mean batch 256 -> 110, p99 2 -> 8-60 ms,
  // profiles/archive/r2_slo_controller_ab.txt).
  const bool full = mean_batch >= 0.9 * b;
  if (p99_ms > cfg_.slo_p99_ms) {
    if (backlog || full) {
      b = std::min(maxb, b + std::max(1, maxb / 8));  // overload: capacity first
    } else {
      b = std::max(minb, b * 3 / 4);
      w = std::max(min_wait, w * 7 / 10);
    }
  } else if (p99_ms < 0.8 * cfg_.slo_p99_ms) {
    b = std::min(maxb, b + std::max(1, maxb / 16));
    w = std::min(max_wait, w * 5 / 4 + 20000);
  } else {
    return;
  }
  eff_batch_ = b;
  eff_wait_ns_ = w;
  ++slo_adjustments_;
}

void Engine::watchdog_loop() {
  int tick = 0;
  while (running_ && !workers_done_) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (cfg_.slo_p99_ms > 0 && (++tick & 1) == 0) slo_step();
    const int64_t now = mono_ns();
    for (auto& rs : replicas_) {
      std::vector<InRecord> back;
      {
        std::lock_guard<std::mutex> lk(rs->mu);
        if (!rs->alive || rs->inflight.empty()) continue;
        const int64_t t0 = rs->inflight.front()->t_submit_ns;
        if (t0 == 0 || now - t0 < (int64_t)cfg_.watchdog_ms * 1000000) continue;
        rs->alive = false;
        rs->watchdog_killed = true;
        for (auto& b : rs->inflight)
          for (const InRecord& r : b->recs) back.push_back(r);
        rs->inflight.clear();
      }
      fprintf(stderr, "[gale watchdog] replica %d (%s) exceeded %d ms: marked dead, %zu records "
              "re-queued\n", rs->index, rs->rep->name().c_str(), cfg_.watchdog_ms, back.size());
      ++replica_failures_;
      requeued_ += (int64_t)back.size();
      batchers_[(size_t)rs->slot]->requeue(std::move(back));
    }
  }
}

void Engine::finish_batch(ReplicaSlot* rs, Batch& b) {
  h_device_us_.add((b.t_done_ns - b.t_submit_ns) / 1000);
  h_batch_images_.add(b.images);
  if (cfg_.slo_p99_ms > 0) h_slo_batch_.add(b.images);
  rs->batches++;
  rs->images += b.images;
  rs->records += (int64_t)b.recs.size();
  kafka::Producer* prod = producer_for(rs->index);
  const bool js = cfg_.value_format == "json-string";
  const bool java8 = cfg_.float_format == "java8";
  auto encode_ok = [&](const InRecord& r, int img, std::string& out, bool jstr) {
    if (b.pred_text)
      codec::encode_predictions_text(b.pred_text + (size_t)img * cfg_.classes * 16, r.images,
                                     cfg_.classes, jstr, out);
    else
      codec::encode_predictions(b.probs + (size_t)img * cfg_.classes, r.images, cfg_.classes,
                                jstr, out, java8);
  };
  int img = 0;
  std::string out;
  // The batch's outputs leave as ONE record group: one producer call and one acknowledgement
  // for the batch's records, in order (the producer splits the group by partition when its
  // partitioner chooses per record). Records sent one by one cost ~1 us each in allocations,
  // producer lock round trips and per-record callbacks, at 1.5 M records/s ~1.5 cores.
  kafka::RecordGroup g;
  g.off.reserve(b.recs.size() + 1);
  g.off.push_back(0);
  g.values.reserve(b.recs.size() * (size_t)(cfg_.classes * 13 + 24));
  const bool keyed = cfg_.output_key == "input";
  if (keyed) g.koff.push_back(0);
  if (cfg_.type_id_header) g.headers.push_back({"__TypeId__", "java.lang.String", false});
  auto metas = std::make_shared<std::vector<InRecord>>();
  metas->reserve(b.recs.size());
  for (size_t i = 0; i < b.recs.size(); ++i) {
    InRecord& r = b.recs[i];
    if (r.status == codec::OK && i < b.dev_status.size()) r.status = b.dev_status[i];
    if (r.split) {  // a fragment of an oversized record: its rows join the others'
      std::string rows;
      if (r.status == codec::OK) {
        encode_ok(r, img, out, false);
        rows.assign(out, 16, out.size() - 18);  // {"predictions":[ rows ]}
      }
      fragment_done(r, std::move(rows), r.status, prod);
      img += r.images;
      continue;
    }
    InRecord meta;
    meta.partition = r.partition;
    meta.offset = r.offset;
    meta.timestamp_ms = r.timestamp_ms;
    meta.t_fetch_ns = r.t_fetch_ns;
    meta.t_take_ns = b.t_take_ns;
    meta.t_ready_ns = r.t_ready_ns;
    meta.t_done_ns = b.t_done_ns;
    meta.images = r.status == codec::OK ? r.images : 0;
    bool null_value = false;
    if (r.status != codec::OK) {
      ++errors_;
      err_by_status_[r.status & 15]++;
      if (cfg_.on_error == "drop") {
        ++dropped_;
        complete_record(meta, true);
        img += r.images;
        continue;
      }
      if (cfg_.on_error == "null") {
        null_value = true;
      } else {
        codec::encode_error(r.status, "", js, out);
        g.values += out;
      }
    } else {
      encode_ok(r, img, out, js);
      g.values += out;
    }
    img += r.images;
    g.off.push_back((uint32_t)g.values.size());
    if (null_value) {
      if (g.null_value.empty()) g.null_value.assign(metas->size(), 0);
      g.null_value.push_back(1);
    } else if (!g.null_value.empty()) {
      g.null_value.push_back(0);
    }
    if (keyed) {
      const bool has = r.key_len >= 0 && r.key;
      if (has) g.keys.append(reinterpret_cast<const char*>(r.key), (size_t)r.key_len);
      g.koff.push_back((uint32_t)g.keys.size());
      g.key_null.push_back(has ? 0 : 1);
    }
    metas->push_back(meta);
  }
  if (metas->empty()) return;
  const bool ff = cfg_.sink_mode == "fire-and-forget";
  kafka::GroupCallback cb;
  if (!ff)
    cb = [this, metas](int16_t err, int32_t, int64_t, size_t) {
      complete_records(*metas, err == 0);
    };
  try {
    prod->send_group(cfg_.output_topic, cfg_.output_partition, std::move(g), std::move(cb));
  } catch (const std::exception& e) {
    fprintf(stderr, "[gale sink] send failed: %s\n", e.what());
    complete_records(*metas, false);
    return;
  }
  if (ff) complete_records(*metas, true);  // KafkaBolt fire-and-forget acks immediately
  if (cfg_.sink_mode == "sync") prod->flush();
}

// ---------------------------------------------------------------------------------------------
// sink
// ---------------------------------------------------------------------------------------------

// A record group's acknowledgement: one pending-window update for all of its records.
void Engine::complete_records(const std::vector<InRecord>& rs, bool ok) {
  const int64_t now = mono_ns();
  if (!ok && cfg_.delivery == "at-least-once") {
    undelivered(rs);
  } else {
    std::lock_guard<std::mutex> lk(pend_mu_);
    for (const InRecord& r : rs) {
      auto it = pending_.find(r.partition);
      if (it != pending_.end()) it->second.done(r.offset);
    }
  }
  const int64_t wall = wall_ms_now();
  int64_t imgs = 0;
  if (ok) {
    for (const InRecord& r : rs) {
      imgs += r.images;
      h_engine_e2e_us_.add((now - r.t_fetch_ns) / 1000);
      if (cfg_.slo_p99_ms > 0) h_slo_win_us_.add((now - r.t_fetch_ns) / 1000);
      if (r.timestamp_ms > 0) h_record_e2e_ms_.add(wall - r.timestamp_ms);
    }
    records_out_ += (int64_t)rs.size();
    images_out_ += imgs;
  } else {
    produce_failures_ += (int64_t)rs.size();
  }
  t_last_ns_ = now;
  if (ok && ack_log_on_.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> lk(ack_mu_);
    for (size_t i = 0; i < rs.size() && ack_n_ < ack_cap_; ++i)
      ack_push({rs[i].partition, rs[i].offset, now, rs[i].t_fetch_ns, rs[i].t_take_ns,
                rs[i].t_done_ns, rs[i].t_ready_ns});
  }
  note_completed(completed_ += (int64_t)rs.size(), now);
}

void Engine::undelivered(const std::vector<InRecord>& rs) {
  if (rs.empty()) return;
  undelivered_ += (int64_t)rs.size();
  if (!delivery_failed_.exchange(true))
    fprintf(stderr, "[gale sink] at-least-once: %zu output(s) not acknowledged after %d "
            "retr%s (first: input partition %d offset %lld); their offsets stay uncommitted, "
            "delivery_failed raised\n", rs.size(), cfg_.producer_retries,
            cfg_.producer_retries == 1 ? "y" : "ies", rs[0].partition,
            (long long)rs[0].offset);
}

void Engine::note_completed(int64_t c, int64_t now) {
  const int64_t target = wait_target_.load(std::memory_order_relaxed);
  if ((cfg_.max_records > 0 && c >= cfg_.max_records) || (target > 0 && c >= target)) {
    std::lock_guard<std::mutex> lk(done_mu_);
    if (target > 0 && c >= target && hit_target_ != target) {
      hit_target_ = target;
      hit_ns_ = now;
      hit_c_ = c;
    }
    done_cv_.notify_all();
  }
}

void Engine::complete_record(const InRecord& r, bool ok) {
  if (!ok && cfg_.delivery == "at-least-once") {
    undelivered({r});
  } else {
    std::lock_guard<std::mutex> lk(pend_mu_);
    auto it = pending_.find(r.partition);
    if (it != pending_.end()) it->second.done(r.offset);
  }
  const int64_t now = mono_ns();
  if (ok) {
    ++records_out_;
    images_out_ += r.images;
    h_engine_e2e_us_.add((now - r.t_fetch_ns) / 1000);
    if (cfg_.slo_p99_ms > 0) h_slo_win_us_.add((now - r.t_fetch_ns) / 1000);
    if (r.timestamp_ms > 0) h_record_e2e_ms_.add(wall_ms_now() - r.timestamp_ms);
  } else {
    ++produce_failures_;
  }
  t_last_ns_ = now;
  if (ack_log_on_.load(std::memory_order_relaxed) && ok) {
    std::lock_guard<std::mutex> lk(ack_mu_);
    if (ack_n_ < ack_cap_)
      ack_push({r.partition, r.offset, now, r.t_fetch_ns, r.t_take_ns, r.t_done_ns,
                r.t_ready_ns});
  }
  note_completed(++completed_, now);
}

void Engine::set_ack_log(bool on, size_t capacity) {
  std::lock_guard<std::mutex> lk(ack_mu_);
  if (on) {
    ack_n_ = 0;
    ack_cap_ = capacity;
    // blocks allocated and touched now, before the window: no page faults or copies inside it
    const size_t nb = (std::min<size_t>(capacity, 16u << 20) + kAckBlock - 1) / kAckBlock;
    while (ack_blocks_.size() < nb) {
      ack_blocks_.emplace_back(new AckSample[kAckBlock]);
      memset(ack_blocks_.back().get(), 0, sizeof(AckSample) * kAckBlock);
    }
  }
  ack_log_on_ = on;
}

void Engine::ack_push(const AckSample& a) {
  const size_t b = ack_n_ / kAckBlock;
  if (b >= ack_blocks_.size()) ack_blocks_.emplace_back(new AckSample[kAckBlock]);
  ack_blocks_[b][ack_n_ % kAckBlock] = a;
  ++ack_n_;
}

std::vector<AckSample> Engine::take_ack_log() {
  std::lock_guard<std::mutex> lk(ack_mu_);
  std::vector<AckSample> out(ack_n_);
  for (size_t i = 0; i < ack_n_; i += kAckBlock)
    memcpy(out.data() + i, ack_blocks_[i / kAckBlock].get(),
           sizeof(AckSample) * std::min(kAckBlock, ack_n_ - i));
  ack_n_ = 0;
  return out;
}

bool Engine::wait_completed(int64_t n, int64_t timeout_ms) {
  wait_target_ = n;
  std::unique_lock<std::mutex> lk(done_mu_);
  auto pred = [&] { return !running_ || stopping_ || completed_.load() >= n; };
  if (timeout_ms < 0) done_cv_.wait(lk, pred);
  else done_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred);
  wait_target_ = 0;
  last_wait_ns_ = hit_target_ == n ? hit_ns_ : 0;
  last_wait_c_ = hit_target_ == n ? hit_c_ : 0;
  return completed_.load() >= n;
}

void Engine::emit(InRecord& r, std::string value, bool null_value, kafka::Producer* prod) {
  std::vector<kafka::Header> hs;
  if (cfg_.type_id_header) hs.push_back({"__TypeId__", "java.lang.String", false});
  // the callback keeps only what completion needs (not the fetch buffer)
  InRecord meta;
  meta.partition = r.partition;
  meta.offset = r.offset;
  meta.timestamp_ms = r.timestamp_ms;
  meta.t_fetch_ns = r.t_fetch_ns;
  meta.images = r.status == codec::OK ? r.images : 0;
  const bool ff = cfg_.sink_mode == "fire-and-forget";
  std::string key;
  const bool keyed = cfg_.output_key == "input" && r.key_len >= 0 && r.key;
  if (keyed) key.assign(reinterpret_cast<const char*>(r.key), (size_t)r.key_len);
  kafka::SendCallback cb;
  if (!ff) {
    cb = [this, meta](const kafka::SendResult& res) {
      complete_record(meta, res.error == 0);
    };
  }
  try {
    prod->send(cfg_.output_topic, cfg_.output_partition, keyed ? &key : nullptr,
               std::move(value), null_value, std::move(hs), -1, std::move(cb));
  } catch (const std::exception& e) {
    fprintf(stderr, "[gale sink] send failed: %s\n", e.what());
    complete_record(meta, false);
    return;
  }
  if (ff) complete_record(meta, true);  // KafkaBolt fire-and-forget acks immediately
}

bool Engine::split_record(InRecord& r, std::vector<InRecord>& good) {
  std::vector<std::pair<uint32_t, uint32_t>> spans;
  const uint8_t* arr = r.value + r.arr_off;
  if (!codec::split_instances(arr, (size_t)r.arr_len, spans) || (int)spans.size() != r.images)
    return false;
  const int mb = cfg_.max_batch;
  const int parts = (r.images + mb - 1) / mb;
  auto sp = std::make_shared<SplitRecord>();
  sp->parent = r;
  sp->parent.buf.reset();
  sp->parent.value = nullptr;
  sp->parent.dev_value = nullptr;
  if (r.key && r.key_len >= 0) {
    sp->key.assign(reinterpret_cast<const char*>(r.key), (size_t)r.key_len);
    sp->parent.key = reinterpret_cast<const uint8_t*>(sp->key.data());
  }
  sp->parts = parts;
  sp->rows.resize((size_t)parts);
  for (int k = 0; k < parts; ++k) {
    const int i0 = k * mb, i1 = std::min(r.images, i0 + mb);
    const size_t b = spans[(size_t)i0].first, e = spans[(size_t)i1 - 1].second;
    // a complete InstObj of its own: {"instances":[ images ]}
    static const char kHead[] = "{\"instances\":[";
    const size_t hl = sizeof(kHead) - 1;
    const size_t n = hl + (e - b) + 2;
    std::shared_ptr<uint8_t> buf = kafka::heap_alloc(n);
    memcpy(buf.get(), kHead, hl);
    memcpy(buf.get() + hl, arr + b, e - b);
    buf.get()[n - 2] = ']';
    buf.get()[n - 1] = '}';
    InRecord f;
    f.buf = std::move(buf);
    f.value = f.buf.get();
    f.len = (int32_t)n;
    f.arr_off = (int64_t)hl - 1;
    f.arr_len = (int64_t)(e - b) + 2;
    f.images = i1 - i0;
    f.status = codec::OK;
    f.partition = r.partition;
    f.offset = r.offset;
    f.timestamp_ms = r.timestamp_ms;
    f.t_fetch_ns = r.t_fetch_ns;
    f.source = r.source;
    f.split = sp;
    f.split_index = k;
    good.push_back(std::move(f));
  }
  ++split_records_;
  split_fragments_ += parts;
  return true;
}

void Engine::fragment_done(const InRecord& frag, std::string rows, int status,
                           kafka::Producer* prod) {
  SplitRecord& sp = *frag.split;
  {
    std::lock_guard<std::mutex> lk(sp.mu);
    if (status != codec::OK && sp.status == codec::OK) sp.status = status;
    sp.rows[(size_t)frag.split_index] = std::move(rows);
    if (++sp.done < sp.parts) return;
  }
  // the last fragment: one output record for the input record, rows in image order
  if (sp.status != codec::OK) {
    emit_error(sp.parent, sp.status, prod);
    return;
  }
  const bool js = cfg_.value_format == "json-string";
  const char* q = js ? "\\\"" : "\"";
  size_t total = 32;
  for (const std::string& x : sp.rows) total += x.size() + 1;
  std::string v;
  v.reserve(total);
  if (js) v.push_back('"');
  v += '{';
  v += q;
  v += "predictions";
  v += q;
  v += ":[";
  for (size_t k = 0; k < sp.rows.size(); ++k) {
    if (k) v.push_back(',');
    v += sp.rows[k];
  }
  v += "]}";
  if (js) v.push_back('"');
  emit(sp.parent, std::move(v), false, prod);
}

void Engine::emit_error(InRecord& r, int status, kafka::Producer* prod) {
  ++errors_;
  err_by_status_[status & 15]++;
  if (cfg_.on_error == "drop") {
    ++dropped_;
    InRecord meta = r;
    meta.images = 0;
    complete_record(meta, true);
    return;
  }
  if (cfg_.on_error == "null") {
    emit(r, std::string(), true, prod);
    return;
  }
  std::string v;
  codec::encode_error(status, "", cfg_.value_format == "json-string", v);
  emit(r, std::move(v), false, prod);
}

// ---------------------------------------------------------------------------------------------
// metrics
// ---------------------------------------------------------------------------------------------

std::map<std::string, double> Engine::stats() const {
  std::map<std::string, double> s;
  s["records_in"] = (double)records_in_;
  s["images_in"] = (double)images_in_;
  s["bytes_in"] = (double)bytes_in_;
  s["records_out"] = (double)records_out_;
  s["images_out"] = (double)images_out_;
  s["completed"] = (double)completed_;
  s["errors"] = (double)errors_;
  s["produce_failures"] = (double)produce_failures_;
  s["undelivered"] = (double)undelivered_;
  s["delivery_failed"] = delivery_failed_ ? 1.0 : 0.0;
  {
    std::lock_guard<std::mutex> lk(prod_mu_);
    int64_t retried = prod_retried_, req_failed = prod_req_failed_;
    for (const auto& p : producers_) {
      const kafka::ProducerStats ps = p->stats();
      retried += ps.records_retried;
      req_failed += ps.requests_failed;
    }
    s["produce_retried_records"] = (double)retried;
    s["produce_failed_requests"] = (double)req_failed;
  }
  s["dropped"] = (double)dropped_;
  s["requeued"] = (double)requeued_;
  s["replica_failures"] = (double)replica_failures_;
  s["replica_restarts"] = (double)replica_restarts_;
  s["commits"] = (double)commits_;
  s["converted_batches"] = (double)converted_batches_;
  s["poison_batches"] = (double)poison_batches_;
  s["poison_records"] = (double)poison_records_;
  s["poison_unknown_span"] = (double)poison_unknown_span_;
  s["split_records"] = (double)split_records_;
  s["sparse_fetches"] = (double)sparse_fetches_;
  s["restored_fetches"] = (double)restored_fetches_;
  {
    PinnedPool::Stats ps;
    for (const auto& pool : pools_)
      if (pool) {
        const PinnedPool::Stats q = pool->stats();
        ps.chunks += q.chunks;
        ps.in_use_max += q.in_use_max;
        ps.heap_too_large += q.heap_too_large;
        ps.heap_budget += q.heap_budget;
        ps.no_mirror += q.no_mirror;
        ps.waits += q.waits;
        ps.wait_us += q.wait_us;
      }
    s["pinned_chunks"] = (double)ps.chunks;
    s["pinned_in_use_max"] = (double)ps.in_use_max;
    s["pinned_heap_too_large"] = (double)ps.heap_too_large;
    s["pinned_heap_budget"] = (double)ps.heap_budget;
    s["pinned_no_mirror"] = (double)ps.no_mirror;
    s["pinned_waits"] = (double)ps.waits;
    s["pinned_wait_s"] = (double)ps.wait_us * 1e-6;
  }
  s["split_fragments"] = (double)split_fragments_;
  {
    int64_t lag = 0, fetch_lag = 0, lag_max = 0;
    for (const PartitionOffsets& o : partition_offsets()) {
      lag += o.lag;
      fetch_lag += o.fetch_lag;
      lag_max = std::max(lag_max, o.lag);
    }
    s["lag_records"] = (double)lag;              // storm-kafka spoutLag, summed over partitions
    s["lag_records_max"] = (double)lag_max;
    s["fetch_lag_records"] = (double)fetch_lag;  // log end - next fetch
  }
  s["batches"] = (double)batches_total_;
  size_t queued = 0;
  for (auto& q : batchers_) queued += q->size();
  s["queue_records"] = (double)queued;
  s["locality_slots"] = (double)batchers_.size();
  s["steals"] = (double)steals_;
  for (int i = 1; i < codec::kStatusCount; ++i)
    s[std::string("err_") + codec::status_name(i)] = (double)err_by_status_[i];
  const double el = (double)(t_last_ns_ - t_first_ns_) * 1e-9;
  s["elapsed_s"] = el > 0 ? el : 0;
  s["images_per_s"] = el > 0 ? (double)images_out_ / el : 0;
  auto q = [&](const char* n, const Histogram& h) {
    s[std::string(n) + "_p50"] = h.quantile(0.5);
    s[std::string(n) + "_p90"] = h.quantile(0.9);
    s[std::string(n) + "_p99"] = h.quantile(0.99);
    s[std::string(n) + "_max"] = (double)h.max();
    s[std::string(n) + "_mean"] = h.mean();
  };
  q("queue_us", h_queue_us_);
  q("device_us", h_device_us_);
  q("e2e_us", h_engine_e2e_us_);
  q("record_e2e_ms", h_record_e2e_ms_);
  q("batch_images", h_batch_images_);
  int alive = 0;
  for (auto& r : replicas_) alive += r->alive ? 1 : 0;
  s["replicas_alive"] = alive;
  s["rebalances"] = (double)rebalances_;
  s["lag_rebalances"] = (double)lag_rebalances_;
  s["lag_rebalances_skipped"] = (double)lag_rebalances_skipped_;
  s["capacity_rps"] = capacity_rps_.load();
  s["generation"] = (double)generation_;
  s["assigned_partitions"] = cfg_.group_membership ? (double)assigned_partitions_
                                                   : (double)partition_offsets().size();
  s["ingested_records"] = (double)ingested_records_;
  s["ingest_parsed_records"] = (double)ingest_parsed_;
  {
    int64_t step = 0, fwd = 0, pre = 0, tab = 0;
    for (auto& r : replicas_) {
      step += r->rep->graph_step_batches();
      fwd += r->rep->graph_forward_batches();
      pre += r->rep->preparsed_records();
      tab += r->rep->table_batches();
    }
    s["table_batches"] = (double)tab;  // steps = one forward launch, inputs in kernel arguments
    s["graph_step_batches"] = (double)step;
    s["graph_forward_batches"] = (double)fwd;
    s["preparsed_records"] = (double)pre;  // records the step took parsed from the ingest arena
  }
  {
    int64_t text = 0, link = 0;
    for (auto& kv : ingests_) {
      int64_t t = 0, l = 0;
      kv.second->link_bytes(t, l);
      text += t;
      link += l;
    }
    s["ingest_text_bytes"] = (double)text;
    s["ingest_link_bytes"] = (double)link;
  }
  s["thread_s_ingest"] = ingest_ns_ * 1e-9;
  {
    Ingest::Timing t;
    for (auto& kv : ingests_) {
      const Ingest::Timing q = kv.second->timing();
      t.runs += q.runs;
      t.prep_ns += q.prep_ns;
      t.plan_ns += q.plan_ns;
      t.wait_ns += q.wait_ns;
      t.post_ns += q.post_ns;
      t.dev_runs += q.dev_runs;
      t.dev_copy_ns += q.dev_copy_ns;
      t.dev_count_ns += q.dev_count_ns;
      t.dev_parse_ns += q.dev_parse_ns;
      t.dev_wait_ns += q.dev_wait_ns;
      t.plan_in_chunk += q.plan_in_chunk;
    }
    // per fetch, microseconds: waiting for a lane, the lane's host work before / after the
    // device, and the device wait itself
    const double n = (double)std::max<int64_t>(1, t.runs);
    s["ingest_fetches"] = (double)t.runs;
    s["ingest_lane_wait_us"] = (double)ns_lane_wait_ / n / 1e3;
    s["ingest_prep_us"] = (double)t.prep_ns / n / 1e3;
    s["ingest_device_wait_us"] = (double)t.wait_ns / n / 1e3;
    s["ingest_post_us"] = (double)t.post_ns / n / 1e3;
    s["ingest_lane_us"] = (double)ingest_ns_ / n / 1e3;  // a lane's whole turn, scan to push
    // the same as running totals (s), for per-window deltas
    s["ingest_lane_wait_s"] = (double)ns_lane_wait_ * 1e-9;
    s["ingest_prep_s"] = (double)t.prep_ns * 1e-9;
    s["ingest_plan_s"] = (double)t.plan_ns * 1e-9;
    s["ingest_device_wait_s"] = (double)t.wait_ns * 1e-9;
    s["ingest_post_s"] = (double)t.post_ns * 1e-9;
    // sampled device spans (GALE_INGEST_DEV_TIMING), running totals
    s["ingest_plan_in_chunk"] = (double)t.plan_in_chunk;
    s["ingest_dev_runs"] = (double)t.dev_runs;
    s["ingest_dev_copy_s"] = (double)t.dev_copy_ns * 1e-9;
    s["ingest_dev_count_s"] = (double)t.dev_count_ns * 1e-9;
    s["ingest_dev_parse_s"] = (double)t.dev_parse_ns * 1e-9;
    s["ingest_dev_wait_s"] = (double)t.dev_wait_ns * 1e-9;
  }
  s["eff_max_batch"] = (double)eff_batch_;
  s["eff_max_wait_us"] = (double)eff_wait_ns_ / 1000.0;
  s["slo_adjustments"] = (double)slo_adjustments_;
  s["thread_s_poll"] = ns_poll_ * 1e-9;
  s["thread_s_handoff"] = ns_handoff_ * 1e-9;
  s["thread_s_decode"] = ns_decode_ * 1e-9;
  s["thread_s_take"] = ns_take_ * 1e-9;
  s["thread_s_submit"] = ns_submit_ * 1e-9;
  s["thread_s_wait"] = ns_wait_ * 1e-9;
  s["thread_s_finish"] = ns_finish_ * 1e-9;
  return s;
}

std::vector<ReplicaStats> Engine::replica_stats() const {
  std::vector<ReplicaStats> v;
  for (auto& r : replicas_) {
    ReplicaStats s;
    s.name = r->rep->name();
    s.device = r->rep->device();
    s.alive = r->alive;
    s.batches = r->batches;
    s.images = r->images;
    s.records = r->records;
    s.restarts = r->restarts;
    s.slot = r->slot;
    s.resident_records = r->rep->resident_records();
    s.host_records = r->rep->host_records();
    v.push_back(s);
  }
  return v;
}

std::vector<PartitionOffsets> Engine::partition_offsets() const {
  std::vector<PartitionOffsets> v;
  std::lock_guard<std::mutex> lk(const_cast<std::mutex&>(pend_mu_));
  for (const auto& kv : next_fetch_) {
    PartitionOffsets o;
    o.partition = kv.first;
    o.fetched = kv.second;
    auto pit = pending_.find(kv.first);
    o.committed = (pit != pending_.end() && !pit->second.empty()) ? pit->second.first()
                                                                  : kv.second;
    auto hit = high_watermark_.find(kv.first);
    o.high_watermark = hit != high_watermark_.end() ? hit->second : -1;
    if (o.high_watermark >= 0) {
      o.lag = std::max<int64_t>(0, o.high_watermark - o.committed);
      o.fetch_lag = std::max<int64_t>(0, o.high_watermark - o.fetched);
    }
    v.push_back(o);
  }
  return v;
}

void Engine::reset_stats() {
  h_queue_us_.reset();
  h_device_us_.reset();
  h_engine_e2e_us_.reset();
  h_record_e2e_ms_.reset();
  h_batch_images_.reset();
  images_out_ = 0;
  records_out_ = 0;
  bytes_in_ = 0;  // (json MB/s of a window = bytes fetched inside it)
  ns_poll_ = ns_decode_ = ns_take_ = ns_submit_ = ns_wait_ = ns_finish_ = ns_handoff_ = 0;
  t_first_ns_ = mono_ns();
  t_last_ns_ = t_first_ns_.load();
}

}  // namespace gale
