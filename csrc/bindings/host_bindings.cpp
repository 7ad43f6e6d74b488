// Python bindings of the host runtime: JSON codec, Kafka wire protocol / broker / client.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <time.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

#include "../codec/json_codec.h"
#include "gale/llc_pair.h"
#include "../codec/text_pack.h"
#include "../kafka/broker.h"
#include "../kafka/client.h"
#include "../kafka/compress.h"
#include "../kafka/fetch_framing.h"
#include "../runtime/pack_tap.h"
#include "../kafka/protocol.h"
#include "../kafka/wire.h"

namespace py = pybind11;

namespace gale {

void bind_engine(py::module_& m);  // engine_bindings.cpp

namespace {

using namespace gale::kafka;

std::string_view view(const py::bytes& b) {
  char* p;
  Py_ssize_t n;
  PyBytes_AsStringAndSize(b.ptr(), &p, &n);
  return std::string_view(p, (size_t)n);
}

py::object opt_bytes(const uint8_t* base, int64_t off, int32_t len) {
  if (len < 0) return py::none();
  return py::bytes(reinterpret_cast<const char*>(base + off), (size_t)len);
}

py::list records_to_py(const uint8_t* base, const std::vector<RecordRef>& recs) {
  py::list out;
  for (const RecordRef& r : recs) {
    py::dict d;
    d["partition"] = r.partition;
    d["offset"] = r.offset;
    d["timestamp"] = r.timestamp;
    d["key"] = opt_bytes(base, r.key_off, r.key_len);
    d["value"] = opt_bytes(base, r.value_off, r.value_len);
    py::list hs;
    for (const Header& h : decode_headers(base, r))
      hs.append(py::make_tuple(h.key, h.value_null ? py::object(py::none())
                                                   : py::object(py::bytes(h.value))));
    d["headers"] = hs;
    if (r.poison) d["poison"] = true;
    out.append(d);
  }
  return out;
}

// decode_records, falling back to the consumer's normalisation (compress.h) for compressed /
// legacy / corrupt blobs; `hold` keeps the normalised bytes the records point into
const uint8_t* decode_any(const std::string_view s, int64_t min_offset, bool check_crc,
                          std::string& hold, std::vector<RecordRef>& recs) {
  const uint8_t* base = reinterpret_cast<const uint8_t*>(s.data());
  try {
    decode_records(base, 0, s.size(), min_offset, check_crc, recs);
    return base;
  } catch (const ProtocolError&) {
    recs.clear();
    NormalizeStats st;
    hold = normalize_records(base, s.size(), min_offset, check_crc, (size_t)1 << 30, st);
    const uint8_t* hb = reinterpret_cast<const uint8_t*>(hold.data());
    decode_records(hb, 0, hold.size(), min_offset, false, recs, nullptr, true);
    return hb;
  }
}

std::vector<Header> headers_from_py(const py::object& o) {
  std::vector<Header> hs;
  if (o.is_none()) return hs;
  for (auto item : o) {
    auto t = item.cast<py::tuple>();
    Header h;
    h.key = t[0].cast<std::string>();
    if (t[1].is_none()) h.value_null = true;
    else h.value = std::string(view(t[1].cast<py::bytes>()));
    hs.push_back(std::move(h));
  }
  return hs;
}

// Batch encode from python: records = [(key|None, value|None, timestamp, headers|None), ...]
py::bytes py_encode_batch(py::list records, int64_t base_offset, int64_t base_ts) {
  std::vector<std::string> keys(records.size()), vals(records.size());
  std::vector<std::vector<Header>> hdrs(records.size());
  std::vector<RecordIn> ins(records.size());
  for (size_t i = 0; i < records.size(); ++i) {
    auto t = records[i].cast<py::tuple>();
    if (!t[0].is_none()) {
      keys[i] = std::string(view(t[0].cast<py::bytes>()));
      ins[i].key = keys[i];
      ins[i].key_null = false;
    }
    if (t[1].is_none()) {
      ins[i].value_null = true;
    } else {
      vals[i] = std::string(view(t[1].cast<py::bytes>()));
      ins[i].value = vals[i];
    }
    ins[i].timestamp = t.size() > 2 ? t[2].cast<int64_t>() : -1;
    if (t.size() > 3) {
      hdrs[i] = headers_from_py(t[3]);
      if (!hdrs[i].empty()) ins[i].headers = &hdrs[i];
    }
  }
  Writer w;
  encode_batch(w, ins.data(), ins.size(), base_offset, base_ts);
  return py::bytes(w.buf);
}

// Pre-encoded RecordBatch v2 blobs held natively and appended to the embedded broker by
// reference (bench preloading / open-loop feeding): the distinct payload is materialised once.
struct BatchSet {
  std::vector<std::shared_ptr<const std::string>> batches;
  std::vector<int32_t> records;  // records per batch
  int64_t images_per_record = 1;
  size_t bytes = 0;
};

// Open-loop producer of the benchmark's offered load: appends the batches of a BatchSet (by
// reference) to an embedded broker's partitions at a fixed record rate, round-robin over the
// partitions, and logs each append as (partition, base offset, records, CLOCK_MONOTONIC ns). The
// log is the "record appended" end of the record-level latency (bench.py latency phase); the
// engine's ack log (Engine::ack_log) is the other end - both on the same monotonic clock.
class RateFeeder {
 public:
  RateFeeder(std::shared_ptr<Broker> b, std::string topic, std::vector<int> parts,
             std::shared_ptr<BatchSet> set)
      : b_(std::move(b)), topic_(std::move(topic)), parts_(std::move(parts)),
        set_(std::move(set)) {
    if (parts_.empty() || !set_ || set_->batches.empty())
      throw std::invalid_argument("RateFeeder: no partitions or empty BatchSet");
  }
  ~RateFeeder() { stop(); }
  void start(double records_per_s, int64_t start_batch) {
    if (t_.joinable()) throw std::logic_error("RateFeeder: already running");
    if (records_per_s <= 0) throw std::invalid_argument("RateFeeder: rate must be > 0");
    stop_ = false;
    next_ = start_batch;
    {
      // room for a long window up front: the appends are timestamped, a growth copy would
      // delay the next ones
      std::lock_guard<std::mutex> lk(mu_);
      for (auto* v : {&lp_, &ln_}) v->reserve(1 << 18);
      for (auto* v : {&lbase_, &lt_}) v->reserve(1 << 18);
    }
    t_ = std::thread([this, records_per_s] { run(records_per_s); });
  }
  void stop() {
    stop_ = true;
    if (t_.joinable()) t_.join();
  }
  int64_t next_batch() const { return next_; }
  // (partition, base_offset, records, t_ns) arrays; clears the log
  py::tuple take_log() {
    std::vector<int32_t> p;
    std::vector<int64_t> base, t;
    std::vector<int32_t> n;
    {
      std::lock_guard<std::mutex> lk(mu_);
      p.swap(lp_);
      base.swap(lbase_);
      n.swap(ln_);
      t.swap(lt_);
    }
    return py::make_tuple(py::array_t<int32_t>(p.size(), p.data()),
                          py::array_t<int64_t>(base.size(), base.data()),
                          py::array_t<int32_t>(n.size(), n.data()),
                          py::array_t<int64_t>(t.size(), t.data()));
  }
  int64_t appended_records() const { return appended_; }

 private:
  static int64_t now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
  }
  void run(double rate) {
    const int64_t t0 = now_ns();
    const int64_t m = (int64_t)set_->batches.size();
    size_t pi = 0;
    int64_t sent = 0;
    while (!stop_) {
      const double due = (double)(now_ns() - t0) * 1e-9 * rate;
      while (!stop_) {
        const size_t k = (size_t)(((next_ % m) + m) % m);
        const int32_t nrec = set_->records[k];
        if ((double)(sent + nrec) > due) break;
        const int part = parts_[pi++ % parts_.size()];
        const int64_t base = b_->append_shared(topic_, part, set_->batches[k]);
        const int64_t t = now_ns();
        {
          std::lock_guard<std::mutex> lk(mu_);
          lp_.push_back(part);
          lbase_.push_back(base);
          ln_.push_back(nrec);
          lt_.push_back(t);
        }
        sent += nrec;
        appended_ += nrec;
        ++next_;
      }
      // sleep until the next batch is due (at least 20 us: a loop that polls the clock would
      // take a core from the pipeline under test)
      const int32_t nrec = set_->records[(size_t)(((next_ % m) + m) % m)];
      const double wait_s = ((double)(sent + nrec) - (double)(now_ns() - t0) * 1e-9 * rate) / rate;
      std::this_thread::sleep_for(std::chrono::nanoseconds(
          std::max<int64_t>(20000, (int64_t)(wait_s * 1e9))));
    }
  }
  std::shared_ptr<Broker> b_;
  std::string topic_;
  std::vector<int> parts_;
  std::shared_ptr<BatchSet> set_;
  std::thread t_;
  std::atomic<bool> stop_{true};
  std::atomic<int64_t> next_{0}, appended_{0};
  std::mutex mu_;
  std::vector<int32_t> lp_, ln_;
  std::vector<int64_t> lbase_, lt_;
};

// Encode images [N, H, W, C] as InstObj JSON records (images_per_record each, Java float text)
// grouped records_per_batch per Kafka batch, on `threads` threads. key_prefix non-empty: record
// j (0-based over the whole set) gets key "<key_prefix><j>".
std::shared_ptr<BatchSet> synthetic_batches(const float* x, int64_t n, int H, int W, int C,
                                            int ipr, int rpb, int threads,
                                            const std::string& key_prefix) {
  if (ipr <= 0 || rpb <= 0 || n <= 0) throw std::invalid_argument("synthetic_batches: bad sizes");
  auto bs = std::make_shared<BatchSet>();
  bs->images_per_record = ipr;
  const int64_t nrec = (n + ipr - 1) / ipr;
  const int64_t nb = (nrec + rpb - 1) / rpb;
  bs->batches.resize((size_t)nb);
  bs->records.resize((size_t)nb);
  const size_t img = (size_t)H * W * C;
  std::atomic<int64_t> next{0};
  auto work = [&] {
    std::vector<std::string> vals, keys;
    std::vector<RecordIn> ins;
    for (int64_t b; (b = next++) < nb;) {
      const int64_t r0 = b * rpb, r1 = std::min<int64_t>(nrec, r0 + rpb);
      vals.assign((size_t)(r1 - r0), std::string());
      keys.assign((size_t)(r1 - r0), std::string());
      ins.assign((size_t)(r1 - r0), RecordIn());
      for (int64_t r = r0; r < r1; ++r) {
        const int64_t i0 = r * ipr, cnt = std::min<int64_t>(ipr, n - i0);
        codec::encode_instances(x + (size_t)i0 * img, (int)cnt, H, W, C, vals[(size_t)(r - r0)]);
        RecordIn& ri = ins[(size_t)(r - r0)];
        ri.value = vals[(size_t)(r - r0)];
        if (!key_prefix.empty()) {
          keys[(size_t)(r - r0)] = key_prefix + std::to_string(r);
          ri.key = keys[(size_t)(r - r0)];
          ri.key_null = false;
        }
      }
      Writer w;
      encode_batch(w, ins.data(), ins.size(), 0, 0);
      bs->records[(size_t)b] = (int32_t)(r1 - r0);
      bs->batches[(size_t)b] = std::make_shared<const std::string>(std::move(w.buf));
    }
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < std::max(1, threads); ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  for (auto& b : bs->batches) bs->bytes += b->size();
  return bs;
}

std::vector<std::string> strs(const py::handle& o) { return o.cast<std::vector<std::string>>(); }

// Encode a request body by message name (golden-byte tests of the protocol layer).
py::bytes py_encode(const std::string& name, py::dict d) {
  Writer w;
  if (name == "request_header") {
    RequestHeader h;
    h.api_key = d["api_key"].cast<int16_t>();
    h.api_version = d["api_version"].cast<int16_t>();
    h.correlation_id = d["correlation_id"].cast<int32_t>();
    h.client_id = d["client_id"].cast<std::string>();
    encode_request_header(w, h);
  } else if (name == "metadata_request") {
    MetadataRequest m;
    if (d["topics"].is_none()) m.all_topics = true;
    else m.topics = strs(d["topics"]);
    m.allow_auto_topic_creation = d["allow_auto_topic_creation"].cast<bool>();
    encode_metadata_request(w, m);
  } else if (name == "fetch_request") {
    FetchRequest m;
    m.max_wait_ms = d["max_wait_ms"].cast<int32_t>();
    m.min_bytes = d["min_bytes"].cast<int32_t>();
    m.max_bytes = d["max_bytes"].cast<int32_t>();
    FetchTopic t;
    t.name = d["topic"].cast<std::string>();
    for (auto p : d["partitions"].cast<py::list>()) {
      auto tp = p.cast<py::tuple>();
      t.partitions.push_back({tp[0].cast<int32_t>(), tp[1].cast<int64_t>(), tp[2].cast<int32_t>()});
    }
    m.topics.push_back(t);
    encode_fetch_request(w, m);
  } else if (name == "produce_request") {
    ProduceRequest m;
    m.acks = d["acks"].cast<int16_t>();
    m.timeout_ms = d["timeout_ms"].cast<int32_t>();
    ProduceTopic t;
    t.name = d["topic"].cast<std::string>();
    ProducePartition pp;
    pp.index = d["partition"].cast<int32_t>();
    pp.records = std::string(view(d["records"].cast<py::bytes>()));
    t.partitions.push_back(pp);
    m.topics.push_back(t);
    encode_produce_request(w, m);
  } else if (name == "list_offsets_request") {
    ListOffsetsRequest m;
    m.topics.push_back({d["topic"].cast<std::string>(),
                        {{d["partition"].cast<int32_t>(), d["timestamp"].cast<int64_t>()}}});
    encode_list_offsets_request(w, m);
  } else if (name == "offset_commit_request") {
    OffsetCommitRequest m;
    m.group_id = d["group_id"].cast<std::string>();
    CommitTopic t;
    t.name = d["topic"].cast<std::string>();
    CommitPartition cp;
    cp.index = d["partition"].cast<int32_t>();
    cp.offset = d["offset"].cast<int64_t>();
    t.partitions.push_back(cp);
    m.topics.push_back(t);
    encode_offset_commit_request(w, m);
  } else {
    throw std::invalid_argument("unknown message " + name);
  }
  return py::bytes(w.buf);
}

py::dict py_decode(const std::string& name, py::bytes b) {
  const std::string_view s = view(b);
  Reader r(s);
  py::dict d;
  if (name == "metadata_response") {
    const MetadataResponse m = decode_metadata_response(r);
    py::list brokers;
    for (auto& n : m.brokers) brokers.append(py::make_tuple(n.node_id, n.host, n.port));
    d["brokers"] = brokers;
    d["cluster_id"] = m.cluster_id;
    d["controller_id"] = m.controller_id;
    py::dict topics;
    for (auto& t : m.topics) {
      py::list parts;
      for (auto& p : t.partitions) parts.append(py::make_tuple(p.index, p.leader, p.error));
      topics[py::str(t.name)] = py::make_tuple(t.error, parts);
    }
    d["topics"] = topics;
  } else if (name == "produce_response") {
    const ProduceResponse m = decode_produce_response(r);
    py::list parts;
    for (auto& t : m.topics)
      for (auto& p : t.partitions)
        parts.append(py::make_tuple(t.name, p.index, p.error, p.base_offset));
    d["partitions"] = parts;
    d["throttle_ms"] = m.throttle_ms;
  } else if (name == "fetch_response") {
    const FetchResponse m = decode_fetch_response(r);
    py::list parts;
    for (auto& t : m.topics)
      for (auto& p : t.partitions) {
        std::vector<RecordRef> recs;
        if (p.records_len > 0)
          decode_records(reinterpret_cast<const uint8_t*>(s.data()), p.records_off,
                         (size_t)p.records_len, 0, true, recs);
        parts.append(py::make_tuple(t.name, p.index, p.error, p.high_watermark,
                                    records_to_py(reinterpret_cast<const uint8_t*>(s.data()), recs)));
      }
    d["partitions"] = parts;
  } else if (name == "api_versions_response") {
    const ApiVersionsResponse m = decode_api_versions_response(r);
    d["error"] = m.error;
    py::dict apis;
    for (auto& a : m.apis) apis[py::int_(a.key)] = py::make_tuple(a.min_version, a.max_version);
    d["apis"] = apis;
  } else {
    throw std::invalid_argument("unknown message " + name);
  }
  return d;
}

// Python callables held by C++ must be released with the GIL held.
std::shared_ptr<py::object> hold(py::object o) {
  return std::shared_ptr<py::object>(new py::object(std::move(o)), [](py::object* p) {
    py::gil_scoped_acquire g;
    delete p;
  });
}

}  // namespace

void bind_host(py::module_& m) {
  // ---- JSON codec ----
  m.def("status_name", &codec::status_name);
  m.def("scan_instances", [](py::bytes b, int H, int W, int C) {
    const std::string_view s = view(b);
    const codec::Scan sc =
        codec::scan_instances(reinterpret_cast<const uint8_t*>(s.data()), s.size(), H, W, C);
    return py::make_tuple(sc.status, sc.arr_off, sc.arr_len, sc.images);
  });
  m.def("parse_instances_host", [](py::bytes b, int H, int W, int C, int max_images) {
    const std::string_view s = view(b);
    const codec::Scan sc =
        codec::scan_instances(reinterpret_cast<const uint8_t*>(s.data()), s.size(), H, W, C);
    const int n = sc.status == codec::OK ? sc.images : 0;
    py::array_t<float> out({(py::ssize_t)n, (py::ssize_t)H, (py::ssize_t)W, (py::ssize_t)C});
    int images = 0;
    int st = sc.status;
    if (st == codec::OK)
      st = codec::parse_instances_host(reinterpret_cast<const uint8_t*>(s.data()), s.size(), H, W,
                                       C, out.mutable_data(), max_images, &images);
    return py::make_tuple(st, out);
  }, py::arg("data"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("max_images") = -1);
  // ---- nibble transport (text_pack.h) ----
  m.def("text_pack_fast", &codec::text_pack_fast);
  // L3-domain pairing (gale/llc_pair.h), for tests: each call acts on the calling thread
  m.def("llc_pin_self_next_domain", &llc::pin_self_next_domain);
  m.def("llc_register_local_port", &llc::register_local_port);
  m.def("llc_pin_self_for_peer", &llc::pin_self_for_peer);
  m.def("set_pack_stream_stores", &codec::set_pack_stream_stores,
        "non-temporal stores for the packed stream (default on; A/B switch)");
  m.def("text_pack", [](py::bytes b, bool force_scalar) {
    const std::string_view s = view(b);
    std::string out(codec::pack_bound(s.size()), '\0');
    py::array_t<uint32_t> tab((py::ssize_t)(2 * codec::pack_groups(s.size())));
    const size_t n = codec::text_pack(reinterpret_cast<const uint8_t*>(s.data()), s.size(),
                                      reinterpret_cast<uint8_t*>(out.data()), tab.mutable_data(),
                                      force_scalar);
    out.resize(n);
    return py::make_tuple(py::bytes(out), tab);
  }, py::arg("data"), py::arg("force_scalar") = false);
  m.def("text_pack_chunked", [](py::bytes b, std::vector<size_t> cuts) {
    // resumable packing as a receive loop drives it: progress at every cut, then finish
    const std::string_view s = view(b);
    const auto* src = reinterpret_cast<const uint8_t*>(s.data());
    std::string out(codec::pack_bound(s.size()), '\0');
    py::array_t<uint32_t> tab((py::ssize_t)(2 * codec::pack_groups(s.size())));
    codec::PackState st;
    auto* dst = reinterpret_cast<uint8_t*>(out.data());
    for (size_t c : cuts)
      codec::text_pack_blocks(src, std::min(c, s.size()) / codec::kPackBlock, dst,
                              tab.mutable_data(), st);
    out.resize(codec::text_pack_finish(src, s.size(), dst, tab.mutable_data(), st));
    return py::make_tuple(py::bytes(out), tab);
  });
  m.def("text_unpack_host", [](py::bytes packed, py::array_t<uint32_t, py::array::c_style> tab,
                               size_t n) {
    std::string out(n, '\0');
    codec::text_unpack_host(reinterpret_cast<const uint8_t*>(view(packed).data()), tab.data(), n,
                            reinterpret_cast<uint8_t*>(out.data()));
    return py::bytes(out);
  });
  m.def("text_pack_bench_ptr", [](uintptr_t src, size_t n, uintptr_t dst, uintptr_t tab,
                                  int iters) {
    // seconds per pass: packing between caller-provided buffers (e.g. pinned vs pageable)
    size_t out = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i)
      out = codec::text_pack(reinterpret_cast<const uint8_t*>(src), n,
                             reinterpret_cast<uint8_t*>(dst), reinterpret_cast<uint32_t*>(tab));
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return py::make_tuple(dt / std::max(1, iters), out);
  });
  m.def("text_pack_bench", [](py::bytes b, int iters, bool force_scalar) {
    // seconds per pass over b (host packing throughput)
    const std::string_view s = view(b);
    std::vector<uint8_t> out(codec::pack_bound(s.size()) + 64);
    std::vector<uint32_t> tab(2 * codec::pack_groups(s.size()) + 2);
    size_t n = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i)
      n = codec::text_pack(reinterpret_cast<const uint8_t*>(s.data()), s.size(), out.data(),
                           tab.data(), force_scalar);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return py::make_tuple(dt / std::max(1, iters), n);
  }, py::arg("data"), py::arg("iters") = 10, py::arg("force_scalar") = false);
  m.def("format_float_java8", [](float v) {
    char buf[48];
    return std::string(buf, (size_t)codec::format_float_java8(v, buf));
  });
  m.def("format_float_java", [](float v) {
    char buf[48];
    return std::string(buf, (size_t)codec::format_float_java(v, buf));
  });
  m.def("encode_predictions", [](py::array_t<float, py::array::c_style | py::array::forcecast> p,
                                 bool json_string, bool java8) {
    if (p.ndim() != 2) throw std::invalid_argument("predictions must be [N, classes]");
    std::string out;
    codec::encode_predictions(p.data(), (int)p.shape(0), (int)p.shape(1), json_string, out,
                              java8);
    return py::bytes(out);
  }, py::arg("probs"), py::arg("json_string") = false, py::arg("java8") = false);
  m.def("encode_predictions_text", [](py::bytes text16, int n, int classes, bool json_string) {
    const std::string t = text16;
    if (n < 0 || classes <= 0 || t.size() != (size_t)n * classes * 16)
      throw std::invalid_argument("text16 must hold n * classes 16-byte slots");
    for (size_t i = 15; i < t.size(); i += 16)
      if ((unsigned char)t[i] > 15) throw std::invalid_argument("slot length > 15");
    std::string out;
    codec::encode_predictions_text(reinterpret_cast<const uint8_t*>(t.data()), n, classes,
                                   json_string, out);
    return py::bytes(out);
  }, py::arg("text16"), py::arg("n"), py::arg("classes"), py::arg("json_string") = false);
  m.def("encode_instances", [](py::array_t<float, py::array::c_style | py::array::forcecast> x) {
    if (x.ndim() != 4) throw std::invalid_argument("instances must be [N, H, W, C]");
    std::string out;
    {
      py::gil_scoped_release nogil;
      codec::encode_instances(x.data(), (int)x.shape(0), (int)x.shape(1), (int)x.shape(2),
                              (int)x.shape(3), out);
    }
    return py::bytes(out);
  });
  m.def("encode_error", [](int status, const std::string& detail, bool json_string) {
    std::string out;
    codec::encode_error(status, detail.c_str(), json_string, out);
    return py::bytes(out);
  });

  // ---- Kafka wire ----
  py::module_ k = m.def_submodule("kafka", "Kafka wire protocol, embedded broker and client");
  k.def("crc32c", [](py::bytes b) {
    const std::string_view s = view(b);
    return crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  k.def("group_assign", &GroupMember::assign, py::arg("assignor"), py::arg("members"),
        py::arg("partitions"));
  k.def("group_assign_load_aware", [](std::vector<std::string> members, py::dict loads, int n) {
    // loads: member -> (capacity records/s, [owned partitions])
    std::map<std::string, MemberLoad> m;
    for (auto kv : loads) {
      auto t = kv.second.cast<py::tuple>();
      MemberLoad ml;
      ml.capacity = t[0].cast<double>();
      ml.owned = t[1].cast<std::vector<int32_t>>();
      m[kv.first.cast<std::string>()] = ml;
    }
    return GroupMember::assign_load_aware(members, m, n);
  }, py::arg("members"), py::arg("loads"), py::arg("partitions"));
  k.def("member_load_roundtrip", [](double cap, std::vector<int32_t> owned) {
    MemberLoad ml;
    ml.capacity = cap;
    ml.owned = owned;
    const MemberLoad r = decode_member_load(encode_member_load(ml));
    return py::make_tuple(r.capacity, r.owned);
  });
  k.def("crc32c_device_tables", [] {
    std::vector<uint32_t> t(kCrcDeviceTableWords);
    crc32c_device_tables(t.data());
    return t;
  });
  k.def("crc32c_shift", &crc32c_shift, py::arg("raw"), py::arg("nbytes"));
  k.def("crc32c_combine", &crc32c_combine, py::arg("crc_a"), py::arg("crc_b"), py::arg("len_b"));
  k.def("murmur2", [](py::bytes b) {
    const std::string_view s = view(b);
    return murmur2(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  py::class_<BatchSet, std::shared_ptr<BatchSet>>(k, "BatchSet")
      .def_static("from_bytes", [](py::list blobs) {
        auto bs = std::make_shared<BatchSet>();
        for (auto o : blobs) {
          const std::string_view v = view(o.cast<py::bytes>());
          const BatchInfo bi = peek_batch(reinterpret_cast<const uint8_t*>(v.data()), v.size(),
                                          false);
          bs->batches.push_back(std::make_shared<const std::string>(v));
          bs->records.push_back(bi.records);
          bs->bytes += v.size();
        }
        return bs;
      })
      .def("__len__", [](const BatchSet& b) { return b.batches.size(); })
      .def_property_readonly("bytes", [](const BatchSet& b) { return b.bytes; })
      .def_property_readonly("records", [](const BatchSet& b) {
        int64_t n = 0;
        for (int32_t r : b.records) n += r;
        return n;
      })
      .def_property_readonly("images_per_record",
                             [](const BatchSet& b) { return b.images_per_record; })
      .def("records_in", [](const BatchSet& b, size_t i) { return b.records.at(i); })
      .def("batch", [](const BatchSet& b, size_t i) { return py::bytes(*b.batches.at(i)); });
  k.def("synthetic_batches", [](py::array_t<float, py::array::c_style | py::array::forcecast> x,
                                int ipr, int rpb, int threads, const std::string& key_prefix) {
    if (x.ndim() != 4) throw std::invalid_argument("images must be [N, H, W, C]");
    const float* p = x.data();
    const int64_t n = x.shape(0);
    const int H = (int)x.shape(1), W = (int)x.shape(2), C = (int)x.shape(3);
    py::gil_scoped_release nogil;
    return synthetic_batches(p, n, H, W, C, ipr, rpb, threads, key_prefix);
  }, py::arg("images"), py::arg("images_per_record") = 1, py::arg("records_per_batch") = 64,
     py::arg("threads") = 8, py::arg("key_prefix") = "");
  k.def("encode_batch", &py_encode_batch, py::arg("records"), py::arg("base_offset") = 0,
        py::arg("base_timestamp") = 0);
  k.def("decode_records", [](py::bytes b, int64_t min_offset, bool check_crc) {
    const std::string_view s = view(b);
    std::vector<RecordRef> recs;
    std::string hold;
    const uint8_t* base = decode_any(s, min_offset, check_crc, hold, recs);
    return records_to_py(base, recs);
  }, py::arg("data"), py::arg("min_offset") = 0, py::arg("check_crc") = true,
     "records of a records blob (any message format / compression; undecodable batches come "
     "back as {'poison': True, 'value': None} records)");
  // ---- compression codecs and message-format conversion (kafka/compress.h)
  k.def("codec_available", [](const std::string& c) { return codec_available(codec_from_name(c)); });
  k.def("compress", [](const std::string& c, py::bytes data) {
    const std::string_view s = view(data);
    std::string out;
    {
      py::gil_scoped_release nogil;
      out = compress(codec_from_name(c), reinterpret_cast<const uint8_t*>(s.data()), s.size());
    }
    return py::bytes(out);
  }, py::arg("codec"), py::arg("data"));
  k.def("decompress", [](const std::string& c, py::bytes data, size_t limit) {
    const std::string_view s = view(data);
    std::string out, err;
    if (!decompress(codec_from_name(c), reinterpret_cast<const uint8_t*>(s.data()), s.size(), out,
                    limit, &err))
      throw std::runtime_error(err.empty() ? "corrupt " + c + " data" : err);
    return py::bytes(out);
  }, py::arg("codec"), py::arg("data"), py::arg("limit") = (size_t)1 << 30);
  k.def("snappy_compress_raw", [](py::bytes data) {
    const std::string_view s = view(data);
    return py::bytes(snappy_compress_raw(reinterpret_cast<const uint8_t*>(s.data()), s.size()));
  });
  k.def("xxh32", [](py::bytes data, uint32_t seed) {
    const std::string_view s = view(data);
    return xxh32(reinterpret_cast<const uint8_t*>(s.data()), s.size(), seed);
  }, py::arg("data"), py::arg("seed") = 0);
  k.def("compress_batch", [](py::bytes batch, const std::string& c) {
    return py::bytes(compress_batch(std::string(view(batch)), codec_from_name(c)));
  }, py::arg("batch"), py::arg("codec"));
  k.def("encode_message_set", [](int magic, py::list values, int64_t base_offset,
                                 const std::string& c, py::object keys, int64_t timestamp) {
    std::vector<LegacyRecord> recs(values.size());
    for (size_t i = 0; i < values.size(); ++i) {
      if (values[i].is_none()) recs[i].value_null = true;
      else recs[i].value = std::string(view(values[i].cast<py::bytes>()));
      if (!keys.is_none() && !keys.cast<py::list>()[i].is_none()) {
        recs[i].key = std::string(view(keys.cast<py::list>()[i].cast<py::bytes>()));
        recs[i].key_null = false;
      }
      recs[i].timestamp = timestamp;
    }
    return py::bytes(encode_message_set(magic, recs, base_offset, codec_from_name(c)));
  }, py::arg("magic"), py::arg("values"), py::arg("base_offset") = 0, py::arg("codec") = "none",
     py::arg("keys") = py::none(), py::arg("timestamp") = -1);
  k.def("normalize_records", [](py::bytes data, int64_t min_offset, bool check_crc, size_t limit) {
    const std::string_view s = view(data);
    NormalizeStats st;
    const std::string out = normalize_records(reinterpret_cast<const uint8_t*>(s.data()),
                                              s.size(), min_offset, check_crc, limit, st);
    py::dict d;
    d["converted_batches"] = st.converted_batches;
    d["poison_batches"] = st.poison_batches;
    d["poison_records"] = st.poison_records;
    d["poison_unknown_span"] = st.poison_unknown_span;
    d["last_error"] = st.last_error;
    return py::make_tuple(py::bytes(out), d);
  }, py::arg("data"), py::arg("min_offset") = 0, py::arg("check_crc") = true,
     py::arg("limit") = (size_t)1 << 30);
  k.def("encode", &py_encode);
  k.def("decode", &py_decode);
  k.def("api_version", [](int key) { return kVersion((ApiKey)key); });
  k.def("error_name", &error_name);

  py::class_<Broker, std::shared_ptr<Broker>>(k, "Broker")
      .def(py::init([](const std::string& host, int port, int node_id, int default_partitions,
                       bool auto_create, int64_t max_message_bytes, int64_t retention_bytes,
                       bool check_crcs, bool zero_copy, bool log_append_time) {
             BrokerConfig c;
             c.zero_copy = zero_copy;
             c.log_append_time = log_append_time;
             c.host = host;
             c.port = port;
             c.node_id = node_id;
             c.default_partitions = default_partitions;
             c.auto_create_topics = auto_create;
             c.max_message_bytes = max_message_bytes;
             c.retention_bytes = retention_bytes;
             c.check_crcs = check_crcs;
             return std::make_shared<Broker>(c);
           }),
           py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("node_id") = 0,
           py::arg("default_partitions") = 1, py::arg("auto_create_topics") = true,
           py::arg("max_message_bytes") = 64ll << 20, py::arg("retention_bytes") = 4ll << 30,
           py::arg("check_crcs") = true, py::arg("zero_copy") = false,
           py::arg("log_append_time") = false)
      .def("start", &Broker::start)
      .def("stop", [](Broker& b) {
        py::gil_scoped_release nogil;
        b.stop();
      })
      .def_property_readonly("port", &Broker::port)
      .def_property_readonly("node_id", &Broker::node_id)
      .def_property_readonly("host", [](Broker& b) { return b.config().host; })
      .def("set_cluster", [](Broker& b, py::list nodes) {
        std::vector<BrokerNode> v;
        for (auto n : nodes) {
          auto t = n.cast<py::tuple>();
          v.push_back({t[0].cast<int32_t>(), t[1].cast<std::string>(), t[2].cast<int32_t>()});
        }
        b.set_cluster(v);
      })
      .def("leads", &Broker::leads)
      .def("create_topic", &Broker::create_topic)
      .def("topics", &Broker::topics)
      .def("partitions", &Broker::partitions)
      .def("append", [](Broker& b, const std::string& topic, int partition, py::list values,
                        py::object keys) {
        std::vector<std::string> vals(values.size()), ks(values.size());
        std::vector<RecordIn> ins(values.size());
        for (size_t i = 0; i < values.size(); ++i) {
          if (values[i].is_none()) {
            ins[i].value_null = true;
          } else {
            vals[i] = std::string(view(values[i].cast<py::bytes>()));
            ins[i].value = vals[i];
          }
          if (!keys.is_none() && !keys.cast<py::list>()[i].is_none()) {
            ks[i] = std::string(view(keys.cast<py::list>()[i].cast<py::bytes>()));
            ins[i].key = ks[i];
            ins[i].key_null = false;
          }
        }
        py::gil_scoped_release nogil;
        return b.append(topic, partition, ins);
      }, py::arg("topic"), py::arg("partition"), py::arg("values"), py::arg("keys") = py::none())
      .def("append_legacy", [](Broker& b, const std::string& topic, int partition, int magic,
                               py::list values, const std::string& codec, py::object keys,
                               int64_t timestamp) {
        std::vector<LegacyRecord> recs(values.size());
        for (size_t i = 0; i < values.size(); ++i) {
          if (values[i].is_none()) recs[i].value_null = true;
          else recs[i].value = std::string(view(values[i].cast<py::bytes>()));
          if (!keys.is_none() && !keys.cast<py::list>()[i].is_none()) {
            recs[i].key = std::string(view(keys.cast<py::list>()[i].cast<py::bytes>()));
            recs[i].key_null = false;
          }
          recs[i].timestamp = timestamp;
        }
        py::gil_scoped_release nogil;
        return b.append_legacy(topic, partition, magic, recs, codec_from_name(codec));
      }, py::arg("topic"), py::arg("partition"), py::arg("magic"), py::arg("values"),
         py::arg("codec") = "none", py::arg("keys") = py::none(), py::arg("timestamp") = -1,
         "append one old-format message set (magic 0/1, optionally compressed)")
      .def("append_batch_repeated", [](Broker& b, const std::string& topic, int partition,
                                       py::bytes batch, int64_t times) {
        // append one pre-encoded batch `times` times, sharing its bytes (bench preloading)
        auto s = std::make_shared<const std::string>(view(batch));
        py::gil_scoped_release nogil;
        int64_t first = -1;
        for (int64_t i = 0; i < times; ++i) {
          const int64_t o = b.append_shared(topic, partition, s);
          if (i == 0) first = o;
        }
        return first;
      })
      .def("append_cycled", [](Broker& b, const std::string& topic, int partition,
                               const BatchSet& set, int64_t n_batches, int64_t start) {
        // append n_batches of `set` by reference, cycling from index `start`; returns
        // (first offset, records appended)
        if (set.batches.empty()) throw std::invalid_argument("empty BatchSet");
        int64_t first = -1, recs = 0;
        {
          py::gil_scoped_release nogil;
          const int64_t m = (int64_t)set.batches.size();
          for (int64_t i = 0; i < n_batches; ++i) {
            const size_t k = (size_t)(((start + i) % m + m) % m);
            const int64_t o = b.append_shared(topic, partition, set.batches[k]);
            if (i == 0) first = o;
            recs += set.records[k];
          }
        }
        return py::make_tuple(first, recs);
      }, py::arg("topic"), py::arg("partition"), py::arg("batches"), py::arg("n_batches"),
         py::arg("start") = 0)
      .def("fail_produce", &Broker::fail_produce, py::arg("topic"), py::arg("n"),
           py::arg("error") = (int16_t)NOT_LEADER_FOR_PARTITION)
      .def("describe_group", [](Broker& b, const std::string& g) {
        const GroupInfo gi = b.describe_group(g);
        py::dict d;
        d["state"] = gi.state;
        d["generation"] = gi.generation;
        d["leader"] = gi.leader;
        d["protocol"] = gi.protocol;
        d["members"] = gi.members;
        return d;
      })
      .def("log_start", &Broker::log_start)
      .def("log_end", &Broker::log_end)
      .def("committed", &Broker::committed)
      .def("read", [](Broker& b, const std::string& topic, int partition, int64_t offset,
                      int64_t max_bytes) {
        const std::string raw = b.read_raw(topic, partition, offset, max_bytes);
        std::vector<RecordRef> recs;
        std::string hold;
        const uint8_t* base = decode_any(raw, offset, true, hold, recs);
        for (auto& r : recs) r.partition = partition;
        return records_to_py(base, recs);
      }, py::arg("topic"), py::arg("partition"), py::arg("offset") = 0,
         py::arg("max_bytes") = 64ll << 20)
      .def("stats", [](Broker& b) {
        const BrokerStats s = b.stats();
        py::dict d;
        d["requests"] = s.requests;
        d["produce_requests"] = s.produce_requests;
        d["fetch_requests"] = s.fetch_requests;
        d["bytes_in"] = s.bytes_in;
        d["bytes_out"] = s.bytes_out;
        d["bytes_spliced"] = s.bytes_spliced;
        d["records_in"] = s.records_in;
        d["connections"] = s.connections;
        return d;
      })
      .def("take_probes", [](Broker& b) {
        const BrokerProbes p = b.take_probes();
        py::dict d;
        d["wake_max_us"] = p.wake_max_us;
        d["wake_slow"] = p.wake_slow;
        d["flush_max_us"] = p.flush_max_us;
        d["flush_slow"] = p.flush_slow;
        d["lock_max_us"] = p.lock_max_us;
        d["lock_slow"] = p.lock_slow;
        return d;
      }, "latency-tail probes since the last call (max us, count > 1 ms): parked-fetch "
         "wake-up, response write, append lock wait");

  py::class_<RateFeeder, std::shared_ptr<RateFeeder>>(k, "RateFeeder")
      .def(py::init<std::shared_ptr<Broker>, std::string, std::vector<int>,
                    std::shared_ptr<BatchSet>>(),
           py::arg("broker"), py::arg("topic"), py::arg("partitions"), py::arg("batches"))
      .def("start", &RateFeeder::start, py::arg("records_per_s"), py::arg("start_batch") = 0)
      .def("stop", [](RateFeeder& f) {
        py::gil_scoped_release nogil;
        f.stop();
      })
      .def("take_log", &RateFeeder::take_log)
      .def_property_readonly("next_batch", &RateFeeder::next_batch)
      .def_property_readonly("appended_records", &RateFeeder::appended_records);

  py::class_<Producer, std::shared_ptr<Producer>>(k, "Producer")
      .def(py::init([](const std::string& bootstrap, int acks, int linger_ms, int batch_size,
                       const std::string& client_id, int request_timeout_ms, int max_in_flight,
                       int max_request_size, const std::string& compression, int retries,
                       int retry_backoff_ms, int delivery_timeout_ms, double fail_p) {
             ProducerConfig c;
             c.retries = retries;
             c.retry_backoff_ms = retry_backoff_ms;
             c.delivery_timeout_ms = delivery_timeout_ms;
             c.fail_p = fail_p;
             c.compression = codec_from_name(compression);
             c.max_request_size = max_request_size;
             c.bootstrap = bootstrap;
             c.acks = acks;
             c.linger_ms = linger_ms;
             c.batch_size = batch_size;
             c.client_id = client_id;
             c.request_timeout_ms = request_timeout_ms;
             c.max_in_flight = max_in_flight;
             py::gil_scoped_release nogil;
             return std::make_shared<Producer>(c);
           }),
           py::arg("bootstrap"), py::arg("acks") = 1, py::arg("linger_ms") = 0,
           py::arg("batch_size") = 16384, py::arg("client_id") = "gale-producer",
           py::arg("request_timeout_ms") = 30000, py::arg("max_in_flight") = 5,
           py::arg("max_request_size") = 64 << 20, py::arg("compression") = "none",
           py::arg("retries") = 0, py::arg("retry_backoff_ms") = 100,
           py::arg("delivery_timeout_ms") = 120000, py::arg("fail_p") = 0.0)
      .def("send", [](Producer& p, const std::string& topic, py::object value, py::object key,
                      int partition, py::object headers, int64_t timestamp, py::object callback) {
        std::string v;
        bool vnull = value.is_none();
        if (!vnull) v = std::string(view(value.cast<py::bytes>()));
        std::string ks;
        const bool has_key = !key.is_none();
        if (has_key) ks = std::string(view(key.cast<py::bytes>()));
        SendCallback cb;
        if (!callback.is_none()) {
          auto held = hold(callback);
          cb = [held](const SendResult& r) {
            py::gil_scoped_acquire g;
            try {
              (*held)(r.error, r.partition, r.offset);
            } catch (py::error_already_set& e) {
              e.discard_as_unraisable(__func__);
            }
          };
        }
        auto hs = headers_from_py(headers);
        py::gil_scoped_release nogil;
        p.send(topic, partition, has_key ? &ks : nullptr, std::move(v), vnull, std::move(hs),
               timestamp, std::move(cb));
      }, py::arg("topic"), py::arg("value"), py::arg("key") = py::none(),
         py::arg("partition") = -1, py::arg("headers") = py::none(), py::arg("timestamp") = -1,
         py::arg("callback") = py::none())
      .def("flush", [](Producer& p) {
        py::gil_scoped_release nogil;
        p.flush();
      })
      .def("close", [](Producer& p) {
        py::gil_scoped_release nogil;
        p.close();
      })
      .def("partitions_for", [](Producer& p, const std::string& t) {
        py::gil_scoped_release nogil;
        return p.partitions_for(t);
      })
      .def("stats", [](Producer& p) {
        const ProducerStats s = p.stats();
        py::dict d;
        d["records_sent"] = s.records_sent;
        d["records_acked"] = s.records_acked;
        d["records_failed"] = s.records_failed;
        d["requests"] = s.requests;
        d["bytes"] = s.bytes;
        d["records_retried"] = s.records_retried;
        d["requests_failed"] = s.requests_failed;
        return d;
      });

  py::class_<Consumer, std::shared_ptr<Consumer>>(k, "Consumer")
      .def(py::init([](const std::string& bootstrap, const std::string& group_id, int max_wait_ms,
                       int fetch_max_bytes, int partition_max_bytes, bool check_crcs,
                       const std::string& auto_offset_reset, const std::string& client_id,
                       int recv_lowat, bool bounce_pack, int bounce_window_kb) {
             ConsumerConfig c;
             c.recv_lowat = recv_lowat;
             c.bootstrap = bootstrap;
             c.group_id = group_id;
             c.max_wait_ms = max_wait_ms;
             c.fetch_max_bytes = fetch_max_bytes;
             c.partition_max_bytes = partition_max_bytes;
             c.check_crcs = check_crcs;
             c.auto_offset_reset = auto_offset_reset;
             c.client_id = client_id;
             if (!bounce_pack) return std::make_shared<Consumer>(c);
             // the bounce receive (runtime/pack_tap.h) over heap "chunks" sized like the
             // engine's pinned pool, for host-side tests of the sparse body + packed text
             c.check_crcs = false;  // (the host copy is sparse: the GPU checks the CRCs)
             const size_t chunk =
                 gale::codec::pack_layout_bytes((size_t)c.fetch_max_bytes + (1 << 20)) + 4096;
             auto cons = std::make_shared<Consumer>(
                 c, [chunk](size_t n) { return heap_alloc(std::max(n, chunk)); });
             cons->set_recv_tap(std::make_shared<gale::BouncePackTap>(
                 chunk, [](const uint8_t*) { return true; }, 1,
                 (size_t)std::max(1, bounce_window_kb) << 10));
             return cons;
           }),
           py::arg("bootstrap"), py::arg("group_id") = "", py::arg("max_wait_ms") = 100,
           py::arg("fetch_max_bytes") = 64 << 20, py::arg("partition_max_bytes") = 16 << 20,
           py::arg("check_crcs") = true, py::arg("auto_offset_reset") = "latest",
           py::arg("client_id") = "gale-consumer", py::arg("recv_lowat") = 0,
           py::arg("bounce_pack") = false, py::arg("bounce_window_kb") = 256)
      .def("assign", [](Consumer& c, const std::string& topic, std::vector<int> parts) {
        py::gil_scoped_release nogil;
        c.assign(topic, parts);
      }, py::arg("topic"), py::arg("partitions") = std::vector<int>{})
      .def("assignment", &Consumer::assignment)
      .def("seek_to", [](Consumer& c, const std::string& w) {
        py::gil_scoped_release nogil;
        c.seek_to(w);
      })
      .def("seek", &Consumer::seek)
      .def("position", &Consumer::position)
      .def("format_stats", [](Consumer& c) {
        py::dict d;
        d["converted_batches"] = c.converted_batches();
        d["poison_batches"] = c.poison_batches();
        d["poison_records"] = c.poison_records();
        d["poison_unknown_span"] = c.poison_unknown_span();
        return d;
      }, "record-format conversion counters: compressed / legacy batches rewritten, "
         "undecodable batches skipped as poison records")
      .def("poll", [](Consumer& c) {
        std::vector<Fetched> fs;
        {
          py::gil_scoped_release nogil;
          fs = c.poll();
        }
        py::list out;
        for (auto& f : fs) {
          f.restore();  // (a sparse body: the values are read here)
          for (auto item : records_to_py(f.buf.get(), f.records)) out.append(item);
        }
        return out;
      })
      .def("poll_bodies", [](Consumer& c) {
        // per fetch response: the host copy as received (sparse under the bounce receive), the
        // text expanded from its packed stream, and the records decoded from the host copy
        std::vector<Fetched> fs;
        {
          py::gil_scoped_release nogil;
          fs = c.poll();
        }
        py::list out;
        for (auto& f : fs) {
          py::dict d;
          d["size"] = f.size;
          d["packed_bytes"] = f.tap_result;
          d["sparse"] = f.sparse;
          d["host"] = py::bytes(reinterpret_cast<const char*>(f.buf.get()), f.size);
          py::list recs;
          for (const RecordRef& r : f.records) {
            py::dict x;
            x["partition"] = r.partition;
            x["offset"] = r.offset;
            x["timestamp"] = r.timestamp;
            x["key"] = opt_bytes(f.buf.get(), r.key_off, r.key_len);
            x["value_off"] = r.value_off;
            x["value_len"] = r.value_len;
            py::list hs;
            for (const Header& h : decode_headers(f.buf.get(), r))
              hs.append(py::make_tuple(h.key, h.value_null ? py::object(py::none())
                                                           : py::object(py::bytes(h.value))));
            x["headers"] = hs;
            if (r.value_len >= 0) {
              const gale::codec::Scan sc = gale::codec::scan_envelope(
                  f.buf.get() + r.value_off, (size_t)r.value_len, gale::kafka::FramingWalker::kHead,
                  gale::kafka::FramingWalker::kTail);
              x["scan"] = py::make_tuple(sc.status, sc.arr_off, sc.arr_len);
            }
            recs.append(x);
          }
          d["records"] = recs;
          if (f.tap_result >= 0) {
            std::string full(f.size, '\0');
            gale::codec::text_unpack_host(
                f.buf.get() + gale::codec::pack_offset(f.size),
                reinterpret_cast<const uint32_t*>(f.buf.get() + gale::codec::tab_offset(f.size)),
                f.size, reinterpret_cast<uint8_t*>(&full[0]));
            d["unpacked"] = py::bytes(full);
          }
          out.append(d);
        }
        return out;
      })
      .def("poll_count", [](Consumer& c) {
        // (records, value bytes) of one poll without materialising Python objects: consumer
        // throughput diagnostics
        py::gil_scoped_release nogil;
        int64_t n = 0, bytes = 0;
        for (auto& f : c.poll())
          for (const RecordRef& r : f.records) {
            ++n;
            bytes += r.value_len > 0 ? r.value_len : 0;
          }
        return std::make_pair(n, bytes);
      })
      .def("commit", [](Consumer& c, std::map<int, int64_t> offs) {
        py::gil_scoped_release nogil;
        c.commit(offs);
      })
      .def("committed", [](Consumer& c, int p) {
        py::gil_scoped_release nogil;
        return c.committed(p);
      })
      .def("high_watermarks", &Consumer::high_watermarks)
      .def("set_generation", &Consumer::set_generation, py::arg("generation"),
           py::arg("member_id"));

  py::class_<GroupMember, std::shared_ptr<GroupMember>>(k, "GroupMember")
      .def(py::init([](const std::string& bootstrap, const std::string& group_id,
                       const std::string& topic, int session_timeout_ms,
                       int rebalance_timeout_ms, const std::string& assignor,
                       const std::string& client_id) {
             GroupConfig c;
             c.bootstrap = bootstrap;
             c.group_id = group_id;
             c.topic = topic;
             c.session_timeout_ms = session_timeout_ms;
             c.rebalance_timeout_ms = rebalance_timeout_ms;
             c.assignor = assignor;
             c.client_id = client_id;
             py::gil_scoped_release nogil;
             return std::make_shared<GroupMember>(c);
           }),
           py::arg("bootstrap"), py::arg("group_id"), py::arg("topic"),
           py::arg("session_timeout_ms") = 6000, py::arg("rebalance_timeout_ms") = 8000,
           py::arg("assignor") = "range", py::arg("client_id") = "gale-group")
      .def("join", [](GroupMember& g) {
        py::gil_scoped_release nogil;
        return g.join();
      })
      .def("heartbeat", [](GroupMember& g) {
        py::gil_scoped_release nogil;
        return g.heartbeat();
      })
      .def("leave", [](GroupMember& g) {
        py::gil_scoped_release nogil;
        g.leave();
      })
      .def_property_readonly("member_id", &GroupMember::member_id)
      .def_property_readonly("generation", &GroupMember::generation)
      .def_property_readonly("is_leader", &GroupMember::is_leader);

  py::register_exception<KafkaError>(k, "KafkaError");
  py::register_exception<ProtocolError>(k, "ProtocolError");

  bind_engine(m);
}

}  // namespace gale
