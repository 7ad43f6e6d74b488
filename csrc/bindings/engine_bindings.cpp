// Python bindings of the serving engine (gale._C.Engine).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../runtime/engine.h"
#include "../runtime/gpu_ingest.h"
#include "gale/executor.h"

namespace py = pybind11;

namespace gale {

namespace {

template <typename T>
void opt(const py::dict& d, const char* k, T& dst) {
  if (d.contains(k) && !d[k].is_none()) dst = d[k].cast<T>();
}

EngineConfig config_from_dict(const py::dict& d) {
  EngineConfig c;
  opt(d, "bootstrap", c.bootstrap);
  opt(d, "input_topic", c.input_topic);
  opt(d, "output_topic", c.output_topic);
  opt(d, "output_partition", c.output_partition);
  opt(d, "producer_buffer_bytes", c.producer_buffer_bytes);
  opt(d, "producer_request_bytes", c.producer_request_bytes);
  opt(d, "group_id", c.group_id);
  opt(d, "client_id", c.client_id);
  opt(d, "partitions", c.partitions);
  opt(d, "source_parallelism", c.source_parallelism);
  opt(d, "start_offset", c.start_offset);
  opt(d, "auto_offset_reset", c.auto_offset_reset);
  opt(d, "ingest_parse", c.ingest_parse);
  opt(d, "fetch_max_wait_ms", c.fetch_max_wait_ms);
  opt(d, "fetch_min_bytes", c.fetch_min_bytes);
  opt(d, "fetch_max_bytes", c.fetch_max_bytes);
  opt(d, "partition_max_bytes", c.partition_max_bytes);
  opt(d, "check_crcs", c.check_crcs);
  opt(d, "decode_threads", c.decode_threads);
  opt(d, "pinned_fetch_bytes", c.pinned_fetch_bytes);
  opt(d, "text_pack", c.text_pack);
  opt(d, "text_pack_bounce", c.text_pack_bounce);
  opt(d, "text_pack_window_kb", c.text_pack_window_kb);
  opt(d, "float_format", c.float_format);
  opt(d, "recv_lowat", c.recv_lowat);
  opt(d, "commit_interval_ms", c.commit_interval_ms);
  opt(d, "group_membership", c.group_membership);
  opt(d, "session_timeout_ms", c.session_timeout_ms);
  opt(d, "rebalance_timeout_ms", c.rebalance_timeout_ms);
  opt(d, "heartbeat_interval_ms", c.heartbeat_interval_ms);
  opt(d, "assignor", c.assignor);
  opt(d, "lag_rebalance_records", c.lag_rebalance_records);
  opt(d, "rebalance_cooldown_ms", c.rebalance_cooldown_ms);
  opt(d, "device_cpus", c.device_cpus);
  opt(d, "sink_parallelism", c.sink_parallelism);
  opt(d, "acks", c.acks);
  opt(d, "sink_mode", c.sink_mode);
  opt(d, "delivery", c.delivery);
  opt(d, "producer_retries", c.producer_retries);
  opt(d, "retry_backoff_ms", c.retry_backoff_ms);
  opt(d, "delivery_timeout_ms", c.delivery_timeout_ms);
  opt(d, "linger_ms", c.linger_ms);
  opt(d, "compression", c.compression);
  opt(d, "batch_size", c.batch_size);
  opt(d, "value_format", c.value_format);
  opt(d, "type_id_header", c.type_id_header);
  opt(d, "on_error", c.on_error);
  opt(d, "output_key", c.output_key);
  opt(d, "H", c.H);
  opt(d, "W", c.W);
  opt(d, "C", c.C);
  opt(d, "classes", c.classes);
  opt(d, "max_batch", c.max_batch);
  opt(d, "max_wait_us", c.max_wait_us);
  opt(d, "slo_p99_ms", c.slo_p99_ms);
  opt(d, "queue_depth", c.queue_depth);
  opt(d, "watchdog_ms", c.watchdog_ms);
  opt(d, "max_restarts", c.max_restarts);
  opt(d, "restart_backoff_ms", c.restart_backoff_ms);
  opt(d, "fault", c.fault);
  opt(d, "trace", c.trace);
  opt(d, "max_records", c.max_records);
  opt(d, "seed", c.seed);
  return c;
}

}  // namespace

void bind_engine(py::module_& m) {
  py::class_<Engine, std::shared_ptr<Engine>>(m, "Engine")
      .def(py::init([](py::dict cfg) { return std::make_shared<Engine>(config_from_dict(cfg)); }))
      .def("add_stub_replica",
           [](Engine& e, int max_images, int delay_us, bool compute, int locality) {
             const EngineConfig& c = e.config();
             e.add_replica(std::make_shared<StubReplica>(c.H, c.W, c.C, c.classes, max_images,
                                                         delay_us, compute, locality));
           },
           py::arg("max_images") = 256, py::arg("delay_us") = 0, py::arg("compute") = true,
           py::arg("locality") = -1)
      .def("add_gpu_replica",
           [](Engine& e, std::shared_ptr<Executor> exec, bool use_graph, int wait_poll_us,
              bool gpu_encode, int locality, bool step_graph, bool high_priority,
              bool step_direct) {
             const EngineConfig& c = e.config();
             e.add_replica(std::make_shared<GpuReplica>(std::move(exec), c.H, c.W, c.C,
                                                        c.classes, use_graph, wait_poll_us,
                                                        gpu_encode, locality, step_graph,
                                                        high_priority, step_direct));
           },
           py::arg("executor"), py::arg("use_graph") = true, py::arg("wait_poll_us") = 0,
           py::arg("gpu_encode") = false, py::arg("locality") = -1, py::arg("step_graph") = true,
           py::arg("high_priority") = false, py::arg("step_direct") = false)
      .def("enable_gpu_ingest",
           [](Engine& e, int device, int lanes, int poll_us) {
             e.set_ingest(std::make_shared<GpuIngest>(device, lanes, poll_us));
           },
           py::arg("device"), py::arg("lanes") = 2, py::arg("poll_us") = 20)
      .def("start",
           [](Engine& e) {
             py::gil_scoped_release nogil;
             e.start();
           })
      .def("stop",
           [](Engine& e) {
             py::gil_scoped_release nogil;
             e.stop();
           })
      .def("wait",
           [](Engine& e, int64_t timeout_ms) {
             py::gil_scoped_release nogil;
             return e.wait(timeout_ms);
           },
           py::arg("timeout_ms") = -1)
      .def("last_wait", &Engine::last_wait)
      .def("wait_completed",
           [](Engine& e, int64_t n, int64_t timeout_ms) {
             py::gil_scoped_release nogil;
             return e.wait_completed(n, timeout_ms);
           },
           py::arg("n"), py::arg("timeout_ms") = -1)
      .def_property_readonly("running", &Engine::running)
      .def_property_readonly("completed", &Engine::completed)
      .def("stats", &Engine::stats)
      .def("reset_stats", &Engine::reset_stats)
      .def("set_ack_log", &Engine::set_ack_log, py::arg("on"),
           py::arg("capacity") = (size_t)(8u << 20))
      .def("take_ack_log", [](Engine& e) {
        const std::vector<AckSample> v = e.take_ack_log();
        py::array_t<int32_t> p(v.size());
        py::array_t<int64_t> o(v.size()), t(v.size()), tf(v.size()), tt(v.size()), td(v.size()),
            tr(v.size());
        auto pp = p.mutable_unchecked<1>();
        auto po = o.mutable_unchecked<1>();
        auto pt = t.mutable_unchecked<1>();
        auto pf = tf.mutable_unchecked<1>();
        auto pk = tt.mutable_unchecked<1>();
        auto pd = td.mutable_unchecked<1>();
        auto pr = tr.mutable_unchecked<1>();
        for (size_t i = 0; i < v.size(); ++i) {
          const auto k = (py::ssize_t)i;
          pp(k) = v[i].partition;
          po(k) = v[i].offset;
          pt(k) = v[i].t_ns;
          pf(k) = v[i].t_fetch_ns;
          pk(k) = v[i].t_take_ns;
          pd(k) = v[i].t_done_ns;
          pr(k) = v[i].t_ready_ns;
        }
        // (partition, offset, t_ack, t_fetch, t_take, t_done, t_ready)
        return py::make_tuple(p, o, t, tf, tt, td, tr);
      })
      .def("replica_stats", [](Engine& e) {
        py::list out;
        for (const ReplicaStats& s : e.replica_stats()) {
          py::dict d;
          d["name"] = s.name;
          d["device"] = s.device;
          d["alive"] = s.alive;
          d["batches"] = s.batches;
          d["images"] = s.images;
          d["records"] = s.records;
          d["restarts"] = s.restarts;
          d["slot"] = s.slot;
          d["resident_records"] = s.resident_records;
          d["host_records"] = s.host_records;
          out.append(d);
        }
        return out;
      })
      .def("partition_offsets", [](Engine& e) {
        py::list out;
        for (const PartitionOffsets& o : e.partition_offsets()) {
          py::dict d;
          d["partition"] = o.partition;
          d["high_watermark"] = o.high_watermark;
          d["fetched"] = o.fetched;
          d["committed"] = o.committed;
          d["lag"] = o.lag;
          d["fetch_lag"] = o.fetch_lag;
          out.append(d);
        }
        return out;
      });
}

}  // namespace gale
