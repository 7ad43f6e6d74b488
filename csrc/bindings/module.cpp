// Python bindings of the gale native library (module gale._C).
//
// Kernels take raw device pointers (torch tensors' data_ptr()) and a hipStream_t handle
// (torch.cuda.current_stream().cuda_stream), so they interoperate with PyTorch-ROCm tensors
// without linking libtorch. Long-running calls release the GIL.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../comm/rccl.h"
#include "gale/executor.h"
#include "gale/kernels.h"

namespace py = pybind11;

namespace gale {
void bind_host(py::module_& m);  // codec / kafka / engine bindings (host_bindings.cpp)
}

namespace {

using gale::ConvDesc;

template <typename T>
T get_or(const py::dict& d, const char* k, T dflt) {
  return d.contains(k) ? d[k].cast<T>() : dflt;
}

ConvDesc desc_from_dict(const py::dict& d) {
  ConvDesc c{};
  c.H = d["H"].cast<int>();
  c.W = d["W"].cast<int>();
  c.Cin = d["Cin"].cast<int>();
  c.Ho = d["Ho"].cast<int>();
  c.Wo = d["Wo"].cast<int>();
  c.Cout = d["Cout"].cast<int>();
  c.KH = d["KH"].cast<int>();
  c.KW = d["KW"].cast<int>();
  c.stride = d["stride"].cast<int>();
  c.pad = d["pad"].cast<int>();
  c.K = d["K"].cast<int>();
  c.Kpad = d["Kpad"].cast<int>();
  c.Npad = d["Npad"].cast<int>();
  c.relu = get_or<int>(d, "relu", 0);
  c.has_res = get_or<int>(d, "has_res", 0);
  c.res_H = get_or<int>(d, "res_H", c.Ho);
  c.res_W = get_or<int>(d, "res_W", c.Wo);
  c.res_C = get_or<int>(d, "res_C", c.Cout);
  c.res_stride = get_or<int>(d, "res_stride", 1);
  c.in_f32 = get_or<int>(d, "in_f32", 0);
  c.out_f32 = get_or<int>(d, "out_f32", 0);
  c.fp8 = get_or<int>(d, "fp8", 0);
  c.in_scale = get_or<float>(d, "in_scale", 1.0f);
  c.out_scale = get_or<float>(d, "out_scale", 1.0f);
  c.res_scale = get_or<float>(d, "res_scale", 1.0f);
  c.stem = get_or<int>(d, "stem", 0);
  c.f32 = get_or<int>(d, "f32", 0);
  return c;
}

inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
inline void* P(uintptr_t p) { return reinterpret_cast<void*>(p); }

void chk(hipError_t e, const char* what) { gale::check_hip(e, what); }

gale::PlanOp op_from_dict(const py::dict& d) {
  gale::PlanOp op;
  op.kind = d["kind"].cast<int>();
  if (d.contains("conv")) op.conv = desc_from_dict(d["conv"].cast<py::dict>());
  if (d.contains("p")) {
    auto v = d["p"].cast<std::vector<int>>();
    for (size_t i = 0; i < v.size() && i < 8; ++i) op.p[i] = v[i];
  }
  op.in = d["in"].cast<int>();
  op.out = d["out"].cast<int>();
  op.res = get_or<int>(d, "res", -1);
  op.w = P(get_or<uintptr_t>(d, "w", 0));
  op.bias = static_cast<const float*>(P(get_or<uintptr_t>(d, "bias", 0)));
  op.wscale = static_cast<const float*>(P(get_or<uintptr_t>(d, "wscale", 0)));
  if (d.contains("ptrs"))
    for (auto v : d["ptrs"].cast<std::vector<uintptr_t>>()) op.ptrs.push_back(P(v));
  if (d.contains("scales")) op.scales = d["scales"].cast<std::vector<float>>();
  op.fp8 = get_or<int>(d, "et", get_or<int>(d, "fp8", 0));  // pool/head activation ElemType
  op.scale = get_or<float>(d, "scale", 1.0f);
  if (d.contains("bpi")) {
    auto v = d["bpi"].cast<std::vector<long long>>();
    for (size_t i = 0; i < v.size() && i < 3; ++i) op.bpi[i] = v[i];
  }
  return op;
}

}  // namespace

namespace gale {
void install_crash_handler();  // runtime/crash.cpp
}

namespace {
// Host-mapped pinned memory (hipHostMallocMapped) for tests of the zero-copy kernel paths: the
// GPU ingest reads its plan and the packed text from, and writes its results to, such memory.
struct MappedBuffer {
  uint8_t* p = nullptr;
  size_t n = 0;
  explicit MappedBuffer(size_t bytes) : n(bytes) {
    gale::check_hip(hipHostMalloc(reinterpret_cast<void**>(&p), bytes ? bytes : 1,
                                  hipHostMallocMapped),
                    "hipHostMalloc(mapped)");
    void* dp = nullptr;
    gale::check_hip(hipHostGetDevicePointer(&dp, p, 0), "hipHostGetDevicePointer");
    if (dp != p) throw std::runtime_error("mapped buffer: device address differs from host");
  }
  ~MappedBuffer() {
    if (p) hipHostFree(p);
  }
};
}  // namespace

PYBIND11_MODULE(_C, m) {
  py::class_<MappedBuffer, std::shared_ptr<MappedBuffer>>(
      m, "MappedBuffer", "host-mapped pinned buffer (same address on the host and the GPU)")
      .def(py::init<size_t>())
      .def_property_readonly("ptr", [](const MappedBuffer& b) { return (uintptr_t)b.p; })
      .def_property_readonly("size", [](const MappedBuffer& b) { return b.n; })
      .def("numpy", [](std::shared_ptr<MappedBuffer> b) {
        // a uint8 view that keeps the buffer alive
        return py::array_t<uint8_t>({(py::ssize_t)b->n}, {1}, b->p,
                                    py::capsule(new std::shared_ptr<MappedBuffer>(b), [](void* c) {
                                      delete static_cast<std::shared_ptr<MappedBuffer>*>(c);
                                    }));
      });
  m.doc() = "gale native library: gfx950 kernels, plan executor, host runtime";
  gale::install_crash_handler();

  m.def("conv2d",
        [](py::dict desc, int batch, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t wscale,
           uintptr_t res, uintptr_t y, uintptr_t stream) {
          ConvDesc d = desc_from_dict(desc);
          chk(gale::conv2d(d, batch, P(x), P(w), static_cast<const float*>(P(bias)),
                           static_cast<const float*>(P(wscale)), P(res), P(y), S(stream)),
              "conv2d");
        },
        py::arg("desc"), py::arg("batch"), py::arg("x"), py::arg("w"), py::arg("bias"),
        py::arg("wscale"), py::arg("res"), py::arg("y"), py::arg("stream"));
  m.def("bottleneck56",
        [](int batch, uintptr_t x, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2,
           uintptr_t w3, uintptr_t b3, uintptr_t wd, uintptr_t bd, uintptr_t y, int cin,
           int down, uintptr_t stream) {
          gale::BottleneckParams bp;
          bp.w1 = P(w1); bp.w2 = P(w2); bp.w3 = P(w3); bp.wd = P(wd);
          bp.b1 = static_cast<const float*>(P(b1));
          bp.b2 = static_cast<const float*>(P(b2));
          bp.b3 = static_cast<const float*>(P(b3));
          bp.bd = static_cast<const float*>(P(bd));
          bp.cin = cin;
          bp.down = down;
          chk(gale::bottleneck56(bp, batch, P(x), P(y), S(stream)), "bottleneck56");
        },
        py::arg("batch"), py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("w2"),
        py::arg("b2"), py::arg("w3"), py::arg("b3"), py::arg("wd"), py::arg("bd"), py::arg("y"),
        py::arg("cin"), py::arg("down"), py::arg("stream"));
  m.def("bottleneck56_supported", &gale::bottleneck56_supported, py::arg("H"), py::arg("W"),
        py::arg("cin"), py::arg("cmid"), py::arg("cout"), py::arg("down"));
  m.def("stem_pool",
        [](int batch, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t stream) {
          chk(gale::stem_pool(batch, P(x), P(w), static_cast<const float*>(P(bias)), P(y),
                              S(stream)),
              "stem_pool");
        },
        py::arg("batch"), py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"),
        py::arg("stream"));
  m.def("stem_pack",
        [](int batch, int H, int W, int C, int Wp, int lp, uintptr_t x, uintptr_t y,
           uintptr_t stream) {
          chk(gale::stem_pack(batch, H, W, C, Wp, lp, static_cast<const float*>(P(x)), P(y),
                              S(stream)),
              "stem_pack");
        });
  m.def("maxpool2d",
        [](int batch, int H, int W, int C, int k, int s, int p, int Ho, int Wo, uintptr_t x,
           uintptr_t y, uintptr_t stream, int fp8) {
          chk(gale::maxpool2d(batch, H, W, C, k, s, p, Ho, Wo, P(x), P(y), fp8, S(stream)),
              "maxpool2d");
        },
        py::arg("batch"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("k"), py::arg("s"),
        py::arg("p"), py::arg("Ho"), py::arg("Wo"), py::arg("x"), py::arg("y"), py::arg("stream"),
        py::arg("fp8") = 0);
  m.def("avgpool_global",
        [](int batch, int HW, int C, uintptr_t x, uintptr_t y, uintptr_t stream, int fp8) {
          chk(gale::avgpool_global(batch, HW, C, P(x), P(y), fp8, S(stream)), "avgpool_global");
        },
        py::arg("batch"), py::arg("HW"), py::arg("C"), py::arg("x"), py::arg("y"),
        py::arg("stream"), py::arg("fp8") = 0);
  m.def("head_pool_dense_softmax",
        [](int batch, int HW, int C, int N, uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t out,
           uintptr_t stream, int fp8, float in_scale) {
          chk(gale::head_pool_dense_softmax(batch, HW, C, N, P(x), fp8, in_scale,
                                            static_cast<const float*>(P(w)),
                                            static_cast<const float*>(P(b)),
                                            static_cast<float*>(P(out)), S(stream)),
              "head_pool_dense_softmax");
        },
        py::arg("batch"), py::arg("HW"), py::arg("C"), py::arg("N"), py::arg("x"), py::arg("w"),
        py::arg("b"), py::arg("out"), py::arg("stream"), py::arg("fp8") = 0,
        py::arg("in_scale") = 1.0f);
  m.def("softmax_rows", [](int batch, int N, int ld, uintptr_t x, uintptr_t out, uintptr_t stream) {
    chk(gale::softmax_rows(batch, N, ld, static_cast<const float*>(P(x)),
                           static_cast<float*>(P(out)), S(stream)),
        "softmax_rows");
  });
  m.def("cast_f32_bf16",
        [](int64_t n, float scale, float shift, uintptr_t x, uintptr_t y, uintptr_t stream) {
          chk(gale::cast_f32_bf16(n, scale, shift, static_cast<const float*>(P(x)), P(y),
                                  S(stream)),
              "cast_f32_bf16");
        });
  m.def("bn_act",
        [](int batch, int HW, int Wo, int C, uintptr_t x, uintptr_t scale, uintptr_t shift,
           uintptr_t res, int res_H, int res_W, int res_C, int rs, int relu, uintptr_t y,
           uintptr_t stream) {
          chk(gale::bn_act(batch, HW, Wo, C, P(x), static_cast<const float*>(P(scale)),
                           static_cast<const float*>(P(shift)), P(res), res_H, res_W, res_C, rs,
                           relu, P(y), S(stream)),
              "bn_act");
        });
  m.def("json_parse_instances",
        [](int nrec, int ntiles, uintptr_t recs, uintptr_t tile_rec, uintptr_t bytes, int H,
           int W, int C, uintptr_t tile_counts, uintptr_t out, uintptr_t stream,
           bool count_pass) {
          chk(gale::json_parse_instances(nrec, ntiles, static_cast<gale::JsonRecord*>(P(recs)),
                                         static_cast<const int*>(P(tile_rec)),
                                         static_cast<const uint8_t*>(P(bytes)), H, W, C,
                                         static_cast<int*>(P(tile_counts)),
                                         static_cast<float*>(P(out)), S(stream), count_pass),
              "json_parse_instances");
        },
        py::arg("nrec"), py::arg("ntiles"), py::arg("recs"), py::arg("tile_rec"),
        py::arg("bytes"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("tile_counts"),
        py::arg("out"), py::arg("stream"), py::arg("count_pass") = true);
  m.def("json_tile_count", &gale::json_tile_count);
  py::module_ comm = m.def_submodule("comm", "in-process RCCL communicator (ncclCommInitAll)");
  py::class_<gale::CommGroup, std::shared_ptr<gale::CommGroup>>(comm, "CommGroup")
      .def(py::init([](std::vector<int> devices) {
             py::gil_scoped_release nogil;
             return std::make_shared<gale::CommGroup>(devices);
           }),
           py::arg("devices"))
      .def_property_readonly("size", &gale::CommGroup::size)
      .def_property_readonly("devices", &gale::CommGroup::devices)
      .def("broadcast",
           [](gale::CommGroup& g, uintptr_t send_root, std::vector<uintptr_t> recv, size_t bytes,
              int root) {
             std::vector<void*> r;
             for (uintptr_t p : recv) r.push_back(reinterpret_cast<void*>(p));
             py::gil_scoped_release nogil;
             g.broadcast(reinterpret_cast<const void*>(send_root), r, bytes, root);
           },
           py::arg("send_root"), py::arg("recv"), py::arg("bytes"), py::arg("root") = 0)
      .def("all_reduce_sum_f64",
           [](gale::CommGroup& g, std::vector<uintptr_t> bufs, size_t count) {
             std::vector<double*> b;
             for (uintptr_t p : bufs) b.push_back(reinterpret_cast<double*>(p));
             py::gil_scoped_release nogil;
             g.all_reduce_sum_f64(b, count);
           },
           py::arg("bufs"), py::arg("count"));
  m.def("crc32c_chunks",
        [](uintptr_t bytes, uintptr_t chunks, int n, uintptr_t tables, uintptr_t out,
           uintptr_t stream) {
          gale::check_hip(gale::crc32c_chunks(reinterpret_cast<const uint8_t*>(bytes),
                                              reinterpret_cast<const gale::CrcChunk*>(chunks), n,
                                              reinterpret_cast<const uint32_t*>(tables),
                                              reinterpret_cast<uint32_t*>(out),
                                              reinterpret_cast<hipStream_t>(stream)),
                          "crc32c_chunks");
        });
  m.def("ingest_crc_count",
        [](uintptr_t bytes, uintptr_t chunks, int nchunks, uintptr_t tables, uintptr_t crc_out,
           int nrec, int ngroups, uintptr_t recs, uintptr_t groups, uintptr_t counts,
           uintptr_t gsum, uintptr_t stream, uintptr_t gbad, uintptr_t packed, uintptr_t tab,
           uintptr_t text_out) {
          gale::check_hip(
              gale::ingest_crc_count(reinterpret_cast<const uint8_t*>(bytes),
                                     reinterpret_cast<const gale::CrcChunk*>(chunks), nchunks,
                                     reinterpret_cast<const uint32_t*>(tables),
                                     reinterpret_cast<uint32_t*>(crc_out), nrec, ngroups,
                                     reinterpret_cast<gale::JsonRecord*>(recs),
                                     reinterpret_cast<const int2*>(groups),
                                     reinterpret_cast<int*>(counts),
                                     reinterpret_cast<int*>(gsum),
                                     reinterpret_cast<int*>(gbad),
                                     reinterpret_cast<hipStream_t>(stream),
                                     reinterpret_cast<const uint8_t*>(packed),
                                     reinterpret_cast<const uint32_t*>(tab),
                                     reinterpret_cast<uint8_t*>(text_out)),
              "ingest_crc_count");
        },
        py::arg("bytes"), py::arg("chunks"), py::arg("nchunks"), py::arg("tables"),
        py::arg("crc_out"), py::arg("nrec"), py::arg("ngroups"), py::arg("recs"),
        py::arg("groups"), py::arg("counts"), py::arg("gsum"), py::arg("stream"),
        py::arg("gbad") = 0, py::arg("packed") = 0, py::arg("tab") = 0, py::arg("text_out") = 0,
        "groups: int32 (record, first tile) pairs, GROUP_TILES tiles each; counts: per record "
        "tile0 + grp0 -> [tile counts][group sums]; gsum: one int per group");
  m.attr("GROUP_TILES") = gale::kGroupTiles;
  m.def("text_unpack", [](uintptr_t packed, uintptr_t tab, int64_t n, uintptr_t out,
                          uintptr_t stream) {
    if (out % 16 || packed % 8) throw std::invalid_argument("text_unpack: misaligned buffers");
    gale::check_hip(gale::text_unpack(reinterpret_cast<const uint8_t*>(packed),
                                      reinterpret_cast<const uint32_t*>(tab), n,
                                      reinterpret_cast<uint8_t*>(out),
                                      reinterpret_cast<hipStream_t>(stream)),
                    "text_unpack");
  });
  m.def("format_floats_java", [](int n, uintptr_t x, uintptr_t out16, uintptr_t stream) {
    gale::check_hip(gale::format_floats_java(n, reinterpret_cast<const float*>(x),
                                             reinterpret_cast<void*>(out16),
                                             reinterpret_cast<hipStream_t>(stream)),
                    "format_floats_java");
  });
  m.def("set_conv_path", &gale::set_conv_path);
  m.def("set_conv_patch", &gale::set_conv_patch);
  m.def("conv_patch_supported", [](py::dict desc, int batch, bool has_res) {
    return gale::conv_patch_supported(desc_from_dict(desc), batch, has_res);
  });
  m.def("device_pci_bus_id", [](int device) {
    char buf[64] = {0};
    chk(hipDeviceGetPCIBusId(buf, (int)sizeof(buf), device), "hipDeviceGetPCIBusId");
    return std::string(buf);
  });
  m.def("conv_path", &gale::conv_path);
  m.attr("JSON_TILE_BYTES") = gale::kJsonTileBytes;
  m.attr("JSON_RECORD_BYTES") = (int)sizeof(gale::JsonRecord);
  m.def("memcpy_async",
        [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t stream) {
          chk(hipMemcpyAsync(P(dst), P(src), n, hipMemcpyDefault, S(stream)), "memcpy_async");
        });
  m.def("stream_sync", [](uintptr_t stream) {
    py::gil_scoped_release nogil;
    chk(hipStreamSynchronize(S(stream)), "stream_sync");
  });

  py::class_<gale::Executor, std::shared_ptr<gale::Executor>>(m, "Executor")
      .def(py::init([](int device, py::list ops, std::vector<long long> buf_bytes, int max_batch,
                       int slots, std::vector<int> buckets, int chunk_ops, int chunk_images) {
             gale::PlanSpec spec;
             for (auto o : ops) spec.ops.push_back(op_from_dict(o.cast<py::dict>()));
             spec.buf_bytes_per_image = std::move(buf_bytes);
             spec.max_batch = max_batch;
             spec.slots = slots;
             spec.buckets = std::move(buckets);
             spec.chunk_ops = chunk_ops;
             spec.chunk_images = chunk_images;
             return std::make_shared<gale::Executor>(device, std::move(spec));
           }),
           py::arg("device"), py::arg("ops"), py::arg("buf_bytes"), py::arg("max_batch"),
           py::arg("slots") = 2, py::arg("buckets") = std::vector<int>{}, py::arg("chunk_ops") = 0,
           py::arg("chunk_images") = 0)
      .def("run",
           [](gale::Executor& e, int slot, int batch, uintptr_t stream, bool use_graph) {
             py::gil_scoped_release nogil;
             e.run(slot, batch, S(stream), use_graph);
           },
           py::arg("slot"), py::arg("batch"), py::arg("stream"), py::arg("use_graph") = true)
      .def("run_on",
           [](gale::Executor& e, int batch, uintptr_t in, uintptr_t out, uintptr_t stream) {
             py::gil_scoped_release nogil;
             e.run_on(batch, P(in), P(out), S(stream));
           })
      .def("capture_all",
           [](gale::Executor& e, uintptr_t stream) {
             py::gil_scoped_release nogil;
             e.capture_all(S(stream));
           })
      .def("input_ptr", [](gale::Executor& e, int slot) { return (uintptr_t)e.input(slot); })
      .def("output_ptr", [](gale::Executor& e, int slot) { return (uintptr_t)e.output(slot); })
      .def("bucket_for", &gale::Executor::bucket_for)
      .def_property_readonly("buckets", &gale::Executor::buckets)
      .def_property_readonly("max_batch", &gale::Executor::max_batch)
      .def_property_readonly("slots", &gale::Executor::slots)
      .def_property_readonly("device", &gale::Executor::device)
      .def_property_readonly("graphs_captured", &gale::Executor::graphs_captured)
      .def_property_readonly("graph_pays", &gale::Executor::graph_pays)
      .def_property_readonly("step_out_ok", &gale::Executor::step_out_ok);

  gale::bind_host(m);
}
