// Plan executor (see gale/executor.h).
#include "gale/executor.h"

#include <algorithm>
#include <stdexcept>

namespace gale {

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
  }
}

Executor::Executor(int device, PlanSpec spec) : device_(device), spec_(std::move(spec)) {
  if (spec_.buf_bytes_per_image.size() < 2) throw std::invalid_argument("plan needs >= 2 buffers");
  if (spec_.max_batch <= 0 || spec_.slots <= 0) throw std::invalid_argument("bad max_batch/slots");
  buckets_ = spec_.buckets;
  if (buckets_.empty()) {
    for (int b = 1; b < spec_.max_batch; b *= 2) buckets_.push_back(b);
    buckets_.push_back(spec_.max_batch);
  }
  if (spec_.chunk_ops < 0 || spec_.chunk_ops > (int)spec_.ops.size() || spec_.chunk_images < 0)
    throw std::invalid_argument("bad chunk_ops / chunk_images");
  for (int i = 0; spec_.chunk_images > 0 && i < spec_.chunk_ops; ++i) {
    const PlanOp& op = spec_.ops[i];
    if (op.bpi[0] <= 0 || op.bpi[1] <= 0 || (op.res >= 0 && op.bpi[2] <= 0))
      throw std::invalid_argument("chunked plan op without per-image operand bytes");
  }
  std::sort(buckets_.begin(), buckets_.end());
  buckets_.erase(std::unique(buckets_.begin(), buckets_.end()), buckets_.end());
  if (buckets_.back() < spec_.max_batch) buckets_.push_back(spec_.max_batch);

  check_hip(hipSetDevice(device_), "hipSetDevice");
  const size_t nb = spec_.buf_bytes_per_image.size();
  // activation workspace (ids >= 2) shared by all slots: one compute stream per executor
  size_t ws_total = 0;
  std::vector<size_t> ws_off(nb, 0);
  for (size_t i = 2; i < nb; ++i) {
    ws_off[i] = ws_total;
    const size_t bytes = (size_t)spec_.buf_bytes_per_image[i] * spec_.max_batch;
    ws_total += (bytes + 255) & ~size_t(255);
  }
  if (ws_total) check_hip(hipMalloc(&shared_ws_, ws_total), "hipMalloc(workspace)");
  bufs_.resize(spec_.slots);
  for (int s = 0; s < spec_.slots; ++s) {
    bufs_[s].assign(nb, nullptr);
    for (int i = 0; i < 2; ++i) {
      const size_t bytes = (size_t)spec_.buf_bytes_per_image[i] * spec_.max_batch;
      check_hip(hipMalloc(&bufs_[s][i], bytes ? bytes : 256), "hipMalloc(io)");
      check_hip(hipMemset(bufs_[s][i], 0, bytes ? bytes : 256), "hipMemset(io)");
    }
    for (size_t i = 2; i < nb; ++i) bufs_[s][i] = static_cast<char*>(shared_ws_) + ws_off[i];
  }
}

Executor::~Executor() {
  hipSetDevice(device_);
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  for (auto& s : bufs_) {
    if (s.size() >= 2) {
      hipFree(s[0]);
      hipFree(s[1]);
    }
  }
  if (shared_ws_) hipFree(shared_ws_);
}

int Executor::bucket_for(int batch) const {
  for (int b : buckets_)
    if (b >= batch) return b;
  return -1;
}

void Executor::launch_all(int batch, void* const* bufs, hipStream_t stream, const int* d_batch,
                          const StepOut* so, const float* const* xs) {
  size_t begin = 0;
  const int ch = spec_.chunk_images;
  if (spec_.chunk_ops > 0 && ch > 0 && batch > ch) {
    for (int c0 = 0; c0 < batch; c0 += ch)
      launch_ops(0, spec_.chunk_ops, std::min(ch, batch - c0), bufs, stream, c0);
    begin = spec_.chunk_ops;
  }
  launch_ops(begin, spec_.ops.size(), batch, bufs, stream, 0, d_batch, so, xs);
}

bool Executor::device_batch_ok() const {
  if (spec_.ops.empty() || spec_.chunk_ops > 0) return false;
  for (const PlanOp& op : spec_.ops)
    if (op.kind != OP_RESNET20 && op.kind != OP_LENET5) return false;
  return true;
}

void Executor::launch_device_batch(int slot, const int* d_batch, hipStream_t stream,
                                   const StepOut* so, const float* const* xs) {
  if (!device_batch_ok()) throw std::logic_error("plan does not take a device batch count");
  if (so && !step_out_ok()) throw std::logic_error("plan cannot write the step outputs");
  if (xs && spec_.ops.size() != 1) throw std::logic_error("plan cannot read an input table");
  if (slot < 0 || slot >= spec_.slots) throw std::invalid_argument("bad slot");
  launch_all(spec_.max_batch, bufs_[slot].data(), stream, d_batch, so, xs);
}

void Executor::launch_table(int slot, int batch, const InputTable& tab, hipStream_t stream,
                            const StepOut* so) {
  if (!step_out_ok()) throw std::logic_error("plan cannot read an input table");
  if (slot < 0 || slot >= spec_.slots) throw std::invalid_argument("bad slot");
  if (batch <= 0 || batch > spec_.max_batch || batch > kInputTableImages)
    throw std::invalid_argument("bad table batch");
  launch_ops(0, 1, batch, bufs_[slot].data(), stream, 0, nullptr, so, nullptr, &tab);
}

void Executor::launch_ops(size_t begin, size_t end, int batch, void* const* bufs,
                          hipStream_t stream, int c0, const int* d_batch, const StepOut* so,
                          const float* const* xs, const InputTable* tab) {
  auto at = [&](int id, long long bpi) -> void* {
    return static_cast<char*>(bufs[id]) + (size_t)c0 * (size_t)bpi;
  };
  for (size_t oi = begin; oi < end; ++oi) {
    const PlanOp& op = spec_.ops[oi];
    const void* in = at(op.in, op.bpi[0]);
    void* out = at(op.out, op.bpi[1]);
    void* res = op.res >= 0 ? at(op.res, op.bpi[2]) : nullptr;
    hipError_t e = hipSuccess;
    switch (op.kind) {
      case OP_CONV:
        e = conv2d(op.conv, batch, in, op.w, op.bias, op.wscale, res, out, stream);
        break;
      case OP_MAXPOOL:
        e = maxpool2d(batch, op.p[0], op.p[1], op.p[2], op.p[3], op.p[4], op.p[5], op.p[6], op.p[7],
                      in, out, op.fp8, stream);
        break;
      case OP_AVGPOOL:
        e = avgpool_global(batch, op.p[0], op.p[1], in, out, op.fp8, stream);
        break;
      case OP_HEAD:
        e = head_pool_dense_softmax(batch, op.p[0], op.p[1], op.p[2], in, op.fp8, op.scale,
                                    static_cast<const float*>(op.w), op.bias,
                                    static_cast<float*>(out), stream);
        break;
      case OP_STEM_PACK:
        e = stem_pack(batch, op.p[0], op.p[1], op.p[2], op.p[3], op.p[4],
                      static_cast<const float*>(in), out, stream);
        break;
      case OP_SOFTMAX:
        e = softmax_rows(batch, op.p[0], op.p[1], static_cast<const float*>(in),
                         static_cast<float*>(out), stream);
        break;
      case OP_BN_ACT:
        e = bn_act(batch, op.p[0], op.p[1], op.p[2], in, static_cast<const float*>(op.w), op.bias,
                   res, op.p[4], op.p[5], op.p[6], op.p[7],
                   op.p[3], out, stream, (int)op.fp8);
        break;
      case OP_RESNET20: {
        const bool f8 = op.fp8 != 0;
        if (op.ptrs.size() != (f8 ? 59u : 40u) || (f8 && op.scales.size() != 57))
          throw std::invalid_argument("resnet20 op: bad pointer / scale count");
        ResNet20Params rp{};
        for (int i = 0; i < 19; ++i) {
          rp.w[i] = op.ptrs[i];
          rp.b[i] = static_cast<const float*>(op.ptrs[19 + i]);
        }
        rp.fc_w = static_cast<const float*>(op.ptrs[38]);
        rp.fc_b = static_cast<const float*>(op.ptrs[39]);
        rp.fp8 = f8 ? 1 : 0;
        rp.batch_dev = d_batch;
        rp.xs = xs;
        if (so) rp.so = *so;
        if (f8)
          for (int i = 0; i < 19; ++i) {
            rp.ws[i] = static_cast<const float*>(op.ptrs[40 + i]);
            rp.s_in[i] = op.scales[i];
            rp.s_out[i] = op.scales[19 + i];
            rp.s_res[i] = op.scales[38 + i];
          }
        e = resnet20_fused_forward(rp, batch, static_cast<const float*>(in),
                                   static_cast<float*>(out), stream, tab);
        break;
      }
      case OP_LENET5: {
        if (op.ptrs.size() != 10u) throw std::invalid_argument("lenet5 op: bad pointer count");
        LeNet5Params lp{};
        lp.w1 = op.ptrs[0];
        lp.b1 = static_cast<const float*>(op.ptrs[1]);
        lp.w2 = op.ptrs[2];
        lp.b2 = static_cast<const float*>(op.ptrs[3]);
        lp.w3 = op.ptrs[4];
        lp.b3 = static_cast<const float*>(op.ptrs[5]);
        lp.w4 = op.ptrs[6];
        lp.b4 = static_cast<const float*>(op.ptrs[7]);
        lp.w5 = static_cast<const float*>(op.ptrs[8]);
        lp.b5 = static_cast<const float*>(op.ptrs[9]);
        lp.batch_dev = d_batch;
        lp.xs = xs;
        if (so) lp.so = *so;
        e = lenet5_fused_forward(lp, batch, static_cast<const float*>(in),
                                 static_cast<float*>(out), stream, tab);
        break;
      }
      case OP_BOTTLENECK: {
        const bool down = op.p[1] != 0;
        if (op.ptrs.size() != (down ? 8u : 6u))
          throw std::invalid_argument("bottleneck op: bad pointer count");
        BottleneckParams bp;
        bp.w1 = op.ptrs[0];
        bp.b1 = static_cast<const float*>(op.ptrs[1]);
        bp.w2 = op.ptrs[2];
        bp.b2 = static_cast<const float*>(op.ptrs[3]);
        bp.w3 = op.ptrs[4];
        bp.b3 = static_cast<const float*>(op.ptrs[5]);
        if (down) {
          bp.wd = op.ptrs[6];
          bp.bd = static_cast<const float*>(op.ptrs[7]);
        }
        bp.cin = op.p[0];
        bp.down = down ? 1 : 0;
        e = bottleneck56(bp, batch, in, out, stream);
        break;
      }
      case OP_CONV_PROJ:
        if (op.ptrs.size() != 4u || res == nullptr)
          throw std::invalid_argument("conv_proj op: bad operands");
        e = conv2d_gemm_proj(op.conv, batch, in, op.ptrs[0], static_cast<const float*>(op.ptrs[1]),
                             res, op.p[0], op.p[1], op.p[2], op.p[3], op.p[4], op.ptrs[2],
                             static_cast<const float*>(op.ptrs[3]), out, stream);
        break;
      case OP_STEM_POOL:
        if (!stem_pool_supported(op.conv, op.p[0], op.p[1], op.p[2], op.p[3], op.p[4], op.p[5],
                                 op.p[6], op.p[7]))
          throw std::invalid_argument("stem_pool op: unsupported geometry");
        e = stem_pool(batch, in, op.w, op.bias, out, stream);
        break;
      default:
        throw std::invalid_argument("unknown plan op kind");
    }
    check_hip(e, "plan op launch");
  }
}

void Executor::run_on(int batch, const void* in, void* out, hipStream_t stream) {
  if (batch > spec_.max_batch) throw std::invalid_argument("batch > max_batch");
  std::vector<void*> b = bufs_[0];
  b[0] = const_cast<void*>(in);
  b[1] = out;
  launch_all(batch, b.data(), stream);
}

void Executor::run(int slot, int batch, hipStream_t stream, bool use_graph) {
  if (slot < 0 || slot >= spec_.slots) throw std::invalid_argument("bad slot");
  if (batch <= 0) return;
  if (batch > spec_.max_batch) throw std::invalid_argument("batch > max_batch");
  if (!use_graph || !graph_pays()) {
    launch_all(batch, bufs_[slot].data(), stream);
    return;
  }
  const int bucket = bucket_for(batch);
  hipGraphExec_t exec = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = graphs_.find({bucket, slot});
    if (it != graphs_.end()) exec = it->second;
  }
  if (!exec) {
    // capture on a private non-blocking stream (the legacy null stream cannot capture) that
    // lives only for the capture: serving keeps one stream per replica and per ingest lane, so
    // every stream can own a hardware queue (GPU_MAX_HW_QUEUES) - rocprofv3's queue
    // interception crashed on queues shared by concurrently submitting threads. The
    // instantiated graph is launched on the caller's stream.
    std::lock_guard<std::mutex> cap(capture_mu_);
    hipStream_t cs = nullptr;
    check_hip(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "capture stream");
    hipGraph_t graph = nullptr;
    hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
      try {
        launch_all(bucket, bufs_[slot].data(), cs);
      } catch (...) {
        hipStreamEndCapture(cs, &graph);
        if (graph) hipGraphDestroy(graph);
        hipStreamDestroy(cs);
        throw;
      }
      e = hipStreamEndCapture(cs, &graph);
    }
    hipStreamDestroy(cs);
    check_hip(e, "graph capture");
    check_hip(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0), "GraphInstantiate");
    hipGraphDestroy(graph);
    std::lock_guard<std::mutex> lk(mu_);
    graphs_[{bucket, slot}] = exec;
  }
  check_hip(hipGraphLaunch(exec, stream), "hipGraphLaunch");
}

void Executor::capture_all(hipStream_t stream) {
  if (!graph_pays()) return;
  for (int s = 0; s < spec_.slots; ++s)
    for (int b : buckets_) run(s, b, stream, true);
  check_hip(hipStreamSynchronize(stream), "capture_all sync");
}

int Executor::graphs_captured() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)graphs_.size();
}

}  // namespace gale
