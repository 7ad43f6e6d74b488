// Model plan executor: runs a flat list of gale kernels on one device/stream and replays each
// (batch bucket, I/O slot) pair from a captured hipGraph.
//
// Replaces the reference's per-tuple `sess.runner().feed("input:0").fetch("output/Softmax:0")
// .run()` (InferenceBolt.java:81-85): the model is a static plan built once (R6 prepare,
// InferenceBolt.java:43-62) and every micro-batch is one graph launch.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "gale/kernels.h"

namespace gale {

enum OpKind : int {
  OP_CONV = 0,      // conv2d (also dense layers as 1x1 convs)
  OP_MAXPOOL = 1,   // p[0..6] = H, W, C, k, s, pad, Ho ; p[7] = Wo
  OP_AVGPOOL = 2,   // p[0] = HW, p[1] = C
  OP_HEAD = 3,      // p[0] = HW, p[1] = C, p[2] = N   (pool + dense(fp32 w) + softmax)
  OP_SOFTMAX = 4,   // p[0] = N, p[1] = ld
  OP_RESNET20 = 5,  // whole-network fused CIFAR ResNet-20; ptrs = 19 w, 19 b, fc_w, fc_b
                    // (+ 19 wscale for fp8), scales = 19 s_in, 19 s_out, 19 s_res (fp8)
  OP_STEM_PACK = 6, // p[0..4] = H, W, C, Wp, lp  (fp32 input -> packed-stem bf16 image)
  OP_BN_ACT = 7,    // p[0..7] = HW, Wo, C, relu, res_H, res_W, res_C, res_stride; w = BN scale,
                    // bias = BN shift (unfolded-BN plan: standalone BatchNorm + add + ReLU)
  OP_LENET5 = 8,    // whole-network fused MNIST LeNet-5; ptrs = w1 b1 w2 b2 w3 b3 w4 b4 w5 b5
  OP_BOTTLENECK = 9,  // one whole ResNet-50 56x56 bottleneck (bottleneck56); ptrs = w1 b1 w2 b2
                      // w3 b3 [wd bd]; p[0] = cin, p[1] = down (projection shortcut)
  OP_STEM_POOL = 10,  // ResNet-50 stem conv + max-pool (stem_pool); conv = the stem's desc,
                      // w / bias = its weights; p[0..7] = the max-pool's H W C k s pad Ho Wo
  OP_CONV_PROJ = 11,  // bottleneck conv3 + projection shortcut as one GEMM (conv2d_gemm_proj):
                      // conv = conv3's desc, in = its input, res = the block input (the
                      // projection's source); ptrs = w3 b3 wd bd; p[0..4] = H2 W2 Cin2 stride2 Kpad2
};

// Buffer ids: 0 = network input (fp32 NHWC), 1 = network output (fp32 [B, classes]),
// >= 2 = activation workspace.
struct PlanOp {
  int kind = 0;
  ConvDesc conv{};
  int p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int in = 0, out = 0, res = -1;
  const void* w = nullptr;
  const float* bias = nullptr;
  const float* wscale = nullptr;
  std::vector<const void*> ptrs;  // OP_RESNET20 parameter pointers
  std::vector<float> scales;      // OP_RESNET20 fp8 activation scales
  int fp8 = 0;        // pool / head ops: activation ElemType (0 bf16, 1 e4m3, 2 fp32)
  float scale = 1.f;  // head: input activation scale (fp8)
  long long bpi[3] = {0, 0, 0};  // bytes per image of the in / out / res tensors (chunking)
};

struct PlanSpec {
  std::vector<PlanOp> ops;
  std::vector<long long> buf_bytes_per_image;  // indexed by buffer id (ids 0 and 1 included)
  int max_batch = 256;
  int slots = 2;                               // independent I/O buffer sets (pipelining depth)
  std::vector<int> buckets;                    // graph batch buckets (ascending); empty = powers of 2
  // Batch chunking of the leading ops: ops [0, chunk_ops) run once per chunk of chunk_images
  // images (operands offset by the first image of the chunk times their PlanOp::bpi; activations
  // are batch-major), the
  // rest once over the whole batch. Keeps the wide early tensors (ResNet-50 56x56x256 at batch
  // 256: 411 MB each) small enough to stay in the 256 MB Infinity Cache between producer and
  // consumer. 0 = off. The plan must keep every tensor that outlives the prefix in a buffer no
  // other prefix tensor uses (a later chunk would overwrite it): build_plan(chunk_layers=...).
  int chunk_ops = 0;
  int chunk_images = 0;
};

class Executor {
 public:
  Executor(int device, PlanSpec spec);
  ~Executor();
  Executor(const Executor&) = delete;
  Executor& operator=(const Executor&) = delete;

  int device() const { return device_; }
  int max_batch() const { return spec_.max_batch; }
  int slots() const { return spec_.slots; }
  const std::vector<int>& buckets() const { return buckets_; }
  int bucket_for(int batch) const;

  // Device I/O buffers of a slot (input fp32 [max_batch, ...], output fp32 [max_batch, classes]).
  void* input(int slot) const { return bufs_[slot][0]; }
  void* output(int slot) const { return bufs_[slot][1]; }
  long long input_bytes_per_image() const { return spec_.buf_bytes_per_image[0]; }
  long long output_bytes_per_image() const { return spec_.buf_bytes_per_image[1]; }

  // Enqueue the forward for `batch` images of `slot` on `stream`. use_graph replays (capturing on
  // first use) the graph of the smallest bucket >= batch; otherwise launches kernels eagerly.
  // Plans of at most kMaxDirectOps kernels (the whole-network ResNet-20 kernel) always launch
  // directly: a graph saves nothing there, runs the padded bucket batch, and every replay costs
  // CPU on the HIP runtime's worker thread (~0.9 core at the serving rate, -> 0.16 with direct
  // launches, measured in round 3).
  static constexpr size_t kMaxDirectOps = 2;
  bool graph_pays() const { return spec_.ops.size() > kMaxDirectOps; }
  void run(int slot, int batch, hipStream_t stream, bool use_graph);
  // Eager forward on caller-provided device buffers (tests / ops API; no graph).
  void run_on(int batch, const void* in, void* out, hipStream_t stream);
  void capture_all(hipStream_t stream);  // pre-capture every (bucket, slot) graph
  int graphs_captured() const;
  // Plans whose every op reads its image count from device memory (the whole-network kernels):
  // launch_device_batch enqueues the forward of `slot` sized for max_batch images, the count
  // taken from *d_batch when the kernels run - what a captured per-slot step graph replays
  // for every batch size (GpuReplica step graphs).
  // so (optional): the step outputs the forward kernel writes in its own epilogue (prediction
  // text, parse verdicts; gale/kernels.h StepOut) - only when step_out_ok()
  bool device_batch_ok() const;
  bool step_out_ok() const { return device_batch_ok() && spec_.ops.size() == 1; }
  // xs (optional, device memory): image i's fp32 input at xs[i] instead of the slot's input
  // buffer - images the GPU ingest already parsed (whole-network plans: device_batch_ok())
  void launch_device_batch(int slot, const int* d_batch, hipStream_t stream,
                           const StepOut* so = nullptr, const float* const* xs = nullptr);
  // The forward of `batch` images taken from an input table in the kernel arguments (images the
  // GPU ingest parsed): no metadata in device memory, one launch (step_out_ok() plans)
  void launch_table(int slot, int batch, const InputTable& tab, hipStream_t stream,
                    const StepOut* so = nullptr);

 private:
  void launch_all(int batch, void* const* bufs, hipStream_t stream,
                  const int* d_batch = nullptr, const StepOut* so = nullptr,
                  const float* const* xs = nullptr);
  // ops [begin, end) for images [c0, c0 + batch) of the buffers (c0 > 0: a chunk)
  void launch_ops(size_t begin, size_t end, int batch, void* const* bufs, hipStream_t stream,
                  int c0 = 0, const int* d_batch = nullptr, const StepOut* so = nullptr,
                  const float* const* xs = nullptr, const InputTable* tab = nullptr);
  int device_;
  PlanSpec spec_;
  std::vector<int> buckets_;
  std::vector<std::vector<void*>> bufs_;  // [slot][buffer id]
  void* shared_ws_ = nullptr;             // activation buffers shared by every slot
  std::map<std::pair<int, int>, hipGraphExec_t> graphs_;
  mutable std::mutex mu_;
  std::mutex capture_mu_;
};

void check_hip(hipError_t e, const char* what);

}  // namespace gale
