// Whole-network MNIST LeNet-5 (BASELINE config 1) in one kernel: x fp32 [B,28,28,1] -> softmax
// fp32 [B,10]. The layer-by-layer plan runs seven kernels per batch on activations of a few KB
// per image - conv 5x5 (1->6, pad 2), pool, conv 5x5 (6->16), pool, fc 400->120, fc 120->84,
// fc 84->10 + softmax - so its device time is launch and round-trip latency, not math (0.83 MFLOP
// per image). Here one workgroup (4 waves) carries one image through every layer with all
// activations in LDS (fp32, ~19 KB) and the bf16 packed weights of the serving plan
// (gale/models/graph.py pack_params: conv [Npad][Kpad], k = (ky*KW + kx)*Cin_stored + ci):
//   * conv1 + ReLU + 2x2 max-pool fused: one work item = one (channel, pooled pixel) from a 6x6
//     register patch of the zero-padded input;
//   * conv2 + ReLU + pool fused: one item = one (output channel, pooled pixel), 6 input-channel
//     patches streamed through registers, weights as LDS broadcasts;
//   * the dense layers: two lanes per output neuron, each over half of the 16-byte bf16 weight
//     row, joined by a lane exchange;
//   * logits and the row softmax in LDS.
// The math is fp32 FMA on the vector ALUs: 0.8 MFLOP per image is a few us of a CU's VALU time,
// below what MFMA tiling (16-row minimum, K padded to 32) would save; one image per workgroup
// keeps the per-batch latency at one image's chain (a 4-image workgroup measured 32 us per
// batch of 256, latency-bound).
#include <math.h>

#include "common.cuh"
#include "gale/kernels.h"
#include "java_float.cuh"

namespace gale {
namespace {

constexpr int kT = 256;           // threads per workgroup (one image)
constexpr int kPad = 32;          // zero-padded input row (28 + 2 + 2)
constexpr int kImg = kPad * kPad;
constexpr int kA1 = 6 * 14 * 14;  // conv1 -> pool: [c][y][x]
constexpr int kA2 = 400;          // conv2 -> pool: [(y*5 + x)*16 + c], fc1's k order

// dot of an fp32 LDS vector with a bf16 weight row over [k0, k1) (multiples of 8)
__device__ __forceinline__ float dot_bf16(const float* a, const bf16* row, int k0, int k1) {
  float acc = 0.f;
  for (int k = k0; k < k1; k += 8) {
    const bf16x8 w8 = ld_bf16x8(row + k);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(a[k + j], (float)w8[j], acc);
  }
  return acc;
}

__global__ __launch_bounds__(kT) void lenet5_fused_kernel(LeNet5Params p, int n,
                                                          const float* __restrict__ x,
                                                          float* __restrict__ out,
                                                          InputTable tab) {
  __shared__ float s_img[kImg];
  __shared__ float s_a1[kA1];
  __shared__ float s_a2[kA2];
  __shared__ float s_a3[120];
  __shared__ float s_a4[88];
  __shared__ float s_lg[10];
  __shared__ float s_w1[6 * 25], s_b1[6];
  __shared__ float s_w2[16 * 150], s_b2[16];  // [c][(ky*5 + kx)*6 + ci]
  const int t = threadIdx.x;
  const int img = blockIdx.x;
  if (p.so.status_out && img == 0) step_verdicts(p.so);  // (the parse is done)
  if (p.batch_dev && img >= *p.batch_dev) return;  // (uniform per workgroup, before any barrier)
  const bf16* w1 = static_cast<const bf16*>(p.w1);
  const bf16* w2 = static_cast<const bf16*>(p.w2);
  for (int i = t; i < 150; i += kT) s_w1[i] = (float)w1[(i / 25) * 32 + i % 25];
  if (t < 6) s_b1[t] = p.b1[t];
  for (int i = t; i < 2400; i += kT) {
    const int c = i / 150, r = i % 150;
    s_w2[i] = (float)w2[c * 224 + (r / 6) * 8 + r % 6];
  }
  if (t < 16) s_b2[t] = p.b2[t];
  const float* xi =
      tab.base[0] ? tab.base[tab.code[img] >> 24] + (size_t)(tab.code[img] & 0xffffffu) * 784
      : p.xs      ? p.xs[img]
                  : x + (size_t)img * 784;
  for (int i = t; i < kImg; i += kT) {
    const int y = i / kPad - 2, xx = i % kPad - 2;
    s_img[i] = (y >= 0 && y < 28 && xx >= 0 && xx < 28) ? xi[y * 28 + xx] : 0.f;
  }
  __syncthreads();

  // conv1 (5x5, pad 2) + ReLU + 2x2 max-pool: one (channel, pooled pixel) per item; a wave's
  // lanes share the channel, so every weight read is an LDS broadcast
  for (int o = t; o < kA1; o += kT) {
    const int c = o / 196, q = o % 196, py = q / 14, px = q % 14;
    float patch[6][6];
#pragma unroll
    for (int yy = 0; yy < 6; ++yy)
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) patch[yy][xx] = s_img[(2 * py + yy) * kPad + 2 * px + xx];
    float acc[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[d] = s_b1[c];
#pragma unroll
    for (int ky = 0; ky < 5; ++ky)
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
        const float w = s_w1[c * 25 + ky * 5 + kx];
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[d] = fmaf(patch[(d >> 1) + ky][(d & 1) + kx], w, acc[d]);
      }
    s_a1[c * 196 + q] = fmaxf(fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])), 0.f);
  }
  __syncthreads();

  // conv2 (5x5, valid) + ReLU + 2x2 max-pool: one (output channel, pooled pixel) per item
  for (int o = t; o < kA2; o += kT) {
    const int c = o / 25, q = o % 25, py = q / 5, px = q % 5;
    float acc[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[d] = s_b2[c];
    for (int ci = 0; ci < 6; ++ci) {
      float patch[6][6];
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int xx = 0; xx < 6; ++xx)
          patch[yy][xx] = s_a1[ci * 196 + (2 * py + yy) * 14 + 2 * px + xx];
#pragma unroll
      for (int ky = 0; ky < 5; ++ky)
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) {
          const float w = s_w2[c * 150 + (ky * 5 + kx) * 6 + ci];
#pragma unroll
          for (int d = 0; d < 4; ++d)
            acc[d] = fmaf(patch[(d >> 1) + ky][(d & 1) + kx], w, acc[d]);
        }
    }
    s_a2[q * 16 + c] = fmaxf(fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])), 0.f);
  }
  __syncthreads();

  // fc1 (400 -> 120) + ReLU, weights [128][416] bf16: two lanes per neuron (k halves of 200),
  // joined with one lane exchange
  if (t < 240) {
    const int nn = t >> 1, h = t & 1;
    float acc = dot_bf16(s_a2, static_cast<const bf16*>(p.w3) + (size_t)nn * 416, h * 200,
                         h * 200 + 200);
    acc += __shfl_xor(acc, 1, 64);
    if (!h) s_a3[nn] = fmaxf(acc + p.b3[nn], 0.f);
  }
  __syncthreads();

  // fc2 (120 -> 84) + ReLU, weights [128][128] bf16: k halves [0, 64) and [64, 120)
  if (t < 168) {
    const int nn = t >> 1, h = t & 1;
    float acc = dot_bf16(s_a3, static_cast<const bf16*>(p.w4) + (size_t)nn * 128, h * 64,
                         h ? 120 : 64);
    acc += __shfl_xor(acc, 1, 64);
    if (!h) s_a4[nn] = fmaxf(acc + p.b4[nn], 0.f);
  }
  __syncthreads();

  // fc3 (84 -> 10, fp32 weights [10][88]) and the row softmax
  if (t < 10) {
    float acc = p.b5[t];
    const float* row = p.w5 + t * 88;
    for (int k = 0; k < 84; ++k) acc = fmaf(s_a4[k], row[k], acc);
    s_lg[t] = acc;
  }
  __syncthreads();
  if (t < 10) {
    float m = s_lg[0];
#pragma unroll
    for (int k = 1; k < 10; ++k) m = fmaxf(m, s_lg[k]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 10; ++k) s += expf(s_lg[k] - m);
    const float prob = expf(s_lg[t] - m) / s;
    out[(size_t)img * 10 + t] = prob;
    if (p.so.text) static_cast<uint4*>(p.so.text)[(size_t)img * 10 + t] = java_float_slot(prob);
  }
}

}  // namespace

hipError_t lenet5_fused_forward(const LeNet5Params& p, int batch, const float* x, float* out,
                                hipStream_t stream, const InputTable* tab) {
  if (batch <= 0) return hipSuccess;
  if (!p.w1 || !p.b1 || !p.w2 || !p.b2 || !p.w3 || !p.b3 || !p.w4 || !p.b4 || !p.w5 || !p.b5)
    return hipErrorInvalidValue;
  static const InputTable kNoTable{};
  if (tab && (batch > kInputTableImages || !tab->base[0])) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lenet5_fused_kernel, dim3((unsigned)batch), dim3(kT), 0, stream, p, batch,
                     x, out, tab ? *tab : kNoTable);
  return hipGetLastError();
}

}  // namespace gale
