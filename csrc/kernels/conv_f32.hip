// Reference-precision convolution: fp32 operands on the CDNA4 fp32 matrix core
// (v_mfma_f32_16x16x4_f32), fp32 accumulate, fp32 NHWC activations (--dtype fp32).
//
// The reference runs its TF graph in fp32 on the CPU (InferenceBolt.java:80-86). gale serves in
// bf16 / fp8; this plan exists to pin parity with that fp32 graph: every input, weight,
// activation and epilogue value stays binary32 (no bf16 storage, no xf32 - gfx950 dropped it),
// so the only difference from an fp32 CPU conv is the summation order.
//
// Implicit GEMM D[channel][pixel] = W[channel][k] * X[k][pixel] (same orientation as
// conv_mfma.hip: lane l of an MFMA tile owns channels 4*(l>>4)..+3 of pixel l & 15, so the
// epilogue stores 16-byte float4 rows). A 256-thread workgroup computes 64 channels x 64
// pixels: wave w owns pixels [16w, 16w+16) and all four 16-channel tiles, so each B fragment
// (one LDS read) feeds 4 MFMAs. K is walked in chunks of 16 staged through LDS (weights as
// [64][16+1] and the im2col tile as [16][64+16]: both padded so the fragment reads of a
// half-wave hit 32 distinct banks); each chunk is 4 k-steps of 4.
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

constexpr int kTM = 64;            // pixels per workgroup
constexpr int kTN = 64;            // channels per workgroup
constexpr int kKC = 16;            // K chunk
constexpr int kAS = kKC + 1;       // LDS row stride of the weight tile (floats)
constexpr int kBS = kTM + 16;      // LDS row stride of the im2col tile (floats)

struct F32Args {
  const float* x;
  const float* w;
  const float* bias;
  const float* res;
  float* y;
  int M, H, W, Cin, Ho, Wo, HWo, Cout, KW, stride, pad, K, Kpad, Npad;
  int relu, has_res, res_H, res_W, res_C, res_stride;
};

__device__ __forceinline__ float im2col(const F32Args& a, int n, int ho, int wo, int k) {
  if (k >= a.K) return 0.f;
  const int tap = k / a.Cin, ci = k - tap * a.Cin;
  const int kh = tap / a.KW, kw = tap - kh * a.KW;
  const int hi = ho * a.stride - a.pad + kh, wi = wo * a.stride - a.pad + kw;
  if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) return 0.f;
  return a.x[((size_t)(n * a.H + hi) * a.W + wi) * a.Cin + ci];
}

__global__ __launch_bounds__(256) void conv_f32_kernel(F32Args a) {
  __shared__ float As[kTN * kAS];
  __shared__ float Bs[kKC * kBS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * kTM, n0 = blockIdx.y * kTN;
  // this thread's staging slots: weights row tid/4, k 4*(tid%4)..; im2col pixel tid%64, k
  // 4*(tid/64)..
  const int arow = tid >> 2, akq = (tid & 3) * 4;
  const int bpx = tid & 63, bkq = (tid >> 6) * 4;
  const int m = m0 + bpx;
  const bool mvalid = m < a.M;
  const int n_img = mvalid ? m / a.HWo : 0;
  const int prem = mvalid ? m - n_img * a.HWo : 0;
  const int ho = prem / a.Wo, wo = prem - (prem / a.Wo) * a.Wo;
  const bool vec = (a.Cin & 3) == 0;  // 4 consecutive k = 4 channels of one tap
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < a.Kpad; k0 += kKC) {
    // weights: a 16-byte load per thread (Kpad % 16 == 0, rows >= Npad read as zero)
    float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n0 + arow < a.Npad)
      wv = *reinterpret_cast<const float4*>(a.w + (size_t)(n0 + arow) * a.Kpad + k0 + akq);
    // im2col: 4 consecutive k of one output pixel
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (mvalid) {
      const int k = k0 + bkq;
      if (vec && k < a.K) {
        const int tap = k / a.Cin, ci = k - tap * a.Cin;
        const int kh = tap / a.KW, kw = tap - kh * a.KW;
        const int hi = ho * a.stride - a.pad + kh, wi = wo * a.stride - a.pad + kw;
        if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W) {
          const float4 v = *reinterpret_cast<const float4*>(
              a.x + ((size_t)(n_img * a.H + hi) * a.W + wi) * a.Cin + ci);
          bv[0] = v.x; bv[1] = v.y; bv[2] = v.z; bv[3] = v.w;
        }
      } else if (!vec) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = im2col(a, n_img, ho, wo, k + j);
      }
    }
    __syncthreads();  // (the previous chunk's fragments have been read)
    float* ar = As + arow * kAS + akq;
    ar[0] = wv.x; ar[1] = wv.y; ar[2] = wv.z; ar[3] = wv.w;
#pragma unroll
    for (int j = 0; j < 4; ++j) Bs[(bkq + j) * kBS + bpx] = bv[j];
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kKC; ks += 4) {
      const int kk = ks + (lane >> 4);
      const float b = Bs[kk * kBS + wave * 16 + (lane & 15)];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float av = As[(t * 16 + (lane & 15)) * kAS + kk];
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b, acc[t], 0, 0, 0);
      }
    }
  }
  // epilogue: lane owns channels c..c+3 of pixel p for each channel tile t
  const int p = m0 + wave * 16 + (lane & 15);
  if (p >= a.M) return;
  const int pn = p / a.HWo, pr = p - pn * a.HWo;
  const int pho = pr / a.Wo, pwo = pr - (pr / a.Wo) * a.Wo;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int c = n0 + t * 16 + 4 * (lane >> 4);
    if (c >= a.Cout) continue;  // (Cout % 4 == 0: a row of 4 is all in or all out)
    float v[4] = {acc[t][0], acc[t][1], acc[t][2], acc[t][3]};
    const float4 bb = *reinterpret_cast<const float4*>(a.bias + c);
    v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
    if (a.has_res) {
      const int rh = pho * a.res_stride, rw = pwo * a.res_stride;
      const float* rp = a.res + ((size_t)(pn * a.res_H + rh) * a.res_W + rw) * a.res_C;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c + j < a.res_C) v[j] += rp[c + j];  // option A: zero above res_C
    }
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    *reinterpret_cast<float4*>(a.y + (size_t)p * a.Cout + c) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

}  // namespace

hipError_t conv2d_f32(const ConvDesc& d, int batch, const void* x, const void* w,
                      const float* bias, const void* res, void* y, hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (d.Kpad % kKC || d.Cout % 4 || d.K > d.Kpad || d.Npad < d.Cout || d.fp8 || d.stem)
    return hipErrorInvalidValue;
  if (d.has_res && res && (d.res_stride < 1 || d.res_C > d.Cout || d.res_C % 4))
    return hipErrorInvalidValue;
  F32Args a;
  a.x = static_cast<const float*>(x);
  a.w = static_cast<const float*>(w);
  a.bias = bias;
  a.res = static_cast<const float*>(res);
  a.y = static_cast<float*>(y);
  a.M = batch * d.Ho * d.Wo;
  a.H = d.H; a.W = d.W; a.Cin = d.Cin; a.Ho = d.Ho; a.Wo = d.Wo; a.HWo = d.Ho * d.Wo;
  a.Cout = d.Cout; a.KW = d.KW; a.stride = d.stride; a.pad = d.pad; a.K = d.K; a.Kpad = d.Kpad;
  a.Npad = d.Npad;
  a.relu = d.relu;
  a.has_res = d.has_res && res != nullptr;
  a.res_H = d.res_H; a.res_W = d.res_W; a.res_C = d.res_C; a.res_stride = d.res_stride;
  const dim3 grid((a.M + kTM - 1) / kTM, (d.Cout + kTN - 1) / kTN);
  hipLaunchKernelGGL(conv_f32_kernel, grid, dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace gale
