// Pooling, classifier head and elementwise kernels (NHWC, gfx950).
//
// These cover the MaxPool / AvgPool / MatMul+BiasAdd / Softmax ops of the CNN classifiers the
// reference serves (README.md:16; output tensor "output/Softmax:0", InferenceBolt.java:83).
// All of them are memory-bound: bf16 traffic is vectorised 16 B per lane (8 channels).
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

// 8 channels of one pixel as floats (ET: ElemType; e4m3 values are in units of the tensor's
// scale, which pooling preserves)
template <int ET>
__device__ __forceinline__ void load8f(const void* x, size_t off, float* v) {
  if constexpr (ET == ET_F32) {
    const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x) + off);
    const float4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else if constexpr (ET == ET_FP8) {
    const uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(x) + off);
    v[0] = __builtin_amdgcn_cvt_f32_fp8((int)r.x, 0);
    v[1] = __builtin_amdgcn_cvt_f32_fp8((int)r.x, 1);
    v[2] = __builtin_amdgcn_cvt_f32_fp8((int)r.x, 2);
    v[3] = __builtin_amdgcn_cvt_f32_fp8((int)r.x, 3);
    v[4] = __builtin_amdgcn_cvt_f32_fp8((int)r.y, 0);
    v[5] = __builtin_amdgcn_cvt_f32_fp8((int)r.y, 1);
    v[6] = __builtin_amdgcn_cvt_f32_fp8((int)r.y, 2);
    v[7] = __builtin_amdgcn_cvt_f32_fp8((int)r.y, 3);
  } else {
    const bf16x8 b = ld_bf16x8(reinterpret_cast<const bf16*>(x) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
  }
}

template <int ET>
__device__ __forceinline__ void store8f(void* y, size_t off, const float* v) {
  if constexpr (ET == ET_F32) {
    float4* p = reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + off);
    p[0] = make_float4(v[0], v[1], v[2], v[3]);
    p[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else if constexpr (ET == ET_FP8) {
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(y) + off) =
        make_uint2((uint32_t)lo, (uint32_t)hi);
  } else {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(y) + off) = __builtin_bit_cast(uint4, o);
  }
}

template <int ET>
__global__ __launch_bounds__(256) void maxpool_kernel(int total, int H, int W, int C8, int k, int s,
                                                      int p, int Ho, int Wo, const void* x,
                                                      void* y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cg = i % C8;
  const int pix = i / C8;
  const int wo = pix % Wo;
  const int t = pix / Wo;
  const int ho = t % Ho;
  const int n = t / Ho;
  const int C = C8 * 8;
  float m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = -3.0e38f;
  for (int kh = 0; kh < k; ++kh) {
    const int hi = ho * s - p + kh;
    if ((unsigned)hi >= (unsigned)H) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int wi = wo * s - p + kw;
      if ((unsigned)wi >= (unsigned)W) continue;
      float v[8];
      load8f<ET>(x, ((size_t)(n * H + hi) * W + wi) * C + cg * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], v[j]);
    }
  }
  store8f<ET>(y, (size_t)pix * C + cg * 8, m);  // max of e4m3 values re-encodes exactly
}

template <int ET>
__global__ __launch_bounds__(256) void avgpool_kernel(int total, int HW, int C8, const void* x,
                                                      void* y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cg = i % C8;
  const int n = i / C8;
  const int C = C8 * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const size_t base = (size_t)n * HW * C + cg * 8;
  for (int q = 0; q < HW; ++q) {
    float v[8];
    load8f<ET>(x, base + (size_t)q * C, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += v[j];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] *= inv;
  store8f<ET>(y, (size_t)n * C + cg * 8, s);  // the mean keeps the input's scale
}

// One workgroup per image: pooled[C] -> logits[N] -> softmax, all fp32 in LDS. fp8 inputs are
// pooled in units of their scale, which is applied once to the pooled vector.
template <int ET>
__global__ __launch_bounds__(256) void head_kernel(int HW, int C, int N, const void* x,
                                                   float in_scale, const float* w,
                                                   const float* bias, float* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int C8 = C >> 3;
  const int nps = 256 / C8 > 0 ? 256 / C8 : 1;  // pixel slices summed in parallel
  float* part = reinterpret_cast<float*>(smem);            // [nps][C]
  float* pooled = part + (size_t)nps * C;                  // [C]
  float* logits = pooled + C;                              // [N]
  const int n = blockIdx.x;
  const size_t img = (size_t)n * HW * C;
  for (int t = threadIdx.x; t < nps * C8; t += 256) {
    const int cg = t % C8, ps = t / C8;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int q = ps; q < HW; q += nps) {
      float v[8];
      load8f<ET>(x, img + (size_t)q * C + cg * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[ps * C + cg * 8 + j] = s[j];
  }
  __syncthreads();
  const float inv = in_scale / (float)HW;
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int ps = 0; ps < nps; ++ps) s += part[ps * C + c];
    pooled[c] = s * inv;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o = wave; o < N; o += 4) {
    const float* wr = w + (size_t)o * C;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += wr[c] * pooled[c];
    s = wave_sum(s);
    if (lane == 0) logits[o] = s + bias[o];
  }
  __syncthreads();
  if (wave == 0) {
    float mx = -3.0e38f;
    for (int o = lane; o < N; o += 64) mx = fmaxf(mx, logits[o]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int o = lane; o < N; o += 64) {
      const float e = __expf(logits[o] - mx);
      logits[o] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float r = 1.f / sum;
    for (int o = lane; o < N; o += 64) out[(size_t)n * N + o] = logits[o] * r;
  }
}

// One wave per row.
__global__ __launch_bounds__(256) void softmax_kernel(int B, int N, int ld, const float* x,
                                                      float* out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  const float* xr = x + (size_t)row * ld;
  float mx = -3.0e38f;
  for (int o = lane; o < N; o += 64) mx = fmaxf(mx, xr[o]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int o = lane; o < N; o += 64) sum += __expf(xr[o] - mx);
  sum = wave_sum(sum);
  const float r = 1.f / sum;
  for (int o = lane; o < N; o += 64) out[(size_t)row * N + o] = __expf(xr[o] - mx) * r;
}

__global__ __launch_bounds__(256) void cast_kernel(int64_t n4, float scale, float shift,
                                                   const float* x, bf16* y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4 v = reinterpret_cast<const float4*>(x)[i];
  bf16x4 o;
  o[0] = (bf16)(v.x * scale + shift);
  o[1] = (bf16)(v.y * scale + shift);
  o[2] = (bf16)(v.z * scale + shift);
  o[3] = (bf16)(v.w * scale + shift);
  reinterpret_cast<uint2*>(y)[i] = __builtin_bit_cast(uint2, o);
}

// Standalone inference BatchNorm + residual + ReLU over NHWC bf16 or fp32 (ET; TF
// FusedBatchNorm + Add + Relu): y = act(x * scale[c] + shift[c] + res). The fast path folds BN into the conv weights
// and fuses the rest into the conv epilogue; this kernel serves the unfolded (fold_bn=False)
// plan and the standalone ops. scale == nullptr -> identity affine (plain ReLU / add). The
// residual is read at (ho*rs, wo*rs) with res_C stored channels and zero above them (ResNet
// option-A shortcut when rs == 2). One lane per 8 channels of one pixel (16-byte accesses).
template <int ET>
__global__ __launch_bounds__(256) void bn_act_kernel(int total, int HW, int Wo, int C8,
                                                     const void* x, const float* scale,
                                                     const float* shift, const void* res,
                                                     int res_H, int res_W, int res_C, int rs,
                                                     int relu, void* y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cg = i % C8;
  const int pix = i / C8;
  const size_t off = (size_t)pix * (C8 * 8) + cg * 8;
  float v[8];
  load8f<ET>(x, off, v);
  if (scale) {
    const float4* s4 = reinterpret_cast<const float4*>(scale) + cg * 2;
    const float4* t4 = reinterpret_cast<const float4*>(shift) + cg * 2;
    const float4 s0 = s4[0], s1 = s4[1], t0 = t4[0], t1 = t4[1];
    const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float t[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], s[j], t[j]);
  }
  if (res && cg * 8 < res_C) {
    const int n = pix / HW;
    const int q = pix - n * HW;
    const int ho = q / Wo;
    const int wo = q - ho * Wo;
    float r[8];
    load8f<ET>(res, ((size_t)(n * res_H + ho * rs) * res_W + wo * rs) * res_C + cg * 8, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += r[j];
  }
  if (relu) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
  }
  store8f<ET>(y, off, v);
}

}  // namespace

hipError_t maxpool2d(int batch, int H, int W, int C, int k, int s, int p, int Ho, int Wo,
                     const void* x, void* y, int et, hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (C % 8 || et < 0 || et > 2) return hipErrorInvalidValue;
  const int total = batch * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(et == ET_F32 ? maxpool_kernel<ET_F32>
                     : et == ET_FP8 ? maxpool_kernel<ET_FP8> : maxpool_kernel<ET_BF16>,
                     dim3((total + 255) / 256), dim3(256), 0, stream, total, H, W, C / 8, k, s, p,
                     Ho, Wo, x, y);
  return hipGetLastError();
}

hipError_t avgpool_global(int batch, int HW, int C, const void* x, void* y, int et,
                          hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (C % 8 || et < 0 || et > 2) return hipErrorInvalidValue;
  const int total = batch * (C / 8);
  hipLaunchKernelGGL(et == ET_F32 ? avgpool_kernel<ET_F32>
                     : et == ET_FP8 ? avgpool_kernel<ET_FP8> : avgpool_kernel<ET_BF16>,
                     dim3((total + 255) / 256), dim3(256), 0, stream, total, HW, C / 8, x, y);
  return hipGetLastError();
}

hipError_t head_pool_dense_softmax(int batch, int HW, int C, int N, const void* x, int et,
                                   float in_scale, const float* w, const float* bias, float* out,
                                   hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (C % 8 || C > 4096 || N > 4096 || et < 0 || et > 2) return hipErrorInvalidValue;
  const int C8 = C / 8;
  const int nps = 256 / C8 > 0 ? 256 / C8 : 1;
  const size_t lds = ((size_t)nps * C + C + N) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(et == ET_F32 ? head_kernel<ET_F32>
                     : et == ET_FP8 ? head_kernel<ET_FP8> : head_kernel<ET_BF16>,
                     dim3(batch), dim3(256), lds, stream, HW, C, N, x,
                     et == ET_FP8 ? in_scale : 1.f, w, bias, out);
  return hipGetLastError();
}

hipError_t softmax_rows(int batch, int N, int ld, const float* x, float* out, hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(softmax_kernel, dim3((batch + 3) / 4), dim3(256), 0, stream, batch, N, ld, x,
                     out);
  return hipGetLastError();
}

hipError_t cast_f32_bf16(int64_t n, float scale, float shift, const float* x, void* y,
                         hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (n % 4) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(cast_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream, n4,
                     scale, shift, x, reinterpret_cast<bf16*>(y));
  return hipGetLastError();
}

hipError_t bn_act(int batch, int HW, int Wo, int C, const void* x, const float* scale,
                  const float* shift, const void* res, int res_H, int res_W, int res_C, int rs,
                  int relu, void* y, hipStream_t stream, int et) {
  if (batch <= 0) return hipSuccess;
  if (et != ET_BF16 && et != ET_F32) return hipErrorInvalidValue;
  if (C % 8 || res_C % 8 || HW <= 0 || Wo <= 0 || HW % Wo || (scale && !shift)) return hipErrorInvalidValue;
  if (res && (rs < 1 || res_C > C || (HW / Wo - 1) * rs >= res_H || (Wo - 1) * rs >= res_W))
    return hipErrorInvalidValue;
  const long long total = (long long)batch * HW * (C / 8);
  if (total > 0x7fffffffLL) return hipErrorInvalidValue;
  auto k = et == ET_F32 ? bn_act_kernel<ET_F32> : bn_act_kernel<ET_BF16>;
  hipLaunchKernelGGL(k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, (int)total,
                     HW, Wo, C / 8, x, scale, shift, res, res_H, res_W, res_C, rs, relu, y);
  return hipGetLastError();
}

}  // namespace gale
