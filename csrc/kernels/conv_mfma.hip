// Implicit-GEMM convolution on CDNA4 matrix cores, NHWC, bf16 (v_mfma_f32_16x16x32_bf16) or
// OCP fp8 e4m3 (v_mfma_f32_16x16x32_fp8_fp8).
//
// This is the replacement for the conv/BiasAdd/FusedBatchNorm/Relu/MatMul kernels that the
// reference reaches through TF-Java on the CPU (InferenceBolt.java:81-85, libtensorflow Eigen).
//
// Orientation ("swapped" GEMM): D[channel][pixel] = W[channel][k] * X[k][pixel].
//   * A operand = packed weights, rows = output channels, staged once per workgroup in LDS
//     (row stride padded by 32 B (bf16) / 16 B (fp8): conflict-free fragment reads).
//   * B operand = implicit im2col of the NHWC input: lane l holds 8 consecutive k of pixel
//     (l & 15); with Cin % 8 == 0 those are 8 consecutive channels of ONE tap = one 16-B (bf16)
//     or 8-B (fp8) load.
//   * D layout: col = lane & 15 (pixel), row = 4*(lane >> 4) + r (channel), so each lane owns 4
//     consecutive channels of one pixel -> one 8-B (bf16) / 4-B (fp8) store per (pixel tile,
//     channel tile) and the bias / residual / ReLU epilogue is fused with vector loads.
// A workgroup is 4 waves; each wave owns PR x 16 pixels and all NT x 16 channels of its n-block,
// so every B fragment read from global/L1 feeds NT MFMAs and every A fragment feeds PR. PR is
// picked per launch so that small layers still put >= 4 workgroups on every CU. B fragments of
// U = 8/PR consecutive k-steps are loaded as one group and the next group is prefetched into
// registers while the current one feeds the MFMAs.
// When the whole packed weight block fits the LDS budget the workgroup stages it once and walks
// output tiles grid-stride (weight-stationary: ResNet-20 / LeNet layers); otherwise K is chunked.
//
// fp8 path (BASELINE config 5): weights are e4m3 with a per-output-channel scale (wscale), every
// activation tensor is e4m3 with a per-tensor scale calibrated offline (value = code * scale).
// The epilogue dequantises acc * wscale[c] * in_scale, adds bias and the (dequantised) residual,
// applies ReLU and requantises with 1/out_scale (saturating at +-448), so fp8 halves every
// activation byte moved; the network input stays fp32 and is quantised while it is loaded.
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

constexpr int kThreads = 256;
constexpr int kLdsBudget = 80 * 1024;  // 2 workgroups per CU by LDS

enum { MODE_FAST = 0, MODE_GATHER = 1, MODE_1X1 = 2 };

struct ConvArgs {
  const void* x;
  const void* w;
  const float* bias;
  const float* wscale;  // fp8: per-channel weight scale
  const void* res;
  void* y;
  int M;            // batch * Ho * Wo
  int H, W, Cin, Ho, Wo, HWo, Cout;
  int KW, stride, pad, K, Kpad;
  int cin_shift;    // log2(Cin) in MODE_FAST
  int kw_magic;     // ceil(65536 / KW)
  int relu;
  int has_res, res_H, res_W, res_C, res_stride;
  int BK;           // K chunk staged in LDS (multiple of 32)
  int nkc;          // number of K chunks
  int m_tiles;
  float in_scale;   // fp8: input dequant scale (in_f32: quantisation step of the input)
  float in_qinv;    // 1 / in_scale
  float out_qinv;   // fp8: 1 / out_scale
  float res_scale;  // fp8: residual dequant scale
};

// ---- element traits ----------------------------------------------------------------------
template <bool F8>
struct El;
template <>
struct El<false> {
  typedef bf16x8 frag;  // 8 k-values of one lane
  static constexpr int bytes = 2;
  static __device__ __forceinline__ frag zero() { return zero_bf16x8(); }
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct El<true> {
  typedef long frag;  // 8 e4m3 codes
  static constexpr int bytes = 1;
  static __device__ __forceinline__ frag zero() { return 0; }
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ float sat448(float v) { return fminf(fmaxf(v, -448.f), 448.f); }

// 4 floats -> 4 e4m3 codes (OCP, round to nearest even, saturated)
__device__ __forceinline__ uint32_t pack4_e4m3(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat448(a), sat448(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat448(c), sat448(d), w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ long f32x8_to_e4m3(const float* p, float q) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  const uint32_t lo = pack4_e4m3(a.x * q, a.y * q, a.z * q, a.w * q);
  const uint32_t hi = pack4_e4m3(b.x * q, b.y * q, b.z * q, b.w * q);
  return (long)(((uint64_t)hi << 32) | lo);
}

template <bool F8, bool IN_F32>
__device__ __forceinline__ typename El<F8>::frag load8(const ConvArgs& a, int off) {
  if constexpr (F8) {
    if constexpr (IN_F32) {
      return __builtin_bit_cast(typename El<F8>::frag,
                                f32x8_to_e4m3(reinterpret_cast<const float*>(a.x) + off, a.in_qinv));
    }
    return __builtin_bit_cast(typename El<F8>::frag,
                              *reinterpret_cast<const uint64_t*>(
                                  reinterpret_cast<const uint8_t*>(a.x) + off));
  } else {
    if constexpr (IN_F32)
      return __builtin_bit_cast(typename El<F8>::frag,
                                ld_f32x8_as_bf16(reinterpret_cast<const float*>(a.x) + off));
    return __builtin_bit_cast(typename El<F8>::frag,
                              ld_bf16x8(reinterpret_cast<const bf16*>(a.x) + off));
  }
}

// one element of the input as an operand code (gather mode)
template <bool F8, bool IN_F32>
__device__ __forceinline__ uint32_t load1(const ConvArgs& a, int off) {
  if constexpr (IN_F32) {
    const float v = reinterpret_cast<const float*>(a.x)[off];
    if constexpr (F8) return pack4_e4m3(v * a.in_qinv, 0.f, 0.f, 0.f) & 0xffu;
    return (uint32_t)__builtin_bit_cast(uint16_t, (bf16)v);
  }
  if (F8) return reinterpret_cast<const uint8_t*>(a.x)[off];
  return (uint32_t)__builtin_bit_cast(uint16_t, reinterpret_cast<const bf16*>(a.x)[off]);
}

template <int MODE, bool IN_F32, bool F8>
__device__ __forceinline__ typename El<F8>::frag load_b_frag(const ConvArgs& a, int k, bool ok,
                                                             int base, int h0, int w0) {
  typedef El<F8> E;
  if (MODE == MODE_1X1) {
    if (!ok || k >= a.K) return E::zero();
    return load8<F8, IN_F32>(a, base + k);
  } else if (MODE == MODE_FAST) {
    if (!ok || k >= a.K) return E::zero();
    const int tap = k >> a.cin_shift;
    const int ci = k & ((1 << a.cin_shift) - 1);
    const int kh = div_small(tap, a.kw_magic);
    const int kw = tap - kh * a.KW;
    const int hi = h0 + kh, wi = w0 + kw;
    if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) return E::zero();
    return load8<F8, IN_F32>(a, base + (hi * a.W + wi) * a.Cin + ci);
  } else {  // MODE_GATHER: any Cin (network stems with 1 or 3 input channels)
    uint32_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ok) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = k + j;
        if (kk < a.K) {
          const int tap = kk / a.Cin;
          const int ci = kk - tap * a.Cin;
          const int kh = div_small(tap, a.kw_magic);
          const int kw = tap - kh * a.KW;
          const int hi = h0 + kh, wi = w0 + kw;
          if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
            v[j] = load1<F8, IN_F32>(a, base + (hi * a.W + wi) * a.Cin + ci);
        }
      }
    }
    if constexpr (F8) {
      const uint64_t lo = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
      const uint64_t hi = v[4] | (v[5] << 8) | (v[6] << 16) | (v[7] << 24);
      return __builtin_bit_cast(typename E::frag, (long)((hi << 32) | lo));
    } else {
      const uint4 r = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16),
                                 v[6] | (v[7] << 16));
      return __builtin_bit_cast(typename E::frag, r);
    }
  }
}

template <int NT, int PR, int MODE, bool IN_F32, bool OUT_F32, bool F8>
__global__ __launch_bounds__(kThreads) void conv_mfma_kernel(ConvArgs a) {
  typedef El<F8> E;
  typedef typename E::frag frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint8_t* wl = reinterpret_cast<uint8_t*>(smem);
  constexpr int EB = E::bytes;
  constexpr int BN = NT * 16;
  constexpr int BM = 4 * PR * 16;
  // k-steps whose B fragments are loaded together: U*PR loads in flight per lane, and the next
  // group is fetched while the current one feeds the MFMAs (register double buffer), so a K loop
  // pays ~one memory latency per U steps instead of one per step.
  constexpr int U = 8 / PR;
  const int ldw = (a.BK + 16) * EB;  // LDS row stride in bytes
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4;      // k-group of the B fragment, channel quad of the D fragment
  const int col = lane & 15;    // pixel within a 16-pixel tile / weight row within a channel tile
  const int nb = blockIdx.y;

  auto stage = [&](int kc) {
    const int k0 = kc * a.BK;
    const int kl = min(a.BK, a.Kpad - k0);
    const int chunks = kl * EB / 16;  // 16-B pieces per row
    const uint8_t* src =
        reinterpret_cast<const uint8_t*>(a.w) + ((size_t)nb * BN * a.Kpad + k0) * EB;
    for (int i = threadIdx.x; i < BN * chunks; i += kThreads) {
      const int r = i / chunks, c = i - r * chunks;
      *reinterpret_cast<uint4*>(wl + r * ldw + c * 16) =
          *reinterpret_cast<const uint4*>(src + (size_t)r * a.Kpad * EB + c * 16);
    }
  };

  const bool resident = (a.nkc == 1);
  if (resident) {
    stage(0);
    __syncthreads();
  }

  for (int mt = blockIdx.x; mt < a.m_tiles; mt += gridDim.x) {
    // per pixel-tile coordinates of this lane's pixel (B operand column)
    int pbase[PR], ph0[PR], pw0[PR];
    bool pok[PR];
#pragma unroll
    for (int p = 0; p < PR; ++p) {
      const int m = mt * BM + wave * (PR * 16) + p * 16 + col;
      pok[p] = m < a.M;
      const int mm = pok[p] ? m : 0;
      const int n = mm / a.HWo;
      const int rem = mm - n * a.HWo;
      const int ho = rem / a.Wo;
      const int wo = rem - ho * a.Wo;
      if (MODE == MODE_1X1) {
        pbase[p] = ((n * a.H + ho * a.stride) * a.W + wo * a.stride) * a.Cin;
        ph0[p] = 0;
        pw0[p] = 0;
      } else {
        pbase[p] = n * a.H * a.W * a.Cin;
        ph0[p] = ho * a.stride - a.pad;
        pw0[p] = wo * a.stride - a.pad;
      }
    }

    f32x4 acc[PR][NT];
#pragma unroll
    for (int p = 0; p < PR; ++p)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[p][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kc = 0; kc < a.nkc; ++kc) {
      if (!resident) {
        __syncthreads();
        stage(kc);
        __syncthreads();
      }
      const int k0 = kc * a.BK;
      const int nks = min(a.BK, a.Kpad - k0) >> 5;
      const int ngrp = (nks + U - 1) / U;

      frag bcur[U][PR], bnxt[U][PR];
      auto load_grp = [&](int grp, frag (&dst)[U][PR]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int ks = grp * U + u;
#pragma unroll
          for (int p = 0; p < PR; ++p)
            dst[u][p] = load_b_frag<MODE, IN_F32, F8>(a, k0 + ks * 32 + g * 8,
                                                      pok[p] && ks < nks, pbase[p], ph0[p],
                                                      pw0[p]);
        }
      };
      load_grp(0, bcur);
      for (int grp = 0; grp < ngrp; ++grp) {
        if (grp + 1 < ngrp) load_grp(grp + 1, bnxt);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int ks = grp * U + u;
          if (ks < nks) {
            const int kl = ks * 32 + g * 8;  // k within the chunk for this lane's k-group
            frag afr[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t)
              afr[t] = *reinterpret_cast<const frag*>(wl + (t * 16 + col) * ldw + kl * EB);
#pragma unroll
            for (int p = 0; p < PR; ++p)
#pragma unroll
              for (int t = 0; t < NT; ++t) acc[p][t] = E::mma(afr[t], bcur[u][p], acc[p][t]);
          }
        }
        if (grp + 1 < ngrp) {
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int p = 0; p < PR; ++p) bcur[u][p] = bnxt[u][p];
        }
      }
    }

    // fused epilogue: (dequant) + bias (folded BN) + optional residual + optional ReLU
    // (+ requant), 4 channels per lane
#pragma unroll
    for (int p = 0; p < PR; ++p) {
      const int m = mt * BM + wave * (PR * 16) + p * 16 + col;
      if (m >= a.M) continue;
      int roff = 0;
      if (a.has_res) {
        const int n = m / a.HWo;
        const int rem = m - n * a.HWo;
        const int ho = rem / a.Wo;
        const int wo = rem - ho * a.Wo;
        roff = ((n * a.res_H + ho * a.res_stride) * a.res_W + wo * a.res_stride) * a.res_C;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c = nb * BN + t * 16 + g * 4;
        if (c >= a.Cout) continue;
        const float4 b = *reinterpret_cast<const float4*>(a.bias + c);
        float v0 = acc[p][t][0], v1 = acc[p][t][1], v2 = acc[p][t][2], v3 = acc[p][t][3];
        if (F8) {
          const float4 s = *reinterpret_cast<const float4*>(a.wscale + c);
          v0 *= s.x * a.in_scale; v1 *= s.y * a.in_scale;
          v2 *= s.z * a.in_scale; v3 *= s.w * a.in_scale;
        }
        v0 += b.x; v1 += b.y; v2 += b.z; v3 += b.w;
        if (a.has_res && c < a.res_C) {
          if (F8) {
            const int r = *reinterpret_cast<const int*>(
                reinterpret_cast<const uint8_t*>(a.res) + roff + c);
            v0 += __builtin_amdgcn_cvt_f32_fp8(r, 0) * a.res_scale;
            v1 += __builtin_amdgcn_cvt_f32_fp8(r, 1) * a.res_scale;
            v2 += __builtin_amdgcn_cvt_f32_fp8(r, 2) * a.res_scale;
            v3 += __builtin_amdgcn_cvt_f32_fp8(r, 3) * a.res_scale;
          } else {
            const bf16x4 r = __builtin_bit_cast(
                bf16x4, *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(a.res) +
                                                        roff + c));
            v0 += (float)r[0]; v1 += (float)r[1]; v2 += (float)r[2]; v3 += (float)r[3];
          }
        }
        if (a.relu) {
          v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
        }
        if (OUT_F32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.y) + (size_t)m * a.Cout + c) =
              make_float4(v0, v1, v2, v3);
        } else if (F8) {
          *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.y) + (size_t)m * a.Cout + c) =
              pack4_e4m3(v0 * a.out_qinv, v1 * a.out_qinv, v2 * a.out_qinv, v3 * a.out_qinv);
        } else {
          bf16x4 o;
          o[0] = (bf16)v0; o[1] = (bf16)v1; o[2] = (bf16)v2; o[3] = (bf16)v3;
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(a.y) + (size_t)m * a.Cout + c) =
              __builtin_bit_cast(uint2, o);
        }
      }
    }
  }
}

typedef void (*ConvKernelFn)(ConvArgs);

template <int NT, int MODE, bool IN_F32, bool OUT_F32, bool F8>
ConvKernelFn pick_pr(int pr) {
  switch (pr) {
    case 1: return conv_mfma_kernel<NT, 1, MODE, IN_F32, OUT_F32, F8>;
    case 2: return conv_mfma_kernel<NT, 2, MODE, IN_F32, OUT_F32, F8>;
    default: return conv_mfma_kernel<NT, (NT >= 8 ? 2 : 4), MODE, IN_F32, OUT_F32, F8>;
  }
}

template <int MODE, bool IN_F32, bool OUT_F32, bool F8>
ConvKernelFn pick_nt(int nt, int pr) {
  switch (nt) {
    case 1: return pick_pr<1, MODE, IN_F32, OUT_F32, F8>(pr);
    case 2: return pick_pr<2, MODE, IN_F32, OUT_F32, F8>(pr);
    case 4: return pick_pr<4, MODE, IN_F32, OUT_F32, F8>(pr);
    default: return pick_pr<8, MODE, IN_F32, OUT_F32, F8>(pr);
  }
}

template <bool F8>
ConvKernelFn pick_kernel(int mode, bool in_f32, bool out_f32, int nt, int pr) {
  if (mode == MODE_1X1) {
    if (in_f32) return out_f32 ? pick_nt<MODE_1X1, true, true, F8>(nt, pr)
                               : pick_nt<MODE_1X1, true, false, F8>(nt, pr);
    return out_f32 ? pick_nt<MODE_1X1, false, true, F8>(nt, pr)
                   : pick_nt<MODE_1X1, false, false, F8>(nt, pr);
  }
  if (mode == MODE_FAST)
    return in_f32 ? pick_nt<MODE_FAST, true, false, F8>(nt, pr)
                  : pick_nt<MODE_FAST, false, false, F8>(nt, pr);
  return in_f32 ? pick_nt<MODE_GATHER, true, false, F8>(nt, pr)
                : pick_nt<MODE_GATHER, false, false, F8>(nt, pr);
}

int ilog2_exact(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return ((1 << s) == v) ? s : -1;
}

}  // namespace

int conv_n_tiles(int Cout) {
  // channel tiles per workgroup n-block: whole Cout for the small-channel CNNs, 128 otherwise
  if (Cout <= 16) return 1;
  if (Cout <= 32) return 2;
  if (Cout <= 64) return 4;
  return 8;
}

hipError_t conv2d(const ConvDesc& d, int batch, const void* x, const void* w, const float* bias,
                  const float* wscale, const void* res, void* y, hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (d.f32) return conv2d_f32(d, batch, x, w, bias, d.has_res ? res : nullptr, y, stream);
  const bool f8 = d.fp8 != 0;
  if (d.stem) {
    if (f8 || d.in_f32 || d.out_f32 || d.Cin != 4 || d.KH != 8 || d.KW != 8 || d.K != 256 ||
        d.Kpad != 256 || d.stride != 2 || d.pad != 3 || d.W != 2 * d.Wo + 6 ||
        d.Cout % 64 != 0 || d.Npad % 64 != 0 || (d.has_res && res != nullptr))
      return hipErrorInvalidValue;
    return conv2d_gemm(d, batch, x, w, bias, nullptr, y, stream);
  }
  if (!f8 && conv_patch_supported(d, batch, d.has_res && res != nullptr))
    return conv2d_patch(d, batch, x, w, bias, d.has_res ? res : nullptr, y, stream);
  if (!f8 && conv_gemm_supported(d, batch, d.has_res && res != nullptr))
    return conv2d_gemm(d, batch, x, w, bias, d.has_res ? res : nullptr, y, stream);
  if (f8 && (wscale == nullptr || !(d.in_scale > 0.f) || !(d.out_scale > 0.f)))
    return hipErrorInvalidValue;
  ConvArgs a;
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.wscale = wscale;
  a.res = res;
  a.y = y;
  a.M = batch * d.Ho * d.Wo;
  a.H = d.H; a.W = d.W; a.Cin = d.Cin; a.Ho = d.Ho; a.Wo = d.Wo; a.HWo = d.Ho * d.Wo;
  a.Cout = d.Cout; a.KW = d.KW; a.stride = d.stride; a.pad = d.pad; a.K = d.K; a.Kpad = d.Kpad;
  a.kw_magic = (65536 + d.KW - 1) / d.KW;
  a.relu = d.relu;
  a.has_res = d.has_res && res != nullptr;
  a.res_H = d.res_H; a.res_W = d.res_W; a.res_C = d.res_C; a.res_stride = d.res_stride;
  a.in_scale = f8 ? d.in_scale : 1.f;
  a.in_qinv = f8 ? 1.f / d.in_scale : 1.f;
  a.out_qinv = f8 ? 1.f / d.out_scale : 1.f;
  a.res_scale = f8 ? d.res_scale : 1.f;

  int mode;
  const int cs = ilog2_exact(d.Cin);
  if (d.KH == 1 && d.KW == 1 && d.pad == 0 && d.Cin % 8 == 0) mode = MODE_1X1;
  else if (d.Cin % 8 == 0 && cs >= 0) mode = MODE_FAST;
  else mode = MODE_GATHER;
  a.cin_shift = cs < 0 ? 0 : cs;
  if (d.out_f32 && mode != MODE_1X1) return hipErrorInvalidValue;
  if (d.Cout % 4 != 0 || d.Kpad % 32 != 0) return hipErrorInvalidValue;

  const int nt = conv_n_tiles(d.Cout);
  const int BN = nt * 16;
  if (d.Npad % BN != 0) return hipErrorInvalidValue;
  const int n_blocks = (d.Cout + BN - 1) / BN;
  // pixel tiles per wave: the largest of {4 (2 for 8 channel tiles), 2, 1} that still gives the
  // chip >= 4 workgroups per CU; small layers (late stages, small batches) trade B-fragment reuse
  // for occupancy, which is what bounds them
  const int pr_max = (nt >= 8) ? 2 : 4;
  int PR = pr_max;
  while (PR > 1 && (long long)((a.M + 64 * PR - 1) / (64 * PR)) * n_blocks < 1024) PR >>= 1;
  const int BM = 4 * PR * 16;

  // K chunk: whole K if it fits the LDS budget (weight-stationary), else the largest multiple of
  // 32 that does.
  const int eb = f8 ? 1 : 2;
  int bk = d.Kpad;
  if ((size_t)BN * (bk + 16) * eb > (size_t)kLdsBudget) {
    bk = (kLdsBudget / (BN * eb) - 16) & ~31;
    if (bk < 32) return hipErrorInvalidValue;
  }
  a.BK = bk;
  a.nkc = (d.Kpad + bk - 1) / bk;
  a.m_tiles = (a.M + BM - 1) / BM;
  const size_t lds = (size_t)BN * (bk + 16) * eb;

  int grid_m = a.m_tiles;
  if (a.nkc == 1) {
    // weight-stationary: enough workgroups to fill 256 CUs x 8, each walks several tiles
    const int cap = 2048 / n_blocks > 0 ? 2048 / n_blocks : 1;
    grid_m = a.m_tiles < cap ? a.m_tiles : cap;
  }

  const ConvKernelFn fn = f8 ? pick_kernel<true>(mode, d.in_f32, d.out_f32, nt, PR)
                             : pick_kernel<false>(mode, d.in_f32, d.out_f32, nt, PR);
  hipLaunchKernelGGL(fn, dim3(grid_m, n_blocks), dim3(kThreads), lds, stream, a);
  return hipGetLastError();
}

}  // namespace gale
