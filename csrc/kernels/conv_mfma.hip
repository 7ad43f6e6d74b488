// Implicit-GEMM convolution on CDNA4 matrix cores (v_mfma_f32_16x16x32_bf16), NHWC, bf16.
//
// This is the replacement for the conv/BiasAdd/FusedBatchNorm/Relu/MatMul kernels that the
// reference reaches through TF-Java on the CPU (InferenceBolt.java:81-85, libtensorflow Eigen).
//
// Orientation ("swapped" GEMM): D[channel][pixel] = W[channel][k] * X[k][pixel].
//   * A operand = packed weights, rows = output channels, staged once per workgroup in LDS
//     (row stride padded by 32 B: conflict-free ds_read_b128 for the 4 x 16-lane groups).
//   * B operand = implicit im2col of the NHWC input: lane l holds 8 consecutive k of pixel
//     (l & 15); with Cin % 8 == 0 those are 8 consecutive channels of ONE tap = one 16-B load.
//   * D layout: col = lane & 15 (pixel), row = 4*(lane >> 4) + r (channel), so each lane owns 4
//     consecutive channels of one pixel -> one 8-B store per (pixel tile, channel tile) and the
//     bias / residual / ReLU epilogue is fused with vector loads.
// A workgroup is 4 waves; each wave owns PR x 16 pixels and all NT x 16 channels of its n-block,
// so every B fragment read from global/L1 feeds NT MFMAs and every A fragment feeds PR.
// When the whole packed weight block fits the LDS budget the workgroup stages it once and walks
// output tiles grid-stride (weight-stationary: ResNet-20 / LeNet layers); otherwise K is chunked.
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

constexpr int kThreads = 256;
constexpr int kLdsBudget = 64 * 1024;  // 2 workgroups per CU by LDS

enum { MODE_FAST = 0, MODE_GATHER = 1, MODE_1X1 = 2 };

struct ConvArgs {
  const void* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
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
};

template <int MODE, bool IN_F32>
__device__ __forceinline__ bf16x8 load_b_frag(const ConvArgs& a, int k, bool ok, int base, int h0,
                                              int w0) {
  if (MODE == MODE_1X1) {
    if (!ok || k >= a.K) return zero_bf16x8();
    if (IN_F32) return ld_f32x8_as_bf16(reinterpret_cast<const float*>(a.x) + base + k);
    return ld_bf16x8(reinterpret_cast<const bf16*>(a.x) + base + k);
  } else if (MODE == MODE_FAST) {
    if (!ok || k >= a.K) return zero_bf16x8();
    const int tap = k >> a.cin_shift;
    const int ci = k & ((1 << a.cin_shift) - 1);
    const int kh = div_small(tap, a.kw_magic);
    const int kw = tap - kh * a.KW;
    const int hi = h0 + kh, wi = w0 + kw;
    if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) return zero_bf16x8();
    const int off = base + (hi * a.W + wi) * a.Cin + ci;
    if (IN_F32) return ld_f32x8_as_bf16(reinterpret_cast<const float*>(a.x) + off);
    return ld_bf16x8(reinterpret_cast<const bf16*>(a.x) + off);
  } else {  // MODE_GATHER: any Cin (network stems with 1 or 3 input channels)
    bf16x8 r = zero_bf16x8();
    if (!ok) return r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = k + j;
      if (kk < a.K) {
        const int tap = kk / a.Cin;
        const int ci = kk - tap * a.Cin;
        const int kh = div_small(tap, a.kw_magic);
        const int kw = tap - kh * a.KW;
        const int hi = h0 + kh, wi = w0 + kw;
        if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W) {
          const int off = base + (hi * a.W + wi) * a.Cin + ci;
          r[j] = IN_F32 ? (bf16)(reinterpret_cast<const float*>(a.x)[off])
                        : reinterpret_cast<const bf16*>(a.x)[off];
        }
      }
    }
    return r;
  }
}

template <int NT, int PR, int MODE, bool IN_F32, bool OUT_F32>
__global__ __launch_bounds__(kThreads) void conv_mfma_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* wl = reinterpret_cast<bf16*>(smem);
  constexpr int BN = NT * 16;
  constexpr int BM = 4 * PR * 16;
  const int ldw = a.BK + 16;  // +32 B per row: conflict-free ds_read_b128 (see file header)
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4;      // k-group of the B fragment, channel quad of the D fragment
  const int col = lane & 15;    // pixel within a 16-pixel tile / weight row within a channel tile
  const int nb = blockIdx.y;

  auto stage = [&](int kc) {
    const int k0 = kc * a.BK;
    const int kl = min(a.BK, a.Kpad - k0);
    const int chunks = kl >> 3;  // 16-B pieces per row
    const bf16* src = a.w + (size_t)nb * BN * a.Kpad + k0;
    for (int i = threadIdx.x; i < BN * chunks; i += kThreads) {
      const int r = i / chunks, c = i - r * chunks;
      *reinterpret_cast<uint4*>(wl + r * ldw + c * 8) =
          *reinterpret_cast<const uint4*>(src + (size_t)r * a.Kpad + c * 8);
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

      for (int ks = 0; ks < nks; ++ks) {
        const int kl = ks * 32 + g * 8;  // k within the chunk for this lane's k-group
        bf16x8 bfr[PR];
#pragma unroll
        for (int p = 0; p < PR; ++p)
          bfr[p] = load_b_frag<MODE, IN_F32>(a, k0 + kl, pok[p], pbase[p], ph0[p], pw0[p]);
        bf16x8 afr[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          afr[t] = *reinterpret_cast<const bf16x8*>(wl + (t * 16 + col) * ldw + kl);
#pragma unroll
        for (int p = 0; p < PR; ++p)
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[p][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[t], bfr[p], acc[p][t], 0, 0, 0);
      }
    }

    // fused epilogue: bias (folded BN) + optional residual + optional ReLU, 4 channels per lane
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
        float v0 = acc[p][t][0] + b.x, v1 = acc[p][t][1] + b.y;
        float v2 = acc[p][t][2] + b.z, v3 = acc[p][t][3] + b.w;
        if (a.has_res && c < a.res_C) {
          const bf16x4 r = __builtin_bit_cast(
              bf16x4, *reinterpret_cast<const uint2*>(a.res + roff + c));
          v0 += (float)r[0]; v1 += (float)r[1]; v2 += (float)r[2]; v3 += (float)r[3];
        }
        if (a.relu) {
          v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
        }
        if (OUT_F32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.y) + (size_t)m * a.Cout + c) =
              make_float4(v0, v1, v2, v3);
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

template <int NT, int MODE, bool IN_F32, bool OUT_F32>
ConvKernelFn pick_pr() {
  constexpr int PR = (NT >= 8) ? 2 : 4;
  return conv_mfma_kernel<NT, PR, MODE, IN_F32, OUT_F32>;
}

template <int MODE, bool IN_F32, bool OUT_F32>
ConvKernelFn pick_nt(int nt) {
  switch (nt) {
    case 1: return pick_pr<1, MODE, IN_F32, OUT_F32>();
    case 2: return pick_pr<2, MODE, IN_F32, OUT_F32>();
    case 4: return pick_pr<4, MODE, IN_F32, OUT_F32>();
    default: return pick_pr<8, MODE, IN_F32, OUT_F32>();
  }
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
  (void)wscale;
  if (batch <= 0) return hipSuccess;
  if (d.fp8) return hipErrorNotSupported;  // fp8 convs are routed to conv2d_fp8 by the executor
  ConvArgs a;
  a.x = x;
  a.w = reinterpret_cast<const bf16*>(w);
  a.bias = bias;
  a.res = reinterpret_cast<const bf16*>(res);
  a.y = y;
  a.M = batch * d.Ho * d.Wo;
  a.H = d.H; a.W = d.W; a.Cin = d.Cin; a.Ho = d.Ho; a.Wo = d.Wo; a.HWo = d.Ho * d.Wo;
  a.Cout = d.Cout; a.KW = d.KW; a.stride = d.stride; a.pad = d.pad; a.K = d.K; a.Kpad = d.Kpad;
  a.kw_magic = (65536 + d.KW - 1) / d.KW;
  a.relu = d.relu;
  a.has_res = d.has_res && res != nullptr;
  a.res_H = d.res_H; a.res_W = d.res_W; a.res_C = d.res_C; a.res_stride = d.res_stride;

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
  const int PR = (nt >= 8) ? 2 : 4;
  const int BM = 4 * PR * 16;
  if (d.Npad % BN != 0) return hipErrorInvalidValue;
  const int n_blocks = (d.Cout + BN - 1) / BN;

  // K chunk: whole K if it fits the LDS budget (weight-stationary), else the largest multiple of
  // 32 that does.
  int bk = d.Kpad;
  if ((size_t)BN * (bk + 16) * 2 > (size_t)kLdsBudget) {
    bk = (kLdsBudget / (BN * 2) - 16) & ~31;
    if (bk < 32) return hipErrorInvalidValue;
  }
  a.BK = bk;
  a.nkc = (d.Kpad + bk - 1) / bk;
  a.m_tiles = (a.M + BM - 1) / BM;
  const size_t lds = (size_t)BN * (bk + 16) * 2;

  int grid_m = a.m_tiles;
  if (a.nkc == 1) {
    // weight-stationary: enough workgroups to fill 256 CUs x 2, each walks several tiles
    const int cap = 1024 / n_blocks > 0 ? 1024 / n_blocks : 1;
    grid_m = a.m_tiles < cap ? a.m_tiles : cap;
  }

  ConvKernelFn fn;
  if (mode == MODE_1X1) {
    if (d.in_f32) fn = d.out_f32 ? pick_nt<MODE_1X1, true, true>(nt) : pick_nt<MODE_1X1, true, false>(nt);
    else fn = d.out_f32 ? pick_nt<MODE_1X1, false, true>(nt) : pick_nt<MODE_1X1, false, false>(nt);
  } else if (mode == MODE_FAST) {
    fn = d.in_f32 ? pick_nt<MODE_FAST, true, false>(nt) : pick_nt<MODE_FAST, false, false>(nt);
  } else {
    fn = d.in_f32 ? pick_nt<MODE_GATHER, true, false>(nt) : pick_nt<MODE_GATHER, false, false>(nt);
  }
  hipLaunchKernelGGL(fn, dim3(grid_m, n_blocks), dim3(kThreads), lds, stream, a);
  return hipGetLastError();
}

}  // namespace gale
