// LDS-pipelined implicit-GEMM convolution for the wide layers (Cin % 64 == 0, bf16): the
// ResNet-50 body (BASELINE config 4). conv_mfma.hip keeps the small-channel / odd-shaped layers.
//
// GEMM view (NHWC, swapped so every lane owns 4 consecutive output channels of one pixel):
//   D[channel n][pixel m] = sum_k W[n][k] * X[m][k],  k = (kh*KW + kw)*Cin + ci
// Both operands are K-contiguous rows, so one workgroup tile step stages
//   * BM pixel rows x 64 k  (the im2col rows of one tap (kh, kw) and 64 input channels: one
//     contiguous 128-B run of the NHWC input per pixel, or zeros for a padding tap), and
//   * BN weight rows x 64 k,
// with global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip): 8 lanes per 128-B row, one
// wave-instruction = 8 rows = 1 KiB of LDS. The LDS image is lane-linear, so the bank swizzle is
// applied on the SOURCE side (cdna_hip_programming.md §5.4 rule 21): LDS slot s of row r holds the
// global 16-B chunk s ^ ((r >> 1) & 7), and fragment reads apply the same involution; 16 lanes
// reading 16 consecutive rows at one chunk then hit 16 distinct 4-bank groups (conflict-free).
// Padding taps and rows past M point their source at a zero block.
// Pipeline: two LDS stages, one barrier per 64-deep k-step; the DMA of step k+1 is issued right
// after the barrier and lands while the MFMAs of step k run (v_mfma_f32_16x16x32_bf16, each wave
// owning a (BN/2) x 64 sub-tile = TN x TM 16x16 accumulators).
// Epilogue: folded-BN bias + identity residual + ReLU, bf16 NHWC, staged through LDS so the
// residual loads and output stores are 16-byte, whole-row accesses.
// Grid: one workgroup per (pixel tile, channel tile), remapped so the tiles of one XCD are
// contiguous (T1): the channel tiles of a pixel tile, which re-read the same im2col rows, share an L2.
#include <stdlib.h>

#include <atomic>

#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

__device__ __attribute__((aligned(16))) uint8_t g_zero_rows[64];  // source of padding rows

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gbl_u32x4_t;  // global_load, not flat
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;

struct GemmConvArgs {
  const bf16* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
  void* y;         // bf16 NHWC, or fp32 when out_f32 (classifier logits)
  int M, H, W, Cin, HWo, Wo, Cout, KW, stride, pad, Kpad;
  int nkb;         // 64-deep k-steps = KH*KW*Cin / 64
  int cin_blocks;  // Cin / 64
  int relu, has_res, out_f32;
  int n_tiles, nwg;
  // DUAL (conv2d_gemm_proj): k-steps [nkb1, nkb) read a second 1x1 source - the bottleneck's
  // projection shortcut, x2 [B][H2][W2][Cin2] sampled at stride2, weights w2 [Npad][Kpad2] - so
  // conv3 + projection is one GEMM over the concatenated K, with bias + bias2. Rounding: the
  // projection term stays fp32 inside the accumulator (one bf16 rounding of the sum), while the
  // layered plan (GALE_FUSE_PROJ=0) and bottleneck56's block 0 store the projection as bf16
  // first: the two forms differ by up to one bf16 ulp of the shortcut before the final rounding
  // (tests/test_models_gpu.py pins the fused plan against the fp32 oracle and the
  // layered one). Rounding it here too would need a second accumulator set per tile.
  const bf16* x2;
  const bf16* w2;
  const float* bias2;
  int H2, W2, Cin2, stride2, Kpad2, nkb1;
};

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src), (lds_ptr_t)(lds_base), 16, 0, 0);
}

// STEM: the packed-stem layout (ConvDesc::stem): k-step kb covers kernel rows 2kb and 2kb+1, a
// lane's 16-B chunk c reads row kh = 2kb + (c >> 2), bytes 16*(c & 3) of the 64-B run that
// starts at column 2*wo of the padded image (columns never leave it, rows may: zero rows).
// NST: LDS stages. 2 = double-buffered k-loop; 1 = the single-k-step (K = 64: the 1x1 convs
// on 64 input channels) form, which needs no second stage and so fits 4 workgroups per CU
// instead of 2 - these layers are bound by their epilogue traffic (a 128 x 128 bf16 output tile
// plus the residual per 16 KB of input), which more resident workgroups overlap.
// (Variants measured and removed in round 3 - 256 x 128 tiles with 8 waves, a three-stage
// 128 x 64 ring, register staging instead of LDS-DMA, the single-stage form for 2-4 k-steps: all
// slower at ResNet-50 batch 256, profiles/archive/r2_resnet50_gemm_ab.txt.)
template <int BM, int BN, bool STEM, int NST, bool DUAL = false>
__global__ __launch_bounds__(256, NST == 1 ? 4 : 2)
void conv_gemm_kernel(GemmConvArgs a) {
  constexpr int WM = BM / 64;                   // waves as WM (pixels) x 2 (channels)
  constexpr int WN = 2;
  constexpr int NW = WM * WN;                   // waves per workgroup
  constexpr int TM = BM / WM / 16;              // 16-pixel tiles per wave
  constexpr int TN = BN / WN / 16;              // 16-channel tiles per wave
  constexpr int XI = BM / (8 * NW);             // X wave-instructions (8 rows each) per wave
  constexpr int WI = BN / (8 * NW);             // W wave-instructions per wave
  static_assert(XI >= 1 && WI >= 1, "tile too small for the workgroup");
  constexpr int STAGE = (BM + BN) * 128;        // bytes per LDS stage
  constexpr int EPI = NW * (TM / 2 * 16) * (BN / WN + 4) * 4;  // epilogue staging bytes
  constexpr int LDS_BYTES = NST * STAGE > EPI ? NST * STAGE : EPI;
  __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-contiguous tile order (bijective for any nwg)
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = a.nwg >> 3, r8 = a.nwg & 7;
  const int rid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int mt = rid / a.n_tiles, nt = rid - mt * a.n_tiles;

  // ---- per-lane staging sources ----
  const int srow = lane >> 3;                   // row within a wave-instruction's 8 rows
  const int slot = lane & 7;
  int xoff[XI], xh[XI], xw[XI];
#pragma unroll
  for (int j = 0; j < XI; ++j) {
    const int row = (wave * XI + j) * 8 + srow;
    const int m = mt * BM + row;
    const int chunk = slot ^ ((row >> 1) & 7);
    if (m < a.M) {
      const int n = m / a.HWo;
      const int rem = m - n * a.HWo;
      const int ho = rem / a.Wo;
      const int wo = rem - ho * a.Wo;
      if (STEM) {
        xoff[j] = n * a.H * a.W * 4 + wo * 8 + (chunk & 3) * 8;
        xh[j] = ho * 2 - a.pad + (chunk >> 2);
        xw[j] = 0;
      } else {
        xoff[j] = n * a.H * a.W * a.Cin + chunk * 8;
        xh[j] = ho * a.stride - a.pad;
        xw[j] = wo * a.stride - a.pad;
      }
    } else {
      xoff[j] = 0;
      xh[j] = -(1 << 20);  // every tap out of bounds -> zero rows
      xw[j] = 0;
    }
  }
  const bf16* wsrc[WI];
#pragma unroll
  for (int j = 0; j < WI; ++j) {
    const int row = (wave * WI + j) * 8 + srow;
    const int chunk = slot ^ ((row >> 1) & 7);
    wsrc[j] = a.w + (size_t)(nt * BN + row) * a.Kpad + chunk * 8;
  }
  // DUAL: the second source's row of each staged output pixel (or -1 past M) and weight rows
  int xoff2[DUAL ? XI : 1];
  const bf16* wsrc2[DUAL ? WI : 1];
  if (DUAL) {
#pragma unroll
    for (int j = 0; j < XI; ++j) {
      const int row = (wave * XI + j) * 8 + srow;
      const int m = mt * BM + row;
      const int chunk = slot ^ ((row >> 1) & 7);
      xoff2[j] = -1;
      if (m < a.M) {
        const int n = m / a.HWo;
        const int rem = m - n * a.HWo;
        const int ho = rem / a.Wo;
        const int wo = rem - ho * a.Wo;
        xoff2[j] = ((n * a.H2 + ho * a.stride2) * a.W2 + wo * a.stride2) * a.Cin2 + chunk * 8;
      }
    }
#pragma unroll
    for (int j = 0; j < WI; ++j) {
      const int row = (wave * WI + j) * 8 + srow;
      const int chunk = slot ^ ((row >> 1) & 7);
      wsrc2[j] = a.w2 + (size_t)(nt * BN + row) * a.Kpad2 + chunk * 8;
    }
  }

  // source of im2col piece j (8 rows x 128 B per wave-instruction) of k-step kb
  auto xsrc = [&](int kb, int j) __attribute__((always_inline)) -> const void* {
    if (DUAL && kb >= a.nkb1)
      return xoff2[j] >= 0 ? (const void*)(a.x2 + xoff2[j] + (kb - a.nkb1) * 64)
                           : (const void*)(g_zero_rows + 16 * (lane & 3));
    if (STEM) {
      const int hi = xh[j] + 2 * kb;
      return (unsigned)hi < (unsigned)a.H ? (const void*)(a.x + xoff[j] + hi * a.W * 4)
                                          : (const void*)(g_zero_rows + 16 * (lane & 3));
    }
    const int tap = kb / a.cin_blocks;
    const int cb = kb - tap * a.cin_blocks;
    const int kh = tap / a.KW;
    const int kw = tap - kh * a.KW;
    const int hi = xh[j] + kh, wi = xw[j] + kw;
    const bool ok = (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
    return ok ? (const void*)(a.x + xoff[j] + (hi * a.W + wi) * a.Cin + cb * 64)
              : (const void*)(g_zero_rows + 16 * (lane & 3));
  };
  // LDS-DMA staging: global -> LDS without VGPRs, lane-linear 1 KiB per wave-instruction
  auto stage = [&](int kb, uint8_t* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < XI; ++j) glds16(xsrc(kb, j), buf + (wave * XI + j) * 1024);
#pragma unroll
    for (int j = 0; j < WI; ++j)
      glds16(DUAL && kb >= a.nkb1 ? wsrc2[j] + (kb - a.nkb1) * 64 : wsrc[j] + kb * 64,
             buf + BM * 128 + (wave * WI + j) * 1024);
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (row part; the chunk part depends on the k-step)
  const int fr = lane & 15, fq = lane >> 4;
  int xrow_off[TM], wrow_off[TN], xsw[TM], wsw[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = wm * (BM / WM) + i * 16 + fr;
    xrow_off[i] = row * 128;
    xsw[i] = (row >> 1) & 7;
  }
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int row = wn * (BN / WN) + t * 16 + fr;
    wrow_off[t] = BM * 128 + row * 128;
    wsw[t] = (row >> 1) & 7;
  }

  // epilogue geometry (see below) and the residual prefetch: the residual rows this lane will
  // add are loaded into registers while the last k-step's MFMAs run, so their DRAM latency is
  // hidden instead of stalling the epilogue (the 1x1 expansion convs with a shortcut were
  // latency-bound at ~3 TB/s, profiles/archive/r2_resnet50_layers_pmc.txt)
  constexpr bool PREF = NST >= 2;
  constexpr int CW = BN / WN;      // channels per wave
  constexpr int EPS = CW + 4;      // fp32 row stride (+16 B: conflict-free 16-row writes)
  constexpr int LPR = CW / 8;      // lanes per pixel row on read-back
  constexpr int RPI = 64 / LPR;    // pixel rows per read-back instruction
  constexpr int HALF = TM / 2 * 16;  // pixel rows per half
  constexpr int NRI = HALF / RPI;  // read-back instructions per half
  const int c0 = nt * BN + wn * CW;
  const int mbase = mt * BM + wm * (BM / WM);
  const int cc = (lane % LPR) * 8;
  bf16x8 rpre[2][NRI];
  auto prefetch_res = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < NRI; ++j) {
        const int m = mbase + h * HALF + j * RPI + lane / LPR;
        if (m < a.M && c0 + cc < a.Cout)
          rpre[h][j] = ld_bf16x8(a.res + (size_t)m * a.Cout + c0 + cc);
      }
  };

  stage(0, lds);
  for (int kb = 0; kb < a.nkb; ++kb) {
    uint8_t* cur;
    if (NST == 1) {
      // single stage, serial: refill only after every wave is done with step kb-1 (the
      // overlap comes from the other resident workgroups of the CU)
      if (kb > 0) {
        __syncthreads();
        stage(kb, lds);
      }
      __syncthreads();  // step kb has landed
      cur = lds;
    } else {
      __syncthreads();  // step kb has landed (vmcnt(0)); every wave is done reading step kb-1
      cur = lds + (kb & 1) * STAGE;
      if (kb + 1 < a.nkb) stage(kb + 1, lds + ((kb + 1) & 1) * STAGE);
    }
    if (PREF && kb + 1 == a.nkb && a.has_res) prefetch_res();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fq;
      bf16x8 af[TN], bfr[TM];
#pragma unroll
      for (int t = 0; t < TN; ++t)
        af[t] = *reinterpret_cast<const bf16x8*>(cur + wrow_off[t] + ((chunk ^ wsw[t]) << 4));
#pragma unroll
      for (int i = 0; i < TM; ++i)
        bfr[i] = *reinterpret_cast<const bf16x8*>(cur + xrow_off[i] + ((chunk ^ xsw[i]) << 4));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < TN; ++t)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bfr[i], acc[i][t], 0, 0, 0);
    }
  }

  // ---- epilogue through LDS: full-line global traffic ----
  // A lane's accumulators hold 4 channels of one pixel (8-byte pieces of 16 pixel rows per
  // store); instead each wave writes (acc + bias) as fp32 into its own LDS region, pixel-major,
  // and reads back 8 consecutive channels per lane, so every residual load and output store is
  // a 16-byte access and a wave instruction covers whole 128-byte rows. fp32 in LDS keeps the
  // rounding identical to the register epilogue (one bf16 rounding after the residual/ReLU).
  // Two halves of TM/2 pixel tiles each fit the 2-stage LDS allocation.
  static_assert(NW * HALF * EPS * 4 <= LDS_BYTES, "epilogue staging exceeds the LDS allocation");
  __syncthreads();  // every wave is done with the last k-stage
  float* ep = reinterpret_cast<float*>(lds) + wave * HALF * EPS;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int cl = t * 16 + fq * 4;
      float4 b = *reinterpret_cast<const float4*>(a.bias + c0 + cl);
      if (DUAL) {
        const float4 b2 = *reinterpret_cast<const float4*>(a.bias2 + c0 + cl);
        b = make_float4(b.x + b2.x, b.y + b2.y, b.z + b2.z, b.w + b2.w);
      }
#pragma unroll
      for (int ii = 0; ii < TM / 2; ++ii) {
        const int i = h * (TM / 2) + ii;
        *reinterpret_cast<float4*>(ep + (ii * 16 + fr) * EPS + cl) =
            make_float4(acc[i][t][0] + b.x, acc[i][t][1] + b.y, acc[i][t][2] + b.z,
                        acc[i][t][3] + b.w);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (wave-private region)
#pragma unroll
    for (int j = 0; j < NRI; ++j) {
      const int r0 = j * RPI;
      const int p = r0 + lane / LPR;
      const int m = mbase + h * HALF + p;
      if (m < a.M && c0 + cc < a.Cout) {  // (Cout % 8 == 0; channels >= Cout are padding)
        const float* src = ep + p * EPS + cc;
        const float4 lo = *reinterpret_cast<const float4*>(src);
        const float4 hi = *reinterpret_cast<const float4*>(src + 4);
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const size_t o = (size_t)m * a.Cout + c0 + cc;
        if (a.has_res) {
          const bf16x8 rr = PREF ? rpre[h][j] : ld_bf16x8(a.res + o);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)rr[e];
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (a.out_f32) {  // classifier logits stay fp32 (the softmax op follows)
          float4* yo = reinterpret_cast<float4*>(static_cast<float*>(a.y) + o);
          yo[0] = make_float4(v[0], v[1], v[2], v[3]);
          yo[1] = make_float4(v[4], v[5], v[6], v[7]);
        } else {
          bf16x8 ov;
#pragma unroll
          for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
          *reinterpret_cast<uint4*>(static_cast<bf16*>(a.y) + o) = __builtin_bit_cast(uint4, ov);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next half
  }
}

}  // namespace

// 0 auto, 1 never the GEMM path, 2 GEMM path whenever the shape allows (tests / A-B benches)
static std::atomic<int> g_conv_path{0};
void set_conv_path(int mode) { g_conv_path = mode; }
int conv_path() { return g_conv_path; }

bool conv_gemm_supported(const ConvDesc& d, int batch, bool has_res) {
  if (g_conv_path == 1) return false;
  if (d.fp8 || d.in_f32 || d.f32) return false;
  if (d.Cin % 64 != 0 || d.Cout % 8 != 0 || d.K != d.KH * d.KW * d.Cin || d.Kpad != d.K)
    return false;
  // channel tiles cover Npad (zero weight rows past Cout; the epilogue stores c < Cout only)
  const int bn = (d.Npad % 128 == 0) ? 128 : 64;
  if (d.Npad % bn != 0 || d.Npad < d.Cout) return false;
  if (has_res && (d.res_C != d.Cout || d.res_stride != 1 || d.res_H != d.Ho || d.res_W != d.Wo))
    return false;
  // 32-bit element offsets inside the kernel. (No minimum size: measured faster than conv_mfma
  // from ResNet-50 batch 64 up, including the 98-tile stage-4 layers, profiles/archive/r1_resnet50_*.)
  const long long m = (long long)batch * d.Ho * d.Wo;
  return m < (1ll << 31) && (long long)batch * d.H * d.W * d.Cin < (1ll << 31);
}

hipError_t conv2d_gemm(const ConvDesc& d, int batch, const void* x, const void* w,
                       const float* bias, const void* res, void* y, hipStream_t stream) {
  GemmConvArgs a;
  a.x = static_cast<const bf16*>(x);
  a.w = static_cast<const bf16*>(w);
  a.bias = bias;
  a.res = static_cast<const bf16*>(res);
  a.y = y;
  a.out_f32 = d.out_f32;
  a.M = batch * d.Ho * d.Wo;
  a.H = d.H; a.W = d.W; a.Cin = d.Cin; a.HWo = d.Ho * d.Wo; a.Wo = d.Wo; a.Cout = d.Cout;
  a.KW = d.KW; a.stride = d.stride; a.pad = d.pad; a.Kpad = d.Kpad;
  a.nkb = d.K / 64;
  a.cin_blocks = d.stem ? 1 : d.Cin / 64;
  a.relu = d.relu;
  a.has_res = d.has_res && res != nullptr;
  a.x2 = nullptr; a.w2 = nullptr; a.bias2 = nullptr;
  a.H2 = a.W2 = a.Cin2 = a.stride2 = a.Kpad2 = 0;
  a.nkb1 = a.nkb;
  // 64-channel tiles for the single-k-step (K = 64) 1x1 convs: these are bound by their
  // epilogue traffic, and half-width tiles (24 KB of LDS, 91 VGPRs) put 5 workgroups on a CU
  // instead of 4 (ResNet-50 batch 256: 4.87 -> 4.81 ms; at K = 128 / 256 / 512 the same change
  // costs 0.6 / 1.6 / 2.6 %, profiles/r4_resnet50_layers.txt)
  // (the single-stage form for the K = 128 1x1 convs, with 64- or 128-channel tiles, measured
  // 0.4 / 2.2 % slower in round 4; for the 64-channel K = 256 ones, within noise)
  const int bn = (d.Npad % 128 == 0 && !(d.K == 64 && d.KH == 1 && !d.stem)) ? 128 : 64;
  constexpr int BM = 128;
  const int m_tiles = (a.M + BM - 1) / BM;
  a.n_tiles = d.Npad / bn;
  a.nwg = m_tiles * a.n_tiles;
  // per-shape choice: the packed stem; K = 64 (one k-step: 1x1 convs on 64 channels) in the
  // single-stage form with 64-channel tiles, 5 workgroups per CU; everything else
  // double-buffered, 128-channel tiles when Npad allows, else 64
  const bool one = a.nkb == 1;
  if (d.stem) {
    if (bn == 128)
      hipLaunchKernelGGL((conv_gemm_kernel<BM, 128, true, 2>), dim3(a.nwg), dim3(256), 0, stream,
                         a);
    else
      hipLaunchKernelGGL((conv_gemm_kernel<BM, 64, true, 2>), dim3(a.nwg), dim3(256), 0, stream,
                         a);
  } else if (bn == 128) {
    if (one)
      hipLaunchKernelGGL((conv_gemm_kernel<BM, 128, false, 1>), dim3(a.nwg), dim3(256), 0, stream,
                         a);
    else
      hipLaunchKernelGGL((conv_gemm_kernel<BM, 128, false, 2>), dim3(a.nwg), dim3(256), 0, stream,
                         a);
  } else {
    if (one)
      hipLaunchKernelGGL((conv_gemm_kernel<BM, 64, false, 1>), dim3(a.nwg), dim3(256), 0, stream,
                         a);
    else
      hipLaunchKernelGGL((conv_gemm_kernel<BM, 64, false, 2>), dim3(a.nwg), dim3(256), 0, stream,
                         a);
  }
  return hipGetLastError();
}

// images per launch of the fused projection: every element offset of the launch's x, x2 and y
// (and its pixel count) must stay below 2^31 (max_batch >= ~2675 overflowed the
// stage-2 projection's input)
static int proj_chunk_images(const ConvDesc& d, int H2, int W2, int Cin2) {
  const long long lim = (1ll << 31) - 1;
  long long per = (long long)d.Ho * d.Wo * std::max(d.Cout, 1);
  per = std::max(per, (long long)d.H * d.W * d.Cin);
  per = std::max(per, (long long)H2 * W2 * Cin2);
  return per > 0 ? (int)std::min<long long>(lim / per, 1 << 20) : 0;
}

bool conv_gemm_proj_supported(const ConvDesc& d, int batch, int H2, int W2, int Cin2,
                              int stride2, int Kpad2) {
  // (no conv_path switch: like the fused block kernels this op has no other implementation)
  if (d.fp8 || d.in_f32 || d.f32 || d.out_f32 || d.stem || d.has_res) return false;
  if (d.KH != 1 || d.KW != 1 || d.stride != 1 || d.pad != 0) return false;
  if (d.Cin % 64 != 0 || d.K != d.Cin || d.Kpad != d.K || d.Ho != d.H || d.Wo != d.W) return false;
  if (Cin2 % 64 != 0 || Kpad2 != Cin2 || stride2 < 1) return false;
  if ((H2 - 1) / stride2 + 1 != d.Ho || (W2 - 1) / stride2 + 1 != d.Wo) return false;
  if (d.Npad % 128 != 0 || d.Npad < d.Cout || d.Cout % 8 != 0) return false;
  // (any batch: conv2d_gemm_proj launches chunks whose 32-bit element offsets hold)
  return batch >= 0 && proj_chunk_images(d, H2, W2, Cin2) > 0;
}

hipError_t conv2d_gemm_proj(const ConvDesc& d, int batch, const void* x, const void* w,
                            const float* bias, const void* x2, int H2, int W2, int Cin2,
                            int stride2, int Kpad2, const void* w2, const float* bias2, void* y,
                            hipStream_t stream) {
  if (!conv_gemm_proj_supported(d, batch, H2, W2, Cin2, stride2, Kpad2))
    return hipErrorInvalidValue;
  const int chunk = proj_chunk_images(d, H2, W2, Cin2);
  if (batch > chunk) {  // chunks of images, each with 32-bit offsets (bf16 in and out)
    for (int c0 = 0; c0 < batch; c0 += chunk) {
      const int nb = std::min(chunk, batch - c0);
      const hipError_t e = conv2d_gemm_proj(
          d, nb, static_cast<const bf16*>(x) + (size_t)c0 * d.H * d.W * d.Cin, w, bias,
          static_cast<const bf16*>(x2) + (size_t)c0 * H2 * W2 * Cin2, H2, W2, Cin2, stride2,
          Kpad2, w2, bias2, static_cast<bf16*>(y) + (size_t)c0 * d.Ho * d.Wo * d.Cout, stream);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  GemmConvArgs a;
  a.x = static_cast<const bf16*>(x);
  a.w = static_cast<const bf16*>(w);
  a.bias = bias;
  a.res = nullptr;
  a.y = y;
  a.out_f32 = 0;
  a.M = batch * d.Ho * d.Wo;
  a.H = d.H; a.W = d.W; a.Cin = d.Cin; a.HWo = d.Ho * d.Wo; a.Wo = d.Wo; a.Cout = d.Cout;
  a.KW = 1; a.stride = 1; a.pad = 0; a.Kpad = d.Kpad;
  a.cin_blocks = d.Cin / 64;
  a.nkb1 = d.Cin / 64;
  a.nkb = a.nkb1 + Cin2 / 64;
  a.relu = d.relu;
  a.has_res = 0;
  a.x2 = static_cast<const bf16*>(x2);
  a.w2 = static_cast<const bf16*>(w2);
  a.bias2 = bias2;
  a.H2 = H2; a.W2 = W2; a.Cin2 = Cin2; a.stride2 = stride2; a.Kpad2 = Kpad2;
  constexpr int BM = 128;
  a.n_tiles = d.Npad / 128;
  a.nwg = (a.M + BM - 1) / BM * a.n_tiles;
  hipLaunchKernelGGL((conv_gemm_kernel<BM, 128, false, 2, true>), dim3(a.nwg), dim3(256), 0,
                     stream, a);
  return hipGetLastError();
}

namespace {
// one thread per output pixel (8 bytes) of the packed-stem image
__global__ __launch_bounds__(256) void stem_pack_kernel(int total, int W, int C, int Wp, int lp,
                                                        const float* __restrict__ x,
                                                        uint2* __restrict__ y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int row = i / Wp;  // n * H + h
  const int w = i - row * Wp - lp;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (w >= 0 && w < W) {
    const float* s = x + ((size_t)row * W + w) * C;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < C) v[c] = s[c];
  }
  bf16x4 o;
  o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
  y[i] = __builtin_bit_cast(uint2, o);
}
}  // namespace

hipError_t stem_pack(int batch, int H, int W, int C, int Wp, int lp, const float* x, void* y,
                     hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (C < 1 || C > 4 || lp < 0 || Wp < W + lp) return hipErrorInvalidValue;
  const long long total = (long long)batch * H * Wp;
  if (total >= (1ll << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(stem_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     stream, (int)total, W, C, Wp, lp, x, static_cast<uint2*>(y));
  return hipGetLastError();
}

}  // namespace gale
