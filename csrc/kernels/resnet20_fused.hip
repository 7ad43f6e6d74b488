// Whole-network CIFAR-10 ResNet-20 forward in ONE kernel: a workgroup carries an image through
// all 19 convolutions, the residual adds, the global pool, the dense layer and the softmax with
// every activation resident in LDS (BASELINE config 2/3 flagship; SURVEY.md §7.5 hard part 3:
// "consider whole-block or whole-network fusion (persistent kernel)").
//
// Why: per-layer kernels at serving batch sizes (64-256 images) are latency bound — ~20 launches,
// each re-reading its input through L2 with a 9x implicit-im2col amplification and exposing a
// global-memory latency per K step. Here the only HBM traffic per image is its 12 KB fp32 input
// and 40 B of softmax output; weights (540 KB bf16) stream from L2 as MFMA A fragments.
//
// LDS plan (78,464 B per workgroup -> 2 workgroups per CU), bf16 NHWC with a zero border so the
// 3x3 windows need no bounds checks (padded layouts Hp x Wp x C):
//   R0 [0, 36992)        X1 34x34x16 (stage-1 block input/output)  | stage 3: T3, X3 10x10x64
//   R1 [36992, 78464)    IN 34x34x3 (stem input) -> T1 34x34x16     | stage 2: T2, X2 18x18x32
// Block conv2 writes its output in place over its residual (each lane reads the residual of the
// pixel/channels it then writes, and no other lane reads that buffer in the same conv).
//
// MFMA mapping (v_mfma_f32_16x16x32_bf16, same orientation as conv_mfma.hip): D[channel][pixel];
// A = weights [Cout][Kpad] from global (k = (kh*3 + kw)*Cin + ci), hoisted into registers once
// per conv (each wave owns one 16-channel tile); B = 8 consecutive input channels of one tap of
// one pixel = one ds_read_b128 from the padded LDS image. Each wave walks its pixel tiles four
// at a time (four independent accumulators).
//
// Reference parity: the model the reference serves is an opaque SavedModel fetched as
// "output/Softmax:0" (InferenceBolt.java:81-86); numerics equal the layer-by-layer gale plan
// (same bf16 rounding points) and are checked against the fp32 oracle in tests.
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

constexpr int kR0 = 0;
constexpr int kR1 = 36992;
constexpr int kLds = 78464;
constexpr int kT2 = kR1, kX2 = kR1 + 20736;
constexpr int kT3 = kR0, kX3 = kR0 + 12800;

__device__ __forceinline__ bf16* lds_at(char* smem, int byte_off) {
  return reinterpret_cast<bf16*>(smem + byte_off);
}

// zero the one-pixel border of a padded Hp x Wp x C bf16 image (C % 8 == 0)
template <int HP, int WP, int C>
__device__ __forceinline__ void zero_border(bf16* buf) {
  constexpr int V = C / 8;  // 16-byte vectors per cell
  constexpr int CELLS = 2 * WP + 2 * (HP - 2);
  for (int i = threadIdx.x; i < CELLS * V; i += 256) {
    const int cell = i / V, v = i - cell * V;
    int h, w;
    if (cell < WP) { h = 0; w = cell; }
    else if (cell < 2 * WP) { h = HP - 1; w = cell - WP; }
    else { const int r = cell - 2 * WP; h = 1 + (r >> 1); w = (r & 1) ? WP - 1 : 0; }
    *reinterpret_cast<uint4*>(buf + (h * WP + w) * C + v * 8) = make_uint4(0, 0, 0, 0);
  }
}

// 3x3 pad-1 convolution LDS -> LDS with the folded-BN bias, optional residual and ReLU.
// RES: 0 none, 1 identity (same layout as out), 2 option-A shortcut from the previous stage's
// buffer (stride-2 subsample, channels >= RC are zero).
template <int CIN, int COUT, int S, int HO, int RES, int RC>
__device__ __forceinline__ void conv3x3(const bf16* __restrict__ wg, const float* __restrict__ bias,
                                        const bf16* in, bf16* out, const bf16* res) {
  constexpr int WPI = HO * S + 2;  // padded input width
  constexpr int WPO = HO + 2;      // padded output width
  constexpr int RWP = 2 * HO + 2;  // padded width of an option-A residual source
  constexpr int K = 9 * CIN;
  constexpr int KPAD = (K + 31) / 32 * 32;
  constexpr int KS = KPAD / 32;
  constexpr int CT = COUT / 16;        // channel tiles
  constexpr int PT = HO * HO / 16;     // 16-pixel tiles
  constexpr int WPC = 4 / CT;          // waves per channel tile
  constexpr int PTW = PT / WPC;        // pixel tiles per wave
  static_assert(PTW % 4 == 0, "pixel tiles per wave must be a multiple of 4");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int ct = wave / WPC;
  const int pt0 = (wave % WPC) * PTW;

  bf16x8 afr[KS];
  int koff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = ks * 32 + g * 8;
    afr[ks] = ld_bf16x8(wg + (ct * 16 + col) * KPAD + k);
    int tap = k / CIN;
    const int ci = k - tap * CIN;
    if (tap >= 9) tap = 0;  // K padding: zero weights, any finite input
    koff[ks] = ((tap / 3) * WPI + (tap % 3)) * CIN + ci;
  }
  const int c0 = ct * 16 + g * 4;  // this lane's 4 output channels
  const float4 bv = *reinterpret_cast<const float4*>(bias + c0);

#pragma unroll 1
  for (int pg = 0; pg < PTW; pg += 4) {
    int pbase[4], ho[4], wo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int m = (pt0 + pg + p) * 16 + col;
      ho[p] = m / HO;
      wo[p] = m - ho[p] * HO;
      pbase[p] = (ho[p] * S * WPI + wo[p] * S) * CIN;
    }
    f32x4 acc[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 b[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) b[p] = ld_bf16x8(in + pbase[p] + koff[ks]);
#pragma unroll
      for (int p = 0; p < 4; ++p)
        acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[ks], b[p], acc[p], 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float v0 = acc[p][0] + bv.x, v1 = acc[p][1] + bv.y;
      float v2 = acc[p][2] + bv.z, v3 = acc[p][3] + bv.w;
      const int o = ((ho[p] + 1) * WPO + wo[p] + 1) * COUT + c0;
      if (RES == 1) {
        const bf16x4 r = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(res + o));
        v0 += (float)r[0]; v1 += (float)r[1]; v2 += (float)r[2]; v3 += (float)r[3];
      } else if (RES == 2) {
        if (c0 < RC) {
          const int ro = ((2 * ho[p] + 1) * RWP + 2 * wo[p] + 1) * RC + c0;
          const bf16x4 r = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(res + ro));
          v0 += (float)r[0]; v1 += (float)r[1]; v2 += (float)r[2]; v3 += (float)r[3];
        }
      }
      bf16x4 ov;
      ov[0] = (bf16)fmaxf(v0, 0.f); ov[1] = (bf16)fmaxf(v1, 0.f);
      ov[2] = (bf16)fmaxf(v2, 0.f); ov[3] = (bf16)fmaxf(v3, 0.f);
      *reinterpret_cast<uint2*>(out + o) = __builtin_bit_cast(uint2, ov);
    }
  }
}

// stem: 3x3x3 -> 16 over the 34x34x3 padded input (K = 27 padded to 32: one k step, the 8
// k-values of a lane are 8 scalar LDS reads)
__device__ __forceinline__ void stem(const bf16* __restrict__ wg, const float* __restrict__ bias,
                                     const bf16* in, bf16* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  const bf16x8 a = ld_bf16x8(wg + col * 32 + g * 8);
  int off[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = g * 8 + j;
    const int tap = k < 27 ? k / 3 : 0, ci = k < 27 ? k % 3 : 0;
    off[j] = ((tap / 3) * 34 + tap % 3) * 3 + ci;
  }
  const float4 bv = *reinterpret_cast<const float4*>(bias + g * 4);
#pragma unroll 1
  for (int pg = 0; pg < 16; pg += 4) {
    f32x4 acc[4];
    int ho[4], wo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int m = (wave * 16 + pg + p) * 16 + col;
      ho[p] = m >> 5;
      wo[p] = m & 31;
      const bf16* px = in + (ho[p] * 34 + wo[p]) * 3;
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = px[off[j]];
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      bf16x4 ov;
      ov[0] = (bf16)fmaxf(acc[p][0] + bv.x, 0.f); ov[1] = (bf16)fmaxf(acc[p][1] + bv.y, 0.f);
      ov[2] = (bf16)fmaxf(acc[p][2] + bv.z, 0.f); ov[3] = (bf16)fmaxf(acc[p][3] + bv.w, 0.f);
      *reinterpret_cast<uint2*>(out + ((ho[p] + 1) * 34 + wo[p] + 1) * 16 + g * 4) =
          __builtin_bit_cast(uint2, ov);
    }
  }
}

__global__ __launch_bounds__(256, 2) void resnet20_fused_kernel(ResNet20Params p, const float* x,
                                                                float* out, int batch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* X1 = lds_at(smem, kR0);
  bf16* T1 = lds_at(smem, kR1);
  bf16* IN = lds_at(smem, kR1);
  bf16* T2 = lds_at(smem, kT2);
  bf16* X2 = lds_at(smem, kX2);
  bf16* T3 = lds_at(smem, kT3);
  bf16* X3 = lds_at(smem, kX3);
  float* scratch = reinterpret_cast<float*>(smem + kR1);

  for (int img = blockIdx.x; img < batch; img += gridDim.x) {
    __syncthreads();  // the previous image's head is done with R0/R1
    // ---- stage the fp32 input image as bf16 into the zero-bordered 34x34x3 IN ----
    for (int i = threadIdx.x; i < 34 * 34 * 3; i += 256) {
      const int cell = i / 3;
      const int h = cell / 34, w = cell - h * 34;
      if (h == 0 || h == 33 || w == 0 || w == 33) IN[i] = (bf16)0.f;
    }
    zero_border<34, 34, 16>(X1);
    const float4* xi = reinterpret_cast<const float4*>(x + (size_t)img * 3072);
    for (int i = threadIdx.x; i < 768; i += 256) {
      const float4 v = xi[i];
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int idx = i * 4 + j;  // (h*32 + w)*3 + c
        const int pix = idx / 3, c = idx - pix * 3;
        const int h = pix >> 5, w = pix & 31;
        IN[((h + 1) * 34 + w + 1) * 3 + c] = (bf16)e[j];
      }
    }
    __syncthreads();
    stem(static_cast<const bf16*>(p.w[0]), p.b[0], IN, X1);
    __syncthreads();
    zero_border<34, 34, 16>(T1);  // IN is dead; T1's border overlaps its bytes
    // ---- stage 1: 32x32x16 ----
#pragma unroll 1
    for (int blk = 0; blk < 3; ++blk) {
      conv3x3<16, 16, 1, 32, 0, 16>(static_cast<const bf16*>(p.w[1 + 2 * blk]), p.b[1 + 2 * blk], X1, T1, nullptr);
      __syncthreads();
      conv3x3<16, 16, 1, 32, 1, 16>(static_cast<const bf16*>(p.w[2 + 2 * blk]), p.b[2 + 2 * blk], T1, X1, X1);
      __syncthreads();
    }
    // ---- stage 2: 16x16x32 ----
    zero_border<18, 18, 32>(T2);
    zero_border<18, 18, 32>(X2);
    conv3x3<16, 32, 2, 16, 0, 16>(static_cast<const bf16*>(p.w[7]), p.b[7], X1, T2, nullptr);
    __syncthreads();
    conv3x3<32, 32, 1, 16, 2, 16>(static_cast<const bf16*>(p.w[8]), p.b[8], T2, X2, X1);
    __syncthreads();
#pragma unroll 1
    for (int blk = 1; blk < 3; ++blk) {
      conv3x3<32, 32, 1, 16, 0, 32>(static_cast<const bf16*>(p.w[7 + 2 * blk]), p.b[7 + 2 * blk], X2, T2, nullptr);
      __syncthreads();
      conv3x3<32, 32, 1, 16, 1, 32>(static_cast<const bf16*>(p.w[8 + 2 * blk]), p.b[8 + 2 * blk], T2, X2, X2);
      __syncthreads();
    }
    // ---- stage 3: 8x8x64 ----
    zero_border<10, 10, 64>(T3);
    zero_border<10, 10, 64>(X3);
    conv3x3<32, 64, 2, 8, 0, 32>(static_cast<const bf16*>(p.w[13]), p.b[13], X2, T3, nullptr);
    __syncthreads();
    conv3x3<64, 64, 1, 8, 2, 32>(static_cast<const bf16*>(p.w[14]), p.b[14], T3, X3, X2);
    __syncthreads();
#pragma unroll 1
    for (int blk = 1; blk < 3; ++blk) {
      conv3x3<64, 64, 1, 8, 0, 64>(static_cast<const bf16*>(p.w[13 + 2 * blk]), p.b[13 + 2 * blk], X3, T3, nullptr);
      __syncthreads();
      conv3x3<64, 64, 1, 8, 1, 64>(static_cast<const bf16*>(p.w[14 + 2 * blk]), p.b[14 + 2 * blk], T3, X3, X3);
      __syncthreads();
    }
    // ---- head: global average pool (8x8) -> dense 64 -> 10 -> softmax ----
    {
      const int c = threadIdx.x & 63, q = threadIdx.x >> 6;  // 4 quarters of 16 pixels
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int pix = q * 16 + i;
        const int h = pix >> 3, w = pix & 7;
        s += (float)X3[((h + 1) * 10 + w + 1) * 64 + c];
      }
      scratch[q * 64 + c] = s;  // R1 is free in stage 3's last block (X2 is dead)
      __syncthreads();
      if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const float pooled =
            (scratch[lane] + scratch[64 + lane] + scratch[128 + lane] + scratch[192 + lane]) *
            (1.f / 64.f);
        float logit = -3.0e38f;
        for (int o = 0; o < 10; ++o) {
          const float t = wave_sum(p.fc_w[o * 64 + lane] * pooled);
          if (lane == o) logit = t + p.fc_b[o];
        }
        const float mx = wave_max(lane < 10 ? logit : -3.0e38f);
        const float e = lane < 10 ? __expf(logit - mx) : 0.f;
        const float sum = wave_sum(e);
        if (lane < 10) out[(size_t)img * 10 + lane] = e / sum;
      }
    }
  }
}

}  // namespace

hipError_t resnet20_fused_forward(const ResNet20Params& p, int batch, const float* x, float* out,
                                  hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  static int grid_cap = 0;
  if (grid_cap == 0) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid_cap = 2 * (cus > 0 ? cus : 256);  // 2 resident workgroups per CU (LDS bound)
  }
  const int grid = batch < grid_cap ? batch : grid_cap;
  hipLaunchKernelGGL(resnet20_fused_kernel, dim3(grid), dim3(256), kLds, stream, p, x, out, batch);
  return hipGetLastError();
}

}  // namespace gale
