// Whole-bottleneck kernel for the ResNet-50 56x56 stage (bf16, BASELINE config 4): conv1 (1x1,
// 256 -> 64 or, in block 0, 64 -> 64), conv2 (3x3, 64 -> 64) and conv3 (1x1, 64 -> 256) with its
// shortcut (the block input, or in block 0 the 1x1 projection of it) and both ReLUs, in ONE
// launch. The two 64-channel intermediates never leave the CU.
//
// Why: the layered plan moves every 56x56 tensor through HBM - per identity block the 256-channel
// input is read twice (conv1, conv3's residual) and the two 64-channel intermediates are written
// and read back: 414 us per block at batch 256, 4.0-5.2 TB/s, MFMA busy 5-9 % in the 1x1 layers
// (profiles/r4_resnet50_layers.txt:10-16). Fused, a block reads its input once (+ 2 halo rows in
// 8) and its residual once (block 0: computes it from the input it already reads), and writes
// its output once.
//
// Tiling: one workgroup (8 waves, 1 per CU: 145 KB of LDS) owns TR = 8 output rows x 56 columns
// of one image, all 256 output channels. Its LDS holds
//   H1: conv1's output over the (TR + 2) x (W + 2) halo patch (zero padding ring), 128-B rows;
//       later H2, conv2's output for the TR x W tile (same rows, so no extra space);
//   W2: the nine 64 x 64 conv2 taps (LDS-DMA at the start, landing during phase 1); later W3
//       (and Wd, the block-0 projection) for phase 3.
// Every 128-B LDS row stores its 16-B chunk c at slot c ^ rkey(row) (see rkey): 16 lanes reading
// 16 consecutive rows hit 16 distinct 4-bank groups.
//   phase 1: conv1 on the 10 x 56 halo pixels: per wave up to 5 tiles of 16 pixels x all 64
//            channels; the input fragments (the only HBM stream; 4 k-steps ahead) and conv1's
//            weights (L2; 1 step ahead) are loaded straight into registers; bias + ReLU -> bf16
//            -> H1.
//   phase 2: conv2 from H1 (taps = shifted patch rows) x W2, 4 x 2 waves of 112 pixels x 32
//            channels; the residual (or block-0 input) fragments of phase 3 are issued first so
//            their HBM latency hides under the MFMAs; bias + ReLU -> bf16 -> H2 over H1.
//   phase 3: conv3 (K = 64) from H2 x W3 in four passes of 32 channels per wave; epilogue
//            bias + shortcut + ReLU -> bf16, 8-byte stores (a wave completes each 128-B line).
// Rounding matches the layered plan: H1, H2 and the block-0 projection are rounded to bf16
// exactly where the layered kernels store them.
// Grid: batch x 7 strips, XCD-contiguous (neighbouring strips share 2 halo rows in one L2).
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src), (lds_ptr_t)(lds_base), 16, 0, 0);
}

constexpr int kW = 56, kH = 56, kCM = 64, kCO = 256, kTR = 8;
constexpr int kPW = kW + 2;                      // patch width (zero column each side)
constexpr int kR1 = kTR + 2;                     // patch rows
constexpr int kH1Bytes = kR1 * kPW * 128;        // 74,240
constexpr int kW2Bytes = 9 * kCM * 128;          // 73,728
constexpr int kLdsBytes = kH1Bytes + kW2Bytes;   // 147,968
constexpr int kT1 = kR1 * kW / 16;               // 35 phase-1 pixel tiles
constexpr int kStrips = kH / kTR;                // 7
static_assert(kR1 * kW % 16 == 0 && kTR * kW % (16 * 4) == 0, "tile geometry");
static_assert(kCO * 128 <= kW2Bytes, "W3 must fit the W2 region");
static_assert(kCO * 128 + 8 * 4096 <= kW2Bytes, "two-tile output stages must fit past W3");

struct BneckArgs {
  const bf16* x;   // [B][56][56][CIN]
  const bf16* w1;  // [64][CIN]
  const bf16* w2;  // [64][9 * 64], k = tap * 64 + ci
  const bf16* w3;  // [256][64]
  const bf16* wd;  // [256][64] (block 0)
  const float* b1;
  const float* b2;
  const float* b3;
  const float* bd;
  bf16* y;         // [B][56][56][256]
  int nwg;
};

// XOR key of 128-B LDS row `row`: even values only, so a ds_read_b128 lane group - which mixes
// chunks c and c ^ 1 (fq = 0 / 1 lanes) - never has two lanes on one 4-bank group for ANY 16
// consecutive rows, not just 16-aligned ones: the conv2 taps read the patch at row offsets
// +1 / +2 (bank model: 6.9 -> 4.6 LDS cycles per fragment read, 4 = conflict-free)
__device__ __forceinline__ int rkey(int row) { return ((row >> 1) & 3) << 1; }
// byte offset of 16-B chunk c of 128-B LDS row `row`
__device__ __forceinline__ int swz(int row, int c) { return row * 128 + ((c ^ rkey(row)) << 4); }

// conv3 / projection output channel held by LDS weight row R: within each 64-channel group,
// MFMA tile t row m <- channel (m >> 2) * 16 + t * 4 + (m & 3), so a lane's four channel tiles
// hold 16 CONSECUTIVE channels (fq * 16 ..) of its pixel: 16-byte residual loads and stage stores
__device__ __forceinline__ int perm3(int R) {
  return (R & ~63) | (((R & 15) >> 2) << 4) | (((R >> 4) & 3) << 2) | (R & 3);
}

__device__ __forceinline__ bf16x8 lds16(const uint8_t* lds, int off) {
  return *reinterpret_cast<const bf16x8*>(lds + off);
}

template <int CIN, bool DOWN>
__global__ __launch_bounds__(512, 1) void bottleneck56_kernel(BneckArgs a) {
  constexpr int NC = CIN / 32;  // phase-1 k-steps
  __shared__ __attribute__((aligned(1024))) uint8_t lds[kLdsBytes];
  uint8_t* const h1 = lds;
  uint8_t* const wreg = lds + kH1Bytes;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  // XCD-contiguous tile order (bijective for any nwg)
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = a.nwg >> 3, r8 = a.nwg & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int n = rid / kStrips, y0 = (rid - n * kStrips) * kTR;

  // ---- W1 -> the H1 region (free until conv1's outputs are written): CIN / 64 blocks of 64
  // rows x 128 B, row = k-block * 64 + output channel ----
  constexpr int W1I = CIN / 64;  // wave-instructions per wave (64 * CIN / 64 rows / 8 / 8 waves)
#pragma unroll
  for (int j = 0; j < W1I; ++j) {
    const int wi = wave * W1I + j;
    const int row = wi * 8 + (lane >> 3);
    const int kb = row >> 6, ch = row & 63;
    const int c = (lane & 7) ^ rkey(row);
    glds16(a.w1 + ch * CIN + kb * 64 + c * 8, h1 + wi * 1024);
  }
  // W2 -> LDS (lands during phase 1): 576 rows of 128 B = 72 wave-instructions
  auto stage_w2 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int wi = wave * 9 + j;
      const int rg = wi * 8 + (lane >> 3);  // tap * 64 + output channel
      const int tap = rg >> 6, row = rg & 63;
      const int c = (lane & 7) ^ rkey(row);
      glds16(a.w2 + row * (9 * kCM) + tap * kCM + c * 8, wreg + wi * 1024);
    }
  };

  // ---- phase 1: conv1 over the halo rows y0-1 .. y0+8 -> H1 ----
  {
    const bool t5 = wave < kT1 - 32;  // waves 0..2 own a fifth tile
    const bf16* xr[5];
    int hs[5];
    bool rv[5];
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int t = wave + 8 * s;
      const int qp = (t < kT1 ? t : 0) * 16 + fr;
      const int r = qp / kW, cc = qp - r * kW;
      const int yy = y0 - 1 + r;
      rv[s] = (unsigned)yy < (unsigned)kH;
      const int yc = yy < 0 ? 0 : (yy >= kH ? kH - 1 : yy);
      xr[s] = a.x + ((size_t)(n * kH + yc) * kW + cc) * CIN + fq * 8;
      hs[s] = r * kPW + cc + 1;
    }
    f32x4 acc[5][4];
#pragma unroll
    for (int s = 0; s < 5; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[s][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the input fragments (HBM) run D k-steps ahead; conv1's weights come from LDS
    constexpr int D = NC < 4 ? NC : 4;
    bf16x8 xf[D][5];
    auto ldx = [&](int c) __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < 5; ++s)
        if (s < 4 || t5) xf[c % D][s] = ld_bf16x8(xr[s] + c * 32);
    };
#pragma unroll
    for (int c = 0; c < D - 1; ++c) ldx(c);
    // W1 landed in every wave (its DMA was issued before these >= 4 (D - 1) input loads;
    // vector-memory loads complete in order), then the workgroup barrier
    if constexpr (D - 1 >= 3)
      asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    stage_w2();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c + D - 1 < NC) ldx(c + D - 1);
      bf16x8 wf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[j] = lds16(h1, swz((c >> 1) * 64 + j * 16 + fr, (c & 1) * 4 + fq));
#pragma unroll
      for (int s = 0; s < 5; ++s)
        if (s < 4 || t5)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[s][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[c % D][s], acc[s][j],
                                                                0, 0, 0);
    }
    __syncthreads();  // every wave is done with W1: its region becomes H1
    // zero padding columns of the patch (slots r * 58 and r * 58 + 57)
    if (tid < kR1 * 2 * 8) {
      const int s = tid >> 3, r = s >> 1;
      *reinterpret_cast<uint4*>(h1 + (r * kPW + (s & 1) * (kPW - 1)) * 128 + (tid & 7) * 16) =
          make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 b = *reinterpret_cast<const float4*>(a.b1 + j * 16 + fq * 4);
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        if (s < 4 || t5) {
          bf16x4 o;
          o[0] = (bf16)(rv[s] ? fmaxf(acc[s][j][0] + b.x, 0.f) : 0.f);
          o[1] = (bf16)(rv[s] ? fmaxf(acc[s][j][1] + b.y, 0.f) : 0.f);
          o[2] = (bf16)(rv[s] ? fmaxf(acc[s][j][2] + b.z, 0.f) : 0.f);
          o[3] = (bf16)(rv[s] ? fmaxf(acc[s][j][3] + b.w, 0.f) : 0.f);
          *reinterpret_cast<uint2*>(h1 + swz(hs[s], 2 * j + (fq >> 1)) + (fq & 1) * 8) =
              __builtin_bit_cast(uint2, o);
        }
      }
    }
  }
  __syncthreads();  // H1 complete, W2 landed

  // ---- phase-3 operands fetched now, consumed after phase 2 ----
  const int wm = wave >> 1, wn = wave & 1;
  int gp[7];  // NHWC pixel index of this lane's pixel in each of the wave's 7 tiles
  int pr[7];  // tile pixel (0..447) = H2 row
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int p = (wm * 7 + i) * 16 + fr;
    const int r = p / kW, cc = p - r * kW;
    pr[i] = p;
    gp[i] = (n * kH + y0 + r) * kW + cc;
  }
  // identity: the residual in (perm3) MFMA-output layout, 2 passes x 7 tiles x 16 channels;
  // block 0: the input pixels' 64 channels for the projection (7 tiles x 2 k-halves)
  uint4 res[DOWN ? 1 : 2][7][2];
  bf16x8 xc[DOWN ? 7 : 1][2];
  if constexpr (DOWN) {
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) xc[i][kk] = ld_bf16x8(a.x + (size_t)gp[i] * CIN + kk * 32 + fq * 8);
  } else {
    // (perm3 layout: 16 consecutive channels of the pixel per lane and 64-channel group)
#pragma unroll
    for (int ps = 0; ps < 2; ++ps)
#pragma unroll
      for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          res[ps][i][h] = *reinterpret_cast<const uint4*>(
              a.x + (size_t)gp[i] * kCO + wn * 128 + ps * 64 + fq * 16 + h * 8);
  }

  // ---- phase 2: conv2 (3x3) from H1 -> registers ----
  f32x4 acc2[7][2];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t) acc2[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    int pb[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int r = pr[i] / kW;
      pb[i] = r * kPW + (pr[i] - r * kW);  // patch slot of the pixel at tap (0, 0)
    }
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3;
      const int toff = kh * kPW + (tap - kh * 3);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + fq;
        bf16x8 af[2], bfr[7];
#pragma unroll
        for (int t = 0; t < 2; ++t) af[t] = lds16(wreg, tap * 8192 + swz(wn * 32 + t * 16 + fr, c));
#pragma unroll
        for (int i = 0; i < 7; ++i) bfr[i] = lds16(h1, swz(pb[i] + toff, c));
#pragma unroll
        for (int i = 0; i < 7; ++i)
#pragma unroll
          for (int t = 0; t < 2; ++t)
            acc2[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bfr[i], acc2[i][t], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // every wave is done with H1 and W2

  // W3 -> the W2 region: 256 rows of 128 B each = 32 wave-instructions (block 0's projection
  // weights come from L2 into registers, one 64-channel group per pass)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int wi = wave * 4 + j;
    const int row = wi * 8 + (lane >> 3);
    const int c = (lane & 7) ^ rkey(row);
    const int g = perm3(row);
    glds16(a.w3 + g * kCM + c * 8, wreg + wi * 1024);
  }
  // H2 = bf16(relu(conv2 + b2)) over H1
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float4 b = *reinterpret_cast<const float4*>(a.b2 + wn * 32 + t * 16 + fq * 4);
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      bf16x4 o;
      o[0] = (bf16)fmaxf(acc2[i][t][0] + b.x, 0.f);
      o[1] = (bf16)fmaxf(acc2[i][t][1] + b.y, 0.f);
      o[2] = (bf16)fmaxf(acc2[i][t][2] + b.z, 0.f);
      o[3] = (bf16)fmaxf(acc2[i][t][3] + b.w, 0.f);
      *reinterpret_cast<uint2*>(h1 + swz(pr[i], wn * 4 + t * 2 + (fq >> 1)) + (fq & 1) * 8) =
          __builtin_bit_cast(uint2, o);
    }
  }
  __syncthreads();  // H2 written, W3 / Wd landed

  // ---- phase 3: conv3 + shortcut: per wave 7 tiles of 16 pixels x two 64-channel groups ----
  // Each tile's 16 x 128-B output lines go through a wave-private 2 KB LDS stage (the H1 bytes
  // past H2) so that every global store is 16 B per lane and whole lines per instruction: the
  // MFMA layout's 8-byte pieces of 16 pixels cost ~40 % of the kernel in partial-line writes.
  // Stage: two tiles per wave (4 KB) in the weight region past W3 (fewer serialised LDS round
  // trips than one)
  constexpr int TPS = 2;
  uint8_t* const stg = wreg + kCO * 128 + wave * 4096;
  // (identity: unrolled, so res[ps] indexes registers statically; block 0: one pass at a time)
  constexpr int kPassUnroll = DOWN ? 1 : 2;
#pragma unroll kPassUnroll
  for (int ps = 0; ps < 2; ++ps) {
    const int ch0 = wn * 128 + ps * 64;
    bf16x8 af[4][2], df[DOWN ? 4 : 1][2];  // W3 (and Wd) fragments, reused by the 7 tiles
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        af[t][kk] = lds16(wreg, swz(ch0 + t * 16 + fr, kk * 4 + fq));
        if constexpr (DOWN)
          df[t][kk] = ld_bf16x8(a.wd + perm3(ch0 + t * 16 + fr) * kCM + kk * 32 + fq * 8);
      }
    float4 b3v[4], bdv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      b3v[t] = *reinterpret_cast<const float4*>(a.b3 + ch0 + fq * 16 + t * 4);
      if constexpr (DOWN) bdv[t] = *reinterpret_cast<const float4*>(a.bd + ch0 + fq * 16 + t * 4);
    }
    // one tile: conv3 (+ projection), bias + shortcut + ReLU in fp32, one bf16 rounding (as
    // the layered conv3); lane: 16 consecutive channels of pixel fr -> 32 B of stage row fr
    auto tile = [&](int i, uint8_t* st) __attribute__((always_inline)) {
      f32x4 acc3[4], accd[DOWN ? 4 : 1];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc3[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (DOWN) accd[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 bfr = lds16(h1, swz(pr[i], kk * 4 + fq));
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          acc3[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t][kk], bfr, acc3[t], 0, 0, 0);
          if constexpr (DOWN)
            accd[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(df[t][kk], xc[i][kk], accd[t], 0,
                                                              0, 0);
        }
      }
      bf16x4 o[4];  // channels fq * 16 + t * 4 .. + 4 (perm3)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float sc[4];
        if constexpr (DOWN) {
          // the projection as the layered plan stores it: bf16(wd . x + bd)
          sc[0] = (float)(bf16)(accd[t][0] + bdv[t].x);
          sc[1] = (float)(bf16)(accd[t][1] + bdv[t].y);
          sc[2] = (float)(bf16)(accd[t][2] + bdv[t].z);
          sc[3] = (float)(bf16)(accd[t][3] + bdv[t].w);
        } else {
          const bf16x8 rr = __builtin_bit_cast(bf16x8, res[ps][i][t >> 1]);
#pragma unroll
          for (int e = 0; e < 4; ++e) sc[e] = (float)rr[(t & 1) * 4 + e];
        }
        o[t][0] = (bf16)fmaxf(acc3[t][0] + b3v[t].x + sc[0], 0.f);
        o[t][1] = (bf16)fmaxf(acc3[t][1] + b3v[t].y + sc[1], 0.f);
        o[t][2] = (bf16)fmaxf(acc3[t][2] + b3v[t].z + sc[2], 0.f);
        o[t][3] = (bf16)fmaxf(acc3[t][3] + b3v[t].w + sc[3], 0.f);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = o[2 * h][e];
          v[4 + e] = o[2 * h + 1][e];
        }
        *reinterpret_cast<uint4*>(st + swz(fr, 2 * fq + h)) = __builtin_bit_cast(uint4, v);
      }
    };
    // read back 8 pixels x 128 B per instruction: lane -> pixel (lane >> 3) + 8h, chunk lane & 7
    auto flush = [&](int i, const uint8_t* st) __attribute__((always_inline)) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int px = h * 8 + (lane >> 3), c = lane & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(st + swz(px, c));
        const int p = (wm * 7 + i) * 16 + px;
        const int r = p / kW, cc = p - r * kW;
        *reinterpret_cast<uint4*>(a.y + (size_t)((n * kH + y0 + r) * kW + cc) * kCO + ch0 + c * 8) = v;
      }
    };
#pragma unroll
    for (int i0 = 0; i0 < 7; i0 += TPS) {
#pragma unroll
      for (int u = 0; u < TPS; ++u)
        if (i0 + u < 7) tile(i0 + u, stg + u * 2048);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (wave-private stage)
#pragma unroll
      for (int u = 0; u < TPS; ++u)
        if (i0 + u < 7) flush(i0 + u, stg + u * 2048);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // stage free for the next round
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

}  // namespace

bool bottleneck56_supported(int H, int W, int cin, int cmid, int cout, int down) {
  return H == kH && W == kW && cmid == kCM && cout == kCO &&
         ((down && cin == 64) || (!down && cin == kCO));
}

hipError_t bottleneck56(const BottleneckParams& p, int batch, const void* x, void* y,
                        hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (!p.w1 || !p.w2 || !p.w3 || !p.b1 || !p.b2 || !p.b3 || !x || !y) return hipErrorInvalidValue;
  if (p.down && (!p.wd || !p.bd || p.cin != 64)) return hipErrorInvalidValue;
  if (!p.down && p.cin != kCO) return hipErrorInvalidValue;
  // the kernel's element offsets are 32-bit: launch chunks of <= 2048 images (any max_batch)
  constexpr int kChunk = 2048;
  static_assert((long long)kChunk * kH * kW * kCO < (1ll << 31), "chunk offsets");
  for (int c0 = 0; c0 < batch; c0 += kChunk) {
    const int nb = batch - c0 < kChunk ? batch - c0 : kChunk;
    BneckArgs a;
    a.x = static_cast<const bf16*>(x) + (size_t)c0 * kH * kW * p.cin;
    a.w1 = static_cast<const bf16*>(p.w1);
    a.w2 = static_cast<const bf16*>(p.w2);
    a.w3 = static_cast<const bf16*>(p.w3);
    a.wd = static_cast<const bf16*>(p.wd);
    a.b1 = p.b1; a.b2 = p.b2; a.b3 = p.b3; a.bd = p.bd;
    a.y = static_cast<bf16*>(y) + (size_t)c0 * kH * kW * kCO;
    a.nwg = nb * kStrips;
    if (p.down)
      hipLaunchKernelGGL((bottleneck56_kernel<64, true>), dim3(a.nwg), dim3(512), 0, stream, a);
    else
      hipLaunchKernelGGL((bottleneck56_kernel<256, false>), dim3(a.nwg), dim3(512), 0, stream,
                         a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace gale
