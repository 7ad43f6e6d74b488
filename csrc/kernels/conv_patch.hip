// 3x3 stride-1 convolutions with an LDS-resident input patch (bf16, Cin % 64 == 0): the
// ResNet-50 bottleneck conv2 layers at 56x56, 28x28 and 14x14.
//
// Why: in conv_gemm.hip every k-step stages the im2col rows of ONE tap, so each input pixel
// crosses the vector-memory return path (TA/TD -> LDS) nine times per 64 input channels. The
// per-layer counters show that path, not the MFMA, binding those layers: TD busy 0.6-0.75 of
// the CU cycles against MFMA busy 22-28 % (profiles/archive/r2_resnet50_layers_mem_pmc.txt).
//
// Here a workgroup owns TR whole output rows of one image (TR*W <= 128 pixels: 2 x 56,
// 4 x 28, 7 x 14) and BN output channels. Per 64-channel input block it stages the
// (TR+2) x (W+2) halo patch ONCE (zero rows/columns for the padding), then runs the nine taps as
// nine 64-deep k-steps whose B fragments are the patch rows shifted by (kh, kw). Only the
// weight rows of each tap are staged per step. For a 28x28 tile the input bytes per 64
// channels drop from 9 x 112 to 180 rows.
//
// Pipeline: weights double-buffered per step; the patch is double-buffered per input block, and
// the next block's patch is issued with the last tap's weights. The taps of a block share its
// patch, so the next tap's X fragments are read at the end of a step, before the barrier (3x3
// layers 2-5 % faster; a 3-stage weight ring with counted vmcnt was slower,
// profiles/r5_conv_patch_ab.jsonl). Both go by LDS-DMA
// (global_load_lds_dwordx4), with the same source-side XOR bank swizzle as conv_gemm (slot s of
// LDS row r holds 16-byte chunk s ^ ((r >> 1) & 7)). Fragment rows map pixel p of the tile to
// patch row (p / W + kh) * (W + 2) + p % W + kw; rows past the tile's pixels read a zero row.
// The epilogue (bias, residual, ReLU) is the same as conv_gemm's, staged through LDS.
#include <algorithm>
#include <atomic>

#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

__device__ __attribute__((aligned(16))) uint8_t g_patch_zero[64];

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src), (lds_ptr_t)(lds_base), 16, 0, 0);
}

struct PatchArgs {
  const bf16* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
  bf16* y;
  int H, W, Cin, Cout, Kpad;
  int TR, P, PW, PR;    // rows per tile, pixels per tile (TR * W), patch width W + 2, patch rows
  int rblocks;          // H / TR
  int IMG, PR1, B;      // whole images per tile (> 1 only when TR == H: 7x7), patch rows per
                        // image, batch (the last tile of a multi-image layer may be partial)
  int nsteps;           // 9 * Cin / 64
  int relu, has_res;
  int n_tiles, nwg;
};

// PRR: patch rows held in LDS (>= PR + 1 for the zero row, a multiple of 8 = one
// wave-instruction); compile-time so the two stages are static LDS (2 workgroups per CU).
// (Variants measured and removed in round 3 - 256-row tiles with 8 waves, 64-channel tiles with
// one patch buffer at 4 workgroups per CU, two taps per k-step: none faster than these tiles,
// profiles/archive/r2_conv_patch.txt.)
template <int BN, int PRR>
__global__ __launch_bounds__(256, 2)
void conv_patch_kernel(PatchArgs a) {
  constexpr int WM = 2;              // waves along the pixels
  constexpr int kBM = WM * 64;       // MFMA rows per tile (pixels P <= kBM; the rest read zeros)
  constexpr int WN = 2, NW = WM * WN;
  constexpr int TM = kBM / WM / 16;  // 16-pixel tiles per wave
  constexpr int TN = BN / WN / 16;   // 16-channel tiles per wave
  constexpr int WI = BN / (8 * NW);  // weight wave-instructions per wave per step
  constexpr int NPJ = PRR / 8;       // patch wave-instructions
  constexpr int PJ = (NPJ + NW - 1) / NW;  // ... per wave
  constexpr int SPB = 9;             // k-steps (taps) per 64-channel input block
  constexpr int WST = BN * 128;      // bytes per weight stage
  constexpr int PST = PRR * 128;     // bytes per patch stage
  constexpr int CW = BN / WN;        // epilogue geometry (as conv_gemm)
  constexpr int EPS = CW + 4;
  constexpr int LPR = CW / 8;
  constexpr int RPI = 64 / LPR;
  constexpr int HALF = TM / 2 * 16;
  constexpr int NRI = HALF / RPI;
  constexpr int LDS_BYTES = 2 * WST + 2 * PST;
  static_assert(NW * HALF * EPS * 4 <= LDS_BYTES, "epilogue staging exceeds the LDS allocation");
  static_assert(WI >= 1, "tile too small for the workgroup");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];
  uint8_t* const wbuf = lds;
  uint8_t* const pbuf = lds + 2 * WST;

  // (wave index in an SGPR: the LDS-DMA destinations (M0) are then scalar arithmetic)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-contiguous tile order (bijective for any nwg): the channel tiles of one row block, which
  // stage the same patch, share an L2
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = a.nwg >> 3, r8 = a.nwg & 7;
  const int rid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int mt = rid / a.n_tiles, nt = rid - mt * a.n_tiles;
  const int img = (mt / a.rblocks) * a.IMG, rb = mt - (mt / a.rblocks) * a.rblocks;
  const int y0 = rb * a.TR;
  // pixels of this tile that exist (a partial last multi-image tile has fewer images)
  const int pvalid = a.IMG > 1 ? min(a.P, (a.B - img) * a.H * a.W) : a.P;

  // ---- staging sources ----
  const int srow = lane >> 3, slot = lane & 7;
  int poff[PJ];  // element offset of this lane's 16-byte chunk of its patch row (block 0), or -1
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    const int wi = wave + NW * j;
    const int row = wi * 8 + srow;
    const int chunk = slot ^ ((row >> 1) & 7);
    poff[j] = -1;
    if (wi < NPJ && row < a.PR) {
      const int ii = row / a.PR1, r1 = row - ii * a.PR1;  // image of the tile, row within its patch
      const int py = r1 / a.PW, px = r1 - py * a.PW;
      const int yy = y0 - 1 + py, xx = px - 1;
      if ((unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W && img + ii < a.B)
        poff[j] = (((img + ii) * a.H + yy) * a.W + xx) * a.Cin + chunk * 8;
    }
  }
  // weight rows: a scalar base per step plus a 32-bit per-lane byte offset (the saddr form of
  // the LDS-DMA load: no 64-bit vector address arithmetic in the loop)
  const char* const wtile = reinterpret_cast<const char*>(a.w + (size_t)nt * BN * a.Kpad);
  int wlo[WI];
#pragma unroll
  for (int j = 0; j < WI; ++j) {
    const int row = (wave * WI + j) * 8 + srow;
    const int chunk = slot ^ ((row >> 1) & 7);
    wlo[j] = (row * a.Kpad + chunk * 8) * 2;
  }
  auto stage_patch = [&](int cb, uint8_t* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const int wi = wave + NW * j;
      if (wi < NPJ) {  // (wave-uniform)
        const void* src = poff[j] >= 0 ? (const void*)(a.x + poff[j] + cb * 64)
                                       : (const void*)(g_patch_zero + 16 * (lane & 3));
        glds16(src, buf + wi * 1024);
      }
    }
  };
  // step s = cb * SPB + tap: weight columns k = tap * Cin + cb * 64 (k = (kh*3 + kw)*Cin + ci)
  auto stage_w = [&](int s, uint8_t* buf) __attribute__((always_inline)) {
    const int cb = s / SPB, tap = s - cb * SPB;
    const char* const wk = wtile + (size_t)(tap * a.Cin + cb * 64) * 2;
#pragma unroll
    for (int j = 0; j < WI; ++j) glds16(wk + wlo[j], buf + (wave * WI + j) * 1024);
  };

  // ---- fragment geometry ----
  const int fr = lane & 15, fq = lane >> 4;
  int pbase[TM];  // patch row of the fragment row's pixel at tap (0, 0); -1 past the tile
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = wm * (kBM / WM) + i * 16 + fr;
    if (p < pvalid) {
      const int ii = p / (a.TR * a.W), q1 = p - ii * (a.TR * a.W);
      const int py = q1 / a.W;
      pbase[i] = ii * a.PR1 + py * a.PW + (q1 - py * a.W);
    } else {
      pbase[i] = -1;
    }
  }
  int wrow_off[TN], wsw[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int row = wn * (BN / WN) + t * 16 + fr;
    wrow_off[t] = row * 128;
    wsw[t] = (row >> 1) & 7;
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // X (patch) fragments of tap `tap` from patch buffer pc
  auto read_x = [&](const uint8_t* pc, int tap, bf16x8 (&bx)[2][TM])
      __attribute__((always_inline)) {
    const int kh = tap / 3;
    const int toff = kh * a.PW + (tap - kh * 3);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = pbase[i] >= 0 ? pbase[i] + toff : a.PR;  // (row PR: zeros)
      const int xo = row * 128, xs = (row >> 1) & 7;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        bx[kk][i] = *reinterpret_cast<const bf16x8*>(pc + xo + (((kk * 4 + fq) ^ xs) << 4));
    }
  };
  // One k-step (one tap of 64 input channels). The taps of one input block share its patch,
  // so the next tap's X fragments are read at the end of this step, before the barrier, and
  // only the weight fragments wait for the step's DMA; the next step's DMA is issued right
  // after those reads.
  auto step = [&](int s, bf16x8 (&bx)[2][TM], bf16x8 (&bn)[2][TM])
      __attribute__((always_inline)) {
    // step s has landed (vmcnt(0)); every wave is done with step s-1, whose weight buffer (and,
    // on a block's last tap, the previous block's patch buffer) is refilled below
    __syncthreads();
    const int cb = s / SPB, sl = s - cb * SPB;
    const uint8_t* wcur = wbuf + (s & 1) * WST;
    const uint8_t* pcur = pbuf + (cb & 1) * PST;
    if (sl == 0) read_x(pcur, 0, bx);  // a block's first tap: its patch has just landed
    bf16x8 af[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        af[kk][t] = *reinterpret_cast<const bf16x8*>(wcur + wrow_off[t] +
                                                     (((kk * 4 + fq) ^ wsw[t]) << 4));
    if (s + 1 < a.nsteps) {
      stage_w(s + 1, wbuf + ((s + 1) & 1) * WST);
      if (sl == SPB - 1) stage_patch(cb + 1, pbuf + ((cb + 1) & 1) * PST);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < TN; ++t)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][t], bx[kk][i], acc[i][t],
                                                              0, 0, 0);
    if (sl + 1 < SPB) read_x(pcur, sl + 1, bn);
  };
  bf16x8 xa[2][TM], xb[2][TM];
  stage_patch(0, pbuf);
  stage_w(0, wbuf);
  int s = 0;
  for (; s + 1 < a.nsteps; s += 2) {  // (two steps per iteration: the fragment sets alternate)
    step(s, xa, xb);
    step(s + 1, xb, xa);
  }
  if (s < a.nsteps) step(s, xa, xb);

  // ---- epilogue through LDS (as conv_gemm): fp32 (acc + bias) per wave, read back 8 channels
  // per lane, residual / ReLU, 16-byte bf16 stores of whole 128-byte rows ----
  __syncthreads();  // every wave is done with the last stages
  float* ep = reinterpret_cast<float*>(lds) + wave * HALF * EPS;
  const int c0 = nt * BN + wn * CW;
  const int pw0 = wm * (kBM / WM);
  const int m0 = (img * a.H + y0) * a.W;  // NHWC pixel index of tile pixel 0 (whole rows)
  const int cc = (lane % LPR) * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int cl = t * 16 + fq * 4;
      const float4 b = *reinterpret_cast<const float4*>(a.bias + c0 + cl);
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
      const int pr = j * RPI + lane / LPR;
      const int p = pw0 + h * HALF + pr;
      if (p < pvalid && c0 + cc < a.Cout) {
        const float* src = ep + pr * EPS + cc;
        const float4 lo = *reinterpret_cast<const float4*>(src);
        const float4 hi = *reinterpret_cast<const float4*>(src + 4);
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const size_t o = (size_t)(m0 + p) * a.Cout + c0 + cc;
        if (a.has_res) {
          const bf16x8 rr = ld_bf16x8(a.res + o);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)rr[e];
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        bf16x8 ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
        *reinterpret_cast<uint4*>(a.y + o) = __builtin_bit_cast(uint4, ov);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next half
  }
}

// the patch-row capacities compiled (2 workgroups per CU at BN = 128 up to 184 rows)
constexpr int kPrr[3] = {152, 184, 240};

int patch_tile_rows(const ConvDesc& d) {
  // largest divisor of H whose rows hold <= 128 pixels
  for (int tr = 128 / d.W; tr >= 1; --tr)
    if (d.H % tr == 0) return tr;
  return 0;
}

// whole images per tile: several when one image's rows fill less than half the tile (7x7: 2 x 49
// of 128 MFMA rows)
int patch_images(const ConvDesc& d, int tr) {
  if (tr != d.H) return 1;
  return std::max(1, 128 / (d.H * d.W));
}

int patch_prr(int PR) {
  for (int c : kPrr)
    if (PR + 1 <= c) return c;
  return 0;
}

int patch_bn(const ConvDesc& d) { return (d.Npad % 128 == 0) ? 128 : 64; }

}  // namespace

// conv_patch mode (set_conv_patch): 0 off, 1 (default) the 128-channel tiles (ResNet-50 28x28
// and 14x14 conv2: 90 -> 77 us and 86 -> 76 us per layer at batch 256), 2 also the 64-channel
// tiles (the 56x56 conv2 measured 104-110 -> 125-127 us there: one input block per tile leaves
// the patch load exposed, so those stay on conv_gemm; profiles/archive/r2_conv_patch.txt)
static std::atomic<int> g_conv_patch{1};

void set_conv_patch(int mode) { g_conv_patch = mode; }

bool conv_patch_supported(const ConvDesc& d, int batch, bool has_res) {
  if (!g_conv_patch.load(std::memory_order_relaxed) || conv_path() == 1) return false;
  if (d.stem || d.fp8 || d.f32 || d.in_f32 || d.out_f32) return false;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1) return false;
  if (d.Cin % 64 != 0 || d.K != 9 * d.Cin || d.Kpad != d.K) return false;
  if (d.Ho != d.H || d.Wo != d.W || d.W > 128 || d.Cout % 8 != 0) return false;
  const int bn = patch_bn(d);
  if (d.Npad % bn != 0 || d.Npad < d.Cout) return false;
  if (bn == 64 && g_conv_patch.load(std::memory_order_relaxed) < 2) return false;
  if (has_res && (d.res_C != d.Cout || d.res_stride != 1 || d.res_H != d.H || d.res_W != d.W))
    return false;
  const int tr = patch_tile_rows(d);
  const int img = tr >= 1 ? patch_images(d, tr) : 1;
  // (a tile below 3/4 of its MFMA rows wastes too much)
  if (tr < 1 || img * tr * d.W * 4 < 128 * 3 - 16) return false;
  const int prr = patch_prr(img * (tr + 2) * (d.W + 2));
  if (prr == 0 || (bn == 128 && prr > 184)) return false;
  return (long long)batch * d.H * d.W * d.Cin < (1ll << 31) &&
         (long long)batch * d.H * d.W * d.Cout < (1ll << 31);
}

hipError_t conv2d_patch(const ConvDesc& d, int batch, const void* x, const void* w,
                        const float* bias, const void* res, void* y, hipStream_t stream) {
  PatchArgs a;
  a.x = static_cast<const bf16*>(x);
  a.w = static_cast<const bf16*>(w);
  a.bias = bias;
  a.res = static_cast<const bf16*>(res);
  a.y = static_cast<bf16*>(y);
  a.H = d.H; a.W = d.W; a.Cin = d.Cin; a.Cout = d.Cout; a.Kpad = d.Kpad;
  const int bn = patch_bn(d);
  a.TR = patch_tile_rows(d);
  if (a.TR < 1) return hipErrorInvalidValue;
  a.IMG = patch_images(d, a.TR);
  a.B = batch;
  a.P = a.IMG * a.TR * d.W;
  a.PW = d.W + 2;
  a.PR1 = (a.TR + 2) * a.PW;
  a.PR = a.IMG * a.PR1;
  a.rblocks = d.H / a.TR;
  a.nsteps = 9 * (d.Cin / 64);  // k-steps: one tap of 64 input channels each
  a.relu = d.relu;
  a.has_res = d.has_res && res != nullptr;
  a.n_tiles = d.Npad / bn;
  a.nwg = (batch + a.IMG - 1) / a.IMG * a.rblocks * a.n_tiles;
  const int prr = patch_prr(a.PR);
  if (a.P > 128 || prr == 0) return hipErrorInvalidValue;
  if (bn == 128) {
    if (prr > 184) return hipErrorInvalidValue;
    if (prr == 152)
      hipLaunchKernelGGL((conv_patch_kernel<128, 152>), dim3(a.nwg), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((conv_patch_kernel<128, 184>), dim3(a.nwg), dim3(256), 0, stream, a);
  } else {
    if (prr == 152)
      hipLaunchKernelGGL((conv_patch_kernel<64, 152>), dim3(a.nwg), dim3(256), 0, stream, a);
    else if (prr == 184)
      hipLaunchKernelGGL((conv_patch_kernel<64, 184>), dim3(a.nwg), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((conv_patch_kernel<64, 240>), dim3(a.nwg), dim3(256), 0, stream, a);
  }
  return hipGetLastError();
}

}  // namespace gale
