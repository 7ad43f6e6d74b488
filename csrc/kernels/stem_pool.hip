// ResNet-50 ImageNet stem (7x7/2 conv, 3 -> 64, folded BN, ReLU) and the 3x3/2 max-pool after
// it in ONE kernel (bf16, BASELINE config 4): the 112x112x64 stem output (411 MB at batch 256)
// never goes to HBM.
//
// Layered, the stem GEMM (conv_gemm's packed-stem form) writes that tensor and the max-pool reads
// it back: 242 + 113 us at batch 256 (profiles/r5_resnet50_layers.txt), both bound by the
// 0.5 GB of traffic rather than by their MFMA work (17 % busy).
//
// A workgroup (8 waves, 1 per CU) owns PR = 4 pooled rows (all 56 columns) of one image. It
// computes the 2 * PR + 1 = 9 stem rows those windows cover, all 112 columns (1008 pixels: 12.5 %
// more stem work than the pooled rows own, the shared window row), into LDS, then max-pools
// from LDS. The packed input image (stem_pack: bf16 [224][230][4], 3 zero columns left) makes
// each kernel row of an output pixel one 64-byte run, so an MFMA B fragment (16 pixels x 32 k =
// one kernel row) is a 16-byte global load per lane, two k-steps ahead; the weights (64 x 256,
// 32 KB) sit in LDS. The stem output is ReLU'd (>= 0), so the pool's implicit padding is the same
// as skipping the out-of-image window taps, which is what the epilogue does.
// LDS: weights 32 KB + the stem tile 1008 x 128 B = 158 KB. Grid: batch x 14 strips,
// XCD-contiguous (neighbouring strips of an image share input rows in one L2).
#include "common.cuh"
#include "gale/kernels.h"

namespace gale {
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __attribute__((aligned(16))) uint8_t g_stem_zero[64];

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src), (lds_ptr_t)(lds_base), 16, 0, 0);
}

constexpr int kIH = 224, kIW = 230;      // packed input image
constexpr int kSO = 112, kPO = 56;       // stem output / pooled output side
constexpr int kC = 64, kK = 256;         // channels, GEMM depth (8x8x4 packed kernel)
constexpr int kPR = 4;                   // pooled rows per workgroup
constexpr int kSR = 2 * kPR + 1;         // stem rows per workgroup
constexpr int kNT = kSR * kSO / 16;      // 63 pixel tiles of 16
constexpr int kStrips = kPO / kPR;       // 14
constexpr int kWBytes = kK / 64 * kC * 128;  // 32 KB: 4 k-blocks x 64 rows x 128 B
constexpr int kTileBytes = kSR * kSO * 128;  // 129,024
static_assert(kSR * kSO % 16 == 0 && kPO % kPR == 0, "tile geometry");
static_assert(kWBytes + kTileBytes <= 163840, "LDS");

__device__ __forceinline__ int rkey(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swz(int row, int c) { return row * 128 + ((c ^ rkey(row)) << 4); }

struct StemPoolArgs {
  const bf16* x;   // [B][224][230][4]
  const bf16* w;   // [64][256], k = kh * 32 + kw * 4 + c
  const float* b;  // [64]
  bf16* y;         // [B][56][56][64]
  int nwg;
};

__global__ __launch_bounds__(512, 1) void stem_pool_kernel(StemPoolArgs a) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[kWBytes + kTileBytes];
  uint8_t* const wl = lds;
  uint8_t* const tile = lds + kWBytes;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = a.nwg >> 3, r8 = a.nwg & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int n = rid / kStrips, a0 = (rid - n * kStrips) * kPR;  // first pooled row
  const int ho0 = 2 * a0 - 1;                                   // stem row of tile row 0

  // weights -> LDS: 256 rows (k-block * 64 + channel) of 128 B, 32 wave-instructions
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int wi = wave * 4 + j;
    const int row = wi * 8 + (lane >> 3);
    const int kb = row >> 6, ch = row & 63;
    const int c = (lane & 7) ^ rkey(row);
    glds16(a.w + ch * kK + kb * 64 + c * 8, wl + wi * 1024);
  }

  __syncthreads();  // weights landed
  // this wave's pixel tiles t = wave + 8 s (63 tiles: waves 0..6 own 8, wave 7 owns 7), in two
  // passes of 4 (registers)
  constexpr int NS = 4;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    const bool last = pass == 0 || wave + 8 * 7 < kNT;  // (s = 7 exists for waves 0..6)
    int pbase[NS];  // element offset of (pixel, image row 0, lane's 16-B piece)
    int hrow[NS];   // input row of kernel row 0
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int t = wave + 8 * (pass * NS + u);
      const int q = (t < kNT ? t : 0) * 16 + fr;  // tile pixel: row q / 112, column q % 112
      const int r = q / kSO, wo = q - r * kSO;
      hrow[u] = 2 * (ho0 + r) - 3;
      pbase[u] = ((n * kIH) * kIW + 2 * wo) * 4 + fq * 8;
    }
    auto xsrc = [&](int u, int c) __attribute__((always_inline)) -> const bf16* {
      const int hi = hrow[u] + c;
      return (unsigned)hi < (unsigned)kIH
                 ? a.x + pbase[u] + hi * (kIW * 4)
                 : reinterpret_cast<const bf16*>(g_stem_zero) + (fq & 3) * 8;
    };
    auto live = [&](int u) __attribute__((always_inline)) { return u < NS - 1 || last; };
    f32x4 acc[NS][4];
#pragma unroll
    for (int u = 0; u < NS; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[u][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 xf[2][NS];
#pragma unroll
    for (int u = 0; u < NS; ++u)
      if (live(u)) xf[0][u] = ld_bf16x8(xsrc(u, 0));
#pragma unroll
    for (int c = 0; c < kK / 32; ++c) {  // k-step c = kernel row c
      if (c + 1 < kK / 32) {
#pragma unroll
        for (int u = 0; u < NS; ++u)
          if (live(u)) xf[(c + 1) & 1][u] = ld_bf16x8(xsrc(u, c + 1));
      }
      bf16x8 wf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wf[j] = *reinterpret_cast<const bf16x8*>(wl + swz((c >> 1) * 64 + j * 16 + fr,
                                                         (c & 1) * 4 + fq));
#pragma unroll
      for (int u = 0; u < NS; ++u)
        if (live(u))
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[c & 1][u], acc[u][j],
                                                                0, 0, 0);
    }
    // bias + ReLU -> bf16 stem tile in LDS (row = tile pixel, 128 B)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 bv = *reinterpret_cast<const float4*>(a.b + j * 16 + fq * 4);
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        if (live(u)) {
          const int q = (wave + 8 * (pass * NS + u)) * 16 + fr;
          bf16x4 o;
          o[0] = (bf16)fmaxf(acc[u][j][0] + bv.x, 0.f);
          o[1] = (bf16)fmaxf(acc[u][j][1] + bv.y, 0.f);
          o[2] = (bf16)fmaxf(acc[u][j][2] + bv.z, 0.f);
          o[3] = (bf16)fmaxf(acc[u][j][3] + bv.w, 0.f);
          *reinterpret_cast<uint2*>(tile + swz(q, 2 * j + (fq >> 1)) + (fq & 1) * 8) =
              __builtin_bit_cast(uint2, o);
        }
      }
    }
  }
  __syncthreads();

  // 3x3 / 2 max-pool of the tile: item = (pooled row, pooled column, 8-channel chunk); taps
  // outside the stem output (row -1, column -1) are skipped (values >= 0: same as padding)
  for (int it = tid; it < kPR * kPO * 8; it += 512) {
    const int cg = it & 7, pix = it >> 3;
    const int py = pix / kPO, px = pix - py * kPO;
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = 0.f;
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
      const int r = 2 * py + dr;  // tile row (stem row ho0 + r)
      if (ho0 + r < 0) continue;
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) {
        const int wo = 2 * px - 1 + dc;
        if (wo < 0) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(tile + swz(r * kSO + wo, cg));
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)v[e]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)m[e];
    *reinterpret_cast<uint4*>(a.y + ((size_t)(n * kPO + a0 + py) * kPO + px) * kC + cg * 8) =
        __builtin_bit_cast(uint4, o);
  }
}

}  // namespace

bool stem_pool_supported(const ConvDesc& d, int H, int W, int C, int k, int s, int p, int Ho,
                         int Wo) {
  return d.stem && !d.fp8 && !d.f32 && !d.out_f32 && d.relu && !d.has_res && d.H == kIH &&
         d.W == kIW && d.Ho == kSO && d.Wo == kSO && d.Cout == kC && d.Npad == kC &&
         d.K == kK && d.Kpad == kK && H == kSO && W == kSO && C == kC && k == 3 && s == 2 &&
         p == 1 && Ho == kPO && Wo == kPO;
}

hipError_t stem_pool(int batch, const void* x, const void* w, const float* bias, void* y,
                     hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  if (!x || !w || !bias || !y) return hipErrorInvalidValue;
  // 32-bit element offsets in the kernel: launch chunks of <= 4096 images (any max_batch)
  constexpr int kChunk = 4096;
  static_assert((long long)kChunk * kIH * kIW * 4 < (1ll << 31), "chunk offsets");
  for (int c0 = 0; c0 < batch; c0 += kChunk) {
    const int nb = batch - c0 < kChunk ? batch - c0 : kChunk;
    StemPoolArgs a;
    a.x = static_cast<const bf16*>(x) + (size_t)c0 * kIH * kIW * 4;
    a.w = static_cast<const bf16*>(w);
    a.b = bias;
    a.y = static_cast<bf16*>(y) + (size_t)c0 * kPO * kPO * kC;
    a.nwg = nb * kStrips;
    hipLaunchKernelGGL(stem_pool_kernel, dim3(a.nwg), dim3(512), 0, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace gale
