// Whole-network CIFAR-10 ResNet-20 forward in ONE kernel: a workgroup carries an image through
// all 19 convolutions, the residual adds, the global pool, the dense layer and the softmax with
// every activation resident in LDS (BASELINE configs 2/3/5; SURVEY.md §7.5 hard part 3:
// "consider whole-block or whole-network fusion (persistent kernel)").
//
// Why: per-layer kernels at serving batch sizes (64-256 images) are latency bound — ~20 launches,
// each re-reading its input through L2 with a 9x implicit-im2col amplification and exposing a
// global-memory latency per K step. Here the only HBM traffic per image is its 12 KB fp32 input
// and 40 B of softmax output; weights (540 KB bf16 / 270 KB e4m3) stream from L2 as MFMA A
// fragments.
//
// Two instantiations:
//   bf16: v_mfma_f32_16x16x32_bf16, activations bf16 in LDS (76,576 B -> 2 workgroups per CU)
//   fp8 : v_mfma_f32_16x16x32_fp8_fp8, OCP e4m3 weights (per-channel scale) and activations
//         (per-tensor scales calibrated offline, gale/models/quant.py) -> 38,288 B of LDS
//         (half the bytes per B fragment). Epilogue: acc*wscale[c]*s_in + bias + res*s_res, ReLU,
//         requantise with 1/s_out (saturating at +-448).
// LDS plan (element offsets scale with the element size EB), NHWC with a zero border so the 3x3
// windows need no bounds checks (padded layouts Hp x Wp x C, see Layouts):
//            stage 1                    stage 2                        stage 3
//   R0 [0, 18496)       X1 34x34x16      X2 18x18x32 (after conv 7)     (X2: conv 14's shortcut)
//   R1 [18496, ...)     IN 34x34x3->T1   T2 18x18x32, SC 16x16x16       T3, X3 10x10x64
// SC is the option-A shortcut of block 2.1 (X1 subsampled, channels 0-15), copied out by conv 7
// so that X1 is dead once conv 7 is done and the padded stage-2 images fit.
// Block conv2 writes its output in place over its residual (each lane reads the residual of the
// pixel/channels it then writes, and no other lane reads that buffer in the same conv).
//
// MFMA mapping (same orientation as conv_mfma.hip): D[channel][pixel]; A = weights [Cout][Kpad]
// from global (k = (kh*3 + kw)*Cin + ci), hoisted into registers once per conv (each wave owns
// one 16-channel tile); B = 8 consecutive input channels of one tap of one pixel = one
// ds_read_b128 (bf16) / ds_read_b64 (fp8) from the padded LDS image. Each wave walks its pixel
// tiles four at a time (four independent accumulators).
//
// Reference parity: the model the reference serves is an opaque SavedModel fetched as
// "output/Softmax:0" (InferenceBolt.java:81-86); numerics equal the layer-by-layer gale plan
// (same rounding points) and are checked against the fp32 / fp8-emulation oracles in tests.
#include <stdlib.h>

#include "common.cuh"
#include "gale/kernels.h"
#include "java_float.cuh"

namespace gale {
namespace {

// Padded NHWC image layout in LDS: pixel (h, w) of a padded image starts at h * RP + w * PS
// elements (PS >= C: a pixel may be followed by unused elements, RP >= Wp * PS).
template <int PS_, int RP_>
struct Lay {
  static constexpr int PS = PS_, RP = RP_;
};
// Stage layouts (bf16). The B fragments of a 16-pixel tile are ds_read_b128s whose 16-lane
// groups must hit 16 distinct 16-B slots of the 256-B bank row (tools/lds_bank_model.py):
//   stage 2 pads each 32-channel pixel to 48 elements (96 B = six slots) and each row to 872
//     elements (109 slots): 0 extra cycles for stage 2 and for conv 13's stride-2 reads
//     (dense 64-B pixels: 4 and 12 extra LDS cycles per read);
//   stage 3 pads each 64-channel pixel to 80 elements (ten slots) and each row to 896 (dense: 12).
// fp8 uses the same element counts, i.e. half the bytes: its B fragments are ds_read_b64s whose
// 32-lane halves (lane groups g = 0,1 and 2,3 x 16 pixels) read a 16-B window per pixel, and
// pixel strides of 48 / 80 B (3 / 5 x 16 B, odd) put the 16 windows of a row on 16 distinct 16-B
// positions of the 256-B bank row; the row strides (872 B = 109 x 8 B: two rows for conv 13's
// stride-2 reads land on the other half of the positions; 896 B = 128 mod 256: stage 3's second
// tile row) keep multi-row tiles disjoint too. (Dense fp8 pixels of 32 / 64 B: 2- and 4-way, 14
// extra LDS cycles per LDS instruction measured, profiles/archive/r3_resnet20_fp8_lds.txt.)
template <bool F8>
struct Layouts {
  typedef Lay<16, 34 * 16> S1;  // 34x34x16
  typedef Lay<48, 872> S2;      // 18x18x32
  typedef Lay<80, 896> S3;      // 10x10x64
  typedef Lay<16, 16 * 16> SC;                        // 16x16x16 shortcut, no border
};

// element offsets (multiply by EB for bytes)
constexpr int kR0 = 0;
constexpr int kR1 = 18496;  // 34*34*16
template <bool F8>
struct Plan {
  typedef Layouts<F8> Ls;
  static constexpr int kX2 = kR0, kT2 = kR1;
  static constexpr int kSC = kT2 + 18 * Ls::S2::RP;
  static constexpr int kT3 = kR1, kX3 = kR1 + 10 * Ls::S3::RP;
  static constexpr int kEnd1 = kR1 + 34 * 34 * 16;
  static constexpr int kEnd2 = kSC + 16 * 16 * 16;
  static constexpr int kEnd3 = kX3 + 10 * Ls::S3::RP;
  static_assert(18 * Ls::S2::RP <= kR1, "X2 fits in R0");
};
constexpr int cmax(int a, int b) { return a > b ? a : b; }
// LDS elements per workgroup (the same bound serves both element sizes)
constexpr int kElems = cmax(cmax(Plan<false>::kEnd1, Plan<false>::kEnd2), Plan<false>::kEnd3);
static_assert(Plan<true>::kEnd2 <= kElems && Plan<true>::kEnd3 <= kElems, "fp8 plan fits");

template <bool F8>
struct Ty;
template <>
struct Ty<false> {
  typedef bf16 elem;
  typedef bf16x8 frag;
  static constexpr int EB = 2;
  static __device__ __forceinline__ frag ld(const elem* p) { return ld_bf16x8(p); }
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ void load4(const elem* p, float s, float* v) {
    const bf16x4 r = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(p));
    v[0] = (float)r[0]; v[1] = (float)r[1]; v[2] = (float)r[2]; v[3] = (float)r[3];
    (void)s;
  }
  static __device__ __forceinline__ void store4(elem* p, float q, float a, float b, float c,
                                                float d) {
    (void)q;
    bf16x4 o;
    o[0] = (bf16)a; o[1] = (bf16)b; o[2] = (bf16)c; o[3] = (bf16)d;
    *reinterpret_cast<uint2*>(p) = __builtin_bit_cast(uint2, o);
  }
  static __device__ __forceinline__ elem from_f32(float v, float q) {
    (void)q;
    return (bf16)v;
  }
  static __device__ __forceinline__ float to_f32(elem e) { return (float)e; }
  static __device__ __forceinline__ elem zero() { return (bf16)0.f; }
};
template <>
struct Ty<true> {
  typedef uint8_t elem;
  typedef long frag;
  static constexpr int EB = 1;
  static __device__ __forceinline__ frag ld(const elem* p) {
    return *reinterpret_cast<const long*>(p);
  }
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ void load4(const elem* p, float s, float* v) {
    const int r = *reinterpret_cast<const int*>(p);
    v[0] = __builtin_amdgcn_cvt_f32_fp8(r, 0) * s;
    v[1] = __builtin_amdgcn_cvt_f32_fp8(r, 1) * s;
    v[2] = __builtin_amdgcn_cvt_f32_fp8(r, 2) * s;
    v[3] = __builtin_amdgcn_cvt_f32_fp8(r, 3) * s;
  }
  static __device__ __forceinline__ float sat(float v) { return fminf(fmaxf(v, -448.f), 448.f); }
  static __device__ __forceinline__ void store4(elem* p, float q, float a, float b, float c,
                                                float d) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a * q), sat(b * q), 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c * q), sat(d * q), w, true);
    *reinterpret_cast<int*>(p) = w;
  }
  static __device__ __forceinline__ elem from_f32(float v, float q) {
    return (elem)(__builtin_amdgcn_cvt_pk_fp8_f32(sat(v * q), 0.f, 0, false) & 0xff);
  }
  static __device__ __forceinline__ float to_f32(elem e) {
    return __builtin_amdgcn_cvt_f32_fp8((int)e, 0);
  }
  static __device__ __forceinline__ elem zero() { return 0; }
};

// per-conv quantisation constants (fp8; identity for bf16)
struct Q {
  float deq;    // s_in (acc * wscale[c] * deq)
  float qout;   // 1 / s_out
  float res;    // s_res
};

template <bool F8>
__device__ __forceinline__ Q conv_q(const ResNet20Params& p, int i) {
  if constexpr (F8) return Q{p.s_in[i], 1.f / p.s_out[i], p.s_res[i]};
  (void)p; (void)i;
  return Q{1.f, 1.f, 1.f};
}

// ---- weight prefetch into LDS (8-wave form, one workgroup per CU: 84 KB of LDS spare) ----
// Every conv starts by hoisting its weights (A fragments) into registers; from global memory that
// is an L2/HBM round trip that all waves wait for together, ~19 times per image. In the 8-wave
// form the weights of conv i+1 are copied by LDS-DMA (global_load_lds_dwordx4) while conv i
// computes, so the hoist reads LDS. One 1 KiB wave-instruction per chunk (lanes past the end of
// the tensor are masked off). The copy pads each weight row: the hoist's ds_read_b128 has lane
// (g, col) read 16-B unit (row col, k-group g), and with the dense row of 20/36/72 units (a
// multiple of 4) rows 4 apart land on the same bank quad (2-, 2- and 4-way conflicts,
// tools/lds_bank_model.py --weights). A row stride of S = 2 (mod 4) units spreads the 16 lanes of
// every b128 group over 16 distinct quads. LDS-DMA writes lane l of a wave-instruction to unit
// 64c + l, so the padding is done on the source side: each lane fetches the global unit its LDS
// unit holds (pad units are masked off and never read).
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// padded LDS row stride (16-B units) of a weight row of `upr` units
__host__ __device__ constexpr int wrow_units(int upr) { return upr + ((2 - upr) & 3); }

// the largest conv weight (64 x 576 bf16) with padded rows
constexpr int kWeightLdsBytes = 64 * wrow_units(576 * 2 / 16) * 16;

// conv i's packed weight geometry: rows (Cout) and 16-B units per row (Kpad x EB / 16)
__device__ __forceinline__ int conv_w_rows(int i) { return i <= 6 ? 16 : i <= 12 ? 32 : 64; }
__device__ __forceinline__ int conv_w_upr(int i, int eb) {
  return (i <= 7 ? 160 : i <= 13 ? 288 : 576) * eb / 16;
}

template <int NW>
__device__ __forceinline__ void prefetch_weights(const void* src, int rows, int upr, void* dst) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int S = wrow_units(upr);
  const int units = rows * S;
  const float inv = 1.f / (float)S;
  for (int c = wave; c * 64 < units; c += NW) {
    const int u = c * 64 + lane;
    int row = (int)((float)u * inv);
    if (row * S > u) --row;
    else if ((row + 1) * S <= u) ++row;
    const int k = u - row * S;
    if (u < units && k < upr)
      __builtin_amdgcn_global_load_lds(
          (gbl_ptr_t)(static_cast<const char*>(src) + (row * upr + k) * 16),
          (lds_ptr_t)(static_cast<char*>(dst) + c * 1024), 16, 0, 0);
  }
}

struct WPf {
  void* wl;          // LDS weight buffer (nullptr: hoist from global, no prefetch)
  const void* next;  // weights of the next conv (nullptr: none)
  int next_rows, next_upr;
};

// MFMA accumulator -> store order: lane (g, col) holds channels g*4..+3 of tile pixel col; after
// the exchange of lane bits (2,3) <-> (4,5) lane l holds channel quad (l>>2)&3 of tile pixel
// (l>>4)*4 + (l&3), so each 16-lane ds_write_b64 group stores all quads of 4 pixels
__device__ __forceinline__ uint2 quad_transpose(uint2 w) {
  const int lane = threadIdx.x & 63;
  const int src = (((lane >> 2) & 3) << 4) | (((lane >> 4) & 3) << 2) | (lane & 3);
  w.x = (unsigned)__builtin_amdgcn_ds_bpermute(src << 2, (int)w.x);
  w.y = (unsigned)__builtin_amdgcn_ds_bpermute(src << 2, (int)w.y);
  return w;
}

// zero the one-pixel border of a padded Hp x Wp x C image in layout L (C * EB % 16 == 0); 8-B
// vectors when a row or pixel stride is not a multiple of 16 B (fp8 stage 2: 872-B rows)
template <bool F8, int NW, int HP, int WP, int C, class L>
__device__ __forceinline__ void zero_border(typename Ty<F8>::elem* buf) {
  constexpr int EB = Ty<F8>::EB;
  constexpr int VB = (L::RP * EB) % 16 == 0 && (L::PS * EB) % 16 == 0 ? 16 : 8;
  constexpr int V = C * EB / VB;  // vectors per cell
  constexpr int CELLS = 2 * WP + 2 * (HP - 2);
  for (int i = threadIdx.x; i < CELLS * V; i += 64 * NW) {
    const int cell = i / V, v = i - cell * V;
    int h, w;
    if (cell < WP) { h = 0; w = cell; }
    else if (cell < 2 * WP) { h = HP - 1; w = cell - WP; }
    else { const int r = cell - 2 * WP; h = 1 + (r >> 1); w = (r & 1) ? WP - 1 : 0; }
    char* dst = reinterpret_cast<char*>(buf + h * L::RP + w * L::PS) + v * VB;
    if constexpr (VB == 16)
      *reinterpret_cast<uint4*>(dst) = make_uint4(0, 0, 0, 0);
    else
      *reinterpret_cast<uint2*>(dst) = make_uint2(0, 0);
  }
}

// 3x3 pad-1 convolution LDS -> LDS with the folded-BN bias, optional residual and ReLU.
// RES: 0 none, 1 identity (same layout as out), 2 option-A shortcut from the previous stage's
// buffer (stride-2 subsample, channels >= RC are zero), 3 option-A shortcut from the SC copy
// (layout LR, no border), 4 none, and copy this stride-2 conv's option-A shortcut (channels
// < RC of the input at the subsampled pixels) to `res` in layout LR.
template <bool F8, int NW, int CIN, int COUT, int S, int HO, int RES, int RC, class LI, class LO,
          class LR>
__device__ __forceinline__ void conv3x3(const void* wgv, const float* __restrict__ wscale,
                                        const float* __restrict__ bias, Q q,
                                        const typename Ty<F8>::elem* in,
                                        typename Ty<F8>::elem* out,
                                        const typename Ty<F8>::elem* res, WPf pf) {
  typedef Ty<F8> T;
  typedef typename T::elem elem;
  const elem* wg = static_cast<const elem*>(NW == 8 ? pf.wl : wgv);
  constexpr int K = 9 * CIN;
  constexpr int KPAD = (K + 31) / 32 * 32;
  // weight row stride in elements: dense in global, padded in the LDS copy
  constexpr int WROW = NW == 8 ? wrow_units(KPAD * T::EB / 16) * 16 / T::EB : KPAD;
  constexpr int KS = KPAD / 32;
  constexpr int CT = COUT / 16;        // channel tiles
  constexpr int PT = HO * HO / 16;     // 16-pixel tiles
  constexpr int WPC = NW / CT;         // waves per channel tile
  constexpr int PTW = PT / WPC;        // pixel tiles per wave
  constexpr int G = PTW < 4 ? PTW : 4;  // independent accumulators per pass
  static_assert(WPC >= 1 && PTW >= 1 && PTW % G == 0, "wave partition of the conv");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int ct = wave / WPC;
  const int pt0 = (wave % WPC) * PTW;

  typename T::frag afr[KS];
  int koff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = ks * 32 + g * 8;
    afr[ks] = T::ld(wg + (ct * 16 + col) * WROW + k);
    int tap = k / CIN;
    const int ci = k - tap * CIN;
    if (tap >= 9) tap = 0;  // K padding: zero weights, any finite input
    koff[ks] = (tap / 3) * LI::RP + (tap % 3) * LI::PS + ci;
  }
  const int c0 = ct * 16 + g * 4;  // this lane's 4 output channels
  const float4 bv = *reinterpret_cast<const float4*>(bias + c0);
  float4 sc = make_float4(1.f, 1.f, 1.f, 1.f);
  if constexpr (F8) {
    sc = *reinterpret_cast<const float4*>(wscale + c0);
    sc.x *= q.deq; sc.y *= q.deq; sc.z *= q.deq; sc.w *= q.deq;
  }
  if (pf.wl) {
    // A fragments and epilogue constants in registers (no plain load may be pending once the
    // DMA is in flight), every wave done reading the buffer, then refill it for the next conv
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (pf.next) prefetch_weights<NW>(pf.next, pf.next_rows, pf.next_upr, pf.wl);
  }

#pragma unroll 1
  for (int pg = 0; pg < PTW; pg += G) {
    int pbase[G], ho[G], wo[G];
#pragma unroll
    for (int p = 0; p < G; ++p) {
      const int m = (pt0 + pg + p) * 16 + col;
      ho[p] = m / HO;
      wo[p] = m - ho[p] * HO;
      pbase[p] = ho[p] * S * LI::RP + wo[p] * S * LI::PS;
    }
    f32x4 acc[G];
#pragma unroll
    for (int p = 0; p < G; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      typename T::frag b[G];
#pragma unroll
      for (int p = 0; p < G; ++p) b[p] = T::ld(in + pbase[p] + koff[ks]);
#pragma unroll
      for (int p = 0; p < G; ++p) acc[p] = T::mma(afr[ks], b[p], acc[p]);
      // bound how far the scheduler hoists LDS reads (register pressure -> occupancy)
      if (ks % 3 == 2) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int p = 0; p < G; ++p) {
      float v0 = acc[p][0] * sc.x + bv.x, v1 = acc[p][1] * sc.y + bv.y;
      float v2 = acc[p][2] * sc.z + bv.z, v3 = acc[p][3] * sc.w + bv.w;
      const int o = (ho[p] + 1) * LO::RP + (wo[p] + 1) * LO::PS + c0;
      if (RES == 1 || ((RES == 2 || RES == 3) && c0 < RC)) {
        const int ro = RES == 1   ? o
                       : RES == 2 ? (2 * ho[p] + 1) * LR::RP + (2 * wo[p] + 1) * LR::PS + c0
                                  : ho[p] * LR::RP + wo[p] * LR::PS + c0;
        float r[4];
        T::load4(res + ro, q.res, r);
        v0 += r[0]; v1 += r[1]; v2 += r[2]; v3 += r[3];
      }
      if (RES == 4 && c0 < RC) {  // raw copy: same quantisation scale on both sides
        const elem* src = in + (2 * ho[p] + 1) * LI::RP + (2 * wo[p] + 1) * LI::PS + c0;
        elem* dst = const_cast<elem*>(res) + ho[p] * LR::RP + wo[p] * LR::PS + c0;
        if constexpr (F8)
          *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(src);
        else
          *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(src);
      }
      if constexpr (!F8) {
        // The accumulator puts lane (g, col) on channels g*4..+3 of pixel col: a 16-lane
        // ds_write_b64 group would store one channel quad of 16 pixels, 4-way (8-way for 64-B
        // pixels) on the 32-bank store rule. Exchange lane bits (2,3) <-> (4,5) first
        // (ds_bpermute), so a group stores all four quads of 4 consecutive pixels: 128
        // contiguous bytes for 32-B pixels (stage 1), distinct banks for the padded 160-B
        // pixels (stage 3), 2-way for 64-B pixels (stage 2).
        bf16x4 ov;
        ov[0] = (bf16)fmaxf(v0, 0.f); ov[1] = (bf16)fmaxf(v1, 0.f);
        ov[2] = (bf16)fmaxf(v2, 0.f); ov[3] = (bf16)fmaxf(v3, 0.f);
        const uint2 w = quad_transpose(__builtin_bit_cast(uint2, ov));
        const int mt = (pt0 + pg + p) * 16 + ((lane >> 4) << 2) + (lane & 3);
        const int hot = mt / HO, wot = mt - hot * HO;
        const int ot = (hot + 1) * LO::RP + (wot + 1) * LO::PS + ct * 16 + ((lane >> 2) & 3) * 4;
        *reinterpret_cast<uint2*>(out + ot) = w;
      } else {
        T::store4(out + o, q.qout, fmaxf(v0, 0.f), fmaxf(v1, 0.f), fmaxf(v2, 0.f),
                  fmaxf(v3, 0.f));
      }
    }
  }
  // the next conv's weights have landed before the caller's barrier
  if (pf.wl && pf.next) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// stem: 3x3x3 -> 16 over the 34x34x3 padded input (K = 27 padded to 32: one k step, the 8
// k-values of a lane are 8 scalar LDS reads)
template <bool F8, int NW>
__device__ __forceinline__ void stem(const void* wgv, const float* __restrict__ wscale,
                                     const float* __restrict__ bias, Q q,
                                     const typename Ty<F8>::elem* in,
                                     typename Ty<F8>::elem* out) {
  typedef Ty<F8> T;
  typedef typename T::elem elem;
  const elem* wg = static_cast<const elem*>(wgv);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, col = lane & 15;
  const typename T::frag a = T::ld(wg + col * 32 + g * 8);
  int off[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = g * 8 + j;
    const int tap = k < 27 ? k / 3 : 0, ci = k < 27 ? k % 3 : 0;
    off[j] = ((tap / 3) * 34 + tap % 3) * 3 + ci;
  }
  const float4 bv = *reinterpret_cast<const float4*>(bias + g * 4);
  float4 sc = make_float4(1.f, 1.f, 1.f, 1.f);
  if constexpr (F8) {
    sc = *reinterpret_cast<const float4*>(wscale + g * 4);
    sc.x *= q.deq; sc.y *= q.deq; sc.z *= q.deq; sc.w *= q.deq;
  }
  constexpr int TPW = 64 / NW;  // 16-pixel tiles per wave (64 tiles of 32x32)
#pragma unroll 1
  for (int pg = 0; pg < TPW; pg += 4) {
    f32x4 acc[4];
    int ho[4], wo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int m = (wave * TPW + pg + p) * 16 + col;
      ho[p] = m >> 5;
      wo[p] = m & 31;
      const elem* px = in + (ho[p] * 34 + wo[p]) * 3;
      typename T::frag b;
      if constexpr (F8) {
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) v |= (uint64_t)px[off[j]] << (8 * j);
        b = (long)v;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = px[off[j]];
      }
      acc[p] = T::mma(a, b, f32x4{0.f, 0.f, 0.f, 0.f});
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float v0 = fmaxf(acc[p][0] * sc.x + bv.x, 0.f), v1 = fmaxf(acc[p][1] * sc.y + bv.y, 0.f);
      const float v2 = fmaxf(acc[p][2] * sc.z + bv.z, 0.f), v3 = fmaxf(acc[p][3] * sc.w + bv.w, 0.f);
      if constexpr (!F8) {  // 128 contiguous bytes per ds_write_b64 group (see quad_transpose)
        bf16x4 ov;
        ov[0] = (bf16)v0; ov[1] = (bf16)v1; ov[2] = (bf16)v2; ov[3] = (bf16)v3;
        const uint2 w = quad_transpose(__builtin_bit_cast(uint2, ov));
        const int mt = (wave * TPW + pg + p) * 16 + ((lane >> 4) << 2) + (lane & 3);
        *reinterpret_cast<uint2*>(out + ((mt >> 5) + 1) * 34 * 16 + ((mt & 31) + 1) * 16 +
                                  ((lane >> 2) & 3) * 4) = w;
      } else {
        T::store4(out + ((ho[p] + 1) * 34 + wo[p] + 1) * 16 + g * 4, q.qout, v0, v1, v2, v3);
      }
    }
  }
}

// NW waves per workgroup (one image per workgroup): 4 waves with 2 workgroups per CU, or 8 waves
// with one workgroup per CU (every SIMD still runs 2 waves, but each image has twice the waves:
// half the per-image latency when images are fewer than workgroup slots)
template <bool F8, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void resnet20_fused_kernel(ResNet20Params p,
                                                                         const float* x,
                                                                         float* out, int batch,
                                                                         InputTable tab) {
  typedef Ty<F8> T;
  typedef typename T::elem elem;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  elem* base = reinterpret_cast<elem*>(smem);
  elem* X1 = base + kR0;
  elem* T1 = base + kR1;
  elem* IN = base + kR1;
  typedef Plan<F8> PL;
  elem* T2 = base + PL::kT2;
  elem* X2 = base + PL::kX2;
  elem* SC = base + PL::kSC;
  elem* T3 = base + PL::kT3;
  elem* X3 = base + PL::kX3;
  typedef typename Layouts<F8>::S1 L1;
  typedef typename Layouts<F8>::S2 L2;
  typedef typename Layouts<F8>::S3 L3;
  float* scratch = reinterpret_cast<float*>(base + kR0);
  // 8-wave form: weights of the next conv prefetched into LDS behind the activations
  void* wl = NW == 8 ? static_cast<void*>(smem + kElems * T::EB) : nullptr;
  auto pfw = [&](int i) {
    WPf f;
    f.wl = wl;
    f.next = i < 18 ? p.w[i + 1] : nullptr;
    f.next_rows = i < 18 ? conv_w_rows(i + 1) : 0;
    f.next_upr = i < 18 ? conv_w_upr(i + 1, T::EB) : 0;
    return f;
  };
  const float in_q = F8 ? 1.f / p.s_in[0] : 1.f;  // quantisation of the fp32 network input

  if (p.so.status_out && blockIdx.x == 0) step_verdicts(p.so);  // (the parse is done)
  if (p.batch_dev) batch = min(batch, *p.batch_dev);  // (a captured step graph's batch size)
  for (int img = blockIdx.x; img < batch; img += gridDim.x) {
    __syncthreads();  // the previous image's head is done with R0/R1
    // ---- stage the fp32 input image into the zero-bordered 34x34x3 IN ----
    for (int i = threadIdx.x; i < 34 * 34 * 3; i += 64 * NW) {
      const int cell = i / 3;
      const int h = cell / 34, w = cell - h * 34;
      if (h == 0 || h == 33 || w == 0 || w == 33) IN[i] = T::zero();
    }
    zero_border<F8, NW, 34, 34, 16, L1>(X1);
    const float* src =
        tab.base[0] ? tab.base[tab.code[img] >> 24] + (size_t)(tab.code[img] & 0xffffffu) * 3072
        : p.xs      ? p.xs[img]
                    : x + (size_t)img * 3072;
    const float4* xi = reinterpret_cast<const float4*>(src);
    for (int i = threadIdx.x; i < 768; i += 64 * NW) {
      const float4 v = xi[i];
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int idx = i * 4 + j;  // (h*32 + w)*3 + c
        const int pix = idx / 3, c = idx - pix * 3;
        const int h = pix >> 5, w = pix & 31;
        IN[((h + 1) * 34 + w + 1) * 3 + c] = T::from_f32(e[j], in_q);
      }
    }
    __syncthreads();
    stem<F8, NW>(p.w[0], p.ws[0], p.b[0], conv_q<F8>(p, 0), IN, X1);
    if (wl) {  // conv 1's weights land during the barrier below and the border zeroing
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      prefetch_weights<NW>(p.w[1], conv_w_rows(1), conv_w_upr(1, T::EB), wl);
    }
    __syncthreads();
    zero_border<F8, NW, 34, 34, 16, L1>(T1);  // IN is dead; T1's border overlaps its bytes
    // ---- stage 1: 32x32x16 ----
#pragma unroll 1
    for (int blk = 0; blk < 3; ++blk) {
      const int c1 = 1 + 2 * blk, c2 = c1 + 1;
      conv3x3<F8, NW, 16, 16, 1, 32, 0, 16, L1, L1, L1>(p.w[c1], p.ws[c1], p.b[c1], conv_q<F8>(p, c1), X1, T1,
                                        nullptr, pfw(c1));
      __syncthreads();
      conv3x3<F8, NW, 16, 16, 1, 32, 1, 16, L1, L1, L1>(p.w[c2], p.ws[c2], p.b[c2], conv_q<F8>(p, c2), T1, X1,
                                        X1, pfw(c2));
      __syncthreads();
    }
    // ---- stage 2: 16x16x32 ----
    typedef typename Layouts<F8>::SC LS;
    zero_border<F8, NW, 18, 18, 32, L2>(T2);
    // conv 7 also copies block 2.1's shortcut out of X1 into SC: X1 is dead after it
    conv3x3<F8, NW, 16, 32, 2, 16, 4, 16, L1, L2, LS>(p.w[7], p.ws[7], p.b[7], conv_q<F8>(p, 7), X1, T2, SC, pfw(7));
    __syncthreads();
    zero_border<F8, NW, 18, 18, 32, L2>(X2);  // X2 lives where X1 was
    conv3x3<F8, NW, 32, 32, 1, 16, 3, 16, L2, L2, LS>(p.w[8], p.ws[8], p.b[8], conv_q<F8>(p, 8), T2, X2, SC, pfw(8));
    __syncthreads();
#pragma unroll 1
    for (int blk = 1; blk < 3; ++blk) {
      const int c1 = 7 + 2 * blk, c2 = c1 + 1;
      conv3x3<F8, NW, 32, 32, 1, 16, 0, 32, L2, L2, L2>(p.w[c1], p.ws[c1], p.b[c1], conv_q<F8>(p, c1), X2, T2,
                                        nullptr, pfw(c1));
      __syncthreads();
      conv3x3<F8, NW, 32, 32, 1, 16, 1, 32, L2, L2, L2>(p.w[c2], p.ws[c2], p.b[c2], conv_q<F8>(p, c2), T2, X2,
                                        X2, pfw(c2));
      __syncthreads();
    }
    // ---- stage 3: 8x8x64 ----
    zero_border<F8, NW, 10, 10, 64, L3>(T3);
    zero_border<F8, NW, 10, 10, 64, L3>(X3);
    conv3x3<F8, NW, 32, 64, 2, 8, 0, 32, L2, L3, L2>(p.w[13], p.ws[13], p.b[13], conv_q<F8>(p, 13), X2, T3,
                                     nullptr, pfw(13));
    __syncthreads();
    conv3x3<F8, NW, 64, 64, 1, 8, 2, 32, L3, L3, L2>(p.w[14], p.ws[14], p.b[14], conv_q<F8>(p, 14), T3, X3, X2, pfw(14));
    __syncthreads();
#pragma unroll 1
    for (int blk = 1; blk < 3; ++blk) {
      const int c1 = 13 + 2 * blk, c2 = c1 + 1;
      conv3x3<F8, NW, 64, 64, 1, 8, 0, 64, L3, L3, L3>(p.w[c1], p.ws[c1], p.b[c1], conv_q<F8>(p, c1), X3, T3,
                                       nullptr, pfw(c1));
      __syncthreads();
      conv3x3<F8, NW, 64, 64, 1, 8, 1, 64, L3, L3, L3>(p.w[c2], p.ws[c2], p.b[c2], conv_q<F8>(p, c2), T3, X3,
                                       X3, pfw(c2));
      __syncthreads();
    }
    // ---- head: global average pool (8x8) -> dense 64 -> 10 -> softmax ----
    {
      constexpr int PPW = 64 / NW;  // pooled pixels per wave
      const int c = threadIdx.x & 63, qq = threadIdx.x >> 6;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int pix = qq * PPW + i;
        const int h = pix >> 3, w = pix & 7;
        s += T::to_f32(X3[(h + 1) * L3::RP + (w + 1) * L3::PS + c]);
      }
      scratch[qq * 64 + c] = s;  // R0 is free in stage 3's last block (X2 is dead)
      __syncthreads();
      if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const float pool_scale = (F8 ? p.s_out[18] : 1.f) * (1.f / 64.f);
        float acc = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) acc += scratch[w * 64 + lane];
        const float pooled = acc * pool_scale;
        float logit = -3.0e38f;
        for (int o = 0; o < 10; ++o) {
          const float t = wave_sum(p.fc_w[o * 64 + lane] * pooled);
          if (lane == o) logit = t + p.fc_b[o];
        }
        const float mx = wave_max(lane < 10 ? logit : -3.0e38f);
        const float e = lane < 10 ? __expf(logit - mx) : 0.f;
        const float sum = wave_sum(e);
        if (lane < 10) {
          const float prob = e / sum;
          out[(size_t)img * 10 + lane] = prob;
          // the prediction text in the epilogue (no separate formatting launch per batch)
          if (p.so.text)
            static_cast<uint4*>(p.so.text)[(size_t)img * 10 + lane] = java_float_slot(prob);
        }
      }
    }
  }
}

}  // namespace

hipError_t resnet20_fused_forward(const ResNet20Params& p, int batch, const float* x, float* out,
                                  hipStream_t stream, const InputTable* tab) {
  if (batch <= 0) return hipSuccess;
  static const InputTable kNoTable{};
  if (tab && (batch > kInputTableImages || !tab->base[0])) return hipErrorInvalidValue;
  const InputTable& t = tab ? *tab : kNoTable;
  const bool f8 = p.fp8 != 0;
  if (f8) {
    for (int i = 0; i < 19; ++i)
      if (p.ws[i] == nullptr || !(p.s_in[i] > 0.f) || !(p.s_out[i] > 0.f))
        return hipErrorInvalidValue;
  }
  // (C++11 magic statics: initialised once, thread-safe, as replica workers launch concurrently)
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  // resident workgroups per CU: 2 of 4 waves (bf16: LDS bound; fp8: register bound — its 39 KB
  // of LDS would allow 4, but the hoisted A fragments need more than 128 VGPRs per lane), or 1 of
  // 8 waves. The 4-wave form is the default for both: alone a bf16 batch of <= 256 images is
  // ~8 % faster on 8 waves (52.6 vs 56.9 us at 256; weights prefetched into LDS), but that
  // workgroup takes a CU's whole register file and ~150 KB of its LDS, so nothing else runs
  // beside it. On 4 waves (one per SIMD, 77 KB) two batches share the CUs (2 in flight: 36.6 vs
  // 52.6 us per batch) and the GPU ingest's passes run beside a forward (count / parse 18-21 /
  // 22-25 us vs 25-30 / 27-31 us per fetch under load); config 2 end to end: img/s higher in 4
  // of 6 interleaved pairs, p50 equal (profiles/r6_ab_r20_waves.jsonl). GALE_R20_WAVES=8 selects
  // the 8-wave form for bf16 batches of at most one image per CU (A/B).
  static const bool want8 = [] {
    const char* e = getenv("GALE_R20_WAVES");
    return e && atoi(e) == 8;
  }();
  const int nw = !f8 && batch <= cus && want8 ? 8 : 4;
  const int grid_cap = nw == 8 ? cus : 2 * cus;
  const int grid = batch < grid_cap ? batch : grid_cap;
  const size_t lds = (size_t)kElems * (f8 ? 1 : 2) + (nw == 8 ? (size_t)kWeightLdsBytes : 0);
  const dim3 block(64 * nw);
  if (f8) {
    hipLaunchKernelGGL((resnet20_fused_kernel<true, 4>), dim3(grid), block, lds, stream, p, x,
                       out, batch, t);
  } else if (nw == 8) {
    hipLaunchKernelGGL((resnet20_fused_kernel<false, 8>), dim3(grid), block, lds, stream, p, x,
                       out, batch, t);
  } else {
    hipLaunchKernelGGL((resnet20_fused_kernel<false, 4>), dim3(grid), block, lds, stream, p, x,
                       out, batch, t);
  }
  return hipGetLastError();
}

}  // namespace gale
