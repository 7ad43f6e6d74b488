// Host-visible declarations of the gale CDNA4 (gfx950) kernels.
//
// Every tensor is NHWC. Activations are bf16, the network input is fp32 (as parsed from the
// InstObj JSON contract, /root/reference/src/main/java/dke/model/data/InstObj.java:8) and the
// network output is the fp32 softmax (the reference fetches "output/Softmax:0",
// /root/reference/src/main/java/dke/model/InferenceBolt.java:83).
//
// These launchers never allocate or synchronise, so they can be captured into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gale {

// Geometry of one convolution (or fully connected layer expressed as a 1x1 convolution over a
// 1x1 image). Independent of the batch size, which is a launch argument so one descriptor serves
// every hipGraph batch bucket.
struct ConvDesc {
  int H, W, Cin;        // input spatial size and channel count (channel stride of the input)
  int Ho, Wo, Cout;     // output spatial size; Cout = stored output channels (channel stride of y)
  int KH, KW, stride, pad;
  int K;                // true reduction length KH*KW*Cin
  int Kpad;             // K rounded up to 32 (row stride of the packed weights)
  int Npad;             // rows of the packed weight matrix (multiple of the n-block)
  int relu;             // apply ReLU in the epilogue
  // residual added before the ReLU (ResNet shortcut). res_C < Cout zero-pads the extra channels
  // and res_stride > 1 subsamples: together they are the parameter-free "option A" shortcut.
  int has_res, res_H, res_W, res_C, res_stride;
  int in_f32;           // input tensor is fp32 (network input; converted to bf16 while staging)
  int out_f32;          // output tensor is fp32 (classifier logits)
  int fp8;              // OCP e4m3 operands (fp8 MFMA path): weights per-channel (wscale),
                        // activations per tensor (value = code * scale)
  float in_scale;       // fp8: input scale (in_f32: the input is quantised with this step)
  float out_scale;      // fp8: output scale (ignored for out_f32)
  float res_scale;      // fp8: residual scale
  // 1 = packed-stem layout (ResNet-50 7x7/2 stem, bf16): x is the stem_pack() image
  // [B][H][W][4] bf16 with W = 2*Wo + 6 (3 zero columns left, the rest right), the packed weights
  // are [Npad][256] with k = kh*32 + kw*4 + c over an 8x8x4 zero-padded kernel (KH = KW = 8,
  // K = Kpad = 256), so each kernel row of one output pixel is ONE 64-byte run of x.
  int stem;
  // 1 = reference-precision plan (--dtype fp32): x, w, residual and y are all fp32 and the conv
  // runs on the fp32 matrix core (conv_f32.hip, v_mfma_f32_16x16x4_f32); Kpad % 16 == 0
  int f32;
};

// y[B,Ho,Wo,Cout] = act(conv(x, w) + bias (+ residual)).
// w: [Npad][Kpad] (bf16 or e4m3), k = (kh*KW + kw)*Cin + ci, zero padded.
// bias: [Npad] fp32 (BatchNorm already folded in). wscale: [Npad] fp32 per-output-channel weight
// dequant scale (fp8 path only; nullptr otherwise). In the fp8 path x / res / y are e4m3 tensors
// (x fp32 when in_f32, y fp32 when out_f32).
hipError_t conv2d(const ConvDesc& d, int batch, const void* x, const void* w, const float* bias,
                  const float* wscale, const void* res, void* y, hipStream_t stream);
hipError_t conv2d_f32(const ConvDesc& d, int batch, const void* x, const void* w,
                      const float* bias, const void* res, void* y, hipStream_t stream);

// Activation element types of the pooling / head kernels (their `et` argument; 1 was the old
// fp8 flag, so fp8 callers are unchanged)
enum ElemType : int { ET_BF16 = 0, ET_FP8 = 1, ET_F32 = 2 };

// The LDS-pipelined implicit-GEMM path (conv_gemm.hip) for wide bf16 layers; conv2d() routes
// there by itself when conv_gemm_supported() holds.
bool conv_gemm_supported(const ConvDesc& d, int batch, bool has_res);
// conv path selection (tests / A-B benches): 0 auto, 1 never GEMM, 2 GEMM whenever the shape allows
void set_conv_path(int mode);
int conv_path();
// conv3 of a ResNet bottleneck with its projection shortcut as ONE GEMM over the concatenated
// reduction: y = act(conv1x1(x, w) + bias + conv1x1_stride2(x2, w2) + bias2). d: the 1x1
// stride-1 conv on x (no residual); x2 [B][H2][W2][Cin2] bf16 sampled at stride2 onto d's output
// grid, w2 [Npad][Kpad2]. The projection's output tensor never exists.
bool conv_gemm_proj_supported(const ConvDesc& d, int batch, int H2, int W2, int Cin2,
                              int stride2, int Kpad2);
hipError_t conv2d_gemm_proj(const ConvDesc& d, int batch, const void* x, const void* w,
                            const float* bias, const void* x2, int H2, int W2, int Cin2,
                            int stride2, int Kpad2, const void* w2, const float* bias2, void* y,
                            hipStream_t stream);
hipError_t conv2d_gemm(const ConvDesc& d, int batch, const void* x, const void* w,
                       const float* bias, const void* res, void* y, hipStream_t stream);

// 3x3 stride-1 convs with an LDS-resident input patch per 64-channel block (conv_patch.hip):
// bf16, Cin % 64 == 0, tiles of whole output rows (<= 128 pixels, >= 96). conv2d() routes there
// first when conv_patch_supported() holds. set_conv_patch / GALE_CONV_PATCH: 0 off, 1 (default)
// 128-channel tiles only, 2 also 64-channel tiles.
bool conv_patch_supported(const ConvDesc& d, int batch, bool has_res);
void set_conv_patch(int mode);
hipError_t conv2d_patch(const ConvDesc& d, int batch, const void* x, const void* w,
                        const float* bias, const void* res, void* y, hipStream_t stream);

// One whole ResNet-50 56x56 bottleneck per launch (bottleneck_fused.hip), bf16 NHWC:
// y = relu(conv3(relu(conv2(relu(conv1(x))))) + shortcut), shortcut = x (cin 256) or, with
// down = 1 (block 0, cin 64), the 1x1 projection bf16(wd . x + bd). Packed weights as conv2d's:
// w1 [64][cin], w2 [64][576], w3 / wd [256][64]; biases fp32 with BatchNorm folded in.
struct BottleneckParams {
  const void* w1 = nullptr;
  const void* w2 = nullptr;
  const void* w3 = nullptr;
  const void* wd = nullptr;
  const float* b1 = nullptr;
  const float* b2 = nullptr;
  const float* b3 = nullptr;
  const float* bd = nullptr;
  int cin = 256;
  int down = 0;
};
bool bottleneck56_supported(int H, int W, int cin, int cmid, int cout, int down);
hipError_t bottleneck56(const BottleneckParams& p, int batch, const void* x, void* y,
                        hipStream_t stream);

// ResNet-50 ImageNet stem conv (packed-stem ConvDesc, ReLU) + 3x3/2 max-pool in one launch
// (stem_pool.hip): x = stem_pack() image bf16 [B][224][230][4], w [64][256], y bf16
// [B][56][56][64]. stem_pool_supported: the conv desc + the maxpool op's geometry.
bool stem_pool_supported(const ConvDesc& d, int H, int W, int C, int k, int s, int p, int Ho,
                         int Wo);
hipError_t stem_pool(int batch, const void* x, const void* w, const float* bias, void* y,
                     hipStream_t stream);

// fp32 NHWC [B][H][W][C<=4] -> bf16 [B][H][Wp][4] with `lp` zero columns on the left (and zeros
// up to Wp on the right, channels >= C zero): the input of a packed-stem conv (ConvDesc::stem).
hipError_t stem_pack(int batch, int H, int W, int C, int Wp, int lp, const float* x, void* y,
                     hipStream_t stream);

// Max pooling, NHWC bf16 / e4m3 (the scale passes through) / fp32 by `et` (ElemType), window k,
// stride s, -inf padding p.
hipError_t maxpool2d(int batch, int H, int W, int C, int k, int s, int p, int Ho, int Wo,
                     const void* x, void* y, int et, hipStream_t stream);

// Global average pooling, NHWC [B,H,W,C] -> same type [B,C] (same scale), `et` = ElemType.
hipError_t avgpool_global(int batch, int HW, int C, const void* x, void* y, int et,
                          hipStream_t stream);

// Fused classifier head: optional global average pool over HW, dense layer with fp32 weights
// w[N][C] + bias[N], then row softmax. x: bf16, e4m3 (scale in_scale) or fp32 [B,HW,C] by `et`
// (ElemType); out: fp32 [B,N]. One workgroup per image.
hipError_t head_pool_dense_softmax(int batch, int HW, int C, int N, const void* x, int et,
                                   float in_scale, const float* w, const float* bias, float* out,
                                   hipStream_t stream);

// Whole-network CIFAR-10 ResNet-20 (csrc/kernels/resnet20_fused.hip): x fp32 [B,32,32,3] ->
// The step graph's outputs written by a whole-network forward itself (all null: none): each
// softmax value also as a Java Float.toString slot (kFloatTextSlot bytes, as format_floats_java)
// in text, and, by workgroup 0 before anything else, the batch's parse verdicts handed over:
// status_out[i] = status[i], status[i] = 0 for i < *nrec (status: the parse's device array;
// text and status_out: host-mapped). The replica's step is then parse -> forward, two nodes.
// The inputs of a batch whose images the GPU ingest already parsed into fetch arenas, passed BY
// VALUE in the forward's kernel arguments, so a batch step needs no metadata copy at all: image
// i is at base[code[i] >> 24] + (code[i] & 0xffffff) * (H * W * C) floats. base[0] == null:
// no table (the forward reads x or xs).
constexpr int kInputTableImages = 512, kInputTableBases = 16;
struct InputTable {
  const float* base[kInputTableBases];
  uint32_t code[kInputTableImages];
};

struct StepOut {
  void* text = nullptr;
  int* status = nullptr;
  int* status_out = nullptr;
  const int* nrec = nullptr;
};

// softmax fp32 [B,10], one workgroup per image with every activation in LDS. w/b: the 19 convs
// in network order (packed [Npad][Kpad] + folded-BN fp32 bias), fc_w fp32 [10][64].
// fp8: w are e4m3 codes with per-channel scales ws; s_in / s_out / s_res are the per-tensor
// activation scales of each conv's input / output / residual (s_in[0] quantises the input).
struct ResNet20Params {
  const void* w[19];  // bf16 or e4m3
  const float* b[19];
  const float* fc_w;
  const float* fc_b;
  int fp8;
  const float* ws[19];
  float s_in[19], s_out[19], s_res[19];
  // non-null: the image count is read from device memory at run time (images <= the `batch`
  // the launch is sized for) - a captured step graph replays one launch for every batch size
  const int* batch_dev;
  StepOut so;  // (prediction text + verdict hand-off in the epilogue)
  // non-null: image i's fp32 [32][32][3] input is at xs[i] (images the GPU ingest already parsed
  // into its fetch arenas; device memory) instead of x + i * 3072
  const float* const* xs;
};
hipError_t resnet20_fused_forward(const ResNet20Params& p, int batch, const float* x, float* out,
                                  hipStream_t stream, const InputTable* tab = nullptr);

// Whole-network MNIST LeNet-5 (csrc/kernels/lenet5_fused.hip): x fp32 [B,28,28,1] -> softmax
// fp32 [B,10], one image per 256-thread workgroup (grid = batch) with every activation in LDS. Weights are the serving
// plan's packed bf16 matrices: conv1 [16][32], conv2 [16][224], fc1 [128][416], fc2 [128][128]
// (fp32 biases of Npad entries), fc3 fp32 [10][88] + [10].
struct LeNet5Params {
  const void* w1;
  const float* b1;
  const void* w2;
  const float* b2;
  const void* w3;
  const float* b3;
  const void* w4;
  const float* b4;
  const float* w5;
  const float* b5;
  const int* batch_dev;  // as ResNet20Params::batch_dev
  StepOut so;            // as ResNet20Params::so
  const float* const* xs;  // as ResNet20Params::xs ([28][28][1] images)
};
hipError_t lenet5_fused_forward(const LeNet5Params& p, int batch, const float* x, float* out,
                                hipStream_t stream, const InputTable* tab = nullptr);

// Row softmax, fp32 [B, ld] -> fp32 [B, N] (first N columns of each row).
hipError_t softmax_rows(int batch, int N, int ld, const float* x, float* out, hipStream_t stream);

// fp32 -> bf16 cast with optional affine normalisation y = x*scale + shift (n elements).
// Inference BatchNorm (per-channel scale/shift; nullptr = identity) + optional residual + ReLU
// over NHWC bf16 (et = ET_BF16) or fp32 (ET_F32: the fp32 unfolded-BN plan), [batch,
// HW = Ho*Wo, C stored]. The residual is [batch, res_H, res_W, res_C], read at (ho*rs, wo*rs),
// zero for channels >= res_C. In-place (x == y) is allowed.
hipError_t bn_act(int batch, int HW, int Wo, int C, const void* x, const float* scale,
                  const float* shift, const void* res, int res_H, int res_W, int res_C, int rs,
                  int relu, void* y, hipStream_t stream, int et = 0);

hipError_t cast_f32_bf16(int64_t n, float scale, float shift, const float* x, void* y,
                         hipStream_t stream);


// GPU decoder for the InstObj JSON contract: parses every number of each record's instances
// array into the fp32 NHWC batch tensor and validates the rectangular [N][H][W][C] structure.
// Work is split into kJsonTileBytes tiles of record text (one workgroup each); record i owns the
// global tiles [tile0, tile0 + json_tile_count(off, len)), numbered consecutively over the batch.
// The kernel raises each record's status (host zeroes it): 0 ok, 1 number-count mismatch,
// 2 malformed number / element, 3 bad structure (ragged / wrong rank).
constexpr int kJsonTileBytes = 2048;
constexpr int kGroupTiles = 4;  // tiles per ingest counting workgroup (one per wave) / group sum
struct JsonRecord {
  int64_t off;      // byte offset of the instances array inside the staged byte buffer
  int32_t len;      // array length in bytes
  int32_t slot;     // first image slot of this record inside the batch
  int32_t images;   // images in this record (from the host '[' count)
  int32_t status;   // raised by the kernel
  int32_t tile0;    // first global tile of this record
  // 1: the record's count block is already on the device at bytes + cnt_off (the GPU ingest pass
  // counted it and left it in the fetch buffer's device mirror): its nt tile token counts, then
  // one sum per group of kGroupTiles tiles. The parse skips its counting pass over this record.
  int32_t has_cnt;
  int64_t cnt_off;
  // ingest_crc_count only: groups in the records before this one, so the record's count block
  // starts at counts + tile0 + grp0
  int64_t grp0;
};
static_assert(sizeof(JsonRecord) == 48, "JsonRecord layout (host <-> device tables)");
int json_tile_count(int64_t off, int32_t len);
// tile_rec[t]: index of the record owning global tile t. tile_counts: device scratch of
// >= ntiles ints.
// count_pass = false: every record has_cnt (the counting kernel is not launched at all).
// d_ntiles non-null: the kernels read the tile count from device memory (ntiles = the most the
// launch is sized for; waves past the device count exit) - the captured step graph's form.
// status non-null: the verdicts are raised in status[record] (device memory) instead of
// recs[record].status, and recs / tile_rec / d_ntiles are only read - they may then be
// host-mapped pinned memory (the step graph reads the batch's metadata where the host wrote it,
// with no copy node).
// images < 0 (with has_cnt): the record's image count is taken from the group sums of its count
// block on the device (the GPU ingest parses a fetch right behind its counting launch, before
// the host has read the counts); a total that is not whole images expects nothing (status 1).
// tile_bad non-null (count_pass false): each tile's verdict (0 / 1 / 2 / 3) goes to
// tile_bad[tile] by a plain store instead of raising a record status, so it may be host-mapped
// memory; a record's verdict is the max over its tiles.
hipError_t json_parse_instances(int nrec, int ntiles, JsonRecord* recs, const int* tile_rec,
                                const uint8_t* bytes, int H, int W, int C, int* tile_counts,
                                float* out, hipStream_t stream, bool count_pass = true,
                                const int* d_ntiles = nullptr, int* status = nullptr,
                                int* tile_bad = nullptr);

// Raw (zero initial state, no final inversion) CRC32C of byte windows [end - len, end) of a
// device buffer, one wave per window (len <= kCrcChunkBytes): each lane folds 64 bytes with
// slicing-by-4 tables in LDS, shifts its register over the bytes after its piece (one GF(2)
// multiply by a per-lane constant) and the wave XOR-reduces. The host joins the windows of a
// Kafka record batch with crc = shift(crc, 4096) ^ window_crc and converts to the standard CRC
// (kafka::CrcShift). tables: kafka::crc32c_device_tables() (1088 words) in device memory.
constexpr int kCrcChunkBytes = 4096;
struct CrcChunk {
  int64_t end;  // one past the window's last byte (offset into `bytes`)
  int32_t len;  // window length, 1..kCrcChunkBytes
  int32_t pad_;
};
hipError_t crc32c_chunks(const uint8_t* bytes, const CrcChunk* chunks, int n,
                         const uint32_t* tables, uint32_t* out, hipStream_t stream);

// The GPU ingest pass of one fetch buffer in ONE launch: workgroups [0, crc blocks) fold the CRC
// windows (crc32c_chunks), the rest count the records' number tokens so the host learns each
// record's image count without reading its text: one workgroup per tile group, groups[g] =
// (record, record-relative first tile), kGroupTiles tiles each (a record's last group may be
// shorter). Record i's count block at counts + tile0 + grp0 gets its tile counts and group sums
// (see JsonRecord::has_cnt); gsum[g] = the tokens of group g (the host adds a record's groups);
// invalid bytes raise recs[i].status to 2, or, with gbad non-null, set gbad[g] = 2 (else 0) by a
// plain store and leave recs untouched - chunks, recs, groups, crc_out, gsum and gbad may then
// be host-mapped pinned memory (read and written over the link, no copies); bytes, tables and
// counts are device memory.
// packed non-null: the fetch body is the nibble-packed stream `packed` with its group table
// `tab` (both device memory; csrc/codec/text_pack.h) instead of text at `bytes`: the CRC
// windows and counting waves expand it in registers and the counting waves store every record's
// text (its 16-byte-aligned extent) into text_out - text_unpack folded into this launch.
hipError_t ingest_crc_count(const uint8_t* bytes, const CrcChunk* chunks, int nchunks,
                            const uint32_t* tables, uint32_t* crc_out, int nrec, int ngroups,
                            JsonRecord* recs, const int2* groups, int* counts, int* gsum,
                            int* gbad, hipStream_t stream, const uint8_t* packed = nullptr,
                            const uint32_t* tab = nullptr, uint8_t* text_out = nullptr);

// Expands a nibble-packed span (csrc/codec/text_pack.h: 64-byte blocks, per-2-KiB-group
// {base offset, packed-block mask} pairs in tab) into out[0, n). out must be 16-byte aligned,
// packed 8-byte aligned. packed and tab may be host-mapped pinned memory (the GPU ingest reads the
// small group table from the source's pinned chunk; the packed stream itself is DMA'd first:
// kernel loads over the link expand it ~15x slower than the SDMA copy plus a device pass).
hipError_t text_unpack(const uint8_t* packed, const uint32_t* tab, int64_t n, uint8_t* out,
                       hipStream_t stream);

// ---- prediction text (format.hip) -----------------------------------------------------------
// n binary32 values -> Java Float.toString text (JDK 19+ shortest-digit rules, the same text as
// codec::format_float_java), one 16-byte slot per value: characters from byte 0, length in
// byte 15 (at most 14 characters).
constexpr int kFloatTextSlot = 16;
hipError_t format_floats_java(int n, const float* x, void* out16, hipStream_t stream);
// n = (*d_count) * per values (n <= max_n, the launch size): the step graph's form
hipError_t format_floats_java_dev(int max_n, const int* d_count, int per, const float* x,
                                  void* out16, hipStream_t stream);
// The step graph's last node: format_floats_java_dev, and the batch's parse verdicts handed
// back - status_out[i] = status[i], status[i] = 0 for i < *d_nrec (status: the parse's device
// array, cleared for the slot's next batch; status_out: host-mapped), so the step needs no
// status copy node. max_n must cover max_nrec values (the launch's threads do both).
hipError_t format_floats_java_step(int max_n, const int* d_count, int per, const float* x,
                                   void* out16, const int* d_nrec, int* status, int* status_out,
                                   hipStream_t stream);

}  // namespace gale
