// GpuReplica (see replica.h): staged JSON bytes -> GPU JSON parser -> hipGraph forward ->
// softmax rows on the replica's own streams. Kept apart from the host-only replicas so the
// sanitizer build of the host pipeline (make tsan / make asan) links no GPU code.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>
#include <stdexcept>

#include "../codec/json_codec.h"
#include "metrics.h"
#include "replica.h"

namespace gale {

// ---------------------------------------------------------------------------------------------
// GpuReplica
// ---------------------------------------------------------------------------------------------

GpuReplica::GpuReplica(std::shared_ptr<Executor> exec, int H, int W, int C, int classes,
                       bool use_graph, int wait_poll_us, bool gpu_encode, int locality,
                       bool step_graph, bool high_priority, bool step_direct)
    : exec_(std::move(exec)), H_(H), W_(W), C_(C), classes_(classes), use_graph_(use_graph),
      wait_poll_us_(wait_poll_us), gpu_encode_(gpu_encode), locality_(locality),
      step_direct_(step_direct) {
  step_graph_ = step_graph && use_graph && exec_->device_batch_ok();
  ptr_input_ = step_graph_ && gpu_encode_ && step_direct_ && exec_->step_out_ok();
  if (exec_->input_bytes_per_image() != (long long)H * W * C * 4)
    throw std::invalid_argument("GpuReplica: executor input is not fp32 [H, W, C]");
  if (exec_->output_bytes_per_image() != (long long)classes * 4)
    throw std::invalid_argument("GpuReplica: executor output is not fp32 [classes]");
  check_hip(hipSetDevice(exec_->device()), "hipSetDevice");
  if (high_priority) {
    int least = 0, greatest = 0;
    check_hip(hipDeviceGetStreamPriorityRange(&least, &greatest), "stream priority range");
    check_hip(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest),
              "hipStreamCreateWithPriority");
  } else if (const char* e = getenv("GALE_REPLICA_CU_RESERVE"); e && atoi(e) > 0) {
    // (A/B) the replica's kernels kept off the last N CUs, which the GPU ingest's passes then
    // find free instead of queueing behind whole-chip forward batches
    hipDeviceProp_t prop;
    check_hip(hipGetDeviceProperties(&prop, exec_->device()), "hipGetDeviceProperties");
    const int cus = prop.multiProcessorCount, keep = std::max(1, cus - atoi(e));
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int i = 0; i < keep; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    check_hip(hipExtStreamCreateWithCUMask(&stream_, (uint32_t)mask.size(), mask.data()),
              "hipExtStreamCreateWithCUMask");
  } else {
    check_hip(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
  }
  const int mb = exec_->max_batch();
  slots_.resize((size_t)exec_->slots());
  for (Slot& s : slots_) {
    check_hip(hipHostMalloc(reinterpret_cast<void**>(&s.h_out), sizeof(float) * mb * classes),
              "hipHostMalloc(out)");
    if (gpu_encode_) {
      const size_t tb = (size_t)kFloatTextSlot * mb * classes;
      check_hip(hipHostMalloc(reinterpret_cast<void**>(&s.h_text), tb, hipHostMallocMapped),
                "hipHostMalloc(text)");
      check_hip(hipMalloc(reinterpret_cast<void**>(&s.d_status), sizeof(int) * mb),
                "hipMalloc(status)");
      check_hip(hipMemset(s.d_status, 0, sizeof(int) * mb), "hipMemset(status)");
      s.h_status = static_cast<int*>(mapped_alloc(sizeof(int) * mb, "status"));
    }
    check_hip(hipEventCreateWithFlags(&s.done, hipEventDisableTiming |
                                                   (wait_poll_us_ < 0 ? hipEventBlockingSync : 0)),
              "hipEventCreate");
    // initial text capacity: ~12 bytes per number (Java Float.toString + ",") x a full batch
    ensure_device(s, (size_t)mb * H * W * C * 12 + 4096);
    ensure_tiles(s, (int)(((size_t)mb * H * W * C * 12) / kJsonTileBytes) + 2 * mb, 0);
  }
}

GpuReplica::~GpuReplica() {
  hipSetDevice(exec_->device());
  if (stream_) hipStreamSynchronize(stream_);
  for (Slot& s : slots_) {
    drop_steps(s);
    if (s.h_bytes) hipHostFree(s.h_bytes);
    if (s.d_bytes) hipFree(s.d_bytes);
    if (s.h_hdr) hipHostFree(s.h_hdr);
    if (s.d_hdr) hipFree(s.d_hdr);
    if (s.d_tiles) hipFree(s.d_tiles);
    if (s.h_out) hipHostFree(s.h_out);
    if (s.h_text) hipHostFree(s.h_text);
    if (s.h_status) hipHostFree(s.h_status);
    if (s.d_status) hipFree(s.d_status);
    if (s.done) hipEventDestroy(s.done);
  }
  if (stream_) hipStreamDestroy(stream_);
}

std::string GpuReplica::name() const { return "gpu" + std::to_string(exec_->device()); }

// Host-mapped pinned memory that kernels address with the host pointer (ROCm maps it at the
// same virtual address; anything else is refused rather than silently copied).
void* GpuReplica::mapped_alloc(size_t bytes, const char* what) {
  void* h = nullptr;
  check_hip(hipHostMalloc(&h, bytes, hipHostMallocMapped), what);
  void* d = nullptr;
  check_hip(hipHostGetDevicePointer(&d, h, 0), what);
  if (d != h) {
    hipHostFree(h);
    throw std::runtime_error(std::string("GpuReplica: mapped ") + what +
                             " buffer has another device address");
  }
  return h;
}

void GpuReplica::ensure_host(Slot& s, size_t bytes) {
  if (bytes <= s.h_cap) return;
  const size_t cap = (std::max(bytes, s.h_cap * 2) + 4095) & ~(size_t)4095;
  if (s.h_bytes) {
    check_hip(hipEventSynchronize(s.done), "hipEventSynchronize");
    hipHostFree(s.h_bytes);
  }
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&s.h_bytes), cap), "hipHostMalloc(bytes)");
  s.h_cap = cap;
}

void GpuReplica::drop_steps(Slot& s) {
  for (hipGraphExec_t& g : s.step) {
    if (g) hipGraphExecDestroy(g);
    g = nullptr;
  }
}

size_t GpuReplica::meta_rec_bytes() const {
  return (sizeof(JsonRecord) + sizeof(float*)) * (size_t)exec_->max_batch();
}

// Per-slot parser metadata: [header][JsonRecord x max_batch][input pointer x max_batch]
// [tile -> record index x tiles_cap], pinned on the host and mirrored on the device (one H2D per
// batch), plus the per-tile token counts. Growing keeps the first `keep` records and the input
// pointer table already written into the host copy.
void GpuReplica::ensure_tiles(Slot& s, int ntiles, int keep) {
  if (ntiles <= s.tiles_cap) return;
  const int cap = std::max(ntiles, s.tiles_cap * 2);
  const size_t rec_bytes = meta_rec_bytes();
  const size_t xs_off = sizeof(JsonRecord) * (size_t)exec_->max_batch();
  const size_t bytes = kMetaHdr + rec_bytes + sizeof(int) * (size_t)cap;
  if (s.h_hdr) check_hip(hipEventSynchronize(s.done), "hipEventSynchronize");
  // host-mapped: the copy-free step graph's kernels read the metadata from here
  uint8_t* h = static_cast<uint8_t*>(mapped_alloc(bytes, "meta"));
  memset(h, 0, kMetaHdr);
  if (s.h_hdr) {
    memcpy(h + kMetaHdr, s.h_recs, sizeof(JsonRecord) * (size_t)keep);
    memcpy(h + kMetaHdr + xs_off, s.h_xs, sizeof(float*) * (size_t)exec_->max_batch());
    drop_steps(s);
    hipHostFree(s.h_hdr);
    hipFree(s.d_hdr);
    hipFree(s.d_tiles);
  }
  uint8_t* d = nullptr;
  check_hip(hipMalloc(reinterpret_cast<void**>(&d), bytes), "hipMalloc(meta)");
  s.h_hdr = reinterpret_cast<int32_t*>(h);
  s.d_hdr = reinterpret_cast<int32_t*>(d);
  s.h_recs = reinterpret_cast<JsonRecord*>(h + kMetaHdr);
  s.d_recs = reinterpret_cast<JsonRecord*>(d + kMetaHdr);
  s.h_xs = reinterpret_cast<const float**>(h + kMetaHdr + xs_off);
  s.d_xs = reinterpret_cast<const float**>(d + kMetaHdr + xs_off);
  check_hip(hipMalloc(reinterpret_cast<void**>(&s.d_tiles), sizeof(int) * cap),
            "hipMalloc(tiles)");
  s.h_tile_rec = reinterpret_cast<int*>(reinterpret_cast<char*>(s.h_recs) + rec_bytes);
  s.d_tile_rec = reinterpret_cast<int*>(reinterpret_cast<char*>(s.d_recs) + rec_bytes);
  s.tiles_cap = cap;
}

void GpuReplica::ensure_device(Slot& s, size_t bytes) {
  if (bytes <= s.d_cap) return;
  const size_t cap = (std::max(bytes, s.d_cap * 2) + 4095) & ~(size_t)4095;
  if (s.d_bytes) {
    check_hip(hipEventSynchronize(s.done), "hipEventSynchronize");
    drop_steps(s);
    hipFree(s.d_bytes);
  }
  check_hip(hipMalloc(reinterpret_cast<void**>(&s.d_bytes), cap), "hipMalloc(bytes)");
  s.d_cap = cap;
}

// Stage the batch's JSON text on the device. Records that arrived in pinned fetch buffers are
// DMA'd straight from them: one hipMemcpyAsync per fetch buffer covering the records' span
// (the few Kafka record-header bytes between values ride along); records in pageable memory are
// first gathered into the slot's pinned staging buffer. Offsets keep their position modulo 16,
// so the parser's aligned 16-byte loads see the same layout as on the host.
void GpuReplica::submit(Batch& b) {
  const int slot = next_slot_;
  next_slot_ = (next_slot_ + 1) % (int)slots_.size();
  b.slot = slot;
  Slot& s = slots_[(size_t)slot];
  struct Span {
    const uint8_t* base;
    size_t lo, hi;
  };
  std::vector<Span> spans;
  size_t staged = 0;
  const int my_loc = locality();
  auto resident = [my_loc](const InRecord& r) {
    return r.dev_value != nullptr && r.dev_locality == my_loc;
  };
  // images the GPU ingest already parsed (its arena is in this replica's device memory)
  auto preparsed = [&](const InRecord& r) { return ptr_input_ && resident(r) && r.dev_image; };
  if (ptr_input_ && try_table_step(b, s, slot, preparsed)) return;
  for (const InRecord& r : b.recs) {
    if (resident(r)) continue;  // already in device memory (GPU ingest): nothing to copy
    const uint8_t* base = r.buf.get();
    const size_t lo = (size_t)(r.value + r.arr_off - base), hi = lo + (size_t)r.arr_len;
    if (!r.pinned) {
      staged += ((size_t)r.arr_len + 31) & ~(size_t)15;
      continue;
    }
    Span* sp = nullptr;
    for (Span& x : spans)
      if (x.base == base) sp = &x;
    if (!sp) {
      spans.push_back({base, lo, hi});
    } else {
      sp->lo = std::min(sp->lo, lo);
      sp->hi = std::max(sp->hi, hi);
    }
  }
  size_t dev_total = 16 + staged;
  for (Span& x : spans) {
    x.lo &= ~(size_t)15;
    dev_total += ((x.hi - x.lo) + 15) & ~(size_t)15;
  }
  ensure_device(s, dev_total + 16);
  if (staged) ensure_host(s, staged + 16);
  // device layout: [span 0][span 1]...[staged records]
  std::vector<size_t> span_dev(spans.size());
  size_t doff = 0;
  for (size_t i = 0; i < spans.size(); ++i) {
    span_dev[i] = doff;
    check_hip(hipMemcpyAsync(s.d_bytes + doff, spans[i].base + spans[i].lo,
                             spans[i].hi - spans[i].lo, hipMemcpyHostToDevice, stream_),
              "H2D span");
    doff += ((spans[i].hi - spans[i].lo) + 15) & ~(size_t)15;
  }
  const size_t staged_dev = doff;
  size_t hoff = 0;
  int nrec = 0, img = 0, ntiles = 0, npre = 0;
  bool count_pass = false;
  const int64_t per = (int64_t)H_ * W_ * C_;
  const float* in = static_cast<const float*>(exec_->input(slot));
  s.parse_idx.assign(b.recs.size(), -1);
  if (ptr_input_) ensure_tiles(s, 1, 0);  // (the pointer table lives in the metadata)
  for (size_t ri = 0; ri < b.recs.size(); ++ri) {
    const InRecord& r = b.recs[ri];
    if (img + r.images > exec_->max_batch())
      throw std::logic_error("GpuReplica: batch exceeds max_batch");
    if (preparsed(r)) {  // the forward reads its images where the ingest parsed them
      for (int k = 0; k < r.images; ++k) s.h_xs[img + k] = r.dev_image + k * per;
      img += r.images;
      ++npre;
      continue;
    }
    if (ptr_input_)
      for (int k = 0; k < r.images; ++k) s.h_xs[img + k] = in + (int64_t)(img + k) * per;
    s.parse_idx[ri] = nrec;
    JsonRecord& jr = s.h_recs[nrec++];
    const uint8_t* base = r.buf.get();
    const size_t lo = (size_t)(r.value + r.arr_off - base);
    if (resident(r)) {
      // offsets are relative to the slot's buffer; a mirror elsewhere in device memory is a
      // (signed) distance in the flat address space, 16-byte phase preserved (both bases are
      // 256-byte aligned allocations)
      jr.off = (int64_t)((r.dev_value + r.arr_off) - s.d_bytes);
    } else if (r.pinned) {
      size_t k = 0;
      while (spans[k].base != base) ++k;
      jr.off = (int64_t)(span_dev[k] + (lo - spans[k].lo));
    } else {
      hoff += (lo - hoff) & 15;  // keep the record's alignment modulo 16
      memcpy(s.h_bytes + hoff, r.value + r.arr_off, (size_t)r.arr_len);
      jr.off = (int64_t)(staged_dev + hoff);
      hoff = (hoff + (size_t)r.arr_len + 15) & ~(size_t)15;
    }
    jr.len = (int32_t)r.arr_len;
    jr.slot = img;
    jr.images = r.images;
    jr.status = 0;
    jr.tile0 = ntiles;
    jr.has_cnt = 0;
    jr.cnt_off = 0;
    jr.grp0 = 0;
    if (resident(r) && r.dev_counts) {  // counted by the ingest pass: no counting pass here
      jr.has_cnt = 1;
      jr.cnt_off = (int64_t)(r.dev_counts - s.d_bytes);
    } else {
      count_pass = true;
    }
    ntiles += json_tile_count(jr.off, jr.len);
    img += r.images;
  }
  if (img > exec_->max_batch()) throw std::logic_error("GpuReplica: batch exceeds max_batch");
  {
    int64_t res = 0;
    for (const InRecord& r : b.recs) res += resident(r) ? 1 : 0;
    resident_ += res;
    host_ += (int64_t)b.recs.size() - res;
    preparsed_ += npre;
  }
  b.images = img;
  ensure_tiles(s, ntiles, nrec);
  for (int i = 0; i < nrec; ++i) {
    const JsonRecord& jr = s.h_recs[i];
    const int nt = json_tile_count(jr.off, jr.len);
    for (int t = 0; t < nt; ++t) s.h_tile_rec[jr.tile0 + t] = i;
  }
  if (hoff)
    check_hip(hipMemcpyAsync(s.d_bytes + staged_dev, s.h_bytes, hoff, hipMemcpyHostToDevice,
                             stream_),
              "H2D staged");
  if (step_graph_) {
    // ONE launch for the whole step: the captured graph copies the metadata (header included)
    // and its kernels take the record / tile / image counts from the header
    s.h_hdr[0] = nrec;
    s.h_hdr[1] = ntiles;
    s.h_hdr[2] = img;
    hipGraphExec_t g = (gpu_encode_ && step_direct_) ? nullptr : step_for(s, slot, count_pass);
    if (gpu_encode_) {
      // the metadata this batch uses (header, its records, the input pointer table, its tile
      // map) as one DMA
      const size_t rec_bytes = meta_rec_bytes();
      const size_t used = ntiles > 0 ? kMetaHdr + rec_bytes + sizeof(int) * (size_t)ntiles
                          : ptr_input_ ? kMetaHdr + rec_bytes
                                       : kMetaHdr + sizeof(JsonRecord) * (size_t)nrec;
      check_hip(hipMemcpyAsync(s.d_hdr, s.h_hdr, used, hipMemcpyHostToDevice, stream_),
                "H2D step metadata");
    }
    if (g)
      check_hip(hipGraphLaunch(g, stream_), "hipGraphLaunch(step)");
    else  // (the same kernels launched directly: no graph-launch bookkeeping in the runtime)
      check_hip(enqueue_step(s, slot, count_pass, stream_, nrec > 0, ptr_input_), "step launch");
    b.step_graph = true;
    ++step_batches_;
    check_hip(hipEventRecord(s.done, stream_), "hipEventRecord");
    s.t_submit_ns = mono_ns();
    return;
  }
  const size_t meta = reinterpret_cast<char*>(s.h_tile_rec + ntiles) -
                      reinterpret_cast<char*>(s.h_recs);
  check_hip(hipMemcpyAsync(s.d_recs, s.h_recs, meta, hipMemcpyHostToDevice, stream_),
            "H2D recs");
  check_hip(json_parse_instances(nrec, ntiles, s.d_recs, s.d_tile_rec, s.d_bytes, H_, W_, C_,
                                 s.d_tiles,
                                 static_cast<float*>(exec_->input(slot)), stream_, count_pass),
            "json_parse_instances");
  exec_->run(slot, img, stream_, use_graph_);
  if (use_graph_ && exec_->graph_pays()) ++fwd_graph_batches_;
  if (gpu_encode_) {
    // the prediction text (Java Float.toString per value) is formatted on the stream and comes
    // back instead of the probabilities, so the emitting thread only concatenates slots
    // (format.hip: ~6 us per 256-image batch). The kernel stores the 16-byte slots straight
    // into the pinned (device-mapped, coherent) host buffer: no separate D2H copy.
    check_hip(format_floats_java(img * classes_, static_cast<const float*>(exec_->output(slot)),
                                 s.h_text, stream_),
              "format_floats_java");
  } else {
    check_hip(hipMemcpyAsync(s.h_out, exec_->output(slot), sizeof(float) * img * classes_,
                             hipMemcpyDeviceToHost, stream_),
              "D2H probs");
  }
  check_hip(hipMemcpyAsync(s.h_recs, s.d_recs, sizeof(JsonRecord) * nrec, hipMemcpyDeviceToHost,
                           stream_),
            "D2H status");
  check_hip(hipEventRecord(s.done, stream_), "hipEventRecord");
  s.t_submit_ns = mono_ns();
}

// Every record of the batch parsed by the ingest pass (into at most kInputTableBases arenas):
// the step is ONE launch - the forward, each image addressed through an InputTable in its kernel
// arguments - with no metadata copy (the H2D of a step's metadata ran as a CU blit kernel, ~12 us
// of device time per batch, profiles/r6_e2e_kernel_stats.txt) and no verdict hand-off (the
// ingest judged the records).
template <typename Pre>
bool GpuReplica::try_table_step(Batch& b, Slot& s, int slot, const Pre& preparsed) {
  InputTable tab;
  memset(&tab, 0, sizeof(tab));
  const int64_t per = (int64_t)H_ * W_ * C_;
  int nb = 0, img = 0;
  for (const InRecord& r : b.recs) {
    if (!preparsed(r) || !r.dev_arena || img + r.images > kInputTableImages) return false;
    int bi = 0;
    while (bi < nb && tab.base[bi] != r.dev_arena) ++bi;
    if (bi == nb) {
      if (nb == kInputTableBases) return false;
      tab.base[nb++] = r.dev_arena;
    }
    const int64_t s0 = (r.dev_image - r.dev_arena) / per;
    if (s0 < 0 || s0 + r.images > 0xffffff) return false;
    for (int k = 0; k < r.images; ++k) tab.code[img + k] = ((uint32_t)bi << 24) | (uint32_t)(s0 + k);
    img += r.images;
  }
  if (img <= 0 || img > exec_->max_batch()) return false;
  s.parse_idx.assign(b.recs.size(), -1);
  StepOut so;
  so.text = s.h_text;  // (no status hand-off: status_out null)
  exec_->launch_table(slot, img, tab, stream_, &so);
  b.images = img;
  b.step_graph = true;
  ++step_batches_;
  ++table_batches_;
  preparsed_ += (int64_t)b.recs.size();
  resident_ += (int64_t)b.recs.size();
  check_hip(hipEventRecord(s.done, stream_), "hipEventRecord");
  s.t_submit_ns = mono_ns();
  return true;
}

// The kernels-only step (gpu_encode): [count] -> parse -> forward (+ prediction text and
// verdicts in its epilogue; other plans end with the formatting kernel). The batch's metadata
// is DMA'd just before (submit(): an SDMA copy of the used part only), and the kernels read the
// record / tile / image counts from its header. The r4 step captured a metadata H2D and a status
// D2H as graph nodes, which this runtime runs as CU blit kernels (two per batch, 68 us average
// under the serving load); reading the metadata from host memory instead stretched every kernel
// by 25-40 % under the link's DMA load (profiles/r5_step_ab.txt). Captured once per slot into
// the step graph, or enqueued directly (step_direct).
hipError_t GpuReplica::enqueue_step(Slot& s, int slot, bool count_pass, hipStream_t st,
                                     bool parse, bool xs) {
  const int mb = exec_->max_batch();
  hipError_t c = hipSuccess;
  if (parse)  // (a batch of records the ingest already parsed: the forward alone)
    c = json_parse_instances(mb, s.tiles_cap, s.d_recs, s.d_tile_rec, s.d_bytes, H_, W_, C_,
                             s.d_tiles, static_cast<float*>(exec_->input(slot)), st, count_pass,
                             s.d_hdr + 1, s.d_status);
  const bool fused = exec_->step_out_ok();
  StepOut so;
  so.text = s.h_text;
  so.status = s.d_status;
  so.status_out = s.h_status;
  so.nrec = s.d_hdr;
  if (c == hipSuccess) {
    try {
      exec_->launch_device_batch(slot, s.d_hdr + 2, st, fused ? &so : nullptr,
                                 xs ? s.d_xs : nullptr);
    } catch (const std::exception&) {
      c = hipErrorLaunchFailure;
    }
  }
  if (c == hipSuccess && !fused)
    c = format_floats_java_step(std::max(mb * classes_, mb), s.d_hdr + 2, classes_,
                                static_cast<const float*>(exec_->output(slot)), s.h_text,
                                s.d_hdr, s.d_status, s.h_status, st);
  return c;
}

// The slot's step graph, captured on first use (and after its buffers moved). Sized for the
// largest batch: the parse covers tiles_cap tiles and the forward max_batch images, their waves
// past the header's counts exit at once; the status copy-back is max_batch records.
hipGraphExec_t GpuReplica::step_for(Slot& s, int slot, bool count_pass) {
  hipGraphExec_t& g = s.step[count_pass ? 1 : 0];
  if (g) return g;
  const int mb = exec_->max_batch();
  const size_t meta = kMetaHdr + meta_rec_bytes() + sizeof(int) * s.tiles_cap;
  // capture on a private stream (as Executor::run does), replayed on the replica's stream
  hipStream_t cs = nullptr;
  check_hip(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "capture stream");
  hipGraph_t graph = nullptr;
  hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
  if (e == hipSuccess && gpu_encode_) {
    const hipError_t c = enqueue_step(s, slot, count_pass, cs);
    e = hipStreamEndCapture(cs, &graph);
    if (e == hipSuccess) e = c;
  } else if (e == hipSuccess) {
    hipError_t c = hipMemcpyAsync(s.d_hdr, s.h_hdr, meta, hipMemcpyHostToDevice, cs);
    if (c == hipSuccess)
      c = json_parse_instances(mb, s.tiles_cap, s.d_recs, s.d_tile_rec, s.d_bytes, H_, W_, C_,
                               s.d_tiles, static_cast<float*>(exec_->input(slot)), cs,
                               count_pass, s.d_hdr + 1);
    if (c == hipSuccess) {
      try {
        exec_->launch_device_batch(slot, s.d_hdr + 2, cs);
      } catch (const std::exception&) {
        c = hipErrorLaunchFailure;
      }
    }
    if (c == hipSuccess)
      c = gpu_encode_
              ? format_floats_java_dev(mb * classes_, s.d_hdr + 2, classes_,
                                       static_cast<const float*>(exec_->output(slot)), s.h_text,
                                       cs)
              : hipMemcpyAsync(s.h_out, exec_->output(slot), sizeof(float) * mb * classes_,
                               hipMemcpyDeviceToHost, cs);
    if (c == hipSuccess)
      c = hipMemcpyAsync(s.h_recs, s.d_recs, sizeof(JsonRecord) * mb, hipMemcpyDeviceToHost, cs);
    e = hipStreamEndCapture(cs, &graph);
    if (e == hipSuccess) e = c;
  }
  hipStreamDestroy(cs);
  if (e != hipSuccess && graph) hipGraphDestroy(graph);
  check_hip(e, "step graph capture");
  e = hipGraphInstantiate(&g, graph, nullptr, nullptr, 0);
  hipGraphDestroy(graph);
  check_hip(e, "step graph instantiate");
  return g;
}

void GpuReplica::wait(Batch& b) {
  Slot& s = slots_[(size_t)b.slot];
  if (wait_poll_us_ > 0) {
    // sleep-poll: the thread sleeps while the GPU works (the engine's timer slack is set to
    // 1 us on replica threads, so a sleep is not stretched by the default 50 us slack). It
    // sleeps through most of the expected batch time at once and polls only near the end:
    // polling every 20 us through a 0.5 ms batch cost ~0.25 core per replica (6 replicas:
    // 1.5 of a 16-core host share, which then tipped it into CFS throttling)
    const int64_t due = s.t_submit_ns + expect_ns_ * 85 / 100;
    const int64_t now = mono_ns();
    if (expect_ns_ > 0 && due - now > 2000ll * wait_poll_us_)
      std::this_thread::sleep_for(std::chrono::nanoseconds(due - now));
    for (;;) {
      const hipError_t e = hipEventQuery(s.done);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) check_hip(e, "hipEventQuery(batch)");
      std::this_thread::sleep_for(std::chrono::microseconds(wait_poll_us_));
    }
    const int64_t took = mono_ns() - s.t_submit_ns;
    expect_ns_ = expect_ns_ > 0 ? (expect_ns_ * 7 + took) / 8 : took;
  } else {
    check_hip(hipEventSynchronize(s.done), "hipEventSynchronize(batch)");
  }
  b.dev_status.assign(b.recs.size(), codec::OK);
  const bool copy_free = b.step_graph && gpu_encode_;
  for (size_t i = 0; i < b.recs.size(); ++i) {
    const int k = i < s.parse_idx.size() ? s.parse_idx[i] : (int)i;
    if (k < 0) continue;  // parsed (and judged) by the ingest pass
    const int st = copy_free ? s.h_status[k] : s.h_recs[k].status;
    if (st == 1 || st == 3) b.dev_status[i] = codec::BAD_SHAPE;
    else if (st == 2) b.dev_status[i] = codec::BAD_NUMBER;
  }
  b.probs = gpu_encode_ ? nullptr : s.h_out;
  b.pred_text = gpu_encode_ ? s.h_text : nullptr;
}

void GpuReplica::recover() {
  // drain whatever the failed batches left queued on both streams, then clear the (non-sticky)
  // error state; a sticky device fault makes these calls fail and the supervisor gives up
  check_hip(hipSetDevice(exec_->device()), "recover: hipSetDevice");
  check_hip(hipStreamSynchronize(stream_), "recover: compute stream");
  (void)hipGetLastError();
  next_slot_ = 0;
}

}  // namespace gale
