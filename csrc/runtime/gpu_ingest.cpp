// GpuIngest (see gpu_ingest.h / ingest.h).
#include "gpu_ingest.h"
#include "metrics.h"

#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <stdexcept>
#include <thread>

#include "../codec/json_codec.h"
#include "../codec/text_pack.h"
#include "gale/executor.h"

namespace gale {

GpuIngest::GpuIngest(int device, int lanes, int poll_us)
    : device_(device), poll_us_(poll_us), shift_chunk_(kCrcChunkBytes) {
  check_hip(hipSetDevice(device_), "ingest: hipSetDevice");
  std::vector<uint32_t> t(kafka::kCrcDeviceTableWords);
  kafka::crc32c_device_tables(t.data());
  check_hip(hipMalloc(reinterpret_cast<void**>(&d_tables_), t.size() * 4), "ingest: tables");
  check_hip(hipMemcpy(d_tables_, t.data(), t.size() * 4, hipMemcpyHostToDevice),
            "ingest: tables H2D");
  // (ingest lanes at the highest stream priority were measured and dropped: the replicas' batch
  // kernels then queue behind every fetch's ingest, ResNet-20 device time per batch 0.4 -> 2 ms,
  // profiles/archive/r4_ab_ingest_priority.jsonl)
  for (int i = 0; i < std::max(1, lanes); ++i) {
    auto L = std::make_unique<Lane>();
    check_hip(hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking), "ingest: stream");
    check_hip(hipEventCreateWithFlags(&L->done, hipEventDisableTiming), "ingest: event");
    lanes_.push_back(std::move(L));
  }
  if (const char* e = getenv("GALE_INGEST_DEV_TIMING")) dev_every_ = std::max(0, atoi(e));
  // (tests: the plan's own DMA, the path of a fetch whose plan does not fit behind it)
  if (const char* e = getenv("GALE_INGEST_PLAN_SEPARATE")) plan_separate_ = atoi(e) != 0;
  if (dev_every_ > 0)
    for (auto& L : lanes_)
      for (hipEvent_t& ev : L->tev) check_hip(hipEventCreate(&ev), "ingest: timing event");
}

GpuIngest::~GpuIngest() {
  hipSetDevice(device_);
  for (auto& L : lanes_) {
    if (L->stream) hipStreamSynchronize(L->stream);
    if (L->h_io) hipHostFree(L->h_io);
    if (L->d_io) hipFree(L->d_io);
    if (L->d_counts) hipFree(L->d_counts);
    if (L->done) hipEventDestroy(L->done);
    for (hipEvent_t ev : L->tev)
      if (ev) hipEventDestroy(ev);
    if (L->stream) hipStreamDestroy(L->stream);
  }
  if (d_tables_) hipFree(d_tables_);
}

void GpuIngest::grow(Lane& L, size_t io_bytes, size_t tiles) {
  auto up = [](size_t want, size_t have) {
    return (std::max(want, have * 2) + 4095) & ~(size_t)4095;
  };
  if (io_bytes > L.io_cap) {
    if (L.h_io) hipHostFree(L.h_io);
    if (L.d_io) hipFree(L.d_io);
    L.io_cap = up(io_bytes, L.io_cap);
    check_hip(hipMalloc(reinterpret_cast<void**>(&L.d_io), L.io_cap), "ingest: d_io");
    // the plan (DMA'd to d_io) and the results (stored here by the kernel): host-mapped
    check_hip(hipHostMalloc(reinterpret_cast<void**>(&L.h_io), L.io_cap, hipHostMallocMapped),
              "ingest: h_io");
    void* dp = nullptr;
    check_hip(hipHostGetDevicePointer(&dp, L.h_io, 0), "ingest: h_io device pointer");
    if (dp != L.h_io) throw std::runtime_error("ingest: mapped plan buffer has another address");
  }
  if (tiles * sizeof(int) > L.counts_cap) {
    if (L.d_counts) hipFree(L.d_counts);
    L.counts_cap = up(tiles * sizeof(int), L.counts_cap);
    check_hip(hipMalloc(reinterpret_cast<void**>(&L.d_counts), L.counts_cap), "ingest: counts");
  }
}

void GpuIngest::wait(Lane& L) {
  if (poll_us_ <= 0) {
    check_hip(hipEventSynchronize(L.done), "ingest: hipEventSynchronize");
    return;
  }
  for (;;) {
    const hipError_t e = hipEventQuery(L.done);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) check_hip(e, "ingest: hipEventQuery");
    std::this_thread::sleep_for(std::chrono::microseconds(poll_us_));
  }
}

namespace {
size_t align16(size_t n) { return (n + 15) & ~(size_t)15; }
}  // namespace

void GpuIngest::run(int lane, const kafka::Fetched& f, uint8_t* dev, size_t dev_cap,
                    bool check_crcs, int H, int W, int C, IngestIO& io, float* arena,
                    size_t arena_bytes) {
  Lane& L = *lanes_[(size_t)lane % lanes_.size()];
  std::lock_guard<std::mutex> lk(L.mu);
  const int64_t t_start = mono_ns();
  const size_t nrec_all = f.records.size();
  io.images.assign(nrec_all, 0);
  io.cnt_off.assign(nrec_all, -1);
  io.batch_ok.assign(f.batches.size(), 1);
  io.img.assign(nrec_all, nullptr);
  // ---- plan: CRC windows (aligned to each batch's end) and the records to count
  std::vector<CrcChunk> chunks;
  std::vector<std::pair<size_t, size_t>> batch_chunks;  // (first chunk, count) per batch
  size_t lo = f.size, hi = 0;
  for (const kafka::BatchSpan& b : f.batches) {
    lo = std::min(lo, b.off);
    hi = std::max(hi, b.off + b.len);
    if (!check_crcs) continue;
    const int64_t rs = (int64_t)b.off + kafka::kBatchAttrOffset, re = (int64_t)(b.off + b.len);
    const int64_t len = re - rs;
    const int64_t n = (len + kCrcChunkBytes - 1) / kCrcChunkBytes;
    batch_chunks.emplace_back(chunks.size(), (size_t)n);
    for (int64_t k = 0; k < n; ++k) {
      CrcChunk c;
      c.end = re - (int64_t)kCrcChunkBytes * (n - 1 - k);
      c.len = k == 0 ? (int32_t)(len - (int64_t)kCrcChunkBytes * (n - 1)) : kCrcChunkBytes;
      c.pad_ = 0;
      chunks.push_back(c);
    }
  }
  std::vector<int> rec_of;  // JsonRecord j -> record index
  int ntiles = 0, ngroups = 0;
  for (size_t i = 0; i < nrec_all; ++i) {
    if (io.status[i] != codec::OK) continue;
    const kafka::RecordRef& rr = f.records[i];
    rec_of.push_back((int)i);
    const int nt = json_tile_count(rr.value_off + io.arr_off[i], (int32_t)io.arr_len[i]);
    ntiles += nt;
    ngroups += (nt + kGroupTiles - 1) / kGroupTiles;
    lo = std::min(lo, (size_t)rr.value_off);
    hi = std::max(hi, (size_t)(rr.value_off + rr.value_len));
  }
  const size_t nc = chunks.size(), nr = rec_of.size();
  if (nc == 0 && nr == 0) return;
  // packed body (the source's PackTap, text_pack.h): the whole body crosses the link packed and
  // is expanded in its device mirror; otherwise the span holding batches and records, raw
  const bool packed = f.tap_result >= 0;
  if (packed) {
    lo = 0;
    hi = f.size;
  }
  lo &= ~(size_t)15;
  const size_t span = hi - lo;
  const size_t ng = packed ? codec::pack_groups(span) : 0;
  const size_t link = packed ? (size_t)f.tap_result : span;
  // the per-tile token counts stay with the fetch buffer: at the end of its device mirror when
  // they fit behind the text (and the packed stream), so the parse - here or in the replica that
  // later takes these records - reuses them instead of counting again
  const size_t ncnt = (size_t)ntiles + (size_t)ngroups;  // per record: tile counts, group sums
  int64_t cnt_base = -1;
  if (ntiles > 0) {
    const size_t used = packed ? codec::pack_offset(span) + link : hi;
    const size_t cb = (ncnt * sizeof(int) + 255) & ~(size_t)255;
    if (dev_cap > cb + 256 && ((dev_cap - cb) & ~(size_t)255) >= ((used + 64 + 255) & ~(size_t)255))
      cnt_base = (int64_t)((dev_cap - cb) & ~(size_t)255);
  }
  // parse at ingest: every counted record whose arena slots fit, images taken from its counts on
  // the device (JsonRecord::images = -1), verdicts per tile into host memory
  const int64_t per = (int64_t)H * W * C;
  const int64_t S = 2 * per;
  const bool parse = arena && cnt_base >= 0 && per > 0;
  std::vector<int> pjs;  // parse record p -> counting record j
  int ptiles = 0;
  if (parse) {
    for (size_t j = 0; j < nr; ++j) {
      const size_t i = (size_t)rec_of[j];
      const int64_t off = f.records[i].value_off + io.arr_off[i];
      const int64_t slot = (off + S - 1) / S, cap = io.arr_len[i] / S;
      if (cap <= 0 || (slot + cap) * per * (int64_t)sizeof(float) > (int64_t)arena_bytes) continue;
      pjs.push_back((int)j);
      ptiles += json_tile_count(off, (int32_t)io.arr_len[i]);
    }
  }
  const size_t np = pjs.size();
  const size_t o_chunks = align16(ng * 2 * sizeof(uint32_t));  // (the pack group table first)
  const size_t o_groups = o_chunks + align16(nc * sizeof(CrcChunk));
  const size_t o_recs = o_groups + align16((size_t)ngroups * sizeof(int2));
  const size_t o_precs = o_recs + nr * sizeof(JsonRecord);  // (JsonRecord is 48 bytes)
  const size_t o_ptr = o_precs + np * sizeof(JsonRecord);
  const size_t o_gsum = o_ptr + align16((size_t)ptiles * sizeof(int));
  const size_t o_crc = o_gsum + align16((size_t)ngroups * 4);
  const size_t o_gbad = o_crc + align16(nc * 4);
  const size_t o_pbad = o_gbad + align16((size_t)ngroups * 4);
  const size_t io_bytes = o_pbad + align16((size_t)ptiles * 4);
  check_hip(hipSetDevice(device_), "ingest: hipSetDevice");
  grow(L, io_bytes + 16, ncnt + 1);
  // the plan part [0, o_gsum): written into the fetch's own pinned chunk, behind the bytes the
  // copy moves anyway, when it fits before the counts (the chunk is pinned and mirrored at the
  // same offsets), so ONE DMA carries text and plan; else into the lane's buffer, its own DMA.
  // (Sampled device timing, GALE_INGEST_DEV_TIMING: the copies were the largest device span of
  // a fetch, 40-60 us, mostly per-DMA latency - profiles/r6_ingest_device_split.jsonl)
  // (past every byte of the fetch: host code may still read records this plan skips)
  const size_t used = std::max((size_t)f.size, packed ? codec::pack_offset(span) + link : hi);
  const size_t plan_off = (used + 255) & ~(size_t)255;
  const size_t plan_lim = cnt_base >= 0 ? (size_t)cnt_base : dev_cap;
  const bool plan_in_chunk = !plan_separate_ && plan_off + o_gsum <= plan_lim;
  uint8_t* hpl = plan_in_chunk ? f.buf.get() + plan_off : L.h_io;  // host view of the plan
  uint8_t* dpl = plan_in_chunk ? dev + plan_off : L.d_io;          // device view
  CrcChunk* hc = reinterpret_cast<CrcChunk*>(hpl + o_chunks);
  int2* hg = reinterpret_cast<int2*>(hpl + o_groups);
  JsonRecord* hr = reinterpret_cast<JsonRecord*>(hpl + o_recs);
  if (nc) memcpy(hc, chunks.data(), nc * sizeof(CrcChunk));
  int tile = 0, grp = 0;
  for (size_t j = 0; j < nr; ++j) {
    const size_t i = (size_t)rec_of[j];
    JsonRecord& jr = hr[j];
    jr.off = f.records[i].value_off + io.arr_off[i];
    jr.len = (int32_t)io.arr_len[i];
    jr.slot = 0;
    jr.images = 0;
    jr.status = 0;
    jr.tile0 = tile;
    jr.has_cnt = 0;
    jr.cnt_off = 0;
    jr.grp0 = grp;
    const int nt = json_tile_count(jr.off, jr.len);
    for (int t0 = 0; t0 < nt; t0 += kGroupTiles) {
      hg[grp].x = (int)j;
      hg[grp].y = t0;
      ++grp;
    }
    tile += nt;
  }
  JsonRecord* hp = reinterpret_cast<JsonRecord*>(hpl + o_precs);
  int* hpt = reinterpret_cast<int*>(hpl + o_ptr);
  {
    int pt = 0;
    for (size_t k = 0; k < np; ++k) {
      const JsonRecord& jr = hr[pjs[k]];
      JsonRecord& pr = hp[k];
      pr = jr;
      pr.slot = (int32_t)((jr.off + S - 1) / S);
      pr.images = -1;  // from the counts, on the device
      pr.status = 0;
      pr.tile0 = pt;
      pr.has_cnt = 1;
      pr.cnt_off = cnt_base + (int64_t)(jr.tile0 + jr.grp0) * (int64_t)sizeof(int);
      pr.grp0 = 0;
      const int nt = json_tile_count(pr.off, pr.len);
      for (int t = 0; t < nt; ++t) hpt[pt + t] = (int)k;
      pt += nt;
    }
  }
  // ---- device: text span -> mirror (packed: ONE H2D of the packed stream, expanded in place),
  // plan H2D, CRC windows, token counts [, parse]; the kernels store their results (window CRCs,
  // group sums and verdicts, parse tile verdicts) straight into the lane's host-mapped buffer,
  // so no D2H copy follows. Both copies are DMAs (SDMA engines, no CU time). Kernel READS of
  // host memory stay out of this path: under the serving load the link is busy with these DMAs
  // and every read waits behind them - expanding the packed text straight from the host-mapped
  // chunk made text_unpack 15x slower (device time per batch 0.34 -> 2.9 ms), and reading only
  // the plan and the step's metadata that way still stretched every kernel by 25-40 %
  // (profiles/r5_step_ab.txt).
  hipStream_t st = L.stream;
  const int64_t t_plan = mono_ns();  // plan built; the HIP calls follow
  const bool timed = dev_every_ > 0 && L.nrun++ % dev_every_ == 0;
  if (timed) check_hip(hipEventRecord(L.tev[0], st), "ingest: timing event");
  if (packed) memcpy(hpl, f.buf.get() + codec::tab_offset(span), ng * 2 * sizeof(uint32_t));
  const size_t c_lo = packed ? codec::pack_offset(span) : lo;
  const size_t c_len = packed ? link : span;
  if (plan_in_chunk) {
    check_hip(hipMemcpyAsync(dev + c_lo, f.buf.get() + c_lo, plan_off + o_gsum - c_lo,
                             hipMemcpyHostToDevice, st),
              "ingest: H2D text + plan");
  } else {
    check_hip(hipMemcpyAsync(dev + c_lo, f.buf.get() + c_lo, c_len, hipMemcpyHostToDevice, st),
              "ingest: H2D text");
    check_hip(hipMemcpyAsync(L.d_io, L.h_io, o_gsum, hipMemcpyHostToDevice, st),
              "ingest: H2D plan");
  }
  plan_in_chunk_ += plan_in_chunk;
  if (timed) check_hip(hipEventRecord(L.tev[1], st), "ingest: timing event");
  text_bytes_ += (int64_t)span;
  link_bytes_ += (int64_t)link;
  uint32_t* d_crc = reinterpret_cast<uint32_t*>(L.h_io + o_crc);   // (host-mapped results)
  int* d_gsum = reinterpret_cast<int*>(L.h_io + o_gsum);
  int* d_gbad = reinterpret_cast<int*>(L.h_io + o_gbad);
  int* d_pbad = reinterpret_cast<int*>(L.h_io + o_pbad);
  JsonRecord* d_rec = reinterpret_cast<JsonRecord*>(dpl + o_recs);
  int* d_cnt = cnt_base >= 0 ? reinterpret_cast<int*>(dev + cnt_base) : L.d_counts;
  // CRC windows and token counts: one launch, one pass of workgroups over the buffer. Packed,
  // the same launch expands the text: CRC and counting waves read the packed stream, and the
  // counting waves store each record's text into the mirror for the parse (r4 ran a separate
  // text_unpack pass over the whole body first: a third of the ingest launches, 16 % of the
  // GPU's busy time under the serving load, profiles/r5_step_ab.txt)
  check_hip(ingest_crc_count(dev, reinterpret_cast<const CrcChunk*>(dpl + o_chunks), (int)nc,
                             d_tables_, d_crc, (int)nr, ngroups, d_rec,
                             reinterpret_cast<const int2*>(dpl + o_groups), d_cnt, d_gsum,
                             d_gbad, st, packed ? dev + codec::pack_offset(span) : nullptr,
                             packed ? reinterpret_cast<const uint32_t*>(dpl) : nullptr,
                             packed ? dev : nullptr),
            "ingest: crc32c + count");
  if (timed) check_hip(hipEventRecord(L.tev[2], st), "ingest: timing event");
  // the parse right behind it, same stream (the counts are in place when it starts): the text
  // -> fp32 images in the fetch's arena, so the batch step later runs only the forward
  if (np > 0)
    check_hip(json_parse_instances((int)np, ptiles, reinterpret_cast<JsonRecord*>(dpl + o_precs),
                                   reinterpret_cast<const int*>(dpl + o_ptr), dev, H, W, C,
                                   L.d_counts, arena, st, /*count_pass=*/false, nullptr, nullptr,
                                   d_pbad),
              "ingest: parse");
  if (timed) check_hip(hipEventRecord(L.tev[3], st), "ingest: timing event");
  check_hip(hipEventRecord(L.done, st), "ingest: event");
  const int64_t t_wait = mono_ns();
  wait(L);
  const int64_t t_post = mono_ns();
  ++runs_;
  prep_ns_ += t_wait - t_start;
  plan_ns_ += t_plan - t_start;
  wait_ns_ += t_post - t_wait;
  if (timed) {
    float ms[3] = {0.f, 0.f, 0.f};
    for (int k = 0; k < 3; ++k)
      check_hip(hipEventElapsedTime(&ms[k], L.tev[k], L.tev[k + 1]), "ingest: event time");
    ++dev_runs_;
    dev_copy_ns_ += (int64_t)(ms[0] * 1e6);
    dev_count_ns_ += (int64_t)(ms[1] * 1e6);
    dev_parse_ns_ += (int64_t)(ms[2] * 1e6);
    dev_wait_ns_ += t_post - t_wait;
  }
  // ---- host: join the windows of each batch and compare; images from the element counts
  const uint32_t* crc = reinterpret_cast<const uint32_t*>(L.h_io + o_crc);
  for (size_t b = 0; b < batch_chunks.size(); ++b) {
    const kafka::BatchSpan& bs = f.batches[b];
    uint32_t raw = 0;
    for (size_t k = 0; k < batch_chunks[b].second; ++k) {
      const uint32_t c = crc[batch_chunks[b].first + k];
      raw = k == 0 ? c : shift_chunk_(raw) ^ c;
    }
    // standard CRC32C = raw ^ (initial ~0 carried over the message) ^ final ~0
    const uint64_t len = bs.len - (size_t)kafka::kBatchAttrOffset;
    const uint32_t got = raw ^ kafka::crc32c_shift(0xffffffffu, len) ^ 0xffffffffu;
    kafka::Reader cr(f.buf.get() + bs.off + kafka::kBatchCrcOffset, 4);
    io.batch_ok[b] = got == cr.u32();
  }
  // a record's tokens: the sums of its tile groups (and its verdict: the worst group's)
  const int* gsum = reinterpret_cast<const int*>(L.h_io + o_gsum);
  const int* gbad = reinterpret_cast<const int*>(L.h_io + o_gbad);
  const int* pbad = reinterpret_cast<const int*>(L.h_io + o_pbad);
  std::vector<int> parsed_as(nr, -1);
  for (size_t k = 0; k < np; ++k) parsed_as[(size_t)pjs[k]] = (int)k;
  for (size_t j = 0; j < nr; ++j) {
    const size_t i = (size_t)rec_of[j];
    const int64_t g1 = j + 1 < nr ? hr[j + 1].grp0 : ngroups;
    int64_t tok = 0;
    int bad = 0;
    for (int64_t g = hr[j].grp0; g < g1; ++g) {
      tok += gsum[g];
      bad |= gbad[g];
    }
    if (bad != 0) {
      io.status[i] = codec::BAD_NUMBER;
    } else if (tok == 0) {
      io.status[i] = codec::EMPTY;
    } else if (tok % per != 0) {
      io.status[i] = codec::BAD_SHAPE;
    } else {
      io.images[i] = (int32_t)(tok / per);
      if (cnt_base >= 0)
        io.cnt_off[i] = cnt_base + (hr[j].tile0 + hr[j].grp0) * (int64_t)sizeof(int);
      const int k = parsed_as[j];
      if (k >= 0) {
        // the parse's verdict (structure, element count, numbers): the worst of its tiles, in
        // the replica's mapping (GpuReplica::wait)
        const JsonRecord& pr = hp[k];
        const int nt = json_tile_count(pr.off, pr.len);
        int v = 0;
        for (int t = 0; t < nt; ++t) v = std::max(v, pbad[pr.tile0 + t]);
        if (v == 1 || v == 3) io.status[i] = codec::BAD_SHAPE;
        else if (v == 2) io.status[i] = codec::BAD_NUMBER;
        else io.img[i] = arena + (int64_t)pr.slot * per;
      }
    }
  }
  post_ns_ += mono_ns() - t_post;
}

}  // namespace gale
