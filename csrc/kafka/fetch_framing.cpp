// FramingWalker (see fetch_framing.h).
#include "fetch_framing.h"

#include <string.h>

#include <algorithm>

namespace gale {
namespace kafka {

namespace {

inline uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
inline uint16_t be16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

// zig-zag varint at p (< limit): false = incomplete (*need: the offset that must be available)
inline bool varint(const uint8_t* d, size_t& p, size_t limit, int64_t& v, size_t& need) {
  uint64_t u = 0;
  for (int s = 0; s < 64; s += 7) {
    if (p >= limit) {
      need = p + 1;
      return false;
    }
    const uint8_t b = d[p++];
    u |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) {
      v = (int64_t)((u >> 1) ^ (~(u & 1) + 1));
      return true;
    }
  }
  v = -1;  // malformed: the caller copies the rest of the batch whole
  return true;
}

}  // namespace

void FramingWalker::reset(uint8_t* dst, size_t n) {
  dst_ = dst;
  n_ = n;
  copy_ = skipped_ = 0;
  ilo_ = ihi_ = 0;
  st_ = RESP;
  pos_ = 0;
  topics_left_ = parts_left_ = recs_left_ = 0;
  region_end_ = batch_end_ = 0;
}

size_t FramingWalker::step(size_t limit) {
  // bytes up to `target` are copied whole (no interiors in them): demand them
  auto raw_to = [&](size_t target, State next) -> size_t {
    target = std::min(target, n_);
    if (limit < target) return target;
    pos_ = target;
    st_ = next;
    return 0;
  };
  switch (st_) {
    case RESP:  // throttle_time_ms, topic count
      if (pos_ + 8 > limit) return pos_ + 8;
      topics_left_ = (int32_t)be32(dst_ + pos_ + 4);
      pos_ += 8;
      st_ = TOPIC;
      return 0;
    case TOPIC: {
      if (topics_left_ <= 0) return raw_to(n_, TAIL);
      if (pos_ + 2 > limit) return pos_ + 2;
      const int16_t l = (int16_t)be16(dst_ + pos_);
      const size_t nl = l > 0 ? (size_t)l : 0;
      if (pos_ + 2 + nl + 4 > limit) return pos_ + 2 + nl + 4;
      parts_left_ = (int32_t)be32(dst_ + pos_ + 2 + nl);
      pos_ += 2 + nl + 4;
      --topics_left_;
      st_ = PART;
      return 0;
    }
    case PART: {
      if (parts_left_ <= 0) {
        st_ = TOPIC;
        return 0;
      }
      // index 4, error 2, high watermark 8, last stable offset 8, aborted transactions count 4
      if (pos_ + 26 > limit) return pos_ + 26;
      const int32_t na = (int32_t)be32(dst_ + pos_ + 22);
      const size_t hdr = 26 + 16 * (size_t)std::max(0, na) + 4;
      if (pos_ + hdr > limit) return pos_ + hdr;
      const int32_t rl = (int32_t)be32(dst_ + pos_ + hdr - 4);
      pos_ += hdr;
      region_end_ = std::min(n_, pos_ + (size_t)std::max(0, rl));
      --parts_left_;
      st_ = REGION;
      return 0;
    }
    case REGION: {  // at a batch boundary inside a partition's records
      if (pos_ >= region_end_) {
        st_ = PART;
        return 0;
      }
      if (region_end_ - pos_ < 61) return raw_to(region_end_, PART);  // partial trailing batch
      if (pos_ + 12 > limit) return pos_ + 12;
      const int32_t bl = (int32_t)be32(dst_ + pos_ + 8);
      if (bl < 49 || pos_ + 12 + (size_t)bl > region_end_) return raw_to(region_end_, PART);
      batch_end_ = pos_ + 12 + (size_t)bl;
      st_ = BATCH;
      return 0;
    }
    case BATCH: {
      if (pos_ + 61 > limit) return pos_ + 61;
      const int magic = (int8_t)dst_[pos_ + 16];
      const uint16_t attrs = be16(dst_ + pos_ + 21);
      const int32_t count = (int32_t)be32(dst_ + pos_ + 57);
      if (magic != 2 || (attrs & 7) || (attrs & 0x20) || count < 0)
        return raw_to(batch_end_, REGION);  // compressed / control / other formats: whole
      recs_left_ = count;
      pos_ += 61;
      st_ = RECORD;
      return 0;
    }
    case RECORD: {
      if (recs_left_ <= 0 || pos_ >= batch_end_) return raw_to(batch_end_, REGION);
      size_t p = pos_, need = 0;
      const size_t lim = std::min(limit, batch_end_);
      int64_t rlen, tsd, od, klen, vlen;
      if (!varint(dst_, p, lim, rlen, need)) return need;
      const size_t rend = p + (size_t)std::max<int64_t>(rlen, 0);
      if (rlen < 0 || rend > batch_end_) return raw_to(batch_end_, REGION);
      if (p + 1 > lim) return p + 1;
      ++p;  // attributes
      if (!varint(dst_, p, lim, tsd, need)) return need;
      if (!varint(dst_, p, lim, od, need)) return need;
      if (!varint(dst_, p, lim, klen, need)) return need;
      if (klen > 0) {
        if (p + (size_t)klen > rend) return raw_to(batch_end_, REGION);
        if (p + (size_t)klen > lim) return p + (size_t)klen;  // the key is copied whole
        p += (size_t)klen;
      }
      if (!varint(dst_, p, lim, vlen, need)) return need;
      if (vlen > 0 && p + (size_t)vlen > rend) return raw_to(batch_end_, REGION);
      if (vlen > (int64_t)(kHead + kTail + 64)) {
        ilo_ = p + kHead;
        ihi_ = p + (size_t)vlen - kTail;
      }
      pos_ = rend;
      --recs_left_;
      return 0;
    }
    case TAIL:
    default:
      return raw_to(n_, TAIL);
  }
}

void FramingWalker::feed(const uint8_t* win, size_t from, size_t avail) {
  avail = std::min(avail, n_);
  auto copy_to = [&](size_t e) {
    if (e > copy_) {
      memcpy(dst_ + copy_, win + (copy_ - from), e - copy_);
      copy_ = e;
    }
  };
  for (;;) {
    if (ilo_ < ihi_) {
      if (ilo_ < copy_) ilo_ = copy_;
      if (ilo_ < ihi_) {
        copy_to(std::min(avail, ilo_));
        if (copy_ < ilo_) return;
        if (avail < ihi_) return;  // the interior is still streaming past
        skipped_ += ihi_ - copy_;
        copy_ = ihi_;
      }
      ilo_ = ihi_ = 0;
    }
    if (copy_ >= n_) return;
    const size_t need = step(copy_);
    if (need == 0) continue;
    const size_t e = std::min(std::min(need, n_), avail);
    if (e <= copy_) return;  // (more data needed)
    copy_to(e);
  }
}

}  // namespace kafka
}  // namespace gale
