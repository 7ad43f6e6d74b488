// Inference replicas (see replica.h).
#include "replica.h"

#include <math.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <stdexcept>

#include "../codec/json_codec.h"

namespace gale {

// ---------------------------------------------------------------------------------------------
// StubReplica
// ---------------------------------------------------------------------------------------------

StubReplica::StubReplica(int H, int W, int C, int classes, int max_images, int delay_us,
                         bool compute, int locality)
    : H_(H), W_(W), C_(C), classes_(classes), max_images_(max_images), delay_us_(delay_us),
      compute_(compute), locality_(locality) {
  x_.resize((size_t)max_images * H * W * C);
  probs_.resize((size_t)max_images * classes);
}

void StubReplica::submit(Batch& b) {
  const size_t per = (size_t)H_ * W_ * C_;
  int slot = 0;
  b.dev_status.assign(b.recs.size(), codec::OK);
  if (!compute_) {
    int n = 0;
    for (const InRecord& r : b.recs) n += r.images;
    std::fill(probs_.begin(), probs_.begin() + (size_t)n * classes_, 1.0f / (float)classes_);
    if (delay_us_ > 0) usleep((useconds_t)delay_us_);
    b.probs = probs_.data();
    b.pred_text = nullptr;
    return;
  }
  for (size_t ri = 0; ri < b.recs.size(); ++ri) {
    InRecord& r = b.recs[ri];
    int n = 0;
    const int st = codec::parse_instances_host(r.value, (size_t)r.len, H_, W_, C_,
                                               x_.data() + (size_t)slot * per,
                                               max_images_ - slot, &n);
    if (st != codec::OK) b.dev_status[ri] = st;
    for (int i = 0; i < r.images; ++i) {
      const float* img = x_.data() + (size_t)(slot + i) * per;
      float* out = probs_.data() + (size_t)(slot + i) * classes_;
      if (st != codec::OK) {
        std::fill(out, out + classes_, 0.f);
        continue;
      }
      double mx = -1e300;
      for (int k = 0; k < classes_; ++k) {
        double s = 0;
        for (size_t p = (size_t)(k % C_); p < per; p += (size_t)C_) s += img[p];
        const double logit = (k + 1) * s / (double)(per / (size_t)C_);
        out[k] = (float)logit;
        mx = std::max(mx, logit);
      }
      double sum = 0;
      for (int k = 0; k < classes_; ++k) sum += exp((double)out[k] - mx);
      for (int k = 0; k < classes_; ++k) out[k] = (float)(exp((double)out[k] - mx) / sum);
    }
    slot += r.images;
  }
  if (delay_us_ > 0) usleep((useconds_t)delay_us_);
  b.probs = probs_.data();
  b.pred_text = nullptr;
}

void StubReplica::wait(Batch& b) { (void)b; }

}  // namespace gale
