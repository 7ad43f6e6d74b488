// roctx ranges around the serving pipeline's host stages, so a
// `rocprofv3 --kernel-trace --marker-trace` timeline lines the GPU kernels (JSON parse, fused
// forward) up with fetch / decode / batch / H2D+launch / device-wait / encode+produce.
//
// The reference has no tracing at all (only Storm UI counters, E4). Ranges are off unless
// enabled (GALE_ROCTX=1 or Engine config trace=true): a disabled Range costs one relaxed load.
#pragma once

namespace gale {
namespace trace {

bool enabled();
void set_enabled(bool on);
void push(const char* name);
void pop();
void mark(const char* name);

class Range {
 public:
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) push(name);
  }
  ~Range() {
    if (on_) pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace trace
}  // namespace gale
