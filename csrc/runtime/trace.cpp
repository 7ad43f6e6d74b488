// roctx tracing (see trace.h).
#include "trace.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>

#include <rocprofiler-sdk-roctx/roctx.h>

namespace gale {
namespace trace {
namespace {
std::atomic<int> g_on{-1};  // -1: not yet read from the environment
}

bool enabled() {
  int v = g_on.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("GALE_ROCTX");
    v = (e && *e && strcmp(e, "0") != 0) ? 1 : 0;
    g_on.store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

void set_enabled(bool on) { g_on.store(on ? 1 : 0, std::memory_order_relaxed); }
void push(const char* name) { roctxRangePushA(name); }
void pop() { roctxRangePop(); }
void mark(const char* name) {
  if (enabled()) roctxMarkA(name);
}

}  // namespace trace
}  // namespace gale
