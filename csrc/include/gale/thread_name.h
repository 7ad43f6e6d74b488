// Names the calling thread (visible in /proc/<pid>/task/*/comm, top -H, perf, rocprofv3 traces)
// so the host pipeline's CPU time can be attributed per stage: bench.py sums utime+stime of the
// process's threads by name prefix (gl-src, gl-dec, gl-rep, gl-sink, gl-brk, ...).
#pragma once
#include <pthread.h>

#include <string>

namespace gale {

inline void name_thread(const char* prefix, int index = -1) {
  std::string n(prefix);
  if (index >= 0) n += std::to_string(index);
  if (n.size() > 15) n.resize(15);  // the kernel keeps 15 characters + NUL
  pthread_setname_np(pthread_self(), n.c_str());
}

}  // namespace gale
