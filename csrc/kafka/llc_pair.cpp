// L3-domain pairing of loopback connections: see gale/llc_pair.h.
#include "gale/llc_pair.h"

#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace gale {
namespace llc {
namespace {

std::mutex g_mu;
std::unordered_map<int, std::vector<int>> g_ports;  // local port -> CPUs of the reader's domain
std::atomic<unsigned> g_next{0};
thread_local std::vector<int> t_domain;  // CPUs of the domain this thread was pinned to

std::vector<int> parse_cpu_list(const char* s) {
  std::vector<int> out;
  while (*s) {
    char* end = nullptr;
    const long a = strtol(s, &end, 10);
    if (end == s) break;
    long b = a;
    s = end;
    if (*s == '-') {
      b = strtol(s + 1, &end, 10);
      s = end;
    }
    for (long c = a; c <= b; ++c) out.push_back((int)c);
    while (*s == ',' || *s == '\n' || *s == ' ') ++s;
  }
  return out;
}

// L3 domains (CPU lists) of the CPUs in `mask`, each restricted to the mask, by lowest CPU id
std::map<int, std::vector<int>> domains_of(const cpu_set_t& mask) {
  std::map<int, std::vector<int>> out;
  std::map<std::string, bool> seen;
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &mask)) continue;
    // (GALE_SYSFS_CPU: another root with the same layout, for tests of other topologies)
    static const char* root = getenv("GALE_SYSFS_CPU") ? getenv("GALE_SYSFS_CPU")
                                                        : "/sys/devices/system/cpu";
    char path[512];
    snprintf(path, sizeof(path), "%s/cpu%d/cache/index3/shared_cpu_list", root, c);
    FILE* f = fopen(path, "r");
    if (!f) return {};
    char buf[1024] = {0};
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    if (seen.count(buf)) continue;
    seen[buf] = true;
    std::vector<int> cpus;
    for (int d : parse_cpu_list(buf))
      if (d >= 0 && d < CPU_SETSIZE && CPU_ISSET(d, &mask)) cpus.push_back(d);
    if (!cpus.empty()) out[cpus.front()] = cpus;
  }
  return out;
}

bool pin_to(const std::vector<int>& cpus) {
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  return sched_setaffinity(0, sizeof(set), &set) == 0;
}

}  // namespace

bool enabled() {
  static const bool on = [] {
    const char* e = getenv("GALE_LLC_PAIR");
    return e && e[0] == '1';
  }();
  return on;
}

int pin_self_next_domain() {
  if (!enabled()) return -1;
  cpu_set_t mask;
  if (sched_getaffinity(0, sizeof(mask), &mask) != 0) return -1;
  const std::map<int, std::vector<int>> doms = domains_of(mask);
  if (doms.size() < 2) return -1;
  auto it = doms.begin();
  std::advance(it, g_next.fetch_add(1) % doms.size());
  if (!pin_to(it->second)) return -1;
  t_domain = it->second;
  return it->first;
}

void register_local_port(int local_port) {
  if (!enabled() || t_domain.empty() || local_port <= 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  g_ports[local_port] = t_domain;
}

bool pin_self_for_peer(int peer_port) {
  if (!enabled() || peer_port <= 0) return false;
  std::vector<int> cpus;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_ports.find(peer_port);
    if (it == g_ports.end()) return false;
    cpus = it->second;
  }
  return pin_to(cpus);
}

}  // namespace llc
}  // namespace gale
