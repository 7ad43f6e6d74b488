// Host micro-benchmark for the nibble-transport receive path (csrc/codec/text_pack.h): how many
// CPU seconds per GB does a consumer spend receiving Kafka fetch bodies over loopback TCP from a
// zero-copy sender (vmsplice of DRAM-resident stored text, as the embedded broker serves), for
//   raw     recv() straight into a large buffer pool (today's default: the text lands in pinned
//           memory, which the GPU then reads over the link),
//   pack2   recv() into the pool, then pack the received piece into the same chunk (round 3's
//           --text-pack; a second pass over memory),
//   bounce  recv() into a small per-thread bounce buffer (cache resident), pack each piece from
//           there into the pool: only the packed half is written to memory.
// The sender either splices the stored pages (zero copy) or copies them with send() as the
// broker's default writev path does; sender and receiver of a pair can be pinned to two cores of
// one CCD (shared L3: the receive copy reads what the sender just wrote from L3) or of two CCDs.
// Usage: recv_bounce_bench <mode> <pairs> <seconds> [piece_kb] [splice|copy] [none|same|cross]
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../codec/text_pack.h"

namespace {

constexpr size_t kBody = 8u << 20;  // one fetch body
std::atomic<bool> g_stop{false};

double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

double thread_cpu_s() {
  timespec t;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

// stored text: JSON-number-like bytes (the packable alphabet), DRAM resident (256 MB per sender)
std::vector<uint8_t> make_store(size_t n, unsigned seed) {
  std::vector<uint8_t> s(n);
  const char* a = "0123456789[],-.E";
  uint64_t x = seed * 0x9e3779b97f4a7c15ull + 1;
  for (size_t i = 0; i < n; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    s[i] = (uint8_t)a[x & 15];
  }
  return s;
}

void pin_to(int cpu) {
  if (cpu < 0) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

std::atomic<double> g_send_cpu{0};

void add_send_cpu(double c);

void sender_copy(int fd, unsigned seed, int cpu) {
  pin_to(cpu);
  std::vector<uint8_t> store = make_store(256u << 20, seed);
  const double c0 = thread_cpu_s();
  size_t pos = 0;
  while (!g_stop) {
    if (pos + (1u << 20) > store.size()) pos = 0;
    const ssize_t k = send(fd, store.data() + pos, 1u << 20, 0);
    if (k <= 0) break;
    pos += (size_t)k;
  }
  add_send_cpu(thread_cpu_s() - c0);
}

void add_send_cpu(double c) {
  double cur = g_send_cpu.load();
  while (!g_send_cpu.compare_exchange_weak(cur, cur + c)) {
  }
}

void sender(int fd, unsigned seed, int cpu) {
  pin_to(cpu);
  std::vector<uint8_t> store = make_store(256u << 20, seed);
  const double c0 = thread_cpu_s();
  struct Acc {
    double c0;
    ~Acc() { add_send_cpu(thread_cpu_s() - c0); }
  } acc{c0};
  int p[2];
  if (pipe(p) != 0) return;
  fcntl(p[1], F_SETPIPE_SZ, 1 << 20);
  size_t pos = 0;
  while (!g_stop) {
    // one body: vmsplice the stored pages into the pipe, splice the pipe into the socket
    size_t left = kBody;
    while (left && !g_stop) {
      if (pos + 65536 > store.size()) pos = 0;
      iovec iv{store.data() + pos, std::min<size_t>(left, 1 << 20)};
      if (pos + iv.iov_len > store.size()) iv.iov_len = store.size() - pos;
      ssize_t m = vmsplice(p[1], &iv, 1, 0);
      if (m <= 0) return;
      size_t in_pipe = (size_t)m;
      while (in_pipe) {
        ssize_t k = splice(p[0], nullptr, fd, nullptr, in_pipe, SPLICE_F_MORE);
        if (k <= 0) return;
        in_pipe -= (size_t)k;
      }
      pos += (size_t)m;
      left -= (size_t)m;
    }
  }
}

struct Result {
  double bytes = 0, cpu = 0;
};

void receiver(int fd, const char* mode, size_t piece, Result* res, int cpu) {
  pin_to(cpu);
  // pool: 64 chunks of (body + packed + tab), cycled, so writes stream to DRAM
  const size_t chunk = gale::codec::pack_layout_bytes(kBody) + 4096;
  const int nchunks = 64;
  std::vector<uint8_t*> pool(nchunks);
  for (auto& c : pool) {
    c = static_cast<uint8_t*>(aligned_alloc(4096, chunk));
    memset(c, 0, chunk);
  }
  std::vector<uint8_t> bounce(piece + 128);
  const bool raw = !strcmp(mode, "raw"), pack2 = !strcmp(mode, "pack2");
  double c0 = thread_cpu_s();
  size_t total = 0;
  int ci = 0;
  while (!g_stop) {
    uint8_t* buf = pool[(size_t)ci++ % nchunks];
    uint8_t* packed = buf + gale::codec::pack_offset(kBody);
    uint32_t* tab = reinterpret_cast<uint32_t*>(buf + gale::codec::tab_offset(kBody));
    gale::codec::PackState st;
    size_t got = 0;
    size_t bb_base = 0, bb_fill = 0;  // bounce: body offset of bounce[0], bytes held
    while (got < kBody) {
      if (raw || pack2) {
        const ssize_t m = recv(fd, buf + got, std::min(piece, kBody - got), 0);
        if (m <= 0) goto out;
        got += (size_t)m;
        if (pack2) gale::codec::text_pack_blocks(buf, got / 64, packed, tab, st);
      } else {
        const ssize_t m = recv(fd, bounce.data() + bb_fill, std::min(piece, kBody - got), 0);
        if (m <= 0) goto out;
        got += (size_t)m;
        bb_fill += (size_t)m;
        const size_t upto = (bb_base + bb_fill) / 64;
        gale::codec::text_pack_blocks(bounce.data() - bb_base, upto, packed, tab, st);
        const size_t keep = bb_base + bb_fill - upto * 64;  // partial block carried over
        memmove(bounce.data(), bounce.data() + bb_fill - keep, keep);
        bb_base = upto * 64;
        bb_fill = keep;
      }
    }
    if (!raw) gale::codec::text_pack_finish(pack2 ? buf : bounce.data() - bb_base, kBody, packed,
                                            tab, st);
    total += kBody;
  }
out:
  res->bytes = (double)total;
  res->cpu = thread_cpu_s() - c0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s raw|pack2|bounce pairs seconds [piece_kb]\n", argv[0]);
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  const char* mode = argv[1];
  const int pairs = atoi(argv[2]);
  const double secs = atof(argv[3]);
  const size_t piece = (size_t)(argc > 4 ? atoi(argv[4]) : 256) << 10;
  const bool copy = argc > 5 && !strcmp(argv[5], "copy");
  const char* pin = argc > 6 ? argv[6] : "none";
  // receivers on the first core of every other CCD (8 cores per CCD, node 0 = CPUs 0-63);
  // senders on the next core of the same CCD, or on the next CCD
  auto rcpu = [&](int i) { return strcmp(pin, "none") ? (i * 16) % 64 : -1; };
  auto scpu = [&](int i) {
    return !strcmp(pin, "same") ? (i * 16) % 64 + 1 : !strcmp(pin, "cross") ? (i * 16) % 64 + 8
                                                                            : -1;
  };
  std::vector<std::thread> th;
  std::vector<Result> res((size_t)pairs);
  std::vector<int> fds;
  for (int i = 0; i < pairs; ++i) {
    int sv[2];
    // loopback TCP pair
    int ls = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a));
    socklen_t al = sizeof(a);
    getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);
    listen(ls, 1);
    sv[0] = socket(AF_INET, SOCK_STREAM, 0);
    connect(sv[0], reinterpret_cast<sockaddr*>(&a), sizeof(a));
    sv[1] = accept(ls, nullptr, nullptr);
    close(ls);
    int bufsz = 8 << 20;
    setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &bufsz, sizeof(bufsz));
    setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &bufsz, sizeof(bufsz));
    fds.push_back(sv[0]);
    fds.push_back(sv[1]);
    if (copy)
      th.emplace_back(sender_copy, sv[0], (unsigned)i + 1, scpu(i));
    else
      th.emplace_back(sender, sv[0], (unsigned)i + 1, scpu(i));
    th.emplace_back(receiver, sv[1], mode, piece, &res[(size_t)i], rcpu(i));
  }
  const double t0 = now_s();
  std::this_thread::sleep_for(std::chrono::milliseconds((int)(secs * 1000)));
  g_stop = true;
  const double el = now_s() - t0;
  for (int fd : fds) shutdown(fd, SHUT_RDWR);
  for (auto& t : th) t.join();
  double bytes = 0, cpu = 0;
  for (auto& r : res) {
    bytes += r.bytes;
    cpu += r.cpu;
  }
  printf("{\"mode\": \"%s\", \"sender\": \"%s\", \"pin\": \"%s\", \"pairs\": %d, "
         "\"piece_kb\": %zu, \"gb_s\": %.2f, \"recv_cores\": %.2f, "
         "\"gb_per_recv_core_s\": %.2f, \"send_cores\": %.2f}\n",
         mode, copy ? "copy" : "splice", pin, pairs, piece >> 10, bytes / el / 1e9, cpu / el,
         bytes / 1e9 / cpu, g_send_cpu.load() / el);
  return 0;
}
