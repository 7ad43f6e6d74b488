// Fatal-signal reporter (SURVEY.md §5.1/§5.3 diagnostics): on SIGSEGV / SIGBUS / SIGILL / SIGFPE
// / SIGABRT, write the signal, the faulting address, the crashing thread's name (gl-src<i>,
// gl-rep<i>, ... : which pipeline stage) and the native backtrace to stderr, then hand the
// signal to whatever handler was installed before (Python's faulthandler, a profiler's) and
// re-raise it. Installed once when gale._C is imported; GALE_CRASH_HANDLER=0 leaves it out.
//
// Async-signal safety: the report is built with write(2) from a fixed name table and hand-made
// number formatting (no stdio, no strsignal); backtrace() is warmed up at install time (its
// first call may load the unwinder and allocate) and backtrace_symbols_fd() writes without
// malloc. A SIGABRT raised from inside the allocator (heap corruption) skips the backtrace
// unless GALE_CRASH_BACKTRACE=1, so a corrupt heap cannot deadlock the report. The importing
// thread gets an alternate signal stack, so a stack overflow on it is still reported.
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <unistd.h>

namespace gale {

namespace {

constexpr int kSignals[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
constexpr const char* kNames[] = {"SIGSEGV (segmentation fault)", "SIGBUS (bus error)",
                                  "SIGILL (illegal instruction)",
                                  "SIGFPE (arithmetic exception)", "SIGABRT (aborted)"};
constexpr size_t kN = sizeof(kSignals) / sizeof(kSignals[0]);
struct sigaction g_prev[kN];
volatile sig_atomic_t g_in_handler = 0;
bool g_abort_backtrace = false;

void put(const char* s) {
  const ssize_t r = write(2, s, strlen(s));
  (void)r;
}

void put_num(unsigned long v, int base) {
  char buf[24];
  int i = 23;
  buf[i] = '\0';
  do {
    buf[--i] = "0123456789abcdef"[v % (unsigned long)base];
    v /= (unsigned long)base;
  } while (v && i > 2);
  if (base == 16) {
    buf[--i] = 'x';
    buf[--i] = '0';
  }
  put(buf + i);
}

void handler(int sig, siginfo_t* info, void* ctx) {
  size_t k = 0;
  while (k < kN && kSignals[k] != sig) ++k;
  if (!g_in_handler) {
    g_in_handler = 1;
    char name[17] = {0};
    prctl(PR_GET_NAME, name, 0, 0, 0);
    put("\n[gale crash] fatal signal ");
    put_num((unsigned long)sig, 10);
    put(" (");
    put(k < kN ? kNames[k] : "?");
    put(") at address ");
    put_num((unsigned long)(info ? info->si_addr : nullptr), 16);
    put(" in thread '");
    put(name);
    put("'\n");
    if (sig != SIGABRT || g_abort_backtrace) {
      put("[gale crash] native backtrace:\n");
      void* frames[64];
      const int n = backtrace(frames, 64);
      backtrace_symbols_fd(frames, n, 2);
      put("[gale crash] end of backtrace\n");
    }
  }
  // chain: the previous handler (faulthandler prints the Python stacks), else the default
  if (k < kN) {
    const struct sigaction& p = g_prev[k];
    const bool dfl_or_ign = !(p.sa_flags & SA_SIGINFO) &&
                            (p.sa_handler == SIG_DFL || p.sa_handler == SIG_IGN);
    if (!dfl_or_ign) {
      if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction) {
        p.sa_sigaction(sig, info, ctx);
        return;
      }
      if (!(p.sa_flags & SA_SIGINFO) && p.sa_handler) {
        p.sa_handler(sig);
        return;
      }
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

void install_crash_handler() {
  static bool done = false;
  if (done) return;
  done = true;
  const char* off = getenv("GALE_CRASH_HANDLER");
  if (off && off[0] == '0') return;
  const char* bt = getenv("GALE_CRASH_BACKTRACE");
  g_abort_backtrace = bt && bt[0] == '1';
  void* warm[2];
  backtrace(warm, 2);  // load the unwinder now, not inside the handler
  // alternate stack for this (the importing) thread: a stack overflow can still be reported
  static char* alt = nullptr;
  if (!alt) {
    const size_t sz = 64 * 1024;
    alt = static_cast<char*>(malloc(sz));
    if (alt) {
      stack_t ss;
      memset(&ss, 0, sizeof(ss));
      ss.ss_sp = alt;
      ss.ss_size = sz;
      sigaltstack(&ss, nullptr);
    }
  }
  for (size_t k = 0; k < kN; ++k) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kSignals[k], &sa, &g_prev[k]);
  }
}

}  // namespace gale
