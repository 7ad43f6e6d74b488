// Fatal-signal reporter (SURVEY.md §5.1/§5.3 diagnostics): on SIGSEGV / SIGBUS / SIGILL / SIGFPE
// / SIGABRT, write the signal, the faulting address, the crashing thread's name (gl-src<i>,
// gl-rep<i>, ... : which pipeline stage) and the native backtrace to stderr, then hand the
// signal to whatever handler was installed before (Python's faulthandler, a profiler's) and
// re-raise it. Installed once when gale._C is imported.
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/prctl.h>
#include <unistd.h>

namespace gale {

namespace {

constexpr int kSignals[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
struct sigaction g_prev[sizeof(kSignals) / sizeof(kSignals[0])];
volatile sig_atomic_t g_in_handler = 0;

void put(const char* s) {
  const ssize_t r = write(2, s, strlen(s));
  (void)r;
}

void put_hex(unsigned long v) {
  char buf[24];
  int i = 23;
  buf[i] = '\0';
  do {
    buf[--i] = "0123456789abcdef"[v & 15];
    v >>= 4;
  } while (v && i > 2);
  buf[--i] = 'x';
  buf[--i] = '0';
  put(buf + i);
}

void handler(int sig, siginfo_t* info, void* ctx) {
  size_t k = 0;
  while (k < sizeof(kSignals) / sizeof(kSignals[0]) && kSignals[k] != sig) ++k;
  if (!g_in_handler) {
    g_in_handler = 1;
    char name[17] = {0};
    prctl(PR_GET_NAME, name, 0, 0, 0);
    put("\n[gale crash] fatal signal ");
    char num[8];
    snprintf(num, sizeof(num), "%d", sig);
    put(num);
    put(" (");
    put(strsignal(sig));
    put(") at address ");
    put_hex((unsigned long)(info ? info->si_addr : nullptr));
    put(" in thread '");
    put(name);
    put("'\n[gale crash] native backtrace:\n");
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    put("[gale crash] end of backtrace\n");
  }
  // chain: the previous handler (faulthandler prints the Python stacks), else the default
  if (k < sizeof(kSignals) / sizeof(kSignals[0])) {
    const struct sigaction& p = g_prev[k];
    if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction) {
      p.sa_sigaction(sig, info, ctx);
      return;
    }
    if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
      p.sa_handler(sig);
      return;
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
  void* warm[2];
  backtrace(warm, 2);  // load the unwinder now, not inside the handler
  for (size_t k = 0; k < sizeof(kSignals) / sizeof(kSignals[0]); ++k) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kSignals[k], &sa, &g_prev[k]);
  }
}

}  // namespace gale
