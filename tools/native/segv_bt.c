/* Diagnostic (not product code): on SIGSEGV / SIGABRT print the native backtrace of the faulting
 * thread to stderr, then re-raise with the default action.  Loaded with ctypes.CDLL by
 * tools/probes/graph_queue_probe.py before a captured step is replayed. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <stdio.h>
#include <unistd.h>

static void on_fault(int sig, siginfo_t* info, void* ctx) {
  (void)ctx;
  void* frames[128];
  const char msg[] = "\n[segv_bt] native backtrace:\n";
  write(2, msg, sizeof(msg) - 1);
  const int n = backtrace(frames, 128);
  backtrace_symbols_fd(frames, n, 2);
  char buf[64];
  const int m = snprintf(buf, sizeof(buf), "[segv_bt] signal %d addr %p\n", sig, info ? info->si_addr : 0);
  write(2, buf, m > 0 ? m : 0);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
}
