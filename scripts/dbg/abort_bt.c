/* Debug aid: on SIGABRT print the native backtrace to stderr (loaded with ctypes by
   tests/conftest.py when GF_ABORT_BT=1), then re-raise with the default action. */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_abort(int sig) {
  void* f[64];
  const int n = backtrace(f, 64);
  const char m[] = "\n=== native backtrace (SIGABRT) ===\n";
  write(2, m, sizeof m - 1);
  backtrace_symbols_fd(f, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) void gf_install_abort_bt(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_abort;
  sigaction(SIGABRT, &sa, 0);
}
