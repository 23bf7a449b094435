// Debug aid (not product code): load with ctypes.CDLL before a run; on SIGABRT
// or SIGSEGV it prints the native backtrace of the faulting thread to stderr.
//   g++ -O1 -g -shared -fPIC -rdynamic tools/dbg/abrt_bt.cpp -o tools/dbg/libabrt_bt.so
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_sig(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char* m = sig == SIGABRT ? "abrt_bt: SIGABRT\n" : "abrt_bt: SIGSEGV\n";
  (void)!write(2, m, strlen(m));
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void install() {
  signal(SIGABRT, on_sig);
  signal(SIGSEGV, on_sig);
}
