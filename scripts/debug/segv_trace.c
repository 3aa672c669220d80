// Debug aid (not product): print a native backtrace on SIGSEGV.  Loaded with ctypes before a test run.
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <unistd.h>
static void handler(int sig) {
    void* frames[64];
    int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    _exit(128 + sig);
}
__attribute__((constructor)) static void install(void) { signal(SIGSEGV, handler); }
