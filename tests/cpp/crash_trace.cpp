// Test-harness helper (oracle/Makefile `harness`), linked into the
// reference's test executables built against both libraries: on SIGSEGV,
// SIGABRT or SIGBUS it writes the faulting thread's backtrace (one frame per
// line, backtrace_symbols_fd: async-signal-safe, no heap) to the file named
// by LPHY_CRASH_TRACE (stderr when unset) and re-raises the signal with its
// default action, so the exit status is unchanged.
// tests/test_gpu_ref_harness.py reads the trace to pin where
// sync_word_test's fault lands (its heap overflow, sync_word_test.cpp:27-29).
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

namespace {

int g_fd = 2;

void put(const char* s) {
    const ssize_t n = (ssize_t)strlen(s);
    if (write(g_fd, s, (size_t)n) != n) return;
}

void on_fatal(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    put("lphy-crash-trace: signal ");
    put(sig == SIGSEGV ? "SIGSEGV\n" : sig == SIGABRT ? "SIGABRT\n" : "SIGBUS\n");
    backtrace_symbols_fd(frames, n, g_fd);
    put("lphy-crash-trace: end\n");
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) void install() {
    void* warm[2];
    (void)backtrace(warm, 2);  // loads the unwinder now, not inside the handler
    if (const char* p = getenv("LPHY_CRASH_TRACE")) {
        const int fd = open(p, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd >= 0) g_fd = fd;
    }
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = on_fatal;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESETHAND | SA_NODEFER;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGABRT, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
}

}  // namespace
