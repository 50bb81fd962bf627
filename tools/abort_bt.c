/* Diagnostics for host-side aborts (glibc heap checks) in a GPU test process:
 * loaded by tests/conftest.py when PRK_ABORT_BT=1, it installs a SIGABRT
 * handler that writes the native backtrace (addresses + the owning library
 * and offset, symbolised offline with addr2line) to stderr, then hands the
 * signal to the handler that was there before (Python's faulthandler when
 * run with -X faulthandler, which adds the Python stacks).  Host code only.
 *   gcc -O1 -g -fPIC -shared -o tools/libabort_bt.so tools/abort_bt.c */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_prev;

static void on_abort(int sig, siginfo_t *info, void *uc) {
    static const char hdr[] = "\n[abort_bt] SIGABRT native backtrace:\n";
    void *frames[64];
    const int n = backtrace(frames, 64);
    (void)!write(2, hdr, sizeof(hdr) - 1);
    backtrace_symbols_fd(frames, n, 2);
    sigaction(SIGABRT, &g_prev, NULL);
    if (g_prev.sa_flags & SA_SIGINFO) {
        if (g_prev.sa_sigaction) g_prev.sa_sigaction(sig, info, uc);
    } else if (g_prev.sa_handler != SIG_DFL && g_prev.sa_handler != SIG_IGN) {
        g_prev.sa_handler(sig);
    }
    signal(SIGABRT, SIG_DFL);
    raise(SIGABRT);
}

static void install(void);
static void reinstall_at_exit(void) { install(); }

/* Also re-installed by a C atexit hook: Python's finalisation restores the
 * handlers faulthandler replaced, and the C exit handlers (the HIP runtime's,
 * RCCL's, registered earlier) run after this one. */
int abort_bt_install(void) {
    static int once;
    install();
    if (!once) {
        once = 1;
        atexit(reinstall_at_exit);
    }
    return 0;
}

static void install(void) {
    void *warm[2];
    backtrace(warm, 2); /* loads the unwinder now, not inside the handler */
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_abort;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigemptyset(&sa.sa_mask);
    struct sigaction prev;
    sigaction(SIGABRT, &sa, &prev);
    if (prev.sa_sigaction != on_abort) g_prev = prev;
}
