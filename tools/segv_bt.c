/* segv_bt.c -- TEST HELPER: on SIGSEGV / SIGBUS / SIGABRT, print the native
 * stack (glibc backtrace) of the faulting thread to stderr, then die with the
 * signal as before.  Python's faulthandler shows only Python frames; this
 * names the HIP / RCCL / libmvx function a host-side crash happened in.
 * Loaded with ctypes by tests/mp_worker.py when MVX_SEGV_BT=1.
 *   gcc -O2 -shared -fPIC tools/segv_bt.c -o tools/libsegv_bt.so */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig, siginfo_t *si, void *uc)
{
    void *pc[64];
    int n = backtrace(pc, 64);
    static const char head[] = "\n*** native backtrace (segv_bt) ***\n";
    (void)uc;
    (void)si;
    if (write(2, head, sizeof head - 1) < 0) { /* nothing to do */ }
    backtrace_symbols_fd(pc, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int segv_bt_install(void)
{
    struct sigaction sa;
    void *warm[1];
    backtrace(warm, 1);        /* load libgcc's unwinder now, not inside the handler */
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_fault;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    return sigaction(SIGSEGV, &sa, NULL) | sigaction(SIGBUS, &sa, NULL) | sigaction(SIGABRT, &sa, NULL);
}
