/* In-process sampling profiler for host code (tools/, not product): SIGPROF every `us`
 * microseconds of CPU time records the interrupted instruction pointer; the Python driver
 * (tools/host_profile.py) maps the samples to symbols of the loaded libraries.  No perf or
 * gdb in this image.
 * build: gcc -O2 -shared -fPIC -o tools/libsampler.so tools/sampler.c */
#define _GNU_SOURCE
#include <signal.h>
#include <stdint.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>

#define CAP (1 << 20)
static uint64_t g_ips[CAP];
static volatile size_t g_n = 0;

static void on_prof(int sig, siginfo_t* si, void* ctx) {
    (void)sig;
    (void)si;
    ucontext_t* uc = (ucontext_t*)ctx;
    size_t n = g_n;
    if (n < CAP) {
        g_ips[n] = (uint64_t)uc->uc_mcontext.gregs[REG_RIP];
        g_n = n + 1;
    }
}

int sampler_start(int us) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGPROF, &sa, 0) != 0) return -1;
    struct itimerval it;
    it.it_interval.tv_sec = 0;
    it.it_interval.tv_usec = us;
    it.it_value = it.it_interval;
    g_n = 0;
    return setitimer(ITIMER_PROF, &it, 0);
}

size_t sampler_stop(uint64_t* out, size_t cap) {
    struct itimerval it;
    memset(&it, 0, sizeof(it));
    setitimer(ITIMER_PROF, &it, 0);
    size_t n = g_n < cap ? g_n : cap;
    memcpy(out, g_ips, n * sizeof(uint64_t));
    return n;
}
