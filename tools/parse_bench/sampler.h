// CPU-time sampling profiler for parse_bench (-DH2J_SAMPLE): a POSIX CPU-time timer delivers
// SIGPROF every 50 us of wall time (single-threaded runs); the handler records the interrupted instruction
// pointer.  At exit the addresses are written to $H2J_SAMPLE_OUT (one hex address per line) for
// tools/parse_bench/sample_report.py (addr2line, per source line and per inlined function).
#pragma once
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <ucontext.h>

namespace h2j_sample {
static unsigned long g_pc[1 << 22];
static volatile unsigned long g_n = 0;

static void on_prof(int, siginfo_t*, void* ctx) {
    const ucontext_t* uc = static_cast<const ucontext_t*>(ctx);
    const unsigned long n = g_n;
    if (n < (1ul << 22)) {
        g_pc[n] = static_cast<unsigned long>(uc->uc_mcontext.gregs[REG_RIP]);
        g_n = n + 1;
    }
}

static void dump() {
    const char* out = std::getenv("H2J_SAMPLE_OUT");
    FILE* f = std::fopen(out ? out : "samples.txt", "w");
    if (!f) return;
    for (unsigned long i = 0; i < g_n; i++) std::fprintf(f, "%lx\n", g_pc[i]);
    std::fclose(f);
    std::fprintf(stderr, "sampler: %lu samples\n", static_cast<unsigned long>(g_n));
}

static void start() {
    struct sigaction sa = {};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, nullptr);
    sigevent sev = {};
    sev.sigev_notify = SIGEV_SIGNAL;
    sev.sigev_signo = SIGPROF;
    timer_t t;
    timer_create(CLOCK_MONOTONIC, &sev, &t);
    itimerspec its = {};
    its.it_interval.tv_nsec = 50000;
    its.it_value.tv_nsec = 50000;
    timer_settime(t, 0, &its, nullptr);
    std::atexit(dump);
}
}  // namespace h2j_sample
