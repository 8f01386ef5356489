// Host-only timing of the entropy decoders (no GPU): parses every stream of
// the argument list `reps` times on T threads (each with its own FrameJob,
// streams dealt round-robin) and prints ms/frame (wall / frames, and per
// thread) and TUs/frame.
//   g++ -O2 -std=c++11 -pthread -I../../include -I../../h264-h265-to-jpeg_amd/csrc/host parse_bench.cpp \
//       ../../h264-h265-to-jpeg_amd/csrc/host/{bitstream,cabac_tables,hevc_parser,h264_parser}.cpp
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "bitstream.h"
#include "cabac.h"
#include "job.h"
#ifdef H2J_SAMPLE
#include "sampler.h"
#endif

#ifdef H2J_CORO
#include "coro.h"
namespace h2j {
thread_local void (*g_h2j_yield)() = nullptr;
}
namespace {
// -c: the stream list parsed by two coroutines on this thread (even / odd entries), switched
// before every residual block; the other one alone once a coroutine has run out of pictures
struct CoPair {
    h2j_coro::Co co[2], main;
    int cur = 0;
    const std::vector<std::vector<uint8_t>>* streams;
    int reps;
    double best[2];
};
thread_local CoPair* g_pair = nullptr;
void co_yield() {
    CoPair& p = *g_pair;
    const int o = p.cur ^ 1;
    if (p.co[o].done) return;
    const int me = p.cur;
    p.cur = o;
    h2j_ctx_swap(&p.co[me].sp, p.co[o].sp);
}
void co_body(void* arg) {
    CoPair& p = *g_pair;
    const int me = static_cast<int>(reinterpret_cast<intptr_t>(arg));
    h2j::FrameJob job;
    for (int r = 0; r < p.reps; r++)
        for (size_t i = me; i < p.streams->size(); i += 2) {
            const auto& s = (*p.streams)[i];
            if (h2j::hevc_parse_picture(s.data(), s.size(), job)) std::abort();
        }
    p.co[me].done = true;
    const int o = me ^ 1;
    if (!p.co[o].done) {
        p.cur = o;
        h2j_ctx_swap(&p.co[me].sp, p.co[o].sp);
    }
    h2j_ctx_swap(&p.co[me].sp, p.main.sp);
    std::abort();
}
}  // namespace
#endif
#ifdef H2J_CABAC_COUNT
namespace h2j {
thread_local unsigned long long g_bins_ctx = 0, g_bins_byp = 0;
}
#endif

int main(int argc, char** argv) {
#ifdef H2J_SAMPLE
    h2j_sample::start();
#endif
    if (argc < 2) {
        std::fprintf(stderr, "usage: parse_bench file... [-r reps] [-t threads] [-d (output digest)]\n");
        return 2;
    }
    int reps = 3, threads = 1, pthreads = 1;
    bool coro = false;
    (void)coro;
    bool want_digest = false, want_hist = false, want_min = false;
    std::vector<std::vector<uint8_t>> streams;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "-r" && i + 1 < argc) {
            reps = std::atoi(argv[++i]);
            continue;
        }
        if (a == "-d") {
            want_digest = true;
            continue;
        }
        if (a == "-c") {  // coroutine-paired parse (-DH2J_CORO builds)
            coro = true;
            continue;
        }
        if (a == "-m") {  // min-of-reps per stream (robust to a noisy host): sum of per-stream minima
            want_min = true;
            continue;
        }
        if (a == "-s") {  // transform-block histogram by (component, size, cbf)
            want_hist = true;
            continue;
        }
        if (a == "-p" && i + 1 < argc) {  // threads inside one picture (independent slices)
            pthreads = std::atoi(argv[++i]);
            continue;
        }
        if (a == "-t" && i + 1 < argc) {
            threads = std::atoi(argv[++i]);
            continue;
        }
        FILE* f = std::fopen(argv[i], "rb");
        if (!f) continue;
        std::vector<uint8_t> d;
        uint8_t buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + n);
        std::fclose(f);
        streams.push_back(d);
    }
#ifdef H2J_CORO
    if (coro) {  // paired (two coroutines) vs sequential, interleaved rounds, one thread
        for (int round = 0; round < 3; round++) {
            auto t0 = std::chrono::steady_clock::now();
            {
                h2j::FrameJob job;
                for (int r = 0; r < reps; r++)
                    for (const auto& s : streams)
                        if (h2j::hevc_parse_picture(s.data(), s.size(), job)) return 1;
            }
            const double seq = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            CoPair p;
            p.streams = &streams;
            p.reps = reps;
            g_pair = &p;
            h2j::g_h2j_yield = co_yield;
            h2j_coro::make(p.co[0], 8 << 20, co_body, reinterpret_cast<void*>(0));
            h2j_coro::make(p.co[1], 8 << 20, co_body, reinterpret_cast<void*>(1));
            t0 = std::chrono::steady_clock::now();
            p.cur = 0;
            h2j_ctx_swap(&p.main.sp, p.co[0].sp);
            const double par = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            h2j::g_h2j_yield = nullptr;
            std::free(p.co[0].stack);
            std::free(p.co[1].stack);
            const double nf = static_cast<double>(reps) * streams.size();
            std::printf("round %d: sequential %.4f ms/frame, paired %.4f ms/frame (%+.1f %%)\n", round, seq / nf, par / nf,
                        100.0 * (par - seq) / seq);
        }
        return 0;
    }
#endif
    if (want_min) {
        h2j::FrameJob job;
        double sum = 0;
        for (const auto& s : streams) {
            double best = 1e30;
            for (int r = 0; r < reps; r++) {
                const auto t0 = std::chrono::steady_clock::now();
                const int codec = h2j::detect_codec(s.data(), s.size());
                const int rc = codec == 265 ? h2j::hevc_parse_picture(s.data(), s.size(), job)
                                            : h2j::h264_parse_picture(s.data(), s.size(), job);
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                if (rc) return 1;
                best = std::min(best, ms);
            }
            sum += best;
        }
        std::printf("min-of-%d: %.4f ms/frame\n", reps, sum / static_cast<double>(streams.size()));
        return 0;
    }
    const int total = reps * static_cast<int>(streams.size());
    std::atomic<int> next(0), failed(0);
    std::atomic<size_t> tus(0), coefs(0), bytes(0);
    std::atomic<unsigned long long> bins_ctx(0), bins_byp(0);
    std::atomic<unsigned long long> digest(0);  // order-independent checksum of all parse outputs
    std::atomic<unsigned long long> hist[2][4][2];
    for (auto& a : hist) for (auto& b : a) for (auto& c : b) c = 0;
    auto worker = [&]() {
        h2j::FrameJob job;
        job.threads = pthreads;
        size_t t = 0, c = 0, b = 0;
        for (int i = next++; i < total; i = next++) {
            const auto& s = streams[i % streams.size()];
            const int codec = h2j::detect_codec(s.data(), s.size());
            const int rc = codec == 265 ? h2j::hevc_parse_picture(s.data(), s.size(), job)
                                        : h2j::h264_parse_picture(s.data(), s.size(), job);
            if (rc) {
                std::fprintf(stderr, "parse error %d: %s\n", rc, job.message.c_str());
                failed++;
                return;
            }
            t += job.tus.size();
            if (want_hist)
                for (const h2j_tu& u : job.tus)
                    if (u.log2n >= 2 && u.log2n <= 5) hist[u.c ? 1 : 0][u.log2n - 2][(u.flags & H2J_TU_CBF) ? 1 : 0]++;
            c += job.coefs.size();
            b += s.size();
            if (!want_digest) continue;
            unsigned long long hsh = 1469598103934665603ull;
            auto mix = [&](const void* p, size_t n) {
                const unsigned char* q = static_cast<const unsigned char*>(p);
                for (size_t j = 0; j < n; j++) hsh = (hsh ^ q[j]) * 1099511628211ull;
            };
            mix(job.tus.data(), job.tus.size() * sizeof(h2j_tu));
            mix(job.coefs.data(), job.coefs.size() * sizeof(h2j_coef));
            mix(job.ctbs.data(), job.ctbs.size() * sizeof(h2j_ctb));
            mix(job.slices.data(), job.slices.size() * sizeof(h2j_slice));
            mix(&job.hdr, sizeof(job.hdr));
            digest += hsh;
        }
        tus += t;
        coefs += c;
        bytes += b;
#ifdef H2J_CABAC_COUNT
        bins_ctx += h2j::g_bins_ctx;
        bins_byp += h2j::g_bins_byp;
#endif
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    // one thread: parse on the main thread (the -DH2J_SAMPLE process timer signals the main thread)
    if (threads == 1) worker();
    else
        for (int k = 0; k < threads; k++) pool.emplace_back(worker);
    for (auto& th : pool) th.join();
    if (failed) return 1;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const double nf = total;
    std::printf("%d thr: %.3f ms/frame wall, %.3f ms/frame/thread  %.0f TUs/frame  %.0f coefs/frame  %.1f MB/s  digest %016llx\n",
                threads, ms / nf, ms * threads / nf, tus / nf, coefs / nf, bytes / (ms / 1e3) / 1e6,
                static_cast<unsigned long long>(digest));
    if (want_hist)
        for (int c = 0; c < 2; c++)
            for (int l = 0; l < 4; l++)
                std::printf("%s %2dx%-2d: %8.0f TBs/frame, %8.0f with residual\n", c ? "chroma" : "luma  ", 4 << l, 4 << l,
                            (hist[c][l][0] + hist[c][l][1]) / nf, hist[c][l][1] / nf);
    if (bins_ctx + bins_byp)
        std::printf("bins/frame: %.0f context-coded, %.0f bypass; %.2f ns per bin\n", bins_ctx / nf, bins_byp / nf,
                    ms * 1e6 * threads / static_cast<double>(bins_ctx + bins_byp));
    return 0;
}
