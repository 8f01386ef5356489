// Two independent CABAC arithmetic-decoder chains, one after the other vs interleaved bin by bin
// on one thread (the ceiling of VERDICT r02 #1's two-picture interleave).  Decodes
// 400k context-coded bins from two real bitstreams' bytes with a significance-map-like context
// pattern; prints ns per bin, minimum of 15 runs.
//   g++ -O3 -march=x86-64-v3 -std=c++11 -I../../include -I../../h264-h265-to-jpeg_amd/csrc/host \
//       interleave_bench.cpp ../../h264-h265-to-jpeg_amd/csrc/host/cabac_tables.cpp -o interleave_bench
//   ./interleave_bench ../../tests/golden/bench/hevc1080_00.h265 ../../tests/golden/bench/hevc1080_04.h265
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "cabac.h"

using namespace h2j;

static std::vector<uint8_t> read_file(const char* p) {
    std::vector<uint8_t> d;
    FILE* f = std::fopen(p, "rb");
    if (!f) return d;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + n);
    std::fclose(f);
    return d;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: interleave_bench a.h265 b.h265\n");
        return 2;
    }
    const std::vector<uint8_t> a = read_file(argv[1]), b = read_file(argv[2]);
    if (a.size() < 4096 || b.size() < 4096) return 2;
    const int N = 400000;
    static const int pat[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2};
    double best_seq = 1e9, best_il = 1e9;
    for (int rep = 0; rep < 15; rep++) {
        CabacState ca[3], cb[3], da[3], db[3];
        for (int i = 0; i < 3; i++) ca[i] = cb[i] = da[i] = db[i] = cabac_init_word(-5, 60 + i * 10, 30);
        Cabac A, B, A2, B2;
        A.init(a.data() + 200, a.data() + a.size());
        B.init(b.data() + 200, b.data() + b.size());
        A2.init(a.data() + 200, a.data() + a.size());
        B2.init(b.data() + 200, b.data() + b.size());
        unsigned s1 = 0, s2 = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; i++) s1 += A.decision(ca[pat[i & 15]]);
        for (int i = 0; i < N; i++) s1 += B.decision(cb[pat[i & 15]]);
        const auto t1 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; i++) {
            s2 += A2.decision(da[pat[i & 15]]);
            s2 += B2.decision(db[pat[i & 15]]);
        }
        const auto t2 = std::chrono::steady_clock::now();
        if (s1 != s2) std::printf("mismatch\n");
        const double seq = std::chrono::duration<double, std::nano>(t1 - t0).count() / (2.0 * N);
        const double il = std::chrono::duration<double, std::nano>(t2 - t1).count() / (2.0 * N);
        if (seq < best_seq) best_seq = seq;
        if (il < best_il) best_il = il;
    }
    std::printf("one chain after the other %.3f ns/bin, two chains interleaved %.3f ns/bin (%.2fx)\n", best_seq, best_il,
                best_seq / best_il);
    return 0;
}
