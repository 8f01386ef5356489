// Host-only timing of the entropy decoders (no GPU): parses every stream of
// a directory N times on one thread and prints ms/frame and TUs/frame.
//   g++ -O2 -std=c++11 -I../../include -I../../h264-h265-to-jpeg_amd/csrc/host parse_bench.cpp \
//       ../../h264-h265-to-jpeg_amd/csrc/host/{bitstream,cabac_tables,hevc_parser,h264_parser}.cpp
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "bitstream.h"
#include "job.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: parse_bench file... [-r reps]\n");
        return 2;
    }
    int reps = 3;
    std::vector<std::vector<uint8_t>> streams;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "-r" && i + 1 < argc) {
            reps = std::atoi(argv[++i]);
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
    h2j::FrameJob job;
    size_t tus = 0, coefs = 0, bytes = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++)
        for (auto& s : streams) {
            const int codec = h2j::detect_codec(s.data(), s.size());
            const int rc = codec == 265 ? h2j::hevc_parse_picture(s.data(), s.size(), job)
                                        : h2j::h264_parse_picture(s.data(), s.size(), job);
            if (rc) {
                std::fprintf(stderr, "parse error %d: %s\n", rc, job.message.c_str());
                return 1;
            }
            tus += job.tus.size();
            coefs += job.coefs.size();
            bytes += s.size();
        }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const double nf = static_cast<double>(reps) * streams.size();
    std::printf("%.3f ms/frame  %.0f TUs/frame  %.0f coefs/frame  %.1f MB/s\n", ms / nf, tus / nf, coefs / nf,
                bytes / (ms / 1e3) / 1e6);
    return 0;
}
