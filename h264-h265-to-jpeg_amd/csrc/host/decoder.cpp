// IDecoder facade — drop-in for the reference's Decoder
// (/root/reference/src/Decoder.cpp:39-53 getInstance, :115-361 H265ToJpeg)
// and Encoder (/root/reference/src/Encoder.cpp:104-362).  Same contract:
// borrowed C-string paths, fresh instance per getInstance(), false + a LOG
// line on any failure, output written with fopen("wb+") + fwrite.
// Differences (documented in DESIGN.md): no probe-decode, no fixed 2 MiB
// output buffer (the reference's writeCallback has no bounds check,
// src/Encoder.cpp:29), decoder-delay streams are handled (the first picture
// is decoded directly), 10-bit input is converted with
// v8 = min(255, (v + 2) >> 2) instead of producing a corrupted JPEG.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <memory>
#include <mutex>
#include <vector>

#include "IDecoder.h"
#include "h2j.h"

void LOG(const char* format, ...) {
    char log[1024] = {0};
    va_list ap;
    va_start(ap, format);
    vsnprintf(log, sizeof(log), format, ap);
    va_end(ap);
    time_t ts;
    time(&ts);
    struct tm tmv;
    localtime_r(&ts, &tmv);  // the reference's localtime() is not thread-safe
    char now[64];
    strftime(now, sizeof(now), "%Y-%m-%d %H:%M:%S", &tmv);
    printf("%s | %s\n", now, log);
}

namespace {

// One engine per process (per GPU 0); IDecoder instances are cheap handles.
std::mutex g_engine_mu;
h2j_engine* g_engine = nullptr;

h2j_engine* shared_engine() {
    if (!g_engine) g_engine = h2j_engine_create(0, 0);
    return g_engine;
}

bool read_file(const char* path, std::vector<uint8_t>& buf) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return false; }
    long n = ftell(f);
    if (n < 0) { fclose(f); return false; }
    rewind(f);
    buf.resize(static_cast<size_t>(n));
    size_t got = n ? fread(buf.data(), 1, static_cast<size_t>(n), f) : 0;
    fclose(f);
    return got == static_cast<size_t>(n);
}

class Decoder : public IDecoder {
public:
    Decoder() { LOG("%s", __PRETTY_FUNCTION__); }
    ~Decoder() override = default;
    bool H265ToJpeg(const char* inputFilePath, const char* outputFilePath) override;
};

bool Decoder::H265ToJpeg(const char* const in, const char* const out) {
    if (in == nullptr || out == nullptr || strlen(in) == 0 || strlen(out) == 0) {
        LOG("input or output path is empty: input:%s, output:%s", in ? in : "(null)", out ? out : "(null)");
        return false;
    }
    std::vector<uint8_t> data;
    if (!read_file(in, data)) {
        LOG("cannot open input file: %s", in);
        return false;
    }
    std::vector<uint8_t> jpeg;
    {
        std::lock_guard<std::mutex> g(g_engine_mu);
        h2j_engine* e = shared_engine();
        if (!e) {
            LOG("no HIP device available: the MI355X pipeline cannot run");
            return false;
        }
        const uint8_t* d = data.data();
        size_t sz = data.size(), off = 0, len = 0;
        int status = 0;
        size_t cap = 1 << 20;
        for (int attempt = 0; attempt < 2; attempt++) {
            cap = std::max(cap, sz * 4 + (8u << 20));
            jpeg.resize(cap);
            int r = h2j_engine_transcode(e, 1, &d, &sz, jpeg.data(), cap, &off, &len, &status);
            if (r == 0 && status == 0) break;
            if (status == -50) { cap *= 4; continue; }
            LOG("transcode failed (%d/%d): %s", r, status, h2j_engine_error(e));
            return false;
        }
        if (status != 0) return false;
        jpeg.erase(jpeg.begin(), jpeg.begin() + static_cast<long>(off));
        jpeg.resize(len);
    }
    FILE* f = fopen(out, "wb+");
    if (!f) {
        LOG("failed to encode Yuv to Jpeg: cannot open %s", out);
        return false;
    }
    size_t w = fwrite(jpeg.data(), 1, jpeg.size(), f);
    fclose(f);
    if (w != jpeg.size()) {
        LOG("failed to write Jpeg file %s", out);
        return false;
    }
    LOG("saved Jpeg data to file %s", out);
    return true;
}

}  // namespace

std::shared_ptr<IDecoder> IDecoder::getInstance() { return std::make_shared<Decoder>(); }
