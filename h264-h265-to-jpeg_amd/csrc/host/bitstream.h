// Annex-B NAL unit splitting, emulation-prevention removal and an RBSP bit
// reader for the host entropy stage.
//
// Replaces the raw h264/hevc demuxer + parser the reference gets from FFmpeg
// through avformat_open_input / av_read_frame (/root/reference/src/Decoder.cpp:137,298):
// the whole file is scanned once, NAL units of the first access unit are
// handed to the syntax parsers.  No probe-decode (the reference's
// avformat_find_stream_info at :153 decodes the frame a second time).
#pragma once
#include <cstddef>
#include <algorithm>
#include <cstdint>
#include <vector>

namespace h2j {

struct Nal {
    const uint8_t* p;  // NAL header onward, still escaped
    size_t n;
};

// Split an Annex-B byte stream; trailing zero bytes of each NAL are dropped.
void split_annexb(const uint8_t* d, size_t n, std::vector<Nal>& out);

// Remove emulation_prevention_three_byte; returns RBSP length written to dst.
size_t unescape_rbsp(const uint8_t* src, size_t n, uint8_t* dst);

class BitReader {
public:
    BitReader() : p_(nullptr), n_(0), pos_(0) {}
    BitReader(const uint8_t* p, size_t n) : p_(p), n_(n), pos_(0) {}
    uint32_t u(int bits) {
        uint32_t v = 0;
        for (int i = 0; i < bits; i++) v = (v << 1) | bit();
        return v;
    }
    uint32_t bit() {
        size_t byte = pos_ >> 3;
        uint32_t v = byte < n_ ? (p_[byte] >> (7 - (pos_ & 7))) & 1u : 0u;
        pos_++;
        return v;
    }
    uint32_t ue() {
        int lz = 0;
        while (!bit()) {
            if (++lz > 31) { overrun_ = true; return 0; }
        }
        return ((1u << lz) - 1u) + u(lz);
    }
    int32_t se() {
        uint32_t k = ue();
        return (k & 1) ? static_cast<int32_t>((k + 1) >> 1) : -static_cast<int32_t>(k >> 1);
    }
    void align() { pos_ = (pos_ + 7) & ~static_cast<size_t>(7); }
    size_t byte_pos() const { return pos_ >> 3; }
    size_t bit_pos() const { return pos_; }
    bool overrun() const { return overrun_ || (pos_ >> 3) > n_; }
    const uint8_t* data() const { return p_; }
    size_t size() const { return n_; }
    bool more_rbsp_data() const;

private:
    const uint8_t* p_;
    size_t n_;
    size_t pos_;
    bool overrun_ = false;
};

inline int ceil_log2(int v) {
    int r = 0;
    while ((1 << r) < v) r++;
    return r;
}

// The left crop of a decoded picture as FFmpeg 4.3 applies it: decode.c apply_cropping calls
// av_frame_apply_cropping (libavutil/frame.c) without AV_FRAME_CROP_UNALIGNED, which lowers
// crop_left until every cropped plane's data pointer keeps the alignment of FFmpeg's frame pool
// (linesizes are multiples of STRIDE_ALIGN >= 32, so the left part of each plane offset decides):
// crop_left &= ~((1 << (5 + log2(crop_left alignment) - min plane log2 alignment)) - 1) when a
// plane offset is less than 32-byte aligned, AVERROR_BUG when the crop's alignment is below a
// plane's.  yuv420p / yuv420pN (chroma at crop_left >> 1), bps bytes per sample.
// Returns the effective left crop, -1 for AVERROR_BUG (avcodec_receive_frame fails).
inline int ff_crop_left(int cl, int bps) {
    if (cl <= 0) return cl;
    const int lca = __builtin_ctz(static_cast<unsigned>(cl));
    int m = 1000;
    const long part[2] = {static_cast<long>(cl) * bps, static_cast<long>(cl >> 1) * bps};
    for (long v : part)
        if (v && __builtin_ctzl(static_cast<unsigned long>(v)) < 5) m = std::min(m, __builtin_ctzl(static_cast<unsigned long>(v)));
    if (m == 1000) return cl;
    if (lca < m) return -1;
    return cl & ~((1 << (5 + lca - m)) - 1);
}

// 0 unknown, 264, 265 — content probe in the spirit of FFmpeg's raw
// h264/hevc probes (parameter-set NAL units with valid headers).
int detect_codec(const uint8_t* d, size_t n);

}  // namespace h2j
