#include "bitstream.h"

namespace h2j {

void split_annexb(const uint8_t* d, size_t n, std::vector<Nal>& out) {
    out.clear();
    size_t i = 0;
    long start = -1;
    while (i + 2 < n) {
        // fast skip: a start code needs d[i+2] <= 1
        if (d[i + 2] > 1) {
            i += 3;
            continue;
        }
        if (d[i] == 0 && d[i + 1] == 0 && d[i + 2] == 1) {
            if (start >= 0) {
                size_t e = i;
                while (e > static_cast<size_t>(start) && d[e - 1] == 0) e--;
                out.push_back(Nal{d + start, e - start});
            }
            i += 3;
            start = static_cast<long>(i);
            continue;
        }
        i++;
    }
    if (start >= 0 && static_cast<size_t>(start) < n) {
        size_t e = n;
        while (e > static_cast<size_t>(start) && d[e - 1] == 0) e--;
        out.push_back(Nal{d + start, e - start});
    }
}

size_t unescape_rbsp(const uint8_t* src, size_t n, uint8_t* dst) {
    size_t o = 0;
    int zeros = 0;
    for (size_t i = 0; i < n; i++) {
        uint8_t b = src[i];
        if (zeros >= 2 && b == 3) {
            zeros = 0;
            continue;
        }
        dst[o++] = b;
        zeros = (b == 0) ? zeros + 1 : 0;
    }
    return o;
}

bool BitReader::more_rbsp_data() const {
    long last = static_cast<long>(n_) - 1;
    while (last >= 0 && p_[last] == 0) last--;
    if (last < 0) return false;
    int tz = 0;
    while (!((p_[last] >> tz) & 1)) tz++;
    size_t stop = static_cast<size_t>(last) * 8 + (7 - tz);
    return pos_ < stop;
}

int detect_codec(const uint8_t* d, size_t n) {
    std::vector<Nal> nals;
    split_annexb(d, n < (1u << 16) ? n : (1u << 16), nals);
    int hv = 0, hs = 0, hp = 0, as = 0, ap = 0;
    for (const Nal& nal : nals) {
        if (nal.n < 2) continue;
        uint8_t h0 = nal.p[0], h1 = nal.p[1];
        if (h0 & 0x80) continue;
        int t = (h0 >> 1) & 63, layer = ((h0 & 1) << 5) | (h1 >> 3), tid = h1 & 7;
        if (layer == 0 && tid >= 1) {
            if (t == 32) hv++;
            if (t == 33) hs++;
            if (t == 34) hp++;
        }
        int t4 = h0 & 31;
        if (t4 == 7) as++;
        if (t4 == 8) ap++;
    }
    if (hv && hs && hp) return 265;
    if (as && ap) return 264;
    return 0;
}

}  // namespace h2j
