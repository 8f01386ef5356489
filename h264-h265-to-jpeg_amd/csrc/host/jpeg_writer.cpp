#include "jpeg_writer.h"

#include <cstring>

namespace h2j {

const char* const kLavcIdent = "Lavc58.117.101";

namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// DHT order of FFmpeg: DC luma (0x00), DC chroma (0x01), AC luma (0x10), AC chroma (0x11)
const int kDhtOrder[4][2] = {{0, 0x00}, {1, 0x01}, {2, 0x10}, {3, 0x11}};

size_t header_size(const h2j_jstat& st, const char* com) {
    size_t n = 2;                                              // SOI
    if (com) n += 4 + std::strlen(com) + 1;                    // COM
    n += 4 + 65;                                               // DQT
    n += 4;                                                    // DHT marker + length
    for (int t = 0; t < 4; t++) n += 17 + st.nval[t];
    n += 2 + 17;                                               // SOF0
    n += 2 + 12;                                               // SOS
    return n;
}

size_t count_ff(const uint8_t* p, size_t n) {
    size_t c = 0;
    const uint8_t* end = p + n;
    while (p < end) {
        const void* q = std::memchr(p, 0xFF, static_cast<size_t>(end - p));
        if (!q) break;
        c++;
        p = static_cast<const uint8_t*>(q) + 1;
    }
    return c;
}

inline uint8_t* u16(uint8_t* o, int v) {
    o[0] = static_cast<uint8_t>(v >> 8);
    o[1] = static_cast<uint8_t>(v);
    return o + 2;
}

}  // namespace

size_t jpeg_container_size(const h2j_jstat& st, const uint8_t* payload, const char* com) {
    return header_size(st, com) + st.nbytes + count_ff(payload, st.nbytes) + 2;
}

size_t jpeg_write_container(const h2j_jstat& st, const uint8_t* payload, int w, int h, const char* com,
                            uint8_t* out) {
    uint8_t* o = out;
    o = u16(o, 0xFFD8);
    if (com) {
        const int n = static_cast<int>(std::strlen(com)) + 1;
        o = u16(o, 0xFFFE);
        o = u16(o, n + 2);
        std::memcpy(o, com, n);
        o += n;
    }
    o = u16(o, 0xFFDB);
    o = u16(o, 67);
    *o++ = 0;
    for (int i = 0; i < 64; i++) *o++ = st.dqt[kZigzag[i]];
    int dhtlen = 2;
    for (int t = 0; t < 4; t++) dhtlen += 17 + static_cast<int>(st.nval[t]);
    o = u16(o, 0xFFC4);
    o = u16(o, dhtlen);
    for (int k = 0; k < 4; k++) {
        const int t = kDhtOrder[k][0];
        *o++ = static_cast<uint8_t>(kDhtOrder[k][1]);
        for (int l = 1; l <= 16; l++) *o++ = st.bits[t][l];
        std::memcpy(o, st.val[t], st.nval[t]);
        o += st.nval[t];
    }
    o = u16(o, 0xFFC0);
    o = u16(o, 17);
    *o++ = 8;
    o = u16(o, h);
    o = u16(o, w);
    static const uint8_t sof[10] = {3, 1, 0x22, 0, 2, 0x11, 0, 3, 0x11, 0};
    std::memcpy(o, sof, 10);
    o += 10;
    o = u16(o, 0xFFDA);
    o = u16(o, 12);
    static const uint8_t sos[10] = {3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0};
    std::memcpy(o, sos, 10);
    o += 10;
    // payload with byte stuffing: copy runs between 0xFF bytes
    const uint8_t* p = payload;
    const uint8_t* end = payload + st.nbytes;
    while (p < end) {
        const uint8_t* q = static_cast<const uint8_t*>(std::memchr(p, 0xFF, static_cast<size_t>(end - p)));
        const size_t run = (q ? q + 1 : end) - p;
        std::memcpy(o, p, run);
        o += run;
        p += run;
        if (q) *o++ = 0x00;
    }
    o = u16(o, 0xFFD9);
    return static_cast<size_t>(o - out);
}

}  // namespace h2j
