#include "jpeg_writer.h"

#include <cstring>

namespace h2j {

const char* const kLavcIdent = "Lavc58.117.101";

namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct PT {
    int value, prob;
};
struct HL {
    int code, length;
};

// libavutil/qsort.h AV_QSORT: median-of-three quicksort with an explicit
// stack.  Not stable, so equal-count symbols land in FFmpeg's exact order.
template <typename T, typename Cmp>
void av_qsort(T* p, int num, Cmp cmp) {
    T* stack[64][2];
    int sp = 1;
    if (num <= 0) return;
    stack[0][0] = p;
    stack[0][1] = p + num - 1;
    while (sp) {
        T* start = stack[--sp][0];
        T* end = stack[sp][1];
        while (start < end) {
            if (start < end - 1) {
                int checksort = 0;
                T* right = end - 2;
                T* left = start + 1;
                T* mid = start + ((end - start) >> 1);
                if (cmp(start, end) > 0) {
                    if (cmp(end, mid) > 0) std::swap(*start, *mid);
                    else std::swap(*start, *end);
                } else {
                    if (cmp(start, mid) > 0) std::swap(*start, *mid);
                    else checksort = 1;
                }
                if (cmp(mid, end) > 0) {
                    std::swap(*mid, *end);
                    checksort = 0;
                }
                if (start == end - 2) break;
                std::swap(end[-1], *mid);
                while (left <= right) {
                    while (left <= right && cmp(left, end - 1) < 0) left++;
                    while (left <= right && cmp(right, end - 1) > 0) right--;
                    if (left <= right) {
                        std::swap(*left, *right);
                        left++;
                        right--;
                    }
                }
                std::swap(end[-1], *left);
                if (checksort && (mid == left - 1 || mid == left)) {
                    mid = start;
                    while (mid < end && cmp(mid, mid + 1) <= 0) mid++;
                    if (mid == end) break;
                }
                if (end - left < left - start) {
                    stack[sp][0] = start;
                    stack[sp++][1] = right;
                    start = left + 1;
                } else {
                    stack[sp][0] = left + 1;
                    stack[sp++][1] = end;
                    end = right;
                }
            } else {
                if (cmp(start, end) > 0) std::swap(*start, *end);
                break;
            }
        }
    }
}

struct PMList {
    int nitems;
    int item_idx[515];
    int probability[514];
    int items[257 * 16];
};

// package-merge with max code length 16, FFmpeg mjpegenc_huffman.c semantics
void compute_bits(PT* prob, HL* distincts, int size, int max_length) {
    PMList la, lb;
    PMList* to = &la;
    PMList* from = &lb;
    int nbits[257] = {0};
    int i = 0;
    av_qsort(prob, size, [](const PT* a, const PT* b) { return a->prob - b->prob; });
    to->nitems = 1;
    to->item_idx[0] = 0;
    from->nitems = 0;
    for (int times = 0; times <= max_length; times++) {
        to->nitems = 0;
        to->item_idx[0] = 0;
        int j = 0;
        if (times < max_length) i = 0;
        while (i < size || j + 1 < from->nitems) {
            to->nitems++;
            to->item_idx[to->nitems] = to->item_idx[to->nitems - 1];
            if (i < size && (j + 1 >= from->nitems || prob[i].prob < from->probability[j] + from->probability[j + 1])) {
                to->items[to->item_idx[to->nitems]++] = prob[i].value;
                to->probability[to->nitems - 1] = prob[i].prob;
                i++;
            } else {
                for (int k = from->item_idx[j]; k < from->item_idx[j + 2]; k++)
                    to->items[to->item_idx[to->nitems]++] = from->items[k];
                to->probability[to->nitems - 1] = from->probability[j] + from->probability[j + 1];
                j += 2;
            }
        }
        std::swap(to, from);
    }
    const int mn = (size - 1 < from->nitems) ? size - 1 : from->nitems;
    for (i = 0; i < from->item_idx[mn]; i++) nbits[from->items[i]]++;
    int j = 0;
    for (i = 0; i < 256; i++)
        if (nbits[i] > 0) {
            distincts[j].code = i;
            distincts[j].length = nbits[i];
            j++;
        }
}

struct BitWriter {
    std::vector<uint8_t>& out;
    uint64_t acc = 0;
    int n = 0;
    explicit BitWriter(std::vector<uint8_t>& o) : out(o) {}
    inline void put(uint32_t v, int bits) {
        acc = (acc << bits) | (v & ((1u << bits) - 1u));
        n += bits;
        while (n >= 8) {
            const uint8_t b = static_cast<uint8_t>(acc >> (n - 8));
            n -= 8;
            out.push_back(b);
            if (b == 0xFF) out.push_back(0x00);
        }
    }
    void flush_ones() {
        if (n) put((1u << (8 - n)) - 1u, 8 - n);
    }
};

inline int nbits_of(int v) {
    unsigned a = static_cast<unsigned>(v < 0 ? -v : v);
    return a ? 32 - __builtin_clz(a) : 0;
}

void u16(std::vector<uint8_t>& o, int v) {
    o.push_back(static_cast<uint8_t>(v >> 8));
    o.push_back(static_cast<uint8_t>(v));
}

}  // namespace

int huffman_optimal(const uint32_t* counts, uint8_t bits[17], uint8_t* val) {
    PT pt[257];
    HL d[256];
    int nval = 0;
    for (int i = 0; i < 256; i++)
        if (counts[i]) {
            pt[nval].value = i;
            pt[nval].prob = static_cast<int>(counts[i]);
            nval++;
        }
    pt[nval].value = 256;
    pt[nval].prob = 0;
    compute_bits(pt, d, nval + 1, 16);
    av_qsort(d, nval, [](const HL* a, const HL* b) { return a->length - b->length; });
    std::memset(bits, 0, 17);
    for (int i = 0; i < nval; i++) {
        val[i] = static_cast<uint8_t>(d[i].code);
        bits[d[i].length]++;
    }
    return nval;
}

size_t jpeg_assemble(const int16_t* coefs, int w, int h, const h2j_jstat& st, const char* com,
                     std::vector<uint8_t>& out) {
    const size_t start = out.size();
    const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4, nmcu = mbw * mbh;
    uint8_t bits[4][17], val[4][256];
    uint16_t code[4][256];
    uint8_t len[4][256];
    for (int t = 0; t < 4; t++) {
        huffman_optimal(st.hist[t], bits[t], val[t]);
        int c = 0, k = 0;
        std::memset(len[t], 0, 256);
        for (int l = 1; l <= 16; l++) {
            for (int i = 0; i < bits[t][l]; i++, k++) {
                code[t][val[t][k]] = static_cast<uint16_t>(c++);
                len[t][val[t][k]] = static_cast<uint8_t>(l);
            }
            c <<= 1;
        }
    }
    out.reserve(out.size() + 4096 + static_cast<size_t>(w) * h / 4);
    u16(out, 0xFFD8);
    if (com) {
        const int n = static_cast<int>(std::strlen(com)) + 1;
        u16(out, 0xFFFE);
        u16(out, n + 2);
        out.insert(out.end(), com, com + n);
    }
    u16(out, 0xFFDB);
    u16(out, 67);
    out.push_back(0);
    for (int i = 0; i < 64; i++) out.push_back(st.dqt[kZigzag[i]]);
    int dhtlen = 2;
    for (int t = 0; t < 4; t++) {
        int n = 0;
        for (int l = 1; l <= 16; l++) n += bits[t][l];
        dhtlen += 17 + n;
    }
    u16(out, 0xFFC4);
    u16(out, dhtlen);
    static const int order[4][2] = {{0, 0x00}, {1, 0x01}, {2, 0x10}, {3, 0x11}};
    for (int o = 0; o < 4; o++) {
        const int t = order[o][0];
        int n = 0;
        out.push_back(static_cast<uint8_t>(order[o][1]));
        for (int l = 1; l <= 16; l++) {
            out.push_back(bits[t][l]);
            n += bits[t][l];
        }
        out.insert(out.end(), val[t], val[t] + n);
    }
    u16(out, 0xFFC0);
    u16(out, 17);
    out.push_back(8);
    u16(out, h);
    u16(out, w);
    const uint8_t sof[10] = {3, 1, 0x22, 0, 2, 0x11, 0, 3, 0x11, 0};
    out.insert(out.end(), sof, sof + 10);
    u16(out, 0xFFDA);
    u16(out, 12);
    const uint8_t sos[10] = {3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0};
    out.insert(out.end(), sos, sos + 10);
    BitWriter bw(out);
    int last_dc[3] = {128, 128, 128};
    for (int m = 0; m < nmcu; m++)
        for (int b = 0; b < 6; b++) {
            const int16_t* z = coefs + (static_cast<size_t>(m) * 6 + b) * 64;
            const int comp = b < 4 ? 0 : b - 3, tab = b < 4 ? 0 : 1;
            const int diff = z[0] - last_dc[comp];
            last_dc[comp] = z[0];
            const int nb = nbits_of(diff);
            bw.put(code[tab][nb], len[tab][nb]);
            if (nb) bw.put(static_cast<uint32_t>(diff < 0 ? diff - 1 : diff), nb);
            int last = 63;
            while (last > 0 && !z[last]) last--;
            int run = 0;
            const uint16_t* ac = code[2 + tab];
            const uint8_t* al = len[2 + tab];
            for (int i = 1; i <= last; i++) {
                const int v = z[i];
                if (!v) {
                    run++;
                    continue;
                }
                while (run >= 16) {
                    bw.put(ac[0xF0], al[0xF0]);
                    run -= 16;
                }
                const int n = nbits_of(v);
                const int sym = (run << 4) | n;
                bw.put(ac[sym], al[sym]);
                bw.put(static_cast<uint32_t>(v < 0 ? v - 1 : v), n);
                run = 0;
            }
            if (last < 63) bw.put(ac[0], al[0]);
        }
    bw.flush_ones();
    u16(out, 0xFFD9);
    return out.size() - start;
}

}  // namespace h2j
