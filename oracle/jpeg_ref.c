/*
 * ORACLE — test infrastructure only. Never linked into the product.
 *
 * CPU restatement of the reference's YUV420p8 -> baseline JPEG step:
 *   Encoder::yuv2Jpeg (/root/reference/src/Encoder.cpp:104-308), which drives
 *   FFmpeg's mjpeg encoder (libavcodec 58.117.101, binary-only in
 *   /root/reference/lib/ffmpeg/x86_64_shared) through avcodec_send_frame
 *   (src/Encoder.cpp:250) / avcodec_receive_packet (:259) with the defaults
 *   listed in SURVEY.md §5 (bit_rate 200000, qmin 2, qmax 31, i_quant_factor
 *   -0.8, dct AUTO -> ff_fdct_sse2) and time_base 1/25 (:201), pix fmt
 *   YUVJ420P (:162).
 *
 * The arithmetic follows SURVEY.md Appendix A (A.1 pad, A.2 rate control,
 * A.3 DQT, A.4 AP-922 FDCT, A.5 16-bit quantiser, A.6 optimal Huffman + file
 * layout).  Parity is pinned by the reference's own fixtures
 * test/img/img01.h26{4,5}.jpeg (tests/golden/): the Huffman/bitstream half
 * by re-emitting the fixtures' own coefficients byte-exactly, the
 * FDCT/quant/RC half by encoding the decoded fixture pictures.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---------------------------------------------------------------- tables */
static const uint8_t k_zigzag[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* MPEG-1 default intra matrix, natural order */
static const uint8_t k_mpeg1_intra[64] = {
    8,  16, 19, 22, 26, 27, 29, 34, 16, 16, 22, 24, 27, 29, 34, 37,
    19, 22, 26, 27, 29, 34, 34, 38, 22, 22, 26, 27, 29, 34, 37, 40,
    22, 26, 27, 29, 32, 35, 40, 48, 26, 27, 29, 32, 35, 40, 48, 58,
    26, 27, 29, 34, 38, 46, 56, 69, 27, 29, 35, 38, 46, 56, 69, 83};

const uint8_t *oracle_zigzag(void) { return k_zigzag; }

/* --------------------------------------------------------------- A.4 FDCT */
static inline int16_t sat16(int32_t v) {
    return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}
static inline int16_t mulhi(int16_t a, int16_t c) {
    return (int16_t)(((int32_t)a * (int32_t)c) >> 16);
}

#define TG1 13036
#define TG2 27146
#define TG3 (-21746)
#define COS4 23170

static const int16_t k_rowset[4][7] = {
    {22725, 21407, 19266, 16384, 12873, 8867, 4520},
    {31521, 29692, 26722, 22725, 17855, 12299, 6270},
    {29692, 27969, 25172, 21407, 16819, 11585, 5906},
    {26722, 25172, 22654, 19266, 15137, 10426, 5315}};
static const int k_rowsel[8] = {0, 1, 2, 3, 0, 3, 2, 1};

void oracle_fdct(int16_t *blk) {
    int16_t tmp[64];
    for (int x = 0; x < 8; x++) {
        const int16_t x0 = blk[0 * 8 + x], x1 = blk[1 * 8 + x], x2 = blk[2 * 8 + x],
                      x3 = blk[3 * 8 + x], x4 = blk[4 * 8 + x], x5 = blk[5 * 8 + x],
                      x6 = blk[6 * 8 + x], x7 = blk[7 * 8 + x];
        int16_t t0 = sat16(sat16(x0 + x7) * 8), t1 = sat16(sat16(x1 + x6) * 8);
        int16_t t2 = sat16(sat16(x2 + x5) * 8), t3 = sat16(sat16(x3 + x4) * 8);
        int16_t tp03 = sat16(t0 + t3), tm03 = sat16(t0 - t3);
        int16_t tp12 = sat16(t1 + t2), tm12 = sat16(t1 - t2);
        int16_t y0 = sat16(tp03 + tp12), y4 = sat16(tp03 - tp12);
        int16_t y2 = (int16_t)(sat16(tm03 + mulhi(tm12, TG2)) | 1);
        int16_t y6 = (int16_t)(sat16(mulhi(tm03, TG2) - tm12) | 1);
        int16_t d16 = sat16(sat16(x1 - x6) * 16), d25 = sat16(sat16(x2 - x5) * 16);
        int16_t tp65 = (int16_t)(mulhi(sat16(d16 + d25), COS4) | 1);
        int16_t tm65 = mulhi(sat16(d16 - d25), COS4);
        int16_t t4 = sat16(sat16(x3 - x4) * 8), t7 = sat16(sat16(x0 - x7) * 8);
        int16_t tp465 = sat16(t4 + tm65), tm465 = sat16(t4 - tm65);
        int16_t tp765 = sat16(t7 + tp65), tm765 = sat16(t7 - tp65);
        int16_t y1 = (int16_t)(sat16(tp765 + mulhi(tp465, TG1)) | 1);
        int16_t y7 = sat16(mulhi(tp765, TG1) - tp465);
        int16_t y3 = sat16(tm765 - sat16(mulhi(tm465, TG3) + tm465));
        int16_t y5 = sat16(sat16(mulhi(tm765, TG3) + tm765) + tm465);
        tmp[0 * 8 + x] = y0; tmp[1 * 8 + x] = y1; tmp[2 * 8 + x] = y2; tmp[3 * 8 + x] = y3;
        tmp[4 * 8 + x] = y4; tmp[5 * 8 + x] = y5; tmp[6 * 8 + x] = y6; tmp[7 * 8 + x] = y7;
    }
    for (int r = 0; r < 8; r++) {
        const int16_t *c = k_rowset[k_rowsel[r]];
        const int32_t C1 = c[0], C2 = c[1], C3 = c[2], C4 = c[3], C5 = c[4], C6 = c[5], C7 = c[6];
        const int16_t *x = tmp + r * 8;
        int32_t s0 = sat16(x[0] + x[7]), s1 = sat16(x[1] + x[6]);
        int32_t s2 = sat16(x[2] + x[5]), s3 = sat16(x[3] + x[4]);
        int32_t d0 = sat16(x[0] - x[7]), d1 = sat16(x[1] - x[6]);
        int32_t d2 = sat16(x[2] - x[5]), d3 = sat16(x[3] - x[4]);
        int32_t Y[8];
        Y[0] = C4 * s0 + C4 * s1 + C4 * s2 + C4 * s3;
        Y[4] = C4 * s0 - C4 * s1 - C4 * s2 + C4 * s3;
        Y[2] = C2 * s0 + C6 * s1 - C6 * s2 - C2 * s3;
        Y[6] = C6 * s0 - C2 * s1 + C2 * s2 - C6 * s3;
        Y[1] = C1 * d0 + C3 * d1 + C5 * d2 + C7 * d3;
        Y[3] = C3 * d0 - C7 * d1 - C1 * d2 - C5 * d3;
        Y[5] = C5 * d0 - C1 * d1 + C7 * d2 + C3 * d3;
        Y[7] = C7 * d0 - C5 * d1 + C3 * d2 - C1 * d3;
        for (int k = 0; k < 8; k++) blk[r * 8 + k] = sat16((Y[k] + 65536) >> 17);
    }
}

/* ------------------------------------------------------- A.2 rate control */
static int64_t mb_variance_sum(const uint8_t *y, int w, int h, int stride) {
    /* padded picture: replicate last column / row (A.1) */
    const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
    int64_t V = 0;
    for (int my = 0; my < mbh; my++)
        for (int mx = 0; mx < mbw; mx++) {
            uint32_t s = 0, n = 0;
            for (int j = 0; j < 16; j++) {
                int yy = my * 16 + j;
                if (yy >= h) yy = h - 1;
                for (int i = 0; i < 16; i++) {
                    int xx = mx * 16 + i;
                    if (xx >= w) xx = w - 1;
                    uint32_t p = y[(size_t)yy * stride + xx];
                    s += p;
                    n += p * p;
                }
            }
            int var = (int)((n - ((s * s) >> 8) + 500 + 128) >> 8);
            V += var;
        }
    return V;
}

int oracle_jpeg_qscale_from_var(int64_t V, int *lambda_out) {
    const double qp2l = 118.0, qs = 2.0 * 118.0;
    int T = (int)(qp2l * 7.0 * sqrt((double)V) / qs);
    double bits = sqrt((double)T * qs) + 1.0;
    double q = qs * (double)(T + 1) / (bits > 0.9 ? bits : 0.9);
    q = 0.8 * q;
    q = (0.0005 + q) / 1.0005;
    if (q < 189.0) q = 189.0;
    if (q > 2926.0) q = 2926.0;
    int lambda = (int)(q + 0.5);
    int qscale = (lambda * 139 + 128 * 64) >> 14;
    if (qscale < 2) qscale = 2;
    if (qscale > 31) qscale = 31;
    if (lambda_out) *lambda_out = lambda;
    return qscale;
}

int oracle_jpeg_qscale(const uint8_t *y, int w, int h, int stride, int64_t *V_out,
                       int *lambda_out) {
    int64_t V = mb_variance_sum(y, w, h, stride);
    if (V_out) *V_out = V;
    return oracle_jpeg_qscale_from_var(V, lambda_out);
}

/* ------------------------------------------------ A.3 / A.5 quant tables */
void oracle_jpeg_matrix(int qscale, uint8_t M[64], uint16_t q16[64], uint16_t b16[64]) {
    M[0] = 8;
    for (int i = 1; i < 64; i++) {
        int v = (k_mpeg1_intra[i] * qscale) >> 3;
        M[i] = (uint8_t)(v > 255 ? 255 : v);
    }
    for (int i = 0; i < 64; i++) {
        int den = 16 * M[i];
        int q = (2 << 16) / den;
        if (q == 0 || q == 128 * 256) q = 128 * 256 - 1;
        q16[i] = (uint16_t)q;
        int a = 96 * 256;
        b16[i] = (uint16_t)((a + (q >> 1)) / q);
    }
}

/* quantise one FDCT'd block (natural order) into zigzag order */
static void quant_block(const int16_t *X, const uint16_t *q16, const uint16_t *b16,
                        int16_t *outzz) {
    int16_t nat[64];
    nat[0] = (int16_t)(((X[0] >> 2) + 8) / 16);
    for (int i = 1; i < 64; i++) {
        int a = X[i] < 0 ? -X[i] : X[i];
        uint32_t t = (uint32_t)a + b16[i];
        if (t > 65535) t = 65535;
        int L = (int)((t * q16[i]) >> 16);
        if (L > 1023) L = 1023; /* clip_coeffs: max_qcoeff 1023 (never hit at 8 bit) */
        nat[i] = (int16_t)(X[i] < 0 ? -L : L);
    }
    for (int k = 0; k < 64; k++) outzz[k] = nat[k_zigzag[k]];
}

/* Produce quantised zigzag coefficients for the whole picture.
 * Layout: coefs[mcu][6][64], MCU raster, blocks Y00 Y01 Y10 Y11 Cb Cr. */
int oracle_jpeg_coeffs(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h,
                       int ystride, int cstride, int16_t *coefs, int *qscale_out) {
    int qscale = oracle_jpeg_qscale(y, w, h, ystride, NULL, NULL);
    uint8_t M[64];
    uint16_t q16[64], b16[64];
    oracle_jpeg_matrix(qscale, M, q16, b16);
    const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
    const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    int16_t blk[64];
    for (int my = 0; my < mbh; my++)
        for (int mx = 0; mx < mbw; mx++) {
            int16_t *mcu = coefs + ((size_t)my * mbw + mx) * 6 * 64;
            for (int b = 0; b < 6; b++) {
                const uint8_t *pl;
                int pw, ph, st, x0, y0;
                if (b < 4) {
                    pl = y; pw = w; ph = h; st = ystride;
                    x0 = mx * 16 + (b & 1) * 8; y0 = my * 16 + (b >> 1) * 8;
                } else {
                    pl = b == 4 ? u : v; pw = cw; ph = ch; st = cstride;
                    x0 = mx * 8; y0 = my * 8;
                }
                for (int j = 0; j < 8; j++) {
                    int yy = y0 + j;
                    if (yy >= ph) yy = ph - 1;
                    for (int i = 0; i < 8; i++) {
                        int xx = x0 + i;
                        if (xx >= pw) xx = pw - 1;
                        blk[j * 8 + i] = pl[(size_t)yy * st + xx];
                    }
                }
                oracle_fdct(blk);
                quant_block(blk, q16, b16, mcu + b * 64);
            }
        }
    if (qscale_out) *qscale_out = qscale;
    return mbw * mbh;
}

/* ------------------------------------------------------ A.6 Huffman build */
typedef struct { int value, prob; } PTable;
typedef struct { int code, length; } HuffLen;
typedef struct {
    int nitems;
    int item_idx[515];
    int probability[514];
    int items[257 * 16];
} PMList;

static int cmp_prob(const PTable *a, const PTable *b) { return a->prob - b->prob; }
static int cmp_len(const HuffLen *a, const HuffLen *b) { return a->length - b->length; }

/* FFmpeg libavutil/qsort.h AV_QSORT, restated as a macro-instantiated
 * function (the exact pivot / partition order matters: it is not stable). */
#define DEFINE_QSORT(NAME, type, cmp)                                               \
    static void NAME(type *p, int num) {                                            \
        type *stack[64][2];                                                         \
        int sp = 1;                                                                 \
        type tmpv;                                                                  \
        if (num <= 0) return;                                                       \
        stack[0][0] = p;                                                            \
        stack[0][1] = p + num - 1;                                                  \
        while (sp) {                                                                \
            type *start = stack[--sp][0];                                           \
            type *end = stack[sp][1];                                               \
            while (start < end) {                                                   \
                if (start < end - 1) {                                              \
                    int checksort = 0;                                              \
                    type *right = end - 2;                                          \
                    type *left = start + 1;                                         \
                    type *mid = start + ((end - start) >> 1);                       \
                    if (cmp(start, end) > 0) {                                      \
                        if (cmp(end, mid) > 0) { tmpv = *start; *start = *mid; *mid = tmpv; } \
                        else { tmpv = *start; *start = *end; *end = tmpv; }         \
                    } else {                                                        \
                        if (cmp(start, mid) > 0) { tmpv = *start; *start = *mid; *mid = tmpv; } \
                        else checksort = 1;                                         \
                    }                                                               \
                    if (cmp(mid, end) > 0) {                                        \
                        tmpv = *mid; *mid = *end; *end = tmpv;                      \
                        checksort = 0;                                              \
                    }                                                               \
                    if (start == end - 2) break;                                    \
                    tmpv = end[-1]; end[-1] = *mid; *mid = tmpv;                    \
                    while (left <= right) {                                         \
                        while (left <= right && cmp(left, end - 1) < 0) left++;     \
                        while (left <= right && cmp(right, end - 1) > 0) right--;   \
                        if (left <= right) {                                        \
                            tmpv = *left; *left = *right; *right = tmpv;            \
                            left++;                                                 \
                            right--;                                                \
                        }                                                           \
                    }                                                               \
                    tmpv = end[-1]; end[-1] = *left; *left = tmpv;                  \
                    if (checksort && (mid == left - 1 || mid == left)) {            \
                        mid = start;                                                \
                        while (mid < end && cmp(mid, mid + 1) <= 0) mid++;          \
                        if (mid == end) break;                                      \
                    }                                                               \
                    if (end - left < left - start) {                                \
                        stack[sp][0] = start;                                       \
                        stack[sp++][1] = right;                                     \
                        start = left + 1;                                           \
                    } else {                                                        \
                        stack[sp][0] = left + 1;                                    \
                        stack[sp++][1] = end;                                       \
                        end = right;                                                \
                    }                                                               \
                } else {                                                            \
                    if (cmp(start, end) > 0) { tmpv = *start; *start = *end; *end = tmpv; } \
                    break;                                                          \
                }                                                                   \
            }                                                                       \
        }                                                                           \
    }

DEFINE_QSORT(qsort_ptable, PTable, cmp_prob)
DEFINE_QSORT(qsort_hufflen, HuffLen, cmp_len)

/* package-merge, max length 16 (FFmpeg mjpegenc_huffman.c) */
static void compute_bits(PTable *prob, HuffLen *distincts, int size, int max_length) {
    static __thread PMList la, lb; /* per thread: the CPU baseline runs several transcodes at once */
    PMList *to = &la, *from = &lb, *t;
    int nbits[257] = {0};
    int i = 0, j, k;
    qsort_ptable(prob, size);
    to->nitems = 1;
    to->item_idx[0] = 0;
    from->nitems = 0;
    for (int times = 0; times <= max_length; times++) {
        to->nitems = 0;
        to->item_idx[0] = 0;
        j = 0;
        k = 0;
        if (times < max_length) i = 0;
        while (i < size || j + 1 < from->nitems) {
            to->nitems++;
            to->item_idx[to->nitems] = to->item_idx[to->nitems - 1];
            if (i < size && (j + 1 >= from->nitems ||
                             prob[i].prob < from->probability[j] + from->probability[j + 1])) {
                to->items[to->item_idx[to->nitems]++] = prob[i].value;
                to->probability[to->nitems - 1] = prob[i].prob;
                i++;
            } else {
                for (k = from->item_idx[j]; k < from->item_idx[j + 2]; k++)
                    to->items[to->item_idx[to->nitems]++] = from->items[k];
                to->probability[to->nitems - 1] = from->probability[j] + from->probability[j + 1];
                j += 2;
            }
        }
        t = to; to = from; from = t;
    }
    int mn = (size - 1 < from->nitems) ? size - 1 : from->nitems;
    for (i = 0; i < from->item_idx[mn]; i++) nbits[from->items[i]]++;
    j = 0;
    for (i = 0; i < 256; i++)
        if (nbits[i] > 0) {
            distincts[j].code = i;
            distincts[j].length = nbits[i];
            j++;
        }
}

/* counts[256] -> bits[17], val[] (returns nval) */
int oracle_huff_build(const uint32_t *counts, uint8_t bits[17], uint8_t *val) {
    PTable pt[257];
    HuffLen d[256];
    int nval = 0;
    for (int i = 0; i < 256; i++)
        if (counts[i]) {
            pt[nval].value = i;
            pt[nval].prob = (int)counts[i];
            nval++;
        }
    pt[nval].value = 256;
    pt[nval].prob = 0;
    compute_bits(pt, d, nval + 1, 16);
    qsort_hufflen(d, nval);
    memset(bits, 0, 17);
    for (int i = 0; i < nval; i++) {
        val[i] = (uint8_t)d[i].code;
        bits[d[i].length]++;
    }
    return nval;
}

/* --------------------------------------------------------- bit writer */
typedef struct {
    uint8_t *buf;
    long cap, pos;
    uint64_t acc;
    int nacc;
    int err;
} BW;

static void bw_byte(BW *b, uint8_t v) {
    if (b->pos < b->cap) b->buf[b->pos] = v;
    else b->err = 1;
    b->pos++;
}
/* entropy-coded bits with 0xFF00 stuffing */
static void bw_bits(BW *b, uint32_t v, int n) {
    if (n == 0) return;
    b->acc = (b->acc << n) | (v & ((1u << n) - 1));
    b->nacc += n;
    while (b->nacc >= 8) {
        uint8_t byte = (uint8_t)(b->acc >> (b->nacc - 8));
        b->nacc -= 8;
        bw_byte(b, byte);
        if (byte == 0xFF) bw_byte(b, 0x00);
    }
}
static void bw_flush_ones(BW *b) {
    if (b->nacc) bw_bits(b, (1u << (8 - b->nacc)) - 1, 8 - b->nacc);
}
static void bw_u16(BW *b, int v) { bw_byte(b, (uint8_t)(v >> 8)); bw_byte(b, (uint8_t)v); }

static int nbits_of(int v) {
    int a = v < 0 ? -v : v, n = 0;
    while (a) { n++; a >>= 1; }
    return n;
}

typedef struct {
    uint16_t code[256];
    uint8_t len[256];
} HCode;

static void canon_codes(const uint8_t bits[17], const uint8_t *val, HCode *hc) {
    int code = 0, k = 0;
    memset(hc, 0, sizeof(*hc));
    for (int l = 1; l <= 16; l++) {
        for (int i = 0; i < bits[l]; i++, k++) {
            hc->code[val[k]] = (uint16_t)code++;
            hc->len[val[k]] = (uint8_t)l;
        }
        code <<= 1;
    }
}

/* symbol statistics over the coefficient array, tables: 0 DC-luma,
 * 1 DC-chroma, 2 AC-luma, 3 AC-chroma */
void oracle_jpeg_count(const int16_t *coefs, int nmcu, uint32_t counts[4][256]) {
    memset(counts, 0, 4 * 256 * sizeof(uint32_t));
    int last_dc[3] = {128, 128, 128};
    for (int m = 0; m < nmcu; m++)
        for (int b = 0; b < 6; b++) {
            const int16_t *z = coefs + ((size_t)m * 6 + b) * 64;
            int comp = b < 4 ? 0 : b - 3, tab = b < 4 ? 0 : 1;
            int diff = z[0] - last_dc[comp];
            last_dc[comp] = z[0];
            counts[tab][nbits_of(diff)]++;
            int last = 0;
            for (int i = 63; i >= 1; i--)
                if (z[i]) { last = i; break; }
            int run = 0;
            for (int i = 1; i <= last; i++) {
                if (!z[i]) { run++; continue; }
                while (run >= 16) { counts[2 + tab][0xF0]++; run -= 16; }
                counts[2 + tab][(run << 4) | nbits_of(z[i])]++;
                run = 0;
            }
            if (last < 63) counts[2 + tab][0]++;
        }
}

static void put_sym(BW *b, const HCode *h, int sym) { bw_bits(b, h->code[sym], h->len[sym]); }

long oracle_jpeg_from_coeffs(const int16_t *coefs, int w, int h, int qscale, const char *com,
                             uint8_t *out, long cap) {
    const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4, nmcu = mbw * mbh;
    uint32_t counts[4][256];
    uint8_t bits[4][17], val[4][256];
    HCode hc[4];
    uint8_t M[64];
    uint16_t q16[64], b16[64];
    oracle_jpeg_matrix(qscale, M, q16, b16);
    oracle_jpeg_count(coefs, nmcu, counts);
    for (int t = 0; t < 4; t++) {
        oracle_huff_build(counts[t], bits[t], val[t]);
        canon_codes(bits[t], val[t], &hc[t]);
    }
    BW b = {out, cap, 0, 0, 0, 0};
    bw_u16(&b, 0xFFD8);
    if (com) {
        int n = (int)strlen(com) + 1;
        bw_u16(&b, 0xFFFE);
        bw_u16(&b, n + 2);
        for (int i = 0; i < n; i++) bw_byte(&b, (uint8_t)com[i]);
    }
    bw_u16(&b, 0xFFDB);
    bw_u16(&b, 67);
    bw_byte(&b, 0);
    for (int i = 0; i < 64; i++) bw_byte(&b, M[k_zigzag[i]]);
    /* DHT: DC0, DC1, AC0, AC1 in one segment */
    int dhtlen = 2;
    for (int t = 0; t < 4; t++) {
        int n = 0;
        for (int l = 1; l <= 16; l++) n += bits[t][l];
        dhtlen += 17 + n;
    }
    bw_u16(&b, 0xFFC4);
    bw_u16(&b, dhtlen);
    static const int order[4][2] = {{0, 0x00}, {1, 0x01}, {2, 0x10}, {3, 0x11}};
    for (int o = 0; o < 4; o++) {
        int t = order[o][0], n = 0;
        bw_byte(&b, (uint8_t)order[o][1]);
        for (int l = 1; l <= 16; l++) { bw_byte(&b, bits[t][l]); n += bits[t][l]; }
        for (int i = 0; i < n; i++) bw_byte(&b, val[t][i]);
    }
    bw_u16(&b, 0xFFC0);
    bw_u16(&b, 17);
    bw_byte(&b, 8);
    bw_u16(&b, h);
    bw_u16(&b, w);
    bw_byte(&b, 3);
    bw_byte(&b, 1); bw_byte(&b, 0x22); bw_byte(&b, 0);
    bw_byte(&b, 2); bw_byte(&b, 0x11); bw_byte(&b, 0);
    bw_byte(&b, 3); bw_byte(&b, 0x11); bw_byte(&b, 0);
    bw_u16(&b, 0xFFDA);
    bw_u16(&b, 12);
    bw_byte(&b, 3);
    bw_byte(&b, 1); bw_byte(&b, 0x00);
    bw_byte(&b, 2); bw_byte(&b, 0x11);
    bw_byte(&b, 3); bw_byte(&b, 0x11);
    bw_byte(&b, 0); bw_byte(&b, 63); bw_byte(&b, 0);
    int last_dc[3] = {128, 128, 128};
    for (int m = 0; m < nmcu; m++)
        for (int blk = 0; blk < 6; blk++) {
            const int16_t *z = coefs + ((size_t)m * 6 + blk) * 64;
            int comp = blk < 4 ? 0 : blk - 3, tab = blk < 4 ? 0 : 1;
            int diff = z[0] - last_dc[comp];
            last_dc[comp] = z[0];
            int nb = nbits_of(diff);
            put_sym(&b, &hc[tab], nb);
            if (nb) bw_bits(&b, (uint32_t)(diff < 0 ? diff - 1 : diff), nb);
            int last = 0;
            for (int i = 63; i >= 1; i--)
                if (z[i]) { last = i; break; }
            int run = 0;
            for (int i = 1; i <= last; i++) {
                int v = z[i];
                if (!v) { run++; continue; }
                while (run >= 16) { put_sym(&b, &hc[2 + tab], 0xF0); run -= 16; }
                int n = nbits_of(v);
                put_sym(&b, &hc[2 + tab], (run << 4) | n);
                bw_bits(&b, (uint32_t)(v < 0 ? v - 1 : v), n);
                run = 0;
            }
            if (last < 63) put_sym(&b, &hc[2 + tab], 0);
        }
    bw_flush_ones(&b);
    bw_u16(&b, 0xFFD9);
    if (b.err) return -b.pos; /* needed size, negated */
    return b.pos;
}

long oracle_jpeg_encode(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h,
                        int ystride, int cstride, const char *com, uint8_t *out, long cap) {
    const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
    int16_t *coefs = (int16_t *)malloc((size_t)mbw * mbh * 6 * 64 * sizeof(int16_t));
    if (!coefs) return 0;
    int qscale = 0;
    oracle_jpeg_coeffs(y, u, v, w, h, ystride, cstride, coefs, &qscale);
    long n = oracle_jpeg_from_coeffs(coefs, w, h, qscale, com, out, cap);
    free(coefs);
    return n;
}

/* ---------------------------------------------- baseline JPEG parser (tests)
 * Decodes the entropy-coded data of a 3-component 4:2:0 baseline JPEG (the
 * fixtures' exact layout) into quantised zigzag coefficients (DC absolute,
 * predictor 128).  Returns number of MCUs, fills w/h and DQT. */
typedef struct {
    const uint8_t *p;
    long n, pos;
    uint32_t acc;
    int nacc;
} BR;

static int br_bit(BR *r) {
    if (r->nacc == 0) {
        if (r->pos >= r->n) return 0;
        uint8_t byte = r->p[r->pos++];
        if (byte == 0xFF) {
            if (r->pos < r->n && r->p[r->pos] == 0x00) r->pos++;
        }
        r->acc = byte;
        r->nacc = 8;
    }
    r->nacc--;
    return (r->acc >> r->nacc) & 1;
}
static int br_bits(BR *r, int n) {
    int v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | br_bit(r);
    return v;
}

typedef struct {
    int mincode[17], maxcode[18], valptr[17];
    uint8_t val[256];
} HDec;

static void hdec_build(HDec *h, const uint8_t *bits, const uint8_t *val) {
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        h->valptr[l] = k;
        h->mincode[l] = code;
        code += bits[l];
        k += bits[l];
        h->maxcode[l] = bits[l] ? code - 1 : -1;
        code <<= 1;
    }
    h->maxcode[17] = 0x7FFFFFFF;
    memcpy(h->val, val, (size_t)k);
}
static int hdec_sym(BR *r, const HDec *h) {
    int code = 0;
    for (int l = 1; l <= 16; l++) {
        code = (code << 1) | br_bit(r);
        if (code <= h->maxcode[l]) return h->val[h->valptr[l] + code - h->mincode[l]];
    }
    return -1;
}
static int extend(int v, int n) { return (n && v < (1 << (n - 1))) ? v - (1 << n) + 1 : v; }

int oracle_jpeg_parse(const uint8_t *jpg, long n, int *w_out, int *h_out, uint8_t dqt_zz[64],
                      int16_t *coefs, int max_mcu) {
    HDec hd[2][4];
    int w = 0, h = 0;
    long pos = 2;
    if (n < 4 || jpg[0] != 0xFF || jpg[1] != 0xD8) return -1;
    while (pos + 4 <= n) {
        if (jpg[pos] != 0xFF) return -2;
        int mk = jpg[pos + 1];
        int len = (jpg[pos + 2] << 8) | jpg[pos + 3];
        const uint8_t *seg = jpg + pos + 4;
        if (mk == 0xDB) {
            memcpy(dqt_zz, seg + 1, 64);
        } else if (mk == 0xC4) {
            const uint8_t *s = seg;
            while (s < seg + len - 2) {
                int tc = s[0] >> 4, th = s[0] & 15, cnt = 0;
                uint8_t bits[17] = {0};
                for (int l = 1; l <= 16; l++) { bits[l] = s[l]; cnt += s[l]; }
                hdec_build(&hd[tc][th], bits, s + 17);
                s += 17 + cnt;
            }
        } else if (mk == 0xC0) {
            h = (seg[1] << 8) | seg[2];
            w = (seg[3] << 8) | seg[4];
        } else if (mk == 0xDA) {
            pos += 2 + len;
            break;
        }
        pos += 2 + len;
    }
    const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4, nmcu = mbw * mbh;
    if (w_out) *w_out = w;
    if (h_out) *h_out = h;
    if (!coefs) return nmcu;
    if (nmcu > max_mcu) return -3;
    BR r = {jpg, n, pos, 0, 0};
    int pred[3] = {128, 128, 128};
    for (int m = 0; m < nmcu; m++)
        for (int b = 0; b < 6; b++) {
            int16_t *z = coefs + ((size_t)m * 6 + b) * 64;
            int comp = b < 4 ? 0 : b - 3, tab = b < 4 ? 0 : 1;
            memset(z, 0, 64 * sizeof(int16_t));
            int s = hdec_sym(&r, &hd[0][tab]);
            if (s < 0) return -4;
            int d = extend(br_bits(&r, s), s);
            pred[comp] += d;
            z[0] = (int16_t)pred[comp];
            for (int k = 1; k < 64;) {
                int rs = hdec_sym(&r, &hd[1][tab]);
                if (rs < 0) return -5;
                int run = rs >> 4, sz = rs & 15;
                if (sz == 0) {
                    if (run == 15) { k += 16; continue; }
                    break;
                }
                k += run;
                if (k > 63) return -6;
                z[k] = (int16_t)extend(br_bits(&r, sz), sz);
                k++;
            }
        }
    return nmcu;
}
