/*
 * ORACLE — test infrastructure only.  Annex-B NAL splitting, emulation
 * prevention removal and an RBSP bit reader shared by the oracle decoders
 * (ITU-T H.264/H.265 Annex B + 7.3.1/7.4.2 NAL unit syntax).  The reference
 * delegates this to FFmpeg's raw h264/hevc demuxers + parsers
 * (avformat_open_input / av_read_frame, /root/reference/src/Decoder.cpp:137,298).
 */
#ifndef H2J_ORACLE_BITS_H
#define H2J_ORACLE_BITS_H
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    const uint8_t *p; /* NAL payload including header, still escaped */
    long n;
} OraNal;

/* split an Annex-B byte stream into NAL units; returns count (<= max) */
static inline int ora_split_annexb(const uint8_t *d, long n, OraNal *out, int max) {
    int cnt = 0;
    long i = 0, start = -1;
    while (i + 2 < n) {
        if (d[i] == 0 && d[i + 1] == 0 && d[i + 2] == 1) {
            if (start >= 0 && cnt < max) {
                long e = i;
                while (e > start && d[e - 1] == 0) e--;
                out[cnt].p = d + start;
                out[cnt].n = e - start;
                cnt++;
            }
            i += 3;
            start = i;
            continue;
        }
        i++;
    }
    if (start >= 0 && start < n && cnt < max) {
        long e = n;
        while (e > start && d[e - 1] == 0) e--;
        out[cnt].p = d + start;
        out[cnt].n = e - start;
        cnt++;
    }
    return cnt;
}

/* remove emulation_prevention_three_byte; returns RBSP length */
static inline long ora_unescape(const uint8_t *src, long n, uint8_t *dst) {
    long o = 0;
    int zeros = 0;
    for (long i = 0; i < n; i++) {
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

typedef struct {
    const uint8_t *p;
    long n;    /* bytes */
    long pos;  /* bit position */
} OraBits;

static inline int ob_bit(OraBits *b) {
    long byte = b->pos >> 3;
    int v = byte < b->n ? (b->p[byte] >> (7 - (b->pos & 7))) & 1 : 0;
    b->pos++;
    return v;
}
static inline uint32_t ob_u(OraBits *b, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | (uint32_t)ob_bit(b);
    return v;
}
static inline uint32_t ob_ue(OraBits *b) {
    int lz = 0;
    while (!ob_bit(b)) {
        lz++;
        if (lz > 31) return 0xFFFFFFFFu;
    }
    return ((1u << lz) - 1) + ob_u(b, lz);
}
static inline int32_t ob_se(OraBits *b) {
    uint32_t k = ob_ue(b);
    return (k & 1) ? (int32_t)((k + 1) >> 1) : -(int32_t)(k >> 1);
}
static inline int ob_more_rbsp(OraBits *b) {
    /* true if there is more data before the rbsp_stop_one_bit */
    long last = b->n - 1;
    while (last >= 0 && b->p[last] == 0) last--;
    if (last < 0) return 0;
    int tz = 0;
    while (!((b->p[last] >> tz) & 1)) tz++;
    long stop = last * 8 + (7 - tz);
    return b->pos < stop;
}
/* FFmpeg 4.3 av_frame_apply_cropping (libavutil/frame.c) as decode.c applies it to every decoded
 * frame (AVCodecContext.apply_cropping 1, no AV_CODEC_FLAG_UNALIGNED): the left crop is lowered
 * until the cropped planes' data pointers keep the alignment FFmpeg's frame pool gives them
 * (linesizes are multiples of STRIDE_ALIGN >= 32, so only the left part of each plane's offset
 * decides): crop_left &= ~((1 << (5 + log2_crop_align - min_log2_align)) - 1) when
 * min_log2_align < 5, and AVERROR_BUG (no frame) when log2_crop_align < min_log2_align.
 * yuv420p / yuv420pN: planes at crop_left and crop_left >> 1, bps bytes per sample.  Returns the
 * effective left crop, -1 for AVERROR_BUG. */
static inline int ora_ff_crop_left(int cl, int bps) {
    if (cl <= 0) return cl;
    const int lca = __builtin_ctz((unsigned)cl);
    int m = 1000;
    const long part[2] = {(long)cl * bps, (long)(cl >> 1) * bps};
    for (int i = 0; i < 2; i++)
        if (part[i] && __builtin_ctzl((unsigned long)part[i]) < 5 && __builtin_ctzl((unsigned long)part[i]) < m)
            m = __builtin_ctzl((unsigned long)part[i]);
    if (m == 1000) return cl; /* every offset 32-byte aligned: unchanged */
    if (lca < m) return -1;
    return cl & ~((1 << (5 + lca - m)) - 1);
}

static inline int ora_ceil_log2(int v) {
    int r = 0;
    while ((1 << r) < v) r++;
    return r;
}
#endif
