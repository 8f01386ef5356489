/*
 * ORACLE — test infrastructure only.  Never linked into the product.
 *
 * Restates Decoder::H265ToJpeg (/root/reference/src/Decoder.cpp:115-361) on an
 * in-memory stream: codec auto-detection (the reference lets
 * avformat_open_input probe the raw h264/hevc demuxers, :137), decode of the
 * first picture only (:298-355), then Encoder::yuv2Jpeg
 * (src/Encoder.cpp:104-308).  The reference has no valid behaviour for
 * 10-bit pictures (it feeds LE16 samples to a YUVJ420P
 * encoder); the build's documented rule is v8 = min(255, (v + 2) >> 2).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bits.h"
#include "oracle.h"

/* 0 = unknown, 264 / 265 */
int oracle_detect_codec(const uint8_t *data, long size) {
    OraNal nals[64];
    int n = ora_split_annexb(data, size, nals, 64);
    int hv = 0, hs = 0, hp = 0, as = 0, ap = 0;
    for (int i = 0; i < n; i++) {
        if (nals[i].n < 2) continue;
        uint8_t h0 = nals[i].p[0], h1 = nals[i].p[1];
        if (!(h0 & 0x80)) {
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
    }
    if (hv && hs && hp) return 265;
    if (as && ap) return 264;
    return 0;
}

long oracle_transcode(const uint8_t *data, long size, const char *com, uint8_t *out, long cap) {
    OraclePicture p;
    int codec = oracle_detect_codec(data, size);
    int r;
    if (codec == 265) r = oracle_hevc_decode(data, size, 0, &p);
    else if (codec == 264) r = oracle_h264_decode(data, size, 0, &p);
    else return -100;
    if (r < 0) return r - 200;
    int w = p.width, h = p.height, cw = w / 2, ch = h / 2;
    uint8_t *pl[3];
    for (int c = 0; c < 3; c++) {
        int pw = c ? cw : w, ph = c ? ch : h;
        pl[c] = (uint8_t *)malloc((size_t)pw * ph);
        for (int y = 0; y < ph; y++)
            for (int x = 0; x < pw; x++) {
                int v = p.planes[c][(size_t)y * p.stride[c] + x];
                if (p.bit_depth > 8) {
                    v = (v + (1 << (p.bit_depth - 9))) >> (p.bit_depth - 8);
                    if (v > 255) v = 255;
                }
                pl[c][(size_t)y * pw + x] = (uint8_t)v;
            }
    }
    long n = oracle_jpeg_encode(pl[0], pl[1], pl[2], w, h, w, cw, com, out, cap);
    for (int c = 0; c < 3; c++) free(pl[c]);
    oracle_free_picture(&p);
    return n;
}
