/*
 * h264gen — deterministic H.264 (progressive 4:2:0, 8/10-bit, CABAC) intra
 * still-picture ENCODER used only to mint test vectors and benchmark inputs.
 * Test infrastructure: never linked into the product.  (The reference ships
 * libx264.a as a prebuilt binary, which this build may not load.)
 *
 * One IDR picture: SPS (Main 77, High 100 or High10 110) + PPS + N slices.
 * Macroblock decisions are heuristic (variance + SAD) with seeded random
 * choices that exercise: I4x4 / I8x8 (transform_size_8x8_flag) / I16x16 /
 * I_PCM, all prediction modes legal for the available neighbours, chroma
 * modes, mb_qp_delta, chroma QP offsets, multiple slices, deblocking
 * offsets / disable_deblocking_filter_idc.  Quantisation is generic
 * least-squares against the decoder's own reconstruction basis, so the
 * encoder reconstruction equals the decoder's by construction; the
 * reconstruction is written with --recon for the tests.
 *
 * usage: h264gen in.yuv W H bitdepth qp seed out.h264 [options]
 *   --t8x8 0|1 --pcm 0|1 --qpdelta 0|1 --slices N(MB rows, 0 = one)
 *   --alpha A --beta B (div2 offsets) --dbidc 0|1|2 --cqp N --cqp2 N --cavlc 0|1 --recon out.yuv
 *   --sm 0..3 (scaling matrices, see write_matrices)
 *   --nonidr 1 (first picture: non-IDR I, nal_unit_type 1)
 *   --delay K (VUI max_num_reorder_frames = K, then K + 1 all-skip P pictures)
 *   --mono 1 (4:0:0, chroma_format_idc 0: no chroma syntax; the reconstruction's chroma planes are
 *             1 << (bitdepth - 1), FFmpeg's output for monochrome streams)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/bits.h"
#include "../../oracle/cabac_tables.h"
#include "cavlc_tables.h"

static uint64_t g_rng = 1;
static uint32_t rnd(void) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (uint32_t)(g_rng >> 11);
}
static int rndn(int n) { return (int)(rnd() % (uint32_t)n); }
static int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

/* ------------------------------------------------------------ bit writer / NAL */
typedef struct {
    uint8_t *buf;
    size_t cap, n;
    uint32_t acc;
    int nb;
} BW;
static void bw_init(BW *b) { b->cap = 1 << 16; b->buf = (uint8_t *)malloc(b->cap); b->n = 0; b->acc = 0; b->nb = 0; }
static void bw_byte(BW *b, uint8_t v) {
    if (b->n == b->cap) { b->cap *= 2; b->buf = (uint8_t *)realloc(b->buf, b->cap); }
    b->buf[b->n++] = v;
}
static void bw_put(BW *b, uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) {
        b->acc = (b->acc << 1) | ((v >> i) & 1);
        if (++b->nb == 8) { bw_byte(b, (uint8_t)b->acc); b->acc = 0; b->nb = 0; }
    }
}
static void bw_ue(BW *b, uint32_t v) {
    uint32_t x = v + 1;
    int len = 0;
    while ((x >> len) > 1) len++;
    bw_put(b, 0, len);
    bw_put(b, x, len + 1);
}
static void bw_se(BW *b, int v) { bw_ue(b, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
static void bw_trailing(BW *b) { bw_put(b, 1, 1); while (b->nb) bw_put(b, 0, 1); }
static void bw_align_zero(BW *b) { while (b->nb) bw_put(b, 0, 1); }
static void write_nal(FILE *f, int ref_idc, int type, const uint8_t *p, size_t n) {
    static const uint8_t sc[4] = {0, 0, 0, 1};
    fwrite(sc, 1, 4, f);
    uint8_t h = (uint8_t)((ref_idc << 5) | type);
    fwrite(&h, 1, 1, f);
    int zeros = 0;
    for (size_t i = 0; i < n; i++) {
        if (zeros >= 2 && p[i] <= 3) { uint8_t e = 3; fwrite(&e, 1, 1, f); zeros = 0; }
        fwrite(&p[i], 1, 1, f);
        zeros = p[i] == 0 ? zeros + 1 : 0;
    }
}

/* ------------------------------------------------------------ CABAC encoder */
typedef struct {
    BW *bw;
    uint32_t low, range;
    int bits_left, nbuf;
    uint32_t bufbyte;
} Enc;
static void ce_start(Enc *e, BW *bw) { e->bw = bw; e->low = 0; e->range = 510; e->bits_left = 23; e->nbuf = 0; e->bufbyte = 0xff; }
static void ce_writeout(Enc *e) {
    uint32_t lead = e->low >> (24 - e->bits_left);
    e->bits_left += 8;
    e->low &= 0xffffffffu >> e->bits_left;
    if (lead == 0xff) { e->nbuf++; return; }
    if (e->nbuf > 0) {
        uint32_t carry = lead >> 8, byte = e->bufbyte + carry;
        e->bufbyte = lead & 0xff;
        bw_put(e->bw, byte, 8);
        byte = (0xff + carry) & 0xff;
        while (e->nbuf > 1) { bw_put(e->bw, byte, 8); e->nbuf--; }
    } else {
        e->nbuf = 1;
        e->bufbyte = lead;
    }
}
static void ce_test(Enc *e) { if (e->bits_left < 12) ce_writeout(e); }
static const uint8_t k_renorm[32] = {6, 5, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
static void ce_bin(Enc *e, uint8_t *ctx, int bin) {
    int s = *ctx >> 1, mps = *ctx & 1;
    uint32_t lps = ora_lps_table[s][(e->range >> 6) & 3];
    e->range -= lps;
    if (bin != mps) {
        int nb = k_renorm[lps >> 3];
        e->low = (e->low + e->range) << nb;
        e->range = lps << nb;
        if (s == 0) mps = 1 - mps;
        s = ora_trans_lps[s];
        e->bits_left -= nb;
    } else {
        if (s < 62) s++;
        *ctx = (uint8_t)((s << 1) | mps);
        if (e->range >= 256) return;
        e->low <<= 1;
        e->range <<= 1;
        e->bits_left--;
    }
    *ctx = (uint8_t)((s << 1) | mps);
    ce_test(e);
}
static void ce_byp(Enc *e, int bin) { e->low <<= 1; if (bin) e->low += e->range; e->bits_left--; ce_test(e); }
static void ce_term(Enc *e, int bin) {
    e->range -= 2;
    if (bin) { e->low += e->range; e->low <<= 7; e->range = 2 << 7; e->bits_left -= 7; }
    else if (e->range >= 256) return;
    else { e->low <<= 1; e->range <<= 1; e->bits_left--; }
    ce_test(e);
}
static void ce_finish(Enc *e) {
    if (e->low >> (32 - e->bits_left)) {
        bw_put(e->bw, e->bufbyte + 1, 8);
        while (e->nbuf > 1) { bw_put(e->bw, 0x00, 8); e->nbuf--; }
        e->low -= 1u << (32 - e->bits_left);
    } else {
        if (e->nbuf > 0) bw_put(e->bw, e->bufbyte, 8);
        while (e->nbuf > 1) { bw_put(e->bw, 0xff, 8); e->nbuf--; }
    }
    bw_put(e->bw, e->low >> 8, 24 - e->bits_left);
}

/* ------------------------------------------------------------ CABAC init (I) */
#include "h264_init_I.inc"

static const uint8_t k_sig8x8[64] = {0, 1, 2, 3, 4, 5, 5, 4, 4, 3, 3, 4, 4, 4, 5, 5, 4, 4, 4, 4, 3, 3,
                                     6, 7, 7, 7, 8, 9, 10, 9, 8, 7, 7, 6, 11, 12, 13, 11, 6, 7, 8, 9, 14, 10,
                                     9, 8, 6, 11, 12, 13, 11, 6, 9, 14, 10, 9, 11, 12, 13, 11, 14, 10, 12};
static const uint8_t k_last8x8[64] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2,
                                      2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4,
                                      4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8, 8};
static const uint8_t k_zz4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
/* field scans (field macroblocks, 8.5.6 / 8.5.7) and the field-coded 8x8 significance contexts (Table 9-43) */
static const uint8_t k_fld4[16] = {0, 4, 1, 8, 12, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
static const uint8_t k_fld8[64] = {0, 8, 16, 1, 9, 24, 32, 17, 2, 25, 40, 48, 56, 33, 10, 3, 18, 41, 49, 57, 26, 11,
                                   4, 19, 34, 42, 50, 58, 27, 12, 5, 20, 35, 43, 51, 59, 28, 13, 6, 21, 36, 44,
                                   52, 60, 29, 14, 22, 37, 45, 53, 61, 30, 7, 15, 38, 46, 54, 62, 23, 31, 39, 47, 55, 63};
static const uint8_t k_sig8x8_fld[63] = {0, 1, 1, 2, 2, 3, 3, 4, 5, 6, 7, 7, 7, 8, 4, 5, 6, 9, 10, 10, 8, 11,
                                         12, 11, 9, 9, 10, 10, 8, 11, 12, 11, 9, 9, 10, 10, 8, 11, 12, 11, 9, 9,
                                         10, 10, 8, 13, 13, 9, 9, 10, 10, 8, 13, 13, 9, 9, 10, 10, 14, 14, 14, 14, 14};
static const uint8_t k_zz8[64] = {0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
                                  41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                                  30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
static const uint8_t k_blk_x[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
static const uint8_t k_blk_y[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
static const uint8_t k_blk_of[4][4] = {{0, 1, 4, 5}, {2, 3, 6, 7}, {8, 9, 12, 13}, {10, 11, 14, 15}};

/* ------------------------------------------------------------ state */
typedef struct {
    int slice, mb_type, t8x8, cbp, qp, cpm;
    uint8_t ipm[16], cbf[16], cbf_c[2][4], cbf_dc[3];
    uint8_t tc[16], tcc[2][4];  /* CAVLC TotalCoeff per luma / chroma AC 4x4 block */
    int field, vx, vy;          /* --mbaff: the pair's mb_field_decoding_flag; grid position (vy = 2 pair row + bottom) */
} Mb;

typedef struct {
    int W, H, outW, outH, mbw, mbh, bd, qp, t8x8, pcm, qpdelta, slice_rows, alpha, beta, dbidc, cqp, cqp2, cavlc, sm, nonidr, delay, firstmb, vuireorder, vuicpb, ilsps, lossless, mbaff, cur_field, paff, onefield, mono;
    long long rawcrop[4];
    uint16_t *src[3], *rec[3];
    int st[3];
    Mb *mb;
    int mbx, mby, cur_slice;
    uint8_t ctx[460];
    Enc ce;
    int cur_qp, prev_qpd_nz;
} G;

static Mb *mb_in_slice(G *g, int x, int y) {
    if (x < 0 || y < 0 || x >= g->mbw || y >= g->mbh) return NULL;
    Mb *m = &g->mb[y * g->mbw + x];
    return m->slice == g->cur_slice ? m : NULL;
}
/* 6.4.12: macroblock covering (xN, yN) relative to the current MB (maxW x maxH) and the location
 * (xW, yW) inside it, NULL if unavailable; --mbaff: 6.4.12.2 / Table 6-4 (the decoder's rules) */
static Mb *nb_loc(G *g, int xN, int yN, int maxW, int maxH, int *xW, int *yW) {
    Mb *cur = &g->mb[g->mby * g->mbw + g->mbx];
    if (yN > maxH - 1 || (xN > maxW - 1 && yN >= 0)) return NULL;
    *xW = (xN + maxW) % maxW;
    if (xN >= 0 && xN <= maxW - 1 && yN >= 0) { *yW = yN; return cur; }
    if (!g->mbaff || g->paff) { /* --paff: the neighbours of a field MB are in its own field */
        *yW = (yN + maxH) % maxH;
        return mb_in_slice(g, g->mbx + (xN < 0 ? -1 : (xN > maxW - 1 ? 1 : 0)), g->mby + (yN < 0 ? (g->paff ? -2 : -1) : 0));
    }
    const int px = g->mbx, py = g->mby >> 1, top = !(g->mby & 1), frame = !cur->field;
    Mb *X = NULL;
    int yM = yN, bot = 0;
    if (xN < 0 && yN < 0) {
        if (frame && !top) { X = mb_in_slice(g, px - 1, 2 * py); if (!X) return NULL; bot = X->field; yM = X->field ? (yN + maxH) >> 1 : yN; }
        else if (frame || !top) { X = mb_in_slice(g, px - 1, 2 * py - 2); bot = 1; }
        else { X = mb_in_slice(g, px - 1, 2 * py - 2); if (!X) return NULL; if (!X->field) { bot = 1; yM = 2 * yN; } }
    } else if (xN < 0) {
        X = mb_in_slice(g, px - 1, 2 * py);
        if (!X) return NULL;
        if (frame) {
            if (!X->field) bot = top ? 0 : 1;
            else { bot = yN & 1; yM = top ? yN >> 1 : (yN + maxH) >> 1; }
        } else if (!X->field) {
            if (yN < maxH / 2) { bot = 0; yM = (yN << 1) + (top ? 0 : 1); }
            else { bot = 1; yM = (yN << 1) + (top ? 0 : 1) - maxH; }
        } else bot = top ? 0 : 1;
    } else if (xN <= maxW - 1) {
        if (frame && !top) X = &g->mb[(2 * py) * g->mbw + px];
        else if (frame || !top) { X = mb_in_slice(g, px, 2 * py - 2); bot = 1; }
        else { X = mb_in_slice(g, px, 2 * py - 2); if (!X) return NULL; if (!X->field) { bot = 1; yM = 2 * yN; } }
    } else {
        if (frame && !top) return NULL;
        if (frame || !top) { X = mb_in_slice(g, px + 1, 2 * py - 2); bot = 1; }
        else { X = mb_in_slice(g, px + 1, 2 * py - 2); if (!X) return NULL; if (!X->field) { bot = 1; yM = 2 * yN; } }
    }
    if (!X) return NULL;
    *yW = (yM + maxH) % maxH;
    return &g->mb[(X->vy + bot) * g->mbw + X->vx];
}
static Mb *nb(G *g, int dx, int dy) {
    int xW, yW;
    return nb_loc(g, dx < 0 ? -1 : (dx > 0 ? 16 : 0), dy < 0 ? -1 : 0, 16, 16, &xW, &yW);
}
static Mb *nb_blk(G *g, int bx, int by, int *nblk) {
    int xW, yW;
    Mb *m = nb_loc(g, bx * 4, by * 4, 16, 16, &xW, &yW);
    *nblk = m ? k_blk_of[yW >> 2][xW >> 2] : 0;
    return m;
}
/* picture position of sample (xW, yW) of component c of macroblock N (field MBs interleave rows) */
static int mb_phys(const G *g, const Mb *N, int c, int xW, int yW) {
    const int S = c ? 8 : 16, X = N->vx * S + xW;
    int Y;
    if (!g->mbaff) Y = N->vy * S + yW;
    else Y = N->field ? 2 * (N->vy >> 1) * S + 2 * yW + (N->vy & 1) : N->vy * S + yW;
    return Y * g->st[c] + X;
}
/* source / reconstruction of the current MB at grid position (x, y) */
static int srcv(G *g, int c, int x, int y) {
    const int S = c ? 8 : 16;
    return g->src[c][mb_phys(g, &g->mb[g->mby * g->mbw + g->mbx], c, x - g->mbx * S, y - g->mby * S)];
}
static void recv_put(G *g, int c, int x, int y, int v) {
    const int S = c ? 8 : 16;
    g->rec[c][mb_phys(g, &g->mb[g->mby * g->mbw + g->mbx], c, x - g->mbx * S, y - g->mby * S)] = (uint16_t)v;
}
static int avail_luma(G *g, int x, int y, int cur_blk4) {
    if (y < 0 && x < 0) return nb(g, -1, -1) != NULL;
    if (y < 0 && x >= 16) return nb(g, 1, -1) != NULL;
    if (y < 0) return nb(g, 0, -1) != NULL;
    if (x < 0) return nb(g, -1, 0) != NULL;
    if (x >= 16) return 0;
    return k_blk_of[y >> 2][x >> 2] < cur_blk4;
}
static int px(G *g, int c, int x, int y) {
    if (!g->mbaff) return g->rec[c][y * g->st[c] + x];
    const int S = c ? 8 : 16;
    int xW, yW;
    Mb *N = nb_loc(g, x - g->mbx * S, y - g->mby * S, S, S, &xW, &yW);
    return N ? g->rec[c][mb_phys(g, N, c, xW, yW)] : 0;
}

/* ------------------------------------------------------------ prediction (same formulas as the decoder) */
typedef struct { int T[16], L[16], C, at, al, ad, atr; } Nb;

static int pred_nxn(int mode, int x, int y, int n, const int *T, const int *L, int C, int dcv) {
#define TT(i) ((i) < 0 ? C : T[i])
#define LL(i) ((i) < 0 ? C : L[i])
    switch (mode) {
    case 0: return T[x];
    case 1: return L[y];
    case 2: return dcv;
    case 3: return (x == n - 1 && y == n - 1) ? (T[2 * n - 2] + 3 * T[2 * n - 1] + 2) >> 2 : (T[x + y] + 2 * T[x + y + 1] + T[x + y + 2] + 2) >> 2;
    case 4:
        if (x > y) return (TT(x - y - 2) + 2 * TT(x - y - 1) + T[x - y] + 2) >> 2;
        if (x < y) return (LL(y - x - 2) + 2 * LL(y - x - 1) + L[y - x] + 2) >> 2;
        return (T[0] + 2 * C + L[0] + 2) >> 2;
    case 5: {
        int z = 2 * x - y;
        if (z >= 0 && !(z & 1)) return (TT(x - (y >> 1) - 1) + T[x - (y >> 1)] + 1) >> 1;
        if (z >= 0) return (TT(x - (y >> 1) - 2) + 2 * TT(x - (y >> 1) - 1) + T[x - (y >> 1)] + 2) >> 2;
        if (z == -1) return (L[0] + 2 * C + T[0] + 2) >> 2;
        return (L[y - 2 * x - 1] + 2 * L[y - 2 * x - 2] + LL(y - 2 * x - 3) + 2) >> 2;
    }
    case 6: {
        int z = 2 * y - x;
        if (z >= 0 && !(z & 1)) return (LL(y - (x >> 1) - 1) + L[y - (x >> 1)] + 1) >> 1;
        if (z >= 0) return (LL(y - (x >> 1) - 2) + 2 * LL(y - (x >> 1) - 1) + L[y - (x >> 1)] + 2) >> 2;
        if (z == -1) return (L[0] + 2 * C + T[0] + 2) >> 2;
        return (T[x - 2 * y - 1] + 2 * T[x - 2 * y - 2] + TT(x - 2 * y - 3) + 2) >> 2;
    }
    case 7: { int i = x + (y >> 1); return !(y & 1) ? (T[i] + T[i + 1] + 1) >> 1 : (T[i] + 2 * T[i + 1] + T[i + 2] + 2) >> 2; }
    default: {
        int z = x + 2 * y, lim = 2 * n - 3;
        if (z > lim) return L[n - 1];
        if (z == lim) return (L[n - 2] + 3 * L[n - 1] + 2) >> 2;
        int i = y + (x >> 1);
        return !(z & 1) ? (L[i] + L[i + 1] + 1) >> 1 : (L[i] + 2 * L[i + 1] + L[i + 2] + 2) >> 2;
    }
    }
#undef TT
#undef LL
}

static void gather4(G *g, int blk, Nb *o) {
    int x0 = k_blk_x[blk] * 4, y0 = k_blk_y[blk] * 4, gx = g->mbx * 16 + x0, gy = g->mby * 16 + y0;
    o->at = avail_luma(g, x0, y0 - 1, blk);
    o->al = avail_luma(g, x0 - 1, y0, blk);
    o->ad = avail_luma(g, x0 - 1, y0 - 1, blk);
    o->atr = avail_luma(g, x0 + 4, y0 - 1, blk);
    for (int i = 0; i < 4; i++) {
        o->T[i] = o->at ? px(g, 0, gx + i, gy - 1) : 0;
        o->L[i] = o->al ? px(g, 0, gx - 1, gy + i) : 0;
    }
    for (int i = 4; i < 8; i++) o->T[i] = o->atr ? px(g, 0, gx + i, gy - 1) : o->T[3];
    o->C = o->ad ? px(g, 0, gx - 1, gy - 1) : 0;
}
static void gather8(G *g, int b8, Nb *o) {
    int x0 = (b8 & 1) * 8, y0 = (b8 >> 1) * 8, gx = g->mbx * 16 + x0, gy = g->mby * 16 + y0, blk4 = b8 * 4;
    int at = avail_luma(g, x0, y0 - 1, blk4), al = avail_luma(g, x0 - 1, y0, blk4), ad = avail_luma(g, x0 - 1, y0 - 1, blk4);
    int atr = avail_luma(g, x0 + 8, y0 - 1, blk4);
    int Tr[16], Lr[8], C = ad ? px(g, 0, gx - 1, gy - 1) : 0;
    for (int i = 0; i < 8; i++) { Tr[i] = at ? px(g, 0, gx + i, gy - 1) : 0; Lr[i] = al ? px(g, 0, gx - 1, gy + i) : 0; }
    for (int i = 8; i < 16; i++) Tr[i] = atr ? px(g, 0, gx + i, gy - 1) : Tr[7];
    memset(o, 0, sizeof(*o));
    o->at = at; o->al = al; o->ad = ad; o->atr = atr;
    if (at) {
        o->T[0] = ad ? (C + 2 * Tr[0] + Tr[1] + 2) >> 2 : (3 * Tr[0] + Tr[1] + 2) >> 2;
        for (int x = 1; x < 15; x++) o->T[x] = (Tr[x - 1] + 2 * Tr[x] + Tr[x + 1] + 2) >> 2;
        o->T[15] = (Tr[14] + 3 * Tr[15] + 2) >> 2;
    }
    o->C = C;
    if (ad) {
        if (at && al) o->C = (Tr[0] + 2 * C + Lr[0] + 2) >> 2;
        else if (at) o->C = (3 * C + Tr[0] + 2) >> 2;
        else if (al) o->C = (3 * C + Lr[0] + 2) >> 2;
    }
    if (al) {
        o->L[0] = ad ? (C + 2 * Lr[0] + Lr[1] + 2) >> 2 : (3 * Lr[0] + Lr[1] + 2) >> 2;
        for (int y = 1; y < 7; y++) o->L[y] = (Lr[y - 1] + 2 * Lr[y] + Lr[y + 1] + 2) >> 2;
        o->L[7] = (Lr[6] + 3 * Lr[7] + 2) >> 2;
    }
}
static int mode_legal(int mode, const Nb *o) {
    switch (mode) {
    case 0: case 3: case 7: return o->at;
    case 1: case 8: return o->al;
    case 2: return 1;
    default: return o->at && o->al && o->ad;
    }
}
static void predict_nxn(G *g, int n, int mode, const Nb *o, int *pred) {
    int dcv, s = 0, lg = n == 4 ? 2 : 3;
    if (o->at && o->al) { for (int i = 0; i < n; i++) s += o->T[i] + o->L[i]; dcv = (s + n) >> (lg + 1); }
    else if (o->al) { for (int i = 0; i < n; i++) s += o->L[i]; dcv = (s + n / 2) >> lg; }
    else if (o->at) { for (int i = 0; i < n; i++) s += o->T[i]; dcv = (s + n / 2) >> lg; }
    else dcv = 1 << (g->bd - 1);
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) pred[y * n + x] = pred_nxn(mode, x, y, n, o->T, o->L, o->C, dcv);
}
static void pred16(G *g, int mode, int *pred) {
    int gx = g->mbx * 16, gy = g->mby * 16;
    int at = nb(g, 0, -1) != NULL, al = nb(g, -1, 0) != NULL, ad = nb(g, -1, -1) != NULL;
    int T[16], L[16], C = ad ? px(g, 0, gx - 1, gy - 1) : 0, maxv = (1 << g->bd) - 1;
    for (int i = 0; i < 16; i++) { T[i] = at ? px(g, 0, gx + i, gy - 1) : 0; L[i] = al ? px(g, 0, gx - 1, gy + i) : 0; }
    if (mode == 0) { for (int i = 0; i < 256; i++) pred[i] = T[i & 15]; return; }
    if (mode == 1) { for (int i = 0; i < 256; i++) pred[i] = L[i >> 4]; return; }
    if (mode == 2) {
        int s = 0;
        if (at && al) { for (int i = 0; i < 16; i++) s += T[i] + L[i]; s = (s + 16) >> 5; }
        else if (al) { for (int i = 0; i < 16; i++) s += L[i]; s = (s + 8) >> 4; }
        else if (at) { for (int i = 0; i < 16; i++) s += T[i]; s = (s + 8) >> 4; }
        else s = 1 << (g->bd - 1);
        for (int i = 0; i < 256; i++) pred[i] = s;
        return;
    }
    int H = 0, V = 0;
    for (int i = 0; i < 8; i++) { H += (i + 1) * (T[8 + i] - (i == 7 ? C : T[6 - i])); V += (i + 1) * (L[8 + i] - (i == 7 ? C : L[6 - i])); }
    int a = 16 * (L[15] + T[15]), b = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
    for (int y = 0; y < 16; y++) for (int x = 0; x < 16; x++) pred[y * 16 + x] = clip3(0, maxv, (a + b * (x - 7) + c * (y - 7) + 16) >> 5);
}
static void predc(G *g, int c, int mode, int *pred) {
    int gx = g->mbx * 8, gy = g->mby * 8;
    int at = nb(g, 0, -1) != NULL, al = nb(g, -1, 0) != NULL, ad = nb(g, -1, -1) != NULL;
    int T[8], L[8], C = ad ? px(g, c, gx - 1, gy - 1) : 0, maxv = (1 << g->bd) - 1;
    for (int i = 0; i < 8; i++) { T[i] = at ? px(g, c, gx + i, gy - 1) : 0; L[i] = al ? px(g, c, gx - 1, gy + i) : 0; }
    if (mode == 0) {
        for (int by = 0; by < 2; by++)
            for (int bx = 0; bx < 2; bx++) {
                int st = 0, sl = 0, s;
                for (int i = 0; i < 4; i++) { st += T[bx * 4 + i]; sl += L[by * 4 + i]; }
                if (bx == by) s = (at && al) ? (st + sl + 4) >> 3 : at ? (st + 2) >> 2 : al ? (sl + 2) >> 2 : 1 << (g->bd - 1);
                else if (bx) s = at ? (st + 2) >> 2 : al ? (sl + 2) >> 2 : 1 << (g->bd - 1);
                else s = al ? (sl + 2) >> 2 : at ? (st + 2) >> 2 : 1 << (g->bd - 1);
                for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) pred[(by * 4 + y) * 8 + bx * 4 + x] = s;
            }
        return;
    }
    if (mode == 1) { for (int i = 0; i < 64; i++) pred[i] = L[i >> 3]; return; }
    if (mode == 2) { for (int i = 0; i < 64; i++) pred[i] = T[i & 7]; return; }
    int H = 0, V = 0;
    for (int i = 0; i < 4; i++) { H += (i + 1) * (T[4 + i] - (i == 3 ? C : T[2 - i])); V += (i + 1) * (L[4 + i] - (i == 3 ? C : L[2 - i])); }
    int a = 16 * (L[7] + T[7]), b = (34 * H + 32) >> 6, cc = (34 * V + 32) >> 6;
    for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) pred[y * 8 + x] = clip3(0, maxv, (a + b * (x - 3) + cc * (y - 3) + 16) >> 5);
}

/* ------------------------------------------------------------ decoder-side residual (dequant + IDCT) */
static const int k_norm4[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
static const int k_norm8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                                  {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
static int norm4(int m, int i, int j) { return (!(i & 1) && !(j & 1)) ? k_norm4[m][0] : ((i & 1) && (j & 1)) ? k_norm4[m][1] : k_norm4[m][2]; }
static int norm8(int m, int i, int j) {
    if (!(i & 3) && !(j & 3)) return k_norm8[m][0];
    if ((i & 1) && (j & 1)) return k_norm8[m][1];
    if ((i & 3) == 2 && (j & 3) == 2) return k_norm8[m][2];
    if ((!(i & 3) && (j & 1)) || ((i & 1) && !(j & 3))) return k_norm8[m][3];
    if ((!(i & 3) && (j & 3) == 2) || ((i & 3) == 2 && !(j & 3))) return k_norm8[m][4];
    return k_norm8[m][5];
}
static int sc4(int l, int ls, int qp) { return qp >= 24 ? (l * ls) << (qp / 6 - 4) : (l * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6); }
static int sc8(int l, int ls, int qp) { return qp >= 36 ? (l * ls) << (qp / 6 - 6) : (l * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6); }
/* conformance (8.5.12.1 / 8.5.13.1): scaled coefficients and transform intermediates fit
 * -2^(7+bitDepth) .. 2^(7+bitDepth)-1 (FFmpeg stores them in int16 at 8-bit) */
static int g_lim = 1 << 15, g_viol;
static void range_check(int v) { if (v < -g_lim || v >= g_lim) g_viol = 1; }
static void idct4(int *b) {
    int t[16];
    for (int i = 0; i < 16; i++) range_check(b[i]);
    for (int i = 0; i < 4; i++) {
        int *r = b + i * 4, e0 = r[0] + r[2], e1 = r[0] - r[2], e2 = (r[1] >> 1) - r[3], e3 = r[1] + (r[3] >> 1);
        t[i * 4] = e0 + e3; t[i * 4 + 1] = e1 + e2; t[i * 4 + 2] = e1 - e2; t[i * 4 + 3] = e0 - e3;
    }
    for (int i = 0; i < 16; i++) range_check(t[i]);
    for (int j = 0; j < 4; j++) {
        int f0 = t[j], f1 = t[4 + j], f2 = t[8 + j], f3 = t[12 + j];
        int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        b[j] = (g0 + g3 + 32) >> 6; b[4 + j] = (g1 + g2 + 32) >> 6; b[8 + j] = (g1 - g2 + 32) >> 6; b[12 + j] = (g0 - g3 + 32) >> 6;
    }
}
static void idct8_1d(const int *d, int *o) {
    int a0 = d[0] + d[4], a4 = d[0] - d[4], a2 = (d[2] >> 1) - d[6], a6 = d[2] + (d[6] >> 1);
    int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
    int a1 = -d[3] + d[5] - d[7] - (d[7] >> 1), a3 = d[1] + d[7] - d[3] - (d[3] >> 1);
    int a5 = -d[1] + d[7] + d[5] + (d[5] >> 1), a7 = d[3] + d[5] + d[1] + (d[1] >> 1);
    int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
    o[0] = b0 + b7; o[1] = b2 + b5; o[2] = b4 + b3; o[3] = b6 + b1; o[4] = b6 - b1; o[5] = b4 - b3; o[6] = b2 - b5; o[7] = b0 - b7;
}
static void idct8(int *b) {
    int t[64], col[8], o[8];
    for (int i = 0; i < 64; i++) range_check(b[i]);
    for (int i = 0; i < 8; i++) idct8_1d(b + i * 8, t + i * 8);
    for (int i = 0; i < 64; i++) range_check(t[i]);
    for (int j = 0; j < 8; j++) {
        for (int i = 0; i < 8; i++) col[i] = t[i * 8 + j];
        idct8_1d(col, o);
        for (int i = 0; i < 8; i++) b[i * 8 + j] = (o[i] + 32) >> 6;
    }
}
/* residual of a 4x4 / 8x8 block from raster levels; w = raster weightScale (8.5.9) */
static void res4(const int *lv, int qp, int *r, const int *w) {
    for (int i = 0; i < 16; i++) r[i] = sc4(lv[i], w[i] * norm4(qp % 6, i >> 2, i & 3), qp);
    idct4(r);
}
static void res8(const int *lv, int qp, int *r, const int *w) {
    for (int i = 0; i < 64; i++) r[i] = sc8(lv[i], w[i] * norm8(qp % 6, i >> 3, i & 7), qp);
    idct8(r);
}
/* MB-wide residual for I16x16 (n = 16, luma) or chroma (n = 8): DC levels at (4i,4j) */
static void res_dc(const int *lv, int n, int qp, int *r, const int *w) {
    int nb = n / 4, dc[16];
    for (int r0 = 0; r0 < nb; r0++)
        for (int q = 0; q < nb; q++) {
            int acc = 0;
            for (int i = 0; i < nb; i++)
                for (int j = 0; j < nb; j++) {
                    int hr = nb == 4 ? ((r0 == 0 || (r0 == 1 && i < 2) || (r0 == 2 && (i == 0 || i == 3)) || (r0 == 3 && !(i & 1))) ? 1 : -1) : ((r0 == 0 || i == 0) ? 1 : -1);
                    int hc = nb == 4 ? ((q == 0 || (q == 1 && j < 2) || (q == 2 && (j == 0 || j == 3)) || (q == 3 && !(j & 1))) ? 1 : -1) : ((q == 0 || j == 0) ? 1 : -1);
                    acc += hr * hc * lv[(i * 4) * n + j * 4];
                }
            int ls0 = w[0] * k_norm4[qp % 6][0];
            dc[r0 * nb + q] = nb == 4 ? (qp >= 36 ? (acc * ls0) << (qp / 6 - 6) : (acc * ls0 + (1 << (5 - qp / 6))) >> (6 - qp / 6))
                                      : ((acc * ls0) << (qp / 6)) >> 5;
            range_check(dc[r0 * nb + q]);
        }
    for (int by = 0; by < nb; by++)
        for (int bx = 0; bx < nb; bx++) {
            int b[16];
            for (int i = 0; i < 16; i++) b[i] = sc4(lv[(by * 4 + (i >> 2)) * n + bx * 4 + (i & 3)], w[i] * norm4(qp % 6, i >> 2, i & 3), qp);
            b[0] = dc[by * nb + bx];
            idct4(b);
            for (int i = 0; i < 16; i++) r[(by * 4 + (i >> 2)) * n + bx * 4 + (i & 3)] = b[i];
        }
}

/* ------------------------------------------------------------ least-squares quantiser against the decoder basis */
typedef struct { float *basis; int n, npos; } Basis; /* basis[pos][sample] for unit level */
static Basis g_b4[88], g_b8[88], g_b16[88], g_bc[2][88]; /* qP up to 51 + QpBdOffset (14-bit: 87) */

/* weightScale matrices in raster order (8.5.6 inverse zig-zag of the active scaling lists):
 * [0..2] Intra Y / Cb / Cr 4x4, g_w8 Intra Y 8x8; flat 16 without scaling matrices */
static int g_w4[3][16], g_w8[64];

static void build_basis(Basis *B, int kind, int qp, const int *w) {
    int n = kind == 0 ? 4 : (kind == 1 ? 8 : (kind == 2 ? 16 : 8));
    if (B->basis) return;
    B->n = n;
    B->npos = n * n;
    B->basis = (float *)calloc((size_t)n * n * n * n, sizeof(float));
    const int L = 64;
    for (int p = 0; p < n * n; p++) {
        int lv[256] = {0}, r[256];
        if ((kind == 2 || kind == 3) && 0) {}
        lv[p] = L;
        if (kind == 0) res4(lv, qp, r, w);
        else if (kind == 1) res8(lv, qp, r, w);
        else res_dc(lv, n, qp, r, w);
        for (int i = 0; i < n * n; i++) B->basis[p * n * n + i] = (float)r[i] / L;
    }
}
/* levels[raster] minimising ||x - Σ l b|| approximately (independent projections + deadzone) */
static void quantize(const Basis *B, const int *x, int *lv, int maxlev) {
    int nn = B->npos;
    for (int p = 0; p < nn; p++) {
        const float *b = B->basis + (size_t)p * nn;
        double dot = 0, bb = 0;
        for (int i = 0; i < nn; i++) { dot += b[i] * x[i]; bb += (double)b[i] * b[i]; }
        double v = bb > 0 ? dot / bb : 0;
        int l = (int)(fabs(v) + 0.6667 - 1.0 + 0.3333 * 0 + 0.0);
        l = (int)(fabs(v) + 1.0 / 3.0);
        if (l > maxlev) l = maxlev;
        lv[p] = v < 0 ? -l : l;
    }
}
/* shrink the levels of a block until its reconstruction stays in the conformant range */
static void fit(int kind, int *lv, int qp, const int *w) {
    int n = kind == 0 ? 4 : (kind == 1 ? 8 : (kind == 2 ? 16 : 8)), r[256];
    for (;;) {
        g_viol = 0;
        if (kind == 0) res4(lv, qp, r, w);
        else if (kind == 1) res8(lv, qp, r, w);
        else res_dc(lv, n, qp, r, w);
        if (!g_viol) return;
        for (int i = 0; i < n * n; i++) lv[i] = lv[i] * 3 / 4;
    }
}

/* ------------------------------------------------------------ CABAC syntax */
static int bin(G *g, int ctx, int v) { ce_bin(&g->ce, &g->ctx[ctx], v); return v; }

/* ------------------------------------------------------------ CAVLC (9.2) */
static int cavlc_nc(int na, int aa, int nb_, int ab) {
    if (aa && ab) return (na + nb_ + 1) >> 1;
    return aa ? na : (ab ? nb_ : 0);
}
/* residual_block_cavlc for coefficients co[0..maxnum-1] in scan order; returns TotalCoeff */
static int enc_block_cavlc(G *g, int nC, int maxnum, const int *co) {
    BW *b = g->ce.bw;
    int idx[16], lv[16], tc = 0;
    for (int i = maxnum - 1; i >= 0; i--)
        if (co[i]) { idx[tc] = i; lv[tc] = co[i]; tc++; }  /* highest frequency first */
    int t1 = 0;
    while (t1 < tc && t1 < 3 && abs(lv[t1]) == 1) t1++;
    if (nC >= 8) {
        bw_put(b, tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u, 6);
    } else {
        int col = nC < 0 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
        bw_put(b, kCoeffTokenCode[col][t1][tc], kCoeffTokenLen[col][t1][tc]);
    }
    if (!tc) return 0;
    for (int i = 0; i < t1; i++) bw_put(b, lv[i] < 0, 1);
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = t1; i < tc; i++) {
        int code = lv[i] > 0 ? 2 * lv[i] - 2 : -2 * lv[i] - 1;
        if (i == t1 && t1 < 3) code -= 2;
        int prefix, ssz, suffix;
        if (sl == 0) {
            if (code < 14) { prefix = code; ssz = 0; suffix = 0; }
            else if (code < 30) { prefix = 14; ssz = 4; suffix = code - 14; }
            else { prefix = 15; ssz = 12; suffix = code - 30; }
        } else if (code < (15 << sl)) {
            prefix = code >> sl; ssz = sl; suffix = code & ((1 << sl) - 1);
        } else {
            prefix = 15; ssz = 12; suffix = code - (15 << sl);
        }
        if (suffix >= 4096) { /* level_prefix >= 16 (high bit depths, 7.4.5.3.2): levelCode adds
                                * (1 << (level_prefix - 3)) - 4096, suffix of level_prefix - 3 bits */
            int base = code - suffix; /* levelCode at level_prefix 15, suffix 0 */
            prefix = 16;
            while (code >= base + (1 << (prefix - 3)) - 4096 + (1 << (prefix - 3)) && prefix < 28) prefix++;
            ssz = prefix - 3;
            suffix = code - (base + (1 << (prefix - 3)) - 4096);
            if (suffix < 0 || suffix >= (1 << ssz)) { fprintf(stderr, "level out of CAVLC range\n"); exit(3); }
        }
        bw_put(b, 1, prefix + 1);  /* prefix zeros then 1 */
        if (ssz) bw_put(b, (uint32_t)suffix, ssz);
        if (sl == 0) sl = 1;
        if (abs(lv[i]) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int zeros = idx[0] + 1 - tc;
    if (tc < maxnum) {
        if (maxnum == 4) bw_put(b, kTotalZerosDcCode[tc - 1][zeros], kTotalZerosDcLen[tc - 1][zeros]);
        else bw_put(b, kTotalZerosCode[tc - 1][zeros], kTotalZerosLen[tc - 1][zeros]);
    }
    for (int i = 0; i < tc - 1 && zeros > 0; i++) {
        int run = idx[i] - idx[i + 1] - 1;
        int zl = zeros < 7 ? zeros : 7;
        bw_put(b, kRunBeforeCode[zl - 1][run], kRunBeforeLen[zl - 1][run]);
        zeros -= run;
    }
    return tc;
}
static int nc_luma(G *g, int blk) {
    int nblk, va = 0, vb = 0;
    Mb *A = nb_blk(g, k_blk_x[blk] - 1, k_blk_y[blk], &nblk);
    if (A) va = A->mb_type == 25 ? 16 : A->tc[nblk];
    Mb *B = nb_blk(g, k_blk_x[blk], k_blk_y[blk] - 1, &nblk);
    if (B) vb = B->mb_type == 25 ? 16 : B->tc[nblk];
    return cavlc_nc(va, A != NULL, vb, B != NULL);
}
static int nc_chroma(G *g, Mb *m, int c, int b4) {
    int bx = b4 & 1, by = b4 >> 1, va = 0, vb = 0, aa = 1, ab = 1;
    if (bx) va = m->tcc[c][b4 - 1];
    else { int xW, yW; Mb *A = nb_loc(g, -1, by * 4, 8, 8, &xW, &yW); if (!A) aa = 0; else va = A->mb_type == 25 ? 16 : A->tcc[c][(yW >> 2) * 2 + (xW >> 2)]; }
    if (by) vb = m->tcc[c][b4 - 2];
    else { int xW, yW; Mb *B = nb_loc(g, bx * 4, -1, 8, 8, &xW, &yW); if (!B) ab = 0; else vb = B->mb_type == 25 ? 16 : B->tcc[c][(yW >> 2) * 2 + (xW >> 2)]; }
    return cavlc_nc(va, aa, vb, ab);
}

static int cbf_cond(int cat, Mb *N, int nblk, int icbcr) {
    if (!N) return 1;
    if (N->mb_type == 25) return 1;
    switch (cat) {
    case 0: return (N->mb_type >= 1 && N->mb_type <= 24) ? N->cbf_dc[0] : 0;
    case 1: case 2: return ((N->cbp >> (nblk >> 2)) & 1) ? N->cbf[nblk] : 0;
    case 3: return (N->cbp >> 4) ? N->cbf_dc[1 + icbcr] : 0;
    case 4: return (N->cbp >> 4) == 2 ? N->cbf_c[icbcr][nblk] : 0;
    }
    return 0;
}

/* coeffs in scan order; returns coded */
static int enc_block(G *g, int cat, int cbf_inc, int maxnum, const int *co) {
    static const int cbf_off[5] = {0, 4, 8, 12, 16}, sig_off[6] = {0, 15, 29, 44, 47, 0}, abs_off[6] = {0, 10, 20, 30, 39, 0};
    int last = -1;
    for (int i = 0; i < maxnum; i++) if (co[i]) last = i;
    int coded = last >= 0;
    if (cat != 5) bin(g, 85 + cbf_off[cat] + cbf_inc, coded);
    if (!coded) return 0;
    const int fld = g->mb[g->mby * g->mbw + g->mbx].field, s0 = fld ? 277 : 105, l0 = fld ? 338 : 166;
    for (int i = 0; i < maxnum - 1; i++) {
        int sc, lc;
        if (cat == 5) { sc = fld ? 436 + k_sig8x8_fld[i] : 402 + k_sig8x8[i]; lc = (fld ? 451 : 417) + k_last8x8[i]; }
        else if (cat == 3) { int inc = i < 2 ? i : 2; sc = s0 + sig_off[3] + inc; lc = l0 + sig_off[3] + inc; }
        else { sc = s0 + sig_off[cat] + i; lc = l0 + sig_off[cat] + i; }
        bin(g, sc, co[i] != 0);
        if (co[i]) { bin(g, lc, i == last); if (i == last) break; }
    }
    int eq1 = 0, gt1 = 0, absb = cat == 5 ? 426 : 227 + abs_off[cat];
    for (int i = last; i >= 0; i--) {
        if (!co[i]) continue;
        int a = abs(co[i]) - 1;
        int inc = gt1 ? 0 : (eq1 + 1 < 4 ? eq1 + 1 : 4);
        bin(g, absb + inc, a > 0);
        if (a > 0) {
            int inc2 = 5 + (gt1 < 4 - (cat == 3) ? gt1 : 4 - (cat == 3));
            int pre = a < 14 ? a : 14;
            for (int k = 1; k < pre; k++) bin(g, absb + inc2, 1);
            if (a < 14) bin(g, absb + inc2, 0);
            else {
                int s = a - 14, k = 0;
                while (s >= (1 << k)) { ce_byp(&g->ce, 1); s -= 1 << k; k++; }
                ce_byp(&g->ce, 0);
                while (k--) ce_byp(&g->ce, (s >> k) & 1);
            }
        }
        if (a == 0) eq1++; else gt1++;
        ce_byp(&g->ce, co[i] < 0);
    }
    return 1;
}

/* ------------------------------------------------------------ macroblock encode */
static int chroma_qp(int qpi) {
    static const int t[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
    return qpi < 30 ? qpi : t[qpi - 30];
}

static long var16(G *g) {
    long s = 0, s2 = 0;
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) { int v = srcv(g, 0, g->mbx * 16 + x, g->mby * 16 + y); s += v; s2 += (long)v * v; }
    return (s2 - s * s / 256) / 256;
}

/* --lossless: the inverse of the decoder's 8.5.15 accumulation (vertical: differences down each
 * column, horizontal: along each row) for horizontal / vertical intra predictions; dir 0 / 1 */
static void dpcm_diff(const int *r, int *c, int n, int dir) {
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            int v = r[y * n + x];
            if (dir == 0 && y > 0) v -= r[(y - 1) * n + x];
            if (dir == 1 && x > 0) v -= r[y * n + x - 1];
            c[y * n + x] = v;
        }
}

static void put(G *g, int c, int gx, int gy, int n, const int *pred, const int *r) {
    int maxv = (1 << g->bd) - 1;
    for (int y = 0; y < n; y++) for (int x = 0; x < n; x++) recv_put(g, c, gx + x, gy + y, clip3(0, maxv, pred[y * n + x] + r[y * n + x]));
}

static void encode_mb(G *g) {
    Mb *m = &g->mb[g->mby * g->mbw + g->mbx];
    memset(m, 0, sizeof(*m));
    m->slice = g->cur_slice;
    m->vx = g->mbx;
    m->vy = g->mby;
    m->field = g->mbaff ? g->cur_field : 0;
    const int gx = g->mbx * 16, gy = g->mby * 16;
    long v = var16(g);
    int scale = 1 << (2 * (g->bd - 8));
    int pcm = g->pcm && rndn(40) == 0;
    int is16 = !pcm && (v < (long)(g->qp * 2) * scale || rndn(12) == 0);
    int t8 = !pcm && !is16 && g->t8x8 && rndn(2);
    /* mb_type */
    Mb *A = nb(g, -1, 0), *B = nb(g, 0, -1);
    int ctx = (A && A->mb_type != 0) + (B && B->mb_type != 0);
    /* decide I16x16 mode and levels first (mb_type carries cbp) */
    int lv16[256] = {0}, lvc[2][64], pred[256], r[256], src[256];
    int mode16 = 2, qpd = 0;
    /* mb_qp_delta choice */
    int new_qp = g->cur_qp;
    if (g->qpdelta && rndn(4) == 0) new_qp = clip3(-6 * (g->bd - 8), 51, g->qp + rndn(7) - 3);
    if (pcm) {
        if (g->cavlc) {
            bw_ue(g->ce.bw, 25);
        } else {
            bin(g, 3 + ctx, 1);
            ce_term(&g->ce, 1);
            ce_finish(&g->ce);
            bw_put(g->ce.bw, 1, 1);
        }
        bw_align_zero(g->ce.bw);
        for (int y = 0; y < 16; y++) for (int x = 0; x < 16; x++) {
            int s = srcv(g, 0, gx + x, gy + y);
            bw_put(g->ce.bw, (uint32_t)s, g->bd);
            recv_put(g, 0, gx + x, gy + y, s);
        }
        for (int c = 1; c < 3; c++) for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) {
            int s = srcv(g, c, gx / 2 + x, gy / 2 + y); /* --mono: the flat chroma source, not coded */
            if (!g->mono) bw_put(g->ce.bw, (uint32_t)s, g->bd);
            recv_put(g, c, gx / 2 + x, gy / 2 + y, s);
        }
        if (!g->cavlc) { BW *bw = g->ce.bw; ce_start(&g->ce, bw); }
        m->mb_type = 25; m->qp = g->cur_qp; m->cbp = 0x2F;
        memset(m->tc, 16, sizeof(m->tc)); memset(m->tcc, 16, sizeof(m->tcc));
        memset(m->cbf, 1, 16); memset(m->cbf_c, 1, sizeof(m->cbf_c)); memset(m->cbf_dc, 1, 3);
        for (int i = 0; i < 16; i++) m->ipm[i] = 2;
        g->prev_qpd_nz = 0;
        return;
    }
    int qp_use = new_qp; /* QP used for quantisation if the MB ends up coding a delta */
    int qpl = qp_use + 6 * (g->bd - 8);
    int maxlev = 2047;
    if (is16) {
        int at = B != NULL, al = A != NULL, ad = nb(g, -1, -1) != NULL;
        long best = -1;
        for (int md = 0; md < 4; md++) {
            if ((md == 0 && !at) || (md == 1 && !al) || (md == 3 && !(at && al && ad))) continue;
            pred16(g, md, pred);
            long c = 0;
            for (int i = 0; i < 256; i++) c += abs(srcv(g, 0, gx + (i & 15), gy + (i >> 4)) - pred[i]);
            if (best < 0 || c < best) { best = c; mode16 = md; }
        }
        pred16(g, mode16, pred);
        for (int i = 0; i < 256; i++) src[i] = srcv(g, 0, gx + (i & 15), gy + (i >> 4)) - pred[i];
        if (g->lossless) {  /* transform bypass: the levels are the residual (DPCM for modes 0 / 1) */
            if (mode16 <= 1) dpcm_diff(src, lv16, 16, mode16);
            else memcpy(lv16, src, sizeof(lv16));
        } else {
            Basis *Bs = &g_b16[qpl];
            build_basis(Bs, 2, qpl, g_w4[0]);
            quantize(Bs, src, lv16, maxlev);
            fit(2, lv16, qpl, g_w4[0]);
        }
    }
    /* chroma mode + levels need the chroma QP of the final QP */
    int at = B != NULL, al = A != NULL, ad = nb(g, -1, -1) != NULL;
    int cpm = rndn(4);
    if ((cpm == 1 && !al) || (cpm == 2 && !at) || (cpm == 3 && !(at && al && ad))) cpm = 0;
    if (g->mono) cpm = 0; /* no intra_chroma_pred_mode: the flat chroma source predicts exactly */
    /* chroma residual is computed after luma (recon order doesn't matter: chroma pred uses neighbour MBs only) */
    int qpc[2];
    for (int c = 0; c < 2; c++) qpc[c] = chroma_qp(clip3(-6 * (g->bd - 8), 51, qp_use + (c ? g->cqp2 : g->cqp))) + 6 * (g->bd - 8);
    int predc_[2][64];
    for (int c = 0; c < 2; c++) {
        predc(g, 1 + c, cpm, predc_[c]);
        int x[64];
        for (int i = 0; i < 64; i++) x[i] = srcv(g, 1 + c, gx / 2 + (i & 7), gy / 2 + (i >> 3)) - predc_[c][i];
        if (g->lossless) {  /* intra_chroma_pred_mode 1 horizontal, 2 vertical */
            if (cpm == 1 || cpm == 2) dpcm_diff(x, lvc[c], 8, cpm == 2 ? 0 : 1);
            else memcpy(lvc[c], x, sizeof(x));
            continue;
        }
        Basis *Bs = &g_bc[c][qpc[c]];
        build_basis(Bs, 3, qpc[c], g_w4[1 + c]);
        quantize(Bs, x, lvc[c], maxlev);
        fit(3, lvc[c], qpc[c], g_w4[1 + c]);
        if (rndn(5) == 0) for (int i = 0; i < 64; i++) if ((i & 3) || (i >> 3) & 3) lvc[c][i] = 0; /* DC-only chroma */
    }
    int chroma_dc = 0, chroma_ac = 0;
    for (int c = 0; c < 2; c++) for (int i = 0; i < 64; i++) if (lvc[c][i]) { if ((i & 3) == 0 && ((i >> 3) & 3) == 0) chroma_dc = 1; else chroma_ac = 1; }
    int cbp_c = chroma_ac ? 2 : (chroma_dc ? 1 : 0);
    if (cbp_c < 2) for (int c = 0; c < 2; c++) for (int i = 0; i < 64; i++) if ((i & 3) || ((i >> 3) & 3)) lvc[c][i] = 0;
    if (cbp_c == 0) memset(lvc, 0, sizeof(lvc));
    if (is16) {
        int ac = 0;
        for (int i = 0; i < 256; i++) if (lv16[i] && ((i & 3) || ((i >> 4) & 3))) ac = 1;
        if (!ac) for (int i = 0; i < 256; i++) if ((i & 3) || ((i >> 4) & 3)) lv16[i] = 0;
        m->mb_type = 1 + mode16 + 4 * cbp_c + (ac ? 12 : 0);
        m->cbp = (cbp_c << 4) | (ac ? 15 : 0);
        if (g->cavlc) {
            bw_ue(g->ce.bw, (uint32_t)m->mb_type);
        } else {
            bin(g, 3 + ctx, 1);
            ce_term(&g->ce, 0);
            bin(g, 6, ac);
            bin(g, 7, cbp_c != 0);
            if (cbp_c) bin(g, 8, cbp_c == 2);
            bin(g, 9, mode16 >> 1);
            bin(g, 10, mode16 & 1);
        }
    } else {
        m->mb_type = 0;
        if (g->cavlc) {
            bw_ue(g->ce.bw, 0);
            if (g->t8x8) bw_put(g->ce.bw, (uint32_t)t8, 1);
        } else {
            bin(g, 3 + ctx, 0);
            if (g->t8x8) {
                int c8 = (A && A->t8x8) + (B && B->t8x8);
                bin(g, 399 + c8, t8);
            }
        }
        m->t8x8 = t8;
    }
    /* luma NxN: choose modes + levels block by block with reconstruction */
    int lv4[16][16], lv8[4][64];
    memset(lv4, 0, sizeof(lv4));
    memset(lv8, 0, sizeof(lv8));
    if (!is16) {
        int nblk = t8 ? 4 : 16;
        for (int i = 0; i < nblk; i++) {
            int blk = t8 ? i * 4 : i, n = t8 ? 8 : 4;
            int bx = t8 ? (i & 1) * 8 : k_blk_x[blk] * 4, by = t8 ? (i >> 1) * 8 : k_blk_y[blk] * 4;
            Nb o;
            if (t8) gather8(g, i, &o); else gather4(g, blk, &o);
            long best = -1;
            int bm = 2, p[64];
            for (int md = 0; md < 9; md++) {
                if (!mode_legal(md, &o)) continue;
                if (md > 2 && rndn(3) == 0) continue;
                predict_nxn(g, n, md, &o, p);
                long c = 0;
                for (int k = 0; k < n * n; k++) c += abs(srcv(g, 0, gx + bx + k % n, gy + by + k / n) - p[k]);
                if (best < 0 || c < best) { best = c; bm = md; }
            }
            /* signal */
            int nblkA, nblkB;
            Mb *NA = nb_blk(g, k_blk_x[blk] - 1, k_blk_y[blk], &nblkA);
            int ma = !NA ? -1 : (NA->mb_type != 0 ? 2 : NA->ipm[nblkA]);
            Mb *NB = nb_blk(g, k_blk_x[blk], k_blk_y[blk] - 1, &nblkB);
            int mb2 = !NB ? -1 : (NB->mb_type != 0 ? 2 : NB->ipm[nblkB]);
            int pm = (ma < 0 || mb2 < 0) ? 2 : (ma < mb2 ? ma : mb2);
            if (g->cavlc) {
                bw_put(g->ce.bw, bm == pm, 1);
                if (bm != pm) bw_put(g->ce.bw, (uint32_t)(bm < pm ? bm : bm - 1), 3);
            } else {
                bin(g, 68, bm == pm);
                if (bm != pm) {
                    int rem = bm < pm ? bm : bm - 1;
                    bin(g, 69, rem & 1); bin(g, 69, (rem >> 1) & 1); bin(g, 69, (rem >> 2) & 1);
                }
            }
            if (t8) for (int k = 0; k < 4; k++) m->ipm[blk + k] = (uint8_t)bm;
            else m->ipm[blk] = (uint8_t)bm;
            /* residual + recon now (later blocks predict from it) */
            predict_nxn(g, n, bm, &o, p);
            int x[64], rr[64];
            for (int k = 0; k < n * n; k++) x[k] = srcv(g, 0, gx + bx + k % n, gy + by + k / n) - p[k];
            int *lv = t8 ? lv8[i] : lv4[blk];
            if (g->lossless) {  /* transform bypass: exact reconstruction */
                if (bm <= 1) dpcm_diff(x, lv, n, bm);
                else memcpy(lv, x, sizeof(int) * (size_t)(n * n));
                memcpy(rr, x, sizeof(int) * (size_t)(n * n));
            } else {
                Basis *Bs = t8 ? &g_b8[qpl] : &g_b4[qpl];
                build_basis(Bs, t8 ? 1 : 0, qpl, t8 ? g_w8 : g_w4[0]);
                quantize(Bs, x, lv, maxlev);
                fit(t8 ? 1 : 0, lv, qpl, t8 ? g_w8 : g_w4[0]);
                if (t8) res8(lv, qpl, rr, g_w8); else res4(lv, qpl, rr, g_w4[0]);
            }
            put(g, 0, gx + bx, gy + by, n, p, rr);
        }
    }
    /* cbp for NxN */
    if (!is16) {
        int cbp = cbp_c << 4;
        for (int b8 = 0; b8 < 4; b8++) {
            int nz = 0;
            if (t8) { for (int k = 0; k < 64; k++) nz |= lv8[b8][k] != 0; }
            else for (int b4 = 0; b4 < 4; b4++) for (int k = 0; k < 16; k++) nz |= lv4[b8 * 4 + b4][k] != 0;
            cbp |= nz << b8;
        }
        m->cbp = cbp;
    }
    /* chroma pred mode (none in 4:0:0) */
    if (!g->mono) {
        int c2 = (A && A->mb_type != 25 && A->cpm != 0) + (B && B->mb_type != 25 && B->cpm != 0);
        if (g->cavlc) {
            bw_ue(g->ce.bw, (uint32_t)cpm);
        } else {
            bin(g, 64 + c2, cpm != 0);
            if (cpm) { bin(g, 67, cpm > 1); if (cpm > 1) bin(g, 67, cpm > 2); }
        }
        m->cpm = cpm;
    }
    if (!is16 && g->cavlc) {
        static const uint8_t k_gray[16] = {15, 0, 7, 11, 13, 14, 3, 5, 10, 12, 1, 2, 4, 8, 6, 9}; /* Table 9-4, 4:0:0 */
        int cn = 0;
        if (g->mono) while (k_gray[cn] != m->cbp) cn++;
        else while (kCbpIntra[cn] != m->cbp) cn++;
        bw_ue(g->ce.bw, (uint32_t)cn);
    } else if (!is16) {
        int cbp = m->cbp;
        for (int b8 = 0; b8 < 4; b8++) {
            int bx = b8 & 1, by = b8 >> 1, ca, cb;
            int xW, yW;
            Mb *N8;
            if (bx == 0) { N8 = nb_loc(g, -1, by * 8, 16, 16, &xW, &yW);
                           ca = N8 ? (N8->mb_type == 25 ? 0 : !((N8->cbp >> ((yW >> 3) * 2 + (xW >> 3))) & 1)) : 0; }
            else ca = !((cbp >> (b8 - 1)) & 1);
            if (by == 0) { N8 = nb_loc(g, bx * 8, -1, 16, 16, &xW, &yW);
                           cb = N8 ? (N8->mb_type == 25 ? 0 : !((N8->cbp >> ((yW >> 3) * 2 + (xW >> 3))) & 1)) : 0; }
            else cb = !((cbp >> (b8 - 2)) & 1);
            bin(g, 73 + ca + 2 * cb, (cbp >> b8) & 1);
        }
        int ac = A ? (A->mb_type == 25 ? 2 : (A->cbp >> 4)) : 0, bc = B ? (B->mb_type == 25 ? 2 : (B->cbp >> 4)) : 0;
        if (!g->mono) {
            bin(g, 77 + (ac > 0) + 2 * (bc > 0), cbp_c != 0);
            if (cbp_c) bin(g, 77 + 4 + (ac == 2) + 2 * (bc == 2), cbp_c == 2);
        }
    }
    /* mb_qp_delta: the levels were quantised at qp_use; if the MB codes a
     * delta it must be qp_use - cur_qp, else QP stays cur_qp (only possible
     * when nothing is coded, so the residual is zero either way) */
    if ((m->cbp & 15) || (m->cbp >> 4) || is16) {
        qpd = qp_use - g->cur_qp;
        int k = qpd > 0 ? 2 * qpd - 1 : -2 * qpd;
        int c0 = g->prev_qpd_nz ? 1 : 0;
        if (g->cavlc) {
            bw_se(g->ce.bw, qpd);
        } else {
            bin(g, 60 + c0, k > 0);
            if (k > 0) {
                for (int i = 1; i < k; i++) bin(g, 60 + (i == 1 ? 2 : 3), 1);
                bin(g, 60 + (k == 1 ? 2 : 3), 0);
            }
        }
        g->cur_qp = qp_use;
    } else if (qp_use != g->cur_qp) {
        /* nothing coded: re-encode impossible; residual is all zero so recon matches */
    }
    g->prev_qpd_nz = qpd != 0;
    m->qp = g->cur_qp;
    /* residual syntax (field MBs: field scans) */
    int co[64];
    const uint8_t *z4 = m->field ? k_fld4 : k_zz4, *z8 = m->field ? k_fld8 : k_zz8;
    if (is16) {
        for (int k = 0; k < 16; k++) { int rr = z4[k]; co[k] = lv16[(rr >> 2) * 4 * 16 + (rr & 3) * 4]; }
        if (g->cavlc) enc_block_cavlc(g, nc_luma(g, 0), 16, co);
        else m->cbf_dc[0] = (uint8_t)enc_block(g, 0, cbf_cond(0, A, 0, 0) + 2 * cbf_cond(0, B, 0, 0), 16, co);
    }
    for (int b8 = 0; b8 < 4; b8++) {
        if (!((m->cbp >> b8) & 1)) continue;
        if (t8 && g->cavlc) {
            for (int i4 = 0; i4 < 4; i4++) {
                for (int k = 0; k < 16; k++) co[k] = lv8[b8][z8[4 * k + i4]];
                m->tc[b8 * 4 + i4] = (uint8_t)enc_block_cavlc(g, nc_luma(g, b8 * 4 + i4), 16, co);
            }
            continue;
        }
        if (t8) {
            for (int k = 0; k < 64; k++) co[k] = lv8[b8][z8[k]];
            enc_block(g, 5, 0, 64, co);
            for (int k = 0; k < 4; k++) m->cbf[b8 * 4 + k] = 1;
            continue;
        }
        for (int b4 = 0; b4 < 4; b4++) {
            int blk = b8 * 4 + b4, bx = k_blk_x[blk], by = k_blk_y[blk], nb1;
            Mb *NA = nb_blk(g, bx - 1, by, &nb1);
            int ca = cbf_cond(is16 ? 1 : 2, NA, nb1, 0);
            Mb *NB = nb_blk(g, bx, by - 1, &nb1);
            int cb = cbf_cond(is16 ? 1 : 2, NB, nb1, 0);
            if (is16) {
                for (int k = 0; k < 15; k++) { int rr = z4[k + 1]; co[k] = lv16[(by * 4 + (rr >> 2)) * 16 + bx * 4 + (rr & 3)]; }
                if (g->cavlc) m->tc[blk] = (uint8_t)enc_block_cavlc(g, nc_luma(g, blk), 15, co);
                else m->cbf[blk] = (uint8_t)enc_block(g, 1, ca + 2 * cb, 15, co);
            } else {
                for (int k = 0; k < 16; k++) co[k] = lv4[blk][z4[k]];
                if (g->cavlc) m->tc[blk] = (uint8_t)enc_block_cavlc(g, nc_luma(g, blk), 16, co);
                else m->cbf[blk] = (uint8_t)enc_block(g, 2, ca + 2 * cb, 16, co);
            }
        }
    }
    if (m->cbp >> 4) {
        for (int c = 0; c < 2; c++) {
            for (int k = 0; k < 4; k++) co[k] = lvc[c][(k >> 1) * 4 * 8 + (k & 1) * 4];
            if (g->cavlc) enc_block_cavlc(g, -1, 4, co);
            else m->cbf_dc[1 + c] = (uint8_t)enc_block(g, 3, cbf_cond(3, A, 0, c) + 2 * cbf_cond(3, B, 0, c), 4, co);
        }
    }
    if ((m->cbp >> 4) == 2) {
        for (int c = 0; c < 2; c++)
            for (int b4 = 0; b4 < 4; b4++) {
                int bx = b4 & 1, by = b4 >> 1;
                int xW, yW, ca, cb;
                if (bx) ca = m->cbf_c[c][b4 - 1];
                else { Mb *N = nb_loc(g, -1, by * 4, 8, 8, &xW, &yW); ca = cbf_cond(4, N, N ? (yW >> 2) * 2 + (xW >> 2) : 0, c); }
                if (by) cb = m->cbf_c[c][b4 - 2];
                else { Mb *N = nb_loc(g, bx * 4, -1, 8, 8, &xW, &yW); cb = cbf_cond(4, N, N ? (yW >> 2) * 2 + (xW >> 2) : 0, c); }
                for (int k = 0; k < 15; k++) { int rr = z4[k + 1]; co[k] = lvc[c][(by * 4 + (rr >> 2)) * 8 + bx * 4 + (rr & 3)]; }
                if (g->cavlc) m->tcc[c][b4] = (uint8_t)enc_block_cavlc(g, nc_chroma(g, m, c, b4), 15, co);
                else m->cbf_c[c][b4] = (uint8_t)enc_block(g, 4, ca + 2 * cb, 15, co);
            }
    }
    /* reconstruction of I16x16 luma and chroma */
    if (is16) {
        pred16(g, mode16, pred);
        if (g->lossless) for (int i = 0; i < 256; i++) r[i] = srcv(g, 0, gx + (i & 15), gy + (i >> 4)) - pred[i];
        else res_dc(lv16, 16, qpl, r, g_w4[0]);
        put(g, 0, gx, gy, 16, pred, r);
    }
    for (int c = 0; c < 2; c++) {
        int rr[64];
        if (g->lossless) for (int i = 0; i < 64; i++) rr[i] = srcv(g, 1 + c, gx / 2 + (i & 7), gy / 2 + (i >> 3)) - predc_[c][i];
        else res_dc(lvc[c], 8, qpc[c], rr, g_w4[1 + c]);
        put(g, 1 + c, gx / 2, gy / 2, 8, predc_[c], rr);
    }
    if (!is16) for (int i = 0; i < 16; i++) if (t8) {} /* ipm already set */
    if (is16) for (int i = 0; i < 16; i++) m->ipm[i] = 2;
}

/* ------------------------------------------------------------ scaling matrices (7.3.2.1.1.1) */
/* --sm: 0 none; 1 SPS matrices (fall-back rule A); 2 SPS matrices + PPS matrices (fall-back
 * rule B); 3 PPS matrices only (fall-back rule A in the PPS).  Each list is, at random: not
 * present (fall-back), useDefaultScalingMatrixFlag (first delta gives 0), or DPCM-coded values,
 * sometimes ended early by a 0 (the rest repeats the last value). */
static const uint8_t k_def4[2][16] = {{6, 13, 13, 20, 20, 20, 28, 28, 28, 28, 32, 32, 32, 37, 37, 42},
                                      {10, 14, 14, 20, 20, 20, 24, 24, 24, 24, 27, 27, 27, 30, 30, 34}};
static const uint8_t k_def8[2][64] = {
    {6,  10, 10, 13, 11, 13, 16, 16, 16, 16, 18, 18, 18, 18, 18, 23, 23, 23, 23, 23, 23, 25,
     25, 25, 25, 25, 25, 25, 27, 27, 27, 27, 27, 27, 27, 27, 29, 29, 29, 29, 29, 29, 29, 31,
     31, 31, 31, 31, 31, 33, 33, 33, 33, 33, 36, 36, 36, 36, 38, 38, 38, 40, 40, 42},
    {9,  13, 13, 15, 13, 15, 17, 17, 17, 17, 19, 19, 19, 19, 19, 21, 21, 21, 21, 21, 21, 22,
     22, 22, 22, 22, 22, 22, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 27,
     27, 27, 27, 27, 27, 28, 28, 28, 28, 28, 30, 30, 30, 30, 32, 32, 32, 33, 33, 35}};
typedef struct { uint8_t l4[6][16], l8[2][64]; } Mat; /* scan (zig-zag) order */
static Mat g_sps_m, g_pps_m;
static int g_sps_m_on;

static void write_list(BW *b, uint8_t *list, int n, const uint8_t *def) {
    int r = rndn(8);
    if (r == 0) { bw_se(b, -8); memcpy(list, def, (size_t)n); return; } /* useDefaultScalingMatrixFlag */
    const int wild = r == 1, base = 6 + rndn(24), slope = rndn(4), stop = rndn(3) == 0 ? 1 + rndn(n - 1) : n;
    int last = 8;
    for (int j = 0; j < n; j++) {
        if (j == stop) { /* nextScale 0: the rest repeats lastScale */
            int d = -last;
            if (d < -128) d += 256;
            bw_se(b, d);
            for (; j < n; j++) list[j] = (uint8_t)last;
            return;
        }
        int v = wild ? 1 + rndn(255) : clip3(1, 255, base + slope * j * (n == 16 ? 2 : 1) / 2 + rndn(5) - 2);
        int d = v - last;
        if (d > 127) d -= 256;
        if (d < -128) d += 256;
        bw_se(b, d);
        list[j] = (uint8_t)v;
        last = v;
    }
}
/* scaling lists 0..5 (4x4) and 6..6+n8-1 (8x8); fb = fall-back rule B source (NULL: rule A) */
static void write_matrices(BW *b, Mat *M, const Mat *fb, int n8) {
    for (int i = 0; i < 6; i++) {
        int pres = rndn(3) != 0;
        bw_put(b, (uint32_t)pres, 1);
        if (pres) write_list(b, M->l4[i], 16, k_def4[i >= 3]);
        else if (i == 0 || i == 3) memcpy(M->l4[i], fb ? fb->l4[i] : k_def4[i >= 3], 16);
        else memcpy(M->l4[i], M->l4[i - 1], 16);
    }
    for (int i = 0; i < n8; i++) {
        int pres = rndn(3) != 0;
        bw_put(b, (uint32_t)pres, 1);
        if (pres) write_list(b, M->l8[i], 64, k_def8[i]);
        else memcpy(M->l8[i], fb ? fb->l8[i] : k_def8[i], 64);
    }
}
static void set_weights(const Mat *M) {
    for (int c = 0; c < 3; c++)
        for (int k = 0; k < 16; k++) g_w4[c][k_zz4[k]] = M ? M->l4[c][k] : 16;
    for (int k = 0; k < 64; k++) g_w8[k_zz8[k]] = M ? M->l8[0][k] : 16;
}

/* ------------------------------------------------------------ parameter sets */
static void write_sps(FILE *f, G *g, int profile) {
    BW b; bw_init(&b);
    bw_put(&b, (uint32_t)profile, 8);
    bw_put(&b, 0, 8);
    bw_put(&b, 40, 8);
    bw_ue(&b, 0);
    if (profile >= 100) {
        bw_ue(&b, g->mono ? 0 : 1); /* chroma_format_idc */
        bw_ue(&b, (uint32_t)(g->bd - 8)); bw_ue(&b, (uint32_t)(g->bd - 8));
        bw_put(&b, (uint32_t)g->lossless, 1); /* qpprime_y_zero_transform_bypass_flag (--lossless) */
        g_sps_m_on = g->sm == 1 || g->sm == 2;
        bw_put(&b, (uint32_t)g_sps_m_on, 1); /* seq_scaling_matrix_present_flag */
        if (g_sps_m_on) write_matrices(&b, &g_sps_m, NULL, 2);
    }
    set_weights(g_sps_m_on ? &g_sps_m : NULL);
    bw_ue(&b, 0);     /* log2_max_frame_num - 4 */
    bw_ue(&b, 0);     /* poc type 0 */
    bw_ue(&b, 0);     /* log2_max_poc_lsb - 4 */
    bw_ue(&b, 1);     /* max_num_ref_frames */
    bw_put(&b, 0, 1);
    bw_ue(&b, (uint32_t)(g->mbw - 1));
    /* --ilsps 1: an interlace-capable SPS (frame_mbs_only_flag 0, mb_adaptive_frame_field_flag 0)
     * coding a frame picture: the height is sent in field MB rows (map units) and the vertical
     * crop in units of 4 rows (7.4.2.1.1) */
    bw_ue(&b, (uint32_t)(g->ilsps ? g->mbh / 2 - 1 : g->mbh - 1));
    bw_put(&b, (uint32_t)!g->ilsps, 1); /* frame_mbs_only */
    if (g->ilsps) bw_put(&b, (uint32_t)(g->mbaff && !g->paff), 1); /* mb_adaptive_frame_field_flag (--mbaff: MBAFF frame) */
    bw_put(&b, 1, 1); /* direct_8x8_inference */
    int crop = g->outW != g->W || g->outH != g->H;
    if (g->rawcrop[0] >= 0) { /* --crop l,r,t,b: raw frame_crop offsets (malformed-SPS vectors) */
        bw_put(&b, 1, 1);
        for (int i = 0; i < 4; i++) bw_ue(&b, (uint32_t)g->rawcrop[i]);
    } else {
        bw_put(&b, (uint32_t)crop, 1);
        /* CropUnitX / CropUnitY: 2 / 2 (2 - frame_mbs_only) in 4:2:0, 1 / 2 - frame_mbs_only in 4:0:0 */
        const int ux = g->mono ? 1 : 2, uy = (g->mono ? 1 : 2) * (g->ilsps ? 2 : 1);
        if (crop) { bw_ue(&b, 0); bw_ue(&b, (uint32_t)(g->W - g->outW) / ux); bw_ue(&b, 0); bw_ue(&b, (uint32_t)(g->H - g->outH) / uy); }
    }
    /* --vuireorder K: the VUI's reorder depth alone (no extra pictures; malformed-SPS vectors use
     * K > 16); --vuicpb K: a NAL HRD with cpb_cnt_minus1 = K (K > 31 is malformed) */
    const int reorder = g->vuireorder >= 0 ? g->vuireorder : g->delay;
    const int vui = g->delay > 0 || g->vuireorder >= 0 || g->vuicpb >= 0;
    bw_put(&b, (uint32_t)vui, 1); /* vui_parameters_present_flag */
    if (vui) { /* E.1.1: bitstream_restriction carrying the reorder depth (+ an optional NAL HRD) */
        bw_put(&b, 0, 5);       /* aspect, overscan, video signal, chroma loc, timing */
        bw_put(&b, g->vuicpb >= 0, 1); /* nal_hrd_parameters_present_flag */
        if (g->vuicpb >= 0) {   /* E.1.2 */
            bw_ue(&b, (uint32_t)g->vuicpb);
            bw_put(&b, 0, 8);   /* bit_rate_scale, cpb_size_scale */
            for (int i = 0; i <= g->vuicpb && i < 40; i++) { bw_ue(&b, 1000); bw_ue(&b, 1000); bw_put(&b, 0, 1); }
            bw_put(&b, 0x5AD6B, 20); /* four 5-bit lengths */
        }
        bw_put(&b, 0, 1);       /* vcl_hrd_parameters_present_flag */
        if (g->vuicpb >= 0) bw_put(&b, 0, 1); /* low_delay_hrd_flag */
        bw_put(&b, 0, 1);       /* pic_struct_present_flag */
        bw_put(&b, 1, 1);       /* bitstream_restriction_flag */
        bw_put(&b, 1, 1);       /* motion_vectors_over_pic_boundaries_flag */
        bw_ue(&b, 0); bw_ue(&b, 0); bw_ue(&b, 15); bw_ue(&b, 15);
        bw_ue(&b, (uint32_t)reorder);     /* max_num_reorder_frames */
        bw_ue(&b, (uint32_t)reorder + 1); /* max_dec_frame_buffering */
    }
    bw_trailing(&b);
    write_nal(f, 3, 7, b.buf, b.n);
    free(b.buf);
}
static void write_pps(FILE *f, G *g, int high, int id) {
    BW b; bw_init(&b);
    bw_ue(&b, (uint32_t)id); bw_ue(&b, 0);
    bw_put(&b, (uint32_t)(!g->cavlc && id == 0), 1); /* entropy_coding_mode_flag (PPS 1: CAVLC skip pictures) */
    bw_put(&b, 0, 1);
    bw_ue(&b, 0);     /* slice groups */
    bw_ue(&b, 0); bw_ue(&b, 0);
    bw_put(&b, 0, 1); bw_put(&b, 0, 2);
    bw_se(&b, 0);     /* init qp 26 */
    bw_se(&b, 0);
    bw_se(&b, g->cqp);
    bw_put(&b, 1, 1); /* deblocking filter control present */
    bw_put(&b, 0, 1); /* constrained intra */
    bw_put(&b, 0, 1); /* redundant pic cnt */
    if (high) {
        bw_put(&b, (uint32_t)g->t8x8, 1);
        int pm = g->sm >= 2;
        bw_put(&b, (uint32_t)pm, 1); /* pic_scaling_matrix_present_flag */
        if (pm) {
            g_pps_m = g_sps_m; /* 8x8 lists stay the SPS ones without transform_8x8_mode */
            if (!g_sps_m_on) for (int i = 0; i < 2; i++) memset(g_pps_m.l8[i], 16, 64);
            write_matrices(&b, &g_pps_m, g_sps_m_on ? &g_sps_m : NULL, g->t8x8 ? 2 : 0);
            set_weights(&g_pps_m);
        }
        bw_se(&b, g->cqp2);
    }
    bw_trailing(&b);
    write_nal(f, 3, 8, b.buf, b.n);
    free(b.buf);
}

static int opt_int(int argc, char **argv, const char *n, int d) { for (int i = 1; i + 1 < argc; i++) if (!strcmp(argv[i], n)) return atoi(argv[i + 1]); return d; }
static const char *opt_str(int argc, char **argv, const char *n) { for (int i = 1; i + 1 < argc; i++) if (!strcmp(argv[i], n)) return argv[i + 1]; return NULL; }

int main(int argc, char **argv) {
    if (argc < 8) { fprintf(stderr, "usage: h264gen in.yuv W H bitdepth qp seed out.h264 [options]\n"); return 2; }
    G *g = (G *)calloc(1, sizeof(G));
    g->outW = atoi(argv[2]); g->outH = atoi(argv[3]); g->bd = atoi(argv[4]); g->qp = atoi(argv[5]);
    g_rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)atoll(argv[6]) * 0x100000001B3ull;
    g->t8x8 = opt_int(argc, argv, "--t8x8", 1);
    g->pcm = opt_int(argc, argv, "--pcm", 0);
    g->qpdelta = opt_int(argc, argv, "--qpdelta", 1);
    g->slice_rows = opt_int(argc, argv, "--slices", 0);
    g->alpha = opt_int(argc, argv, "--alpha", 0);
    g->beta = opt_int(argc, argv, "--beta", 0);
    g->dbidc = opt_int(argc, argv, "--dbidc", 0);
    g->cqp = opt_int(argc, argv, "--cqp", 0);
    g->cqp2 = opt_int(argc, argv, "--cqp2", g->cqp);
    g->cavlc = opt_int(argc, argv, "--cavlc", 0);
    g->sm = opt_int(argc, argv, "--sm", 0);
    g->nonidr = opt_int(argc, argv, "--nonidr", 0);
    g->delay = opt_int(argc, argv, "--delay", 0);
    g->firstmb = opt_int(argc, argv, "--firstmb", -1);
    g->vuireorder = opt_int(argc, argv, "--vuireorder", -1);
    g->vuicpb = opt_int(argc, argv, "--vuicpb", -1);
    g->ilsps = opt_int(argc, argv, "--ilsps", 0);
    /* --mbaff 1: an MBAFF frame (frame_mbs_only_flag 0, mb_adaptive_frame_field_flag 1): macroblock
     * pairs, each coded as two frame or two field macroblocks (random per pair, --fieldpct % field) */
    g->mbaff = opt_int(argc, argv, "--mbaff", 0);
    if (g->mbaff) g->ilsps = 1;
    int fieldpct = opt_int(argc, argv, "--fieldpct", 50);
    /* --paff 1: a field pair (field_pic_flag 1): the first field an IDR (or --nonidr) I field, the
     * second field (the other parity, nal type 1) an I field; --paff 2: bottom field first.  Held
     * like an MBAFF frame of field pairs: field MB (x, fy) of parity f at grid (x, 2 fy + f) */
    g->paff = opt_int(argc, argv, "--paff", 0);
    if (g->paff) g->mbaff = g->ilsps = 1;
    g->onefield = opt_int(argc, argv, "--onefield", 0); /* --paff with the first field only (malformed) */
    /* --lossless 1: High 4:4:4 Predictive (profile_idc 244) with qpprime_y_zero_transform_bypass_flag,
     * every macroblock at QP'Y 0 (TransformBypassModeFlag), residual DPCM for H / V predictions */
    g->lossless = opt_int(argc, argv, "--lossless", 0);
    g->mono = opt_int(argc, argv, "--mono", 0);
    if (g->lossless) { g->qp = -6 * (g->bd - 8); g->qpdelta = 0; }
    g->rawcrop[0] = -1;
    if (opt_str(argc, argv, "--crop"))
        sscanf(opt_str(argc, argv, "--crop"), "%lld,%lld,%lld,%lld", &g->rawcrop[0], &g->rawcrop[1], &g->rawcrop[2], &g->rawcrop[3]);
    if (g->delay > 6) { fprintf(stderr, "--delay <= 6 (4-bit POC lsb)\n"); return 2; }
    int profile = opt_int(argc, argv, "--profile", (g->lossless || g->bd > 10) ? 244 : g->bd > 8 ? 110 : (g->t8x8 || g->cqp2 != g->cqp || g->sm || g->mono ? 100 : 77));
    g_lim = 1 << (7 + g->bd);
    g->W = (g->outW + 15) & ~15; g->H = g->ilsps ? (g->outH + 31) & ~31 : (g->outH + 15) & ~15;
    if (g->ilsps && (g->H - g->outH) % 4) { fprintf(stderr, "--ilsps: the height must crop in 4-row units\n"); return 2; }
    g->mbw = g->W / 16; g->mbh = g->H / 16;
    FILE *fi = fopen(argv[1], "rb");
    if (!fi) { perror("input"); return 1; }
    for (int c = 0; c < 3; c++) {
        int w = c ? g->W / 2 : g->W, h = c ? g->H / 2 : g->H, iw = c ? g->outW / 2 : g->outW, ih = c ? g->outH / 2 : g->outH;
        g->st[c] = w;
        g->src[c] = (uint16_t *)calloc((size_t)w * h, 2);
        g->rec[c] = (uint16_t *)calloc((size_t)w * h, 2);
        for (int y = 0; y < ih; y++) for (int x = 0; x < iw; x++) {
            int v = g->bd == 8 ? fgetc(fi) : (fgetc(fi) | (fgetc(fi) << 8));
            g->src[c][y * w + x] = (uint16_t)(v < 0 ? 0 : v);
        }
        for (int y = 0; y < h; y++) for (int x = 0; x < w; x++) g->src[c][y * w + x] = g->src[c][(y < ih ? y : ih - 1) * w + (x < iw ? x : iw - 1)];
        if (c && g->mono) for (int i = 0; i < w * h; i++) g->src[c][i] = (uint16_t)(1 << (g->bd - 1));
    }
    fclose(fi);
    g->mb = (Mb *)calloc((size_t)g->mbw * g->mbh, sizeof(Mb));
    for (int i = 0; i < g->mbw * g->mbh; i++) g->mb[i].slice = -1;
    FILE *fo = fopen(argv[7], "wb");
    write_sps(fo, g, profile);
    write_pps(fo, g, profile >= 100, 0);
    if (g->delay) write_pps(fo, g, 0, 1);
    const int fh = g->paff ? g->mbh / 2 : g->mbh; /* MB rows per coded picture (--paff: per field) */
    int rows = g->slice_rows > 0 ? g->slice_rows : fh;
    if (g->mbaff && !g->paff) rows = (rows + 1) & ~1; /* slices start at pair rows */
    int nslice = 0;
    for (int fld = 0; fld < (g->paff ? 2 - g->onefield : 1); fld++) {
    const int par = fld ^ (g->paff == 2), idr = !g->nonidr && fld == 0;
    for (int r0 = 0; r0 < fh; r0 += rows, nslice++) {
        BW b; bw_init(&b);
        bw_ue(&b, (uint32_t)(r0 == 0 && g->firstmb >= 0 ? g->firstmb : (g->mbaff && !g->paff ? r0 / 2 : r0) * g->mbw)); /* first_mb (MBAFF: pair index; --firstmb: malformed) */
        bw_ue(&b, 7);                         /* I (all slices I) */
        bw_ue(&b, 0);                         /* pps */
        bw_put(&b, 0, 4);                     /* frame_num */
        if (g->ilsps) bw_put(&b, (uint32_t)!!g->paff, 1); /* field_pic_flag */
        if (g->paff) bw_put(&b, (uint32_t)par, 1);        /* bottom_field_flag */
        if (idr) bw_ue(&b, 0);                /* idr_pic_id */
        bw_put(&b, (uint32_t)fld, 4);         /* poc lsb */
        if (idr) { bw_put(&b, 0, 1); bw_put(&b, 0, 1); } /* dec_ref_pic_marking (IDR) */
        else bw_put(&b, 0, 1);                /* adaptive_ref_pic_marking_mode_flag */
        int sqp = clip3(-6 * (g->bd - 8), 51, g->qp + (nslice && !g->lossless ? rndn(5) - 2 : 0));
        bw_se(&b, sqp - 26);
        int idc = g->dbidc;
        bw_ue(&b, (uint32_t)idc);
        if (idc != 1) { bw_se(&b, g->alpha); bw_se(&b, g->beta); }
        if (!g->cavlc) while (b.nb) bw_put(&b, 1, 1);  /* cabac_alignment_one_bit */
        for (int i = 0; i < 460; i++) {
            int mm = k_init_I[i][0], nn = k_init_I[i][1];
            int pre = clip3(1, 126, ((mm * clip3(0, 51, sqp)) >> 4) + nn), mps = pre <= 63 ? 0 : 1;
            g->ctx[i] = (uint8_t)(((mps ? pre - 64 : 63 - pre) << 1) | mps);
        }
        ce_start(&g->ce, &b);
        g->cur_slice = nslice;
        g->cur_qp = sqp;
        g->prev_qpd_nz = 0;
        int r1 = r0 + rows < fh ? r0 + rows : fh;
        if (g->paff) { /* field MBs in raster order of the field */
            for (int my = r0; my < r1; my++)
                for (int mx = 0; mx < g->mbw; mx++) {
                    g->mbx = mx; g->mby = 2 * my + par;
                    g->mb[g->mby * g->mbw + mx].slice = nslice;
                    g->cur_field = 1;
                    encode_mb(g);
                    if (!g->cavlc) ce_term(&g->ce, my == r1 - 1 && mx == g->mbw - 1);
                }
        } else if (g->mbaff) { /* pairs in raster order, top MB then bottom MB (7.3.4) */
            for (int pr = r0 / 2; pr < r1 / 2; pr++)
                for (int mx = 0; mx < g->mbw; mx++)
                    for (int bt = 0; bt < 2; bt++) {
                        g->mbx = mx; g->mby = 2 * pr + bt;
                        g->mb[g->mby * g->mbw + mx].slice = nslice;
                        if (!bt) { /* mb_field_decoding_flag: ctxIdx 70 + left / upper pair are field pairs */
                            g->cur_field = rndn(100) < fieldpct;
                            Mb *PA = mb_in_slice(g, mx - 1, 2 * pr), *PB = mb_in_slice(g, mx, 2 * pr - 2);
                            if (g->cavlc) bw_put(g->ce.bw, (uint32_t)g->cur_field, 1);
                            else bin(g, 70 + (PA && PA->field) + (PB && PB->field), g->cur_field);
                        }
                        encode_mb(g);
                        if (!g->cavlc) ce_term(&g->ce, pr == r1 / 2 - 1 && mx == g->mbw - 1 && bt == 1);
                    }
        } else
        for (int my = r0; my < r1; my++)
            for (int mx = 0; mx < g->mbw; mx++) {
                g->mbx = mx; g->mby = my;
                g->mb[my * g->mbw + mx].slice = nslice;
                encode_mb(g);
                if (!g->cavlc) ce_term(&g->ce, my == r1 - 1 && mx == g->mbw - 1);
            }
        if (!g->cavlc) ce_finish(&g->ce);
        bw_put(&b, 1, 1);
        bw_align_zero(&b);
        write_nal(fo, 3, idr ? 5 : 1, b.buf, b.n);
        free(b.buf);
    }
    }
    /* decoder delay: delay + 1 all-skip P pictures (CAVLC, PPS 1), output order != decoding order:
     * frame_num 1, 2, ..., POC 2(delay+1), 2, 4, ... */
    for (int k = 1; g->delay && k <= g->delay + 1; k++) {
        BW b; bw_init(&b);
        bw_ue(&b, 0);                                   /* first_mb_in_slice */
        bw_ue(&b, 5);                                   /* P (all slices) */
        bw_ue(&b, 1);                                   /* pps 1 */
        bw_put(&b, (uint32_t)k, 4);                     /* frame_num */
        bw_put(&b, (uint32_t)(k == 1 ? 2 * (g->delay + 1) : 2 * (k - 1)), 4); /* poc lsb */
        bw_put(&b, 0, 1);                               /* num_ref_idx_active_override_flag */
        bw_put(&b, 0, 1);                               /* ref_pic_list_modification_flag_l0 */
        bw_put(&b, 0, 1);                               /* adaptive_ref_pic_marking_mode_flag */
        bw_se(&b, 0);                                   /* slice_qp_delta */
        bw_ue(&b, 0); bw_se(&b, 0); bw_se(&b, 0);       /* deblocking */
        bw_ue(&b, (uint32_t)(g->mbw * g->mbh));         /* mb_skip_run: the whole picture */
        bw_trailing(&b);
        write_nal(fo, 2, 1, b.buf, b.n);
        free(b.buf);
    }
    fclose(fo);
    const char *rp = opt_str(argc, argv, "--recon");
    if (rp) {
        FILE *fr = fopen(rp, "wb");
        for (int c = 0; c < 3; c++) {
            int iw = c ? g->outW / 2 : g->outW, ih = c ? g->outH / 2 : g->outH;
            for (int y = 0; y < ih; y++) for (int x = 0; x < iw; x++) {
                uint16_t v = g->rec[c][y * g->st[c] + x];
                if (g->bd == 8) fputc(v, fr); else { fputc(v & 255, fr); fputc(v >> 8, fr); }
            }
        }
        fclose(fr);
    }
    return 0;
}
