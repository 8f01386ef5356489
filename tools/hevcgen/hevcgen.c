/*
 * hevcgen — deterministic HEVC (H.265 Main / Main10, 4:2:0) all-intra
 * still-picture ENCODER used only to mint test vectors and benchmark inputs
 * (the container has no HEVC encoder; the reference's
 * lib/ffmpeg/x86_64_static/libx265.a is a missing blob).  Test
 * infrastructure: never linked into the product.
 *
 * Produces one IDR picture: VPS + SPS + PPS + N slices.  Decisions are
 * heuristic (variance-driven CU split, SAD intra mode search, scalar
 * quantisation) with seeded random choices that exercise the syntax the
 * decoder must handle: CU 8..64, NxN, TU split depth, transform_skip,
 * cu_qp_delta, sign data hiding, SAO band/edge/merge, PCM, transquant
 * bypass, multiple slices, deblocking offsets.  The encoder's own
 * reconstruction is written out (--recon) so tests can check that the
 * oracle decoder reproduces it bit-exactly.
 *
 * usage: hevcgen in.yuv W H bitdepth qp seed out.h265 [options]
 *   input: planar 4:2:0, 8-bit (1 B/sample) or >8-bit (2 B LE/sample)
 *   options: --sdh 0|1 --tskip 0|1 --qpdelta 0|1 --sao 0|1 --pcm 0|1
 *            --bypass 0|1 --slices N(ctb rows per slice, 0=one)
 *            --depth D (max_transform_hierarchy_depth_intra) --ctb 16|32|64
 *            --beta B --tc T --recon out.yuv --cbqp N --crqp N
 *            --sl 0..4 (scaling lists, see write_scaling_list_data)
 *   range extensions (H.265 v2): --profile P (general_profile_idc; default 1 / 2 / 4 for
 *            8 / 10 / other bit depths), --vui 1 (a VUI with HRD parameters),
 *            --rext MASK (sps_range_extension flags: 1 transform_skip_rotation, 2
 *            transform_skip_context, 4 implicit_rdpcm, 8 explicit_rdpcm, 16
 *            extended_precision_processing, 32 intra_smoothing_disabled, 64
 *            high_precision_offsets, 128 persistent_rice_adaptation, 256
 *            cabac_bypass_alignment), --maxts L (log2_max_transform_skip_block_size),
 *            --saoscale L,C (log2_sao_offset_scale luma, chroma), --cqo 1|2 (chroma QP offset
 *            list in the PPS; 2: also enabled in the slice header, so every chroma QP offset
 *            group codes cu_chroma_qp_offset_flag / _idx with a random choice), --cqolist
 *            cb0,cr0[,cb1,cr1...] (up to 6 pairs; default -2,3,4,-1), --cqodepth D
 *            (diff_cu_chroma_qp_offset_depth, default 1), --ppsext 1 (write the
 *            pps_range_extension even when the profile is not RExt: decoders then ignore it)
 *   The encoder uses the tools as the decoder will see them.  extended_precision_processing and
 *   cabac_bypass_alignment are written but coded as FFmpeg 4.3 decodes them (as if 0: "not yet
 *   implemented"); with extended precision the level escapes stay short enough that the spec's
 *   limited EGk reads them the same way (checked: the encoder stops otherwise).  A chroma QP
 *   offset index equal to chroma_qp_offset_list_len_minus1 < 5 is never coded: FFmpeg 4.3 reads the
 *   index with cMax 5 whatever the list length, the spec with cMax len_minus1.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/bits.h"
#include "../../oracle/cabac_tables.h"

/* ------------------------------------------------------------ rng */
static uint64_t g_rng = 1;
static uint32_t rnd(void) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (uint32_t)(g_rng >> 11);
}
static int rndn(int n) { return (int)(rnd() % (uint32_t)n); }

/* ------------------------------------------------------------ bit writer */
typedef struct {
    uint8_t *buf;
    size_t cap, n; /* bytes */
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
static void bw_trailing(BW *b) {
    bw_put(b, 1, 1);
    while (b->nb) bw_put(b, 0, 1);
}
static void bw_align_zero(BW *b) { while (b->nb) bw_put(b, 0, 1); }

/* NAL with emulation prevention */
static void write_nal(FILE *f, int type, const uint8_t *p, size_t n) {
    static const uint8_t sc[4] = {0, 0, 0, 1};
    fwrite(sc, 1, 4, f);
    uint8_t h[2] = {(uint8_t)(type << 1), 1};
    fwrite(h, 1, 2, f);
    int zeros = 0;
    for (size_t i = 0; i < n; i++) {
        if (zeros >= 2 && p[i] <= 3) {
            uint8_t e = 3;
            fwrite(&e, 1, 1, f);
            zeros = 0;
        }
        fwrite(&p[i], 1, 1, f);
        zeros = p[i] == 0 ? zeros + 1 : 0;
    }
}

/* ------------------------------------------------------------ CABAC encoder (HM style) */
typedef struct {
    BW *bw;
    uint32_t low, range;
    int bits_left, nbuf;
    uint32_t bufbyte;
} Enc;
static void ce_start(Enc *e, BW *bw) {
    e->bw = bw; e->low = 0; e->range = 510; e->bits_left = 23; e->nbuf = 0; e->bufbyte = 0xff;
}
static void ce_writeout(Enc *e) {
    uint32_t lead = e->low >> (24 - e->bits_left);
    e->bits_left += 8;
    e->low &= 0xffffffffu >> e->bits_left;
    if (lead == 0xff) {
        e->nbuf++;
    } else {
        if (e->nbuf > 0) {
            uint32_t carry = lead >> 8;
            uint32_t byte = e->bufbyte + carry;
            e->bufbyte = lead & 0xff;
            bw_put(e->bw, byte, 8);
            byte = (0xff + carry) & 0xff;
            while (e->nbuf > 1) { bw_put(e->bw, byte, 8); e->nbuf--; }
        } else {
            e->nbuf = 1;
            e->bufbyte = lead;
        }
    }
}
static void ce_test(Enc *e) { if (e->bits_left < 12) ce_writeout(e); }
static const uint8_t k_renorm[32] = {6, 5, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
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
static void ce_byp(Enc *e, int bin) {
    e->low <<= 1;
    if (bin) e->low += e->range;
    e->bits_left--;
    ce_test(e);
}
static void ce_bypn(Enc *e, uint32_t v, int n) { for (int i = n - 1; i >= 0; i--) ce_byp(e, (v >> i) & 1); }
static void ce_term(Enc *e, int bin) {
    e->range -= 2;
    if (bin) {
        e->low += e->range;
        e->low <<= 7;
        e->range = 2 << 7;
        e->bits_left -= 7;
    } else if (e->range >= 256) {
        return;
    } else {
        e->low <<= 1;
        e->range <<= 1;
        e->bits_left--;
    }
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

/* ------------------------------------------------------------ contexts (same layout as the oracle) */
enum {
    C_SAO_MERGE = 0, C_SAO_TYPE = 1, C_SPLIT_CU = 2, C_TQ_BYPASS = 5, C_PART_MODE = 6, C_PREV_INTRA = 7,
    C_CHROMA_MODE = 8, C_SPLIT_TF = 9, C_CBF_LUMA = 12, C_CBF_CHROMA = 14, C_TSKIP = 18, C_LAST_X = 20,
    C_LAST_Y = 38, C_CSBF = 56, C_SIG = 60, C_GT1 = 104, C_GT2 = 128, C_QP_DELTA = 134, C_CQO_FLAG = 136,
    C_CQO_IDX = 137, NUM_CTX = 138
};
static const uint8_t k_init_I[NUM_CTX] = {
    153, 200, 139, 141, 157, 154, 184, 184, 63, 153, 138, 138, 111, 141, 94, 138, 182, 154, 139, 139,
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    91, 171, 134, 141,
    111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141,
    179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153,
    136, 139, 111, 136, 139, 111, 141, 111,
    140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166,
    182, 140, 227, 122, 197, 138, 153, 136, 167, 152, 152, 154, 154, 154, 154};

/* ------------------------------------------------------------ options + state */
typedef struct {
    int W, H, CW, CH; /* coded size (luma), padded to min CB */
    int outW, outH;
    int bd;
    int qp;
    int sdh, tskip, qpdelta, sao, pcm, bypass, slice_rows, depth, log2ctb, beta, tc, cbqp, crqp, wpp;
    int tile_cols, tile_rows, lf_tiles; /* uniform tile grid (1 x 1 = no tiles) */
    int strong;
    int log2maxtb;
    int sl; /* scaling-list mode (--sl) */
    int nut;   /* NAL unit type of the (intra) first picture: 19 IDR_W_RADL, 21 CRA, 16 BLA_W_LP */
    int delay; /* sps_max_num_reorder_pics; the stream then carries delay + 1 all-skip P pictures */
    long long rawconf[4]; /* --conf: raw conformance window offsets (-1: derived from the size) */
    int wdelta;           /* --wdelta: subtracted from the signalled picture width */
    int profile, vui, rext, maxts, sao_scale[2], cqo, ppsext;
    int cqo_len, cqo_depth, cqo_cb[6], cqo_cr[6]; /* chroma QP offset list (--cqolist, --cqodepth) */
    int eff_maxts;        /* log2 max transform-skip size the decoder uses (2 without the PPS range ext) */
} Opt;
#define RX_ROT 1
#define RX_CTX 2
#define RX_RDPCM 4
#define RX_EXTPREC 16
#define RX_NOSMOOTH 32
#define RX_RICE 128

typedef struct {
    Opt o;
    uint16_t *src[3];
    uint16_t *rec[3];
    int st[3];
    int ctbs, ctbW, ctbH, mw, mh;
    int8_t *qpm;
    uint8_t *ipm, *ctd;
    int *ctb_slice; /* slice index per CTB (-1 = not coded) */
    int *rs2ts, *ts2rs, *tile_id, *col_bd; /* tile scan (6.5.1); identity without tiles */
    /* state */
    uint8_t ctx[NUM_CTX];
    Enc ce;
    int slice_idx, slice_qp;
    int qg_pred, qpd_val, is_qpd_coded, first_qg, last_cu_qp, qp_y, target_qp;
    int cu_bypass;
    int cqo_on;                      /* cu_chroma_qp_offset_enabled_flag of the slice */
    int cqo_coded, cqo_choice;       /* IsCuChromaQpOffsetCoded; the group's choice: -1 flag 0, else idx */
    int qpbd;
    int stat[4]; /* StatCoeff (persistent_rice_adaptation) */
} G;

static int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

static void init_contexts(G *g, int qp) {
    qp = clip3(0, 51, qp);
    for (int i = 0; i < NUM_CTX; i++) {
        int iv = k_init_I[i];
        int m = (iv >> 4) * 5 - 45, n = ((iv & 15) << 3) - 16;
        int pre = clip3(1, 126, ((m * qp) >> 4) + n);
        int mps = pre <= 63 ? 0 : 1;
        g->ctx[i] = (uint8_t)(((mps ? pre - 64 : 63 - pre) << 1) | mps);
    }
    memset(g->stat, 0, sizeof(g->stat));
}

static int zs(G *g, int x, int y) {
    int ctb = (y >> g->o.log2ctb) * g->ctbW + (x >> g->o.log2ctb);
    int xi = (x & (g->ctbs - 1)) >> 2, yi = (y & (g->ctbs - 1)) >> 2, z = 0;
    for (int i = 0; i < 5; i++) z |= (((xi >> i) & 1) << (2 * i)) | (((yi >> i) & 1) << (2 * i + 1));
    return (g->rs2ts[ctb] << (2 * (g->o.log2ctb - 2))) + z; /* decoding order */
}
static int avail(G *g, int xc, int yc, int xn, int yn) {
    if (xn < 0 || yn < 0 || xn >= g->o.CW || yn >= g->o.CH) return 0;
    int cn = (yn >> g->o.log2ctb) * g->ctbW + (xn >> g->o.log2ctb);
    int cc = (yc >> g->o.log2ctb) * g->ctbW + (xc >> g->o.log2ctb);
    if (g->ctb_slice[cn] < 0 || g->ctb_slice[cn] != g->ctb_slice[cc]) return 0;
    if (g->tile_id[cn] != g->tile_id[cc]) return 0;
    return zs(g, xn, yn) <= zs(g, xc, yc);
}

/* ------------------------------------------------------------ transforms */
static int8_t tm32[32][32];
static void init_tm(void) {
    static const int C[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                              61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
    for (int m = 0; m < 32; m++)
        for (int n = 0; n < 32; n++) {
            int a = ((2 * n + 1) * m) % 128;
            if (a > 64) a = 128 - a;
            tm32[m][n] = (int8_t)(a > 32 ? -C[64 - a] : C[a]);
        }
}
static const int k_dst[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
static int coefm(int dst, int n, int j, int i) { return dst ? k_dst[j][i] : tm32[j * (32 / n)][i]; }

/* forward 2-D transform (HM: shift1 = log2n + bd - 9, shift2 = log2n + 6) */
static void fwd_transform(const int *res, int *coef, int n, int log2n, int dst, int bd) {
    int tmp[32 * 32];
    int s1 = log2n + bd - 9, s2 = log2n + 6;
    for (int y = 0; y < n; y++)
        for (int k = 0; k < n; k++) { /* horizontal: row y */
            long s = 0;
            for (int x = 0; x < n; x++) s += (long)coefm(dst, n, k, x) * res[y * n + x];
            tmp[y * n + k] = (int)((s + (1L << (s1 - 1))) >> s1);
        }
    for (int x = 0; x < n; x++)
        for (int k = 0; k < n; k++) {
            long s = 0;
            for (int y = 0; y < n; y++) s += (long)coefm(dst, n, k, y) * tmp[y * n + x];
            coef[k * n + x] = (int)((s + (1L << (s2 - 1))) >> s2);
        }
}
static void inv_transform(const int *d, int *r, int n, int dst, int bd) {
    int tmp[32 * 32];
    for (int x = 0; x < n; x++)
        for (int y = 0; y < n; y++) {
            long s = 0;
            for (int j = 0; j < n; j++) s += (long)coefm(dst, n, j, y) * d[j * n + x];
            tmp[y * n + x] = clip3(-32768, 32767, (int)((s + 64) >> 7));
        }
    int bdShift = 20 - bd;
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            long s = 0;
            for (int j = 0; j < n; j++) s += (long)coefm(dst, n, j, x) * tmp[y * n + j];
            r[y * n + x] = (int)((s + (1L << (bdShift - 1))) >> bdShift);
        }
}

/* ------------------------------------------------------------ intra prediction (8.4.4.2) */
static const int k_angle[35] = {0,   0,   32,  26,  21,  17,  13,  9,  5,  2,  0,  -2,
                                -5,  -9,  -13, -17, -21, -26, -32, -26, -21, -17, -13, -9,
                                -5,  -2,  0,   2,   5,   9,   13,  17,  21,  26,  32};
static const int k_inv_angle[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482,
                                    -390, -315, -256, -315, -390, -482, -630, -910, -1638, -4096};

typedef struct { int seq[129]; int n; } Refs;

static void build_refs(G *g, int c, int x0, int y0, int log2n, Refs *R) {
    const int n = 1 << log2n, sh = c ? 1 : 0, bd = g->o.bd;
    const uint16_t *pl = g->rec[c];
    const int st = g->st[c];
    int av[129], any = 0;
    int L = 4 * n + 1;
    for (int k = 0; k < L; k++) {
        int xn, yn;
        if (k < 2 * n) { xn = x0 - 1; yn = y0 + (2 * n - 1 - k); }
        else if (k == 2 * n) { xn = x0 - 1; yn = y0 - 1; }
        else { xn = x0 + (k - 2 * n - 1); yn = y0 - 1; }
        av[k] = avail(g, x0 << sh, y0 << sh, xn << sh, yn << sh);
        R->seq[k] = av[k] ? pl[yn * st + xn] : 0;
        any |= av[k];
    }
    if (!any) {
        for (int k = 0; k < L; k++) R->seq[k] = 1 << (bd - 1);
    } else {
        if (!av[0]) { int f = 1; while (!av[f]) f++; R->seq[0] = R->seq[f]; }
        for (int k = 1; k < L; k++) if (!av[k]) R->seq[k] = R->seq[k - 1];
    }
    R->n = n;
}

static void filter_refs(G *g, int c, int mode, Refs *R) {
    const int n = R->n, bd = g->o.bd;
    if (c != 0 || mode == 1 || n == 4 || (g->o.rext & RX_NOSMOOTH)) return;
    int d26 = abs(mode - 26), d10 = abs(mode - 10), md = d26 < d10 ? d26 : d10;
    int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
    if (!(mode == 0 || md > thr)) return;
    int *s = R->seq, f[129], L = 4 * n + 1, corner = s[2 * n];
    if (g->o.strong && n == 32 && abs(corner + s[4 * n] - 2 * s[3 * n]) < (1 << (bd - 5)) &&
        abs(corner + s[0] - 2 * s[n]) < (1 << (bd - 5))) {
        for (int k = 0; k < L; k++) {
            if (k == 0 || k == 4 * n || k == 2 * n) f[k] = s[k];
            else if (k < 2 * n) { int y = 2 * n - 1 - k; f[k] = ((63 - y) * corner + (y + 1) * s[0] + 32) >> 6; }
            else { int x = k - 2 * n - 1; f[k] = ((63 - x) * corner + (x + 1) * s[4 * n] + 32) >> 6; }
        }
    } else {
        f[0] = s[0];
        f[L - 1] = s[L - 1];
        for (int k = 1; k < L - 1; k++) f[k] = (s[k - 1] + 2 * s[k] + s[k + 1] + 2) >> 2;
    }
    memcpy(s, f, sizeof(int) * L);
}

static void predict(G *g, int c, int mode, const Refs *Rf, int *pred) {
    const int n = Rf->n, maxv = (1 << g->o.bd) - 1;
    int log2n = 0;
    while ((1 << log2n) < n) log2n++;
    const int *R = Rf->seq;
#define PL(y) R[2 * n - 1 - (y)]
#define PT(x) R[2 * n + 1 + (x)]
    if (mode == 0) {
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++)
                pred[y * n + x] = ((n - 1 - x) * PL(y) + (x + 1) * PT(n) + (n - 1 - y) * PT(x) + (y + 1) * PL(n) + n) >> (log2n + 1);
        return;
    }
    if (mode == 1) {
        int sum = n;
        for (int k = 0; k < n; k++) sum += PT(k) + PL(k);
        int dc = sum >> (log2n + 1);
        for (int i = 0; i < n * n; i++) pred[i] = dc;
        if (c == 0 && n < 32) {
            pred[0] = (PL(0) + 2 * dc + PT(0) + 2) >> 2;
            for (int x = 1; x < n; x++) pred[x] = (PT(x) + 3 * dc + 2) >> 2;
            for (int y = 1; y < n; y++) pred[y * n] = (PL(y) + 3 * dc + 2) >> 2;
        }
        return;
    }
    int angle = k_angle[mode], inv = k_inv_angle[mode];
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            int pv;
            if (mode >= 18) {
                int idx = ((y + 1) * angle) >> 5, fr = ((y + 1) * angle) & 31;
                int k1 = x + idx + 1, k2 = k1 + 1;
                int r1 = k1 >= 0 ? R[2 * n + k1] : R[2 * n - ((k1 * inv + 128) >> 8)];
                int r2 = k2 >= 0 ? R[2 * n + k2] : R[2 * n - ((k2 * inv + 128) >> 8)];
                pv = fr ? ((32 - fr) * r1 + fr * r2 + 16) >> 5 : r1;
                if (mode == 26 && c == 0 && n < 32 && x == 0) pv = clip3(0, maxv, PT(0) + ((PL(y) - R[2 * n]) >> 1));
            } else {
                int idx = ((x + 1) * angle) >> 5, fr = ((x + 1) * angle) & 31;
                int k1 = y + idx + 1, k2 = k1 + 1;
                int r1 = k1 >= 0 ? R[2 * n - k1] : R[2 * n + ((k1 * inv + 128) >> 8)];
                int r2 = k2 >= 0 ? R[2 * n - k2] : R[2 * n + ((k2 * inv + 128) >> 8)];
                pv = fr ? ((32 - fr) * r1 + fr * r2 + 16) >> 5 : r1;
                if (mode == 10 && c == 0 && n < 32 && y == 0) pv = clip3(0, maxv, PL(0) + ((PT(x) - R[2 * n]) >> 1));
            }
            pred[y * n + x] = pv;
        }
#undef PL
#undef PT
}

/* SAD of predicting with mode m vs source */
static long mode_cost(G *g, int c, int x0, int y0, int log2n, int mode, const Refs *raw) {
    Refs R = *raw;
    int pred[1024];
    filter_refs(g, c, mode, &R);
    predict(g, c, mode, &R, pred);
    const int n = 1 << log2n, st = g->st[c];
    long s = 0;
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) s += abs(g->src[c][(y0 + y) * st + x0 + x] - pred[y * n + x]);
    return s;
}

/* ------------------------------------------------------------ scans */
static uint8_t scan_diag[4][64][2], scan_hor[4][64][2], scan_ver[4][64][2];
static void init_scans(void) {
    for (int l = 0; l < 4; l++) {
        int bs = 1 << l, i = 0, x = 0, y = 0;
        while (i < bs * bs) {
            while (y >= 0) {
                if (x < bs && y < bs) { scan_diag[l][i][0] = (uint8_t)x; scan_diag[l][i][1] = (uint8_t)y; i++; }
                y--; x++;
            }
            y = x; x = 0;
        }
        i = 0;
        for (y = 0; y < bs; y++) for (x = 0; x < bs; x++, i++) { scan_hor[l][i][0] = (uint8_t)x; scan_hor[l][i][1] = (uint8_t)y; }
        i = 0;
        for (x = 0; x < bs; x++) for (y = 0; y < bs; y++, i++) { scan_ver[l][i][0] = (uint8_t)x; scan_ver[l][i][1] = (uint8_t)y; }
    }
}

/* ------------------------------------------------------------ residual coding (7.3.8.11) */
static void enc_last_prefix(G *g, int base, int log2n, int c, int v) {
    int off, shift;
    if (c == 0) { off = 3 * (log2n - 2) + ((log2n - 1) >> 2); shift = (log2n + 1) >> 2; }
    else { off = 15; shift = log2n - 2; }
    int maxv = (log2n << 1) - 1;
    for (int i = 0; i < v; i++) ce_bin(&g->ce, &g->ctx[base + off + (i >> shift)], 1);
    if (v < maxv) ce_bin(&g->ce, &g->ctx[base + off + (v >> shift)], 0);
}
static void pos_to_prefix(int p, int *prefix, int *suffix, int *sbits) {
    /* inverse of: prefix<=3 -> p ; else (1<<nb)*(2+(prefix&1)) + suffix, nb=(prefix>>1)-1 */
    if (p < 4) { *prefix = p; *sbits = 0; *suffix = 0; return; }
    for (int pr = 4; pr < 10; pr++) {
        int nb = (pr >> 1) - 1, base = (1 << nb) * (2 + (pr & 1));
        if (p >= base && p < base + (1 << nb)) { *prefix = pr; *sbits = nb; *suffix = p - base; return; }
    }
}
static void enc_alr(G *g, int v, int rice) {
    /* coeff_abs_level_remaining with the decoder's prefix/suffix structure */
    if ((v >> rice) < 3) {
        int pre = v >> rice;
        for (int i = 0; i < pre; i++) ce_byp(&g->ce, 1);
        ce_byp(&g->ce, 0);
        ce_bypn(&g->ce, (uint32_t)(v & ((1 << rice) - 1)), rice);
        return;
    }
    /* value = (((1<<pm3)+2) << rice) + suffix(pm3 + rice bits), prefix = pm3 + 3 */
    int pm3 = 0;
    while ((((1 << (pm3 + 1)) + 2) << rice) <= v) pm3++;
    if ((g->o.rext & RX_EXTPREC) && pm3 >= 12) {
        fprintf(stderr, "level escape too long for extended_precision_processing (limited EGk)\n");
        exit(3);
    }
    int base = ((1 << pm3) + 2) << rice;
    for (int i = 0; i < pm3 + 3; i++) ce_byp(&g->ce, 1);
    ce_byp(&g->ce, 0);
    ce_bypn(&g->ce, (uint32_t)(v - base), pm3 + rice);
}

/* coef[y*n+x] levels; mode for scan; writes syntax */
static void enc_residual(G *g, int *coef, int log2n, int c, int pred_mode, int tskip) {
    const int n = 1 << log2n;
    if (g->o.tskip && !g->cu_bypass && log2n <= g->o.eff_maxts) ce_bin(&g->ce, &g->ctx[C_TSKIP + (c ? 1 : 0)], tskip);
    const int ts_ctx = (g->o.rext & RX_CTX) && (tskip || g->cu_bypass);
    const int rdpcm_ts = (g->o.rext & RX_RDPCM) && tskip && (pred_mode == 10 || pred_mode == 26);
    const int rice_on = (g->o.rext & RX_RICE) != 0, sb_type = 2 * (c == 0) + ((tskip || g->cu_bypass) ? 1 : 0);
    int scanIdx = 0;
    if (log2n == 2 || (log2n == 3 && c == 0)) {
        if (pred_mode >= 6 && pred_mode <= 14) scanIdx = 2;
        else if (pred_mode >= 22 && pred_mode <= 30) scanIdx = 1;
    }
    const uint8_t(*sc)[64][2] = scanIdx == 0 ? scan_diag : (scanIdx == 1 ? scan_hor : scan_ver);
    const int lsb = log2n - 2, nsb = 1 << (2 * lsb);
    /* last significant position in scan order */
    int lastSub = -1, lastPos = -1;
    for (int i = nsb - 1; i >= 0 && lastSub < 0; i--) {
        int xs = sc[lsb][i][0], ys = sc[lsb][i][1];
        for (int k = 15; k >= 0; k--) {
            int xc = (xs << 2) + sc[2][k][0], yc = (ys << 2) + sc[2][k][1];
            if (coef[yc * n + xc]) { lastSub = i; lastPos = k; break; }
        }
    }
    int lx = (sc[lsb][lastSub][0] << 2) + sc[2][lastPos][0];
    int ly = (sc[lsb][lastSub][1] << 2) + sc[2][lastPos][1];
    if (scanIdx == 2) { int t = lx; lx = ly; ly = t; }
    int px, sx, bx, py, sy, by;
    pos_to_prefix(lx, &px, &sx, &bx);
    pos_to_prefix(ly, &py, &sy, &by);
    enc_last_prefix(g, C_LAST_X, log2n, c, px);
    enc_last_prefix(g, C_LAST_Y, log2n, c, py);
    if (px > 3) ce_bypn(&g->ce, (uint32_t)sx, bx);
    if (py > 3) ce_bypn(&g->ce, (uint32_t)sy, by);
    uint8_t csbf[8][8];
    memset(csbf, 0, sizeof(csbf));
    int greater1_ctx = 1;
    for (int i = lastSub; i >= 0; i--) {
        int xs = sc[lsb][i][0], ys = sc[lsb][i][1];
        int lv[16];
        int anynz = 0;
        for (int k = 0; k < 16; k++) {
            int xc = (xs << 2) + sc[2][k][0], yc = (ys << 2) + sc[2][k][1];
            lv[k] = coef[yc * n + xc];
            if (lv[k]) anynz = 1;
        }
        int infer_dc = 0;
        if (i < lastSub && i > 0) {
            int csr = (xs + 1 < (1 << lsb)) ? csbf[xs + 1][ys] : 0;
            int csb = (ys + 1 < (1 << lsb)) ? csbf[xs][ys + 1] : 0;
            csbf[xs][ys] = (uint8_t)anynz;
            ce_bin(&g->ce, &g->ctx[C_CSBF + (csr | csb) + (c ? 2 : 0)], anynz);
            infer_dc = 1;
        } else {
            csbf[xs][ys] = 1;
        }
        int nstart = (i == lastSub) ? lastPos - 1 : 15;
        int prevCsbf = 0;
        if (xs + 1 < (1 << lsb)) prevCsbf |= csbf[xs + 1][ys];
        if (ys + 1 < (1 << lsb)) prevCsbf |= csbf[xs][ys + 1] << 1;
        if (csbf[xs][ys]) {
            /* if DC would be inferred but is zero, we cannot signal it: the
             * inference only triggers when all other sig flags are 0 -> then
             * anynz implies DC nonzero. */
            for (int nn = nstart; nn >= 0; nn--) {
                int xp = sc[2][nn][0], yp = sc[2][nn][1];
                int xC = (xs << 2) + xp, yC = (ys << 2) + yp;
                if (nn > 0 || !infer_dc) {
                    int sigCtx;
                    if (ts_ctx) {
                        sigCtx = c == 0 ? 42 : 16;
                    } else if (log2n == 2) {
                        static const uint8_t m[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
                        sigCtx = m[(yC << 2) + xC];
                    } else if (xC + yC == 0) {
                        sigCtx = 0;
                    } else {
                        if (prevCsbf == 0) sigCtx = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
                        else if (prevCsbf == 1) sigCtx = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
                        else if (prevCsbf == 2) sigCtx = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
                        else sigCtx = 2;
                        if (c == 0) {
                            if (xs > 0 || ys > 0) sigCtx += 3;
                            sigCtx += (log2n == 3) ? ((scanIdx == 0) ? 9 : 15) : 21;
                        } else {
                            sigCtx += (log2n == 3) ? 9 : 12;
                        }
                    }
                    int s = lv[nn] != 0;
                    ce_bin(&g->ce, &g->ctx[C_SIG + (c == 0 ? sigCtx : 27 + sigCtx)], s);
                    if (s) infer_dc = 0;
                }
            }
        }
        if (!anynz) continue;
        int ctxSet = (i == 0 || c > 0) ? 0 : 2;
        if (greater1_ctx == 0) ctxSet++;
        greater1_ctx = 1;
        int numG1 = 0, lastG1 = -1, firstSig = 16, lastSig = -1;
        int g1[16] = {0};
        for (int nn = 15; nn >= 0; nn--) {
            if (!lv[nn]) continue;
            if (numG1 < 8) {
                int f = abs(lv[nn]) > 1;
                ce_bin(&g->ce, &g->ctx[C_GT1 + ctxSet * 4 + greater1_ctx + (c ? 16 : 0)], f);
                g1[nn] = f;
                numG1++;
                if (f) { greater1_ctx = 0; if (lastG1 == -1) lastG1 = nn; }
                else if (greater1_ctx > 0 && greater1_ctx < 3) greater1_ctx++;
            }
            if (lastSig == -1) lastSig = nn;
            firstSig = nn;
        }
        int signHidden = !g->cu_bypass && !rdpcm_ts && (lastSig - firstSig > 3);
        int g2 = 0;
        if (lastG1 != -1) {
            g2 = abs(lv[lastG1]) > 2;
            ce_bin(&g->ce, &g->ctx[C_GT2 + ctxSet + (c ? 4 : 0)], g2);
        }
        for (int nn = 15; nn >= 0; nn--)
            if (lv[nn] && (!g->o.sdh || !signHidden || nn != firstSig)) ce_byp(&g->ce, lv[nn] < 0);
        int numSig = 0, rice = rice_on ? g->stat[sb_type] / 4 : 0, stat_done = 0;
        for (int nn = 15; nn >= 0; nn--) {
            if (!lv[nn]) continue;
            int base = 1 + g1[nn] + (nn == lastG1 ? g2 : 0);
            if (base == ((numSig < 8) ? ((nn == lastG1) ? 3 : 2) : 1)) {
                int rem = abs(lv[nn]) - base;
                enc_alr(g, rem, rice);
                if (abs(lv[nn]) > 3 * (1 << rice)) rice = rice_on ? rice + 1 : (rice < 4 ? rice + 1 : 4);
                if (rice_on && !stat_done) { /* StatCoeff update (9.3.3.11) */
                    int ri = g->stat[sb_type] / 4;
                    if (rem >= (3 << ri)) g->stat[sb_type]++;
                    else if (2 * rem < (1 << ri) && g->stat[sb_type] > 0) g->stat[sb_type]--;
                    stat_done = 1;
                }
            }
            numSig++;
        }
    }
}

/* sign data hiding: make each hidden sign recoverable from the parity of
 * the subblock's absolute sum (decoder rule in residual_coding) by growing
 * the highest-frequency coefficient of the subblock by one.  Applied before
 * reconstruction so encoder and decoder agree. */
static void sdh_fix(G *g, int *coef, int log2n, int c, int pred_mode, int tskip) {
    const int n = 1 << log2n;
    if (!g->o.sdh || g->cu_bypass) return;
    if ((g->o.rext & RX_RDPCM) && tskip && (pred_mode == 10 || pred_mode == 26)) return; /* no hiding */
    int scanIdx = 0;
    if (log2n == 2 || (log2n == 3 && c == 0)) {
        if (pred_mode >= 6 && pred_mode <= 14) scanIdx = 2;
        else if (pred_mode >= 22 && pred_mode <= 30) scanIdx = 1;
    }
    const uint8_t(*sc)[64][2] = scanIdx == 0 ? scan_diag : (scanIdx == 1 ? scan_hor : scan_ver);
    const int lsb = log2n - 2, nsb = 1 << (2 * lsb);
    for (int i = 0; i < nsb; i++) {
        int xs = sc[lsb][i][0], ys = sc[lsb][i][1];
        int first = -1, last = -1, sum = 0;
        for (int k = 0; k < 16; k++) {
            int xc = (xs << 2) + sc[2][k][0], yc = (ys << 2) + sc[2][k][1];
            int v = coef[yc * n + xc];
            if (v) { if (first < 0) first = k; last = k; sum += abs(v); }
        }
        if (first < 0 || last - first <= 3) continue;
        int fx = (xs << 2) + sc[2][first][0], fy = (ys << 2) + sc[2][first][1];
        int neg = coef[fy * n + fx] < 0;
        if ((sum & 1) != neg) {
            int lx = (xs << 2) + sc[2][last][0], ly = (ys << 2) + sc[2][last][1];
            coef[ly * n + lx] += coef[ly * n + lx] > 0 ? 1 : -1;
        }
    }
}

/* ------------------------------------------------------------ scaling lists (7.3.4, 7.4.5) */
/* --sl: 0 off; 1 scaling_list_enabled with the default lists (no data in SPS or PPS);
 * 2 explicit SPS lists; 3 explicit SPS lists overridden by explicit PPS lists; 4 default SPS
 * lists overridden by explicit PPS lists.  Explicit lists mix the three ways of coding each
 * (sizeId, matrixId): pred_mode 0 with delta 0 (default list), pred_mode 0 with a
 * scaling_list_pred_matrix_id_delta copy of an earlier matrix (DC included), and DPCM-coded
 * values (with scaling_list_dc_coef_minus8 for 16x16 / 32x32). */
typedef struct { uint8_t sl[4][6][64]; uint8_t dc[4][6]; } SList; /* sl in up-right diagonal order */
static const uint8_t k_sl_def_intra[64] = {
    16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18, 17, 18, 18, 17, 18, 21,
    19, 20, 21, 20, 19, 21, 24, 22, 22, 24, 24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29,
    31, 35, 35, 31, 29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115};
static const uint8_t k_sl_def_inter[64] = {
    16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18, 18, 18, 18, 18, 18, 20,
    20, 20, 20, 20, 20, 20, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28,
    28, 28, 28, 28, 28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91};
static int g_sl_on;                 /* scaling_list_enabled_flag */
static uint16_t g_sf[4][3][1024];   /* ScalingFactor m[x][y] (raster y*n+x) per sizeId, cIdx (intra) */

static void sl_default(SList *L) {
    for (int m = 0; m < 6; m++) {
        memset(L->sl[0][m], 16, 16);
        L->dc[0][m] = 16;
        for (int s = 1; s < 4; s++) {
            memcpy(L->sl[s][m], m < 3 ? k_sl_def_intra : k_sl_def_inter, 64);
            L->dc[s][m] = 16;
        }
    }
}

/* scaling_list_data(): random lists, written and applied to L */
static void write_scaling_list_data(BW *b, SList *L) {
    sl_default(L);
    for (int sizeId = 0; sizeId < 4; sizeId++) {
        const int step = sizeId == 3 ? 3 : 1, n = sizeId ? 64 : 16;
        for (int m = 0; m < 6; m += step) {
            int how = rndn(5); /* 0 default, 1 copy, else explicit */
            if (how == 1 && m < step) how = 2;
            if (how <= 1) {
                bw_put(b, 0, 1);
                if (how == 0) { bw_ue(b, 0); continue; } /* default (already in L) */
                int delta = 1 + rndn(m / step);
                bw_ue(b, (uint32_t)delta);
                int ref = m - delta * step;
                memcpy(L->sl[sizeId][m], L->sl[sizeId][ref], (size_t)n);
                L->dc[sizeId][m] = L->dc[sizeId][ref];
                continue;
            }
            bw_put(b, 1, 1);
            int next = 8;
            if (sizeId > 1) {
                int dcv = 1 + rndn(rndn(6) == 0 ? 255 : 40);
                bw_se(b, dcv - 8);
                next = dcv;
                L->dc[sizeId][m] = (uint8_t)dcv;
            }
            /* smooth, frequency-increasing lists with jitter; now and then a wild one */
            const int wild = rndn(6) == 0, base = 6 + rndn(20), slope = rndn(6);
            for (int i = 0; i < n; i++) {
                int x = scan_diag[sizeId ? 3 : 2][i][0], y = scan_diag[sizeId ? 3 : 2][i][1];
                int v = wild ? 1 + rndn(255) : clip3(1, 255, base + slope * (x + y) * (sizeId ? 1 : 2) + rndn(5) - 2);
                int d = v - next;
                if (d > 127) d -= 256;
                if (d < -128) d += 256;
                bw_se(b, d);
                next = v;
                L->sl[sizeId][m][i] = (uint8_t)v;
            }
        }
    }
}

/* ScalingFactor (7.4.5) of the active lists, intra matrices (matrixId = cIdx) */
static void sl_expand(const SList *L) {
    for (int sizeId = 0; sizeId < 4; sizeId++) {
        const int n = 4 << sizeId;
        for (int c = 0; c < 3; c++) {
            if (sizeId == 3 && c) break; /* no 32x32 chroma TBs in 4:2:0 */
            for (int i = 0; i < (sizeId ? 64 : 16); i++) {
                int x = scan_diag[sizeId ? 3 : 2][i][0], y = scan_diag[sizeId ? 3 : 2][i][1];
                int r = sizeId <= 1 ? 1 : (sizeId == 2 ? 2 : 4);
                for (int yy = 0; yy < r; yy++)
                    for (int xx = 0; xx < r; xx++) g_sf[sizeId][c][(y * r + yy) * n + x * r + xx] = L->sl[sizeId][c][i];
            }
            if (sizeId >= 2) g_sf[sizeId][c][0] = L->dc[sizeId][c];
        }
    }
}
/* m[x][y] of a TB (8.6.4.2); 16 when scaling lists are off */
static int sf(int c, int log2n, int i) { return g_sl_on ? g_sf[log2n - 2][c][i] : 16; }

/* ------------------------------------------------------------ quant / recon of one TB */
static const int k_qscale[6] = {26214, 23302, 20560, 18396, 16384, 14564};
static const int k_ls[6] = {40, 45, 51, 57, 64, 72};

/* RExt residual DPCM (8.6.8): accumulate down the columns (mode 26) / along the rows (mode 10),
 * int16 as in the decoder's coefficient buffer; diff_dpcm is its inverse (encoder side) */
static void acc_dpcm(int *r, int n, int vertical) {
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            if (vertical ? y == 0 : x == 0) continue;
            r[y * n + x] = (int16_t)(r[y * n + x] + (vertical ? r[(y - 1) * n + x] : r[y * n + x - 1]));
        }
}
static void diff_dpcm(int *r, int n, int vertical) {
    for (int y = n - 1; y >= 0; y--)
        for (int x = n - 1; x >= 0; x--) {
            if (vertical ? y == 0 : x == 0) continue;
            r[y * n + x] -= vertical ? r[(y - 1) * n + x] : r[y * n + x - 1];
        }
}
static int uses_rdpcm(G *g, int mode) { return (g->o.rext & RX_RDPCM) && (mode == 10 || mode == 26); }

/* Encode-side processing of one transform block: prediction already in
 * rec; computes levels into coef, reconstructs rec.  Returns cbf. */
static int code_block(G *g, int c, int x0, int y0, int log2n, int pred_mode, int qp, int *coef, int *tskip_out,
                      const int *pred) {
    const int n = 1 << log2n, st = g->st[c], bd = g->o.bd, maxv = (1 << bd) - 1;
    int res[1024];
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) res[y * n + x] = g->src[c][(y0 + y) * st + x0 + x] - pred[y * n + x];
    int nz = 0;
    int tskip = 0;
    int dst = (c == 0 && log2n == 2);
    (void)maxv;
    if (g->cu_bypass) {
        if (uses_rdpcm(g, pred_mode)) diff_dpcm(res, n, pred_mode == 26); /* lossless: levels = differences */
        for (int i = 0; i < n * n; i++) { coef[i] = res[i]; nz |= res[i] != 0; }
    } else {
        int tc[1024];
        if (g->o.tskip && log2n <= g->o.eff_maxts && rndn(log2n == 2 ? 5 : 3) == 0) tskip = 1;
        if (tskip) {
            if (uses_rdpcm(g, pred_mode)) diff_dpcm(res, n, pred_mode == 26); /* open-loop DPCM */
            int shift = 15 - bd - log2n; /* HM: transformSkipShift */
            for (int i = 0; i < n * n; i++) tc[i] = shift >= 0 ? res[i] * (1 << shift) : res[i] >> -shift;
            if ((g->o.rext & RX_ROT) && n == 4)
                for (int i = 0; i < 8; i++) { int t = tc[i]; tc[i] = tc[15 - i]; tc[15 - i] = t; }
        } else {
            fwd_transform(res, tc, n, log2n, dst, bd);
        }
        int qbits = 14 + qp / 6 + (15 - bd - log2n);
        long add = (171L << (qbits - 9));
        for (int i = 0; i < n * n; i++) {
            long a = labs((long)tc[i]);
            int m = (tskip && n > 4) ? 16 : sf(c, log2n, i);
            int l = (int)((a * k_qscale[qp % 6] * 16 / m + add) >> qbits);
            if (l > 32767) l = 32767;
            coef[i] = tc[i] < 0 ? -l : l;
            nz |= l != 0;
        }
    }
    *tskip_out = tskip;
    return nz;
}

static void recon_block(G *g, int c, int x0, int y0, int log2n, int qp, const int *coef, int tskip, const int *pred,
                        int cbf, int mode) {
    const int n = 1 << log2n, st = g->st[c], bd = g->o.bd, maxv = (1 << bd) - 1;
    int r[1024];
    memset(r, 0, sizeof(int) * n * n);
    if (cbf) {
        if (g->cu_bypass) {
            for (int i = 0; i < n * n; i++) r[i] = coef[i];
            if (uses_rdpcm(g, mode)) acc_dpcm(r, n, mode == 26);
        } else {
            int d[1024];
            int bdShift = bd + log2n - 5;
            for (int i = 0; i < n * n; i++) {
                int m = (tskip && n > 4) ? 16 : sf(c, log2n, i);
                long v = (long)coef[i] * m * k_ls[qp % 6];
                v = (v << (qp / 6)) + (1L << (bdShift - 1));
                v >>= bdShift;
                d[i] = (int)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
            }
            if (tskip) {
                if ((g->o.rext & RX_ROT) && n == 4)
                    for (int i = 0; i < 8; i++) { int t = d[i]; d[i] = d[15 - i]; d[15 - i] = t; }
                int sh = 15 - bd - log2n;
                for (int i = 0; i < n * n; i++) r[i] = sh > 0 ? (d[i] + (1 << (sh - 1))) >> sh : (int16_t)(d[i] * (1 << -sh));
                if (uses_rdpcm(g, mode)) acc_dpcm(r, n, mode == 26);
            } else {
                inv_transform(d, r, n, c == 0 && log2n == 2, bd);
            }
        }
    }
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
            g->rec[c][(y0 + y) * st + x0 + x] = (uint16_t)clip3(0, maxv, pred[y * n + x] + r[y * n + x]);
}

static int chroma_qp_table(int qpi) {
    static const int t[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    return t[qpi - 30];
}

static void set_map(G *g, uint8_t *m, int x0, int y0, int n, uint8_t v) {
    for (int y = y0 >> 2; y < ((y0 + n) >> 2) && y < g->mh; y++)
        for (int x = x0 >> 2; x < ((x0 + n) >> 2) && x < g->mw; x++) m[y * g->mw + x] = v;
}
static void set_qp(G *g, int x0, int y0, int n, int qp) {
    for (int y = y0 >> 2; y < ((y0 + n) >> 2) && y < g->mh; y++)
        for (int x = x0 >> 2; x < ((x0 + n) >> 2) && x < g->mw; x++) g->qpm[y * g->mw + x] = (int8_t)qp;
}

/* ------------------------------------------------------------ CU coding */
typedef struct {
    int x0, y0, log2cb, cm; /* chroma mode */
} Cu;

static void write_qp_delta(G *g) {
    int v = g->target_qp - g->qg_pred;
    int a = abs(v);
    ce_bin(&g->ce, &g->ctx[C_QP_DELTA], a > 0);
    if (a > 0) {
        int pre = a < 5 ? a : 5;
        for (int i = 1; i < pre; i++) ce_bin(&g->ce, &g->ctx[C_QP_DELTA + 1], 1);
        if (pre < 5) ce_bin(&g->ce, &g->ctx[C_QP_DELTA + 1], 0);
        if (a >= 5) { /* EG0 of a - 5 */
            int s = a - 5, k = 0;
            while (s >= (1 << k)) { ce_byp(&g->ce, 1); s -= 1 << k; k++; }
            ce_byp(&g->ce, 0);
            ce_bypn(&g->ce, (uint32_t)s, k);
        }
        ce_byp(&g->ce, v < 0);
    }
    g->is_qpd_coded = 1;
    g->qpd_val = v;
}

/* Full transform-tree coding.  Because cbf flags precede residuals in the
 * syntax, each node is first computed (prediction + quantisation +
 * reconstruction in decoding order) and then written. */
typedef struct {
    int split;
    int cbf_cb, cbf_cr, cbf_l;
    int tsl, tscb, tscr;
    int coef_l[1024], coef_cb[256], coef_cr[256];
    int child[4];
} TNode;

static TNode *g_nodes;
static int g_nnodes;

static int tree_compute(G *g, Cu *cu, int x0, int y0, int xb, int yb, int log2n, int depth, int blk, int max_depth,
                        int intra_split) {
    int id = g_nnodes++;
    TNode *t = &g_nodes[id];
    int split;
    if (log2n <= g->o.log2maxtb && log2n > 2 && depth < max_depth && !(intra_split && depth == 0))
        split = (log2n > 3 && rndn(3) == 0) ? 1 : 0; /* random TU split for coverage */
    else
        split = log2n > g->o.log2maxtb || (intra_split && depth == 0);
    t->split = split;
    t->cbf_cb = t->cbf_cr = t->cbf_l = 0;
    if (split) {
        int h = 1 << (log2n - 1);
        int c0 = tree_compute(g, cu, x0, y0, x0, y0, log2n - 1, depth + 1, 0, max_depth, intra_split);
        int c1 = tree_compute(g, cu, x0 + h, y0, x0, y0, log2n - 1, depth + 1, 1, max_depth, intra_split);
        int c2 = tree_compute(g, cu, x0, y0 + h, x0, y0, log2n - 1, depth + 1, 2, max_depth, intra_split);
        int c3 = tree_compute(g, cu, x0 + h, y0 + h, x0, y0, log2n - 1, depth + 1, 3, max_depth, intra_split);
        t = &g_nodes[id];
        t->child[0] = c0; t->child[1] = c1; t->child[2] = c2; t->child[3] = c3;
        if (log2n > 2 + 1) { /* children have their own chroma: parent cbf = OR */
            for (int k = 0; k < 4; k++) { t->cbf_cb |= g_nodes[t->child[k]].cbf_cb; t->cbf_cr |= g_nodes[t->child[k]].cbf_cr; }
        } else {
            /* children are 4x4 luma: chroma 4x4 coded at blk 3 with this node's cbf */
            t->cbf_cb = g_nodes[t->child[3]].cbf_cb;
            t->cbf_cr = g_nodes[t->child[3]].cbf_cr;
        }
        return id;
    }
    /* leaf: luma */
    int lmode = g->ipm[(y0 >> 2) * g->mw + (x0 >> 2)];
    int pred[1024];
    Refs R;
    build_refs(g, 0, x0, y0, log2n, &R);
    filter_refs(g, 0, lmode, &R);
    predict(g, 0, lmode, &R, pred);
    int qpy = g->target_qp + g->qpbd;
    t->cbf_l = code_block(g, 0, x0, y0, log2n, lmode, qpy, t->coef_l, &t->tsl, pred);
    if (t->cbf_l) sdh_fix(g, t->coef_l, log2n, 0, lmode, t->tsl);
    recon_block(g, 0, x0, y0, log2n, qpy, t->coef_l, t->tsl, pred, t->cbf_l, lmode);
    int qpc[2];
    for (int k = 0; k < 2; k++) {
        int off = k == 0 ? g->o.cbqp : g->o.crqp;
        /* the group's chroma QP offset: coded before the group's first chroma residual */
        if (g->cqo_on && g->cqo_choice >= 0) off += k == 0 ? g->o.cqo_cb[g->cqo_choice] : g->o.cqo_cr[g->cqo_choice];
        qpc[k] = chroma_qp_table(clip3(-g->qpbd, 57, g->target_qp + off)) + g->qpbd;
    }
    int cm = cu->cm;
    if (log2n > 2 || blk == 3) {
        int xc = (log2n > 2 ? x0 : xb) >> 1, yc = (log2n > 2 ? y0 : yb) >> 1, l2 = log2n > 2 ? log2n - 1 : 2;
        for (int c = 1; c <= 2; c++) {
            build_refs(g, c, xc, yc, l2, &R);
            predict(g, c, cm, &R, pred);
            int *co = c == 1 ? t->coef_cb : t->coef_cr;
            int *ts = c == 1 ? &t->tscb : &t->tscr;
            int cbf = code_block(g, c, xc, yc, l2, cm, qpc[c - 1], co, ts, pred);
            if (cbf) sdh_fix(g, co, l2, c, cm, *ts);
            recon_block(g, c, xc, yc, l2, qpc[c - 1], co, *ts, pred, cbf, cm);
            if (c == 1) t->cbf_cb = cbf; else t->cbf_cr = cbf;
        }
    }
    return id;
}

static void tree_write(G *g, Cu *cu, int id, int x0, int y0, int xb, int yb, int log2n, int depth, int blk,
                       int max_depth, int intra_split, int pcb, int pcr) {
    TNode *t = &g_nodes[id];
    if (log2n <= g->o.log2maxtb && log2n > 2 && depth < max_depth && !(intra_split && depth == 0))
        ce_bin(&g->ce, &g->ctx[C_SPLIT_TF + 5 - log2n], t->split);
    int cbf_cb = 0, cbf_cr = 0;
    if (log2n > 2) {
        if (depth == 0 || pcb) { cbf_cb = t->cbf_cb; ce_bin(&g->ce, &g->ctx[C_CBF_CHROMA + depth], cbf_cb); }
        if (depth == 0 || pcr) { cbf_cr = t->cbf_cr; ce_bin(&g->ce, &g->ctx[C_CBF_CHROMA + depth], cbf_cr); }
    } else {
        cbf_cb = pcb;
        cbf_cr = pcr;
    }
    if (t->split) {
        int h = 1 << (log2n - 1);
        tree_write(g, cu, t->child[0], x0, y0, x0, y0, log2n - 1, depth + 1, 0, max_depth, intra_split, cbf_cb, cbf_cr);
        tree_write(g, cu, t->child[1], x0 + h, y0, x0, y0, log2n - 1, depth + 1, 1, max_depth, intra_split, cbf_cb, cbf_cr);
        tree_write(g, cu, t->child[2], x0, y0 + h, x0, y0, log2n - 1, depth + 1, 2, max_depth, intra_split, cbf_cb, cbf_cr);
        tree_write(g, cu, t->child[3], x0 + h, y0 + h, x0, y0, log2n - 1, depth + 1, 3, max_depth, intra_split, cbf_cb, cbf_cr);
        return;
    }
    ce_bin(&g->ce, &g->ctx[C_CBF_LUMA + (depth == 0 ? 1 : 0)], t->cbf_l);
    if ((t->cbf_l || cbf_cb || cbf_cr) && g->o.qpdelta && !g->is_qpd_coded) write_qp_delta(g);
    if ((cbf_cb || cbf_cr) && g->cqo_on && !g->cu_bypass && !g->cqo_coded) {
        ce_bin(&g->ce, &g->ctx[C_CQO_FLAG], g->cqo_choice >= 0);
        if (g->cqo_choice >= 0 && g->o.cqo_len > 1) {
            /* truncated unary; idx < cMax for both FFmpeg (5) and the spec (len_minus1) unless idx == 5 */
            for (int i = 0; i < g->cqo_choice; i++) ce_bin(&g->ce, &g->ctx[C_CQO_IDX], 1);
            if (g->cqo_choice < 5) ce_bin(&g->ce, &g->ctx[C_CQO_IDX], 0);
        }
        g->cqo_coded = 1;
    }
    int lmode = g->ipm[(y0 >> 2) * g->mw + (x0 >> 2)];
    if (t->cbf_l) enc_residual(g, t->coef_l, log2n, 0, lmode, t->tsl);
    if (log2n > 2) {
        if (cbf_cb) enc_residual(g, t->coef_cb, log2n - 1, 1, cu->cm, t->tscb);
        if (cbf_cr) enc_residual(g, t->coef_cr, log2n - 1, 2, cu->cm, t->tscr);
    } else if (blk == 3) {
        if (cbf_cb) enc_residual(g, t->coef_cb, 2, 1, cu->cm, t->tscb);
        if (cbf_cr) enc_residual(g, t->coef_cr, 2, 2, cu->cm, t->tscr);
    }
}

static long block_var(G *g, int x0, int y0, int n) {
    long s = 0, s2 = 0;
    int cnt = 0;
    for (int y = y0; y < y0 + n && y < g->o.CH; y++)
        for (int x = x0; x < x0 + n && x < g->o.CW; x++) {
            int v = g->src[0][y * g->st[0] + x];
            s += v; s2 += (long)v * v; cnt++;
        }
    if (!cnt) return 0;
    return (s2 - s * s / cnt) / cnt;
}

static void coding_unit(G *g, int x0, int y0, int log2cb) {
    const int n = 1 << log2cb;
    Cu cu = {x0, y0, log2cb, 0};
    g->cu_bypass = 0;
    if (g->o.bypass) {
        g->cu_bypass = rndn(40) == 0;
        ce_bin(&g->ce, &g->ctx[C_TQ_BYPASS], g->cu_bypass);
    }
    int part_nxn = 0;
    if (log2cb == 3) {
        long v = block_var(g, x0, y0, 8);
        part_nxn = v > (long)(g->o.qp * g->o.qp) * (1 << (2 * (g->o.bd - 8))) / 6 || rndn(8) == 0;
        ce_bin(&g->ce, &g->ctx[C_PART_MODE], !part_nxn);
    }
    g->qp_y = ((g->qg_pred + g->qpd_val + 52 + 2 * g->qpbd) % (52 + g->qpbd)) - g->qpbd;
    set_qp(g, x0, y0, n, g->qp_y);
    int pcm = 0;
    if (!part_nxn && g->o.pcm && log2cb >= 3 && log2cb <= 4) {
        pcm = rndn(30) == 0;
        ce_term(&g->ce, pcm);
    }
    if (pcm) {
        set_map(g, g->ipm, x0, y0, n, 1);
        /* pcm_flag: flush, align, raw samples (8-bit PCM depth = bd), restart */
        ce_finish(&g->ce);
        bw_put(g->ce.bw, 1, 1);
        bw_align_zero(g->ce.bw);
        for (int c = 0; c < 3; c++) {
            int cn = c ? n / 2 : n, xs = c ? x0 / 2 : x0, ys = c ? y0 / 2 : y0;
            for (int y = 0; y < cn; y++)
                for (int x = 0; x < cn; x++) {
                    int v = g->src[c][(ys + y) * g->st[c] + xs + x];
                    bw_put(g->ce.bw, (uint32_t)v, g->o.bd);
                    g->rec[c][(ys + y) * g->st[c] + xs + x] = (uint16_t)v;
                }
        }
        {
            BW *bw = g->ce.bw;
            ce_start(&g->ce, bw);
        }
        g->last_cu_qp = g->qp_y;
        return;
    }
    int np = part_nxn ? 4 : 1, pb = part_nxn ? n / 2 : n;
    int modes[4], prevf[4], mpmi[4], remv[4];
    for (int i = 0; i < np; i++) {
        int xp = x0 + (i & 1) * pb, yp = y0 + (i >> 1) * pb;
        /* candidate list */
        int ca = 1, cb = 1;
        if (avail(g, xp, yp, xp - 1, yp)) ca = g->ipm[(yp >> 2) * g->mw + ((xp - 1) >> 2)];
        if (avail(g, xp, yp, xp, yp - 1) && ((yp - 1) >> g->o.log2ctb) == (yp >> g->o.log2ctb))
            cb = g->ipm[((yp - 1) >> 2) * g->mw + (xp >> 2)];
        int cand[3];
        if (ca == cb) {
            if (ca < 2) { cand[0] = 0; cand[1] = 1; cand[2] = 26; }
            else { cand[0] = ca; cand[1] = 2 + ((ca + 29) % 32); cand[2] = 2 + ((ca - 2 + 1) % 32); }
        } else {
            cand[0] = ca; cand[1] = cb;
            cand[2] = (ca != 0 && cb != 0) ? 0 : ((ca != 1 && cb != 1) ? 1 : 26);
        }
        /* mode search at the TU size the PB will be predicted with (<= 32) */
        int l2 = 0;
        while ((1 << l2) < pb) l2++;
        int l2t = l2 > g->o.log2maxtb ? g->o.log2maxtb : l2;
        Refs R;
        build_refs(g, 0, xp, yp, l2t, &R);
        long best = -1;
        int bm = 0;
        for (int m = 0; m < 35; m++) {
            if (rndn(4) == 0 && m > 1) continue; /* sub-sampled search: speed + variety */
            long cst = mode_cost(g, 0, xp, yp, l2t, m, &R);
            if (m == cand[0] || m == cand[1] || m == cand[2]) cst -= cst / 16;
            if (best < 0 || cst < best) { best = cst; bm = m; }
        }
        modes[i] = bm;
        /* neighbours of later PBs in this CU see this PB's mode */
        set_map(g, g->ipm, xp, yp, pb, (uint8_t)bm);
        if (bm == cand[0] || bm == cand[1] || bm == cand[2]) {
            prevf[i] = 1;
            mpmi[i] = bm == cand[0] ? 0 : (bm == cand[1] ? 1 : 2);
        } else {
            prevf[i] = 0;
            int s[3] = {cand[0], cand[1], cand[2]}, t;
            if (s[0] > s[1]) { t = s[0]; s[0] = s[1]; s[1] = t; }
            if (s[0] > s[2]) { t = s[0]; s[0] = s[2]; s[2] = t; }
            if (s[1] > s[2]) { t = s[1]; s[1] = s[2]; s[2] = t; }
            int r = bm;
            for (int k = 2; k >= 0; k--) if (r > s[k]) r--;
            remv[i] = r;
        }
    }
    for (int i = 0; i < np; i++) ce_bin(&g->ce, &g->ctx[C_PREV_INTRA], prevf[i]);
    for (int i = 0; i < np; i++) {
        if (prevf[i]) {
            ce_byp(&g->ce, mpmi[i] > 0);
            if (mpmi[i] > 0) ce_byp(&g->ce, mpmi[i] > 1);
        } else {
            ce_bypn(&g->ce, (uint32_t)remv[i], 5);
        }
    }
    /* chroma mode */
    int lm = modes[0];
    int icpm = rndn(3) == 0 ? rndn(5) : 4;
    static const int cmodes[4] = {0, 26, 10, 1};
    if (icpm == 4) cu.cm = lm;
    else cu.cm = cmodes[icpm] == lm ? 34 : cmodes[icpm];
    ce_bin(&g->ce, &g->ctx[C_CHROMA_MODE], icpm != 4);
    if (icpm != 4) ce_bypn(&g->ce, (uint32_t)icpm, 2);
    /* transform tree */
    int max_depth = g->o.depth + part_nxn;
    g_nnodes = 0;
    int root = tree_compute(g, &cu, x0, y0, x0, y0, log2cb, 0, 0, max_depth, part_nxn);
    tree_write(g, &cu, root, x0, y0, x0, y0, log2cb, 0, 0, max_depth, part_nxn, 0, 0);
    /* CU QP after the (possible) delta */
    g->qp_y = ((g->qg_pred + g->qpd_val + 52 + 2 * g->qpbd) % (52 + g->qpbd)) - g->qpbd;
    set_qp(g, x0, y0, n, g->qp_y);
    g->last_cu_qp = g->qp_y;
}

static void qg_start(G *g, int xq, int yq) {
    int prev = g->first_qg ? g->slice_qp : g->last_cu_qp;
    g->first_qg = 0;
    int ctb = (yq >> g->o.log2ctb) * g->ctbW + (xq >> g->o.log2ctb);
    int qa = prev, qb = prev;
    if (avail(g, xq, yq, xq - 1, yq) && (yq >> g->o.log2ctb) * g->ctbW + ((xq - 1) >> g->o.log2ctb) == ctb)
        qa = g->qpm[(yq >> 2) * g->mw + ((xq - 1) >> 2)];
    if (avail(g, xq, yq, xq, yq - 1) && ((yq - 1) >> g->o.log2ctb) * g->ctbW + (xq >> g->o.log2ctb) == ctb)
        qb = g->qpm[((yq - 1) >> 2) * g->mw + (xq >> 2)];
    g->qg_pred = (qa + qb + 1) >> 1;
    g->qpd_val = 0;
    g->is_qpd_coded = 0;
    /* QP this quantisation group will be coded at */
    if (g->o.qpdelta) {
        int d = rndn(4) == 0 ? rndn(7) - 3 : 0;
        int t = g->o.qp + d;
        g->target_qp = clip3(-g->qpbd, 51, t);
    } else {
        g->target_qp = g->qg_pred;
    }
}

static void coding_quadtree(G *g, int x0, int y0, int log2cb, int depth, int log2qg) {
    const int n = 1 << log2cb;
    int split;
    if (x0 + n <= g->o.CW && y0 + n <= g->o.CH && log2cb > 3) {
        long v = block_var(g, x0, y0, n);
        long thr = (long)(4 + g->o.qp) * (1 << (2 * (g->o.bd - 8))) * (log2cb == 6 ? 2 : 3);
        if (log2cb == 6) split = v > thr / 4 || rndn(2);
        else split = v > thr || rndn(10) == 0;
        int inc = 0;
        if (avail(g, x0, y0, x0 - 1, y0) && g->ctd[(y0 >> 2) * g->mw + ((x0 - 1) >> 2)] > depth) inc++;
        if (avail(g, x0, y0, x0, y0 - 1) && g->ctd[((y0 - 1) >> 2) * g->mw + (x0 >> 2)] > depth) inc++;
        ce_bin(&g->ce, &g->ctx[C_SPLIT_CU + inc], split);
    } else {
        split = log2cb > 3;
    }
    if (log2cb >= log2qg) qg_start(g, x0, y0);
    if (g->cqo_on && log2cb >= g->o.log2ctb - g->o.cqo_depth) {
        /* a new chroma QP offset group: flag 0, or an index FFmpeg and the spec read alike */
        int nidx = g->o.cqo_len - (g->o.cqo_len < 6 && g->o.cqo_len > 1 ? 1 : 0);
        g->cqo_coded = 0;
        g->cqo_choice = rndn(nidx + 1) - 1;
    }
    if (split) {
        int h = n >> 1;
        coding_quadtree(g, x0, y0, log2cb - 1, depth + 1, log2qg);
        if (x0 + h < g->o.CW) coding_quadtree(g, x0 + h, y0, log2cb - 1, depth + 1, log2qg);
        if (y0 + h < g->o.CH) coding_quadtree(g, x0, y0 + h, log2cb - 1, depth + 1, log2qg);
        if (x0 + h < g->o.CW && y0 + h < g->o.CH) coding_quadtree(g, x0 + h, y0 + h, log2cb - 1, depth + 1, log2qg);
    } else {
        set_map(g, g->ctd, x0, y0, n, (uint8_t)depth);
        coding_unit(g, x0, y0, log2cb);
    }
}

/* SAO syntax: random-but-plausible parameters (valid for every CTB) */
typedef struct { int type[3], band[3], eo[3], off[3][4]; } Sao;

static void write_sao(G *g, int rx, int ry, Sao *tab) {
    int ctb = ry * g->ctbW + rx;
    Sao *s = &tab[ctb];
    memset(s, 0, sizeof(*s));
    int bd = g->o.bd, cmax = (1 << ((bd < 10 ? bd : 10) - 5)) - 1;
    if (rx > 0 && g->ctb_slice[ctb - 1] == g->ctb_slice[ctb] && g->tile_id[ctb - 1] == g->tile_id[ctb]) {
        int m = rndn(4) == 0;
        ce_bin(&g->ce, &g->ctx[C_SAO_MERGE], m);
        if (m) { *s = tab[ctb - 1]; return; }
    }
    if (ry > 0 && g->ctb_slice[ctb - g->ctbW] == g->ctb_slice[ctb] && g->tile_id[ctb - g->ctbW] == g->tile_id[ctb]) {
        int m = rndn(4) == 0;
        ce_bin(&g->ce, &g->ctx[C_SAO_MERGE], m);
        if (m) { *s = tab[ctb - g->ctbW]; return; }
    }
    for (int c = 0; c < 3; c++) {
        if (c == 2) { s->type[2] = s->type[1]; s->eo[2] = s->eo[1]; }
        else {
            int t = rndn(3);
            s->type[c] = t;
            ce_bin(&g->ce, &g->ctx[C_SAO_TYPE], t != 0);
            if (t) ce_byp(&g->ce, t == 2);
        }
        if (!s->type[c]) continue;
        int lim = cmax < 3 ? cmax : 3;
        int a[4];
        for (int i = 0; i < 4; i++) {
            a[i] = rndn(lim + 1);
            for (int k = 0; k < a[i]; k++) ce_byp(&g->ce, 1);
            if (a[i] < cmax) ce_byp(&g->ce, 0);
        }
        if (s->type[c] == 1) {
            for (int i = 0; i < 4; i++) {
                int neg = a[i] && rndn(2);
                if (a[i]) ce_byp(&g->ce, neg);
                s->off[c][i] = neg ? -a[i] : a[i];
            }
            s->band[c] = rndn(32);
            ce_bypn(&g->ce, (uint32_t)s->band[c], 5);
        } else {
            s->off[c][0] = a[0]; s->off[c][1] = a[1]; s->off[c][2] = -a[2]; s->off[c][3] = -a[3];
            if (c == 0) { s->eo[0] = rndn(4); ce_bypn(&g->ce, (uint32_t)s->eo[0], 2); }
            if (c == 1) { s->eo[1] = rndn(4); ce_bypn(&g->ce, (uint32_t)s->eo[1], 2); }
        }
    }
}

/* ------------------------------------------------------------ parameter sets */
static void ptl(BW *b, int prof) {
    bw_put(b, 0, 2);          /* profile space */
    bw_put(b, 0, 1);          /* tier */
    bw_put(b, (uint32_t)prof, 5);
    for (int j = 0; j < 32; j++) bw_put(b, (j == prof || (prof == 1 && j == 2)) ? 1 : 0, 1);
    bw_put(b, 1, 1); /* progressive */
    bw_put(b, 0, 1);
    bw_put(b, 0, 1);
    bw_put(b, 1, 1); /* frame only */
    bw_put(b, 0, 32);
    bw_put(b, 0, 11);
    bw_put(b, 0, 1);
    bw_put(b, 123, 8); /* level 4.1 */
}

static void write_vps(FILE *f, int prof, int delay) {
    BW b; bw_init(&b);
    bw_put(&b, 0, 4); bw_put(&b, 1, 1); bw_put(&b, 1, 1); bw_put(&b, 0, 6); bw_put(&b, 0, 3); bw_put(&b, 1, 1);
    bw_put(&b, 0xffff, 16);
    ptl(&b, prof);
    bw_put(&b, 0, 1); /* sub layer ordering info present */
    bw_ue(&b, (uint32_t)(delay ? delay + 1 : 0)); bw_ue(&b, (uint32_t)delay); bw_ue(&b, 0); /* dpb size, reorder, latency */
    bw_put(&b, 0, 6); bw_ue(&b, 0); bw_put(&b, 0, 1); bw_put(&b, 0, 1);
    bw_trailing(&b);
    write_nal(f, 32, b.buf, b.n);
    free(b.buf);
}

static void write_sps(FILE *f, const Opt *o) {
    BW b; bw_init(&b);
    bw_put(&b, 0, 4); bw_put(&b, 0, 3); bw_put(&b, 1, 1);
    ptl(&b, o->profile);
    bw_ue(&b, 0);          /* sps id */
    bw_ue(&b, 1);          /* 4:2:0 */
    bw_ue(&b, (uint32_t)(o->CW - o->wdelta)); /* --wdelta: malformed (not a MinCbSize multiple) */
    bw_ue(&b, (uint32_t)o->CH);
    int crop = o->CW != o->outW || o->CH != o->outH;
    if (o->rawconf[0] >= 0) { /* --conf l,r,t,b: raw conformance_window offsets (malformed-SPS vectors) */
        bw_put(&b, 1, 1);
        for (int i = 0; i < 4; i++) bw_ue(&b, (uint32_t)o->rawconf[i]);
    } else {
        bw_put(&b, (uint32_t)crop, 1);
        if (crop) { bw_ue(&b, 0); bw_ue(&b, (uint32_t)(o->CW - o->outW) / 2); bw_ue(&b, 0); bw_ue(&b, (uint32_t)(o->CH - o->outH) / 2); }
    }
    bw_ue(&b, (uint32_t)(o->bd - 8)); bw_ue(&b, (uint32_t)(o->bd - 8));
    bw_ue(&b, 4);          /* log2_max_poc_lsb - 4 */
    bw_put(&b, 0, 1);      /* sub layer ordering info present */
    bw_ue(&b, (uint32_t)(o->delay ? o->delay + 1 : 0)); bw_ue(&b, (uint32_t)o->delay); bw_ue(&b, 0);
    bw_ue(&b, 0);          /* log2 min cb - 3 */
    bw_ue(&b, (uint32_t)(o->log2ctb - 3));
    bw_ue(&b, 0);          /* log2 min tb - 2 */
    bw_ue(&b, (uint32_t)(o->log2maxtb - 2)); /* max tb */
    bw_ue(&b, 0);          /* depth inter */
    bw_ue(&b, (uint32_t)o->depth);
    bw_put(&b, o->sl != 0, 1); /* scaling_list_enabled_flag */
    if (o->sl) {
        static SList L;
        bw_put(&b, o->sl == 2 || o->sl == 3, 1); /* sps_scaling_list_data_present_flag */
        if (o->sl == 2 || o->sl == 3) write_scaling_list_data(&b, &L);
        else sl_default(&L);
        sl_expand(&L);
    }
    bw_put(&b, 0, 1);      /* amp */
    bw_put(&b, (uint32_t)o->sao, 1);
    bw_put(&b, (uint32_t)o->pcm, 1);
    if (o->pcm) { bw_put(&b, (uint32_t)(o->bd - 1), 4); bw_put(&b, (uint32_t)(o->bd - 1), 4); bw_ue(&b, 0); bw_ue(&b, 1); bw_put(&b, 1, 1); }
    bw_ue(&b, 0);          /* num st rps */
    bw_put(&b, 0, 1);      /* long term */
    bw_put(&b, 0, 1);      /* temporal mvp */
    bw_put(&b, (uint32_t)o->strong, 1);
    bw_put(&b, (uint32_t)o->vui, 1); /* vui_parameters_present_flag */
    if (o->vui) { /* E.2.1 with every optional part present, HRD (E.2.2) with NAL + VCL parameters */
        bw_put(&b, 1, 1); bw_put(&b, 255, 8); bw_put(&b, 4, 16); bw_put(&b, 3, 16); /* EXTENDED_SAR 4:3 */
        bw_put(&b, 1, 1); bw_put(&b, 0, 1);                                         /* overscan */
        bw_put(&b, 1, 1); bw_put(&b, 5, 3); bw_put(&b, 1, 1);                       /* video signal, full range */
        bw_put(&b, 1, 1); bw_put(&b, 1, 8); bw_put(&b, 1, 8); bw_put(&b, 1, 8);     /* BT.709 */
        bw_put(&b, 1, 1); bw_ue(&b, 1); bw_ue(&b, 2);                               /* chroma loc */
        bw_put(&b, 0, 3);
        bw_put(&b, 1, 1); bw_ue(&b, 2); bw_ue(&b, 0); bw_ue(&b, 1); bw_ue(&b, 3);   /* default display window */
        bw_put(&b, 1, 1); bw_put(&b, 1001, 32); bw_put(&b, 60000, 32);              /* timing */
        bw_put(&b, 1, 1); bw_ue(&b, 0);                                             /* poc proportional */
        bw_put(&b, 1, 1);                                                           /* hrd_parameters */
        bw_put(&b, 1, 1); bw_put(&b, 1, 1); bw_put(&b, 1, 1);                       /* nal, vcl, sub_pic */
        bw_put(&b, 23, 8); bw_put(&b, 4, 5); bw_put(&b, 0, 1); bw_put(&b, 6, 5);
        bw_put(&b, 3, 4); bw_put(&b, 5, 4); bw_put(&b, 2, 4);
        bw_put(&b, 23, 5); bw_put(&b, 23, 5); bw_put(&b, 4, 5);
        bw_put(&b, 0, 1); bw_put(&b, 1, 1); bw_ue(&b, 0);                           /* fixed within cvs */
        bw_ue(&b, 1);                                                               /* cpb_cnt_minus1 */
        for (int k = 0; k < 2; k++)
            for (int j = 0; j < 2; j++) { bw_ue(&b, 1000 + j); bw_ue(&b, 2000); bw_ue(&b, 300); bw_ue(&b, 77); bw_put(&b, j, 1); }
        bw_put(&b, 1, 1); bw_put(&b, 5, 3);                                         /* bitstream restriction */
        bw_ue(&b, 0); bw_ue(&b, 2); bw_ue(&b, 1); bw_ue(&b, 15); bw_ue(&b, 15);
    }
    bw_put(&b, o->rext != 0, 1); /* sps_extension_present_flag */
    if (o->rext) {
        bw_put(&b, 1, 1);        /* sps_range_extension_flag */
        bw_put(&b, 0, 7);
        for (int k = 0; k < 9; k++) bw_put(&b, (uint32_t)((o->rext >> k) & 1), 1);
    }
    bw_trailing(&b);
    write_nal(f, 33, b.buf, b.n);
    free(b.buf);
}

static void write_pps(FILE *f, const Opt *o) {
    BW b; bw_init(&b);
    bw_ue(&b, 0); bw_ue(&b, 0);
    bw_put(&b, 0, 1);  /* dependent slices */
    bw_put(&b, 0, 1);  /* output flag */
    bw_put(&b, 0, 3);
    bw_put(&b, (uint32_t)o->sdh, 1);
    bw_put(&b, 0, 1);  /* cabac init present */
    bw_ue(&b, 0); bw_ue(&b, 0);
    bw_se(&b, 0);      /* init qp 26 */
    bw_put(&b, 0, 1);  /* constrained intra */
    bw_put(&b, (uint32_t)o->tskip, 1);
    bw_put(&b, (uint32_t)o->qpdelta, 1);
    if (o->qpdelta) bw_ue(&b, 1);
    bw_se(&b, o->cbqp); bw_se(&b, o->crqp);
    bw_put(&b, 0, 1);  /* slice chroma qp offsets present */
    bw_put(&b, 0, 1); bw_put(&b, 0, 1);
    bw_put(&b, (uint32_t)o->bypass, 1);
    int tiles = o->tile_cols > 1 || o->tile_rows > 1;
    bw_put(&b, (uint32_t)tiles, 1);
    bw_put(&b, (uint32_t)o->wpp, 1);  /* entropy_coding_sync (WPP) */
    if (tiles) {
        bw_ue(&b, (uint32_t)(o->tile_cols - 1));
        bw_ue(&b, (uint32_t)(o->tile_rows - 1));
        bw_put(&b, 1, 1); /* uniform_spacing */
        bw_put(&b, (uint32_t)o->lf_tiles, 1);
    }
    bw_put(&b, 1, 1);  /* loop filter across slices */
    int dfc = o->beta != 0 || o->tc != 0;
    bw_put(&b, (uint32_t)dfc, 1);
    if (dfc) { bw_put(&b, 0, 1); bw_put(&b, 0, 1); bw_se(&b, o->beta); bw_se(&b, o->tc); }
    bw_put(&b, o->sl >= 3, 1); /* pps_scaling_list_data_present_flag */
    if (o->sl >= 3) {
        static SList L;
        write_scaling_list_data(&b, &L);
        sl_expand(&L); /* the PPS lists replace the SPS lists */
    }
    bw_put(&b, 0, 1); bw_ue(&b, 0); bw_put(&b, 0, 1);
    bw_put(&b, (uint32_t)o->ppsext, 1); /* pps_extension_present_flag */
    if (o->ppsext) {
        bw_put(&b, 1, 1); /* pps_range_extension_flag */
        bw_put(&b, 0, 7);
        if (o->tskip) bw_ue(&b, (uint32_t)(o->maxts - 2));
        bw_put(&b, 0, 1); /* cross_component_prediction_enabled_flag */
        bw_put(&b, o->cqo != 0, 1);
        if (o->cqo) {
            bw_ue(&b, (uint32_t)o->cqo_depth); bw_ue(&b, (uint32_t)(o->cqo_len - 1));
            for (int i = 0; i < o->cqo_len; i++) { bw_se(&b, o->cqo_cb[i]); bw_se(&b, o->cqo_cr[i]); }
        }
        bw_ue(&b, (uint32_t)o->sao_scale[0]); bw_ue(&b, (uint32_t)o->sao_scale[1]);
    }
    bw_trailing(&b);
    write_nal(f, 34, b.buf, b.n);
    free(b.buf);
}

/* ------------------------------------------------------------ all-skip P picture (--delay) */
/* One P slice (TRAIL_R) whose CUs are all cu_skip_flag = 1 with MaxNumMergeCand = 1, so the
 * slice data is split_cu_flag / cu_skip_flag / end_of_slice_segment_flag bins only (initType 1
 * contexts, Tables 9-11 / 9-13).  Its short-term RPS references the first picture. */
static void skip_quadtree(G *g, uint8_t *ctx, int x0, int y0, int log2cb, int depth) {
    const int n = 1 << log2cb;
    int split;
    if (x0 + n <= g->o.CW && y0 + n <= g->o.CH && log2cb > 3) {
        int inc = (x0 > 0 && g->ctd[(y0 >> 2) * g->mw + ((x0 - 1) >> 2)] > depth) +
                  (y0 > 0 && g->ctd[((y0 - 1) >> 2) * g->mw + (x0 >> 2)] > depth);
        split = 0;
        ce_bin(&g->ce, &ctx[inc], split);
    } else {
        split = log2cb > 3;
    }
    if (split) {
        int h = n >> 1;
        skip_quadtree(g, ctx, x0, y0, log2cb - 1, depth + 1);
        if (x0 + h < g->o.CW) skip_quadtree(g, ctx, x0 + h, y0, log2cb - 1, depth + 1);
        if (y0 + h < g->o.CH) skip_quadtree(g, ctx, x0, y0 + h, log2cb - 1, depth + 1);
        if (x0 + h < g->o.CW && y0 + h < g->o.CH) skip_quadtree(g, ctx, x0 + h, y0 + h, log2cb - 1, depth + 1);
        return;
    }
    set_map(g, g->ctd, x0, y0, n, (uint8_t)depth);
    ce_bin(&g->ce, &ctx[3 + (x0 > 0) + (y0 > 0)], 1); /* cu_skip_flag: both neighbours skipped */
}

static void write_skip_picture(G *g, FILE *fo, int poc) {
    static const uint8_t init[6] = {107, 139, 126, 197, 185, 201}; /* split_cu_flag, cu_skip_flag (initType 1) */
    uint8_t ctx[6];
    const int qp = g->o.qp;
    for (int i = 0; i < 6; i++) {
        int m = (init[i] >> 4) * 5 - 45, nn = ((init[i] & 15) << 3) - 16;
        int pre = clip3(1, 126, ((m * clip3(0, 51, qp)) >> 4) + nn), mps = pre <= 63 ? 0 : 1;
        ctx[i] = (uint8_t)(((mps ? pre - 64 : 63 - pre) << 1) | mps);
    }
    BW b; bw_init(&b);
    bw_put(&b, 1, 1);  /* first_slice_segment_in_pic_flag */
    bw_ue(&b, 0);      /* pps id */
    bw_ue(&b, 1);      /* P */
    bw_put(&b, (uint32_t)poc, 8);
    bw_put(&b, 0, 1);  /* short_term_ref_pic_set_sps_flag */
    bw_ue(&b, 1); bw_ue(&b, 0); bw_ue(&b, (uint32_t)(poc - 1)); bw_put(&b, 1, 1); /* {POC 0}, used */
    if (g->o.sao) { bw_put(&b, 0, 1); bw_put(&b, 0, 1); }
    bw_put(&b, 0, 1);  /* num_ref_idx_active_override_flag */
    bw_ue(&b, 4);      /* five_minus_max_num_merge_cand */
    bw_se(&b, qp - 26);
    bw_put(&b, 1, 1);  /* slice_loop_filter_across_slices_enabled_flag */
    if (g->o.wpp || g->o.tile_cols > 1 || g->o.tile_rows > 1) { fprintf(stderr, "--delay needs one substream\n"); exit(2); }
    bw_put(&b, 1, 1);  /* byte_alignment */
    bw_align_zero(&b);
    memset(g->ctd, 0, (size_t)g->mw * g->mh);
    ce_start(&g->ce, &b);
    const int nctb = g->ctbW * g->ctbH;
    for (int rs = 0; rs < nctb; rs++) {
        if (g->o.bypass) { fprintf(stderr, "--delay without --bypass\n"); exit(2); }
        skip_quadtree(g, ctx, (rs % g->ctbW) << g->o.log2ctb, (rs / g->ctbW) << g->o.log2ctb, g->o.log2ctb, 0);
        ce_term(&g->ce, rs == nctb - 1);
    }
    ce_finish(&g->ce);
    bw_put(&b, 1, 1);
    bw_align_zero(&b);
    write_nal(fo, 1, b.buf, b.n); /* TRAIL_R */
    free(b.buf);
}

/* ------------------------------------------------------------ main */
static int opt_int(int argc, char **argv, const char *name, int def) {
    for (int i = 1; i + 1 < argc; i++) if (!strcmp(argv[i], name)) return atoi(argv[i + 1]);
    return def;
}
static const char *opt_str(int argc, char **argv, const char *name) {
    for (int i = 1; i + 1 < argc; i++) if (!strcmp(argv[i], name)) return argv[i + 1];
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: hevcgen in.yuv W H bitdepth qp seed out.h265 [options]\n");
        return 2;
    }
    init_tm();
    init_scans();
    G *g = (G *)calloc(1, sizeof(G));
    Opt *o = &g->o;
    o->outW = atoi(argv[2]);
    o->outH = atoi(argv[3]);
    o->bd = atoi(argv[4]);
    o->qp = atoi(argv[5]);
    g_rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)atoll(argv[6]) * 0x100000001B3ull;
    if (!g_rng) g_rng = 1;
    o->sdh = opt_int(argc, argv, "--sdh", 1);
    o->tskip = opt_int(argc, argv, "--tskip", 1);
    o->qpdelta = opt_int(argc, argv, "--qpdelta", 1);
    o->sao = opt_int(argc, argv, "--sao", 1);
    o->pcm = opt_int(argc, argv, "--pcm", 0);
    o->bypass = opt_int(argc, argv, "--bypass", 0);
    o->slice_rows = opt_int(argc, argv, "--slices", 0);
    o->depth = opt_int(argc, argv, "--depth", 1);
    o->beta = opt_int(argc, argv, "--beta", 0);
    o->tc = opt_int(argc, argv, "--tc", 0);
    o->cbqp = opt_int(argc, argv, "--cbqp", 0);
    o->crqp = opt_int(argc, argv, "--crqp", 0);
    o->wpp = opt_int(argc, argv, "--wpp", 0);
    o->tile_cols = opt_int(argc, argv, "--tilecols", 1);
    o->tile_rows = opt_int(argc, argv, "--tilerows", 1);
    o->lf_tiles = opt_int(argc, argv, "--lftiles", 1);
    o->sl = opt_int(argc, argv, "--sl", 0);
    o->nut = opt_int(argc, argv, "--nut", 19);
    o->delay = opt_int(argc, argv, "--delay", 0);
    o->wdelta = opt_int(argc, argv, "--wdelta", 0);
    o->rawconf[0] = -1;
    if (opt_str(argc, argv, "--conf"))
        sscanf(opt_str(argc, argv, "--conf"), "%lld,%lld,%lld,%lld", &o->rawconf[0], &o->rawconf[1], &o->rawconf[2], &o->rawconf[3]);
    o->profile = opt_int(argc, argv, "--profile", o->bd == 8 ? 1 : (o->bd == 10 ? 2 : 4));
    o->vui = opt_int(argc, argv, "--vui", 0);
    o->rext = opt_int(argc, argv, "--rext", 0);
    o->maxts = opt_int(argc, argv, "--maxts", 2);
    o->cqo = opt_int(argc, argv, "--cqo", 0);
    o->cqo_depth = opt_int(argc, argv, "--cqodepth", 1);
    {
        const char *l = opt_str(argc, argv, "--cqolist");
        int v[12], n = 0;
        if (!l) l = "-2,3,4,-1";
        while (n < 12 && sscanf(l, "%d", &v[n]) == 1) {
            n++;
            l = strchr(l, ',');
            if (!l) break;
            l++;
        }
        if (n < 2 || (n & 1)) { fprintf(stderr, "--cqolist wants cb,cr pairs\n"); return 2; }
        o->cqo_len = n / 2;
        for (int i = 0; i < o->cqo_len; i++) { o->cqo_cb[i] = v[2 * i]; o->cqo_cr[i] = v[2 * i + 1]; }
    }
    if (opt_str(argc, argv, "--saoscale")) sscanf(opt_str(argc, argv, "--saoscale"), "%d,%d", &o->sao_scale[0], &o->sao_scale[1]);
    o->ppsext = opt_int(argc, argv, "--ppsext", 0) || o->maxts != 2 || o->cqo || o->sao_scale[0] || o->sao_scale[1];
    /* decoders read the pps_range_extension only for the RExt profile (FFmpeg hevc_ps.c) */
    o->eff_maxts = (o->ppsext && o->profile == 4) ? o->maxts : 2;
    g_sl_on = o->sl != 0;
    o->strong = 1;
    int ctb = opt_int(argc, argv, "--ctb", 64);
    o->log2ctb = ctb == 16 ? 4 : (ctb == 32 ? 5 : 6);
    o->log2maxtb = o->log2ctb < 5 ? o->log2ctb : 5;
    o->CW = (o->outW + 7) & ~7;
    o->CH = (o->outH + 7) & ~7;
    g->qpbd = 6 * (o->bd - 8);
    g->ctbs = 1 << o->log2ctb;
    g->ctbW = (o->CW + g->ctbs - 1) / g->ctbs;
    g->ctbH = (o->CH + g->ctbs - 1) / g->ctbs;
    g->mw = o->CW / 4;
    g->mh = o->CH / 4;
    /* read + pad source */
    FILE *fi = fopen(argv[1], "rb");
    if (!fi) { perror("input"); return 1; }
    for (int c = 0; c < 3; c++) {
        int w = c ? o->CW / 2 : o->CW, h = c ? o->CH / 2 : o->CH;
        int iw = c ? o->outW / 2 : o->outW, ih = c ? o->outH / 2 : o->outH;
        g->st[c] = w;
        g->src[c] = (uint16_t *)calloc((size_t)w * h, 2);
        g->rec[c] = (uint16_t *)calloc((size_t)w * h, 2);
        for (int y = 0; y < ih; y++)
            for (int x = 0; x < iw; x++) {
                int v;
                if (o->bd == 8) { v = fgetc(fi); }
                else { int lo = fgetc(fi), hi = fgetc(fi); v = lo | (hi << 8); }
                if (v < 0) v = 0;
                g->src[c][y * w + x] = (uint16_t)v;
            }
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                int sy = y < ih ? y : ih - 1, sx = x < iw ? x : iw - 1;
                g->src[c][y * w + x] = g->src[c][sy * w + sx];
            }
    }
    fclose(fi);
    size_t m = (size_t)g->mw * g->mh;
    g->qpm = (int8_t *)calloc(m, 1);
    g->ipm = (uint8_t *)calloc(m, 1);
    g->ctd = (uint8_t *)calloc(m, 1);
    int nctb = g->ctbW * g->ctbH;
    g->ctb_slice = (int *)malloc(sizeof(int) * nctb);
    for (int i = 0; i < nctb; i++) g->ctb_slice[i] = -1;
    /* tile scan: uniform column / row boundaries (6.5.1), tiles in raster order, CTBs in
     * raster order inside each tile */
    if (o->tile_cols > g->ctbW) o->tile_cols = g->ctbW;
    if (o->tile_rows > g->ctbH) o->tile_rows = g->ctbH;
    if ((o->tile_cols > 1 || o->tile_rows > 1) && o->slice_rows) { fprintf(stderr, "tiles with --slices unsupported\n"); return 2; }
    g->rs2ts = (int *)malloc(sizeof(int) * nctb);
    g->ts2rs = (int *)malloc(sizeof(int) * nctb);
    g->tile_id = (int *)malloc(sizeof(int) * nctb);
    g->col_bd = (int *)malloc(sizeof(int) * (o->tile_cols + 1));
    {
        int *row_bd = (int *)malloc(sizeof(int) * (o->tile_rows + 1));
        for (int i = 0; i <= o->tile_cols; i++) g->col_bd[i] = i * g->ctbW / o->tile_cols;
        for (int i = 0; i <= o->tile_rows; i++) row_bd[i] = i * g->ctbH / o->tile_rows;
        int ts = 0;
        for (int ty = 0; ty < o->tile_rows; ty++)
            for (int tx = 0; tx < o->tile_cols; tx++)
                for (int y = row_bd[ty]; y < row_bd[ty + 1]; y++)
                    for (int x = g->col_bd[tx]; x < g->col_bd[tx + 1]; x++) {
                        int rs = y * g->ctbW + x;
                        g->rs2ts[rs] = ts;
                        g->ts2rs[ts++] = rs;
                        g->tile_id[rs] = ty * o->tile_cols + tx;
                    }
        free(row_bd);
    }
    g_nodes = (TNode *)malloc(sizeof(TNode) * 128);
    Sao *sao = (Sao *)calloc((size_t)nctb, sizeof(Sao));

    FILE *fo = fopen(argv[7], "wb");
    write_vps(fo, o->profile, o->delay);
    write_sps(fo, o);
    write_pps(fo, o);
    int rows_per_slice = o->slice_rows > 0 ? o->slice_rows : g->ctbH;
    int log2qg = o->log2ctb - 1;
    int nslice = 0;
    for (int r0 = 0; r0 < g->ctbH; r0 += rows_per_slice, nslice++) {
        BW b; bw_init(&b);
        int first = r0 == 0;
        bw_put(&b, (uint32_t)first, 1);
        bw_put(&b, 0, 1); /* no_output_of_prior_pics */
        bw_ue(&b, 0);
        if (!first) {
            int bits = 0;
            while ((1 << bits) < nctb) bits++;
            bw_put(&b, (uint32_t)(r0 * g->ctbW), bits);
        }
        bw_ue(&b, 2); /* I */
        if (o->nut != 19 && o->nut != 20) { /* CRA / BLA: POC lsb + an empty short-term RPS */
            bw_put(&b, 0, 8);               /* slice_pic_order_cnt_lsb */
            bw_put(&b, 0, 1);               /* short_term_ref_pic_set_sps_flag */
            bw_ue(&b, 0); bw_ue(&b, 0);     /* num_negative_pics, num_positive_pics */
        }
        if (o->sao) { bw_put(&b, 1, 1); bw_put(&b, 1, 1); }
        int sqp_delta = 0;
        if (o->qpdelta && nslice > 0) sqp_delta = rndn(5) - 2;
        g->slice_qp = clip3(-g->qpbd, 51, o->qp + sqp_delta);
        bw_se(&b, g->slice_qp - 26);
        if (o->cqo && o->profile == 4) bw_put(&b, o->cqo == 2, 1); /* cu_chroma_qp_offset_enabled_flag */
        g->cqo_on = o->cqo == 2 && o->profile == 4;
        /* pps_loop_filter_across_slices_enabled: signal slice flag */
        if (1) bw_put(&b, (uint32_t)(nslice % 2 == 0), 1);
        /* slice data: one substream per CTB row with WPP (7.3.8.1 end_of_subset_one_bit +
         * byte_alignment; contexts stored after the row's 2nd CTB, 9.3.2.4, and synchronised
         * at the next row's start, 9.3.1), else one */
        int r1 = r0 + rows_per_slice < g->ctbH ? r0 + rows_per_slice : g->ctbH;
        /* CTBs of the slice in decoding (tile-scan) order; a new substream at every tile
         * start and, with WPP, at every CTB row of a tile */
        const int ts0 = r0 * g->ctbW, ts1 = r1 * g->ctbW;
        int nsub = 1, ks = 0;
        for (int ts = ts0 + 1; ts < ts1; ts++) {
            int rs = g->ts2rs[ts], rx = rs % g->ctbW, tc = 0;
            while (rx >= g->col_bd[tc + 1]) tc++;
            if (g->tile_id[rs] != g->tile_id[g->ts2rs[ts - 1]] || (o->wpp && rx == g->col_bd[tc])) nsub++;
        }
        BW *sub = (BW *)calloc((size_t)nsub, sizeof(BW));
        uint8_t wpp_ctx[NUM_CTX];
        int wpp_stat[4] = {0, 0, 0, 0};
        bw_init(&sub[0]);
        init_contexts(g, g->slice_qp);
        ce_start(&g->ce, &sub[0]);
        g->first_qg = 1;
        g->last_cu_qp = g->slice_qp;
        for (int ts = ts0; ts < ts1; ts++) {
            const int rs = g->ts2rs[ts], rx = rs % g->ctbW, ry = rs / g->ctbW;
            int tc = 0;
            while (rx >= g->col_bd[tc + 1]) tc++;
            const int tile_start = ts > ts0 && g->tile_id[rs] != g->tile_id[g->ts2rs[ts - 1]];
            const int row_start = ts > ts0 && o->wpp && rx == g->col_bd[tc];
            if (tile_start || row_start) {
                ce_term(&g->ce, 1); /* end_of_subset_one_bit */
                ce_finish(&g->ce);
                bw_put(&sub[ks], 1, 1);
                bw_align_zero(&sub[ks]);
                bw_init(&sub[++ks]);
                ce_start(&g->ce, &sub[ks]);
                /* 9.3.1: initialise at a tile start; at a WPP row start synchronise with the
                 * contexts after the 2nd CTB of the row above when that CTB is available */
                if (!tile_start && ry > 0 && rx + 1 < g->col_bd[tc + 1] && g->ctb_slice[rs - g->ctbW + 1] == nslice)
                    { memcpy(g->ctx, wpp_ctx, NUM_CTX); memcpy(g->stat, wpp_stat, sizeof(wpp_stat)); }
                else init_contexts(g, g->slice_qp);
                g->first_qg = 1;
                g->last_cu_qp = g->slice_qp; /* qPY_PREV of the first QG (8.6.1) */
            }
            g->ctb_slice[rs] = nslice;
            if (o->sao) write_sao(g, rx, ry, sao);
            coding_quadtree(g, rx << o->log2ctb, ry << o->log2ctb, o->log2ctb, 0, log2qg);
            if (o->wpp && rx == g->col_bd[tc] + 1) { memcpy(wpp_ctx, g->ctx, NUM_CTX); memcpy(wpp_stat, g->stat, sizeof(wpp_stat)); }
            ce_term(&g->ce, ts == ts1 - 1); /* end_of_slice_segment_flag */
        }
        ce_finish(&g->ce);
        bw_put(&sub[ks], 1, 1);
        bw_align_zero(&sub[ks]);
        if (o->wpp || o->tile_cols > 1 || o->tile_rows > 1) {
            /* entry points: substream sizes with their emulation-prevention bytes (every
             * substream ends in a non-zero byte, so each one's escaping is self-contained) */
            uint32_t mx = 1, *sz = (uint32_t *)calloc((size_t)nsub, 4);
            for (int k = 0; k < nsub; k++) {
                int zeros = 0;
                sz[k] = (uint32_t)sub[k].n;
                for (size_t i = 0; i < sub[k].n; i++) {
                    if (zeros >= 2 && sub[k].buf[i] <= 3) { sz[k]++; zeros = 0; }
                    zeros = sub[k].buf[i] == 0 ? zeros + 1 : 0;
                }
                if (k < nsub - 1 && sz[k] > mx) mx = sz[k];
            }
            bw_ue(&b, (uint32_t)(nsub - 1));
            if (nsub > 1) {
                int len = 1;
                while ((1u << len) < mx) len++; /* offsets - 1 fit in len bits */
                bw_ue(&b, (uint32_t)(len - 1));
                for (int k = 0; k < nsub - 1; k++) bw_put(&b, sz[k] - 1, len);
            }
            free(sz);
        }
        bw_put(&b, 1, 1); /* byte_alignment */
        bw_align_zero(&b);
        for (int k = 0; k < nsub; k++) {
            for (size_t i = 0; i < sub[k].n; i++) bw_put(&b, sub[k].buf[i], 8);
            free(sub[k].buf);
        }
        free(sub);
        write_nal(fo, o->nut, b.buf, b.n); /* IDR_W_RADL unless --nut */
        free(b.buf);
    }
    /* decoder delay: delay + 1 trailing P pictures, output order != decoding order */
    for (int k = 1; o->delay && k <= o->delay + 1; k++) write_skip_picture(g, fo, k == 1 ? 2 * (o->delay + 1) : 2 * (k - 1));
    fclose(fo);
    const char *rp = opt_str(argc, argv, "--recon");
    if (rp) {
        FILE *fr = fopen(rp, "wb");
        for (int c = 0; c < 3; c++) {
            int iw = c ? o->outW / 2 : o->outW, ih = c ? o->outH / 2 : o->outH;
            for (int y = 0; y < ih; y++)
                for (int x = 0; x < iw; x++) {
                    uint16_t v = g->rec[c][y * g->st[c] + x];
                    if (o->bd == 8) fputc(v, fr);
                    else { fputc(v & 255, fr); fputc(v >> 8, fr); }
                }
        }
        fclose(fr);
    }
    return 0;
}
