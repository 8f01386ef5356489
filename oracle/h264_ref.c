/*
 * ORACLE — test infrastructure only.  Never linked into the product.
 *
 * Scalar CPU restatement of the H.264 (ITU-T H.264, progressive frames,
 * 4:2:0, 8..10 bit) intra decode the reference performs inside FFmpeg's h264
 * decoder when Decoder::H265ToJpeg calls avcodec_send_packet /
 * avcodec_receive_frame (/root/reference/src/Decoder.cpp:324,342) on the
 * first access unit (:298).  Restates:
 *   7.3 syntax (SPS/PPS/slice header/macroblock layer), 9.3 CABAC (I slices),
 *   8.3 intra prediction (4x4, 8x8 with reference filtering, 16x16, chroma),
 *   8.5 transform decoding (4x4, 8x8, luma/chroma DC), 8.7 deblocking.
 * Pinned by SURVEY.md Appendix B (decoded and pre-deblocking YUV md5 of
 * test/img/img01.h264, Main profile CABAC) and by img01.h264.jpeg.
 * The 8x8 transform / 8x8 CABAC contexts (High profile) are exercised only by
 * generated vectors: parity for those is pinned to this restatement.
 * CAVLC (7.3.5.3.2 / 9.2) with its own hand-typed VLC tables (cavlc_spec.h), checked
 * against the product's generated ones by tests/test_cavlc_tables.py.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bits.h"
#include "cabac_tables.h"
#include "cavlc_spec.h"
#include "oracle.h"

/* ------------------------------------------------------------ CABAC init (I slices) */
static const int8_t k_cabac_init_I[460][2] = {
    /* 0 - 10 */
    {20, -15}, {2, 54}, {3, 74}, {20, -15}, {2, 54}, {3, 74}, {-28, 127}, {-23, 104}, {-6, 53}, {-1, 54}, {7, 51},
    /* 11 - 59: unused in I slices */
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    /* 60 - 69 */
    {0, 41}, {0, 63}, {0, 63}, {0, 63}, {-9, 83}, {4, 86}, {0, 97}, {-7, 72}, {13, 41}, {3, 62},
    /* 70 - 87 */
    {0, 11}, {1, 55}, {0, 69}, {-17, 127}, {-13, 102}, {0, 82}, {-7, 74}, {-21, 107}, {-27, 127}, {-31, 127},
    {-24, 127}, {-18, 95}, {-27, 127}, {-21, 114}, {-30, 127}, {-17, 123}, {-12, 115}, {-16, 122},
    /* 88 - 104 */
    {-11, 115}, {-12, 63}, {-2, 68}, {-15, 84}, {-13, 104}, {-3, 70}, {-8, 93}, {-10, 90}, {-30, 127},
    {-1, 74}, {-6, 97}, {-7, 91}, {-20, 127}, {-4, 56}, {-5, 82}, {-7, 76}, {-22, 125},
    /* 105 - 135 */
    {-7, 93}, {-11, 87}, {-3, 77}, {-5, 71}, {-4, 63}, {-4, 68}, {-12, 84}, {-7, 62}, {-7, 65}, {8, 61},
    {5, 56}, {-2, 66}, {1, 64}, {0, 61}, {-2, 78}, {1, 50}, {7, 52}, {10, 35}, {0, 44}, {11, 38},
    {1, 45}, {0, 46}, {5, 44}, {31, 17}, {1, 51}, {7, 50}, {28, 19}, {16, 33}, {14, 62}, {-13, 108},
    {-15, 100},
    /* 136 - 165 */
    {-13, 101}, {-13, 91}, {-12, 94}, {-10, 88}, {-16, 84}, {-10, 86}, {-7, 83}, {-13, 87}, {-19, 94}, {1, 70},
    {0, 72}, {-5, 74}, {18, 59}, {-8, 102}, {-15, 100}, {0, 95}, {-4, 75}, {2, 72}, {-11, 75}, {-3, 71},
    {15, 46}, {-13, 69}, {0, 62}, {0, 65}, {21, 37}, {-15, 72}, {9, 57}, {16, 54}, {0, 62}, {12, 72},
    /* 166 - 196 */
    {24, 0}, {15, 9}, {8, 25}, {13, 18}, {15, 9}, {13, 19}, {10, 37}, {12, 18}, {6, 29}, {20, 33},
    {15, 30}, {4, 45}, {1, 58}, {0, 62}, {7, 61}, {12, 38}, {11, 45}, {15, 39}, {11, 42}, {13, 44},
    {16, 45}, {12, 41}, {10, 49}, {30, 34}, {18, 42}, {10, 55}, {17, 51}, {17, 46}, {0, 89}, {26, -19},
    {22, -17},
    /* 197 - 226 */
    {26, -17}, {30, -25}, {28, -20}, {33, -23}, {37, -27}, {33, -23}, {40, -28}, {38, -17}, {33, -11}, {40, -15},
    {41, -6}, {38, 1}, {41, 17}, {30, -6}, {27, 3}, {26, 22}, {37, -16}, {35, -4}, {38, -8}, {38, -3},
    {37, 3}, {38, 5}, {42, 0}, {35, 16}, {39, 22}, {14, 48}, {27, 37}, {21, 60}, {12, 68}, {2, 97},
    /* 227 - 251 */
    {-3, 71}, {-6, 42}, {-5, 50}, {-3, 54}, {-2, 62}, {0, 58}, {1, 63}, {-2, 72}, {-1, 74}, {-9, 91},
    {-5, 67}, {-5, 27}, {-3, 39}, {-2, 44}, {0, 46}, {-16, 64}, {-8, 68}, {-10, 78}, {-6, 77}, {-10, 86},
    {-12, 92}, {-15, 55}, {-10, 60}, {-6, 62}, {-4, 65},
    /* 252 - 275 */
    {-12, 73}, {-8, 76}, {-7, 80}, {-9, 88}, {-17, 110}, {-11, 97}, {-20, 84}, {-11, 79}, {-6, 73}, {-4, 74},
    {-13, 86}, {-13, 96}, {-11, 97}, {-19, 117}, {-8, 78}, {-5, 33}, {-4, 48}, {-2, 53}, {-3, 62}, {-13, 71},
    {-10, 79}, {-12, 86}, {-13, 90}, {-14, 97},
    /* 276 (terminate, unused) */
    {0, 0},
    /* 277 - 307 (field coded) */
    {-6, 93}, {-6, 84}, {-8, 79}, {0, 66}, {-1, 71}, {0, 62}, {-2, 60}, {-2, 59}, {-5, 75}, {-3, 62},
    {-4, 58}, {-9, 66}, {-1, 79}, {0, 71}, {3, 68}, {10, 44}, {-7, 62}, {15, 36}, {14, 40}, {16, 27},
    {12, 29}, {1, 44}, {20, 36}, {18, 32}, {5, 42}, {1, 48}, {10, 62}, {17, 46}, {9, 64}, {-12, 104},
    {-11, 97},
    /* 308 - 337 */
    {-16, 96}, {-7, 88}, {-8, 85}, {-7, 85}, {-9, 85}, {-13, 88}, {4, 66}, {-3, 77}, {-3, 76}, {-6, 76},
    {10, 58}, {-1, 76}, {-1, 83}, {-7, 99}, {-14, 95}, {2, 95}, {0, 76}, {-5, 74}, {0, 70}, {-11, 75},
    {1, 68}, {0, 65}, {-14, 73}, {3, 62}, {4, 62}, {-1, 68}, {-13, 75}, {11, 55}, {5, 64}, {12, 70},
    /* 338 - 368 */
    {15, 6}, {6, 19}, {7, 16}, {12, 14}, {18, 13}, {13, 11}, {13, 15}, {15, 16}, {12, 23}, {13, 23},
    {15, 20}, {14, 26}, {14, 44}, {17, 40}, {17, 47}, {24, 17}, {21, 21}, {25, 22}, {31, 27}, {22, 29},
    {19, 35}, {14, 50}, {10, 57}, {7, 63}, {-2, 77}, {-4, 82}, {-3, 94}, {9, 69}, {-12, 109}, {36, -35},
    {36, -34},
    /* 369 - 398 */
    {32, -26}, {37, -30}, {44, -32}, {34, -18}, {34, -15}, {40, -15}, {33, -7}, {35, -5}, {33, 0}, {38, 2},
    {33, 13}, {23, 35}, {13, 58}, {29, -3}, {26, 0}, {22, 30}, {31, -7}, {35, -15}, {34, -3}, {34, 3},
    {36, -1}, {34, 5}, {32, 11}, {35, 5}, {34, 12}, {39, 11}, {30, 29}, {34, 26}, {29, 39}, {19, 66},
    /* 399 - 401 transform_size_8x8_flag */
    {31, 21}, {31, 31}, {25, 50},
    /* 402 - 435 */
    {-17, 120}, {-20, 112}, {-18, 114}, {-11, 85}, {-15, 92}, {-14, 89}, {-26, 71}, {-15, 81}, {-14, 80},
    {0, 68}, {-14, 70}, {-24, 56}, {-23, 68}, {-24, 50}, {-11, 74}, {23, -13}, {26, -13}, {40, -15},
    {49, -14}, {44, 3}, {45, 6}, {44, 34}, {33, 54}, {19, 82}, {-3, 75}, {-1, 23}, {1, 34}, {1, 43},
    {0, 54}, {-2, 55}, {0, 61}, {1, 64}, {0, 68}, {-9, 92},
    /* 436 - 459 */
    {-14, 106}, {-13, 97}, {-15, 90}, {-12, 90}, {-18, 88}, {-10, 73}, {-9, 79}, {-14, 86}, {-10, 73},
    {-10, 70}, {-10, 69}, {-5, 66}, {-9, 64}, {-5, 58}, {2, 59}, {21, -10}, {24, -11}, {28, -8}, {28, -1},
    {29, 3}, {29, 9}, {35, 20}, {29, 36}, {14, 67}};

/* 8x8 significance / last context increments, frame coded (Table 9-43) */
static const uint8_t k_sig8x8[64] = {0,  1,  2,  3,  4,  5,  5,  4,  4,  3,  3,  4,  4,  4,  5,  5,
                                     4,  4,  4,  4,  3,  3,  6,  7,  7,  7,  8,  9,  10, 9,  8,  7,
                                     7,  6,  11, 12, 13, 11, 6,  7,  8,  9,  14, 10, 9,  8,  6,  11,
                                     12, 13, 11, 6,  9,  14, 10, 9,  11, 12, 13, 11, 14, 10, 12};
static const uint8_t k_last8x8[64] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2,
                                      2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4,
                                      4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8, 8};

/* zigzag scans (frame) */
static const uint8_t k_zz4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
/* field scans (Table 8-13 / 8.5.7, field macroblocks): raster index y * n + x per scan position */
static const uint8_t k_fld4[16] = {0, 4, 1, 8, 12, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
static const uint8_t k_fld8[64] = {0,  8,  16, 1,  9,  24, 32, 17, 2,  25, 40, 48, 56, 33, 10, 3,
                                   18, 41, 49, 57, 26, 11, 4,  19, 34, 42, 50, 58, 27, 12, 5,  20,
                                   35, 43, 51, 59, 28, 13, 6,  21, 36, 44, 52, 60, 29, 14, 22, 37,
                                   45, 53, 61, 30, 7,  15, 38, 46, 54, 62, 23, 31, 39, 47, 55, 63};
/* significant_coeff_flag ctxIdxInc of 8x8 blocks in field macroblocks (Table 9-43, field column) */
static const uint8_t k_sig8x8_fld[63] = {0,  1,  1,  2,  2,  3,  3,  4,  5,  6,  7,  7,  7,  8,  4,  5,
                                         6,  9,  10, 10, 8,  11, 12, 11, 9,  9,  10, 10, 8,  11, 12, 11,
                                         9,  9,  10, 10, 8,  11, 12, 11, 9,  9,  10, 10, 8,  13, 13, 9,
                                         9,  10, 10, 8,  13, 13, 9,  9,  10, 10, 14, 14, 14, 14, 14};
static const uint8_t k_zz8[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                  35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                  58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* luma4x4BlkIdx -> (x, y) in 4x4 units */
static const uint8_t k_blk_x[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
static const uint8_t k_blk_y[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};

/* ------------------------------------------------------------ parameter sets */
typedef struct {
    int valid, profile, chroma_format_idc, bit_depth, bit_depth_c;
    int log2_max_frame_num, poc_type, log2_max_poc_lsb, delta_pic_order_always_zero;
    int mb_w, mb_h, frame_mbs_only, mbaff;
    int transform_bypass; /* qpprime_y_zero_transform_bypass_flag */
    int crop_l, crop_r, crop_t, crop_b; /* luma samples */
    int scaling_present;
    uint8_t sl4[6][16], sl8[6][64];
    int sl_flat;
} H4Sps;

typedef struct {
    int valid, sps_id, cabac, bottom_field_pic_order, num_slice_groups;
    int weighted_pred, weighted_bipred, init_qp, chroma_qp_offset, chroma_qp_offset2;
    int deblock_ctrl, constrained_intra, redundant_pic_cnt, transform_8x8;
    int scaling_present;
    uint8_t sl4[6][16], sl8[6][64];
} H4Pps;

static const uint8_t k_def4_intra[16] = {6, 13, 13, 20, 20, 20, 28, 28, 28, 28, 32, 32, 32, 37, 37, 42};
static const uint8_t k_def4_inter[16] = {10, 14, 14, 20, 20, 20, 24, 24, 24, 24, 27, 27, 27, 30, 30, 34};
static const uint8_t k_def8_intra[64] = {
    6,  10, 10, 13, 11, 13, 16, 16, 16, 16, 18, 18, 18, 18, 18, 23, 23, 23, 23, 23, 23, 25,
    25, 25, 25, 25, 25, 25, 27, 27, 27, 27, 27, 27, 27, 27, 29, 29, 29, 29, 29, 29, 29, 31,
    31, 31, 31, 31, 31, 33, 33, 33, 33, 33, 36, 36, 36, 36, 38, 38, 38, 40, 40, 42};
static const uint8_t k_def8_inter[64] = {
    9,  13, 13, 15, 13, 15, 17, 17, 17, 17, 19, 19, 19, 19, 19, 21, 21, 21, 21, 21, 21, 22,
    22, 22, 22, 22, 22, 22, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 27,
    27, 27, 27, 27, 27, 28, 28, 28, 28, 28, 30, 30, 30, 30, 32, 32, 32, 33, 33, 35};

/* scaling_list(): lists stored in zigzag order; fallback rules A/B */
static void parse_sl(OraBits *b, uint8_t *list, int n, const uint8_t *def, const uint8_t *fallback, int present) {
    if (!present) {
        memcpy(list, fallback, (size_t)n);
        return;
    }
    int last = 8, next = 8;
    for (int j = 0; j < n; j++) {
        if (next != 0) {
            int delta = ob_se(b);
            next = (last + delta + 256) % 256;
            if (j == 0 && next == 0) { /* useDefaultScalingMatrixFlag */
                memcpy(list, def, (size_t)n);
                return;
            }
        }
        list[j] = (uint8_t)(next == 0 ? last : next);
        last = list[j];
    }
}

static void parse_matrices(OraBits *b, uint8_t sl4[6][16], uint8_t sl8[6][64], int n8, const uint8_t fb4[6][16],
                           const uint8_t fb8[6][64], int fallback_is_default) {
    static uint8_t flat16[64];
    (void)flat16;
    for (int i = 0; i < 6; i++) {
        int pres = (int)ob_u(b, 1);
        const uint8_t *def = i < 3 ? k_def4_intra : k_def4_inter;
        const uint8_t *fb;
        if (i == 0 || i == 3) fb = fallback_is_default ? def : fb4[i];
        else fb = sl4[i - 1];
        parse_sl(b, sl4[i], 16, def, fb, pres);
    }
    for (int i = 0; i < n8; i++) {
        int pres = (int)ob_u(b, 1);
        const uint8_t *def = (i % 2 == 0) ? k_def8_intra : k_def8_inter;
        const uint8_t *fb;
        if (i < 2) fb = fallback_is_default ? def : fb8[i];
        else fb = sl8[i - 2];
        parse_sl(b, sl8[i], 64, def, fb, pres);
    }
}

/* E.1.1 vui_parameters as far as FFmpeg 4.3 (h264_ps.c decode_vui_parameters /
 * decode_hrd_parameters, behind /root/reference/src/Decoder.cpp:324) can fail the SPS on them:
 * an HRD with cpb_cnt_minus1 > 31 ("cpb_count invalid") or max_num_reorder_frames > 16
 * ("Clipping illegal num_reorder_frames", AVERROR_INVALIDDATA).  A VUI cut short by the end of
 * the SPS counts as no bitstream restriction (FFmpeg resets it).  1 = the SPS fails. */
static int vui_fails(OraBits *b) {
    if (ob_u(b, 1) && ob_u(b, 8) == 255) ob_u(b, 32); /* aspect_ratio_info, Extended_SAR */
    if (ob_u(b, 1)) ob_u(b, 1);                       /* overscan_info */
    if (ob_u(b, 1)) {                                 /* video_signal_type */
        ob_u(b, 4);
        if (ob_u(b, 1)) ob_u(b, 24);                  /* colour description */
    }
    if (ob_u(b, 1)) { ob_ue(b); ob_ue(b); }           /* chroma_loc_info */
    if (ob_u(b, 1)) { ob_u(b, 32); ob_u(b, 32); ob_u(b, 1); } /* timing_info */
    int hrd = 0;
    for (int k = 0; k < 2; k++) {                     /* NAL, then VCL hrd_parameters (E.1.2) */
        if (!ob_u(b, 1)) continue;
        hrd = 1;
        uint32_t cpb_minus1 = ob_ue(b);
        if (cpb_minus1 > 31) return 1;
        ob_u(b, 8);
        for (uint32_t i = 0; i <= cpb_minus1; i++) { ob_ue(b); ob_ue(b); ob_u(b, 1); }
        ob_u(b, 20);
    }
    if (hrd) ob_u(b, 1);                              /* low_delay_hrd_flag */
    ob_u(b, 1);                                       /* pic_struct_present_flag */
    if (!ob_u(b, 1)) return 0;                        /* bitstream_restriction_flag */
    ob_u(b, 1);
    for (int i = 0; i < 4; i++) ob_ue(b);
    uint32_t reorder = ob_ue(b);
    ob_ue(b);                                         /* max_dec_frame_buffering */
    if (b->pos > b->n * 8) return 0;
    return reorder > 16;
}

static int parse_sps(OraBits *b, H4Sps *tab) {
    int profile = (int)ob_u(b, 8);
    ob_u(b, 8);
    ob_u(b, 8);
    int id = (int)ob_ue(b);
    if (id > 31) return -1;
    H4Sps *s = &tab[id];
    memset(s, 0, sizeof(*s));
    s->profile = profile;
    s->chroma_format_idc = 1;
    s->bit_depth = s->bit_depth_c = 8;
    for (int i = 0; i < 6; i++) { memset(s->sl4[i], 16, 16); memset(s->sl8[i], 16, 64); }
    s->sl_flat = 1;
    if (profile == 100 || profile == 110 || profile == 122 || profile == 244 || profile == 44 || profile == 83 ||
        profile == 86 || profile == 118 || profile == 128 || profile == 138 || profile == 139 || profile == 134 ||
        profile == 135) {
        s->chroma_format_idc = (int)ob_ue(b);
        if (s->chroma_format_idc == 3) ob_u(b, 1);
        s->bit_depth = (int)ob_ue(b) + 8;
        s->bit_depth_c = (int)ob_ue(b) + 8;
        s->transform_bypass = (int)ob_u(b, 1); /* qpprime_y_zero_transform_bypass_flag */
        s->scaling_present = (int)ob_u(b, 1);
        if (s->scaling_present) {
            uint8_t fb4[6][16], fb8[6][64];
            parse_matrices(b, s->sl4, s->sl8, s->chroma_format_idc != 3 ? 2 : 6, (const uint8_t(*)[16])fb4,
                           (const uint8_t(*)[64])fb8, 1);
            s->sl_flat = 0;
        }
    }
    s->log2_max_frame_num = (int)ob_ue(b) + 4;
    s->poc_type = (int)ob_ue(b);
    if (s->poc_type == 0) {
        s->log2_max_poc_lsb = (int)ob_ue(b) + 4;
    } else if (s->poc_type == 1) {
        s->delta_pic_order_always_zero = (int)ob_u(b, 1);
        ob_se(b);
        ob_se(b);
        int n = (int)ob_ue(b);
        for (int i = 0; i < n; i++) ob_se(b);
    }
    ob_ue(b); /* max_num_ref_frames */
    ob_u(b, 1);
    s->mb_w = (int)ob_ue(b) + 1;
    s->mb_h = (int)ob_ue(b) + 1; /* map units */
    s->frame_mbs_only = (int)ob_u(b, 1);
    if (!s->frame_mbs_only) s->mbaff = (int)ob_u(b, 1);
    s->mb_h *= 2 - s->frame_mbs_only; /* 7.4.2.1.1: FrameHeightInMbs */
    ob_u(b, 1);                         /* direct_8x8_inference */
    if (ob_u(b, 1)) {
        /* FFmpeg 4.3 h264_ps.c rejects the SPS ("crop values invalid", goto fail) when an
         * offset exceeds INT_MAX / 4 / step or the window leaves no picture (only hevc_ps.c
         * ignores such a window and shows the whole surface) */
        int cx = s->chroma_format_idc == 0 ? 1 : 2, cy = (s->chroma_format_idc == 1 ? 2 : 1) * (2 - s->frame_mbs_only);
        uint64_t cl = ob_ue(b), cr = ob_ue(b), ct = ob_ue(b), cb = ob_ue(b);
        uint64_t lx = 0x7fffffffu / 4 / (unsigned)cx, ly = 0x7fffffffu / 4 / (unsigned)cy;
        if (cl > lx || cr > lx || ct > ly || cb > ly || (cl + cr) * cx >= (uint64_t)s->mb_w * 16 ||
            (ct + cb) * cy >= (uint64_t)s->mb_h * 16)
            return -6;
        s->crop_l = (int)cl * cx;
        s->crop_r = (int)cr * cx;
        s->crop_t = (int)ct * cy;
        s->crop_b = (int)cb * cy;
    }
    if (ob_u(b, 1) && vui_fails(b)) return -7; /* vui_parameters_present_flag */
    if (s->chroma_format_idc != 1 && s->chroma_format_idc != 0) return -4;
    /* FFmpeg 4.3: h264_ps.c fails luma / chroma depths that differ ("Different chroma and luma
     * bit depth") or exceed 14; h264_slice.c get_pixel_format has no 11- or 13-bit format
     * ("Unsupported bit depth") */
    if (s->bit_depth != s->bit_depth_c || s->bit_depth > 14 || s->bit_depth == 11 || s->bit_depth == 13) return -4;
    s->valid = 1;
    return 0;
}

static int parse_pps(OraBits *b, H4Pps *tab, const H4Sps *sps_tab) {
    int id = (int)ob_ue(b);
    if (id > 255) return -1;
    H4Pps *p = &tab[id];
    memset(p, 0, sizeof(*p));
    p->sps_id = (int)ob_ue(b);
    if (p->sps_id > 31) return -1;
    p->cabac = (int)ob_u(b, 1);
    p->bottom_field_pic_order = (int)ob_u(b, 1);
    p->num_slice_groups = (int)ob_ue(b) + 1;
    if (p->num_slice_groups > 1) return -2; /* FMO (Baseline-only) out of scope */
    ob_ue(b);
    ob_ue(b);
    p->weighted_pred = (int)ob_u(b, 1);
    p->weighted_bipred = (int)ob_u(b, 2);
    p->init_qp = 26 + ob_se(b);
    ob_se(b);
    p->chroma_qp_offset = ob_se(b);
    p->deblock_ctrl = (int)ob_u(b, 1);
    p->constrained_intra = (int)ob_u(b, 1);
    p->redundant_pic_cnt = (int)ob_u(b, 1);
    p->chroma_qp_offset2 = p->chroma_qp_offset;
    const H4Sps *s = &sps_tab[p->sps_id];
    for (int i = 0; i < 6; i++) { memcpy(p->sl4[i], s->sl4[i], 16); memcpy(p->sl8[i], s->sl8[i], 64); }
    p->scaling_present = 0;
    if (ob_more_rbsp(b)) {
        p->transform_8x8 = (int)ob_u(b, 1);
        p->scaling_present = (int)ob_u(b, 1);
        if (p->scaling_present) {
            /* fallback rule B when the SPS carried matrices, A otherwise */
            uint8_t fb4[6][16], fb8[6][64];
            memcpy(fb4, s->sl4, sizeof(fb4));
            memcpy(fb8, s->sl8, sizeof(fb8));
            parse_matrices(b, p->sl4, p->sl8, p->transform_8x8 ? (s->chroma_format_idc != 3 ? 2 : 6) : 0,
                           (const uint8_t(*)[16])fb4, (const uint8_t(*)[64])fb8, !s->scaling_present);
        }
        p->chroma_qp_offset2 = ob_se(b);
    }
    p->valid = 1;
    return 0;
}

/* ------------------------------------------------------------ decoder state */
enum { MB_I_NXN = 0, MB_I_PCM = 25 };

typedef struct {
    int slice;          /* slice number, -1 = not decoded */
    int mb_type;        /* 0 NxN, 1..24 I16x16, 25 PCM */
    int t8x8;
    int cbp;            /* bits 0-3 luma, bits 4-5 chroma (0..2) */
    int qp;             /* QPY */
    int cpm;            /* intra_chroma_pred_mode */
    int qpd_nz;         /* mb_qp_delta != 0 */
    uint8_t ipm[16];    /* Intra4x4/8x8 pred modes per 4x4 block (2 for non-NxN) */
    uint8_t cbf[16];    /* luma 4x4 coded_block_flag (8x8: replicated) */
    uint8_t cbf_c[2][4];/* chroma AC */
    uint8_t cbf_dc[3];  /* luma DC (I16x16), Cb DC, Cr DC */
    uint8_t tc[16];     /* CAVLC: TotalCoeff of each luma 4x4 block (I16x16: AC block) */
    uint8_t tcc[2][4];  /* CAVLC: TotalCoeff of each chroma AC block */
    int field;          /* MBAFF: mb_field_decoding_flag of the macroblock's pair */
    int vx, vy;         /* position in the macroblock grid (MBAFF: vy = 2 * pair row + bottom) */
} MbInfo;

typedef struct {
    int disable_deblock, alpha_off, beta_off; /* *2 */
    int chroma_qp_offset, chroma_qp_offset2;
} H4Slice;

typedef struct {
    H4Sps sps[32];
    H4Pps pps[256];
    const H4Sps *s;
    const H4Pps *p;
    int W, H, mbw, mbh, bd, bdc, qpbd, qpbdc;
    int mbaff; /* MbaffFrameFlag: macroblock pairs; MbInfo at (vx, vy = 2 * pair row + bottom) */
    int cur_field; /* mb_field_decoding_flag of the pair being decoded */
    /* PAFF: picture 0 is a field pair (field_pic_flag 1), held in the MBAFF layout as all-field pairs
     * (field MB (x, fy) of parity f at grid (x, 2 fy + f)); neighbours stay inside a field
     * (6.4.12.1 on the field's MB grid) */
    int paff, parity, fields_seen;
    /* 4:0:0 (chroma_format_idc 0, High profiles): no chroma syntax; FFmpeg (h264_cabac.c /
     * h264_cavlc.c decode_chroma = 0) predicts both chroma blocks with DC_128_PRED8x8 and writes
     * 1 << (BitDepth - 1) for I_PCM, into a yuv420p frame */
    int mono;
    uint16_t *pl[3];
    int st[3];
    MbInfo *mb;
    H4Slice sl[256];
    int nslice;
    /* slice decode */
    OraCabac cc;
    OraBits bits;
    uint8_t ctx[460];
    int qp, prev_qpd_nz;
    int mbx, mby;
    int lvl4[16][16];  /* per 4x4 block, raster coeffs */
    int lvl8[4][64];
    int dc_l[16];
    int dc_c[2][4];
    int ac_c[2][4][16];
} H4Dec;

static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

static void init_ctx(H4Dec *d, int qp) {
    for (int i = 0; i < 460; i++) {
        int m = k_cabac_init_I[i][0], n = k_cabac_init_I[i][1];
        int pre = clip3(1, 126, ((m * clip3(0, 51, qp)) >> 4) + n);
        int mps = pre <= 63 ? 0 : 1;
        d->ctx[i] = (uint8_t)(((mps ? pre - 64 : 63 - pre) << 1) | mps);
    }
}
static inline int bin(H4Dec *d, int ctx) { return oc_decision(&d->cc, &d->ctx[ctx]); }
static inline int byp(H4Dec *d) { return oc_bypass(&d->cc); }

/* the macroblock at grid position (x, y) if it is decoded in the current slice */
static MbInfo *mb_in_slice(H4Dec *d, int x, int y) {
    if (x < 0 || y < 0 || x >= d->mbw || y >= d->mbh) return NULL;
    MbInfo *m = &d->mb[y * d->mbw + x];
    MbInfo *c = &d->mb[d->mby * d->mbw + d->mbx];
    return (m->slice < 0 || m->slice != c->slice) ? NULL : m;
}

/* 6.4.12: the macroblock covering location (xN, yN) relative to the current macroblock's
 * upper-left sample (maxW x maxH: 16 x 16 luma, 8 x 8 chroma) and the location (xW, yW) inside
 * it; NULL when not available.  Non-MBAFF: 6.4.12.1 (raster neighbours, decoding order).  MBAFF:
 * 6.4.12.2 -- pairs A / B / C / D left / above / above-right / above-left, then Table 6-4. */
static MbInfo *nb_loc(H4Dec *d, int xN, int yN, int maxW, int maxH, int *xW, int *yW) {
    MbInfo *cur = &d->mb[d->mby * d->mbw + d->mbx];
    if (yN > maxH - 1 || (xN > maxW - 1 && yN >= 0)) return NULL;
    *xW = (xN + maxW) % maxW;
    if (!d->mbaff || d->paff) {
        int dx = xN < 0 ? -1 : (xN > maxW - 1 ? 1 : 0), dy = yN < 0 ? -1 : 0;
        *yW = (yN + maxH) % maxH;
        if (dx == 0 && dy == 0) return cur;
        return mb_in_slice(d, d->mbx + dx, d->mby + (d->paff ? 2 * dy : dy)); /* PAFF: same field */
    }
    const int px = d->mbx, py = d->mby >> 1, top = !(d->mby & 1), frame = !cur->field;
    MbInfo *X = NULL, *N = NULL; /* X: top MB of the neighbouring pair */
    int yM = yN, bot = 0;        /* N = X (bot 0) or X's bottom MB (bot 1) */
    if (xN >= 0 && xN <= maxW - 1 && yN >= 0) {
        *yW = yN;
        return cur;
    }
    if (xN < 0 && yN < 0) { /* D */
        if (frame && !top) {
            /* a bottom frame MB's upper-left neighbour: the left pair's top frame MB, last row, or
             * -- left field pair -- its bottom field MB's middle row (the picture sample above-left;
             * FFmpeg fill_decode_neighbors: topleft_xy += mb_stride, "take top left ... from the
             * middle of the mb") */
            X = mb_in_slice(d, px - 1, 2 * py);
            if (!X) return NULL;
            bot = X->field ? 1 : 0;
            yM = X->field ? (yN + maxH) >> 1 : yN;
        } else if (frame || !top) {
            X = mb_in_slice(d, px - 1, 2 * py - 2);
            bot = 1;
        } else {
            X = mb_in_slice(d, px - 1, 2 * py - 2);
            if (!X) return NULL;
            if (X->field) bot = 0; else { bot = 1; yM = 2 * yN; }
        }
    } else if (xN < 0) { /* A, 0 <= yN <= maxH - 1 */
        X = mb_in_slice(d, px - 1, 2 * py);
        if (!X) return NULL;
        if (frame) {
            if (top) {
                if (!X->field) { bot = 0; yM = yN; }
                else { bot = yN & 1; yM = yN >> 1; }
            } else {
                if (!X->field) { bot = 1; yM = yN; }
                else { bot = yN & 1; yM = (yN + maxH) >> 1; }
            }
        } else {
            if (top) {
                if (!X->field) { if (yN < maxH / 2) { bot = 0; yM = yN << 1; } else { bot = 1; yM = (yN << 1) - maxH; } }
                else { bot = 0; yM = yN; }
            } else {
                if (!X->field) { if (yN < maxH / 2) { bot = 0; yM = (yN << 1) + 1; } else { bot = 1; yM = (yN << 1) + 1 - maxH; } }
                else { bot = 1; yM = yN; }
            }
        }
    } else if (xN <= maxW - 1) { /* B, yN < 0 */
        if (frame && !top) {
            X = &d->mb[(2 * py) * d->mbw + px]; /* CurrMbAddr - 1: the pair's top MB */
            bot = 0;
        } else if (frame || !top) {
            X = mb_in_slice(d, px, 2 * py - 2);
            bot = 1;
        } else {
            X = mb_in_slice(d, px, 2 * py - 2);
            if (!X) return NULL;
            if (X->field) bot = 0; else { bot = 1; yM = 2 * yN; }
        }
    } else { /* C, yN < 0 */
        if (frame && !top) return NULL;
        if (frame || !top) {
            X = mb_in_slice(d, px + 1, 2 * py - 2);
            bot = 1;
        } else {
            X = mb_in_slice(d, px + 1, 2 * py - 2);
            if (!X) return NULL;
            if (X->field) bot = 0; else { bot = 1; yM = 2 * yN; }
        }
    }
    if (!X) return NULL;
    N = &d->mb[(X->vy + bot) * d->mbw + X->vx];
    *yW = (yM + maxH) % maxH;
    return N;
}

/* neighbouring MB (A left, B top, C top-right, D top-left): the MB covering luma location
 * (-1, 0) / (0, -1) / (16, -1) / (-1, -1) (6.4.11.1) */
static MbInfo *nb_mb(H4Dec *d, int dx, int dy) {
    int xW, yW;
    return nb_loc(d, dx < 0 ? -1 : (dx > 0 ? 16 : 0), dy < 0 ? -1 : 0, 16, 16, &xW, &yW);
}

static const uint8_t k_blk_of[4][4] = {{0, 1, 4, 5}, {2, 3, 6, 7}, {8, 9, 12, 13}, {10, 11, 14, 15}};
/* neighbour 4x4 luma block (6.4.11.4): the block covering luma location (4 bx, 4 by) relative to
 * the current MB (bx, by in 4x4 units, may be -1 / 4); returns the MB and the block index */
static MbInfo *nb_blk(H4Dec *d, int bx, int by, int *nblk) {
    int xW, yW;
    MbInfo *m = nb_loc(d, bx * 4, by * 4, 16, 16, &xW, &yW);
    *nblk = m ? k_blk_of[yW >> 2][xW >> 2] : 0;
    return m;
}

/* picture position of sample (xW, yW) of component c of macroblock N (MBAFF field macroblocks
 * interleave the rows of their pair: top field even rows, bottom field odd rows) */
static void mb_phys(const H4Dec *d, const MbInfo *N, int c, int xW, int yW, int *X, int *Y) {
    const int S = c ? 8 : 16;
    *X = N->vx * S + xW;
    if (!d->mbaff) { *Y = N->vy * S + yW; return; }
    const int py = N->vy >> 1, bot = N->vy & 1;
    *Y = N->field ? 2 * py * S + 2 * yW + bot : (2 * py + bot) * S + yW;
}
/* sample store of the current macroblock at grid position (x, y) of component c */
static void put_sample(H4Dec *d, int c, int x, int y, int v) {
    const int S = c ? 8 : 16;
    int X, Y;
    mb_phys(d, &d->mb[d->mby * d->mbw + d->mbx], c, x - d->mbx * S, y - d->mby * S, &X, &Y);
    d->pl[c][Y * d->st[c] + X] = (uint16_t)v;
}

/* ------------------------------------------------------------ CABAC syntax elements */
static int dec_mb_type_I(H4Dec *d) {
    MbInfo *A = nb_mb(d, -1, 0), *B = nb_mb(d, 0, -1);
    int ctx = (A && A->mb_type != MB_I_NXN) + (B && B->mb_type != MB_I_NXN);
    if (!bin(d, 3 + ctx)) return 0;
    if (oc_terminate(&d->cc)) return 25;
    int t = 1;
    t += 12 * bin(d, 6);
    if (bin(d, 7)) t += 4 + 4 * bin(d, 8);
    t += 2 * bin(d, 9);
    t += bin(d, 10);
    return t;
}

static int dec_cbp(H4Dec *d) {
    MbInfo *cur = &d->mb[d->mby * d->mbw + d->mbx];
    (void)cur;
    int cbp = 0;
    for (int b8 = 0; b8 < 4; b8++) {
        int bx = (b8 & 1) * 2, by = (b8 >> 1) * 2;
        int ca, cb;
        /* left / upper neighbour 8x8 block (6.4.11.2: the block covering luma location
         * (x - 1, y) / (x, y - 1); MBAFF through Table 6-4) */
        int xW, yW;
        if (bx == 0) {
            MbInfo *A = nb_loc(d, -1, by * 4, 16, 16, &xW, &yW);
            ca = A ? (A->mb_type == MB_I_PCM ? 0 : !((A->cbp >> ((yW >> 3) * 2 + (xW >> 3))) & 1)) : 0;
        } else {
            ca = !((cbp >> (b8 - 1)) & 1);
        }
        if (by == 0) {
            MbInfo *B = nb_loc(d, bx * 4, -1, 16, 16, &xW, &yW);
            cb = B ? (B->mb_type == MB_I_PCM ? 0 : !((B->cbp >> ((yW >> 3) * 2 + (xW >> 3))) & 1)) : 0;
        } else {
            cb = !((cbp >> (b8 - 2)) & 1);
        }
        cbp |= bin(d, 73 + ca + 2 * cb) << b8;
    }
    if (d->mono) return cbp; /* no CodedBlockPatternChroma bins (9.3.2.4) */
    MbInfo *A = nb_mb(d, -1, 0), *B = nb_mb(d, 0, -1);
    int ac = A ? (A->mb_type == MB_I_PCM ? 2 : (A->cbp >> 4)) : 0;
    int bc = B ? (B->mb_type == MB_I_PCM ? 2 : (B->cbp >> 4)) : 0;
    int ctx = (ac > 0) + 2 * (bc > 0);
    if (bin(d, 77 + ctx)) {
        ctx = 4 + (ac == 2) + 2 * (bc == 2);
        cbp |= (1 + bin(d, 77 + ctx)) << 4;
    }
    return cbp;
}

static int dec_qp_delta(H4Dec *d) {
    int ctx = d->prev_qpd_nz ? 1 : 0;
    int k = 0;
    if (bin(d, 60 + ctx)) {
        k = 1;
        ctx = 2;
        while (bin(d, 60 + ctx)) {
            ctx = 3;
            k++;
            if (k > 200) break;
        }
    }
    return (k & 1) ? (k + 1) / 2 : -(k / 2);
}

static int dec_chroma_pred(H4Dec *d) {
    MbInfo *A = nb_mb(d, -1, 0), *B = nb_mb(d, 0, -1);
    int ctx = (A && A->mb_type != MB_I_PCM && A->cpm != 0) + (B && B->mb_type != MB_I_PCM && B->cpm != 0);
    if (!bin(d, 64 + ctx)) return 0;
    if (!bin(d, 67)) return 1;
    return bin(d, 67) ? 3 : 2;
}

/* coded_block_flag ctxIdxInc condition for a neighbour */
static int cbf_cond(H4Dec *d, int cat, MbInfo *N, int nblk, int icbcr) {
    if (!N) return 1; /* unavailable, current MB intra */
    if (N->mb_type == MB_I_PCM) return 1;
    switch (cat) {
    case 0: return N->mb_type >= 1 && N->mb_type <= 24 ? N->cbf_dc[0] : 0;
    case 1:
    case 2:
        if (!((N->cbp >> (nblk >> 2)) & 1)) return 0;
        return N->cbf[nblk];
    case 3: return (N->cbp >> 4) ? N->cbf_dc[1 + icbcr] : 0;
    case 4: return (N->cbp >> 4) == 2 ? N->cbf_c[icbcr][nblk] : 0;
    }
    (void)d;
    return 0;
}

/* residual_block_cabac: coeffs in scan order into out[0..maxNum-1]; returns coded flag */
static int residual_block(H4Dec *d, int cat, int cbf_inc, int maxNum, int *out) {
    static const int cbf_off[5] = {0, 4, 8, 12, 16};
    static const int sig_off[6] = {0, 15, 29, 44, 47, 0};
    static const int abs_off[6] = {0, 10, 20, 30, 39, 0};
    memset(out, 0, sizeof(int) * maxNum);
    /* field macroblocks (MBAFF): significant / last contexts at ctxIdxOffset 277 / 338 (cat < 5)
     * and 436 / 451 with the field ctxIdxInc table (cat 5) instead of 105 / 166, 402 / 417 */
    const int fld = d->mb[d->mby * d->mbw + d->mbx].field;
    const int sig0 = fld ? 277 : 105, last0 = fld ? 338 : 166;
    if (cat != 5) {
        if (!bin(d, 85 + cbf_off[cat] + cbf_inc)) return 0;
    }
    int sig[64], nsig = 0;
    int last = -1;
    int i;
    for (i = 0; i < maxNum - 1; i++) {
        int sctx, lctx;
        if (cat == 5) {
            sctx = fld ? 436 + k_sig8x8_fld[i] : 402 + k_sig8x8[i];
            lctx = (fld ? 451 : 417) + k_last8x8[i];
        } else if (cat == 3) {
            int inc = i < 2 ? i : 2; /* Min(i / NumC8x8, 2), 4:2:0 */
            sctx = sig0 + sig_off[cat] + inc;
            lctx = last0 + sig_off[cat] + inc;
        } else {
            sctx = sig0 + sig_off[cat] + i;
            lctx = last0 + sig_off[cat] + i;
        }
        if (bin(d, sctx)) {
            sig[nsig++] = i;
            if (bin(d, lctx)) {
                last = i;
                break;
            }
        }
    }
    if (last < 0) sig[nsig++] = maxNum - 1;
    int eq1 = 0, gt1 = 0;
    int absb = cat == 5 ? 426 : 227 + abs_off[cat];
    for (int k = nsig - 1; k >= 0; k--) {
        int inc = gt1 ? 0 : (eq1 + 1 < 4 ? eq1 + 1 : 4);
        int v;
        if (!bin(d, absb + inc)) {
            v = 1;
        } else {
            int inc2 = 5 + (gt1 < (4 - (cat == 3)) ? gt1 : (4 - (cat == 3)));
            int p = 1;
            while (p < 14 && bin(d, absb + inc2)) p++;
            v = p + 1;
            if (p == 14) { /* UEG0 suffix */
                int kk = 0;
                while (byp(d)) {
                    v += 1 << kk;
                    kk++;
                    if (kk > 20) break;
                }
                while (kk--) v += byp(d) << kk;
            }
        }
        if (v == 1) eq1++;
        else gt1++;
        out[sig[k]] = byp(d) ? -v : v;
    }
    return 1;
}

/* ------------------------------------------------------------ dequant / transforms */
static const int k_norm4[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
static const int k_norm8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                                  {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
static int norm4(int m, int i, int j) {
    if ((i & 1) == 0 && (j & 1) == 0) return k_norm4[m][0];
    if ((i & 1) == 1 && (j & 1) == 1) return k_norm4[m][1];
    return k_norm4[m][2];
}
static int norm8(int m, int i, int j) {
    if ((i & 3) == 0 && (j & 3) == 0) return k_norm8[m][0];
    if ((i & 1) == 1 && (j & 1) == 1) return k_norm8[m][1];
    if ((i & 3) == 2 && (j & 3) == 2) return k_norm8[m][2];
    if (((i & 3) == 0 && (j & 1) == 1) || ((i & 1) == 1 && (j & 3) == 0)) return k_norm8[m][3];
    if (((i & 3) == 0 && (j & 3) == 2) || ((i & 3) == 2 && (j & 3) == 0)) return k_norm8[m][4];
    return k_norm8[m][5];
}

/* weightScale in raster order from zigzag list */
static int ws4(const uint8_t *zzlist, int pos /* raster */) {
    for (int k = 0; k < 16; k++)
        if (k_zz4[k] == pos) return zzlist[k];
    return 16;
}
static int ws8(const uint8_t *zzlist, int pos) {
    for (int k = 0; k < 64; k++)
        if (k_zz8[k] == pos) return zzlist[k];
    return 16;
}

static void idct4(int *b) { /* in place, raster 4x4: rows then columns, then (x+32)>>6 */
    int t[16];
    for (int i = 0; i < 4; i++) {
        int *r = b + i * 4;
        int e0 = r[0] + r[2], e1 = r[0] - r[2], e2 = (r[1] >> 1) - r[3], e3 = r[1] + (r[3] >> 1);
        t[i * 4 + 0] = e0 + e3; t[i * 4 + 1] = e1 + e2; t[i * 4 + 2] = e1 - e2; t[i * 4 + 3] = e0 - e3;
    }
    for (int j = 0; j < 4; j++) {
        int f0 = t[j], f1 = t[4 + j], f2 = t[8 + j], f3 = t[12 + j];
        int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        b[j] = (g0 + g3 + 32) >> 6;
        b[4 + j] = (g1 + g2 + 32) >> 6;
        b[8 + j] = (g1 - g2 + 32) >> 6;
        b[12 + j] = (g0 - g3 + 32) >> 6;
    }
}

static void idct8_1d(const int *d, int *o) {
    int a0 = d[0] + d[4], a4 = d[0] - d[4], a2 = (d[2] >> 1) - d[6], a6 = d[2] + (d[6] >> 1);
    int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
    int a1 = -d[3] + d[5] - d[7] - (d[7] >> 1), a3 = d[1] + d[7] - d[3] - (d[3] >> 1);
    int a5 = -d[1] + d[7] + d[5] + (d[5] >> 1), a7 = d[3] + d[5] + d[1] + (d[1] >> 1);
    int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
    o[0] = b0 + b7; o[1] = b2 + b5; o[2] = b4 + b3; o[3] = b6 + b1;
    o[4] = b6 - b1; o[5] = b4 - b3; o[6] = b2 - b5; o[7] = b0 - b7;
}
static void idct8(int *b) {
    int t[64], col[8], o[8];
    for (int i = 0; i < 8; i++) idct8_1d(b + i * 8, t + i * 8);
    for (int j = 0; j < 8; j++) {
        for (int i = 0; i < 8; i++) col[i] = t[i * 8 + j];
        idct8_1d(col, o);
        for (int i = 0; i < 8; i++) b[i * 8 + j] = (o[i] + 32) >> 6;
    }
}

static int chroma_qp(int qpi) {
    static const int t[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
    return qpi < 30 ? qpi : t[qpi - 30];
}

/* ------------------------------------------------------------ intra prediction */
/* sample availability for intra prediction: luma location (x,y) relative to
 * the current MB origin in samples; returns availability of the neighbour
 * sample given the current 4x4/8x8 block index order */
static int avail_luma(H4Dec *d, int x, int y, int cur_blk4) {
    /* x,y in [-1, 31] relative to MB */
    if (y < 0 && x < 0) return nb_mb(d, -1, -1) != NULL;
    if (y < 0 && x >= 16) return nb_mb(d, 1, -1) != NULL;
    if (y < 0) return nb_mb(d, 0, -1) != NULL;
    if (x < 0) return nb_mb(d, -1, 0) != NULL;
    if (x >= 16) return 0;
    /* inside current MB: decoded if its 4x4 block index precedes */
    static const uint8_t blk_of[4][4] = {{0, 1, 4, 5}, {2, 3, 6, 7}, {8, 9, 12, 13}, {10, 11, 14, 15}};
    int b = blk_of[y >> 2][x >> 2];
    return b < cur_blk4;
}

/* sample at grid position (x, y) of component c, seen from the current macroblock (MBAFF: through
 * the 6.4.12.2 neighbour mapping, e.g. a field MB's row above is the row two picture rows up);
 * callers read only positions they found available */
static int px(H4Dec *d, int c, int x, int y) {
    if (!d->mbaff) return d->pl[c][y * d->st[c] + x];
    const int S = c ? 8 : 16;
    int xW, yW, X, Y;
    MbInfo *N = nb_loc(d, x - d->mbx * S, y - d->mby * S, S, S, &xW, &yW);
    if (!N) return 0;
    mb_phys(d, N, c, xW, yW, &X, &Y);
    return d->pl[c][Y * d->st[c] + X];
}

static void pred4x4(H4Dec *d, int blk, int mode, int *pred) {
    int x0 = k_blk_x[blk] * 4, y0 = k_blk_y[blk] * 4;
    int gx = d->mbx * 16 + x0, gy = d->mby * 16 + y0;
    int T[8], L[4], Cn;
    int at = avail_luma(d, x0, y0 - 1, blk), al = avail_luma(d, x0 - 1, y0, blk);
    int ad = avail_luma(d, x0 - 1, y0 - 1, blk);
    int atr = avail_luma(d, x0 + 4, y0 - 1, blk);
    if (blk == 3 || blk == 7 || blk == 11 || blk == 13 || blk == 15 || blk == 5) {
        if (blk != 5) atr = 0;
    }
    for (int i = 0; i < 4; i++) {
        T[i] = at ? px(d, 0, gx + i, gy - 1) : 0;
        L[i] = al ? px(d, 0, gx - 1, gy + i) : 0;
    }
    for (int i = 4; i < 8; i++) T[i] = atr ? px(d, 0, gx + i, gy - 1) : T[3];
    Cn = ad ? px(d, 0, gx - 1, gy - 1) : 0;
    int bd = d->bd;
#define P(x, y) pred[(y) * 4 + (x)]
    switch (mode) {
    case 0: for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) P(x, y) = T[x]; break;
    case 1: for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) P(x, y) = L[y]; break;
    case 2: {
        int s;
        if (at && al) s = (T[0] + T[1] + T[2] + T[3] + L[0] + L[1] + L[2] + L[3] + 4) >> 3;
        else if (al) s = (L[0] + L[1] + L[2] + L[3] + 2) >> 2;
        else if (at) s = (T[0] + T[1] + T[2] + T[3] + 2) >> 2;
        else s = 1 << (bd - 1);
        for (int i = 0; i < 16; i++) pred[i] = s;
        break;
    }
    case 3:
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++)
                P(x, y) = (x == 3 && y == 3) ? (T[6] + 3 * T[7] + 2) >> 2 : (T[x + y] + 2 * T[x + y + 1] + T[x + y + 2] + 2) >> 2;
        break;
    case 4:
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int v;
                if (x > y) { int a = x - y; v = ((a - 2 >= 0 ? T[a - 2] : Cn) + 2 * T[a - 1] + T[a] + 2) >> 2; }
                else if (x < y) { int a = y - x; v = ((a - 2 >= 0 ? L[a - 2] : Cn) + 2 * L[a - 1] + L[a] + 2) >> 2; }
                else v = (T[0] + 2 * Cn + L[0] + 2) >> 2;
                P(x, y) = v;
            }
        break;
    case 5:
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int z = 2 * x - y, v;
                if (z >= 0 && (z & 1) == 0) v = ((x - (y >> 1) - 1 >= 0 ? T[x - (y >> 1) - 1] : Cn) + T[x - (y >> 1)] + 1) >> 1;
                else if (z >= 0) v = ((x - (y >> 1) - 2 >= 0 ? T[x - (y >> 1) - 2] : Cn) + 2 * (x - (y >> 1) - 1 >= 0 ? T[x - (y >> 1) - 1] : Cn) + T[x - (y >> 1)] + 2) >> 2;
                else if (z == -1) v = (L[0] + 2 * Cn + T[0] + 2) >> 2;
                else v = (L[y - 1] + 2 * L[y - 2] + (y - 3 >= 0 ? L[y - 3] : Cn) + 2) >> 2;
                P(x, y) = v;
            }
        break;
    case 6:
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int z = 2 * y - x, v;
                if (z >= 0 && (z & 1) == 0) v = ((y - (x >> 1) - 1 >= 0 ? L[y - (x >> 1) - 1] : Cn) + L[y - (x >> 1)] + 1) >> 1;
                else if (z >= 0) v = ((y - (x >> 1) - 2 >= 0 ? L[y - (x >> 1) - 2] : Cn) + 2 * (y - (x >> 1) - 1 >= 0 ? L[y - (x >> 1) - 1] : Cn) + L[y - (x >> 1)] + 2) >> 2;
                else if (z == -1) v = (L[0] + 2 * Cn + T[0] + 2) >> 2;
                else v = (T[x - 1] + 2 * T[x - 2] + (x - 3 >= 0 ? T[x - 3] : Cn) + 2) >> 2;
                P(x, y) = v;
            }
        break;
    case 7:
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int i = x + (y >> 1);
                P(x, y) = (y & 1) == 0 ? (T[i] + T[i + 1] + 1) >> 1 : (T[i] + 2 * T[i + 1] + T[i + 2] + 2) >> 2;
            }
        break;
    case 8:
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int z = x + 2 * y, v;
                if (z > 5) v = L[3];
                else if (z == 5) v = (L[2] + 3 * L[3] + 2) >> 2;
                else if ((z & 1) == 0) v = (L[y + (x >> 1)] + L[y + (x >> 1) + 1] + 1) >> 1;
                else v = (L[y + (x >> 1)] + 2 * L[y + (x >> 1) + 1] + L[y + (x >> 1) + 2] + 2) >> 2;
                P(x, y) = v;
            }
        break;
    }
#undef P
}

static void pred8x8(H4Dec *d, int b8, int mode, int *pred) {
    int x0 = (b8 & 1) * 8, y0 = (b8 >> 1) * 8;
    int gx = d->mbx * 16 + x0, gy = d->mby * 16 + y0;
    int blk4 = b8 * 4;
    int at = avail_luma(d, x0, y0 - 1, blk4), al = avail_luma(d, x0 - 1, y0, blk4);
    int ad = avail_luma(d, x0 - 1, y0 - 1, blk4);
    int atr = avail_luma(d, x0 + 8, y0 - 1, blk4);
    if (b8 == 3) atr = 0;
    if (b8 == 2) atr = 1; /* block 1 decoded */
    int p[8 + 8 + 1 + 8], *T = p + 9, *L = p; /* L[0..7], corner p[8], T[0..15] */
    int Lr[8], Tr[16], C = 0;
    for (int i = 0; i < 8; i++) {
        Tr[i] = at ? px(d, 0, gx + i, gy - 1) : 0;
        Lr[i] = al ? px(d, 0, gx - 1, gy + i) : 0;
    }
    for (int i = 8; i < 16; i++) Tr[i] = atr ? px(d, 0, gx + i, gy - 1) : Tr[7];
    if (ad) C = px(d, 0, gx - 1, gy - 1);
    (void)T; (void)L; (void)p;
    /* 8.3.2.2.1 reference sample filtering */
    int Tf[16] = {0}, Lf[8] = {0}, Cf = C;  /* read only when available (8.3.2.2) */
    if (at) {
        Tf[0] = ad ? (C + 2 * Tr[0] + Tr[1] + 2) >> 2 : (3 * Tr[0] + Tr[1] + 2) >> 2;
        for (int x = 1; x < 15; x++) Tf[x] = (Tr[x - 1] + 2 * Tr[x] + Tr[x + 1] + 2) >> 2;
        Tf[15] = (Tr[14] + 3 * Tr[15] + 2) >> 2;
    }
    if (ad) {
        if (at && al) Cf = (Tr[0] + 2 * C + Lr[0] + 2) >> 2;
        else if (at) Cf = (3 * C + Tr[0] + 2) >> 2;
        else if (al) Cf = (3 * C + Lr[0] + 2) >> 2;
        else Cf = C;
    }
    if (al) {
        Lf[0] = ad ? (C + 2 * Lr[0] + Lr[1] + 2) >> 2 : (3 * Lr[0] + Lr[1] + 2) >> 2;
        for (int y = 1; y < 7; y++) Lf[y] = (Lr[y - 1] + 2 * Lr[y] + Lr[y + 1] + 2) >> 2;
        Lf[7] = (Lr[6] + 3 * Lr[7] + 2) >> 2;
    }
    int bd = d->bd;
#define P(x, y) pred[(y) * 8 + (x)]
#define TT(i) ((i) < 0 ? Cf : Tf[i])
#define LL(i) ((i) < 0 ? Cf : Lf[i])
    switch (mode) {
    case 0: for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) P(x, y) = Tf[x]; break;
    case 1: for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) P(x, y) = Lf[y]; break;
    case 2: {
        int s = 0;
        if (at && al) { for (int i = 0; i < 8; i++) s += Tf[i] + Lf[i]; s = (s + 8) >> 4; }
        else if (al) { for (int i = 0; i < 8; i++) s += Lf[i]; s = (s + 4) >> 3; }
        else if (at) { for (int i = 0; i < 8; i++) s += Tf[i]; s = (s + 4) >> 3; }
        else s = 1 << (bd - 1);
        for (int i = 0; i < 64; i++) pred[i] = s;
        break;
    }
    case 3:
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++)
                P(x, y) = (x == 7 && y == 7) ? (Tf[14] + 3 * Tf[15] + 2) >> 2 : (Tf[x + y] + 2 * Tf[x + y + 1] + Tf[x + y + 2] + 2) >> 2;
        break;
    case 4:
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                int v;
                if (x > y) v = (TT(x - y - 2) + 2 * TT(x - y - 1) + Tf[x - y] + 2) >> 2;
                else if (x < y) v = (LL(y - x - 2) + 2 * LL(y - x - 1) + Lf[y - x] + 2) >> 2;
                else v = (Tf[0] + 2 * Cf + Lf[0] + 2) >> 2;
                P(x, y) = v;
            }
        break;
    case 5:
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                int z = 2 * x - y, v;
                if (z >= 0 && (z & 1) == 0) v = (TT(x - (y >> 1) - 1) + Tf[x - (y >> 1)] + 1) >> 1;
                else if (z >= 0) v = (TT(x - (y >> 1) - 2) + 2 * TT(x - (y >> 1) - 1) + Tf[x - (y >> 1)] + 2) >> 2;
                else if (z == -1) v = (Lf[0] + 2 * Cf + Tf[0] + 2) >> 2;
                else v = (Lf[y - 2 * x - 1] + 2 * Lf[y - 2 * x - 2] + LL(y - 2 * x - 3) + 2) >> 2;
                P(x, y) = v;
            }
        break;
    case 6:
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                int z = 2 * y - x, v;
                if (z >= 0 && (z & 1) == 0) v = (LL(y - (x >> 1) - 1) + Lf[y - (x >> 1)] + 1) >> 1;
                else if (z >= 0) v = (LL(y - (x >> 1) - 2) + 2 * LL(y - (x >> 1) - 1) + Lf[y - (x >> 1)] + 2) >> 2;
                else if (z == -1) v = (Lf[0] + 2 * Cf + Tf[0] + 2) >> 2;
                else v = (TT(x - 2 * y - 1) + 2 * TT(x - 2 * y - 2) + TT(x - 2 * y - 3) + 2) >> 2;
                P(x, y) = v;
            }
        break;
    case 7:
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                int i = x + (y >> 1);
                P(x, y) = (y & 1) == 0 ? (Tf[i] + Tf[i + 1] + 1) >> 1 : (Tf[i] + 2 * Tf[i + 1] + Tf[i + 2] + 2) >> 2;
            }
        break;
    case 8:
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                int z = x + 2 * y, v;
                if (z > 13) v = Lf[7];
                else if (z == 13) v = (Lf[6] + 3 * Lf[7] + 2) >> 2;
                else if ((z & 1) == 0) v = (Lf[y + (x >> 1)] + Lf[y + (x >> 1) + 1] + 1) >> 1;
                else v = (Lf[y + (x >> 1)] + 2 * Lf[y + (x >> 1) + 1] + Lf[y + (x >> 1) + 2] + 2) >> 2;
                P(x, y) = v;
            }
        break;
    }
#undef P
#undef TT
#undef LL
}

static void pred16x16(H4Dec *d, int mode, int *pred) {
    int gx = d->mbx * 16, gy = d->mby * 16;
    int at = nb_mb(d, 0, -1) != NULL, al = nb_mb(d, -1, 0) != NULL, ad = nb_mb(d, -1, -1) != NULL;
    int T[16], L[16], C = ad ? px(d, 0, gx - 1, gy - 1) : 0;
    for (int i = 0; i < 16; i++) {
        T[i] = at ? px(d, 0, gx + i, gy - 1) : 0;
        L[i] = al ? px(d, 0, gx - 1, gy + i) : 0;
    }
    int maxv = (1 << d->bd) - 1;
    switch (mode) {
    case 0: for (int y = 0; y < 16; y++) for (int x = 0; x < 16; x++) pred[y * 16 + x] = T[x]; break;
    case 1: for (int y = 0; y < 16; y++) for (int x = 0; x < 16; x++) pred[y * 16 + x] = L[y]; break;
    case 2: {
        int s = 0;
        if (at && al) { for (int i = 0; i < 16; i++) s += T[i] + L[i]; s = (s + 16) >> 5; }
        else if (al) { for (int i = 0; i < 16; i++) s += L[i]; s = (s + 8) >> 4; }
        else if (at) { for (int i = 0; i < 16; i++) s += T[i]; s = (s + 8) >> 4; }
        else s = 1 << (d->bd - 1);
        for (int i = 0; i < 256; i++) pred[i] = s;
        break;
    }
    case 3: {
        int H = 0, V = 0;
        for (int i = 0; i < 8; i++) {
            H += (i + 1) * (T[8 + i] - (i == 7 ? C : T[6 - i]));
            V += (i + 1) * (L[8 + i] - (i == 7 ? C : L[6 - i]));
        }
        int a = 16 * (L[15] + T[15]), b = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
        for (int y = 0; y < 16; y++)
            for (int x = 0; x < 16; x++) pred[y * 16 + x] = clip3(0, maxv, (a + b * (x - 7) + c * (y - 7) + 16) >> 5);
        break;
    }
    }
}

static void pred_chroma(H4Dec *d, int c, int mode, int *pred) {
    int gx = d->mbx * 8, gy = d->mby * 8;
    int at = nb_mb(d, 0, -1) != NULL, al = nb_mb(d, -1, 0) != NULL, ad = nb_mb(d, -1, -1) != NULL;
    int T[8], L[8], C = ad ? px(d, c, gx - 1, gy - 1) : 0;
    for (int i = 0; i < 8; i++) {
        T[i] = at ? px(d, c, gx + i, gy - 1) : 0;
        L[i] = al ? px(d, c, gx - 1, gy + i) : 0;
    }
    int maxv = (1 << d->bdc) - 1;
    switch (mode) {
    case 0:
        for (int by = 0; by < 2; by++)
            for (int bx = 0; bx < 2; bx++) {
                int st = 0, sl = 0;
                for (int i = 0; i < 4; i++) { st += T[bx * 4 + i]; sl += L[by * 4 + i]; }
                int s;
                if ((bx == 0 && by == 0) || (bx == 1 && by == 1)) {
                    if (at && al) s = (st + sl + 4) >> 3;
                    else if (at) s = (st + 2) >> 2;
                    else if (al) s = (sl + 2) >> 2;
                    else s = 1 << (d->bdc - 1);
                } else if (bx == 1) { /* xO > 0, yO == 0: prefer top */
                    if (at) s = (st + 2) >> 2;
                    else if (al) s = (sl + 2) >> 2;
                    else s = 1 << (d->bdc - 1);
                } else { /* xO == 0, yO > 0: prefer left */
                    if (al) s = (sl + 2) >> 2;
                    else if (at) s = (st + 2) >> 2;
                    else s = 1 << (d->bdc - 1);
                }
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) pred[(by * 4 + y) * 8 + bx * 4 + x] = s;
            }
        break;
    case 1: for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) pred[y * 8 + x] = L[y]; break;
    case 2: for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) pred[y * 8 + x] = T[x]; break;
    case 3: {
        int H = 0, V = 0;
        for (int i = 0; i < 4; i++) {
            H += (i + 1) * (T[4 + i] - (i == 3 ? C : T[2 - i]));
            V += (i + 1) * (L[4 + i] - (i == 3 ? C : L[2 - i]));
        }
        int a = 16 * (L[7] + T[7]), b = (34 * H + 32) >> 6, cc = (34 * V + 32) >> 6;
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) pred[y * 8 + x] = clip3(0, maxv, (a + b * (x - 3) + cc * (y - 3) + 16) >> 5);
        break;
    }
    }
}

/* ------------------------------------------------------------ macroblock */
static void put_block(H4Dec *d, int c, int gx, int gy, int n, const int *pred, const int *res) {
    int maxv = (1 << (c ? d->bdc : d->bd)) - 1;
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
            put_sample(d, c, gx + x, gy + y, clip3(0, maxv, pred[y * n + x] + (res ? res[y * n + x] : 0)));
}

static int pred_mode_nb(H4Dec *d, int blk, int is8x8, int dir /* 0 A left, 1 B top */) {
    int bx = k_blk_x[blk], by = k_blk_y[blk], nblk;
    MbInfo *N = dir == 0 ? nb_blk(d, bx - 1, by, &nblk) : nb_blk(d, bx, by - 1, &nblk);
    (void)is8x8;
    if (!N) return -1; /* dcPredModePredictedFlag */
    if (N->mb_type != MB_I_NXN) return 2;
    return N->ipm[nblk];
}

/* ---- reconstruction of one macroblock from the parsed levels (8.3, 8.5) ---- */
/* 8.5.15 intra residual transform-bypass: TransformBypassModeFlag (qpprime_y_zero_transform_bypass_flag
 * and QP'Y == 0) with a horizontal / vertical intra prediction accumulates the residual along the
 * prediction direction over the n x n block (FFmpeg h264_mb.c: only for profile_idc 244, through
 * pred*_add per 4x4 block -- the same samples for valid lossless streams).  dir: 0 vertical, 1 horizontal. */
static void bypass_dpcm(int *r, int n, int dir) {
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            if (dir == 0 && y > 0) r[y * n + x] += r[(y - 1) * n + x];
            if (dir == 1 && x > 0) r[y * n + x] += r[y * n + x - 1];
        }
}

/* 4:0:0: both chroma blocks DC_128_PRED8x8 (1 << (BitDepth - 1)), no residual (FFmpeg) */
static int mono_chroma(H4Dec *d, int gx, int gy) {
    for (int c = 1; c < 3; c++)
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) put_sample(d, c, gx / 2 + x, gy / 2 + y, 1 << (d->bd - 1));
    return 0;
}

/* the TransformBypassModeFlag macroblock: residual = the inverse-scanned levels, no scaling, no
 * transform (8.5.12.1 / 8.5.10 / 8.5.11 with TransformBypassModeFlag 1) */
static int recon_mb_bypass(H4Dec *d, MbInfo *m) {
    const int gx = d->mbx * 16, gy = d->mby * 16;
    const int dpcm = d->s->profile == 244;
    int pred[256], r[256];
    if (m->mb_type == MB_I_NXN && !m->t8x8) {
        for (int blk = 0; blk < 16; blk++) {
            pred4x4(d, blk, m->ipm[blk], pred);
            for (int i = 0; i < 16; i++) r[i] = d->lvl4[blk][i];
            if (dpcm && m->ipm[blk] <= 1) bypass_dpcm(r, 4, m->ipm[blk]);
            put_block(d, 0, gx + k_blk_x[blk] * 4, gy + k_blk_y[blk] * 4, 4, pred, r);
        }
    } else if (m->mb_type == MB_I_NXN) {
        for (int b8 = 0; b8 < 4; b8++) {
            pred8x8(d, b8, m->ipm[b8 * 4], pred);
            for (int i = 0; i < 64; i++) r[i] = d->lvl8[b8][i];
            if (dpcm && m->ipm[b8 * 4] <= 1) bypass_dpcm(r, 8, m->ipm[b8 * 4]);
            put_block(d, 0, gx + (b8 & 1) * 8, gy + (b8 >> 1) * 8, 8, pred, r);
        }
    } else {
        const int mode = (m->mb_type - 1) % 4;
        pred16x16(d, mode, pred);
        for (int blk = 0; blk < 16; blk++) { /* 4x4 blocks' levels, DC from the DC matrix */
            int bx = k_blk_x[blk], by = k_blk_y[blk];
            for (int i = 0; i < 16; i++) r[(by * 4 + (i >> 2)) * 16 + bx * 4 + (i & 3)] = i ? d->lvl4[blk][i] : d->dc_l[by * 4 + bx];
        }
        if (dpcm && mode <= 1) bypass_dpcm(r, 16, mode);
        put_block(d, 0, gx, gy, 16, pred, r);
    }
    if (d->mono) return mono_chroma(d, gx, gy);
    for (int c = 0; c < 2; c++) {
        pred_chroma(d, 1 + c, m->cpm, pred);
        for (int b4 = 0; b4 < 4; b4++) {
            int bx = b4 & 1, by = b4 >> 1;
            for (int i = 0; i < 16; i++) r[(by * 4 + (i >> 2)) * 8 + bx * 4 + (i & 3)] = i ? d->ac_c[c][b4][i] : d->dc_c[c][b4];
        }
        /* intra_chroma_pred_mode 1 horizontal, 2 vertical */
        if (dpcm && (m->cpm == 1 || m->cpm == 2)) bypass_dpcm(r, 8, m->cpm == 2 ? 0 : 1);
        put_block(d, 1 + c, gx / 2, gy / 2, 8, pred, r);
    }
    return 0;
}

static int recon_mb(H4Dec *d, MbInfo *m) {
    const int gx = d->mbx * 16, gy = d->mby * 16;
    /* ---- reconstruction ---- */
    const int qp = d->qp + d->qpbd; /* QP'Y */
    if (d->s->transform_bypass && qp == 0) return recon_mb_bypass(d, m);
    const int qm = qp % 6, qd = qp / 6;
    int pred[256], res[64];
    if (m->mb_type == MB_I_NXN && !m->t8x8) {
        const uint8_t *w = d->p->sl4[0];
        for (int blk = 0; blk < 16; blk++) {
            pred4x4(d, blk, m->ipm[blk], pred);
            int r[16];
            for (int i = 0; i < 16; i++) {
                int ls = ws4(w, i) * norm4(qm, i >> 2, i & 3);
                r[i] = qp >= 24 ? (d->lvl4[blk][i] * ls) << (qd - 4) : (d->lvl4[blk][i] * ls + (1 << (3 - qd))) >> (4 - qd);
            }
            idct4(r);
            put_block(d, 0, gx + k_blk_x[blk] * 4, gy + k_blk_y[blk] * 4, 4, pred, r);
        }
    } else if (m->mb_type == MB_I_NXN) {
        const uint8_t *w = d->p->sl8[0];
        for (int b8 = 0; b8 < 4; b8++) {
            pred8x8(d, b8, m->ipm[b8 * 4], pred);
            for (int i = 0; i < 64; i++) {
                int ls = ws8(w, i) * norm8(qm, i >> 3, i & 7);
                res[i] = qp >= 36 ? (d->lvl8[b8][i] * ls) << (qd - 6) : (d->lvl8[b8][i] * ls + (1 << (5 - qd))) >> (6 - qd);
            }
            idct8(res);
            put_block(d, 0, gx + (b8 & 1) * 8, gy + (b8 >> 1) * 8, 8, pred, res);
        }
    } else {
        pred16x16(d, (m->mb_type - 1) % 4, pred);
        const uint8_t *w = d->p->sl4[0];
        /* luma DC: Hadamard then scale */
        int f[16], c4[16];
        memcpy(c4, d->dc_l, sizeof(c4));
        for (int i = 0; i < 4; i++) { /* rows */
            int *r = c4 + i * 4;
            int a = r[0] + r[1], b = r[0] - r[1], cc = r[2] + r[3], dd = r[2] - r[3];
            f[i * 4 + 0] = a + cc; f[i * 4 + 1] = a - cc; f[i * 4 + 2] = b - dd; f[i * 4 + 3] = b + dd;
        }
        int g[16];
        for (int j = 0; j < 4; j++) {
            int a = f[j] + f[4 + j], b = f[j] - f[4 + j], cc = f[8 + j] + f[12 + j], dd = f[8 + j] - f[12 + j];
            g[j] = a + cc; g[4 + j] = a - cc; g[8 + j] = b - dd; g[12 + j] = b + dd;
        }
        int ls0 = ws4(w, 0) * norm4(qm, 0, 0);
        int dcs[16];
        for (int i = 0; i < 16; i++)
            dcs[i] = qp >= 36 ? (g[i] * ls0) << (qd - 6) : (g[i] * ls0 + (1 << (5 - qd))) >> (6 - qd);
        for (int blk = 0; blk < 16; blk++) {
            int bx = k_blk_x[blk], by = k_blk_y[blk];
            int r[16];
            for (int i = 0; i < 16; i++) {
                int ls = ws4(w, i) * norm4(qm, i >> 2, i & 3);
                r[i] = qp >= 24 ? (d->lvl4[blk][i] * ls) << (qd - 4) : (d->lvl4[blk][i] * ls + (1 << (3 - qd))) >> (4 - qd);
            }
            r[0] = dcs[by * 4 + bx];
            idct4(r);
            int p4[16];
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++) p4[y * 4 + x] = pred[(by * 4 + y) * 16 + bx * 4 + x];
            put_block(d, 0, gx + bx * 4, gy + by * 4, 4, p4, r);
        }
    }
    /* chroma */
    if (d->mono) return mono_chroma(d, gx, gy);
    for (int c = 0; c < 2; c++) {
        int off = c == 0 ? d->p->chroma_qp_offset : d->p->chroma_qp_offset2;
        int qpc = chroma_qp(clip3(-d->qpbdc, 51, d->qp + off)) + d->qpbdc;
        int cm = qpc % 6, cd = qpc / 6;
        const uint8_t *w = d->p->sl4[1 + c];
        pred_chroma(d, 1 + c, m->cpm, pred);
        int *dc = d->dc_c[c];
        int f0 = dc[0] + dc[1] + dc[2] + dc[3], f1 = dc[0] - dc[1] + dc[2] - dc[3];
        int f2 = dc[0] + dc[1] - dc[2] - dc[3], f3 = dc[0] - dc[1] - dc[2] + dc[3];
        int fc[4] = {f0, f1, f2, f3};
        int ls0 = ws4(w, 0) * norm4(cm, 0, 0);
        for (int b4 = 0; b4 < 4; b4++) {
            int r[16];
            for (int i = 0; i < 16; i++) {
                int ls = ws4(w, i) * norm4(cm, i >> 2, i & 3);
                r[i] = qpc >= 24 ? (d->ac_c[c][b4][i] * ls) << (cd - 4) : (d->ac_c[c][b4][i] * ls + (1 << (3 - cd))) >> (4 - cd);
            }
            r[0] = ((fc[b4] * ls0) << cd) >> 5;
            idct4(r);
            int bx = b4 & 1, by = b4 >> 1;
            int p4[16];
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++) p4[y * 4 + x] = pred[(by * 4 + y) * 8 + bx * 4 + x];
            put_block(d, 1 + c, gx / 2 + bx * 4, gy / 2 + by * 4, 4, p4, r);
        }
    }
    return 0;
}

/* position the decoder on macroblock address `addr` (MBAFF: pair addr / 2, bottom addr & 1) and,
 * at the top macroblock of an MBAFF pair, read mb_field_decoding_flag (7.3.4: present for the
 * top MB of every pair in I slices; CABAC ctxIdx 70 + condTermFlagA + condTermFlagB, the left /
 * upper pair being available field pairs, 9.3.3.1.1.2) */
static void mb_start(H4Dec *d, int addr, int cabac) {
    if (d->paff) { /* field MB address of the current field */
        d->mbx = addr % d->mbw;
        d->mby = 2 * (addr / d->mbw) + d->parity;
        d->mb[d->mby * d->mbw + d->mbx].slice = d->nslice;
        d->cur_field = 1;
        return;
    }
    if (!d->mbaff) {
        d->mbx = addr % d->mbw;
        d->mby = addr / d->mbw;
        d->mb[addr].slice = d->nslice;
        return;
    }
    const int pair = addr >> 1;
    d->mbx = pair % d->mbw;
    d->mby = 2 * (pair / d->mbw) + (addr & 1);
    d->mb[d->mby * d->mbw + d->mbx].slice = d->nslice;
    if (!(addr & 1)) {
        MbInfo *A = mb_in_slice(d, d->mbx - 1, d->mby), *B = mb_in_slice(d, d->mbx, d->mby - 2);
        d->cur_field = cabac ? bin(d, 70 + (A && A->field) + (B && B->field)) : ob_bit(&d->bits);
    }
}

static int decode_mb(H4Dec *d, int slice_idx) {
    MbInfo *m = &d->mb[d->mby * d->mbw + d->mbx];
    memset(m, 0, sizeof(*m));
    m->slice = slice_idx;
    m->vx = d->mbx;
    m->vy = d->mby;
    m->field = d->mbaff ? d->cur_field : 0;
    m->mb_type = dec_mb_type_I(d);
    const int gx = d->mbx * 16, gy = d->mby * 16;
    if (m->mb_type == MB_I_PCM) {
        OraBits *b = &d->bits;
        b->pos = (b->pos + 7) & ~7L;
        for (int y = 0; y < 16; y++)
            for (int x = 0; x < 16; x++) put_sample(d, 0, gx + x, gy + y, (int)ob_u(b, d->bd));
        for (int c = 1; c < 3; c++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++)
                    put_sample(d, c, gx / 2 + x, gy / 2 + y, d->mono ? 1 << (d->bd - 1) : (int)ob_u(b, d->bdc));
        oc_init(&d->cc, b);
        m->qp = d->qp;
        m->cbp = 0x2F;
        memset(m->cbf, 1, 16);
        memset(m->cbf_c, 1, sizeof(m->cbf_c));
        memset(m->cbf_dc, 1, 3);
        for (int i = 0; i < 16; i++) m->ipm[i] = 2;
        d->prev_qpd_nz = 0;
        return 0;
    }
    int is16 = m->mb_type >= 1 && m->mb_type <= 24;
    if (m->mb_type == MB_I_NXN && d->p->transform_8x8) {
        MbInfo *A = nb_mb(d, -1, 0), *B = nb_mb(d, 0, -1);
        int ctx = (A && A->t8x8) + (B && B->t8x8);
        m->t8x8 = bin(d, 399 + ctx);
    }
    if (m->mb_type == MB_I_NXN) {
        int nb = m->t8x8 ? 4 : 16;
        for (int i = 0; i < nb; i++) {
            int blk = m->t8x8 ? i * 4 : i;
            int prev = bin(d, 68);
            int rem = 0;
            if (!prev) {
                rem = bin(d, 69);
                rem |= bin(d, 69) << 1;
                rem |= bin(d, 69) << 2;
            }
            int a = pred_mode_nb(d, blk, m->t8x8, 0), bb = pred_mode_nb(d, blk, m->t8x8, 1);
            int pm = (a < 0 || bb < 0) ? 2 : (a < bb ? a : bb);
            int mode = prev ? pm : (rem < pm ? rem : rem + 1);
            if (m->t8x8) for (int k = 0; k < 4; k++) m->ipm[blk + k] = (uint8_t)mode;
            else m->ipm[blk] = (uint8_t)mode;
        }
    } else {
        for (int i = 0; i < 16; i++) m->ipm[i] = 2;
    }
    m->cpm = d->mono ? 0 : dec_chroma_pred(d);
    if (is16) {
        int t = m->mb_type - 1;
        m->cbp = ((t / 4) % 3) << 4 | (t >= 12 ? 15 : 0);
    } else {
        m->cbp = dec_cbp(d);
    }
    int qpd = 0;
    if ((m->cbp & 15) || (m->cbp >> 4) || is16) {
        qpd = dec_qp_delta(d);
        d->qp = ((d->qp + qpd + 52 + 2 * d->qpbd) % (52 + d->qpbd)) - d->qpbd;
    }
    d->prev_qpd_nz = qpd != 0;
    m->qpd_nz = qpd != 0;
    m->qp = d->qp;
    /* ---- residual ---- */
    int coef[64];
    const uint8_t *z4 = m->field ? k_fld4 : k_zz4, *z8 = m->field ? k_fld8 : k_zz8; /* 8.5.6 / 8.5.7 */
    memset(d->lvl4, 0, sizeof(d->lvl4));
    memset(d->lvl8, 0, sizeof(d->lvl8));
    memset(d->dc_l, 0, sizeof(d->dc_l));
    memset(d->dc_c, 0, sizeof(d->dc_c));
    memset(d->ac_c, 0, sizeof(d->ac_c));
    if (is16) {
        int nb, ca = cbf_cond(d, 0, nb_mb(d, -1, 0), 0, 0), cb = cbf_cond(d, 0, nb_mb(d, 0, -1), 0, 0);
        (void)nb;
        m->cbf_dc[0] = (uint8_t)residual_block(d, 0, ca + 2 * cb, 16, coef);
        for (int k = 0; k < 16; k++) d->dc_l[z4[k]] = coef[k];
    }
    for (int b8 = 0; b8 < 4; b8++) {
        if (!((m->cbp >> b8) & 1)) continue;
        if (m->t8x8) {
            residual_block(d, 5, 0, 64, coef);
            for (int k = 0; k < 64; k++) d->lvl8[b8][z8[k]] = coef[k];
            for (int k = 0; k < 4; k++) m->cbf[b8 * 4 + k] = 1;
            continue;
        }
        for (int b4 = 0; b4 < 4; b4++) {
            int blk = b8 * 4 + b4, bx = k_blk_x[blk], by = k_blk_y[blk], nblk;
            int cat = is16 ? 1 : 2;
            MbInfo *A = nb_blk(d, bx - 1, by, &nblk);
            int ca = cbf_cond(d, cat, A, nblk, 0);
            MbInfo *B = nb_blk(d, bx, by - 1, &nblk);
            int cb = cbf_cond(d, cat, B, nblk, 0);
            if (is16) {
                m->cbf[blk] = (uint8_t)residual_block(d, 1, ca + 2 * cb, 15, coef);
                for (int k = 0; k < 15; k++) d->lvl4[blk][z4[k + 1]] = coef[k];
            } else {
                m->cbf[blk] = (uint8_t)residual_block(d, 2, ca + 2 * cb, 16, coef);
                for (int k = 0; k < 16; k++) d->lvl4[blk][z4[k]] = coef[k];
            }
        }
    }
    if (!d->mono && (m->cbp >> 4)) {
        for (int c = 0; c < 2; c++) {
            int ca = cbf_cond(d, 3, nb_mb(d, -1, 0), 0, c), cb = cbf_cond(d, 3, nb_mb(d, 0, -1), 0, c);
            m->cbf_dc[1 + c] = (uint8_t)residual_block(d, 3, ca + 2 * cb, 4, coef);
            for (int k = 0; k < 4; k++) d->dc_c[c][k] = coef[k];
        }
    }
    if (!d->mono && (m->cbp >> 4) == 2) {
        for (int c = 0; c < 2; c++)
            for (int b4 = 0; b4 < 4; b4++) {
                int bx = b4 & 1, by = b4 >> 1, ca, cb;
                int xW, yW;
                if (bx > 0) ca = m->cbf_c[c][b4 - 1];
                else { /* 6.4.11.5: the chroma block covering chroma location (-1, 4 by) */
                    MbInfo *A = nb_loc(d, -1, by * 4, 8, 8, &xW, &yW);
                    ca = cbf_cond(d, 4, A, A ? (yW >> 2) * 2 + (xW >> 2) : 0, c);
                }
                if (by > 0) cb = m->cbf_c[c][b4 - 2];
                else {
                    MbInfo *B = nb_loc(d, bx * 4, -1, 8, 8, &xW, &yW);
                    cb = cbf_cond(d, 4, B, B ? (yW >> 2) * 2 + (xW >> 2) : 0, c);
                }
                m->cbf_c[c][b4] = (uint8_t)residual_block(d, 4, ca + 2 * cb, 15, coef);
                for (int k = 0; k < 15; k++) d->ac_c[c][b4][z4[k + 1]] = coef[k];
            }
    }
    return recon_mb(d, m);
}

/* ------------------------------------------------------------ CAVLC (7.3.5.3.2, 9.2) */
/* the index of the first entry (of n) whose code the next bits match; bit by bit, as 9.2 reads */
static int vlc_read(OraBits *b, const uint8_t *lens, const uint8_t *codes, int n) {
    uint32_t code = 0;
    for (int len = 1; len <= 16; len++) {
        code = (code << 1) | (uint32_t)ob_bit(b);
        for (int i = 0; i < n; i++)
            if (lens[i] == len && codes[i] == code) return i;
    }
    return -1;
}

/* coeff_token (9.2.1): returns TotalCoeff, *t1 = TrailingOnes; -1 on error */
static int cavlc_coeff_token(OraBits *b, int nC, int *t1) {
    if (nC >= 8) {
        int v = (int)ob_u(b, 6);
        if (v == 3) { *t1 = 0; return 0; }
        *t1 = v & 3;
        if ((v >> 2) + 1 < *t1) return -1;
        return (v >> 2) + 1;
    }
    /* Table 9-5, indexed TotalCoeff * 4 + TrailingOnes */
    int i = nC < 0 ? vlc_read(b, k_ct_dc_len, k_ct_dc_bits, 4 * 5)
                   : vlc_read(b, k_ct_len[nC < 2 ? 0 : (nC < 4 ? 1 : 2)], k_ct_bits[nC < 2 ? 0 : (nC < 4 ? 1 : 2)], 4 * 17);
    if (i < 0) return -1;
    *t1 = i & 3;
    return i >> 2;
}

/* residual_block_cavlc: coeffLevel[0..maxNum-1] in scan order; returns TotalCoeff (-1 error) */
static int cavlc_block(H4Dec *d, int nC, int maxNum, int *out) {
    OraBits *b = &d->bits;
    memset(out, 0, sizeof(int) * maxNum);
    int t1, tc = cavlc_coeff_token(b, nC, &t1);
    if (tc < 0 || tc > maxNum) return -1;
    if (tc == 0) return 0;
    int level[16], run[16];
    int suffixLength = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; i++) {
        if (i < t1) {
            level[i] = ob_bit(b) ? -1 : 1;
            continue;
        }
        int prefix = 0;
        while (!ob_bit(b)) {
            if (++prefix > 32) return -1;
        }
        int levelCode = (prefix < 15 ? prefix : 15) << suffixLength;
        int sz = (prefix == 14 && suffixLength == 0) ? 4 : (prefix >= 15 ? prefix - 3 : suffixLength);
        if (sz > 0) levelCode += (int)ob_u(b, sz);
        if (prefix >= 15 && suffixLength == 0) levelCode += 15;
        if (prefix >= 16) levelCode += (1 << (prefix - 3)) - 4096;
        if (i == t1 && t1 < 3) levelCode += 2;
        level[i] = (levelCode % 2 == 0) ? (levelCode + 2) >> 1 : (-levelCode - 1) >> 1;
        if (suffixLength == 0) suffixLength = 1;
        if (abs(level[i]) > (3 << (suffixLength - 1)) && suffixLength < 6) suffixLength++;
    }
    int zerosLeft = 0;
    if (tc < maxNum) {
        if (maxNum == 4) zerosLeft = vlc_read(b, k_tz_dc_len[tc - 1], k_tz_dc_bits[tc - 1], 5 - tc);
        else zerosLeft = vlc_read(b, k_tz_len[tc - 1], k_tz_bits[tc - 1], 17 - tc);
        if (zerosLeft < 0 || zerosLeft > maxNum - tc) return -1;
    }
    for (int i = 0; i < tc - 1; i++) {
        if (zerosLeft > 0) {
            int zl = zerosLeft < 7 ? zerosLeft : 7;
            int r = vlc_read(b, k_run_len[zl - 1], k_run_bits[zl - 1], zl < 7 ? zl + 1 : 15);
            if (r < 0 || r > zerosLeft) return -1;
            run[i] = r;
            zerosLeft -= r;
        } else {
            run[i] = 0;
        }
    }
    run[tc - 1] = zerosLeft;
    int coeffNum = -1;
    for (int i = tc - 1; i >= 0; i--) {
        coeffNum += run[i] + 1;
        out[coeffNum] = level[i];
    }
    return tc;
}

/* nC for a luma 4x4 block (9.2.1): neighbours' TotalCoeff, I_PCM = 16 */
static int cavlc_nc_luma(H4Dec *d, int blk) {
    int bx = k_blk_x[blk], by = k_blk_y[blk], na = 0, nb = 0, nblk;
    MbInfo *A = nb_blk(d, bx - 1, by, &nblk);
    if (A) na = A->mb_type == MB_I_PCM ? 16 : A->tc[nblk];
    MbInfo *B = nb_blk(d, bx, by - 1, &nblk);
    if (B) nb = B->mb_type == MB_I_PCM ? 16 : B->tc[nblk];
    if (A && B) return (na + nb + 1) >> 1;
    return A ? na : (B ? nb : 0);
}
static int cavlc_nc_chroma(H4Dec *d, MbInfo *m, int c, int b4) {
    int bx = b4 & 1, by = b4 >> 1, na = 0, nb = 0, aa = 1, ab = 1;
    int xW, yW;
    if (bx) na = m->tcc[c][b4 - 1];
    else { /* 6.4.11.5 */
        MbInfo *A = nb_loc(d, -1, by * 4, 8, 8, &xW, &yW);
        if (!A) aa = 0;
        else na = A->mb_type == MB_I_PCM ? 16 : A->tcc[c][(yW >> 2) * 2 + (xW >> 2)];
    }
    if (by) nb = m->tcc[c][b4 - 2];
    else {
        MbInfo *B = nb_loc(d, bx * 4, -1, 8, 8, &xW, &yW);
        if (!B) ab = 0;
        else nb = B->mb_type == MB_I_PCM ? 16 : B->tcc[c][(yW >> 2) * 2 + (xW >> 2)];
    }
    if (aa && ab) return (na + nb + 1) >> 1;
    return aa ? na : (ab ? nb : 0);
}

static int decode_mb_cavlc(H4Dec *d, int slice_idx) {
    MbInfo *m = &d->mb[d->mby * d->mbw + d->mbx];
    memset(m, 0, sizeof(*m));
    m->slice = slice_idx;
    m->vx = d->mbx;
    m->vy = d->mby;
    m->field = d->mbaff ? d->cur_field : 0;
    OraBits *b = &d->bits;
    uint32_t mbt = ob_ue(b);
    if (mbt > 25) return -1;
    m->mb_type = (int)mbt;
    const int gx = d->mbx * 16, gy = d->mby * 16;
    if (m->mb_type == MB_I_PCM) {
        b->pos = (b->pos + 7) & ~7L;
        for (int y = 0; y < 16; y++)
            for (int x = 0; x < 16; x++) put_sample(d, 0, gx + x, gy + y, (int)ob_u(b, d->bd));
        for (int c = 1; c < 3; c++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++)
                    put_sample(d, c, gx / 2 + x, gy / 2 + y, d->mono ? 1 << (d->bd - 1) : (int)ob_u(b, d->bdc));
        m->qp = d->qp;
        m->cbp = 0x2F;
        memset(m->tc, 16, sizeof(m->tc));
        memset(m->tcc, 16, sizeof(m->tcc));
        for (int i = 0; i < 16; i++) m->ipm[i] = 2;
        return 0;
    }
    int is16 = m->mb_type >= 1 && m->mb_type <= 24;
    if (m->mb_type == MB_I_NXN && d->p->transform_8x8) m->t8x8 = ob_bit(b);
    if (m->mb_type == MB_I_NXN) {
        int nb = m->t8x8 ? 4 : 16;
        for (int i = 0; i < nb; i++) {
            int blk = m->t8x8 ? i * 4 : i;
            int prev = ob_bit(b);
            int rem = prev ? 0 : (int)ob_u(b, 3);
            int a = pred_mode_nb(d, blk, m->t8x8, 0), bb = pred_mode_nb(d, blk, m->t8x8, 1);
            int pm = (a < 0 || bb < 0) ? 2 : (a < bb ? a : bb);
            int mode = prev ? pm : (rem < pm ? rem : rem + 1);
            if (m->t8x8) for (int k = 0; k < 4; k++) m->ipm[blk + k] = (uint8_t)mode;
            else m->ipm[blk] = (uint8_t)mode;
        }
    } else {
        for (int i = 0; i < 16; i++) m->ipm[i] = 2;
    }
    if (!d->mono) {
        uint32_t cpm = ob_ue(b);
        if (cpm > 3) return -1;
        m->cpm = (int)cpm;
    }
    if (is16) {
        int t = m->mb_type - 1;
        m->cbp = ((t / 4) % 3) << 4 | (t >= 12 ? 15 : 0);
    } else {
        uint32_t cn = ob_ue(b);
        /* Table 9-4: ChromaArrayType 0 maps codeNum 0..15 to luma-only patterns */
        static const uint8_t k_cbp_intra_gray[16] = {15, 0, 7, 11, 13, 14, 3, 5, 10, 12, 1, 2, 4, 8, 6, 9};
        if (cn > (d->mono ? 15u : 47u)) return -1;
        m->cbp = d->mono ? k_cbp_intra_gray[cn] : k_cbp_intra[cn];
    }
    if ((m->cbp & 15) || (m->cbp >> 4) || is16) {
        int qpd = ob_se(b);
        d->qp = ((d->qp + qpd + 52 + 2 * d->qpbd) % (52 + d->qpbd)) - d->qpbd;
    }
    m->qp = d->qp;
    int coef[64];
    const uint8_t *z4 = m->field ? k_fld4 : k_zz4, *z8 = m->field ? k_fld8 : k_zz8; /* 8.5.6 / 8.5.7 */
    memset(d->lvl4, 0, sizeof(d->lvl4));
    memset(d->lvl8, 0, sizeof(d->lvl8));
    memset(d->dc_l, 0, sizeof(d->dc_l));
    memset(d->dc_c, 0, sizeof(d->dc_c));
    memset(d->ac_c, 0, sizeof(d->ac_c));
    if (is16) {
        if (cavlc_block(d, cavlc_nc_luma(d, 0), 16, coef) < 0) return -1;
        for (int k = 0; k < 16; k++) d->dc_l[z4[k]] = coef[k];
    }
    for (int b8 = 0; b8 < 4; b8++) {
        if (!((m->cbp >> b8) & 1)) continue;
        if (m->t8x8) {
            for (int i4 = 0; i4 < 4; i4++) {
                int blk = b8 * 4 + i4;
                int tc = cavlc_block(d, cavlc_nc_luma(d, blk), 16, coef);
                if (tc < 0) return -1;
                m->tc[blk] = (uint8_t)tc;
                for (int k = 0; k < 16; k++) d->lvl8[b8][z8[4 * k + i4]] = coef[k];
            }
            continue;
        }
        for (int b4 = 0; b4 < 4; b4++) {
            int blk = b8 * 4 + b4;
            int tc = cavlc_block(d, cavlc_nc_luma(d, blk), is16 ? 15 : 16, coef);
            if (tc < 0) return -1;
            m->tc[blk] = (uint8_t)tc;
            if (is16) for (int k = 0; k < 15; k++) d->lvl4[blk][z4[k + 1]] = coef[k];
            else for (int k = 0; k < 16; k++) d->lvl4[blk][z4[k]] = coef[k];
        }
    }
    if (!d->mono && (m->cbp >> 4)) {
        for (int c = 0; c < 2; c++) {
            if (cavlc_block(d, -1, 4, coef) < 0) return -1;
            for (int k = 0; k < 4; k++) d->dc_c[c][k] = coef[k];
        }
    }
    if (!d->mono && (m->cbp >> 4) == 2) {
        for (int c = 0; c < 2; c++)
            for (int b4 = 0; b4 < 4; b4++) {
                int tc = cavlc_block(d, cavlc_nc_chroma(d, m, c, b4), 15, coef);
                if (tc < 0) return -1;
                m->tcc[c][b4] = (uint8_t)tc;
                for (int k = 0; k < 15; k++) d->ac_c[c][b4][z4[k + 1]] = coef[k];
            }
    }
    return recon_mb(d, m);
}

/* ------------------------------------------------------------ deblocking (8.7) */
static const uint8_t k_alpha[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   4,   4,
                                    5,  6,  7,  8,  9,  10, 12, 13, 15, 17, 20, 22, 25,  28,  32,  36,  40,  45,
                                    50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static const uint8_t k_beta[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  2,  2,
                                   2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7,  7,  8,  8,  9,  9,  10, 10,
                                   11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static const uint8_t k_tc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1},
    {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4},
    {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11},
    {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

/* filter one line across an edge. s: pointer to q0, step: distance p0->q0 */
static void filt_line(uint16_t *q, int step, int bs, int alpha, int beta, int tc0, int chroma, int maxv) {
    int p0 = q[-step], p1 = q[-2 * step], q0 = q[0], q1 = q[step];
    if (!(abs(p0 - q0) < alpha && abs(p1 - p0) < beta && abs(q1 - q0) < beta)) return;
    if (chroma) {
        if (bs < 4) {
            int tc = tc0 + 1;
            int dl = clip3(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
            q[-step] = (uint16_t)clip3(0, maxv, p0 + dl);
            q[0] = (uint16_t)clip3(0, maxv, q0 - dl);
        } else {
            q[-step] = (uint16_t)((2 * p1 + p0 + q1 + 2) >> 2);
            q[0] = (uint16_t)((2 * q1 + q0 + p1 + 2) >> 2);
        }
        return;
    }
    int p2 = q[-3 * step], q2 = q[2 * step];
    int ap = abs(p2 - p0), aq = abs(q2 - q0);
    if (bs < 4) {
        int tc = tc0 + (ap < beta) + (aq < beta);
        int dl = clip3(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
        q[-step] = (uint16_t)clip3(0, maxv, p0 + dl);
        q[0] = (uint16_t)clip3(0, maxv, q0 - dl);
        if (ap < beta) q[-2 * step] = (uint16_t)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 * 2)) >> 1));
        if (aq < beta) q[step] = (uint16_t)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 * 2)) >> 1));
    } else {
        int p3 = q[-4 * step], q3 = q[3 * step];
        if (ap < beta && abs(p0 - q0) < ((alpha >> 2) + 2)) {
            q[-step] = (uint16_t)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
            q[-2 * step] = (uint16_t)((p2 + p1 + p0 + q0 + 2) >> 2);
            q[-3 * step] = (uint16_t)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
        } else {
            q[-step] = (uint16_t)((2 * p1 + p0 + q1 + 2) >> 2);
        }
        if (aq < beta && abs(p0 - q0) < ((alpha >> 2) + 2)) {
            q[0] = (uint16_t)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
            q[step] = (uint16_t)((p0 + q0 + q1 + q2 + 2) >> 2);
            q[2 * step] = (uint16_t)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
        } else {
            q[0] = (uint16_t)((2 * q1 + q0 + p1 + 2) >> 2);
        }
    }
}

static int mb_qp_for_filter(const MbInfo *m) { return m->mb_type == MB_I_PCM ? 0 : m->qp; }

static void deblock_mb(H4Dec *d, int mx, int my) {
    MbInfo *m = &d->mb[my * d->mbw + mx];
    const H4Slice *sl = &d->sl[m->slice];
    if (sl->disable_deblock == 1) return;
    for (int dir = 0; dir < 2; dir++) { /* 0: vertical edges, 1: horizontal */
        MbInfo *n = NULL;
        if (dir == 0 && mx > 0) n = &d->mb[my * d->mbw + mx - 1];
        if (dir == 1 && my > 0) n = &d->mb[(my - 1) * d->mbw + mx];
        int filter_mb_edge = n != NULL;
        if (n && sl->disable_deblock == 2 && n->slice != m->slice) filter_mb_edge = 0;
        for (int e = 0; e < 4; e++) {
            if (e == 0 && !filter_mb_edge) continue;
            if ((e == 1 || e == 3) && m->t8x8) continue;
            int bs = e == 0 ? 4 : 3;
            const MbInfo *pm = e == 0 ? n : m;
            /* luma */
            int qpav = (mb_qp_for_filter(pm) + mb_qp_for_filter(m) + 1) >> 1;
            int ia = clip3(0, 51, qpav + sl->alpha_off), ib = clip3(0, 51, qpav + sl->beta_off);
            int alpha = k_alpha[ia] * (1 << (d->bd - 8)), beta = k_beta[ib] * (1 << (d->bd - 8));
            int tc0 = bs < 4 ? k_tc0[ia][bs - 1] * (1 << (d->bd - 8)) : 0;
            for (int k = 0; k < 16; k++) {
                uint16_t *q;
                int step;
                if (dir == 0) { q = &d->pl[0][(my * 16 + k) * d->st[0] + mx * 16 + e * 4]; step = 1; }
                else { q = &d->pl[0][(my * 16 + e * 4) * d->st[0] + mx * 16 + k]; step = d->st[0]; }
                filt_line(q, step, bs, alpha, beta, tc0, 0, (1 << d->bd) - 1);
            }
            /* chroma: edges 0 and 2 (luma 0, 8) */
            if (e == 0 || e == 2) {
                for (int c = 1; c < 3; c++) {
                    int off = c == 1 ? sl->chroma_qp_offset : sl->chroma_qp_offset2;
                    int qpp = pm->mb_type == MB_I_PCM ? chroma_qp(clip3(-d->qpbdc, 51, 0 + off)) : chroma_qp(clip3(-d->qpbdc, 51, pm->qp + off));
                    int qpq = m->mb_type == MB_I_PCM ? chroma_qp(clip3(-d->qpbdc, 51, 0 + off)) : chroma_qp(clip3(-d->qpbdc, 51, m->qp + off));
                    int qa = (qpp + qpq + 1) >> 1;
                    int ia2 = clip3(0, 51, qa + sl->alpha_off), ib2 = clip3(0, 51, qa + sl->beta_off);
                    int al2 = k_alpha[ia2] * (1 << (d->bdc - 8)), be2 = k_beta[ib2] * (1 << (d->bdc - 8));
                    int tc2 = bs < 4 ? k_tc0[ia2][bs - 1] * (1 << (d->bdc - 8)) : 0;
                    for (int k = 0; k < 8; k++) {
                        uint16_t *q;
                        int step;
                        if (dir == 0) { q = &d->pl[c][(my * 8 + k) * d->st[c] + mx * 8 + e * 2]; step = 1; }
                        else { q = &d->pl[c][(my * 8 + e * 2) * d->st[c] + mx * 8 + k]; step = d->st[c]; }
                        filt_line(q, step, bs, al2, be2, tc2, 1, (1 << d->bdc) - 1);
                    }
                }
            }
        }
    }
}

/* ---- MBAFF deblocking (8.7 with MbaffFrameFlag 1; FFmpeg h264_loopfilter.c, the decoder behind
 * /root/reference/src/Decoder.cpp:324).  Every edge is a set of sample lines in picture
 * coordinates: vertical edges run along picture rows (a field MB's rows are every other picture
 * row, and the p side of its left MB edge is the left pair's MB holding the same picture row);
 * horizontal edges step through the MB's own rows (field MB: 2 picture rows) and its top MB edge
 * reaches up the same way; a frame top MB under a field pair filters its top edge twice in field
 * mode (8.7: "filtered ... with fieldModeInFrameFilteringFlag 1", FFmpeg filter_mb_dir's "special
 * case ... done twice").  All-intra bS: 4 on vertical MB edges and on horizontal MB edges between
 * two frame MBs, 3 otherwise. */
static MbInfo *pair_mb_at_row(H4Dec *d, int px, int py, int c, int Y) {
    const int S = c ? 8 : 16;
    MbInfo *top = &d->mb[(2 * py) * d->mbw + px];
    const int r = Y - 2 * py * S;
    const int bot = top->field ? (r & 1) : (r >= S);
    return &d->mb[(2 * py + bot) * d->mbw + px];
}
static void filt_mbaff(H4Dec *d, int c, uint16_t *q, int step, int bs, const MbInfo *P, const MbInfo *Q, const H4Slice *sl) {
    int qa;
    if (c == 0) {
        qa = (mb_qp_for_filter(P) + mb_qp_for_filter(Q) + 1) >> 1;
    } else {
        int off = c == 1 ? sl->chroma_qp_offset : sl->chroma_qp_offset2;
        int qpp = chroma_qp(clip3(-d->qpbdc, 51, mb_qp_for_filter(P) + off));
        int qpq = chroma_qp(clip3(-d->qpbdc, 51, mb_qp_for_filter(Q) + off));
        qa = (qpp + qpq + 1) >> 1;
    }
    const int bd = c ? d->bdc : d->bd;
    int ia = clip3(0, 51, qa + sl->alpha_off), ib = clip3(0, 51, qa + sl->beta_off);
    int alpha = k_alpha[ia] * (1 << (bd - 8)), beta = k_beta[ib] * (1 << (bd - 8));
    int tc0 = bs < 4 ? k_tc0[ia][bs - 1] * (1 << (bd - 8)) : 0;
    filt_line(q, step, bs, alpha, beta, tc0, c > 0, (1 << bd) - 1);
}
static void deblock_mb_mbaff(H4Dec *d, int mx, int vy) {
    MbInfo *m = &d->mb[vy * d->mbw + mx];
    const H4Slice *sl = &d->sl[m->slice];
    if (sl->disable_deblock == 1) return;
    const int py = vy >> 1, bot = vy & 1;
    /* slice tests on the neighbour of the MB's own parity for field MBs (MBAFF pairs share a
     * slice; the fields of a PAFF pair do not) */
    const int par = m->field ? bot : 0;
    int left = mx > 0;
    if (left) {
        const MbInfo *L = &d->mb[(2 * py + par) * d->mbw + mx - 1];
        if (L->slice < 0 || (sl->disable_deblock == 2 && L->slice != m->slice)) left = 0;
    }
    int top;
    if (!m->field && bot) top = 1; /* the pair's internal edge (CurrMbAddr - 1) */
    else if (py == 0) top = 0;
    else {
        const MbInfo *B = &d->mb[(2 * py - 2 + par) * d->mbw + mx];
        top = B->slice >= 0 && !(sl->disable_deblock == 2 && B->slice != m->slice);
    }
    for (int c = 0; c < 3; c++) {
        const int S = c ? 8 : 16, st = d->st[c];
        uint16_t *pl = d->pl[c];
        for (int dir = 0; dir < 2; dir++) {
            for (int e = 0; e < S; e += 4) {
                if (c == 0 && (e == 4 || e == 12) && m->t8x8) continue;
                if (dir == 0) { /* vertical edge at column e */
                    if (e == 0 && !left) continue;
                    for (int r = 0; r < S; r++) {
                        int X, Y;
                        mb_phys(d, m, c, e, r, &X, &Y);
                        const MbInfo *P = e == 0 ? pair_mb_at_row(d, mx - 1, py, c, Y) : m;
                        filt_mbaff(d, c, &pl[Y * st + X], 1, e == 0 ? 4 : 3, P, m, sl);
                    }
                    continue;
                }
                if (e == 0 && !top) continue;
                int X0, Yq;
                mb_phys(d, m, c, 0, e, &X0, &Yq);
                if (e == 0 && !m->field && !bot && d->mb[(2 * py - 2) * d->mbw + mx].field) {
                    for (int j = 0; j < 2; j++) { /* top field lines, then bottom field lines */
                        const MbInfo *P = &d->mb[(2 * py - 2 + j) * d->mbw + mx];
                        for (int x = 0; x < S; x++) filt_mbaff(d, c, &pl[(Yq + j) * st + X0 + x], 2 * st, 3, P, m, sl);
                    }
                    continue;
                }
                const int step = m->field ? 2 * st : st;
                const MbInfo *P = m;
                int bs = 3;
                if (e == 0) {
                    P = (!m->field && bot) ? &d->mb[(2 * py) * d->mbw + mx]
                                           : pair_mb_at_row(d, mx, py - 1, c, Yq - (m->field ? 2 : 1));
                    bs = (!m->field && !P->field) ? 4 : 3;
                }
                for (int x = 0; x < S; x++) filt_mbaff(d, c, &pl[Yq * st + X0 + x], step, bs, P, m, sl);
            }
        }
    }
}

/* ------------------------------------------------------------ top level */
int oracle_h264_decode(const uint8_t *data, long size, int flags, OraclePicture *out) {
    memset(out, 0, sizeof(*out));
    int maxnal = 4096;
    OraNal *nals = (OraNal *)malloc(sizeof(OraNal) * maxnal);
    int nn = ora_split_annexb(data, size, nals, maxnal);
    H4Dec *d = (H4Dec *)calloc(1, sizeof(H4Dec));
    uint8_t *rbsp = (uint8_t *)malloc((size_t)size + 16);
    int have = 0, ret = -10, first_frame_num = -1, first_idr = -1;
    for (int i = 0; i < nn; i++) {
        if (nals[i].n < 1) continue;
        int nal_ref_idc = (nals[i].p[0] >> 5) & 3;
        int type = nals[i].p[0] & 31;
        long rn = ora_unescape(nals[i].p + 1, nals[i].n - 1, rbsp);
        OraBits b = {rbsp, rn, 0};
        if (type == 7) {
            if (have) break;
            if (parse_sps(&b, d->sps) < 0) { ret = -2; goto done; }
        } else if (type == 8) {
            if (have) break;
            if (parse_pps(&b, d->pps, d->sps) < 0) { ret = -3; goto done; }
        } else if (type == 1 || type == 5) {
            int first_mb = (int)ob_ue(&b);
            int slice_type = (int)ob_ue(&b);
            int pps_id = (int)ob_ue(&b);
            if (pps_id > 255 || !d->pps[pps_id].valid) { ret = -4; goto done; }
            const H4Pps *p = &d->pps[pps_id];
            const H4Sps *s = &d->sps[p->sps_id];
            if (!s->valid) { ret = -4; goto done; }
            int frame_num = (int)ob_u(&b, s->log2_max_frame_num);
            /* field_pic_flag / bottom_field_flag: PAFF.  The reference's FFmpeg outputs no frame for a
             * first field alone (h264dec.c "Wait for second field") and the reference sends one
             * packet, so it returns false for field pictures; restated here is the field pair, the
             * frame FFmpeg outputs once both fields are decoded (the build's default mode) */
            int field_pic = 0, bottom = 0;
            if (!s->frame_mbs_only) {
                field_pic = (int)ob_u(&b, 1);
                if (field_pic) bottom = (int)ob_u(&b, 1);
            }
            if (have && !d->paff && (field_pic || first_mb == 0 || frame_num != first_frame_num || (type == 5) != (first_idr == 1))) break;
            if (have && d->paff) { /* picture 0 = the first field + the other parity's field of the same frame */
                if (!field_pic || frame_num != first_frame_num) break;
                if (first_mb == 0 ? (d->fields_seen >> bottom) & 1 : !((d->fields_seen >> bottom) & 1)) break;
            }
            /* FFmpeg: "first_mb_in_slice overflow" drops the slice; picture 0 is output from the
             * slices already collected, and fails only when none was */
            if (first_mb < 0 || first_mb * (1 + (s->mbaff && !field_pic)) * (1 + field_pic) >= s->mb_w * s->mb_h) {
                if (have) break;
                ret = -6;
                goto done;
            }
            if (slice_type % 5 != 2) { ret = -5; goto done; } /* P/B: the first picture must be intra */
            if (type == 5) ob_ue(&b);                          /* idr_pic_id */
            if (s->poc_type == 0) {
                ob_u(&b, s->log2_max_poc_lsb);
                if (p->bottom_field_pic_order && !field_pic) ob_se(&b);
            } else if (s->poc_type == 1 && !s->delta_pic_order_always_zero) {
                ob_se(&b);
                if (p->bottom_field_pic_order && !field_pic) ob_se(&b);
            }
            if (p->redundant_pic_cnt) ob_ue(&b);
            if (nal_ref_idc) {
                if (type == 5) { ob_u(&b, 1); ob_u(&b, 1); }
                else if (ob_u(&b, 1)) {
                    for (;;) {
                        int op = (int)ob_ue(&b);
                        if (op == 0) break;
                        if (op == 1 || op == 3) ob_ue(&b);
                        if (op == 2) ob_ue(&b);
                        if (op == 3 || op == 6) ob_ue(&b);
                        if (op == 4) ob_ue(&b);
                    }
                }
            }
            int qpd = ob_se(&b);
            H4Slice *sl = &d->sl[d->nslice];
            memset(sl, 0, sizeof(*sl));
            if (p->deblock_ctrl) {
                sl->disable_deblock = (int)ob_ue(&b);
                if (sl->disable_deblock != 1) {
                    sl->alpha_off = ob_se(&b) * 2;
                    sl->beta_off = ob_se(&b) * 2;
                }
            }
            sl->chroma_qp_offset = p->chroma_qp_offset;
            sl->chroma_qp_offset2 = p->chroma_qp_offset2;
            if (!have) {
                d->s = s;
                d->p = p;
                d->mbw = s->mb_w;
                d->mbh = s->mb_h;
                d->W = d->mbw * 16;
                d->H = d->mbh * 16;
                d->bd = s->bit_depth;
                d->bdc = s->bit_depth_c;
                d->mono = s->chroma_format_idc == 0;
                d->qpbd = 6 * (d->bd - 8);
                d->mbaff = s->mbaff || field_pic; /* MbaffFrameFlag; a PAFF field pair uses the same layout */
                d->paff = field_pic;
                d->qpbdc = 6 * (d->bdc - 8);
                for (int c = 0; c < 3; c++) {
                    int w = c ? d->W / 2 : d->W, h = c ? d->H / 2 : d->H;
                    d->st[c] = w;
                    d->pl[c] = (uint16_t *)calloc((size_t)w * h, 2);
                }
                d->mb = (MbInfo *)calloc((size_t)d->mbw * d->mbh, sizeof(MbInfo));
                for (int k = 0; k < d->mbw * d->mbh; k++) d->mb[k].slice = -1;
                have = 1;
                first_frame_num = frame_num;
                first_idr = type == 5;
            }
            d->p = p;
            d->qp = p->init_qp + qpd;
            d->prev_qpd_nz = 0;
            d->parity = bottom;
            d->fields_seen |= field_pic << bottom;
            /* MBAFF: CurrMbAddr = first_mb_in_slice * 2, macroblocks in pair order (top, bottom);
             * PAFF: field MB addresses (mb_start) */
            int mbaddr = first_mb * (1 + (d->mbaff && !d->paff));
            const int nmb = d->paff ? d->mbw * d->mbh / 2 : d->mbw * d->mbh;
            if (p->cabac) {
                /* cabac_alignment_one_bit */
                while (b.pos & 7) ob_u(&b, 1);
                d->bits = b;
                oc_init(&d->cc, &d->bits);
                init_ctx(d, d->qp);
                for (;;) {
                    if (mbaddr >= nmb) { ret = -7; goto done_free; }
                    mb_start(d, mbaddr, 1);
                    decode_mb(d, d->nslice);
                    if (oc_terminate(&d->cc)) break;
                    mbaddr++;
                }
            } else {
                d->bits = b;
                for (;;) {
                    if (mbaddr >= nmb) { ret = -7; goto done_free; }
                    mb_start(d, mbaddr, 0);
                    if (decode_mb_cavlc(d, d->nslice) < 0) { ret = -21; goto done_free; }
                    if (!ob_more_rbsp(&d->bits)) break;
                    mbaddr++;
                }
            }
            d->nslice++;
            if (d->nslice >= 256) { ret = -8; goto done_free; }
        } else if (type == 9 && have) {
            break;
        }
    }
    if (!have) { ret = -9; goto done; }
    if (d->paff && d->fields_seen != 3) { ret = -3; goto done_free; } /* a field without its pair */
    if (!(flags & 1)) {
        if (d->mbaff) { /* macroblock address order: pairs in raster order, top MB then bottom MB */
            for (int pr = 0; pr < d->mbh / 2; pr++)
                for (int mx = 0; mx < d->mbw; mx++)
                    for (int bt = 0; bt < 2; bt++)
                        if (d->mb[(2 * pr + bt) * d->mbw + mx].slice >= 0) deblock_mb_mbaff(d, mx, 2 * pr + bt);
        } else {
            for (int my = 0; my < d->mbh; my++)
                for (int mx = 0; mx < d->mbw; mx++)
                    if (d->mb[my * d->mbw + mx].slice >= 0) deblock_mb(d, mx, my);
        }
    }
    {
        const H4Sps *s = d->s;
        /* decode.c apply_cropping: the left crop as av_frame_apply_cropping aligns it */
        const int cl = ora_ff_crop_left(s->crop_l, d->bd > 8 ? 2 : 1);
        if (cl < 0) { ret = -10; goto done_free; } /* AVERROR_BUG: avcodec_receive_frame fails */
        int w = d->W - cl - s->crop_r, h = d->H - s->crop_t - s->crop_b;
        out->width = w;
        out->height = h;
        out->bit_depth = d->bd;
        out->chroma_format = 1;
        for (int c = 0; c < 3; c++) {
            /* chroma planes of an odd-sized (4:0:0 crop) picture: AV_CEIL_RSHIFT */
            int sh = c ? 1 : 0, cw = (w + sh) >> sh, ch = (h + sh) >> sh;
            out->planes[c] = (uint16_t *)malloc((size_t)cw * ch * 2);
            out->stride[c] = cw;
            for (int y = 0; y < ch; y++)
                memcpy(out->planes[c] + (size_t)y * cw, d->pl[c] + (size_t)(y + (s->crop_t >> sh)) * d->st[c] + (cl >> sh),
                       (size_t)cw * 2);
        }
    }
    ret = 0;
done_free:
    for (int c = 0; c < 3; c++) free(d->pl[c]);
    free(d->mb);
done:
    free(rbsp);
    free(d);
    free(nals);
    return ret;
}
