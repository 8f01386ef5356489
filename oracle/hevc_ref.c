/*
 * ORACLE — test infrastructure only.  Never linked into the product.
 *
 * Scalar CPU restatement of the HEVC (ITU-T H.265 v1, Main / Main10, 4:2:0)
 * intra decode the reference performs inside FFmpeg's hevc decoder when
 * Decoder::H265ToJpeg calls avcodec_send_packet / avcodec_receive_frame
 * (/root/reference/src/Decoder.cpp:324,342) on the first access unit
 * returned by av_read_frame (:298).  FFmpeg (libavcodec 58.117.101) is
 * binary-only in the reference; this file restates the normative decoding
 * process it implements:
 *   7.3 syntax (VPS/SPS/PPS/slice header/slice data), 9.3 CABAC,
 *   8.4.4.2 intra sample prediction, 8.6 scaling + transform,
 *   8.7.2 deblocking, 8.7.3 SAO.
 * Pinned by SURVEY.md Appendix B (decoded / pre-loop-filter YUV md5 of
 * test/img/img01.h265) and by img01.h265.jpeg.
 *
 * Scope: I slices only (the reference uses the first picture only; stills
 * are IDR/CRA), tiles, WPP, dependent slice segments, PCM, transquant
 * bypass, transform skip, scaling lists, sign data hiding; 8/9/10/12-bit
 * 4:2:0 (FFmpeg hevc_ps.c map_pixel_format: no 11-bit format).
 * Range extensions (H.265 v2 7.3.2.2.2 / 7.3.2.3.2), restated as FFmpeg 4.3
 * hevc_ps.c / hevc_cabac.c / hevcpred_template.c decode them for intra 4:2:0:
 *   implicit RDPCM (transform-skip and transquant-bypass TBs, modes 10 / 26),
 *   transform-skip rotation (4x4, transform skip only -- FFmpeg does not rotate
 *   bypass blocks), transform-skip contexts, persistent Rice adaptation
 *   (FFmpeg does not cap the Rice parameter at 4 then), intra smoothing
 *   disabled, log2_max_transform_skip_block_size, log2_sao_offset_scale
 *   (SaoOffsetVal = offset << scale, in place of v1's bitDepth - 10 shift).
 *   Explicit RDPCM / high-precision offsets only act on inter blocks and
 *   cross-component prediction only in 4:4:4 (no effect here).
 *   Rejected (the picture fails, as the product's): extended precision
 *   processing and CABAC bypass alignment (FFmpeg 4.3: "not yet
 *   implemented"), and chroma QP offset lists enabled in a slice.
 * RExt behaviour has no reference-held fixture: parity unpinned.
 */
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "bits.h"
#include "cabac_tables.h"
#include "oracle.h"

#define MAX_SLICES 1024

/* ------------------------------------------------------------ contexts */
enum {
    C_SAO_MERGE = 0,
    C_SAO_TYPE = 1,
    C_SPLIT_CU = 2,      /* 3 */
    C_TQ_BYPASS = 5,
    C_PART_MODE = 6,
    C_PREV_INTRA = 7,
    C_CHROMA_MODE = 8,
    C_SPLIT_TF = 9,      /* 3 */
    C_CBF_LUMA = 12,     /* 2 */
    C_CBF_CHROMA = 14,   /* 4 */
    C_TSKIP = 18,        /* 2 */
    C_LAST_X = 20,       /* 18 */
    C_LAST_Y = 38,       /* 18 */
    C_CSBF = 56,         /* 4 */
    C_SIG = 60,          /* 44 */
    C_GT1 = 104,         /* 24 */
    C_GT2 = 128,         /* 6 */
    C_QP_DELTA = 134,    /* 2 */
    C_CQO_FLAG = 136,    /* 1 */
    C_CQO_IDX = 137,     /* 1 */
    NUM_CTX = 138
};

static const uint8_t k_init_I[NUM_CTX] = {
    153,                                                   /* sao_merge */
    200,                                                   /* sao_type_idx */
    139, 141, 157,                                         /* split_cu_flag */
    154,                                                   /* cu_transquant_bypass */
    184,                                                   /* part_mode */
    184,                                                   /* prev_intra_luma_pred */
    63,                                                    /* intra_chroma_pred_mode */
    153, 138, 138,                                         /* split_transform_flag */
    111, 141,                                              /* cbf_luma */
    94, 138, 182, 154,                                     /* cbf_cb/cr */
    139, 139,                                              /* transform_skip_flag */
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    91, 171, 134, 141,                                     /* coded_sub_block_flag */
    111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141,
    179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153,
    136, 139, 111, 136, 139, 111, 141, 111,                /* sig_coeff_flag */
    140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166,
    182, 140, 227, 122, 197,                               /* greater1 */
    138, 153, 136, 167, 152, 152,                          /* greater2 */
    154, 154,                                              /* cu_qp_delta_abs */
    154,                                                   /* cu_chroma_qp_offset_flag */
    154,                                                   /* cu_chroma_qp_offset_idx */
};

/* ------------------------------------------------------------ param sets */
typedef struct {
    int valid;
    int chroma_format_idc;
    int width, height;
    int conf_l, conf_r, conf_t, conf_b; /* luma samples */
    int bit_depth, bit_depth_c;
    int log2_max_poc_lsb;
    int log2_min_cb, log2_ctb, log2_min_tb, log2_max_tb;
    int max_th_depth_intra;
    int scaling_list_enabled;
    uint8_t sl[4][6][64];
    uint8_t sl_dc[4][6];
    int sao, pcm, pcm_bd, pcm_bd_c, log2_min_pcm, log2_max_pcm, pcm_lf_disabled;
    int num_st_rps;
    int st_num_delta[65];
    int long_term_present, num_lt_sps;
    int temporal_mvp, strong_intra_smoothing;
    int profile_idc; /* general_profile_idc (4 = FF_PROFILE_HEVC_REXT) */
    /* sps_range_extension (7.3.2.2.2) */
    int ts_rotation, ts_context, implicit_rdpcm, explicit_rdpcm, ext_precision, smoothing_disabled,
        high_prec_offsets, persistent_rice, bypass_alignment;
} Sps;

typedef struct {
    int valid, sps_id;
    int dependent_slices, output_flag_present, num_extra_bits, sign_hiding;
    int init_qp, constrained_intra, transform_skip, cu_qp_delta, diff_cu_qp_delta_depth;
    int cb_qp_offset, cr_qp_offset, slice_chroma_qp_present, transquant_bypass;
    int tiles, wpp, ntc, ntr, uniform, lf_across_tiles;
    int col_w[64], row_h[64];
    int lf_across_slices, deblock_override, deblock_disabled, beta_offset, tc_offset;
    int sl_present;
    uint8_t sl[4][6][64];
    uint8_t sl_dc[4][6];
    int slice_header_ext;
    /* pps_range_extension (7.3.2.3.2), read only for the RExt profile as FFmpeg does */
    int log2_max_ts, cross_component, cqo_list_enabled, cqo_depth, cqo_len;
    int cb_qo_list[6], cr_qo_list[6];
    int sao_scale_luma, sao_scale_chroma;
} Pps;

typedef struct {
    int first_in_pic, dependent, address, slice_addr_rs;
    int pps_id, type;
    int sao_luma, sao_chroma;
    int qp_delta, cb_qp_offset, cr_qp_offset;
    int deblock_disabled, beta_offset, tc_offset, lf_across_slices;
    int cu_chroma_qp_offset_enabled;
    int num_entry;
    int slice_qp;
} SliceHdr;

typedef struct {
    int8_t type[3];   /* 0 none, 1 band, 2 edge */
    int8_t band_pos[3];
    int8_t eo_class[3];
    int16_t off[3][4];
} SaoP;

/* default scaling lists (Table 7-5/7-6), up-right diagonal order */
static const uint8_t k_sl_intra[64] = {
    16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18, 17, 18, 18, 17, 18, 21,
    19, 20, 21, 20, 19, 21, 24, 22, 22, 24, 24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29,
    31, 35, 35, 31, 29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115};
static const uint8_t k_sl_inter[64] = {
    16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18, 18, 18, 18, 18, 18, 20,
    20, 20, 20, 20, 20, 20, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28,
    28, 28, 28, 28, 28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91};

static void sl_default(uint8_t sl[4][6][64], uint8_t dc[4][6]) {
    for (int m = 0; m < 6; m++) {
        memset(sl[0][m], 16, 16);
        for (int s = 1; s < 4; s++) {
            memcpy(sl[s][m], m < 3 ? k_sl_intra : k_sl_inter, 64);
            dc[s][m] = 16;
        }
        dc[0][m] = 16;
    }
}

static void parse_scaling_list(OraBits *b, uint8_t sl[4][6][64], uint8_t dc[4][6]) {
    for (int sizeId = 0; sizeId < 4; sizeId++)
        for (int m = 0; m < 6; m += (sizeId == 3) ? 3 : 1) {
            int n = sizeId == 0 ? 16 : 64;
            if (!ob_u(b, 1)) {
                int delta = (int)ob_ue(b);
                if (delta == 0) {
                    if (sizeId == 0) memset(sl[0][m], 16, 16);
                    else memcpy(sl[sizeId][m], m < 3 ? k_sl_intra : k_sl_inter, 64);
                    dc[sizeId][m] = 16;
                } else {
                    int ref = m - delta * (sizeId == 3 ? 3 : 1);
                    memcpy(sl[sizeId][m], sl[sizeId][ref], (size_t)n);
                    dc[sizeId][m] = dc[sizeId][ref];
                }
            } else {
                int next = 8;
                if (sizeId > 1) {
                    next = ob_se(b) + 8;
                    dc[sizeId][m] = (uint8_t)next;
                }
                for (int i = 0; i < n; i++) {
                    next = (next + ob_se(b) + 256) % 256;
                    sl[sizeId][m][i] = (uint8_t)next;
                }
                if (sizeId <= 1) dc[sizeId][m] = sl[sizeId][m][0];
            }
        }
    /* 4:2:0 never uses 32x32 chroma lists; mirror luma for completeness */
    for (int m = 1; m < 6; m++)
        if (m != 3) {
            memcpy(sl[3][m], sl[2][m], 64);
            dc[3][m] = dc[2][m];
        }
}

/* profile_tier_level (7.3.3); returns general_profile_idc, taken from the compatibility flags
 * when it is 0 (FFmpeg hevc_ps.c decode_profile_tier_level) */
static int parse_ptl(OraBits *b, int max_sub_layers_minus1) {
    ob_u(b, 3);       /* profile space, tier */
    int prof = (int)ob_u(b, 5);
    for (int j = 0; j < 32; j++)
        if (ob_u(b, 1) && prof == 0 && j > 0) prof = j;
    ob_u(b, 4);       /* progressive, interlaced, non-packed, frame-only */
    ob_u(b, 32);
    ob_u(b, 11);      /* 43 reserved bits */
    ob_u(b, 1);
    ob_u(b, 8);       /* level */
    int pp[8] = {0}, lp[8] = {0};
    for (int i = 0; i < max_sub_layers_minus1; i++) {
        pp[i] = (int)ob_u(b, 1);
        lp[i] = (int)ob_u(b, 1);
    }
    if (max_sub_layers_minus1 > 0)
        for (int i = max_sub_layers_minus1; i < 8; i++) ob_u(b, 2);
    for (int i = 0; i < max_sub_layers_minus1; i++) {
        if (pp[i]) { ob_u(b, 32); ob_u(b, 32); ob_u(b, 24); }
        if (lp[i]) ob_u(b, 8);
    }
    return prof;
}

/* hrd_parameters (E.2.2) and sub_layer_hrd_parameters (E.2.3): skipped (FFmpeg decode_hrd) */
static int skip_hrd(OraBits *b, int common, int max_sub_layers) {
    int nal = 0, vcl = 0, sub_pic = 0;
    if (common) {
        nal = (int)ob_u(b, 1);
        vcl = (int)ob_u(b, 1);
        if (nal || vcl) {
            sub_pic = (int)ob_u(b, 1);
            if (sub_pic) ob_u(b, 19);
            ob_u(b, 8);
            if (sub_pic) ob_u(b, 4);
            ob_u(b, 15);
        }
    }
    for (int i = 0; i < max_sub_layers; i++) {
        int low_delay = 0;
        uint32_t nb_cpb = 1;
        int fixed = (int)ob_u(b, 1);
        if (!fixed) fixed = (int)ob_u(b, 1);
        if (fixed) ob_ue(b);
        else low_delay = (int)ob_u(b, 1);
        if (!low_delay) {
            nb_cpb = ob_ue(b) + 1;
            if (nb_cpb < 1 || nb_cpb > 32) return -1;
        }
        for (int k = 0; k < nal + vcl; k++)
            for (uint32_t j = 0; j < nb_cpb; j++) {
                ob_ue(b);
                ob_ue(b);
                if (sub_pic) { ob_ue(b); ob_ue(b); }
                ob_u(b, 1);
            }
    }
    return 0;
}

/* vui_parameters (E.2.1), skipped: nothing in it changes the decoded samples (the default display
 * window is not applied by default, FFmpeg's apply_defdispwin = 0) */
static int skip_vui(OraBits *b, int max_sub_layers) {
    if (ob_u(b, 1) && ob_u(b, 8) == 255) ob_u(b, 32); /* aspect_ratio_idc, EXTENDED_SAR */
    if (ob_u(b, 1)) ob_u(b, 1);                        /* overscan */
    if (ob_u(b, 1)) {                                  /* video signal type */
        ob_u(b, 4);
        if (ob_u(b, 1)) ob_u(b, 24);
    }
    if (ob_u(b, 1)) { ob_ue(b); ob_ue(b); }            /* chroma loc */
    ob_u(b, 3); /* neutral chroma, field_seq, frame_field_info */
    if (ob_u(b, 1)) { ob_ue(b); ob_ue(b); ob_ue(b); ob_ue(b); } /* default display window */
    if (ob_u(b, 1)) {                                  /* timing */
        ob_u(b, 32);
        ob_u(b, 32);
        if (ob_u(b, 1)) ob_ue(b);
        if (ob_u(b, 1) && skip_hrd(b, 1, max_sub_layers) < 0) return -1;
    }
    if (ob_u(b, 1)) {                                  /* bitstream restriction */
        ob_u(b, 3);
        for (int i = 0; i < 5; i++) ob_ue(b);
    }
    return 0;
}

static int parse_st_rps(OraBits *b, Sps *s, int idx) {
    int inter = 0;
    if (idx != 0) inter = (int)ob_u(b, 1);
    if (inter) {
        int delta_idx = 1;
        if (idx == s->num_st_rps) delta_idx = (int)ob_ue(b) + 1;
        ob_u(b, 1);  /* delta_rps_sign */
        ob_ue(b);    /* abs_delta_rps_minus1 */
        int ref = idx - delta_idx;
        if (ref < 0) return -1;
        int cnt = 0;
        for (int j = 0; j <= s->st_num_delta[ref]; j++) {
            int used = (int)ob_u(b, 1), use_delta = 1;
            if (!used) use_delta = (int)ob_u(b, 1);
            if (used || use_delta) cnt++;
        }
        s->st_num_delta[idx] = cnt;
    } else {
        int neg = (int)ob_ue(b), pos = (int)ob_ue(b);
        if (neg > 16 || pos > 16) return -1;
        for (int i = 0; i < neg + pos; i++) {
            ob_ue(b);
            ob_u(b, 1);
        }
        s->st_num_delta[idx] = neg + pos;
    }
    return 0;
}

static int parse_sps(OraBits *b, Sps *tab) {
    ob_u(b, 4);
    int msl = (int)ob_u(b, 3);
    ob_u(b, 1);
    int prof = parse_ptl(b, msl);
    int id = (int)ob_ue(b);
    if (id > 15) return -1;
    Sps *s = &tab[id];
    memset(s, 0, sizeof(*s));
    s->profile_idc = prof;
    s->chroma_format_idc = (int)ob_ue(b);
    if (s->chroma_format_idc == 3) ob_u(b, 1);
    uint32_t w = ob_ue(b), h = ob_ue(b);
    if (w == 0 || h == 0 || w > 16888 || h > 16888) return -1;
    s->width = (int)w;
    s->height = (int)h;
    if (ob_u(b, 1)) {
        /* FFmpeg hevc_ps.c: offsets that leave no picture are ignored ("Invalid cropping
         * offsets", "Displaying the whole video surface") unless AV_EF_EXPLODE */
        uint64_t sw = (s->chroma_format_idc == 1 || s->chroma_format_idc == 2) ? 2 : 1;
        uint64_t shh = s->chroma_format_idc == 1 ? 2 : 1;
        uint64_t l = ob_ue(b) * sw, r = ob_ue(b) * sw, t = ob_ue(b) * shh, bo = ob_ue(b) * shh;
        if (l + r < w && t + bo < h) {
            s->conf_l = (int)l;
            s->conf_r = (int)r;
            s->conf_t = (int)t;
            s->conf_b = (int)bo;
        }
    }
    s->bit_depth = (int)ob_ue(b) + 8;
    s->bit_depth_c = (int)ob_ue(b) + 8;
    s->log2_max_poc_lsb = (int)ob_ue(b) + 4;
    int sub = (int)ob_u(b, 1);
    for (int i = sub ? 0 : msl; i <= msl; i++) { ob_ue(b); ob_ue(b); ob_ue(b); }
    s->log2_min_cb = (int)ob_ue(b) + 3;
    s->log2_ctb = s->log2_min_cb + (int)ob_ue(b);
    s->log2_min_tb = (int)ob_ue(b) + 2;
    s->log2_max_tb = s->log2_min_tb + (int)ob_ue(b);
    ob_ue(b); /* max_transform_hierarchy_depth_inter */
    s->max_th_depth_intra = (int)ob_ue(b);
    s->scaling_list_enabled = (int)ob_u(b, 1);
    sl_default(s->sl, s->sl_dc);
    if (s->scaling_list_enabled && ob_u(b, 1)) parse_scaling_list(b, s->sl, s->sl_dc);
    ob_u(b, 1); /* amp */
    s->sao = (int)ob_u(b, 1);
    s->pcm = (int)ob_u(b, 1);
    if (s->pcm) {
        s->pcm_bd = (int)ob_u(b, 4) + 1;
        s->pcm_bd_c = (int)ob_u(b, 4) + 1;
        s->log2_min_pcm = (int)ob_ue(b) + 3;
        s->log2_max_pcm = s->log2_min_pcm + (int)ob_ue(b);
        s->pcm_lf_disabled = (int)ob_u(b, 1);
    }
    s->num_st_rps = (int)ob_ue(b);
    if (s->num_st_rps > 64) return -1;
    for (int i = 0; i < s->num_st_rps; i++)
        if (parse_st_rps(b, s, i) < 0) return -1;
    s->long_term_present = (int)ob_u(b, 1);
    if (s->long_term_present) {
        s->num_lt_sps = (int)ob_ue(b);
        for (int i = 0; i < s->num_lt_sps; i++) {
            ob_u(b, s->log2_max_poc_lsb);
            ob_u(b, 1);
        }
    }
    s->temporal_mvp = (int)ob_u(b, 1);
    s->strong_intra_smoothing = (int)ob_u(b, 1);
    if (ob_u(b, 1) && skip_vui(b, msl + 1) < 0) return -1;
    if (ob_u(b, 1)) {                  /* sps_extension_present_flag */
        int range = (int)ob_u(b, 1);  /* sps_range_extension_flag */
        ob_u(b, 7);                    /* multilayer, 3d, scc, 4bits: not read (FFmpeg 4.3) */
        if (range) {
            s->ts_rotation = (int)ob_u(b, 1);
            s->ts_context = (int)ob_u(b, 1);
            s->implicit_rdpcm = (int)ob_u(b, 1);
            s->explicit_rdpcm = (int)ob_u(b, 1);
            s->ext_precision = (int)ob_u(b, 1);
            s->smoothing_disabled = (int)ob_u(b, 1);
            s->high_prec_offsets = (int)ob_u(b, 1);
            s->persistent_rice = (int)ob_u(b, 1);
            s->bypass_alignment = (int)ob_u(b, 1);
        }
    }
    if (s->chroma_format_idc != 1) return -2;
    /* FFmpeg map_pixel_format: 4:2:0 at 8, 9, 10, 12 bits; luma and chroma depths equal */
    if (s->bit_depth != 8 && s->bit_depth != 9 && s->bit_depth != 10 && s->bit_depth != 12) return -3;
    if (s->bit_depth_c != s->bit_depth) return -3;
    /* extended_precision_processing_flag / cabac_bypass_alignment_enabled_flag: FFmpeg 4.3 hevc_ps.c
     * logs "... not yet implemented" and decodes as if they were 0 (no other effect here either) */
    if (s->log2_ctb > 6 || s->log2_ctb < 4 || s->log2_max_tb > 5) return -3;
    /* FFmpeg hevc_ps.c: "Invalid coded frame dimensions" */
    if ((s->width & ((1 << s->log2_min_cb) - 1)) || (s->height & ((1 << s->log2_min_cb) - 1))) return -1;
    s->valid = 1;
    return 0;
}

static int parse_pps(OraBits *b, Pps *tab, const Sps *stab) {
    int id = (int)ob_ue(b);
    if (id > 63) return -1;
    Pps *p = &tab[id];
    memset(p, 0, sizeof(*p));
    p->sps_id = (int)ob_ue(b);
    if (p->sps_id > 15 || !stab[p->sps_id].valid) return -1; /* FFmpeg: "SPS %u does not exist" */
    const Sps *sps = &stab[p->sps_id];
    p->log2_max_ts = 2;
    p->dependent_slices = (int)ob_u(b, 1);
    p->output_flag_present = (int)ob_u(b, 1);
    p->num_extra_bits = (int)ob_u(b, 3);
    p->sign_hiding = (int)ob_u(b, 1);
    ob_u(b, 1); /* cabac_init_present */
    ob_ue(b);
    ob_ue(b);
    p->init_qp = 26 + ob_se(b);
    p->constrained_intra = (int)ob_u(b, 1);
    p->transform_skip = (int)ob_u(b, 1);
    p->cu_qp_delta = (int)ob_u(b, 1);
    if (p->cu_qp_delta) p->diff_cu_qp_delta_depth = (int)ob_ue(b);
    p->cb_qp_offset = ob_se(b);
    p->cr_qp_offset = ob_se(b);
    p->slice_chroma_qp_present = (int)ob_u(b, 1);
    ob_u(b, 1); /* weighted pred */
    ob_u(b, 1); /* weighted bipred */
    p->transquant_bypass = (int)ob_u(b, 1);
    p->tiles = (int)ob_u(b, 1);
    p->wpp = (int)ob_u(b, 1);
    p->ntc = p->ntr = 1;
    p->uniform = 1;
    p->lf_across_tiles = 1;
    if (p->tiles) {
        p->ntc = (int)ob_ue(b) + 1;
        p->ntr = (int)ob_ue(b) + 1;
        if (p->ntc > 64 || p->ntr > 64) return -1;
        p->uniform = (int)ob_u(b, 1);
        if (!p->uniform) {
            for (int i = 0; i < p->ntc - 1; i++) p->col_w[i] = (int)ob_ue(b) + 1;
            for (int i = 0; i < p->ntr - 1; i++) p->row_h[i] = (int)ob_ue(b) + 1;
        }
        p->lf_across_tiles = (int)ob_u(b, 1);
    }
    p->lf_across_slices = (int)ob_u(b, 1);
    if (ob_u(b, 1)) {
        p->deblock_override = (int)ob_u(b, 1);
        p->deblock_disabled = (int)ob_u(b, 1);
        if (!p->deblock_disabled) {
            p->beta_offset = ob_se(b) * 2;
            p->tc_offset = ob_se(b) * 2;
        }
    }
    p->sl_present = (int)ob_u(b, 1);
    if (p->sl_present) {
        sl_default(p->sl, p->sl_dc);
        parse_scaling_list(b, p->sl, p->sl_dc);
    }
    ob_u(b, 1); /* lists_modification_present */
    ob_ue(b);   /* log2_parallel_merge_level */
    p->slice_header_ext = (int)ob_u(b, 1);
    if (ob_u(b, 1)) {                  /* pps_extension_present_flag */
        int range = (int)ob_u(b, 1);
        ob_u(b, 7);
        if (range && sps->profile_idc == 4) {  /* FFmpeg: only for FF_PROFILE_HEVC_REXT */
            if (p->transform_skip) {
                uint32_t v = ob_ue(b);
                if (v > 3) return -1;
                p->log2_max_ts = (int)v + 2;
            }
            p->cross_component = (int)ob_u(b, 1);
            p->cqo_list_enabled = (int)ob_u(b, 1);
            if (p->cqo_list_enabled) {
                p->cqo_depth = (int)ob_ue(b);
                uint32_t len = ob_ue(b);
                if (len > 5) return -1;
                p->cqo_len = (int)len + 1;
                for (int i = 0; i < p->cqo_len; i++) {
                    p->cb_qo_list[i] = ob_se(b);
                    p->cr_qo_list[i] = ob_se(b);
                }
            }
            uint32_t sl = ob_ue(b), sc = ob_ue(b);
            int lim = sps->bit_depth > 10 ? sps->bit_depth - 10 : 0;
            if (sl > (uint32_t)lim || sc > (uint32_t)lim) return -1;
            p->sao_scale_luma = (int)sl;
            p->sao_scale_chroma = (int)sc;
        }
    }
    p->valid = 1;
    return 0;
}

/* ------------------------------------------------------------ decoder */
typedef struct {
    Sps sps[16];
    Pps pps[64];
    const Sps *s;
    const Pps *p;
    int W, H, log2ctb, ctbs, ctbW, ctbH, nctb, mw, mh; /* mw/mh: 4x4 map dims */
    int bd, bdc, qpbd, qpbdc;
    uint16_t *pl[3];
    int st[3], pw[3], ph[3];
    /* per 4x4 maps */
    int8_t *qp;
    uint8_t *ipm, *ctd, *nofilt, *bsv, *bsh;
    /* per CTB */
    int *ctb_slice, *ctb_addr_rs;    /* slice header index, SliceAddrRs */
    int *rs2ts, *ts2rs, *tile_id, *col_bd, *row_bd;
    SaoP *sao;
    SliceHdr sh[MAX_SLICES];
    int nsh;
    /* slice decoding state */
    SliceHdr *cur;
    OraCabac cc;
    OraBits bits;
    uint8_t ctx[NUM_CTX];
    uint8_t ctx_wpp[NUM_CTX];
    uint8_t ctx_ds[NUM_CTX]; /* end of previous slice segment (dependent slices) */
    /* StatCoeff (persistent_rice_adaptation, 9.3.2.2): initialised, stored and synchronised with
     * the context variables (FFmpeg cabac_init_state / ff_hevc_save_states / load_states) */
    int stat[4], stat_wpp[4], stat_ds[4];
    int have_ds;
    int qp_y, qp_pred_prev, is_qpd_coded, qpd_val, first_qg, qg_pred, last_cu_qp;
    int cu_bypass;
    int cqo_coded, cu_qo_cb, cu_qo_cr; /* IsCuChromaQpOffsetCoded, CuQpOffsetCb / Cr */
    int sl_enabled;
    const uint8_t (*slist)[6][64];
    const uint8_t (*slist_dc)[6];
    int16_t coeff[32 * 32];
} Dec;

static int min_tb_zs(const Dec *d, int x, int y) {
    int ctb = (y >> d->log2ctb) * d->ctbW + (x >> d->log2ctb);
    int xi = (x & (d->ctbs - 1)) >> 2, yi = (y & (d->ctbs - 1)) >> 2, z = 0;
    for (int i = 0; i < 5; i++) z |= (((xi >> i) & 1) << (2 * i)) | (((yi >> i) & 1) << (2 * i + 1));
    return (d->rs2ts[ctb] << (2 * (d->log2ctb - 2))) + z;
}

/* 6.4.1 z-scan order availability */
static int avail(const Dec *d, int xc, int yc, int xn, int yn) {
    if (xn < 0 || yn < 0 || xn >= d->W || yn >= d->H) return 0;
    int cn = (yn >> d->log2ctb) * d->ctbW + (xn >> d->log2ctb);
    int cc = (yc >> d->log2ctb) * d->ctbW + (xc >> d->log2ctb);
    if (d->ctb_slice[cn] < 0) return 0;
    if (min_tb_zs(d, xn, yn) > min_tb_zs(d, xc, yc)) return 0;
    if (d->ctb_addr_rs[cn] != d->ctb_addr_rs[cc]) return 0;
    if (d->tile_id[d->rs2ts[cn]] != d->tile_id[d->rs2ts[cc]]) return 0;
    return 1;
}

static void init_contexts(Dec *d, int qp) {
    if (qp < 0) qp = 0;
    if (qp > 51) qp = 51;
    for (int i = 0; i < NUM_CTX; i++) {
        int iv = k_init_I[i];
        int m = (iv >> 4) * 5 - 45, n = ((iv & 15) << 3) - 16;
        int pre = ((m * qp) >> 4) + n;
        if (pre < 1) pre = 1;
        if (pre > 126) pre = 126;
        int mps = pre <= 63 ? 0 : 1;
        int st = mps ? pre - 64 : 63 - pre;
        d->ctx[i] = (uint8_t)((st << 1) | mps);
    }
    memset(d->stat, 0, sizeof(d->stat));
}

static inline int dec_bin(Dec *d, int ctx) { return oc_decision(&d->cc, &d->ctx[ctx]); }
static inline int dec_byp(Dec *d) { return oc_bypass(&d->cc); }
static inline int dec_bypn(Dec *d, int n) {
    int v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | dec_byp(d);
    return v;
}

/* ------------------------------------------------------------ scans */
static uint8_t scan_diag[4][64][2]; /* log2 size 0..3 */
static uint8_t scan_hor[4][64][2], scan_ver[4][64][2];
static int scans_ready = 0;

static void init_scans(void) {
    if (scans_ready) return;
    for (int l = 0; l < 4; l++) {
        int bs = 1 << l, i = 0, x = 0, y = 0;
        while (i < bs * bs) {
            while (y >= 0) {
                if (x < bs && y < bs) {
                    scan_diag[l][i][0] = (uint8_t)x;
                    scan_diag[l][i][1] = (uint8_t)y;
                    i++;
                }
                y--;
                x++;
            }
            y = x;
            x = 0;
        }
        i = 0;
        for (y = 0; y < bs; y++)
            for (x = 0; x < bs; x++, i++) {
                scan_hor[l][i][0] = (uint8_t)x;
                scan_hor[l][i][1] = (uint8_t)y;
            }
        i = 0;
        for (x = 0; x < bs; x++)
            for (y = 0; y < bs; y++, i++) {
                scan_ver[l][i][0] = (uint8_t)x;
                scan_ver[l][i][1] = (uint8_t)y;
            }
    }
    scans_ready = 1;
}

static const uint8_t (*scan_tab(int scanIdx))[64][2] {
    return scanIdx == 0 ? scan_diag : (scanIdx == 1 ? scan_hor : scan_ver);
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
            int v = a > 32 ? -C[64 - a] : C[a];
            tm32[m][n] = (int8_t)(v > 127 ? 127 : v); /* all |v| <= 90 */
        }
}
static const int k_dst[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};

static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

static void inv_1d(const int *x, int *y, int n, int dst) {
    for (int i = 0; i < n; i++) {
        int64_t s = 0;
        for (int j = 0; j < n; j++) {
            int c = dst ? k_dst[j][i] : tm32[j * (32 / n)][i];
            s += (int64_t)c * x[j];
        }
        y[i] = (int)s;
    }
}

/* d[y*n+x] scaled coeffs -> r residuals (8.6.4.2) */
static void inv_transform(const int *d, int *r, int n, int dst, int bd) {
    int tmp[32 * 32], col[32], out[32];
    for (int x = 0; x < n; x++) {
        for (int y = 0; y < n; y++) col[y] = d[y * n + x];
        inv_1d(col, out, n, dst);
        for (int y = 0; y < n; y++) tmp[y * n + x] = clip3(-32768, 32767, (out[y] + 64) >> 7);
    }
    int bdShift = 20 - bd;
    for (int y = 0; y < n; y++) {
        inv_1d(tmp + y * n, out, n, dst);
        for (int x = 0; x < n; x++) r[y * n + x] = (out[x] + (1 << (bdShift - 1))) >> bdShift;
    }
}

/* ------------------------------------------------------------ intra pred */
static const int k_angle[35] = {0,   0,   32,  26,  21,  17,  13,  9,  5,  2,  0,  -2,
                                -5,  -9,  -13, -17, -21, -26, -32, -26, -21, -17, -13, -9,
                                -5,  -2,  0,   2,   5,   9,   13,  17,  21,  26,  32};
static const int k_inv_angle[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482,
                                    -390, -315, -256, -315, -390, -482, -630, -910, -1638, -4096};

/* 8.4.4.2: predict nT x nT block of component c at (x0,y0) (component coords) */
static void intra_pred(Dec *d, int c, int x0, int y0, int log2n, int mode) {
    const int n = 1 << log2n;
    const int sh = c ? 1 : 0;
    const int bd = c ? d->bdc : d->bd;
    const int maxv = (1 << bd) - 1;
    uint16_t *pl = d->pl[c];
    const int st = d->st[c];
    /* ref samples: p[-1][-1+k] for k=0..2n (left incl corner), p[-1+k][-1] (top incl corner) */
    int ref_l[129] = {0}, ref_t[129] = {0}; /* ref_l[k] = p[-1][k-1] k=0..2n ; ref_t[k] = p[k-1][-1] */
    int av_l[129], av_t[129];
    int xl = x0 << sh, yl = y0 << sh; /* current luma location */
    int cnt = 0;
    for (int k = 0; k <= 2 * n; k++) {
        int yy = y0 + k - 1, xx = x0 - 1;
        int a = avail(d, xl, yl, xx << sh, yy << sh);
        av_l[k] = a;
        ref_l[k] = a ? pl[yy * st + xx] : 0;
        cnt += a;
    }
    for (int k = 1; k <= 2 * n; k++) {
        int yy = y0 - 1, xx = x0 + k - 1;
        int a = avail(d, xl, yl, xx << sh, yy << sh);
        av_t[k] = a;
        ref_t[k] = a ? pl[yy * st + xx] : 0;
        cnt += a;
    }
    av_t[0] = av_l[0];
    ref_t[0] = ref_l[0];
    /* 8.4.4.2.2 substitution */
    if (cnt == 0) {
        for (int k = 0; k <= 2 * n; k++) ref_l[k] = ref_t[k] = 1 << (bd - 1);
    } else {
        /* search order: p[-1][2n-1] up to p[-1][-1], then p[0][-1] .. p[2n-1][-1] */
        int seq[257], av[257], m = 0;
        for (int k = 2 * n; k >= 0; k--) { seq[m] = ref_l[k]; av[m] = av_l[k]; m++; }
        for (int k = 1; k <= 2 * n; k++) { seq[m] = ref_t[k]; av[m] = av_t[k]; m++; }
        if (!av[0]) {
            int f = 1;
            while (!av[f]) f++;
            seq[0] = seq[f];
            av[0] = 1;
        }
        for (int i = 1; i < m; i++)
            if (!av[i]) seq[i] = seq[i - 1];
        m = 0;
        for (int k = 2 * n; k >= 0; k--) ref_l[k] = seq[m++];
        for (int k = 1; k <= 2 * n; k++) ref_t[k] = seq[m++];
        ref_t[0] = ref_l[0];
    }
    /* 8.4.4.2.3 filtering (luma only for 4:2:0; none with RExt intra_smoothing_disabled_flag) */
    if (c == 0 && mode != 1 && n != 4 && !d->s->smoothing_disabled) {
        int mdist = abs(mode - 26) < abs(mode - 10) ? abs(mode - 26) : abs(mode - 10);
        int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
        if (mode == 0 || mdist > thr) {
            int fl[129], ft[129];
            int corner = ref_l[0];
            if (d->s->strong_intra_smoothing && n == 32 &&
                abs(corner + ref_t[2 * n] - 2 * ref_t[n]) < (1 << (bd - 5)) &&
                abs(corner + ref_l[2 * n] - 2 * ref_l[n]) < (1 << (bd - 5))) {
                fl[0] = ft[0] = corner;
                for (int y = 0; y < 63; y++)
                    fl[y + 1] = ((63 - y) * corner + (y + 1) * ref_l[64] + 32) >> 6;
                fl[64] = ref_l[64];
                for (int x = 0; x < 63; x++)
                    ft[x + 1] = ((63 - x) * corner + (x + 1) * ref_t[64] + 32) >> 6;
                ft[64] = ref_t[64];
            } else {
                fl[0] = ft[0] = (ref_l[1] + 2 * corner + ref_t[1] + 2) >> 2;
                for (int k = 1; k < 2 * n; k++) {
                    int up = k == 1 ? corner : ref_l[k - 1];
                    fl[k] = (ref_l[k + 1] + 2 * ref_l[k] + up + 2) >> 2;
                    int lf = k == 1 ? corner : ref_t[k - 1];
                    ft[k] = (ref_t[k + 1] + 2 * ref_t[k] + lf + 2) >> 2;
                }
                fl[2 * n] = ref_l[2 * n];
                ft[2 * n] = ref_t[2 * n];
            }
            memcpy(ref_l, fl, sizeof(int) * (2 * n + 1));
            memcpy(ref_t, ft, sizeof(int) * (2 * n + 1));
        }
    }
    /* p(x,-1) = ref_t[x+1], p(-1,y) = ref_l[y+1], p(-1,-1) = ref_l[0] */
#define PT(x) ref_t[(x) + 1]
#define PL(y) ref_l[(y) + 1]
    int pred[32 * 32];
    if (mode == 0) {
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++)
                pred[y * n + x] = ((n - 1 - x) * PL(y) + (x + 1) * PT(n) + (n - 1 - y) * PT(x) +
                                   (y + 1) * PL(n) + n) >> (log2n + 1);
    } else if (mode == 1) {
        int sum = n;
        for (int k = 0; k < n; k++) sum += PT(k) + PL(k);
        int dc = sum >> (log2n + 1);
        for (int i = 0; i < n * n; i++) pred[i] = dc;
        if (c == 0 && n < 32) {
            pred[0] = (PL(0) + 2 * dc + PT(0) + 2) >> 2;
            for (int x = 1; x < n; x++) pred[x] = (PT(x) + 3 * dc + 2) >> 2;
            for (int y = 1; y < n; y++) pred[y * n] = (PL(y) + 3 * dc + 2) >> 2;
        }
    } else {
        int angle = k_angle[mode];
        int refa[3 * 64 + 1];
        int *ref = refa + 64;
        if (mode >= 18) {
            for (int x = 0; x <= n; x++) ref[x] = x == 0 ? ref_l[0] : PT(x - 1);
            if (angle < 0) {
                if ((n * angle) >> 5 < -1)
                    for (int x = (n * angle) >> 5; x <= -1; x++)
                        ref[x] = ref_l[((x * k_inv_angle[mode] + 128) >> 8)];
            } else {
                for (int x = n + 1; x <= 2 * n; x++) ref[x] = PT(x - 1);
            }
            for (int y = 0; y < n; y++) {
                int idx = ((y + 1) * angle) >> 5, f = ((y + 1) * angle) & 31;
                for (int x = 0; x < n; x++)
                    pred[y * n + x] = f ? ((32 - f) * ref[x + idx + 1] + f * ref[x + idx + 2] + 16) >> 5
                                        : ref[x + idx + 1];
            }
            if (mode == 26 && c == 0 && n < 32)
                for (int y = 0; y < n; y++)
                    pred[y * n] = clip3(0, maxv, PT(0) + ((PL(y) - ref_l[0]) >> 1));
        } else {
            for (int x = 0; x <= n; x++) ref[x] = ref_l[x]; /* p(-1, -1+x) */
            if (angle < 0) {
                if ((n * angle) >> 5 < -1)
                    for (int x = (n * angle) >> 5; x <= -1; x++)
                        ref[x] = ref_t[((x * k_inv_angle[mode] + 128) >> 8)];
            } else {
                for (int x = n + 1; x <= 2 * n; x++) ref[x] = ref_l[x];
            }
            for (int x = 0; x < n; x++) {
                int idx = ((x + 1) * angle) >> 5, f = ((x + 1) * angle) & 31;
                for (int y = 0; y < n; y++)
                    pred[y * n + x] = f ? ((32 - f) * ref[y + idx + 1] + f * ref[y + idx + 2] + 16) >> 5
                                        : ref[y + idx + 1];
            }
            if (mode == 10 && c == 0 && n < 32)
                for (int x = 0; x < n; x++)
                    pred[x] = clip3(0, maxv, PL(0) + ((PT(x) - ref_l[0]) >> 1));
        }
    }
#undef PT
#undef PL
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) pl[(y0 + y) * st + x0 + x] = (uint16_t)pred[y * n + x];
}

/* ------------------------------------------------------------ QP */
static int chroma_qp_table(int qpi) {
    static const int t[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    return t[qpi - 30];
}

static int qp_at(const Dec *d, int x, int y) { return d->qp[(y >> 2) * d->mw + (x >> 2)]; }

/* 8.6.1, invoked at the start of a quantization group */
static void qg_start(Dec *d, int xq, int yq) {
    int prev = d->first_qg ? d->cur->slice_qp : d->qp_pred_prev;
    d->first_qg = 0;
    int ctb = (yq >> d->log2ctb) * d->ctbW + (xq >> d->log2ctb);
    int qa = prev, qb = prev;
    if (avail(d, xq, yq, xq - 1, yq) && ((yq >> d->log2ctb) * d->ctbW + ((xq - 1) >> d->log2ctb)) == ctb)
        qa = qp_at(d, xq - 1, yq);
    if (avail(d, xq, yq, xq, yq - 1) && (((yq - 1) >> d->log2ctb) * d->ctbW + (xq >> d->log2ctb)) == ctb)
        qb = qp_at(d, xq, yq - 1);
    int pred = (qa + qb + 1) >> 1;
    d->qp_y = pred; /* CuQpDeltaVal = 0 */
    d->qpd_val = 0;
    d->is_qpd_coded = 0;
    d->qg_pred = pred;
}

/* ------------------------------------------------------------ residual */
static int decode_last_prefix(Dec *d, int base, int log2n, int c) {
    int off, shift;
    if (c == 0) {
        off = 3 * (log2n - 2) + ((log2n - 1) >> 2);
        shift = (log2n + 1) >> 2;
    } else {
        off = 15;
        shift = log2n - 2;
    }
    int maxv = (log2n << 1) - 1, i = 0;
    while (i < maxv && dec_bin(d, base + off + (i >> shift))) i++;
    return i;
}

static int decode_alr(Dec *d, int rice) {
    int prefix = 0;
    while (prefix < 32 && dec_byp(d)) prefix++;
    if (prefix < 3) return (prefix << rice) + dec_bypn(d, rice);
    int pm3 = prefix - 3;
    return (((1 << pm3) + 3 - 1) << rice) + dec_bypn(d, pm3 + rice);
}

static void residual_coding(Dec *d, int x0, int y0, int log2n, int c, int pred_mode,
                            int *tskip_out) {
    const int n = 1 << log2n;
    int16_t *coef = d->coeff;
    memset(coef, 0, sizeof(int16_t) * n * n);
    int tskip = 0;
    if (d->p->transform_skip && !d->cu_bypass && log2n <= d->p->log2_max_ts) tskip = dec_bin(d, C_TSKIP + (c ? 1 : 0));
    *tskip_out = tskip;
    const Sps *sps = d->s;
    /* RExt: transform-skip / bypass blocks use one significance context per component */
    const int ts_ctx = sps->ts_context && (tskip || d->cu_bypass);
    /* implicit RDPCM (intra, transform skip, mode 10 / 26) turns sign data hiding off */
    const int rdpcm_ts = sps->implicit_rdpcm && tskip && (pred_mode == 10 || pred_mode == 26);
    const int sb_type = 2 * (c == 0 ? 1 : 0) + ((tskip || d->cu_bypass) ? 1 : 0);
    int lx = decode_last_prefix(d, C_LAST_X, log2n, c);
    int ly = decode_last_prefix(d, C_LAST_Y, log2n, c);
    if (lx > 3) {
        int nb = (lx >> 1) - 1;
        lx = (1 << nb) * (2 + (lx & 1)) + dec_bypn(d, nb);
    }
    if (ly > 3) {
        int nb = (ly >> 1) - 1;
        ly = (1 << nb) * (2 + (ly & 1)) + dec_bypn(d, nb);
    }
    int scanIdx = 0;
    if (log2n == 2 || (log2n == 3 && c == 0)) {
        if (pred_mode >= 6 && pred_mode <= 14) scanIdx = 2;
        else if (pred_mode >= 22 && pred_mode <= 30) scanIdx = 1;
    }
    if (scanIdx == 2) {
        int t = lx;
        lx = ly;
        ly = t;
    }
    const uint8_t(*sc)[64][2] = scan_tab(scanIdx);
    const int lsb = log2n - 2;
    int lastSub = (1 << (2 * lsb)) - 1, lastPos = 16;
    int xc, yc;
    do {
        if (lastPos == 0) {
            lastPos = 16;
            lastSub--;
        }
        lastPos--;
        int xs = sc[lsb][lastSub][0], ys = sc[lsb][lastSub][1];
        xc = (xs << 2) + sc[2][lastPos][0];
        yc = (ys << 2) + sc[2][lastPos][1];
    } while (xc != lx || yc != ly);

    uint8_t csbf[8][8];
    memset(csbf, 0, sizeof(csbf));
    int greater1_ctx = 1;
    const int sign_hiding_en = d->p->sign_hiding;
    for (int i = lastSub; i >= 0; i--) {
        int xs = sc[lsb][i][0], ys = sc[lsb][i][1];
        int infer_dc = 0;
        if (i < lastSub && i > 0) {
            int csr = (xs + 1 < (1 << lsb)) ? csbf[xs + 1][ys] : 0;
            int csb = (ys + 1 < (1 << lsb)) ? csbf[xs][ys + 1] : 0;
            int ctx = (csr | csb) + (c ? 2 : 0);
            csbf[xs][ys] = (uint8_t)dec_bin(d, C_CSBF + ctx);
            infer_dc = 1;
        } else {
            csbf[xs][ys] = 1;
        }
        int sig[16];
        memset(sig, 0, sizeof(sig));
        int nstart = 15;
        if (i == lastSub) {
            nstart = lastPos - 1;
            sig[lastPos] = 1;
        }
        int prevCsbf = 0;
        if (xs + 1 < (1 << lsb)) prevCsbf |= csbf[xs + 1][ys];
        if (ys + 1 < (1 << lsb)) prevCsbf |= csbf[xs][ys + 1] << 1;
        for (int nn = nstart; nn >= 0; nn--) {
            int xp = sc[2][nn][0], yp = sc[2][nn][1];
            int xC = (xs << 2) + xp, yC = (ys << 2) + yp;
            if (csbf[xs][ys] && (nn > 0 || !infer_dc)) {
                int sigCtx;
                if (ts_ctx) {
                    sigCtx = c == 0 ? 42 : 16;
                } else if (log2n == 2) {
                    static const uint8_t ctxIdxMap[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
                    sigCtx = ctxIdxMap[(yC << 2) + xC];
                } else if (xC + yC == 0) {
                    sigCtx = 0;
                } else {
                    if (prevCsbf == 0) sigCtx = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
                    else if (prevCsbf == 1) sigCtx = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
                    else if (prevCsbf == 2) sigCtx = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
                    else sigCtx = 2;
                    if (c == 0) {
                        if (xs > 0 || ys > 0) sigCtx += 3;
                        if (log2n == 3) sigCtx += (scanIdx == 0) ? 9 : 15;
                        else sigCtx += 21;
                    } else {
                        if (log2n == 3) sigCtx += 9;
                        else sigCtx += 12;
                    }
                }
                int ctxInc = c == 0 ? sigCtx : 27 + sigCtx;
                sig[nn] = dec_bin(d, C_SIG + ctxInc);
                if (sig[nn]) infer_dc = 0;
            } else {
                if (nn == 0 && infer_dc && csbf[xs][ys]) sig[nn] = 1;
            }
        }
        /* levels */
        int g1[16] = {0}, g2[16] = {0}, sgn[16] = {0};
        int firstSig = 16, lastSig = -1, numG1 = 0, lastG1Pos = -1;
        int any = 0;
        for (int nn = 15; nn >= 0; nn--)
            if (sig[nn]) any = 1;
        if (!any) continue;
        int ctxSet = (i == 0 || c > 0) ? 0 : 2;
        if (greater1_ctx == 0) ctxSet++;
        greater1_ctx = 1;
        for (int nn = 15; nn >= 0; nn--) {
            if (!sig[nn]) continue;
            if (numG1 < 8) {
                int inc = ctxSet * 4 + greater1_ctx + (c ? 16 : 0);
                g1[nn] = dec_bin(d, C_GT1 + inc);
                numG1++;
                if (g1[nn]) {
                    greater1_ctx = 0;
                    if (lastG1Pos == -1) lastG1Pos = nn;
                } else if (greater1_ctx > 0 && greater1_ctx < 3) {
                    greater1_ctx++;
                }
            }
            if (lastSig == -1) lastSig = nn;
            firstSig = nn;
        }
        int signHidden = (d->cu_bypass || rdpcm_ts) ? 0 : (lastSig - firstSig > 3);
        if (lastG1Pos != -1) g2[lastG1Pos] = dec_bin(d, C_GT2 + ctxSet + (c ? 4 : 0));
        for (int nn = 15; nn >= 0; nn--)
            if (sig[nn] && (!sign_hiding_en || !signHidden || nn != firstSig)) sgn[nn] = dec_byp(d);
        /* Rice parameter: 0, or StatCoeff[sbType] / 4 with persistent_rice_adaptation, which also
         * leaves it uncapped (FFmpeg hevc_cabac.c) and updates StatCoeff from the sub-block's
         * first coeff_abs_level_remaining (9.3.3.11) */
        int numSig = 0, sumAbs = 0, rice = sps->persistent_rice ? d->stat[sb_type] / 4 : 0, stat_done = 0;
        for (int nn = 15; nn >= 0; nn--) {
            if (!sig[nn]) continue;
            int base = 1 + g1[nn] + g2[nn];
            int lvl = base;
            if (base == ((numSig < 8) ? ((nn == lastG1Pos) ? 3 : 2) : 1)) {
                int rem = decode_alr(d, rice);
                lvl = base + rem;
                if (lvl > 3 * (1 << rice)) rice = sps->persistent_rice ? rice + 1 : (rice + 1 < 4 ? rice + 1 : 4);
                if (sps->persistent_rice && !stat_done) {
                    int ri = d->stat[sb_type] / 4;
                    if (rem >= (3 << ri)) d->stat[sb_type]++;
                    else if (2 * rem < (1 << ri) && d->stat[sb_type] > 0) d->stat[sb_type]--;
                    stat_done = 1;
                }
            }
            int v = sgn[nn] ? -lvl : lvl;
            if (sign_hiding_en && signHidden) {
                sumAbs += lvl;
                if (nn == firstSig && (sumAbs & 1)) v = -v;
            }
            int xC = (xs << 2) + sc[2][nn][0], yC = (ys << 2) + sc[2][nn][1];
            coef[yC * n + xC] = (int16_t)clip3(-32768, 32767, v);
            numSig++;
        }
    }
    (void)x0;
    (void)y0;
}

/* RExt residual DPCM (8.6.8 / FFmpeg hevcdsp transform_rdpcm): accumulate down the columns
 * (vertical, mode 26) or along the rows (mode 10), in int16 as FFmpeg's coefficient buffer */
static void rdpcm(int *r, int n, int vertical) {
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            if (vertical ? y == 0 : x == 0) continue;
            int prev = vertical ? r[(y - 1) * n + x] : r[y * n + x - 1];
            r[y * n + x] = (int16_t)(r[y * n + x] + prev);
        }
}

/* scale + transform + add (8.6.2-8.6.4); mode: the TB's intra prediction mode (RExt RDPCM) */
static void reconstruct_residual(Dec *d, int c, int x0, int y0, int log2n, int qp, int tskip,
                                 int dst, int mode) {
    const int n = 1 << log2n;
    const int bd = c ? d->bdc : d->bd;
    const int maxv = (1 << bd) - 1;
    const int hv = mode == 10 || mode == 26;
    int r[32 * 32];
    if (d->cu_bypass) {
        for (int i = 0; i < n * n; i++) r[i] = d->coeff[i];
        /* FFmpeg: bypass blocks take implicit RDPCM but no transform-skip rotation */
        if (d->s->implicit_rdpcm && hv) rdpcm(r, n, mode == 26);
    } else {
        static const int ls[6] = {40, 45, 51, 57, 64, 72};
        int dd[32 * 32];
        int bdShift = bd + log2n - 5;
        int use_sl = d->sl_enabled && !(tskip && n > 4);
        int sizeId = log2n - 2, matrixId = c; /* intra */
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++) {
                int m = 16;
                if (use_sl) {
                    if (sizeId == 0) {
                        /* position (x,y) in 4x4 diag scan */
                        int k = 0;
                        while (scan_diag[2][k][0] != x || scan_diag[2][k][1] != y) k++;
                        m = d->slist[0][matrixId][k];
                    } else {
                        int ratio = n / 8, xx = x / ratio, yy = y / ratio, k = 0;
                        while (scan_diag[3][k][0] != xx || scan_diag[3][k][1] != yy) k++;
                        m = d->slist[sizeId][matrixId][k];
                        if (sizeId >= 2 && x == 0 && y == 0) m = d->slist_dc[sizeId][matrixId];
                    }
                }
                int64_t v = (int64_t)d->coeff[y * n + x] * m * ls[qp % 6];
                v = (v << (qp / 6)) + ((int64_t)1 << (bdShift - 1));
                v >>= bdShift;
                dd[y * n + x] = (int)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
            }
        if (tskip) {
            /* rotation (RExt, 4x4): r[x][y] = d[n-1-x][n-1-y] */
            if (d->s->ts_rotation && n == 4)
                for (int i = 0; i < 8; i++) {
                    int t = dd[i];
                    dd[i] = dd[15 - i];
                    dd[15 - i] = t;
                }
            /* tsShift = 5 + log2n, bdShift = 20 - bitDepth; FFmpeg dequant(): one shift by
             * 15 - bitDepth - log2n (left when negative) on the int16 coefficient */
            int sh = 15 - bd - log2n;
            for (int i = 0; i < n * n; i++) r[i] = sh > 0 ? (dd[i] + (1 << (sh - 1))) >> sh : (int16_t)(dd[i] * (1 << -sh));
            if (d->s->implicit_rdpcm && hv) rdpcm(r, n, mode == 26);
        } else {
            inv_transform(dd, r, n, dst, bd);
        }
    }
    uint16_t *pl = d->pl[c];
    int st = d->st[c];
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            uint16_t *p = &pl[(y0 + y) * st + x0 + x];
            *p = (uint16_t)clip3(0, maxv, *p + r[y * n + x]);
        }
}

/* ------------------------------------------------------------ CU parsing */
static void set_map8(Dec *d, uint8_t *m, int x0, int y0, int size, uint8_t v) {
    for (int y = y0 >> 2; y < ((y0 + size) >> 2) && y < d->mh; y++)
        for (int x = x0 >> 2; x < ((x0 + size) >> 2) && x < d->mw; x++) m[y * d->mw + x] = v;
}

static void set_qp_cu(Dec *d, int x0, int y0, int size, int qp) {
    for (int y = y0 >> 2; y < ((y0 + size) >> 2) && y < d->mh; y++)
        for (int x = x0 >> 2; x < ((x0 + size) >> 2) && x < d->mw; x++) d->qp[y * d->mw + x] = (int8_t)qp;
}

/* mark deblocking edges of a transform block (8.7.2.3) */
static void mark_tu_edges(Dec *d, int x0, int y0, int size) {
    if (d->cur->deblock_disabled) return;
    const int ctbmask = d->ctbs - 1;
    for (int k = 0; k < size && y0 + k < d->H; k += 4) {
        /* left edge */
        if ((x0 & 7) == 0 && x0 > 0) {
            int ok = 1;
            int xn = x0 - 1, yn = y0 + k;
            int cn = (yn >> d->log2ctb) * d->ctbW + (xn >> d->log2ctb);
            int cc = (yn >> d->log2ctb) * d->ctbW + (x0 >> d->log2ctb);
            if ((x0 & ctbmask) == 0) {
                if (!d->cur->lf_across_slices && d->ctb_addr_rs[cn] != d->ctb_addr_rs[cc]) ok = 0;
                if (!d->p->lf_across_tiles && d->tile_id[d->rs2ts[cn]] != d->tile_id[d->rs2ts[cc]]) ok = 0;
            }
            if (ok) d->bsv[(yn >> 2) * d->mw + (x0 >> 2)] = 2;
        }
    }
    for (int k = 0; k < size && x0 + k < d->W; k += 4) {
        if ((y0 & 7) == 0 && y0 > 0) {
            int ok = 1;
            int xn = x0 + k, yn = y0 - 1;
            int cn = (yn >> d->log2ctb) * d->ctbW + (xn >> d->log2ctb);
            int cc = (y0 >> d->log2ctb) * d->ctbW + (xn >> d->log2ctb);
            if ((y0 & ctbmask) == 0) {
                if (!d->cur->lf_across_slices && d->ctb_addr_rs[cn] != d->ctb_addr_rs[cc]) ok = 0;
                if (!d->p->lf_across_tiles && d->tile_id[d->rs2ts[cn]] != d->tile_id[d->rs2ts[cc]]) ok = 0;
            }
            if (ok) d->bsh[(y0 >> 2) * d->mw + (xn >> 2)] = 2;
        }
    }
}

typedef struct {
    int x0, y0, log2cb;
    int intra_chroma_mode; /* derived IntraPredModeC */
} CuCtx;

static int luma_mode_at(Dec *d, int x, int y) { return d->ipm[(y >> 2) * d->mw + (x >> 2)]; }

static void transform_unit_recon(Dec *d, CuCtx *cu, int x0, int y0, int xb, int yb, int log2n,
                                 int blk, int cbf_l, int cbf_cb, int cbf_cr) {
    int tskip = 0;
    if ((cbf_l || cbf_cb || cbf_cr) && d->p->cu_qp_delta && !d->is_qpd_coded) {
        int v = 0;
        if (dec_bin(d, C_QP_DELTA)) {
            v = 1;
            while (v < 5 && dec_bin(d, C_QP_DELTA + 1)) v++;
            if (v == 5) {
                int k = 0;
                while (dec_byp(d)) k++;
                v += ((1 << k) - 1) + dec_bypn(d, k);
            }
        }
        if (v && dec_byp(d)) v = -v;
        d->is_qpd_coded = 1;
        d->qpd_val = v;
        d->qp_y = ((d->qg_pred + v + 52 + 2 * d->qpbd) % (52 + d->qpbd)) - d->qpbd;
        set_qp_cu(d, cu->x0, cu->y0, 1 << cu->log2cb, d->qp_y);
    }
    /* FFmpeg 4.3 hls_transform_unit: cu_chroma_qp_offset_flag once per chroma QP offset group, at
     * the first TU with a chroma cbf of a CU without transquant bypass; the index is read only when
     * chroma_qp_offset_list_len_minus1 > 0, by ff_hevc_cu_chroma_qp_offset_idx as a truncated unary
     * code with cMax FFMAX(5, len_minus1) = 5 (H.265 9.3.3.x: cMax = len_minus1; the two agree unless
     * a stream codes idx == len_minus1 < 5); list entries past the list are 0 (zeroed PPS) */
    if ((cbf_cb || cbf_cr) && d->cur->cu_chroma_qp_offset_enabled && !d->cu_bypass && !d->cqo_coded) {
        if (dec_bin(d, C_CQO_FLAG)) {
            int idx = 0;
            if (d->p->cqo_len > 1)
                while (idx < 5 && dec_bin(d, C_CQO_IDX)) idx++;
            d->cu_qo_cb = d->p->cb_qo_list[idx];
            d->cu_qo_cr = d->p->cr_qo_list[idx];
        } else {
            d->cu_qo_cb = d->cu_qo_cr = 0;
        }
        d->cqo_coded = 1;
    }
    const int qpy = d->qp_y + d->qpbd;
    int qpc[2];
    for (int k = 0; k < 2; k++) {
        /* H.265 8.6.1: CuQpOffsetCb / Cr enter the dequantisation QP only (deblocking uses
         * pps_cb_qp_offset alone, 8.7.2.5.5; FFmpeg chroma_tc likewise) */
        int off = k == 0 ? d->p->cb_qp_offset + d->cur->cb_qp_offset + d->cu_qo_cb
                         : d->p->cr_qp_offset + d->cur->cr_qp_offset + d->cu_qo_cr;
        int qpi = clip3(-d->qpbdc, 57, d->qp_y + off);
        qpc[k] = chroma_qp_table(qpi) + d->qpbdc;
    }
    /* luma */
    int mode = luma_mode_at(d, x0, y0);
    intra_pred(d, 0, x0, y0, log2n, mode);
    if (cbf_l) {
        residual_coding(d, x0, y0, log2n, 0, mode, &tskip);
        reconstruct_residual(d, 0, x0, y0, log2n, qpy, tskip, log2n == 2 && !tskip, mode);
    }
    mark_tu_edges(d, x0, y0, 1 << log2n);
    int cm = cu->intra_chroma_mode;
    if (log2n > 2) {
        int xc = x0 >> 1, yc = y0 >> 1, l2 = log2n - 1;
        intra_pred(d, 1, xc, yc, l2, cm);
        if (cbf_cb) {
            residual_coding(d, xc, yc, l2, 1, cm, &tskip);
            reconstruct_residual(d, 1, xc, yc, l2, qpc[0], tskip, 0, cm);
        }
        intra_pred(d, 2, xc, yc, l2, cm);
        if (cbf_cr) {
            residual_coding(d, xc, yc, l2, 2, cm, &tskip);
            reconstruct_residual(d, 2, xc, yc, l2, qpc[1], tskip, 0, cm);
        }
    } else if (blk == 3) {
        int xc = xb >> 1, yc = yb >> 1;
        intra_pred(d, 1, xc, yc, 2, cm);
        if (cbf_cb) {
            residual_coding(d, xc, yc, 2, 1, cm, &tskip);
            reconstruct_residual(d, 1, xc, yc, 2, qpc[0], tskip, 0, cm);
        }
        intra_pred(d, 2, xc, yc, 2, cm);
        if (cbf_cr) {
            residual_coding(d, xc, yc, 2, 2, cm, &tskip);
            reconstruct_residual(d, 2, xc, yc, 2, qpc[1], tskip, 0, cm);
        }
    }
}

static void transform_tree(Dec *d, CuCtx *cu, int x0, int y0, int xb, int yb, int log2n, int depth,
                           int blk, int max_depth, int intra_split, int pcb, int pcr) {
    int split;
    if (log2n <= d->s->log2_max_tb && log2n > d->s->log2_min_tb && depth < max_depth &&
        !(intra_split && depth == 0)) {
        split = dec_bin(d, C_SPLIT_TF + 5 - log2n);
    } else {
        split = log2n > d->s->log2_max_tb || (intra_split && depth == 0);
    }
    int cbf_cb = 0, cbf_cr = 0;
    if (log2n > 2) {
        if (depth == 0 || pcb) cbf_cb = dec_bin(d, C_CBF_CHROMA + depth);
        if (depth == 0 || pcr) cbf_cr = dec_bin(d, C_CBF_CHROMA + depth);
    } else {
        cbf_cb = pcb;
        cbf_cr = pcr;
    }
    if (split) {
        int h = 1 << (log2n - 1);
        transform_tree(d, cu, x0, y0, x0, y0, log2n - 1, depth + 1, 0, max_depth, intra_split, cbf_cb, cbf_cr);
        transform_tree(d, cu, x0 + h, y0, x0, y0, log2n - 1, depth + 1, 1, max_depth, intra_split, cbf_cb, cbf_cr);
        transform_tree(d, cu, x0, y0 + h, x0, y0, log2n - 1, depth + 1, 2, max_depth, intra_split, cbf_cb, cbf_cr);
        transform_tree(d, cu, x0 + h, y0 + h, x0, y0, log2n - 1, depth + 1, 3, max_depth, intra_split, cbf_cb, cbf_cr);
    } else {
        int cbf_l = dec_bin(d, C_CBF_LUMA + (depth == 0 ? 1 : 0));
        transform_unit_recon(d, cu, x0, y0, xb, yb, log2n, blk, cbf_l, cbf_cb, cbf_cr);
    }
}

static void pcm_sample(Dec *d, int x0, int y0, int log2cb) {
    OraBits *b = &d->bits;
    /* position after terminate: align */
    b->pos = (b->pos + 7) & ~7L;
    int n = 1 << log2cb;
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
            d->pl[0][(y0 + y) * d->st[0] + x0 + x] = (uint16_t)(ob_u(b, d->s->pcm_bd) << (d->bd - d->s->pcm_bd));
    for (int c = 1; c < 3; c++)
        for (int y = 0; y < n / 2; y++)
            for (int x = 0; x < n / 2; x++)
                d->pl[c][(y0 / 2 + y) * d->st[c] + x0 / 2 + x] =
                    (uint16_t)(ob_u(b, d->s->pcm_bd_c) << (d->bdc - d->s->pcm_bd_c));
    oc_init(&d->cc, b);
}

static void coding_unit(Dec *d, int x0, int y0, int log2cb) {
    const int n = 1 << log2cb;
    CuCtx cu = {x0, y0, log2cb, 0};
    d->cu_bypass = 0;
    if (d->p->transquant_bypass) d->cu_bypass = dec_bin(d, C_TQ_BYPASS);
    int part_nxn = 0;
    if (log2cb == d->s->log2_min_cb) part_nxn = !dec_bin(d, C_PART_MODE);
    /* the CU's QP before any delta in it (QpY = qPY_PRED + CuQpDeltaVal) */
    d->qp_y = ((d->qg_pred + d->qpd_val + 52 + 2 * d->qpbd) % (52 + d->qpbd)) - d->qpbd;
    set_qp_cu(d, x0, y0, n, d->qp_y);
    int pcm = 0;
    if (!part_nxn && d->s->pcm && log2cb >= d->s->log2_min_pcm && log2cb <= d->s->log2_max_pcm)
        pcm = oc_terminate(&d->cc);
    uint8_t nf = (uint8_t)(d->cu_bypass || (pcm && d->s->pcm_lf_disabled));
    set_map8(d, d->nofilt, x0, y0, n, nf);
    if (pcm) {
        set_map8(d, d->ipm, x0, y0, n, 1); /* PCM: neighbours see DC */
        pcm_sample(d, x0, y0, log2cb);
        mark_tu_edges(d, x0, y0, n);
    } else {
        int np = part_nxn ? 4 : 1, pb = part_nxn ? n / 2 : n;
        int prev[4], mpm[4], rem[4];
        for (int i = 0; i < np; i++) prev[i] = dec_bin(d, C_PREV_INTRA);
        for (int i = 0; i < np; i++) {
            if (prev[i]) {
                mpm[i] = 0;
                if (dec_byp(d)) mpm[i] = dec_byp(d) ? 2 : 1;
            } else {
                rem[i] = dec_bypn(d, 5);
            }
        }
        for (int i = 0; i < np; i++) {
            int xp = x0 + (i & 1) * pb, yp = y0 + (i >> 1) * pb;
            int ca = 1, cb = 1;
            if (avail(d, xp, yp, xp - 1, yp)) ca = luma_mode_at(d, xp - 1, yp);
            if (avail(d, xp, yp, xp, yp - 1) && ((yp - 1) >> d->log2ctb) == (yp >> d->log2ctb))
                cb = luma_mode_at(d, xp, yp - 1);
            int cand[3];
            if (ca == cb) {
                if (ca < 2) { cand[0] = 0; cand[1] = 1; cand[2] = 26; }
                else { cand[0] = ca; cand[1] = 2 + ((ca + 29) % 32); cand[2] = 2 + ((ca - 2 + 1) % 32); }
            } else {
                cand[0] = ca;
                cand[1] = cb;
                cand[2] = (ca != 0 && cb != 0) ? 0 : ((ca != 1 && cb != 1) ? 1 : 26);
            }
            int mode;
            if (prev[i]) {
                mode = cand[mpm[i]];
            } else {
                int t;
                if (cand[0] > cand[1]) { t = cand[0]; cand[0] = cand[1]; cand[1] = t; }
                if (cand[0] > cand[2]) { t = cand[0]; cand[0] = cand[2]; cand[2] = t; }
                if (cand[1] > cand[2]) { t = cand[1]; cand[1] = cand[2]; cand[2] = t; }
                mode = rem[i];
                for (int k = 0; k < 3; k++)
                    if (mode >= cand[k]) mode++;
            }
            set_map8(d, d->ipm, xp, yp, pb, (uint8_t)mode);
        }
        int icpm = 4;
        if (dec_bin(d, C_CHROMA_MODE)) icpm = dec_bypn(d, 2);
        int lm = luma_mode_at(d, x0, y0);
        if (icpm == 4) cu.intra_chroma_mode = lm;
        else {
            static const int cmodes[4] = {0, 26, 10, 1};
            cu.intra_chroma_mode = cmodes[icpm] == lm ? 34 : cmodes[icpm];
        }
        int max_depth = d->s->max_th_depth_intra + part_nxn;
        transform_tree(d, &cu, x0, y0, x0, y0, log2cb, 0, 0, max_depth, part_nxn, 0, 0);
    }
    d->last_cu_qp = d->qp_y;
}

static void coding_quadtree(Dec *d, int x0, int y0, int log2cb, int depth) {
    const int n = 1 << log2cb;
    int split;
    if (x0 + n <= d->W && y0 + n <= d->H && log2cb > d->s->log2_min_cb) {
        int inc = 0;
        if (avail(d, x0, y0, x0 - 1, y0) && d->ctd[(y0 >> 2) * d->mw + ((x0 - 1) >> 2)] > depth) inc++;
        if (avail(d, x0, y0, x0, y0 - 1) && d->ctd[((y0 - 1) >> 2) * d->mw + (x0 >> 2)] > depth) inc++;
        split = dec_bin(d, C_SPLIT_CU + inc);
    } else {
        split = log2cb > d->s->log2_min_cb;
    }
    if (d->p->cu_qp_delta && log2cb >= d->log2ctb - d->p->diff_cu_qp_delta_depth) {
        d->qp_pred_prev = d->last_cu_qp;
        qg_start(d, x0, y0);
    } else if (!d->p->cu_qp_delta && log2cb == d->log2ctb) {
        d->qp_pred_prev = d->last_cu_qp;
        qg_start(d, x0, y0);
    }
    if (d->cur->cu_chroma_qp_offset_enabled && log2cb >= d->log2ctb - d->p->cqo_depth) d->cqo_coded = 0;
    if (split) {
        int h = n >> 1;
        coding_quadtree(d, x0, y0, log2cb - 1, depth + 1);
        if (x0 + h < d->W) coding_quadtree(d, x0 + h, y0, log2cb - 1, depth + 1);
        if (y0 + h < d->H) coding_quadtree(d, x0, y0 + h, log2cb - 1, depth + 1);
        if (x0 + h < d->W && y0 + h < d->H) coding_quadtree(d, x0 + h, y0 + h, log2cb - 1, depth + 1);
    } else {
        set_map8(d, d->ctd, x0, y0, n, (uint8_t)depth);
        coding_unit(d, x0, y0, log2cb);
    }
}

static void parse_sao(Dec *d, int rx, int ry) {
    int ctb = ry * d->ctbW + rx;
    SaoP *sp = &d->sao[ctb];
    memset(sp, 0, sizeof(*sp));
    if (!d->cur->sao_luma && !d->cur->sao_chroma) return;
    int x0 = rx << d->log2ctb, y0 = ry << d->log2ctb;
    if (rx > 0) {
        int l = ctb - 1;
        if (d->ctb_addr_rs[l] == d->ctb_addr_rs[ctb] && d->tile_id[d->rs2ts[l]] == d->tile_id[d->rs2ts[ctb]] &&
            d->ctb_slice[l] >= 0) {
            if (dec_bin(d, C_SAO_MERGE)) {
                *sp = d->sao[l];
                return;
            }
        }
    }
    if (ry > 0) {
        int u = ctb - d->ctbW;
        if (d->ctb_addr_rs[u] == d->ctb_addr_rs[ctb] && d->tile_id[d->rs2ts[u]] == d->tile_id[d->rs2ts[ctb]] &&
            d->ctb_slice[u] >= 0) {
            if (dec_bin(d, C_SAO_MERGE)) {
                *sp = d->sao[u];
                return;
            }
        }
    }
    (void)x0;
    (void)y0;
    for (int c = 0; c < 3; c++) {
        if ((c == 0 && !d->cur->sao_luma) || (c > 0 && !d->cur->sao_chroma)) continue;
        if (c == 2) {
            sp->type[2] = sp->type[1];
            sp->eo_class[2] = sp->eo_class[1];
        } else {
            int t = 0;
            if (dec_bin(d, C_SAO_TYPE)) t = dec_byp(d) ? 2 : 1;
            sp->type[c] = (int8_t)t;
        }
        if (sp->type[c] == 0) continue;
        int bd = c ? d->bdc : d->bd;
        int cmax = (1 << ((bd < 10 ? bd : 10) - 5)) - 1;
        int abs_[4];
        for (int i = 0; i < 4; i++) {
            int v = 0;
            while (v < cmax && dec_byp(d)) v++;
            abs_[i] = v;
        }
        /* SaoOffsetVal = offset << log2OffsetScale (FFmpeg hls_sao_param: the PPS range extension's
         * log2_sao_offset_scale, 0 without it -- not v1's bitDepth - Min(bitDepth, 10)) */
        int shift = c ? d->p->sao_scale_chroma : d->p->sao_scale_luma;
        if (sp->type[c] == 1) {
            for (int i = 0; i < 4; i++) {
                if (abs_[i] && dec_byp(d)) abs_[i] = -abs_[i];
            }
            sp->band_pos[c] = (int8_t)dec_bypn(d, 5);
            for (int i = 0; i < 4; i++) sp->off[c][i] = (int16_t)(abs_[i] * (1 << shift));
        } else {
            sp->off[c][0] = (int16_t)(abs_[0] << shift);
            sp->off[c][1] = (int16_t)(abs_[1] << shift);
            sp->off[c][2] = (int16_t)(-(abs_[2] << shift));
            sp->off[c][3] = (int16_t)(-(abs_[3] << shift));
            if (c == 0) sp->eo_class[0] = (int8_t)dec_bypn(d, 2);
            if (c == 1) sp->eo_class[1] = (int8_t)dec_bypn(d, 2);
        }
    }
}

/* ------------------------------------------------------------ tiles */
static void setup_tiles(Dec *d) {
    const Pps *p = d->p;
    int cbd[65], rbd[65];
    int colw[64], rowh[64];
    for (int i = 0; i < p->ntc; i++) {
        if (p->uniform) colw[i] = ((i + 1) * d->ctbW) / p->ntc - (i * d->ctbW) / p->ntc;
        else if (i < p->ntc - 1) colw[i] = p->col_w[i];
    }
    if (!p->uniform) {
        int s = 0;
        for (int i = 0; i < p->ntc - 1; i++) s += colw[i];
        colw[p->ntc - 1] = d->ctbW - s;
    }
    for (int j = 0; j < p->ntr; j++) {
        if (p->uniform) rowh[j] = ((j + 1) * d->ctbH) / p->ntr - (j * d->ctbH) / p->ntr;
        else if (j < p->ntr - 1) rowh[j] = p->row_h[j];
    }
    if (!p->uniform) {
        int s = 0;
        for (int j = 0; j < p->ntr - 1; j++) s += rowh[j];
        rowh[p->ntr - 1] = d->ctbH - s;
    }
    cbd[0] = 0;
    for (int i = 0; i < p->ntc; i++) cbd[i + 1] = cbd[i] + colw[i];
    rbd[0] = 0;
    for (int j = 0; j < p->ntr; j++) rbd[j + 1] = rbd[j] + rowh[j];
    for (int rs = 0; rs < d->nctb; rs++) {
        int tbx = rs % d->ctbW, tby = rs / d->ctbW, tx = 0, ty = 0;
        for (int i = 0; i < p->ntc; i++)
            if (tbx >= cbd[i]) tx = i;
        for (int j = 0; j < p->ntr; j++)
            if (tby >= rbd[j]) ty = j;
        int v = 0;
        for (int i = 0; i < tx; i++) v += rowh[ty] * colw[i];
        for (int j = 0; j < ty; j++) v += d->ctbW * rowh[j];
        v += (tby - rbd[ty]) * colw[tx] + tbx - cbd[tx];
        d->rs2ts[rs] = v;
        d->ts2rs[v] = rs;
    }
    int tid = 0;
    for (int j = 0; j < p->ntr; j++)
        for (int i = 0; i < p->ntc; i++, tid++)
            for (int y = rbd[j]; y < rbd[j + 1]; y++)
                for (int x = cbd[i]; x < cbd[i + 1]; x++) d->tile_id[d->rs2ts[y * d->ctbW + x]] = tid;
    for (int i = 0; i <= p->ntc; i++) d->col_bd[i] = cbd[i];
    for (int j = 0; j <= p->ntr; j++) d->row_bd[j] = rbd[j];
}

/* ------------------------------------------------------------ picture */
static int alloc_picture(Dec *d) {
    const Sps *s = d->s;
    d->W = s->width;
    d->H = s->height;
    d->log2ctb = s->log2_ctb;
    d->ctbs = 1 << s->log2_ctb;
    d->ctbW = (d->W + d->ctbs - 1) >> d->log2ctb;
    d->ctbH = (d->H + d->ctbs - 1) >> d->log2ctb;
    d->nctb = d->ctbW * d->ctbH;
    d->mw = (d->W + 3) >> 2;
    d->mh = (d->H + 3) >> 2;
    d->bd = s->bit_depth;
    d->bdc = s->bit_depth_c;
    d->qpbd = 6 * (d->bd - 8);
    d->qpbdc = 6 * (d->bdc - 8);
    for (int c = 0; c < 3; c++) {
        d->pw[c] = c ? d->W / 2 : d->W;
        d->ph[c] = c ? d->H / 2 : d->H;
        d->st[c] = d->pw[c];
        d->pl[c] = (uint16_t *)calloc((size_t)d->pw[c] * d->ph[c], 2);
    }
    size_t m = (size_t)d->mw * d->mh;
    d->qp = (int8_t *)calloc(m, 1);
    d->ipm = (uint8_t *)calloc(m, 1);
    d->ctd = (uint8_t *)calloc(m, 1);
    d->nofilt = (uint8_t *)calloc(m, 1);
    d->bsv = (uint8_t *)calloc(m, 1);
    d->bsh = (uint8_t *)calloc(m, 1);
    d->ctb_slice = (int *)malloc(sizeof(int) * d->nctb);
    d->ctb_addr_rs = (int *)malloc(sizeof(int) * d->nctb);
    for (int i = 0; i < d->nctb; i++) d->ctb_slice[i] = d->ctb_addr_rs[i] = -1;
    d->rs2ts = (int *)malloc(sizeof(int) * d->nctb);
    d->ts2rs = (int *)malloc(sizeof(int) * d->nctb);
    d->tile_id = (int *)malloc(sizeof(int) * d->nctb);
    d->col_bd = (int *)malloc(sizeof(int) * 66);
    d->row_bd = (int *)malloc(sizeof(int) * 66);
    d->sao = (SaoP *)calloc((size_t)d->nctb, sizeof(SaoP));
    return 0;
}

static void free_picture(Dec *d) {
    free(d->qp); free(d->ipm); free(d->ctd); free(d->nofilt); free(d->bsv); free(d->bsh);
    free(d->ctb_slice); free(d->ctb_addr_rs); free(d->rs2ts); free(d->ts2rs); free(d->tile_id);
    free(d->col_bd); free(d->row_bd); free(d->sao);
}

/* ------------------------------------------------------------ slice data */
static void ctb_start_contexts(Dec *d, SliceHdr *sh, int ctbAddrRs, int ctbAddrTs, int first_in_seg) {
    int rx = ctbAddrRs % d->ctbW;
    int x0 = rx << d->log2ctb, y0 = (ctbAddrRs / d->ctbW) << d->log2ctb;
    int tile_start = ctbAddrTs == 0 || d->tile_id[ctbAddrTs] != d->tile_id[ctbAddrTs - 1];
    int row_start = 0;
    if (d->p->wpp) {
        for (int i = 0; i < d->p->ntc; i++)
            if (rx == d->col_bd[i]) row_start = 1;
    }
    if (!(first_in_seg || tile_start || row_start)) return;
    if (tile_start) {
        init_contexts(d, sh->slice_qp);
    } else if (row_start) {
        int xr = x0 + d->ctbs, yr = y0 - d->ctbs;
        /* the CTB must belong to the current slice for 6.4.1: mark it first */
        if (xr < d->W && yr >= 0 && avail(d, x0, y0, xr, yr)) {
            memcpy(d->ctx, d->ctx_wpp, NUM_CTX);
            memcpy(d->stat, d->stat_wpp, sizeof(d->stat));
        } else {
            init_contexts(d, sh->slice_qp);
        }
    } else if (sh->dependent && d->have_ds) {
        memcpy(d->ctx, d->ctx_ds, NUM_CTX);
        memcpy(d->stat, d->stat_ds, sizeof(d->stat));
    } else {
        init_contexts(d, sh->slice_qp);
    }
    /* qPY_PREV = SliceQpY for the first QG of a tile / of a CTB row under WPP (8.6.1): also for
     * the QG-size call that follows the CTB-level one (FFmpeg hevcdec first_qp_group) */
    if (tile_start || row_start) { d->first_qg = 1; d->last_cu_qp = d->cur->slice_qp; }
}

static int decode_slice_data(Dec *d, int shi) {
    SliceHdr *sh = &d->sh[shi];
    d->cur = sh;
    oc_init(&d->cc, &d->bits);
    int ctbAddrRs = sh->address;
    int ctbAddrTs = d->rs2ts[ctbAddrRs];
    if (!sh->dependent) {
        d->first_qg = 1;
        d->last_cu_qp = sh->slice_qp;
    }
    d->sl_enabled = d->s->scaling_list_enabled;
    if (d->p->sl_present) {
        d->slist = (const uint8_t(*)[6][64])d->p->sl;
        d->slist_dc = (const uint8_t(*)[6])d->p->sl_dc;
    } else {
        d->slist = (const uint8_t(*)[6][64])d->s->sl;
        d->slist_dc = (const uint8_t(*)[6])d->s->sl_dc;
    }
    int first = 1;
    for (;;) {
        int rx = ctbAddrRs % d->ctbW, ry = ctbAddrRs / d->ctbW;
        int x0 = rx << d->log2ctb, y0 = ry << d->log2ctb;
        d->ctb_slice[ctbAddrRs] = shi;
        d->ctb_addr_rs[ctbAddrRs] = sh->slice_addr_rs;
        ctb_start_contexts(d, sh, ctbAddrRs, ctbAddrTs, first);
        first = 0;
        parse_sao(d, rx, ry);
        coding_quadtree(d, x0, y0, d->log2ctb, 0);
        int end = oc_terminate(&d->cc);
        if (d->p->wpp) {
            int second = 0;
            for (int i = 0; i < d->p->ntc; i++)
                if (rx == d->col_bd[i] + 1 && d->col_bd[i] + 1 < d->col_bd[i + 1]) second = 1;
            if (second) {
                memcpy(d->ctx_wpp, d->ctx, NUM_CTX);
                memcpy(d->stat_wpp, d->stat, sizeof(d->stat));
            }
        }
        ctbAddrTs++;
        if (end) break;
        if (ctbAddrTs >= d->nctb) return -1;
        int nextRs = d->ts2rs[ctbAddrTs];
        int new_tile = d->tile_id[ctbAddrTs] != d->tile_id[ctbAddrTs - 1];
        int new_row = 0;
        if (d->p->wpp) {
            int nrx = nextRs % d->ctbW;
            for (int i = 0; i < d->p->ntc; i++)
                if (nrx == d->col_bd[i]) new_row = 1;
        }
        if (new_tile || new_row) {
            oc_terminate(&d->cc); /* end_of_subset_one_bit */
            d->bits.pos = (d->bits.pos + 7) & ~7L;
            oc_init(&d->cc, &d->bits);
        }
        ctbAddrRs = nextRs;
    }
    memcpy(d->ctx_ds, d->ctx, NUM_CTX);
    memcpy(d->stat_ds, d->stat, sizeof(d->stat));
    d->have_ds = 1;
    return 0;
}

static int parse_slice_header(Dec *d, OraBits *b, int nal_type, SliceHdr *sh, const SliceHdr *prev) {
    memset(sh, 0, sizeof(*sh));
    sh->first_in_pic = (int)ob_u(b, 1);
    if (nal_type >= 16 && nal_type <= 23) ob_u(b, 1);
    sh->pps_id = (int)ob_ue(b);
    if (sh->pps_id > 63 || !d->pps[sh->pps_id].valid) return -1;
    const Pps *p = &d->pps[sh->pps_id];
    const Sps *s = &d->sps[p->sps_id];
    if (!s->valid) return -1;
    if (!sh->first_in_pic) {
        if (p->dependent_slices) sh->dependent = (int)ob_u(b, 1);
        int ctbs = 1 << s->log2_ctb;
        int n = ((s->width + ctbs - 1) / ctbs) * ((s->height + ctbs - 1) / ctbs);
        sh->address = (int)ob_u(b, ora_ceil_log2(n));
    }
    if (sh->dependent) {
        if (!prev) return -1;
        int addr = sh->address, dep = sh->dependent, first = sh->first_in_pic;
        *sh = *prev;
        sh->address = addr;
        sh->dependent = dep;
        sh->first_in_pic = first;
    } else {
        sh->slice_addr_rs = sh->address;
        for (int i = 0; i < p->num_extra_bits; i++) ob_u(b, 1);
        sh->type = (int)ob_ue(b);
        if (p->output_flag_present) ob_u(b, 1);
        if (nal_type != 19 && nal_type != 20) {
            ob_u(b, s->log2_max_poc_lsb);
            int sps_flag = (int)ob_u(b, 1);
            if (!sps_flag) {
                Sps tmp = *s;
                if (parse_st_rps(b, &tmp, s->num_st_rps) < 0) return -1;
            } else if (s->num_st_rps > 1) {
                ob_u(b, ora_ceil_log2(s->num_st_rps));
            }
            if (s->long_term_present) {
                int nsps = 0;
                if (s->num_lt_sps > 0) nsps = (int)ob_ue(b);
                int npics = (int)ob_ue(b);
                for (int i = 0; i < nsps + npics; i++) {
                    if (i < nsps) {
                        if (s->num_lt_sps > 1) ob_u(b, ora_ceil_log2(s->num_lt_sps));
                    } else {
                        ob_u(b, s->log2_max_poc_lsb);
                        ob_u(b, 1);
                    }
                    if (ob_u(b, 1)) ob_ue(b);
                }
            }
            if (s->temporal_mvp) ob_u(b, 1);
        }
        if (s->sao) {
            sh->sao_luma = (int)ob_u(b, 1);
            sh->sao_chroma = (int)ob_u(b, 1);
        }
        if (sh->type != 2) return -2; /* P/B slices: unsupported (stills) */
        sh->qp_delta = ob_se(b);
        if (p->slice_chroma_qp_present) {
            sh->cb_qp_offset = ob_se(b);
            sh->cr_qp_offset = ob_se(b);
        }
        if (p->cqo_list_enabled) sh->cu_chroma_qp_offset_enabled = (int)ob_u(b, 1);
        int override = 0;
        if (p->deblock_override) override = (int)ob_u(b, 1);
        sh->deblock_disabled = p->deblock_disabled;
        sh->beta_offset = p->beta_offset;
        sh->tc_offset = p->tc_offset;
        if (override) {
            sh->deblock_disabled = (int)ob_u(b, 1);
            if (!sh->deblock_disabled) {
                sh->beta_offset = ob_se(b) * 2;
                sh->tc_offset = ob_se(b) * 2;
            }
        }
        sh->lf_across_slices = p->lf_across_slices;
        if (p->lf_across_slices && (sh->sao_luma || sh->sao_chroma || !sh->deblock_disabled))
            sh->lf_across_slices = (int)ob_u(b, 1);
        sh->slice_qp = p->init_qp + sh->qp_delta;
    }
    if (p->tiles || p->wpp) {
        sh->num_entry = (int)ob_ue(b);
        if (sh->num_entry > 0) {
            int len = (int)ob_ue(b) + 1;
            for (int i = 0; i < sh->num_entry; i++) ob_u(b, len);
        }
    }
    if (p->slice_header_ext) {
        int len = (int)ob_ue(b);
        for (int i = 0; i < len; i++) ob_u(b, 8);
    }
    /* byte_alignment() */
    ob_u(b, 1);
    while (b->pos & 7) ob_u(b, 1);
    return 0;
}

/* ------------------------------------------------------------ deblocking */
static const int k_beta[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                               8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                               34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
static const int k_tc[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,  1,  1,  1,  1,  1, 1,
                             2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

static const SliceHdr *slice_at(const Dec *d, int x, int y) {
    int ctb = (y >> d->log2ctb) * d->ctbW + (x >> d->log2ctb);
    return &d->sh[d->ctb_slice[ctb] < 0 ? 0 : d->ctb_slice[ctb]];
}

/* filter one luma edge segment of 4 lines. P(i,k) / Q(i,k): i = distance
 * from the edge (0..3), k = line (0..3) */
static void filter_luma_seg(Dec *d, int vert, int xe, int ye) {
    uint16_t *pl = d->pl[0];
    const int st = d->st[0];
    int xp = vert ? xe - 1 : xe, yp = vert ? ye : ye - 1;
    int qpq = qp_at(d, xe, ye), qpp = qp_at(d, xp, yp);
    int qpl = (qpq + qpp + 1) >> 1;
    const SliceHdr *sh = slice_at(d, xe, ye);
    int bs = 2;
    int Q = clip3(0, 51, qpl + sh->beta_offset);
    int beta = k_beta[Q] * (1 << (d->bd - 8));
    Q = clip3(0, 53, qpl + 2 * (bs - 1) + sh->tc_offset);
    int tc = k_tc[Q] * (1 << (d->bd - 8));
    const int maxv = (1 << d->bd) - 1;
#define PIX(i, k) (vert ? &pl[(ye + (k)) * st + xe - 1 - (i)] : &pl[(ye - 1 - (i)) * st + xe + (k)])
#define QIX(i, k) (vert ? &pl[(ye + (k)) * st + xe + (i)] : &pl[(ye + (i)) * st + xe + (k)])
#define P(i, k) (*PIX(i, k))
#define Qs(i, k) (*QIX(i, k))
    int dp0 = abs(P(2, 0) - 2 * P(1, 0) + P(0, 0)), dp3 = abs(P(2, 3) - 2 * P(1, 3) + P(0, 3));
    int dq0 = abs(Qs(2, 0) - 2 * Qs(1, 0) + Qs(0, 0)), dq3 = abs(Qs(2, 3) - 2 * Qs(1, 3) + Qs(0, 3));
    int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3, dd = dpq0 + dpq3;
    if (dd >= beta) return;
    int dsam0 = (2 * dpq0 < (beta >> 2)) && (abs(P(3, 0) - P(0, 0)) + abs(Qs(0, 0) - Qs(3, 0)) < (beta >> 3)) &&
                (abs(P(0, 0) - Qs(0, 0)) < ((5 * tc + 1) >> 1));
    int dsam3 = (2 * dpq3 < (beta >> 2)) && (abs(P(3, 3) - P(0, 3)) + abs(Qs(0, 3) - Qs(3, 3)) < (beta >> 3)) &&
                (abs(P(0, 3) - Qs(0, 3)) < ((5 * tc + 1) >> 1));
    int dE = (dsam0 && dsam3) ? 2 : 1;
    int dEp = dp < ((beta + (beta >> 1)) >> 3);
    int dEq = dq < ((beta + (beta >> 1)) >> 3);
    int nfp = d->nofilt[(yp >> 2) * d->mw + (xp >> 2)];
    int nfq = d->nofilt[(ye >> 2) * d->mw + (xe >> 2)];
    for (int k = 0; k < 4; k++) {
        int p0 = P(0, k), p1 = P(1, k), p2 = P(2, k), p3 = P(3, k);
        int q0 = Qs(0, k), q1 = Qs(1, k), q2 = Qs(2, k), q3 = Qs(3, k);
        if (dE == 2) {
            if (!nfp) {
                *PIX(0, k) = (uint16_t)clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
                *PIX(1, k) = (uint16_t)clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2);
                *PIX(2, k) = (uint16_t)clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
            }
            if (!nfq) {
                *QIX(0, k) = (uint16_t)clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
                *QIX(1, k) = (uint16_t)clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2);
                *QIX(2, k) = (uint16_t)clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3);
            }
        } else {
            int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (abs(delta) < tc * 10) {
                delta = clip3(-tc, tc, delta);
                if (!nfp) *PIX(0, k) = (uint16_t)clip3(0, maxv, p0 + delta);
                if (!nfq) *QIX(0, k) = (uint16_t)clip3(0, maxv, q0 - delta);
                if (dEp && !nfp) {
                    int dpv = clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1);
                    *PIX(1, k) = (uint16_t)clip3(0, maxv, p1 + dpv);
                }
                if (dEq && !nfq) {
                    int dqv = clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1);
                    *QIX(1, k) = (uint16_t)clip3(0, maxv, q1 + dqv);
                }
            }
        }
    }
#undef PIX
#undef QIX
#undef P
#undef Qs
}

/* chroma edge segment: 4 chroma lines at chroma position (xc,yc) */
static void filter_chroma_seg(Dec *d, int c, int vert, int xc, int yc) {
    uint16_t *pl = d->pl[c];
    const int st = d->st[c];
    int xl = xc * 2, yl = yc * 2;
    int xp = vert ? xl - 1 : xl, yp = vert ? yl : yl - 1;
    int qpq = qp_at(d, xl, yl), qpp = qp_at(d, xp, yp);
    int off = c == 1 ? d->p->cb_qp_offset : d->p->cr_qp_offset;
    int qpi = ((qpq + qpp + 1) >> 1) + off;
    int qpc = chroma_qp_table(qpi);
    const SliceHdr *sh = slice_at(d, xl, yl);
    int Q = clip3(0, 53, qpc + 2 + sh->tc_offset);
    int tc = k_tc[Q] * (1 << (d->bdc - 8));
    const int maxv = (1 << d->bdc) - 1;
    int nfp = d->nofilt[(yp >> 2) * d->mw + (xp >> 2)];
    int nfq = d->nofilt[(yl >> 2) * d->mw + (xl >> 2)];
    for (int k = 0; k < 4; k++) {
        uint16_t *pp0, *pp1, *pq0, *pq1;
        if (vert) {
            if (yc + k >= d->ph[c]) break;
            pp0 = &pl[(yc + k) * st + xc - 1]; pp1 = pp0 - 1;
            pq0 = &pl[(yc + k) * st + xc]; pq1 = pq0 + 1;
        } else {
            if (xc + k >= d->pw[c]) break;
            pp0 = &pl[(yc - 1) * st + xc + k]; pp1 = pp0 - st;
            pq0 = &pl[yc * st + xc + k]; pq1 = pq0 + st;
        }
        int p0 = *pp0, p1 = *pp1, q0 = *pq0, q1 = *pq1;
        int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
        if (!nfp) *pp0 = (uint16_t)clip3(0, maxv, p0 + delta);
        if (!nfq) *pq0 = (uint16_t)clip3(0, maxv, q0 - delta);
    }
}

static void deblock(Dec *d) {
    for (int pass = 0; pass < 2; pass++) {
        int vert = pass == 0;
        uint8_t *bs = vert ? d->bsv : d->bsh;
        /* luma */
        for (int y4 = 0; y4 < d->mh; y4++)
            for (int x4 = 0; x4 < d->mw; x4++) {
                if (!bs[y4 * d->mw + x4]) continue;
                int xe = x4 * 4, ye = y4 * 4;
                if (ye + 3 >= d->H || xe + 3 >= d->W) {
                    /* partial segments only at picture edges not multiple of 4: W,H multiples of 8 */
                }
                filter_luma_seg(d, vert, xe, ye);
            }
        /* chroma: edges on the 8x8 chroma grid (16 luma) */
        for (int c = 1; c < 3; c++) {
            for (int y4 = 0; y4 < d->mh; y4 += 2)
                for (int x4 = 0; x4 < d->mw; x4 += 2) {
                    int xe = x4 * 4, ye = y4 * 4;
                    if (vert) {
                        if (xe % 16) continue;
                        if (!bs[y4 * d->mw + x4]) continue;
                    } else {
                        if (ye % 16) continue;
                        if (!bs[y4 * d->mw + x4]) continue;
                    }
                    filter_chroma_seg(d, c, vert, xe / 2, ye / 2);
                }
        }
    }
}

/* ------------------------------------------------------------ SAO */
static void apply_sao(Dec *d) {
    uint16_t *src[3];
    for (int c = 0; c < 3; c++) {
        size_t n = (size_t)d->pw[c] * d->ph[c];
        src[c] = (uint16_t *)malloc(n * 2);
        memcpy(src[c], d->pl[c], n * 2);
    }
    static const int hpos[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}};
    static const int vpos[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
    for (int ctb = 0; ctb < d->nctb; ctb++) {
        if (d->ctb_slice[ctb] < 0) continue;
        const SaoP *sp = &d->sao[ctb];
        const SliceHdr *sh = &d->sh[d->ctb_slice[ctb]];
        int rx = ctb % d->ctbW, ry = ctb / d->ctbW;
        for (int c = 0; c < 3; c++) {
            if (!sp->type[c]) continue;
            if ((c == 0 && !sh->sao_luma) || (c > 0 && !sh->sao_chroma)) continue;
            int sh_ = c ? 1 : 0;
            int bd = c ? d->bdc : d->bd, maxv = (1 << bd) - 1;
            int cs = d->ctbs >> sh_;
            int x0 = rx * cs, y0 = ry * cs;
            for (int y = y0; y < y0 + cs && y < d->ph[c]; y++)
                for (int x = x0; x < x0 + cs && x < d->pw[c]; x++) {
                    int xl = x << sh_, yl = y << sh_;
                    if (d->nofilt[(yl >> 2) * d->mw + (xl >> 2)]) continue;
                    int v = src[c][y * d->st[c] + x];
                    int off = 0;
                    if (sp->type[c] == 1) {
                        int bshift = bd - 5;
                        int band = v >> bshift;
                        int k = (band - sp->band_pos[c]) & 31;
                        if (k < 4) off = sp->off[c][k];
                    } else {
                        int cls = sp->eo_class[c];
                        int ok = 1, nb[2];
                        for (int k = 0; k < 2; k++) {
                            int xn = x + hpos[cls][k], yn = y + vpos[cls][k];
                            if (xn < 0 || yn < 0 || xn >= d->pw[c] || yn >= d->ph[c]) { ok = 0; break; }
                            int xnl = xn << sh_, ynl = yn << sh_;
                            int cn = (ynl >> d->log2ctb) * d->ctbW + (xnl >> d->log2ctb);
                            if (cn != ctb) {
                                const SliceHdr *shn = &d->sh[d->ctb_slice[cn] < 0 ? 0 : d->ctb_slice[cn]];
                                if (d->ctb_addr_rs[cn] != d->ctb_addr_rs[ctb]) {
                                    int zn = min_tb_zs(d, xnl, ynl), zc = min_tb_zs(d, xl, yl);
                                    if (zn < zc && !sh->lf_across_slices) ok = 0;
                                    if (zc < zn && !shn->lf_across_slices) ok = 0;
                                }
                                if (!d->p->lf_across_tiles && d->tile_id[d->rs2ts[cn]] != d->tile_id[d->rs2ts[ctb]]) ok = 0;
                            }
                            if (!ok) break;
                            nb[k] = src[c][yn * d->st[c] + xn];
                        }
                        if (ok) {
                            int s0 = (v > nb[0]) - (v < nb[0]), s1 = (v > nb[1]) - (v < nb[1]);
                            int e = 2 + s0 + s1;
                            static const int remap[5] = {1, 2, 0, 3, 4};
                            e = remap[e];
                            if (e) off = sp->off[c][e - 1];
                        }
                    }
                    d->pl[c][y * d->st[c] + x] = (uint16_t)clip3(0, maxv, v + off);
                }
        }
    }
    for (int c = 0; c < 3; c++) free(src[c]);
}

/* ------------------------------------------------------------ top level */
static void init_tables(void) {
    init_scans();
    init_tm();
}
static pthread_once_t tables_once = PTHREAD_ONCE_INIT; /* the CPU baseline calls from several threads */

int oracle_hevc_decode(const uint8_t *data, long size, int flags, OraclePicture *out) {
    pthread_once(&tables_once, init_tables);
    memset(out, 0, sizeof(*out));
    int maxnal = 4096;
    OraNal *nals = (OraNal *)malloc(sizeof(OraNal) * maxnal);
    int nn = ora_split_annexb(data, size, nals, maxnal);
    Dec *d = (Dec *)calloc(1, sizeof(Dec));
    uint8_t *rbsp = (uint8_t *)malloc((size_t)size + 16);
    int have_pic = 0, ret = -10;
    const SliceHdr *prev = NULL;
    for (int i = 0; i < nn; i++) {
        if (nals[i].n < 2) continue;
        int type = (nals[i].p[0] >> 1) & 63;
        long rn = ora_unescape(nals[i].p + 2, nals[i].n - 2, rbsp);
        OraBits b = {rbsp, rn, 0};
        if (type == 33) {
            if (have_pic) break;
            {
                int e = parse_sps(&b, d->sps);
                if (e < 0) { ret = e == -11 ? -11 : -2; goto done; }
            }
        } else if (type == 34) {
            if (have_pic) break;
            if (parse_pps(&b, d->pps, d->sps) < 0) { ret = -3; goto done; }
        } else if (type <= 21) {
            if (type >= 10 && type <= 15) continue; /* reserved */
            int first = (rbsp[0] >> 7) & 1;
            if (first && have_pic) break; /* next picture */
            if (!first && !have_pic) continue;
            if (d->nsh >= MAX_SLICES) { ret = -4; goto done; }
            SliceHdr *sh = &d->sh[d->nsh];
            int r = parse_slice_header(d, &b, type, sh, prev);
            if (r < 0) { ret = r == -2 ? -5 : -6; goto done; }
            if (!have_pic) {
                d->p = &d->pps[sh->pps_id];
                d->s = &d->sps[d->p->sps_id];
                alloc_picture(d);
                setup_tiles(d);
                have_pic = 1;
            }
            d->p = &d->pps[sh->pps_id];
            d->bits = b;
            if (decode_slice_data(d, d->nsh) < 0) { ret = -7; goto done_free; }
            prev = sh;
            d->nsh++;
        } else if (type == 35 && have_pic) {
            break; /* AUD: new access unit */
        }
    }
    if (!have_pic) { ret = -8; goto done; }
    if (!(flags & 1)) {
        deblock(d);
        if (d->s->sao) apply_sao(d);
    }
    /* crop */
    {
        const Sps *s = d->s;
        /* decode.c apply_cropping: the left offset as av_frame_apply_cropping aligns it (4:2:0
         * offsets are even: never AVERROR_BUG) */
        const int cl = ora_ff_crop_left(s->conf_l, d->bd > 8 ? 2 : 1);
        int w = d->W - cl - s->conf_r, h = d->H - s->conf_t - s->conf_b;
        out->width = w;
        out->height = h;
        out->bit_depth = d->bd;
        out->chroma_format = 1;
        for (int c = 0; c < 3; c++) {
            int sh = c ? 1 : 0, cw = w >> sh, ch = h >> sh;
            out->planes[c] = (uint16_t *)malloc((size_t)cw * ch * 2);
            out->stride[c] = cw;
            for (int y = 0; y < ch; y++)
                memcpy(out->planes[c] + (size_t)y * cw,
                       d->pl[c] + (size_t)(y + (s->conf_t >> sh)) * d->st[c] + (cl >> sh), (size_t)cw * 2);
        }
    }
    ret = 0;
done_free:
    for (int c = 0; c < 3; c++) free(d->pl[c]);
    free_picture(d);
done:
    if (ret != 0 && have_pic == 0) { /* nothing allocated */ }
    free(rbsp);
    free(d);
    free(nals);
    return ret;
}

void oracle_free_picture(OraclePicture *pic) {
    for (int c = 0; c < 3; c++) {
        free(pic->planes[c]);
        pic->planes[c] = NULL;
    }
}
