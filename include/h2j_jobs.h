/*
 * h2j_jobs.h — the job records the host entropy decoders ship to HBM.
 *
 * This is the data contract between the C++11 host side (Annex-B parsing +
 * CABAC/CAVLC on pinned host threads) and the CDNA4 HIP pixel pipeline.  It
 * replaces what happens inside FFmpeg between avcodec_send_packet and the
 * decoded AVFrame in the reference (/root/reference/src/Decoder.cpp:324-342):
 * the host emits, per picture, one record per transform block (position,
 * size, intra mode, QP, flags) plus the sparse quantised coefficients; the
 * GPU does dequantisation, inverse transform, intra prediction, deblocking,
 * SAO and the JPEG forward path.
 *
 * Plain C, POD only, fixed-width fields: the same bytes are read by hipcc
 * device code and gcc host code.
 */
#ifndef H2J_JOBS_H
#define H2J_JOBS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum h2j_codec { H2J_CODEC_NONE = 0, H2J_CODEC_H264 = 264, H2J_CODEC_HEVC = 265 };

/* TU record flags */
enum {
    H2J_TU_CBF = 1u << 0,     /* residual present (ncoef entries) */
    H2J_TU_TSKIP = 1u << 1,   /* HEVC transform_skip_flag */
    H2J_TU_BYPASS = 1u << 2,  /* cu_transquant_bypass / H.264 lossless: residual = levels */
    H2J_TU_PCM = 1u << 3,     /* coefficients hold raw samples (already scaled to bit depth) */
    H2J_TU_EDGE_L = 1u << 4,  /* left edge is a deblocking edge (filterEdgeFlag && on 8 grid) */
    H2J_TU_EDGE_T = 1u << 5,  /* top edge is a deblocking edge */
    H2J_TU_NOFILT = 1u << 6,  /* samples excluded from deblock/SAO (pcm+lf disabled, bypass) */
    H2J_TU_DST = 1u << 7,     /* HEVC 4x4 luma intra: DST-VII instead of DCT */
    /* H.264 transform-bypass TBs (H2J_TU_BYPASS) with a vertical / horizontal intra prediction:
     * the residual accumulates down the columns / along the rows (8.5.15); the bits are HEVC's
     * deblocking-edge flags, which H.264 records do not use */
    H2J_TU_DPCM_V = 1u << 4,
    H2J_TU_DPCM_H = 1u << 5
};
/* H.264 coefficient entries carry 24-bit levels (10- to 14-bit video: levels up to
 * +-2^(7 + bitDepth)): (pos << 24) | (level & 0xFFFFFF); HEVC entries and PCM samples keep
 * (pos << 16) | (uint16_t)value */
#define H2J_COEF264(pos, level) ((((uint32_t)(pos)) << 24) | (((uint32_t)(level)) & 0xFFFFFFu))

/* One transform block of one colour component, in decoding order.
 * HEVC: every luma/chroma TB of the picture (prediction happens per TB even
 * when cbf == 0).  x, y, log2n are in the component's sample grid. */
typedef struct {
    uint16_t x, y;
    uint8_t log2n;   /* 2..5 */
    uint8_t c;       /* 0 Y, 1 Cb, 2 Cr */
    uint8_t mode;    /* intra prediction mode (HEVC 0..34) */
    uint8_t flags;   /* H2J_TU_* */
    int8_t qp;       /* qP for scaling (Qp'Y / Qp'Cb / Qp'Cr, includes QpBdOffset) */
    int8_t qpy;      /* QpY of the coding unit (deblocking), luma TBs */
    uint16_t ncoef;  /* entries in the coefficient stream */
    uint32_t coef;   /* first entry (frame-relative) */
} h2j_tu;

/* coefficient entry: (pos << 16) | (uint16_t)level, pos = y * n + x (H.264 levels: H2J_COEF264) */
typedef uint32_t h2j_coef;

/* One HEVC CTB or one H.264 macroblock (log2ctb 4). */
typedef struct {
    int8_t type[3];     /* HEVC SAO: 0 off, 1 band, 2 edge */
    int8_t band_pos[3];
    int8_t eo_class[3];
    uint8_t slice;      /* index into the frame's slice table */
    int16_t off[3][4];  /* HEVC SaoOffsetVal[1..4] */
    uint16_t tile;      /* tile id */
    int8_t qp;          /* H.264: QPY of the macroblock (deblocking) */
    uint8_t mbflags;    /* H.264: bit0 I_PCM, bit1 transform_size_8x8_flag, bit2 decoded, bit3 MBAFF field MB */
    uint32_t ts;        /* CtbAddrRsToTs (H.264: macroblock address) */
} h2j_ctb;

typedef struct {
    int8_t beta_offset;     /* HEVC slice_beta_offset_div2 * 2 | H.264 FilterOffsetB */
    int8_t tc_offset;       /* HEVC slice_tc_offset_div2 * 2   | H.264 FilterOffsetA */
    uint8_t sao_luma, sao_chroma;
    uint8_t lf_across_slices;
    uint8_t deblock_disabled; /* HEVC flag | H.264 disable_deblocking_filter_idc (0, 1, 2) */
    int8_t cqp_offset[2];   /* H.264 chroma_qp_index_offset, second_chroma_qp_index_offset */
    int32_t slice_addr_rs;  /* first CTB / macroblock of the slice */
} h2j_slice;

/* One picture.  Offsets are relative to the start of the batch's arrays. */
typedef struct {
    int32_t codec;                  /* h2j_codec */
    int32_t width, height;          /* coded size (luma) */
    int32_t crop_x, crop_y;         /* conformance window origin (luma) */
    int32_t out_w, out_h;           /* cropped output size (luma) */
    int32_t bit_depth, bit_depth_c;
    int32_t log2ctb, ctb_w, ctb_h;
    int32_t strong_smoothing;       /* bit 0 strong_intra_smoothing; H2J_NO_INTRA_SMOOTHING (RExt) */
    int32_t sao_enabled;
    int32_t lf_across_tiles;
    int32_t cb_qp_offset, cr_qp_offset; /* pps offsets (deblocking) */
    int32_t scaling_list;           /* 1: scaling factors at sl */
    uint32_t tu, ntu;               /* h2j_tu range */
    uint32_t coef;                  /* base of this frame's coefficient entries */
    uint32_t ctb;                   /* h2j_ctb base (ctb_w * ctb_h records) */
    uint32_t slice, nslice;         /* h2j_slice range */
    uint32_t sl;                    /* uint8 scaling factor tables: [sizeId 0..3][c 0..2][32*32]... see DESIGN.md */
    uint32_t topo;                  /* 1: several slices / tiles, or not starting at CTB 0 (availability needs the CTB records) */
    /* device arena offsets (bytes), filled by the pipeline */
    uint64_t pic;                   /* reconstruction / deblocking planes */
    uint64_t pic2;                  /* SAO output planes (final decoded picture) */
    uint64_t maps;                  /* per-4x4 deblocking maps: flags (u8) then qp (i8) */
    uint64_t jcoef;                 /* JPEG coefficients int16 [mcu][6][64] */
    uint64_t jstat;                 /* JPEG per-frame stats (h2j_jstat) */
    uint64_t res;                   /* int16 residual planes (K0 -> K1): HEVC tiled by K1 quadrant
                                       (h2j_res_q in h2j_gpu.h), H.264 the picture's raster layout */
    uint64_t aux;                   /* K0 -> K1: uint64 reference-availability mask per TU */
    uint64_t ctbrng;                /* K0 -> K1: uint32 [first, end) TU range per CTB (zeroed) */
    int32_t pic_stride[3];          /* elements */
    int32_t pic_off[3];             /* element offset of each plane inside pic / pic2 */
    int32_t mw, mh;                 /* 4x4 map dims */
    int32_t status;                 /* device-side error code */
    int32_t k1bands;                /* H.264 K1: workgroups (16-row bands) this picture runs on */
    uint64_t xline;                 /* H.264 K1 band boundaries: bottom rows handed to the next band (uint16) */
    int32_t mbaff;                  /* H.264 MBAFF frame: macroblock pairs (h2j_ctb.mbflags bit 3: field
                                       pair), TU records in the MB grid (grid row = 2 pair row + bottom),
                                       availability masks from the host (h2j_tu.qpy bits 0-3) */
    int32_t rext;                   /* HEVC range-extension residual tools K0 applies: H2J_REXT_* */
} h2j_frame;

/* h2j_frame.strong_smoothing bit 1: RExt intra_smoothing_disabled_flag (no reference filtering) */
#define H2J_NO_INTRA_SMOOTHING 2
/* h2j_frame.rext: implicit RDPCM of transform-skip / bypass TBs predicted with mode 10 / 26;
 * 180-degree rotation of 4x4 transform-skip residuals (FFmpeg 4.3: not of bypass blocks) */
#define H2J_REXT_RDPCM 1
#define H2J_REXT_TS_ROT 2

/* per-frame JPEG statistics written by the GPU */
typedef struct {
    int64_t var_sum;        /* Σ MB variance */
    int32_t qscale, lambda;
    uint32_t hist[4][256];  /* DC-Y, DC-C, AC-Y, AC-C symbol counts */
    uint16_t q16[64];       /* quantiser reciprocal (A.5), natural order */
    uint16_t b16[64];       /* quantiser bias (A.5) */
    uint8_t dqt[64];        /* DQT entries, natural order (A.3) */
    /* optimal Huffman tables (K5a, FFmpeg mjpegenc_huffman.c semantics) */
    uint8_t bits[4][20];    /* [t][1..16] code counts per length */
    uint8_t val[4][256];    /* symbols in DHT order */
    uint8_t len[4][256];    /* code length per symbol */
    uint16_t code[4][256];  /* code per symbol */
    uint32_t nval[4];       /* symbols per table */
    /* entropy-coded segment (K5b-K5d) */
    uint32_t nbits;         /* payload bits before the 1-padding */
    uint32_t nbytes;        /* padded payload bytes (no 0xFF stuffing) */
    uint64_t seg_off;       /* byte offset of the payload in the segment pool */
    uint32_t dev_error;     /* device-side failure flags: a progress wait timed out (bit 0 H.264 K1 band hand-off,
                               1 H.264 deblocking band hand-off, 2 HEVC K1 row, 3 H.264 K1 row, 4 H.264
                               deblocking row); the picture fails with status -52 */
    uint32_t pad_e;
} h2j_jstat;

#ifdef __cplusplus
}
#endif
#endif
