/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(),
 * bench.py's cpu_baseline leg).  Never linked into the product library.
 *
 * CPU restatement of the reference's hot path (BornToDeath/h264-h265-to-jpeg,
 * src/Decoder.cpp:115-361 + src/Encoder.cpp:104-308, arithmetic inside the
 * binary-only FFmpeg git-2021-01-28-6fd0116 / libavcodec 58.117.101).
 * See DESIGN.md "Oracle" for how each piece is pinned.
 */
#ifndef H2J_ORACLE_H
#define H2J_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- JPEG (jpeg_ref.c) ---- */
const uint8_t *oracle_zigzag(void);
void oracle_fdct(int16_t *blk);
int oracle_jpeg_qscale_from_var(int64_t V, int *lambda_out);
int oracle_jpeg_qscale(const uint8_t *y, int w, int h, int stride, int64_t *V_out, int *lambda_out);
void oracle_jpeg_matrix(int qscale, uint8_t M[64], uint16_t q16[64], uint16_t b16[64]);
int oracle_jpeg_coeffs(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h,
                       int ystride, int cstride, int16_t *coefs, int *qscale_out);
void oracle_jpeg_count(const int16_t *coefs, int nmcu, uint32_t counts[4][256]);
int oracle_huff_build(const uint32_t *counts, uint8_t bits[17], uint8_t *val);
long oracle_jpeg_from_coeffs(const int16_t *coefs, int w, int h, int qscale, const char *com,
                             uint8_t *out, long cap);
long oracle_jpeg_encode(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h,
                        int ystride, int cstride, const char *com, uint8_t *out, long cap);
int oracle_jpeg_parse(const uint8_t *jpg, long n, int *w_out, int *h_out, uint8_t dqt_zz[64],
                      int16_t *coefs, int max_mcu);

/* ---- HEVC intra decode (hevc_ref.c) ----
 * Decodes the first picture of an Annex-B stream.  Output planes are
 * 16-bit samples (8-bit content stored in uint16) cropped to the
 * conformance window.  flags bit0: skip loop filters (deblock + SAO).
 * Returns 0 on success, <0 on error. */
typedef struct {
    int width, height;       /* cropped output size (luma) */
    int bit_depth;           /* luma bit depth */
    int chroma_format;       /* 1 = 4:2:0 */
    uint16_t *planes[3];     /* malloc'ed, owned by caller (oracle_free_picture) */
    int stride[3];
} OraclePicture;

int oracle_hevc_decode(const uint8_t *data, long size, int flags, OraclePicture *pic);
int oracle_h264_decode(const uint8_t *data, long size, int flags, OraclePicture *pic);
void oracle_free_picture(OraclePicture *pic);

/* Full reference behaviour of IDecoder::H265ToJpeg on an in-memory stream:
 * detect codec, decode picture 0, 10->8 if needed, encode JPEG.  Returns
 * JPEG size (>0), or <=0 on failure. */
long oracle_transcode(const uint8_t *data, long size, const char *com, uint8_t *out, long cap);

#ifdef __cplusplus
}
#endif
#endif
