/*
 * h2j_gpu.h — thin C ABI of libh2j_hip.so, the MI355X (gfx950) pixel
 * pipeline.  Plain pointers and sizes; no torch / HIP types in signatures
 * (streams and events are opaque void*).
 *
 * Boundary: these entry points replace what the reference does inside
 * FFmpeg after entropy decoding, i.e. the arithmetic behind
 *   avcodec_send_packet/avcodec_receive_frame (/root/reference/src/Decoder.cpp:324,342):
 *     dequant + inverse transform + intra prediction   -> h2j_gpu_recon
 *     deblocking                                       -> h2j_gpu_deblock
 *     SAO                                              -> h2j_gpu_sao
 *   avcodec_send_frame (/root/reference/src/Encoder.cpp:250), mjpeg encoder:
 *     pad + MB variance + rate control + FDCT + quantiser + zigzag + symbol
 *     statistics                                       -> h2j_gpu_jpeg
 * The host (libH265ToJpeg.so) builds the optimal Huffman tables from the
 * statistics and emits the JPEG bitstream (avcodec_receive_packet, :259).
 *
 * All functions return 0 on success, a negative code on failure; the text
 * of the last failure is available from h2j_gpu_last_error().
 */
#ifndef H2J_GPU_H
#define H2J_GPU_H
#include <stddef.h>
#include <stdint.h>

#include "h2j_jobs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* device / memory / stream plumbing */
int h2j_gpu_device_count(void);
int h2j_gpu_set_device(int device);
/* PCI bus id "dddd:bb:dd.f" of a device (locates its NUMA node in sysfs for host-thread pinning) */
int h2j_gpu_pci_bus_id(int device, char *buf, int len);
void *h2j_gpu_malloc(size_t bytes);
int h2j_gpu_free(void *p);
int h2j_gpu_mem_info(size_t *free_bytes, size_t *total_bytes); /* current device */
void *h2j_gpu_host_alloc(size_t bytes); /* pinned */
int h2j_gpu_host_free(void *p);
void *h2j_gpu_stream_create(void);
int h2j_gpu_stream_destroy(void *stream);
int h2j_gpu_stream_sync(void *stream);
int h2j_gpu_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int h2j_gpu_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int h2j_gpu_memset(void *dst, int value, size_t bytes, void *stream);
void *h2j_gpu_event_create(void);
int h2j_gpu_event_destroy(void *ev);
int h2j_gpu_event_record(void *ev, void *stream);
/* `stream` runs nothing enqueued after this call until `ev` (recorded on another stream) has completed */
int h2j_gpu_stream_wait_event(void *stream, void *ev);
float h2j_gpu_event_elapsed_ms(void *start, void *stop);
const char *h2j_gpu_last_error(void);

#ifdef __cplusplus
/* HEVC residual planes (K0 writes, K1 reads) in quadrant tiles: each component in tiles of
 * 2^q x 2^q int16 samples (q = the K1 quadrant size: min(log2ctb, 5) for luma, one less for
 * chroma), tiles in raster order, planes Y, Cb, Cr back to back.  A K1 quadrant is then one
 * contiguous tile (2 KB luma, 512 B per chroma plane) and every TB lies inside one tile.
 * (constexpr: host and device code share it) */
constexpr int h2j_res_q(int log2ctb, int c) { return (log2ctb < 5 ? log2ctb : 5) - (c ? 1 : 0); }
constexpr long long h2j_res_tiles(int n, int q) { return (n + (1 << q) - 1) >> q; }
constexpr long long h2j_res_plane(int w, int h, int q) { return (h2j_res_tiles(w, q) * h2j_res_tiles(h, q)) << (2 * q); }
/* int16 elements of the three tiled planes of a w x h 4:2:0 picture */
constexpr long long h2j_res_elems(int w, int h, int log2ctb) {
    return h2j_res_plane(w, h, h2j_res_q(log2ctb, 0)) + 2 * h2j_res_plane(w / 2, h / 2, h2j_res_q(log2ctb, 1));
}
/* K3 SAO sums the JPEG rate control's MB variances of a picture (K4a skips it) when the picture
 * has SAO (its own output plane) and its 16x16 output MB grid is aligned with the CTB grid.
 * (constexpr: host and device code share it) */
constexpr bool h2j_sao_folds_variance(const h2j_frame &f) {
    return f.codec == H2J_CODEC_HEVC && f.pic2 != f.pic && (f.crop_x & 15) == 0 && (f.crop_y & 15) == 0 &&
           (f.out_w & 15) == 0;
}
#endif

/* JPEG symbol stream (production path): per frame, one tile of H2J_JTILE_BYTES per 256 blocks
 * at h2j_frame.jcoef (the dense int16 plane occupies the same region on the inspection path). */
#define H2J_JSYM_MAX 68
#define H2J_JTILE_BYTES (H2J_JSYM_MAX * 256 * 4 + 256 + 512)

#define H2J_SAO_GROUPS 4

/* One batch of pictures resident in HBM.  All pointers are device pointers. */
typedef struct {
    int32_t nframes;
    int32_t max_w, max_h;       /* max coded luma size over the batch */
    int32_t max_mcu;            /* max JPEG MCUs over the batch */
    int32_t max_ntu;            /* max transform-block records over the batch */
    int32_t has_hevc, has_h264; /* codecs present in the batch */
    int32_t max_ctbs;           /* max CTBs of one HEVC picture over the batch */
    int32_t k1wgs;              /* H.264 K1 workgroups (sum of h2j_frame.k1bands over H.264 pictures) */
    const uint32_t *k1map;      /* H.264 K1 workgroup -> (frame << 8) | band, dependency order */
    int32_t hevc_pels;          /* HEVC sample types present: bit 0 8-bit, bit 1 high bit depth */
    int32_t k1all_n;            /* entries of k1all */
    const uint32_t *k1all;      /* mixed-batch K1 workgroups, longest chains first: HEVC pictures
                                   (1u << 31) | (frame << 8), then H.264 (frame << 8) | band */
    const h2j_frame *frames;
    const h2j_tu *tus;
    const h2j_coef *coefs;
    const h2j_ctb *ctbs;
    const h2j_slice *slices;
    const uint8_t *sl;
    uint8_t *arena;             /* pictures, maps, JPEG coefficients + stats */
    /* JPEG entropy stage (h2j_gpu_entropy) */
    uint8_t *seg;               /* entropy-coded segment pool, frames packed at jstat.seg_off */
    uint64_t seg_cap;           /* pool bytes */
    uint32_t *tile_bits;        /* scratch: nframes x ceil(max_mcu*6/256) */
    uint64_t *seg_total;        /* device scalar: pool bytes used (16-byte units x16) */
    int32_t jpeg_dense;         /* 1: K4 writes the dense int16 coefficient plane (inspection), no K5 */
    int32_t k4a_frames;         /* frames whose MB variances K4a sums (the others are summed by K3 SAO,
                                   h2j_sao_folds_variance); 0: K4a is not launched */
    int32_t has_mbaff;          /* H.264 MBAFF frames present (K1 runs h2j_k1_recon_h264_mbaff for them) */
    int32_t h264_pels;          /* non-MBAFF H.264 sample types present: bit 0 8-bit, bit 1 high bit depth */
    /* K3 SAO: one launch per CTB-count class of the HEVC pictures with SAO (a mixed batch's 720p,
       1080p and 4K pictures each get a grid of their own width instead of the largest one's) */
    int32_t sao_groups;         /* launches (0..H2J_SAO_GROUPS) */
    int32_t sao_first[H2J_SAO_GROUPS], sao_count[H2J_SAO_GROUPS], sao_ctbs[H2J_SAO_GROUPS];
    const uint32_t *sao_map;    /* frame indices of the HEVC pictures with SAO, most CTBs first */
    /* H.264 K1 launch of kAvcK1Waves-wave workgroups (h2j_k1_recon_h264): tall pictures in bands of
       as many rows as the workgroup has waves (one row round per band), band-major */
    int32_t k1wgs8;
    const uint32_t *k1map8;     /* workgroup -> (frame << 8) | band of 8 macroblock rows */
    /* the HEVC entries of k1all alone, same order: a mixed batch's HEVC K1 (h2j_k1_recon_any) beside
       the H.264 K1 (h2j_k1_recon_h264 on k1map8) on a companion stream */
    int32_t k1hevc_n;
    const uint32_t *k1hevc;
} h2j_gpu_batch;

/* K0 + K1: K0 (all TUs in parallel) availability masks, CTB->TU ranges,
 * deblocking maps, PCM samples and residuals (dequantisation + inverse
 * transform) into frame.res; K1 (CTB-row wavefront, one workgroup per
 * picture) intra prediction + residual -> the pre-loop-filter picture in
 * frame.pic.  HEVC and H.264. */
int h2j_gpu_recon(const h2j_gpu_batch *b, void *stream);
/* the two halves of h2j_gpu_recon: K0 alone, then K1 alone */
int h2j_gpu_prep(const h2j_gpu_batch *b, void *stream);
int h2j_gpu_predict(const h2j_gpu_batch *b, void *stream);
/* Diagnostics: K1 cycle counters of a -DH2J_PROF build (`make prof`); -1 otherwise. */
int h2j_gpu_prof(unsigned long long *out, int n, int reset);
/* K2: deblocking (vertical edges, then horizontal edges), in place on frame.pic */
int h2j_gpu_deblock(const h2j_gpu_batch *b, void *stream);
/* K3: SAO frame.pic -> frame.pic2 (copies when SAO is off) */
int h2j_gpu_sao(const h2j_gpu_batch *b, void *stream);
/* K4: JPEG forward path on frame.pic2 -> frame.jcoef / frame.jstat
 * (variance, rate control, FDCT + quantiser + zigzag, symbol histograms) */
int h2j_gpu_jpeg(const h2j_gpu_batch *b, void *stream);
/* K4d alone: Huffman symbol histograms of frame.jcoef -> jstat.hist */
int h2j_gpu_histogram(const h2j_gpu_batch *b, void *stream);
/* K5: optimal Huffman tables (jstat.bits/val/code/len) and the entropy-coded
 * payload of every frame, packed into b->seg at jstat.seg_off (jstat.nbytes
 * bytes, 1-padded, no 0xFF stuffing).  *b->seg_total = bytes used. */
int h2j_gpu_entropy(const h2j_gpu_batch *b, void *stream);

#ifdef __cplusplus
}
#endif
#endif
