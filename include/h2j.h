/*
 * h2j.h — C ABI of libH265ToJpeg.so beyond the reference's C++ surface.
 *
 * The reference exports exactly two entry points for this path
 * (SURVEY.md §8b):
 *   - IDecoder::getInstance() / virtual bool H265ToJpeg(in, out)
 *       (/root/reference/export_inc/IDecoder.h:29,35)       -> include/IDecoder.h
 *   - Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decode
 *       (/root/reference/src/jni/com_autonavi_socol_occtiltedserver_service_H265DecodeService.h:15-16)
 * Both are kept verbatim.  The functions below are the batch engine those
 * entry points sit on; they are what an FFI binding (ctypes, cgo, N-API)
 * would bind for throughput, see INTEGRATION.md.
 *
 * Return values: 0 success, < 0 error (message via h2j_engine_error).
 */
#ifndef H2J_H
#define H2J_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct h2j_engine h2j_engine;

/* Visible HIP devices (0: the MI355X pipeline cannot run). */
int h2j_device_count(void);

/* device: HIP device ordinal; host_threads: entropy/Huffman threads (the caller's thread
 * included).  > 0: exactly that many.  0: automatic -- the process's CPUs on the device's NUMA
 * node, split between the visible devices of that node, bounded by the cgroup CPU quota and 64;
 * the pool's workers are pinned to that NUMA-local slice (H2J_PIN=0: not pinned).  -k: as 0,
 * for one of k engines in this process (they share the cgroup quota). */
h2j_engine *h2j_engine_create(int device, int host_threads);
void h2j_engine_destroy(h2j_engine *e);
const char *h2j_engine_error(h2j_engine *e);
/* Message of picture i of the last h2j_engine_transcode ("" if it succeeded).  The string stays
 * valid until the calling thread's next h2j_engine_frame_error call. */
const char *h2j_engine_frame_error(h2j_engine *e, int i);
/* Host placement: out[0] threads (incl. the caller), [1] the device's NUMA node (-1 unknown),
 * [2] CPUs the workers are pinned to (0: not pinned), [3] first of those CPUs. */
int h2j_engine_host_info(h2j_engine *e, int *out, int n);

/* Transcode n independent Annex-B stills (H.264 or H.265, first picture of
 * each) to baseline JPEG.  JPEG i is written at out + out_off[i], length
 * out_len[i]; status[i] = 0 on success, < 0 on failure for that item.
 * Returns 0 if the batch ran (per-item failures reported in status), < 0
 * if the batch could not run (e.g. no GPU, out_cap too small). */
int h2j_engine_transcode(h2j_engine *e, int n, const uint8_t *const *data, const size_t *sizes,
                         uint8_t *out, size_t out_cap, size_t *out_off, size_t *out_len, int *status);

/* Asynchronous batches.  h2j_engine_submit queues a batch (same arguments and per-item
 * semantics as h2j_engine_transcode) and returns a ticket (> 0) at once; the engine parses
 * batches in submission order on its thread pool and runs their GPU work and JPEG assembly on a
 * driver thread, so one batch's GPU tail overlaps the next batch's entropy decoding.  A
 * submitted batch is cut into chunks of up to 1024 pictures (K1 then reconstructs up to four
 * pictures per workgroup).  Every pointer passed to submit must stay valid until
 * h2j_engine_wait returns for that ticket; h2j_engine_wait returns what h2j_engine_transcode
 * would have.  h2j_engine_transcode is submit + wait with smaller, latency-oriented chunks.
 * Stats, chunk times and frame errors describe the last batch that finished. */
int64_t h2j_engine_submit(h2j_engine *e, int n, const uint8_t *const *data, const size_t *sizes,
                          uint8_t *out, size_t out_cap, size_t *out_off, size_t *out_len, int *status);
int h2j_engine_wait(h2j_engine *e, int64_t ticket);

/* Test / inspection entry points (one picture).
 * stage: 0 final decoded picture, 1 pre-loop-filter, 2 deblocked (pre-SAO).
 * planes_out: uint16 Y (w*h) then U, V ((w/2)*(h/2)) of the cropped picture.
 * info[0..2] = w, h, bit_depth. */
int h2j_engine_decode(h2j_engine *e, const uint8_t *data, size_t size, int stage, uint16_t *planes_out,
                      size_t cap_elems, int *info);
/* The same for picture `pick` of n pictures reconstructed as ONE GPU batch (the launch shapes of
 * a production chunk of n pictures: K1's picture pool with up to 4 pictures per workgroup at
 * n >= 1024), so parity tests can read planes from inside a bench-sized batch. */
int h2j_engine_decode_batch(h2j_engine *e, int n, const uint8_t *const *data, const size_t *sizes, int stage,
                            int pick, uint16_t *planes_out, size_t cap_elems, int *info);
/* JPEG coefficients int16 [mcu][6][64] zigzag of the decoded picture;
 * info[0..3] = w, h, qscale, nmcu. */
int h2j_engine_jpeg_coeffs(h2j_engine *e, const uint8_t *data, size_t size, int16_t *out, size_t cap_elems,
                           int *info);
/* Timing of the batch the last h2j_engine_transcode / h2j_engine_wait returned, milliseconds:
 * [0] parse (host, wall, from submission)  [1] h2d  [2] recon  [3] deblock  [4] sao
 * [5] jpeg (GPU)  [6] d2h  [7] huffman (host, wall)  [8] total (wall)
 * [9] frames  [10] algorithmic bytes of the GPU pixel path  [11] GPU entropy
 * [12] K0 prep  [13] chunks  [14] record packing (host)  [15] parse (host, wall, first to last
 * picture of the batch: without the wait behind the previous batch). */
int h2j_engine_stats(h2j_engine *e, double *out, int n);
/* Per chunk (one GPU launch of each stage) of the last h2j_engine_transcode, in order:
 * out[3i] pictures, out[3i+1] K1 ms, out[3i+2] K0..K5 ms (HIP events on the chunk's stream).
 * Returns the number of chunks (entries beyond max_chunks are not written). */
int h2j_engine_chunk_times(h2j_engine *e, double *out, int max_chunks);

/* In-memory and batch entry points beside IDecoder (the reference has only the
 * file-path call, /root/reference/export_inc/IDecoder.h:29).
 * Both go through the same process-wide batching engine as IDecoder, so
 * concurrent callers share GPU batches.
 * h2j_h265_to_jpeg_mem: one Annex-B still (H.264 or H.265) -> JPEG bytes in
 *   *jpeg (malloc'ed, release with h2j_free), 0 on success, < 0 on failure.
 * h2j_h265_to_jpeg_batch: n (input, output) file pairs transcoded as one
 *   batch; ok[i] = 1 where output i was written (may be NULL); returns the
 *   number written.  Per-file behaviour (empty paths, unreadable input, LOG
 *   lines) is that of IDecoder::H265ToJpeg. */
int h2j_h265_to_jpeg_mem(const uint8_t *data, size_t size, uint8_t **jpeg, size_t *jpeg_len);
int h2j_h265_to_jpeg_batch(const char *const *in_paths, const char *const *out_paths, int n, int *ok);
void h2j_free(void *p);

/* Library self-description (version, arch, build). */
const char *h2j_version(void);

#ifdef __cplusplus
}
#endif
#endif
