// Host-side JPEG assembly: optimal Huffman tables from the GPU's symbol
// histograms and the baseline bitstream from the GPU's quantised zigzag
// coefficients.  Restates what FFmpeg's mjpeg encoder does after
// quantisation (ff_mjpeg_build_optimal_huffman, ff_mjpeg_encode_picture_header,
// ff_mjpeg_encode_mb, ff_mjpeg_escape_FF / trailer), reached by the reference
// through avcodec_send_frame / avcodec_receive_packet
// (/root/reference/src/Encoder.cpp:250,259); layout per SURVEY.md A.6.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "h2j_jobs.h"

namespace h2j {

// libavcodec identification string the reference's x86_64 build writes in
// the COM segment (LIBAVCODEC_IDENT of libavcodec 58.117.101).
extern const char* const kLavcIdent;

// FFmpeg mjpegenc_huffman: counts[256] -> BITS[1..16], HUFFVAL; returns nval
int huffman_optimal(const uint32_t* counts, uint8_t bits[17], uint8_t* val);

// Assemble one JPEG.  coefs: int16 [nmcu][6][64] zigzag, DC absolute.
// Appends to out; returns bytes written.
size_t jpeg_assemble(const int16_t* coefs, int w, int h, const h2j_jstat& st, const char* com,
                     std::vector<uint8_t>& out);

}  // namespace h2j
