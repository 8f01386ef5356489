// Host-side JPEG container: the GPU (h2j_gpu_entropy) produces the optimal
// Huffman tables and the entropy-coded payload; the host wraps them in the
// marker segments FFmpeg's mjpeg encoder writes and applies the 0xFF -> 0xFF
// 0x00 byte stuffing while copying the payload (ff_mjpeg_encode_picture_header,
// ff_mjpeg_escape_FF and the trailer, reached by the reference through
// avcodec_send_frame / avcodec_receive_packet, /root/reference/src/Encoder.cpp:250,259;
// layout per SURVEY.md A.6).
#pragma once
#include <cstddef>
#include <cstdint>

#include "h2j_jobs.h"

namespace h2j {

// libavcodec identification string the reference's x86_64 build writes in
// the COM segment (LIBAVCODEC_IDENT of libavcodec 58.117.101).
extern const char* const kLavcIdent;

// Exact size of the JPEG for a payload of st.nbytes bytes.
size_t jpeg_container_size(const h2j_jstat& st, const uint8_t* payload, const char* com);

// Write the JPEG (SOI, COM, DQT, DHT x4, SOF0, SOS, stuffed payload, EOI)
// into out (at least jpeg_container_size bytes).  Returns bytes written.
size_t jpeg_write_container(const h2j_jstat& st, const uint8_t* payload, int w, int h, const char* com,
                            uint8_t* out);

}  // namespace h2j
