// Host-side container for one picture's job records (see include/h2j_jobs.h).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "h2j_jobs.h"

namespace h2j {

struct FrameJob {
    h2j_frame hdr{};
    std::vector<h2j_tu> tus;
    std::vector<h2j_coef> coefs;
    std::vector<h2j_ctb> ctbs;
    std::vector<h2j_slice> slices;
    std::vector<uint8_t> sl;  // scaling factors (2032 B) when hdr.scaling_list
    int error = 0;            // 0 ok, <0 parse error
    std::string message;
    int threads = 1;          // threads the parser may use inside this picture (independent slices)
    // the SPS signals output reordering (H.264 VUI max_num_reorder_frames > 0, H.265
    // sps_max_num_reorder_pics[HighestTid] > 0): FFmpeg holds the picture back until more
    // pictures or a flush arrive (only H2J_STRICT_REFERENCE acts on it)
    bool reorder_delay = false;
    // H.264 PAFF: picture 0 is a field pair (two field pictures).  FFmpeg outputs the frame after
    // the second field; the reference sends one packet (one field) and returns false (only
    // H2J_STRICT_REFERENCE acts on it)
    bool field_pair = false;

    void clear() {
        hdr = h2j_frame{};
        tus.clear();
        coefs.clear();
        ctbs.clear();
        slices.clear();
        sl.clear();
        error = 0;
        message.clear();
        reorder_delay = false;
        field_pair = false;
    }
};

// Offsets of the scaling-factor tables inside FrameJob::sl
enum { H2J_SL_S0 = 0, H2J_SL_S1 = 48, H2J_SL_S2 = 240, H2J_SL_S3 = 1008, H2J_SL_BYTES = 2032 };
// H.264 weight-scale tables inside FrameJob::sl (raster order): 4x4 intra Y/Cb/Cr, 8x8 intra Y
enum { H2J_SL264_4 = 0, H2J_SL264_8 = 48, H2J_SL264_BYTES = 112 };

// Parse the first picture of an HEVC Annex-B stream into job records.
// Returns 0 on success.
int hevc_parse_picture(const uint8_t* data, size_t size, FrameJob& job);
// Same for H.264.
int h264_parse_picture(const uint8_t* data, size_t size, FrameJob& job);

}  // namespace h2j
