// H.264 intra entropy decoding on the host (CABAC / CAVLC; progressive, MBAFF and PAFF; 4:2:0 and
// 4:0:0 -- the latter's chroma is FFmpeg's DC_128 / 1 << (BitDepth - 1), see decode_mb).
//
// Replaces the parsing half of FFmpeg's h264 decoder reached through
// avcodec_send_packet (/root/reference/src/Decoder.cpp:324): SPS/PPS/slice
// header (H.264 7.3), CABAC macroblock layer for I slices (9.3: mb_type,
// transform_size_8x8_flag, intra 4x4/8x8 mode prediction, intra chroma mode,
// coded_block_pattern, mb_qp_delta, residual blocks incl. coded_block_flag
// contexts), I_PCM.  Emits one h2j_tu per prediction/transform unit:
//   luma I4x4 -> 16 records (log2n 2), I8x8 -> 4 (log2n 3), I16x16 -> 1
//   (log2n 4, DC levels stored at the (4i,4j) positions), I_PCM -> 1 (PCM);
//   chroma -> 1 record per component (log2n 3, DC levels at (4i,4j)).
// Macroblocks reuse the h2j_ctb record (log2ctb 4): slice, address, QPY,
// I_PCM / transform_size_8x8 flags for intra availability and deblocking.
#include <algorithm>
#include <atomic>
#include <memory>
#include <thread>
#include <cstdlib>
#include <cstring>

#include "bitstream.h"
#include "cabac.h"
#include "cavlc_tables.h"
#include "job.h"

namespace h2j {
namespace {

// (m, n) for ctxIdx 0..459, I slices (H.264 Tables 9-12 .. 9-33)
const int8_t kInitI[460][2] = {
    {20, -15}, {2, 54}, {3, 74}, {20, -15}, {2, 54}, {3, 74}, {-28, 127}, {-23, 104}, {-6, 53}, {-1, 54}, {7, 51},
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0},
    {0, 41}, {0, 63}, {0, 63}, {0, 63}, {-9, 83}, {4, 86}, {0, 97}, {-7, 72}, {13, 41}, {3, 62},
    {0, 11}, {1, 55}, {0, 69}, {-17, 127}, {-13, 102}, {0, 82}, {-7, 74}, {-21, 107}, {-27, 127}, {-31, 127},
    {-24, 127}, {-18, 95}, {-27, 127}, {-21, 114}, {-30, 127}, {-17, 123}, {-12, 115}, {-16, 122},
    {-11, 115}, {-12, 63}, {-2, 68}, {-15, 84}, {-13, 104}, {-3, 70}, {-8, 93}, {-10, 90}, {-30, 127},
    {-1, 74}, {-6, 97}, {-7, 91}, {-20, 127}, {-4, 56}, {-5, 82}, {-7, 76}, {-22, 125},
    {-7, 93}, {-11, 87}, {-3, 77}, {-5, 71}, {-4, 63}, {-4, 68}, {-12, 84}, {-7, 62}, {-7, 65}, {8, 61},
    {5, 56}, {-2, 66}, {1, 64}, {0, 61}, {-2, 78}, {1, 50}, {7, 52}, {10, 35}, {0, 44}, {11, 38},
    {1, 45}, {0, 46}, {5, 44}, {31, 17}, {1, 51}, {7, 50}, {28, 19}, {16, 33}, {14, 62}, {-13, 108},
    {-15, 100},
    {-13, 101}, {-13, 91}, {-12, 94}, {-10, 88}, {-16, 84}, {-10, 86}, {-7, 83}, {-13, 87}, {-19, 94}, {1, 70},
    {0, 72}, {-5, 74}, {18, 59}, {-8, 102}, {-15, 100}, {0, 95}, {-4, 75}, {2, 72}, {-11, 75}, {-3, 71},
    {15, 46}, {-13, 69}, {0, 62}, {0, 65}, {21, 37}, {-15, 72}, {9, 57}, {16, 54}, {0, 62}, {12, 72},
    {24, 0}, {15, 9}, {8, 25}, {13, 18}, {15, 9}, {13, 19}, {10, 37}, {12, 18}, {6, 29}, {20, 33},
    {15, 30}, {4, 45}, {1, 58}, {0, 62}, {7, 61}, {12, 38}, {11, 45}, {15, 39}, {11, 42}, {13, 44},
    {16, 45}, {12, 41}, {10, 49}, {30, 34}, {18, 42}, {10, 55}, {17, 51}, {17, 46}, {0, 89}, {26, -19},
    {22, -17},
    {26, -17}, {30, -25}, {28, -20}, {33, -23}, {37, -27}, {33, -23}, {40, -28}, {38, -17}, {33, -11}, {40, -15},
    {41, -6}, {38, 1}, {41, 17}, {30, -6}, {27, 3}, {26, 22}, {37, -16}, {35, -4}, {38, -8}, {38, -3},
    {37, 3}, {38, 5}, {42, 0}, {35, 16}, {39, 22}, {14, 48}, {27, 37}, {21, 60}, {12, 68}, {2, 97},
    {-3, 71}, {-6, 42}, {-5, 50}, {-3, 54}, {-2, 62}, {0, 58}, {1, 63}, {-2, 72}, {-1, 74}, {-9, 91},
    {-5, 67}, {-5, 27}, {-3, 39}, {-2, 44}, {0, 46}, {-16, 64}, {-8, 68}, {-10, 78}, {-6, 77}, {-10, 86},
    {-12, 92}, {-15, 55}, {-10, 60}, {-6, 62}, {-4, 65},
    {-12, 73}, {-8, 76}, {-7, 80}, {-9, 88}, {-17, 110}, {-11, 97}, {-20, 84}, {-11, 79}, {-6, 73}, {-4, 74},
    {-13, 86}, {-13, 96}, {-11, 97}, {-19, 117}, {-8, 78}, {-5, 33}, {-4, 48}, {-2, 53}, {-3, 62}, {-13, 71},
    {-10, 79}, {-12, 86}, {-13, 90}, {-14, 97},
    {0, 0},
    {-6, 93}, {-6, 84}, {-8, 79}, {0, 66}, {-1, 71}, {0, 62}, {-2, 60}, {-2, 59}, {-5, 75}, {-3, 62},
    {-4, 58}, {-9, 66}, {-1, 79}, {0, 71}, {3, 68}, {10, 44}, {-7, 62}, {15, 36}, {14, 40}, {16, 27},
    {12, 29}, {1, 44}, {20, 36}, {18, 32}, {5, 42}, {1, 48}, {10, 62}, {17, 46}, {9, 64}, {-12, 104},
    {-11, 97},
    {-16, 96}, {-7, 88}, {-8, 85}, {-7, 85}, {-9, 85}, {-13, 88}, {4, 66}, {-3, 77}, {-3, 76}, {-6, 76},
    {10, 58}, {-1, 76}, {-1, 83}, {-7, 99}, {-14, 95}, {2, 95}, {0, 76}, {-5, 74}, {0, 70}, {-11, 75},
    {1, 68}, {0, 65}, {-14, 73}, {3, 62}, {4, 62}, {-1, 68}, {-13, 75}, {11, 55}, {5, 64}, {12, 70},
    {15, 6}, {6, 19}, {7, 16}, {12, 14}, {18, 13}, {13, 11}, {13, 15}, {15, 16}, {12, 23}, {13, 23},
    {15, 20}, {14, 26}, {14, 44}, {17, 40}, {17, 47}, {24, 17}, {21, 21}, {25, 22}, {31, 27}, {22, 29},
    {19, 35}, {14, 50}, {10, 57}, {7, 63}, {-2, 77}, {-4, 82}, {-3, 94}, {9, 69}, {-12, 109}, {36, -35},
    {36, -34},
    {32, -26}, {37, -30}, {44, -32}, {34, -18}, {34, -15}, {40, -15}, {33, -7}, {35, -5}, {33, 0}, {38, 2},
    {33, 13}, {23, 35}, {13, 58}, {29, -3}, {26, 0}, {22, 30}, {31, -7}, {35, -15}, {34, -3}, {34, 3},
    {36, -1}, {34, 5}, {32, 11}, {35, 5}, {34, 12}, {39, 11}, {30, 29}, {34, 26}, {29, 39}, {19, 66},
    {31, 21}, {31, 31}, {25, 50},
    {-17, 120}, {-20, 112}, {-18, 114}, {-11, 85}, {-15, 92}, {-14, 89}, {-26, 71}, {-15, 81}, {-14, 80},
    {0, 68}, {-14, 70}, {-24, 56}, {-23, 68}, {-24, 50}, {-11, 74}, {23, -13}, {26, -13}, {40, -15},
    {49, -14}, {44, 3}, {45, 6}, {44, 34}, {33, 54}, {19, 82}, {-3, 75}, {-1, 23}, {1, 34}, {1, 43},
    {0, 54}, {-2, 55}, {0, 61}, {1, 64}, {0, 68}, {-9, 92},
    {-14, 106}, {-13, 97}, {-15, 90}, {-12, 90}, {-18, 88}, {-10, 73}, {-9, 79}, {-14, 86}, {-10, 73},
    {-10, 70}, {-10, 69}, {-5, 66}, {-9, 64}, {-5, 58}, {2, 59}, {21, -10}, {24, -11}, {28, -8}, {28, -1},
    {29, 3}, {29, 9}, {35, 20}, {29, 36}, {14, 67}};

const uint8_t kSig8x8[64] = {0,  1,  2,  3,  4,  5,  5,  4,  4,  3,  3,  4,  4,  4,  5,  5,  4,  4,  4,  4,  3,  3,
                             6,  7,  7,  7,  8,  9,  10, 9,  8,  7,  7,  6,  11, 12, 13, 11, 6,  7,  8,  9,  14, 10,
                             9,  8,  6,  11, 12, 13, 11, 6,  9,  14, 10, 9,  11, 12, 13, 11, 14, 10, 12};
const uint8_t kLast8x8[64] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2,
                              2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4,
                              4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8, 8};
const uint8_t kZz4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
const uint8_t kZz8[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                          41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                          30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
const uint8_t kBlkX[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
const uint8_t kBlkY[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
const uint8_t kBlkOf[4][4] = {{0, 1, 4, 5}, {2, 3, 6, 7}, {8, 9, 12, 13}, {10, 11, 14, 15}};
// field macroblocks (MBAFF): field scans (8.5.6 / 8.5.7, raster index per scan position) and the
// field-coded significant_coeff_flag ctxIdxInc of 8x8 blocks (Table 9-43)
const uint8_t kFld4[16] = {0, 4, 1, 8, 12, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
const uint8_t kFld8[64] = {0,  8,  16, 1,  9,  24, 32, 17, 2,  25, 40, 48, 56, 33, 10, 3,  18, 41, 49, 57, 26, 11,
                           4,  19, 34, 42, 50, 58, 27, 12, 5,  20, 35, 43, 51, 59, 28, 13, 6,  21, 36, 44, 52, 60,
                           29, 14, 22, 37, 45, 53, 61, 30, 7,  15, 38, 46, 54, 62, 23, 31, 39, 47, 55, 63};
const uint8_t kSig8x8Fld[64] = {0, 1,  1,  2,  2,  3,  3,  4,  5,  6,  7,  7,  7,  8,  4,  5,  6,  9,  10, 10, 8,  11,
                                12, 11, 9, 9, 10, 10, 8,  11, 12, 11, 9,  9,  10, 10, 8,  11, 12, 11, 9,  9,  10, 10,
                                8,  13, 13, 9, 9, 10, 10, 8,  13, 13, 9,  9,  10, 10, 14, 14, 14, 14, 14, 0};

const uint8_t kDef4Intra[16] = {6, 13, 13, 20, 20, 20, 28, 28, 28, 28, 32, 32, 32, 37, 37, 42};
const uint8_t kDef4Inter[16] = {10, 14, 14, 20, 20, 20, 24, 24, 24, 24, 27, 27, 27, 30, 30, 34};
const uint8_t kDef8Intra[64] = {6,  10, 10, 13, 11, 13, 16, 16, 16, 16, 18, 18, 18, 18, 18, 23, 23, 23, 23, 23, 23, 25,
                                25, 25, 25, 25, 25, 25, 27, 27, 27, 27, 27, 27, 27, 27, 29, 29, 29, 29, 29, 29, 29, 31,
                                31, 31, 31, 31, 31, 33, 33, 33, 33, 33, 36, 36, 36, 36, 38, 38, 38, 40, 40, 42};
const uint8_t kDef8Inter[64] = {9,  13, 13, 15, 13, 15, 17, 17, 17, 17, 19, 19, 19, 19, 19, 21, 21, 21, 21, 21, 21, 22,
                                22, 22, 22, 22, 22, 22, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 27,
                                27, 27, 27, 27, 27, 28, 28, 28, 28, 28, 30, 30, 30, 30, 32, 32, 32, 33, 33, 35};

struct Sps {
    bool valid = false;
    int profile = 0, chroma_format_idc = 1, bit_depth = 8, bit_depth_c = 8;
    int log2_max_frame_num = 4, poc_type = 0, log2_max_poc_lsb = 4, delta_pic_order_always_zero = 0;
    int mb_w = 0, mb_h = 0;          // frame size in MBs (FrameHeightInMbs: map units x (2 - frame_mbs_only))
    int frame_mbs_only = 1, mbaff = 0;
    int transform_bypass = 0;        // qpprime_y_zero_transform_bypass_flag
    int crop_l = 0, crop_r = 0, crop_t = 0, crop_b = 0;
    int num_reorder_frames = 0;  // VUI bitstream_restriction (0 when absent)
    bool scaling_present = false;
    uint8_t sl4[6][16];
    uint8_t sl8[6][64];
};

// E.1.2 hrd_parameters (skipped); false on cpb_cnt_minus1 > 31, which FFmpeg 4.3 h264_ps.c
// rejects ("cpb_count %d invalid": the VUI and with it the SPS fail)
bool skip_hrd(BitReader& b) {
    const uint32_t cnt = b.ue();
    if (cnt > 31) return false;
    b.u(8);  // bit_rate_scale, cpb_size_scale
    for (uint32_t i = 0; i <= cnt; i++) {
        b.ue();
        b.ue();
        b.u(1);
    }
    b.u(20);  // initial_cpb_removal_delay_length .. time_offset_length (4 x 5 bits)
    return true;
}

// E.1.1 vui_parameters, read as far as max_num_reorder_frames: FFmpeg (h264_slice.c) takes the
// output delay from it when bitstream_restriction_flag is set.  Returns the reorder depth, 0 when
// the VUI carries none or is truncated (FFmpeg then keeps no delay either), -1 where FFmpeg 4.3
// h264_ps.c fails the SPS: an HRD with more than 32 CPBs, or max_num_reorder_frames > 16
// ("Clipping illegal num_reorder_frames", AVERROR_INVALIDDATA).
int parse_vui_reorder(BitReader& b) {
    if (b.u(1) && b.u(8) == 255) b.u(32);  // aspect_ratio_idc, Extended_SAR
    if (b.u(1)) b.u(1);                    // overscan
    if (b.u(1)) {                          // video_signal_type
        b.u(4);
        if (b.u(1)) b.u(24);
    }
    if (b.u(1)) {  // chroma_loc_info
        b.ue();
        b.ue();
    }
    if (b.u(1)) b.u(32), b.u(32), b.u(1);  // timing_info
    const bool nal = b.u(1) != 0;
    if (nal && !skip_hrd(b)) return -1;
    const bool vcl = b.u(1) != 0;
    if (vcl && !skip_hrd(b)) return -1;
    if (nal || vcl) b.u(1);  // low_delay_hrd_flag
    b.u(1);                  // pic_struct_present_flag
    if (!b.u(1)) return 0;   // bitstream_restriction_flag
    b.u(1);
    b.ue();
    b.ue();
    b.ue();
    b.ue();
    const uint32_t reorder = b.ue();
    b.ue();  // max_dec_frame_buffering
    if (b.overrun()) return 0;
    return reorder > 16 ? -1 : static_cast<int>(reorder);
}

struct Pps {
    bool valid = false;
    int sps_id = 0, cabac = 0, bottom_field_pic_order = 0, init_qp = 26, cqp = 0, cqp2 = 0;
    int deblock_ctrl = 0, redundant_pic_cnt = 0, transform_8x8 = 0, scaling_present = 0;
    uint8_t sl4[6][16];
    uint8_t sl8[6][64];
};

void parse_sl(BitReader& b, uint8_t* list, int n, const uint8_t* def, const uint8_t* fallback, bool present) {
    if (!present) {
        std::memcpy(list, fallback, static_cast<size_t>(n));
        return;
    }
    int last = 8, next = 8;
    for (int j = 0; j < n; j++) {
        if (next != 0) {
            next = (last + b.se() + 256) % 256;
            if (j == 0 && next == 0) {
                std::memcpy(list, def, static_cast<size_t>(n));
                return;
            }
        }
        list[j] = static_cast<uint8_t>(next == 0 ? last : next);
        last = list[j];
    }
}

void parse_matrices(BitReader& b, uint8_t sl4[6][16], uint8_t sl8[6][64], int n8, const uint8_t fb4[6][16],
                    const uint8_t fb8[6][64], bool fallback_default) {
    for (int i = 0; i < 6; i++) {
        bool pres = b.u(1) != 0;
        const uint8_t* def = i < 3 ? kDef4Intra : kDef4Inter;
        const uint8_t* fb = (i == 0 || i == 3) ? (fallback_default ? def : fb4[i]) : sl4[i - 1];
        parse_sl(b, sl4[i], 16, def, fb, pres);
    }
    for (int i = 0; i < n8; i++) {
        bool pres = b.u(1) != 0;
        const uint8_t* def = (i % 2 == 0) ? kDef8Intra : kDef8Inter;
        const uint8_t* fb = i < 2 ? (fallback_default ? def : fb8[i]) : sl8[i - 2];
        parse_sl(b, sl8[i], 64, def, fb, pres);
    }
}

int parse_sps(BitReader& b, Sps* tab) {
    const int profile = static_cast<int>(b.u(8));
    b.u(8);
    b.u(8);
    const uint32_t id = b.ue();
    if (id > 31) return -1;
    Sps& s = tab[id];
    s = Sps();
    s.profile = profile;
    for (int i = 0; i < 6; i++) {
        std::memset(s.sl4[i], 16, 16);
        std::memset(s.sl8[i], 16, 64);
    }
    if (profile == 100 || profile == 110 || profile == 122 || profile == 244 || profile == 44 || profile == 83 ||
        profile == 86 || profile == 118 || profile == 128 || profile == 138 || profile == 139 || profile == 134 ||
        profile == 135) {
        s.chroma_format_idc = static_cast<int>(b.ue());
        if (s.chroma_format_idc == 3) b.u(1);
        s.bit_depth = static_cast<int>(b.ue()) + 8;
        s.bit_depth_c = static_cast<int>(b.ue()) + 8;
        s.transform_bypass = static_cast<int>(b.u(1));  // qpprime_y_zero_transform_bypass_flag
        s.scaling_present = b.u(1) != 0;
        if (s.scaling_present) {
            uint8_t fb4[6][16], fb8[6][64];
            parse_matrices(b, s.sl4, s.sl8, s.chroma_format_idc != 3 ? 2 : 6, fb4, fb8, true);
        }
    }
    // ranges of 7.4.2.1.1 (FFmpeg h264_ps.c rejects the SPS outside them)
    const uint32_t lfn = b.ue();
    if (lfn > 12) return -1;
    s.log2_max_frame_num = static_cast<int>(lfn) + 4;
    const uint32_t poc_type = b.ue();
    if (poc_type > 2) return -1;
    s.poc_type = static_cast<int>(poc_type);
    if (s.poc_type == 0) {
        const uint32_t lpl = b.ue();
        if (lpl > 12) return -1;
        s.log2_max_poc_lsb = static_cast<int>(lpl) + 4;
    } else if (s.poc_type == 1) {
        s.delta_pic_order_always_zero = static_cast<int>(b.u(1));
        b.se();
        b.se();
        const uint32_t n = b.ue();
        if (n > 255) return -1;
        for (uint32_t i = 0; i < n; i++) b.se();
    }
    b.ue();
    b.u(1);
    const uint32_t mbw1 = b.ue(), mbh1 = b.ue();
    if (mbw1 >= 512 || mbh1 >= 512) return -5;
    s.frame_mbs_only = static_cast<int>(b.u(1));
    if (!s.frame_mbs_only) s.mbaff = static_cast<int>(b.u(1));  // mb_adaptive_frame_field_flag
    s.mb_w = static_cast<int>(mbw1) + 1;
    s.mb_h = (static_cast<int>(mbh1) + 1) * (2 - s.frame_mbs_only);  // 7.4.2.1.1 FrameHeightInMbs
    b.u(1);
    if (b.u(1)) {
        // frame cropping in CropUnitX = 2 / CropUnitY = 2 * (2 - frame_mbs_only) sample units
        // (4:2:0, 7.4.2.1.1; 4:0:0: 1 and 2 - frame_mbs_only).  FFmpeg 4.3 h264_ps.c
        // (libavcodec 58.x, the reference's decoder) rejects the SPS ("crop values invalid",
        // goto fail) when an offset exceeds INT_MAX / 4 / step or the window leaves no
        // picture, so no frame is decoded; only its HEVC SPS parser ignores such a window.
        const uint32_t cl = b.ue(), cr = b.ue(), ct = b.ue(), cb = b.ue();
        const uint64_t w = static_cast<uint64_t>(s.mb_w) * 16, h = static_cast<uint64_t>(s.mb_h) * 16;
        const uint32_t ux = s.chroma_format_idc == 0 ? 1u : 2u;
        const uint32_t uy = (s.chroma_format_idc == 0 ? 1u : 2u) * (2u - static_cast<uint32_t>(s.frame_mbs_only));
        const uint32_t lim = 0x7fffffffu / 4 / ux, limy = 0x7fffffffu / 4 / uy;
        if (cl > lim || cr > lim || ct > limy || cb > limy || (static_cast<uint64_t>(cl) + cr) * ux >= w ||
            (static_cast<uint64_t>(ct) + cb) * uy >= h)
            return -6;
        s.crop_l = static_cast<int>(cl * ux);
        s.crop_r = static_cast<int>(cr * ux);
        s.crop_t = static_cast<int>(ct * uy);
        s.crop_b = static_cast<int>(cb * uy);
    }
    if (b.overrun()) return -1;
    if (b.u(1)) {
        s.num_reorder_frames = parse_vui_reorder(b);
        if (s.num_reorder_frames < 0) return -1;
    }
    // FFmpeg 4.3 decodes 4:2:0 and 4:0:0 (into yuv420p) at 8, 9, 10, 12 and 14 bits with equal
    // luma / chroma depths (h264_ps.c "Different chroma and luma bit depth"; h264_slice.c
    // get_pixel_format has no 11- or 13-bit format, "Unsupported bit depth")
    if ((s.chroma_format_idc != 1 && s.chroma_format_idc != 0) || s.bit_depth_c != s.bit_depth || s.bit_depth > 14 ||
        s.bit_depth == 11 || s.bit_depth == 13)
        return -4;
    s.valid = true;
    return 0;
}

int parse_pps(BitReader& b, Pps* tab, const Sps* sps) {
    const uint32_t id = b.ue();
    if (id > 255) return -1;
    Pps& p = tab[id];
    p = Pps();
    p.sps_id = static_cast<int>(b.ue());
    if (p.sps_id > 31) return -1;
    p.cabac = static_cast<int>(b.u(1));
    p.bottom_field_pic_order = static_cast<int>(b.u(1));
    if (b.ue() != 0) return -2;  // FMO
    b.ue();
    b.ue();
    b.u(1);
    b.u(2);
    p.init_qp = 26 + b.se();
    b.se();
    p.cqp = b.se();
    if (p.cqp < -12 || p.cqp > 12) return -1;
    p.deblock_ctrl = static_cast<int>(b.u(1));
    b.u(1);
    p.redundant_pic_cnt = static_cast<int>(b.u(1));
    p.cqp2 = p.cqp;
    const Sps& s = sps[p.sps_id];
    std::memcpy(p.sl4, s.sl4, sizeof(p.sl4));
    std::memcpy(p.sl8, s.sl8, sizeof(p.sl8));
    if (b.more_rbsp_data()) {
        p.transform_8x8 = static_cast<int>(b.u(1));
        p.scaling_present = static_cast<int>(b.u(1));
        if (p.scaling_present) {
            uint8_t fb4[6][16], fb8[6][64];
            std::memcpy(fb4, s.sl4, sizeof(fb4));
            std::memcpy(fb8, s.sl8, sizeof(fb8));
            parse_matrices(b, p.sl4, p.sl8, p.transform_8x8 ? 2 : 0, fb4, fb8, !s.scaling_present);
        }
        p.cqp2 = b.se();
        if (p.cqp2 < -12 || p.cqp2 > 12) return -1;
    }
    p.valid = true;
    return 0;
}

struct Mb {
    int slice = -1;
    int mb_type = 0;  // 0 NxN, 1..24 I16x16, 25 PCM
    int t8x8 = 0;
    int cbp = 0;
    int qp = 0;
    int cpm = 0;
    uint8_t ipm[16];
    uint8_t cbf[16];
    uint8_t cbf_c[2][4];
    uint8_t cbf_dc[3];
    uint8_t tc[16];     // CAVLC TotalCoeff per luma 4x4 block (I16x16: AC block)
    uint8_t tcc[2][4];  // CAVLC TotalCoeff per chroma AC block
    int field = 0;      // MBAFF: mb_field_decoding_flag of the pair
    int vx = 0, vy = 0; // grid position (MBAFF: vy = 2 * pair row + bottom)
};

// MSB-first reader over one slice's RBSP for CAVLC: 64-bit window, peek/skip.
class VlcBits {
public:
    void init(const uint8_t* p, size_t n, size_t bitpos) {
        p_ = p;
        n_ = n;
        pos_ = bitpos;
    }
    inline uint32_t peek32() const {
        const size_t byte = pos_ >> 3;
        uint64_t w = 0;
        if (byte + 8 <= n_) {
            for (int i = 0; i < 8; i++) w = (w << 8) | p_[byte + i];
        } else {
            for (int i = 0; i < 8; i++) w = (w << 8) | (byte + i < n_ ? p_[byte + i] : 0u);
        }
        return static_cast<uint32_t>((w << (pos_ & 7)) >> 32);
    }
    inline void skip(int n) { pos_ += static_cast<size_t>(n); }
    inline uint32_t u(int n) {
        if (!n) return 0;
        const uint32_t v = peek32() >> (32 - n);
        pos_ += static_cast<size_t>(n);
        return v;
    }
    inline uint32_t ue() {
        const uint32_t w = peek32();
        if (!w) { pos_ = n_ * 8 + 1; return 0; }
        const int lz = __builtin_clz(w);
        if (lz > 15) {  // long code: two steps
            pos_ += static_cast<size_t>(lz + 1);
            return ((1u << lz) - 1u) + u(lz);
        }
        pos_ += static_cast<size_t>(2 * lz + 1);
        return (w >> (31 - 2 * lz)) - 1u;
    }
    inline int32_t se() {
        const uint32_t k = ue();
        return (k & 1) ? static_cast<int32_t>((k + 1) >> 1) : -static_cast<int32_t>(k >> 1);
    }
    void align() { pos_ = (pos_ + 7) & ~static_cast<size_t>(7); }
    size_t pos() const { return pos_; }
    size_t byte_pos() const { return pos_ >> 3; }
    bool overrun() const { return pos_ > n_ * 8; }
    // more_rbsp_data(): anything before the rbsp_stop_one_bit
    bool more_rbsp_data(size_t stop_bit) const { return pos_ < stop_bit; }

private:
    const uint8_t* p_ = nullptr;
    size_t n_ = 0;
    size_t pos_ = 0;
};

// Direct-lookup decoders for the CAVLC VLC tables (built once).
struct CavlcLut {
    // coeff_token: [nC class 0..3][16-bit prefix] -> (len << 10) | (t1 << 5) | tc, 0 = invalid
    std::vector<uint16_t> ct[4];
    uint8_t tz[15][512];    // total_zeros: (len << 4) | value, 9-bit prefix
    uint8_t tzdc[3][8];     // chroma DC total_zeros, 3-bit prefix
    uint8_t rb[7][2048];    // run_before: (len << 4) | run, 11-bit prefix
    CavlcLut() {
        for (int col = 0; col < 4; col++) {
            ct[col].assign(65536, 0);
            for (int t1 = 0; t1 < 4; t1++)
                for (int tc = 0; tc <= 16; tc++) {
                    const int len = kCoeffTokenLen[col][t1][tc];
                    if (!len) continue;
                    const uint32_t base = static_cast<uint32_t>(kCoeffTokenCode[col][t1][tc]) << (16 - len);
                    for (uint32_t k = 0; k < (1u << (16 - len)); k++)
                        ct[col][base + k] = static_cast<uint16_t>((len << 10) | (t1 << 5) | tc);
                }
        }
        std::memset(tz, 0, sizeof(tz));
        for (int t = 0; t < 15; t++)
            for (int z = 0; z < 16; z++) {
                const int len = kTotalZerosLen[t][z];
                if (!len) continue;
                const uint32_t base = static_cast<uint32_t>(kTotalZerosCode[t][z]) << (9 - len);
                for (uint32_t k = 0; k < (1u << (9 - len)); k++) tz[t][base + k] = static_cast<uint8_t>((len << 4) | z);
            }
        std::memset(tzdc, 0, sizeof(tzdc));
        for (int t = 0; t < 3; t++)
            for (int z = 0; z < 4; z++) {
                const int len = kTotalZerosDcLen[t][z];
                if (!len) continue;
                const uint32_t base = static_cast<uint32_t>(kTotalZerosDcCode[t][z]) << (3 - len);
                for (uint32_t k = 0; k < (1u << (3 - len)); k++) tzdc[t][base + k] = static_cast<uint8_t>((len << 4) | z);
            }
        std::memset(rb, 0, sizeof(rb));
        for (int z = 0; z < 7; z++)
            for (int r = 0; r < 15; r++) {
                const int len = kRunBeforeLen[z][r];
                if (!len) continue;
                const uint32_t base = static_cast<uint32_t>(kRunBeforeCode[z][r]) << (11 - len);
                for (uint32_t k = 0; k < (1u << (11 - len)); k++) rb[z][base + k] = static_cast<uint8_t>((len << 4) | r);
            }
    }
};

const CavlcLut& cavlc_lut() {
    static const CavlcLut lut;  // C++11 thread-safe initialisation
    return lut;
}

// slice data kept for the decode pass (after all slice headers of the picture are read)
struct SliceWork {
    bool cabac = true;
    std::vector<uint8_t> data;  // CABAC: bytes after the header (+8 zero bytes); CAVLC: the whole RBSP
    size_t nbytes = 0;          // valid bytes of data
    size_t bitpos = 0;          // CAVLC: first bit of the slice data
    size_t stop_bit = 0;        // CAVLC: position of the rbsp_stop_one_bit
    int qp = 0, first_mb = 0, index = 0, pps_id = 0;
    int parity = 0;  // PAFF: bottom_field_flag
};

class H264Parser {
public:
    explicit H264Parser(FrameJob& job) : job_(&job) {}
    // a worker for other slices of the same picture: picture state copied, its own outputs
    H264Parser(const H264Parser& proto, FrameJob& job) : H264Parser(proto) { job_ = &job; }
    int run(const uint8_t* data, size_t size, int threads);

private:
    H264Parser(const H264Parser&) = default;
    int decode_slice(const SliceWork& w);
    template <bool AFF>
    int mb_loop_cabac(int addr, int nmb);
    template <bool AFF>
    int mb_loop_cavlc(int addr, int nmb);
    FrameJob* job_;
    Sps sps_[32];
    Pps pps_[256];
    const Sps* s_ = nullptr;
    const Pps* p_ = nullptr;
    std::vector<uint8_t> rbsp_;
    std::vector<Mb> mb_;
    int mbw_ = 0, mbh_ = 0, mbx_ = 0, mby_ = 0, qpbd_ = 0;
    int mbaff_ = 0, cur_field_ = 0;  // MbaffFrameFlag; mb_field_decoding_flag of the current pair
    // PAFF field pair: held in the MBAFF layout as all-field pairs (field MB (x, fy) of parity f at
    // grid (x, 2 fy + f)); parity_ = bottom_field_flag of the slice being decoded
    int paff_ = 0, parity_ = 0;
    // 4:0:0: no chroma syntax; chroma TBs are DC predicted without residual (every chroma sample
    // 1 << (BitDepth - 1), as FFmpeg's DC_128_PRED8x8) and I_PCM chroma is that value
    bool mono_ = false;
    int qp_ = 0, prev_qpd_nz_ = 0, cur_slice_ = 0;
    CabacOutlineRefill cc_;
    const uint8_t* end_ = nullptr;
    CabacState ctx_[460];
    int err_ = 0;

    VlcBits vb_;  // CAVLC slice data
    size_t stop_bit_ = 0;
    int dec(int c) { return cc_.decision(ctx_[c]); }
    // CAVLC (7.3.5.3.2 / 9.2)
    int cavlc_block(int nC, int maxnum, uint8_t* pos, int* lvl);
    // AFF: MbaffFrameFlag (MBAFF frames and PAFF field pairs); the macroblock layer is compiled
    // once per value so progressive pictures run no interlace tests
    template <bool AFF>
    int nc_luma(int blk);
    template <bool AFF>
    int nc_chroma(const Mb& m, int c, int b4);
    template <bool AFF>
    void decode_mb_cavlc();
    __attribute__((always_inline)) Mb* mb_in_slice(int x, int y) {
        if (x < 0 || y < 0 || x >= mbw_ || y >= mbh_) return nullptr;
        Mb* m = &mb_[y * mbw_ + x];
        return m->slice == cur_slice_ ? m : nullptr;
    }
    // 6.4.12 (see nb_loc_mbaff): frames and PAFF field pairs inline (every neighbour query of a
    // macroblock goes through here: out of line it cost ~9 % of the progressive parse), MBAFF out
    // of line
    template <bool AFF>
    __attribute__((always_inline)) Mb* nb_loc(int xN, int yN, int maxW, int maxH, int* xW, int* yW) {
        if (AFF && mbaff_ && !paff_) return nb_loc_mbaff(xN, yN, maxW, maxH, xW, yW);
        if (yN > maxH - 1 || (xN > maxW - 1 && yN >= 0)) return nullptr;
        *xW = (xN + maxW) & (maxW - 1);  // maxW, maxH: 8 or 16; xN, yN >= -1
        *yW = (yN + maxH) & (maxH - 1);
        if (xN >= 0 && xN <= maxW - 1 && yN >= 0) return &mb_[mby_ * mbw_ + mbx_];
        return mb_in_slice(mbx_ + (xN < 0 ? -1 : (xN > maxW - 1 ? 1 : 0)), mby_ + (yN < 0 ? (AFF && paff_ ? -2 : -1) : 0));
    }
    __attribute__((noinline)) Mb* nb_loc_mbaff(int xN, int yN, int maxW, int maxH, int* xW, int* yW);
    // MB covering luma location (-1, 0) / (0, -1) / (16, -1) / (-1, -1) (6.4.11.1)
    template <bool AFF>
    __attribute__((always_inline)) Mb* nb(int dx, int dy) {
        int xW, yW;
        return nb_loc<AFF>(dx < 0 ? -1 : (dx > 0 ? 16 : 0), dy < 0 ? -1 : 0, 16, 16, &xW, &yW);
    }
    // the 4x4 luma block covering location (4 bx, 4 by) relative to the MB (6.4.11.4)
    template <bool AFF>
    __attribute__((always_inline)) Mb* nb_blk(int bx, int by, int* nblk) {
        int xW, yW;
        Mb* m = nb_loc<AFF>(bx * 4, by * 4, 16, 16, &xW, &yW);
        *nblk = m ? kBlkOf[yW >> 2][xW >> 2] : 0;
        return m;
    }
    // availability of the sample at luma location (x, y) relative to the MB for intra prediction
    // (inside the MB: earlier in 4x4 block order)
    bool avail_luma(int x, int y, int cur_blk4) {
        int xW, yW;
        if (x >= 16 && y >= 0) return false;
        if (x < 0 || y < 0 || x >= 16) return nb_loc<true>(x, y, 16, 16, &xW, &yW) != nullptr;
        return kBlkOf[y >> 2][x >> 2] < cur_blk4;
    }
    uint8_t mbaff_mask(int xr, int yr, int log2n, int c) {
        const int n = 1 << log2n;
        if (c > 0 || log2n == 4)  // I16x16 / chroma: the MB's neighbours (top, left, top-left)
            return static_cast<uint8_t>((nb<true>(0, -1) ? 1 : 0) | (nb<true>(-1, 0) ? 2 : 0) | (nb<true>(-1, -1) ? 4 : 0));
        const int blk = kBlkOf[yr >> 2][xr >> 2];
        return static_cast<uint8_t>((avail_luma(xr, yr - 1, blk) ? 1 : 0) | (avail_luma(xr - 1, yr, blk) ? 2 : 0) |
                                    (avail_luma(xr - 1, yr - 1, blk) ? 4 : 0) | (avail_luma(xr + n, yr - 1, blk) ? 8 : 0));
    }
    template <bool AFF>
    void mb_start(int addr, bool cabac);
    int cbf_cond(int cat, const Mb* N, int nblk, int icbcr) const;
    // residual_block_cabac (7.3.5.3.3): number of non-zero levels (0: coded_block_flag 0);
    // scan indices in pos[], levels in lvl[]
    // FLD: field macroblock (MBAFF / PAFF) context sets; a compile-time choice, so the frame
    // decoder keeps constant context offsets in its bin loops (r04r: the runtime choice cost the
    // progressive parse ~12 % on the box CPU)
    template <bool FLD>
    int residual_block_t(int cat, int cbf_inc, int max_num, uint8_t* pos, int* lvl);
    template <bool AFF>
    int residual_block(int cat, int cbf_inc, int max_num, uint8_t* pos, int* lvl) {
        return AFF && mb_[mby_ * mbw_ + mbx_].field ? residual_block_t<true>(cat, cbf_inc, max_num, pos, lvl)
                                             : residual_block_t<false>(cat, cbf_inc, max_num, pos, lvl);
    }
    template <bool AFF>
    void decode_mb();
    void emit(int x, int y, int log2n, int c, int mode, uint8_t flags, int qp, const int* lv, int npos, bool pcm);
    // sparse record: entries already (pos << 16) | uint16 level
    template <bool AFF>
    void emit_sparse(int x, int y, int log2n, int c, int mode, int qp, const uint32_t* e, int n);
};

// 6.4.12: the MB covering location (xN, yN) relative to the current MB (maxW x maxH: 16 x 16 luma,
// 8 x 8 chroma) and the location (xW, yW) inside it, nullptr when not available.  Non-MBAFF:
// 6.4.12.1.  MBAFF: 6.4.12.2 (pairs A / B / C / D, Table 6-4); a bottom frame MB's upper-left
// neighbour next to a field pair is that pair's bottom field MB, middle row (the picture sample
// above-left: FFmpeg h264_slice.c fill_decode_neighbors, topleft_xy += mb_stride).  Every
// neighbour sample is then the picture sample next to the MB in its own field / frame view.
Mb* H264Parser::nb_loc_mbaff(int xN, int yN, int maxW, int maxH, int* xW, int* yW) {
    Mb* cur = &mb_[mby_ * mbw_ + mbx_];
    if (yN > maxH - 1 || (xN > maxW - 1 && yN >= 0)) return nullptr;
    *xW = (xN + maxW) % maxW;
    if (xN >= 0 && xN <= maxW - 1 && yN >= 0) {
        *yW = yN;
        return cur;
    }
    if (!mbaff_ || paff_) {  // PAFF: 6.4.12.1 on the field's own MB grid
        *yW = (yN + maxH) % maxH;
        return mb_in_slice(mbx_ + (xN < 0 ? -1 : (xN > maxW - 1 ? 1 : 0)), mby_ + (yN < 0 ? (paff_ ? -2 : -1) : 0));
    }
    const int px = mbx_, py = mby_ >> 1;
    const bool top = !(mby_ & 1), frame = !cur->field;
    Mb* X = nullptr;
    int yM = yN, bot = 0;
    if (xN < 0 && yN < 0) {
        if (frame && !top) {
            X = mb_in_slice(px - 1, 2 * py);
            if (!X) return nullptr;
            bot = X->field;
            yM = X->field ? (yN + maxH) >> 1 : yN;
        } else if (frame || !top) {
            X = mb_in_slice(px - 1, 2 * py - 2);
            bot = 1;
        } else {
            X = mb_in_slice(px - 1, 2 * py - 2);
            if (!X) return nullptr;
            if (!X->field) { bot = 1; yM = 2 * yN; }
        }
    } else if (xN < 0) {
        X = mb_in_slice(px - 1, 2 * py);
        if (!X) return nullptr;
        if (frame) {
            if (!X->field) bot = top ? 0 : 1;
            else { bot = yN & 1; yM = top ? yN >> 1 : (yN + maxH) >> 1; }
        } else if (!X->field) {
            const int o = top ? 0 : 1;
            if (yN < maxH / 2) { bot = 0; yM = (yN << 1) + o; }
            else { bot = 1; yM = (yN << 1) + o - maxH; }
        } else {
            bot = top ? 0 : 1;
        }
    } else if (xN <= maxW - 1) {
        if (frame && !top) {
            X = &mb_[(2 * py) * mbw_ + px];  // CurrMbAddr - 1
        } else if (frame || !top) {
            X = mb_in_slice(px, 2 * py - 2);
            bot = 1;
        } else {
            X = mb_in_slice(px, 2 * py - 2);
            if (!X) return nullptr;
            if (!X->field) { bot = 1; yM = 2 * yN; }
        }
    } else {
        if (frame && !top) return nullptr;
        X = mb_in_slice(px + 1, 2 * py - 2);
        if (!X) return nullptr;
        if (frame || !top) bot = 1;
        else if (!X->field) { bot = 1; yM = 2 * yN; }
    }
    if (!X) return nullptr;
    *yW = (yM + maxH) % maxH;
    return &mb_[(X->vy + bot) * mbw_ + X->vx];
}

// position the parser on macroblock address `addr` (MBAFF: pair addr / 2, bottom addr & 1) and,
// at the top MB of an MBAFF pair, read mb_field_decoding_flag (7.3.4; CABAC ctxIdx 70 + the left /
// upper pair being available field pairs, 9.3.3.1.1.2; CAVLC u(1))
template <bool AFF>
void H264Parser::mb_start(int addr, bool cabac) {
    if (AFF && paff_) {  // field MB address of the current field
        mbx_ = addr % mbw_;
        mby_ = 2 * (addr / mbw_) + parity_;
        mb_[mby_ * mbw_ + mbx_].slice = cur_slice_;
        cur_field_ = 1;
        return;
    }
    if (!AFF || !mbaff_) {
        mbx_ = addr % mbw_;
        mby_ = addr / mbw_;
        return;
    }
    const int pair = addr >> 1;
    mbx_ = pair % mbw_;
    mby_ = 2 * (pair / mbw_) + (addr & 1);
    mb_[mby_ * mbw_ + mbx_].slice = cur_slice_;
    if (!(addr & 1)) {
        Mb* A = mb_in_slice(mbx_ - 1, mby_);
        Mb* B = mb_in_slice(mbx_, mby_ - 2);
        cur_field_ = cabac ? dec(70 + (A && A->field) + (B && B->field)) : static_cast<int>(vb_.u(1));
    }
}

int H264Parser::cbf_cond(int cat, const Mb* N, int nblk, int icbcr) const {
    if (!N) return 1;
    if (N->mb_type == 25) return 1;
    switch (cat) {
    case 0: return (N->mb_type >= 1 && N->mb_type <= 24) ? N->cbf_dc[0] : 0;
    case 1:
    case 2: return ((N->cbp >> (nblk >> 2)) & 1) ? N->cbf[nblk] : 0;
    case 3: return (N->cbp >> 4) ? N->cbf_dc[1 + icbcr] : 0;
    case 4: return (N->cbp >> 4) == 2 ? N->cbf_c[icbcr][nblk] : 0;
    }
    return 0;
}

template <bool FLD>
int H264Parser::residual_block_t(int cat, int cbf_inc, int max_num, uint8_t* pos, int* lvl) {
    static const int kCbfOff[5] = {0, 4, 8, 12, 16};
    static const int kSigOff[6] = {0, 15, 29, 44, 47, 0};
    static const int kAbsOff[6] = {0, 10, 20, 30, 39, 0};
    CabacOutlineRefill cc = cc_;  // engine state in registers for the block
    CabacState* const ctx = ctx_;
    if (cat != 5 && !cc.decision(ctx[85 + kCbfOff[cat] + cbf_inc])) {
        cc_ = cc;
        return 0;
    }
    int nsig = 0;
    bool last_found = false;
    // field macroblocks (MBAFF): significance / last contexts at 277 / 338 (436 / 451 with the
    // field ctxIdxInc table for 8x8 blocks) instead of 105 / 166 (402 / 417), 9.3.3.1.3
    constexpr int sig0 = FLD ? 277 : 105, last0 = FLD ? 338 : 166;
    if (cat == 5) {
        const uint8_t* const sigt = FLD ? kSig8x8Fld : kSig8x8;
        constexpr int s8 = FLD ? 436 : 402, l8 = FLD ? 451 : 417;
        for (int i = 0; i < max_num - 1; i++)
            if (cc.decision(ctx[s8 + sigt[i]])) {
                pos[nsig++] = static_cast<uint8_t>(i);
                if (cc.decision(ctx[l8 + kLast8x8[i]])) { last_found = true; break; }
            }
    } else if (cat == 3) {
        for (int i = 0; i < max_num - 1; i++) {
            const int inc = i < 2 ? i : 2;
            if (cc.decision(ctx[sig0 + kSigOff[3] + inc])) {
                pos[nsig++] = static_cast<uint8_t>(i);
                if (cc.decision(ctx[last0 + kSigOff[3] + inc])) { last_found = true; break; }
            }
        }
    } else {
        CabacState* const sctx = ctx + sig0 + kSigOff[cat];
        CabacState* const lctx = ctx + last0 + kSigOff[cat];
        for (int i = 0; i < max_num - 1; i++)
            if (cc.decision(sctx[i])) {
                pos[nsig++] = static_cast<uint8_t>(i);
                if (cc.decision(lctx[i])) { last_found = true; break; }
            }
    }
    if (!last_found) pos[nsig++] = static_cast<uint8_t>(max_num - 1);
    int eq1 = 0, gt1 = 0;
    CabacState* const absc = ctx + (cat == 5 ? 426 : 227 + kAbsOff[cat]);
    const int gt_cap = 4 - (cat == 3 ? 1 : 0);
    for (int k = nsig - 1; k >= 0; k--) {
        const int inc = gt1 ? 0 : std::min(4, 1 + eq1);
        int v;
        if (!cc.decision(absc[inc])) {
            v = 1;
            eq1++;
        } else {
            CabacState& c2 = absc[5 + std::min(gt_cap, gt1)];
            int p = 1;
            while (p < 14 && cc.decision(c2)) p++;
            v = p + 1;
            if (p == 14) {
                int kk = 0;
                while (cc.bypass()) {
                    v += 1 << kk;
                    if (++kk > 24) { err_ = -30; cc_ = cc; return nsig; }
                }
                while (kk--) v += cc.bypass() << kk;
            }
            gt1++;
        }
        lvl[k] = cc.bypass() ? -v : v;
    }
    cc_ = cc;
    return nsig;
}

template <bool AFF>
void H264Parser::emit_sparse(int x, int y, int log2n, int c, int mode, int qp, const uint32_t* e, int n) {
    // built in place (a local record copied in would wait on store-to-load forwarding of its fields)
    job_->tus.emplace_back();
    h2j_tu& t = job_->tus.back();
    t.x = static_cast<uint16_t>(x);
    t.y = static_cast<uint16_t>(y);
    t.log2n = static_cast<uint8_t>(log2n);
    t.c = static_cast<uint8_t>(c);
    t.mode = static_cast<uint8_t>(mode);
    t.qp = static_cast<int8_t>(qp);
    t.qpy = static_cast<int8_t>(qp_);
    // MBAFF: the reference-availability mask (bits top, left, top-left, top-right) from the 6.4.12.2
    // neighbours, in qpy (H.264 TBs do not use it otherwise); K0 copies it to the mask array
    if (AFF && mbaff_) t.qpy = static_cast<int8_t>(mbaff_mask(x - mbx_ * (c ? 8 : 16), y - mby_ * (c ? 8 : 16), log2n, c));
    t.coef = static_cast<uint32_t>(job_->coefs.size());
    job_->coefs.insert(job_->coefs.end(), e, e + n);
    t.ncoef = static_cast<uint16_t>(n);
    t.flags = n ? H2J_TU_CBF : 0;
    // TransformBypassModeFlag (qpprime_y_zero_transform_bypass_flag and QP'Y 0, 8.5.12 / 8.5.15):
    // the residual is the levels; FFmpeg (h264_mb.c) accumulates it along vertical / horizontal
    // intra predictions only for profile_idc 244.  Luma NxN and 16x16 modes: 0 vertical,
    // 1 horizontal; chroma: 1 horizontal, 2 vertical.
    if (s_->transform_bypass && qp_ + qpbd_ == 0) {
        t.flags |= H2J_TU_BYPASS;
        if (s_->profile == 244) {
            const bool v = c == 0 ? mode == 0 : mode == 2, h = c == 0 ? mode == 1 : mode == 1;
            if (v) t.flags |= H2J_TU_DPCM_V;
            if (h) t.flags |= H2J_TU_DPCM_H;
        }
    }
}

void H264Parser::emit(int x, int y, int log2n, int c, int mode, uint8_t flags, int qp, const int* lv, int npos,
                      bool pcm) {
    job_->tus.emplace_back();
    h2j_tu& t = job_->tus.back();
    t.x = static_cast<uint16_t>(x);
    t.y = static_cast<uint16_t>(y);
    t.log2n = static_cast<uint8_t>(log2n);
    t.c = static_cast<uint8_t>(c);
    t.mode = static_cast<uint8_t>(mode);
    t.qp = static_cast<int8_t>(qp);
    t.qpy = static_cast<int8_t>(qp_);
    t.coef = static_cast<uint32_t>(job_->coefs.size());
    for (int i = 0; i < npos; i++)
        if (lv[i] || pcm) job_->coefs.push_back((static_cast<uint32_t>(i) << 16) | static_cast<uint16_t>(lv[i]));
    t.ncoef = static_cast<uint16_t>(job_->coefs.size() - t.coef);
    t.flags = flags | (t.ncoef ? H2J_TU_CBF : 0);
}

int chroma_qp_264(int qpi) {
    static const int t[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
    return qpi < 30 ? qpi : t[qpi - 30];
}

template <bool AFF>
void H264Parser::decode_mb() {
    Mb& m = mb_[mby_ * mbw_ + mbx_];
    m = Mb();
    m.slice = cur_slice_;
    const int gx = mbx_ * 16, gy = mby_ * 16;
    h2j_ctb& rec = job_->ctbs[mby_ * mbw_ + mbx_];
    rec.slice = static_cast<uint8_t>(cur_slice_);
    m.vx = mbx_;
    m.vy = mby_;
    m.field = AFF && mbaff_ ? cur_field_ : 0;
    rec.mbflags = static_cast<uint8_t>(4 | (m.field ? 8 : 0));  // bit 3: MBAFF field macroblock
    // mb_type (I slice)
    {
        Mb* A = nb<AFF>(-1, 0);
        Mb* B = nb<AFF>(0, -1);
        const int ctx = (A && A->mb_type != 0) + (B && B->mb_type != 0);
        if (!dec(3 + ctx)) {
            m.mb_type = 0;
        } else if (cc_.terminate()) {
            m.mb_type = 25;
        } else {
            int t = 1 + 12 * dec(6);
            if (dec(7)) t += 4 + 4 * dec(8);
            t += 2 * dec(9);
            t += dec(10);
            m.mb_type = t;
        }
    }
    if (m.mb_type == 25) {
        const uint8_t* p = cc_.aligned_pos();
        BitReader b(p, static_cast<size_t>(end_ - p));
        int lv[256];
        for (int i = 0; i < 256; i++) lv[i] = static_cast<int>(b.u(s_->bit_depth));
        emit(gx, gy, 4, 0, 0, H2J_TU_PCM, 0, lv, 256, true);
        for (int c = 1; c < 3; c++) {
            for (int i = 0; i < 64; i++) lv[i] = mono_ ? 1 << (s_->bit_depth - 1) : static_cast<int>(b.u(s_->bit_depth_c));
            emit(gx / 2, gy / 2, 3, c, 0, H2J_TU_PCM, 0, lv, 64, true);
        }
        cc_.init(p + b.byte_pos(), end_);
        m.qp = qp_;
        m.cbp = 0x2F;
        std::memset(m.cbf, 1, sizeof(m.cbf));
        std::memset(m.cbf_c, 1, sizeof(m.cbf_c));
        std::memset(m.cbf_dc, 1, sizeof(m.cbf_dc));
        for (int i = 0; i < 16; i++) m.ipm[i] = 2;
        prev_qpd_nz_ = 0;
        rec.qp = static_cast<int8_t>(qp_);
        rec.mbflags |= 1;
        return;
    }
    const bool is16 = m.mb_type >= 1 && m.mb_type <= 24;
    if (m.mb_type == 0 && p_->transform_8x8) {
        Mb* A = nb<AFF>(-1, 0);
        Mb* B = nb<AFF>(0, -1);
        m.t8x8 = dec(399 + (A && A->t8x8) + (B && B->t8x8));
    }
    if (m.mb_type == 0) {
        const int n = m.t8x8 ? 4 : 16;
        for (int i = 0; i < n; i++) {
            const int blk = m.t8x8 ? i * 4 : i;
            const int prev = dec(68);
            int rem = 0;
            if (!prev) {
                rem = dec(69);
                rem |= dec(69) << 1;
                rem |= dec(69) << 2;
            }
            int nblk;
            const int bx = kBlkX[blk], by = kBlkY[blk];
            Mb* A = nb_blk<AFF>(bx - 1, by, &nblk);
            const int ma = !A ? -1 : (A->mb_type != 0 ? 2 : A->ipm[nblk]);
            Mb* B = nb_blk<AFF>(bx, by - 1, &nblk);
            const int mb = !B ? -1 : (B->mb_type != 0 ? 2 : B->ipm[nblk]);
            const int pm = (ma < 0 || mb < 0) ? 2 : std::min(ma, mb);
            const int mode = prev ? pm : (rem < pm ? rem : rem + 1);
            if (m.t8x8) {
                for (int k = 0; k < 4; k++) m.ipm[blk + k] = static_cast<uint8_t>(mode);
            } else {
                m.ipm[blk] = static_cast<uint8_t>(mode);
            }
        }
    } else {
        for (int i = 0; i < 16; i++) m.ipm[i] = 2;
    }
    if (!mono_) {
        Mb* A = nb<AFF>(-1, 0);
        Mb* B = nb<AFF>(0, -1);
        const int ctx = (A && A->mb_type != 25 && A->cpm != 0) + (B && B->mb_type != 25 && B->cpm != 0);
        if (!dec(64 + ctx)) m.cpm = 0;
        else if (!dec(67)) m.cpm = 1;
        else m.cpm = dec(67) ? 3 : 2;
    }
    if (is16) {
        const int t = m.mb_type - 1;
        m.cbp = (((t / 4) % 3) << 4) | (t >= 12 ? 15 : 0);
    } else {
        int cbp = 0;
        for (int b8 = 0; b8 < 4; b8++) {
            const int bx = b8 & 1, by = b8 >> 1;
            int ca, cb;
            int xW, yW;  // neighbouring 8x8 blocks (6.4.11.2)
            if (bx == 0) {
                Mb* A = nb_loc<AFF>(-1, by * 8, 16, 16, &xW, &yW);
                ca = A ? (A->mb_type == 25 ? 0 : !((A->cbp >> ((yW >> 3) * 2 + (xW >> 3))) & 1)) : 0;
            } else {
                ca = !((cbp >> (b8 - 1)) & 1);
            }
            if (by == 0) {
                Mb* B = nb_loc<AFF>(bx * 8, -1, 16, 16, &xW, &yW);
                cb = B ? (B->mb_type == 25 ? 0 : !((B->cbp >> ((yW >> 3) * 2 + (xW >> 3))) & 1)) : 0;
            } else {
                cb = !((cbp >> (b8 - 2)) & 1);
            }
            cbp |= dec(73 + ca + 2 * cb) << b8;
        }
        if (!mono_) {  // CodedBlockPatternChroma bins (none for ChromaArrayType 0)
            Mb* A = nb<AFF>(-1, 0);
            Mb* B = nb<AFF>(0, -1);
            const int ac = A ? (A->mb_type == 25 ? 2 : (A->cbp >> 4)) : 0;
            const int bc = B ? (B->mb_type == 25 ? 2 : (B->cbp >> 4)) : 0;
            if (dec(77 + (ac > 0) + 2 * (bc > 0))) cbp |= (1 + dec(77 + 4 + (ac == 2) + 2 * (bc == 2))) << 4;
        }
        m.cbp = cbp;
    }
    int qpd = 0;
    if ((m.cbp & 15) || (m.cbp >> 4) || is16) {
        int ctx = prev_qpd_nz_ ? 1 : 0, k = 0;
        if (dec(60 + ctx)) {
            k = 1;
            ctx = 2;
            while (dec(60 + ctx)) {
                ctx = 3;
                if (++k > 104) { err_ = -31; return; }
            }
        }
        qpd = (k & 1) ? (k + 1) / 2 : -(k / 2);
        qp_ = ((qp_ + qpd + 52 + 2 * qpbd_) % (52 + qpbd_)) - qpbd_;
    }
    prev_qpd_nz_ = qpd != 0;
    m.qp = qp_;
    rec.qp = static_cast<int8_t>(qp_);
    if (m.t8x8) rec.mbflags |= 2;
    const int qpl = qp_ + qpbd_;
    // ---- residual + record emission (sparse: (raster pos << 16) | level) ----
    uint8_t pos[64];
    int lvl[64];
    uint32_t mbe[256];  // I16x16: the whole macroblock's levels
    int nmb = 0;
    auto entry = [](int p, int v) { return H2J_COEF264(p, v); };
    const uint8_t* z4 = AFF && m.field ? kFld4 : kZz4;  // field MBs: field scans (8.5.6 / 8.5.7)
    const uint8_t* z8 = AFF && m.field ? kFld8 : kZz8;
    if (is16) {
        Mb* A = nb<AFF>(-1, 0);
        Mb* B = nb<AFF>(0, -1);
        const int n = residual_block<AFF>(0, cbf_cond(0, A, 0, 0) + 2 * cbf_cond(0, B, 0, 0), 16, pos, lvl);
        m.cbf_dc[0] = static_cast<uint8_t>(n != 0);
        for (int k = 0; k < n; k++) {
            const int r = z4[pos[k]];  // raster index of the DC matrix = 4x4 block position
            mbe[nmb++] = entry((r >> 2) * 4 * 16 + (r & 3) * 4, lvl[k]);
        }
    }
    for (int b8 = 0; b8 < 4 && !err_; b8++) {
        const bool coded = (m.cbp >> b8) & 1;
        if (m.t8x8) {
            uint32_t e[64];
            int ne = 0;
            if (coded) {
                const int n = residual_block<AFF>(5, 0, 64, pos, lvl);
                for (int k = 0; k < n; k++) e[ne++] = entry(z8[pos[k]], lvl[k]);
                for (int k = 0; k < 4; k++) m.cbf[b8 * 4 + k] = 1;
            }
            emit_sparse<AFF>(gx + (b8 & 1) * 8, gy + (b8 >> 1) * 8, 3, 0, m.ipm[b8 * 4], qpl, e, ne);
            continue;
        }
        for (int b4 = 0; b4 < 4; b4++) {
            const int blk = b8 * 4 + b4, bx = kBlkX[blk], by = kBlkY[blk];
            uint32_t e[16];
            int ne = 0;
            if (coded) {
                int nblk;
                Mb* A = nb_blk<AFF>(bx - 1, by, &nblk);
                const int ca = cbf_cond(is16 ? 1 : 2, A, nblk, 0);
                Mb* B = nb_blk<AFF>(bx, by - 1, &nblk);
                const int cb = cbf_cond(is16 ? 1 : 2, B, nblk, 0);
                if (is16) {
                    const int n = residual_block<AFF>(1, ca + 2 * cb, 15, pos, lvl);
                    m.cbf[blk] = static_cast<uint8_t>(n != 0);
                    for (int k = 0; k < n; k++) {
                        const int r = z4[pos[k] + 1];
                        mbe[nmb++] = entry((by * 4 + (r >> 2)) * 16 + bx * 4 + (r & 3), lvl[k]);
                    }
                } else {
                    const int n = residual_block<AFF>(2, ca + 2 * cb, 16, pos, lvl);
                    m.cbf[blk] = static_cast<uint8_t>(n != 0);
                    for (int k = 0; k < n; k++) e[ne++] = entry(z4[pos[k]], lvl[k]);
                }
            }
            if (!is16) emit_sparse<AFF>(gx + bx * 4, gy + by * 4, 2, 0, m.ipm[blk], qpl, e, ne);
        }
    }
    if (is16) emit_sparse<AFF>(gx, gy, 4, 0, (m.mb_type - 1) % 4, qpl, mbe, nmb);
    // chroma
    uint32_t ce[2][64];
    int nce[2] = {0, 0};
    if (!mono_ && (m.cbp >> 4)) {
        for (int c = 0; c < 2; c++) {
            Mb* A = nb<AFF>(-1, 0);
            Mb* B = nb<AFF>(0, -1);
            const int n = residual_block<AFF>(3, cbf_cond(3, A, 0, c) + 2 * cbf_cond(3, B, 0, c), 4, pos, lvl);
            m.cbf_dc[1 + c] = static_cast<uint8_t>(n != 0);
            for (int k = 0; k < n; k++) ce[c][nce[c]++] = entry((pos[k] >> 1) * 4 * 8 + (pos[k] & 1) * 4, lvl[k]);
        }
    }
    if (!mono_ && (m.cbp >> 4) == 2) {
        for (int c = 0; c < 2; c++)
            for (int b4 = 0; b4 < 4; b4++) {
                const int bx = b4 & 1, by = b4 >> 1;
                int xW, yW, ca, cb;  // neighbouring chroma 4x4 blocks (6.4.11.5)
                if (bx) ca = m.cbf_c[c][b4 - 1];
                else { const Mb* A = nb_loc<AFF>(-1, by * 4, 8, 8, &xW, &yW); ca = cbf_cond(4, A, A ? (yW >> 2) * 2 + (xW >> 2) : 0, c); }
                if (by) cb = m.cbf_c[c][b4 - 2];
                else { const Mb* B = nb_loc<AFF>(bx * 4, -1, 8, 8, &xW, &yW); cb = cbf_cond(4, B, B ? (yW >> 2) * 2 + (xW >> 2) : 0, c); }
                const int n = residual_block<AFF>(4, ca + 2 * cb, 15, pos, lvl);
                m.cbf_c[c][b4] = static_cast<uint8_t>(n != 0);
                for (int k = 0; k < n; k++) {
                    const int r = z4[pos[k] + 1];
                    ce[c][nce[c]++] = entry((by * 4 + (r >> 2)) * 8 + bx * 4 + (r & 3), lvl[k]);
                }
            }
    }
    for (int c = 0; c < 2; c++) {
        const int off = c == 0 ? p_->cqp : p_->cqp2;
        const int qpi = std::max(-qpbd_, std::min(51, qp_ + off));
        emit_sparse<AFF>(gx / 2, gy / 2, 3, 1 + c, m.cpm, chroma_qp_264(qpi) + qpbd_, ce[c], nce[c]);
    }
}

// ---------------------------------------------------------------- CAVLC
// residual_block_cavlc: number of non-zero levels; scan indices in pos[] and
// levels in lvl[]; -1 on a malformed block.
int H264Parser::cavlc_block(int nC, int maxnum, uint8_t* pos, int* lvl) {
    const CavlcLut& L = cavlc_lut();
    int tc, t1;
    if (nC >= 8) {
        const int v = static_cast<int>(vb_.u(6));
        if (v == 3) return 0;
        tc = (v >> 2) + 1;
        t1 = v & 3;
        if (t1 > tc) return -1;
    } else {
        const int col = nC < 0 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
        const uint16_t e = L.ct[col][vb_.peek32() >> 16];
        if (!e) return -1;
        vb_.skip(e >> 10);
        tc = e & 31;
        t1 = (e >> 5) & 3;
    }
    if (tc == 0) return 0;
    if (tc > maxnum) return -1;
    int level[16], run[16];
    if (t1) {
        const uint32_t sgn = vb_.u(t1);
        for (int i = 0; i < t1; i++) level[i] = ((sgn >> (t1 - 1 - i)) & 1) ? -1 : 1;
    }
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = t1; i < tc; i++) {
        const uint32_t w = vb_.peek32();
        if (!w) return -1;
        const int prefix = __builtin_clz(w);
        vb_.skip(prefix + 1);
        int code = (prefix < 15 ? prefix : 15) << sl;
        const int sz = (prefix == 14 && sl == 0) ? 4 : (prefix >= 15 ? prefix - 3 : sl);
        if (sz > 0) code += static_cast<int>(vb_.u(sz));
        if (prefix >= 15 && sl == 0) code += 15;
        if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
        if (i == t1 && t1 < 3) code += 2;
        level[i] = (code & 1) ? (-code - 1) >> 1 : (code + 2) >> 1;
        if (sl == 0) sl = 1;
        if (std::abs(level[i]) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int zeros = 0;
    if (tc < maxnum) {
        uint8_t e;
        if (maxnum == 4) e = L.tzdc[tc - 1][vb_.peek32() >> 29];
        else e = L.tz[tc - 1][vb_.peek32() >> 23];
        if (!e) return -1;
        vb_.skip(e >> 4);
        zeros = e & 15;
        if (zeros > maxnum - tc) return -1;
    }
    for (int i = 0; i < tc - 1; i++) {
        if (zeros > 0) {
            const int zl = zeros < 7 ? zeros : 7;
            const uint8_t e = L.rb[zl - 1][vb_.peek32() >> 21];
            if (!e) return -1;
            vb_.skip(e >> 4);
            const int r = e & 15;
            if (r > zeros) return -1;
            run[i] = r;
            zeros -= r;
        } else {
            run[i] = 0;
        }
    }
    run[tc - 1] = zeros;
    int coeff = -1;
    for (int i = tc - 1, k = 0; i >= 0; i--, k++) {
        coeff += run[i] + 1;
        pos[k] = static_cast<uint8_t>(coeff);
        lvl[k] = level[i];
    }
    return tc;
}

// nC (9.2.1): average of the neighbours' TotalCoeff, I_PCM counts 16
template <bool AFF>
int H264Parser::nc_luma(int blk) {
    int nblk, cnt_a = 0, cnt_b = 0;
    Mb* A = nb_blk<AFF>(kBlkX[blk] - 1, kBlkY[blk], &nblk);
    if (A) cnt_a = A->mb_type == 25 ? 16 : A->tc[nblk];
    Mb* B = nb_blk<AFF>(kBlkX[blk], kBlkY[blk] - 1, &nblk);
    if (B) cnt_b = B->mb_type == 25 ? 16 : B->tc[nblk];
    if (A && B) return (cnt_a + cnt_b + 1) >> 1;
    return A ? cnt_a : (B ? cnt_b : 0);
}

template <bool AFF>
int H264Parser::nc_chroma(const Mb& m, int c, int b4) {
    const int bx = b4 & 1, by = b4 >> 1;
    int cnt_a = 0, cnt_b = 0;
    bool aa = true, ab = true;
    int xW, yW;  // neighbouring chroma 4x4 blocks (6.4.11.5)
    if (bx) {
        cnt_a = m.tcc[c][b4 - 1];
    } else {
        Mb* A = nb_loc<AFF>(-1, by * 4, 8, 8, &xW, &yW);
        if (!A) aa = false;
        else cnt_a = A->mb_type == 25 ? 16 : A->tcc[c][(yW >> 2) * 2 + (xW >> 2)];
    }
    if (by) {
        cnt_b = m.tcc[c][b4 - 2];
    } else {
        Mb* B = nb_loc<AFF>(bx * 4, -1, 8, 8, &xW, &yW);
        if (!B) ab = false;
        else cnt_b = B->mb_type == 25 ? 16 : B->tcc[c][(yW >> 2) * 2 + (xW >> 2)];
    }
    if (aa && ab) return (cnt_a + cnt_b + 1) >> 1;
    return aa ? cnt_a : (ab ? cnt_b : 0);
}

template <bool AFF>
void H264Parser::decode_mb_cavlc() {
    Mb& m = mb_[mby_ * mbw_ + mbx_];
    m = Mb();
    m.slice = cur_slice_;
    const int gx = mbx_ * 16, gy = mby_ * 16;
    h2j_ctb& rec = job_->ctbs[mby_ * mbw_ + mbx_];
    rec.slice = static_cast<uint8_t>(cur_slice_);
    m.vx = mbx_;
    m.vy = mby_;
    m.field = AFF && mbaff_ ? cur_field_ : 0;
    rec.mbflags = static_cast<uint8_t>(4 | (m.field ? 8 : 0));  // bit 3: MBAFF field macroblock
    const uint32_t mbt = vb_.ue();
    if (mbt > 25) { err_ = -40; return; }
    m.mb_type = static_cast<int>(mbt);
    if (m.mb_type == 25) {
        vb_.align();
        int lv[256];
        for (int i = 0; i < 256; i++) lv[i] = static_cast<int>(vb_.u(s_->bit_depth));
        emit(gx, gy, 4, 0, 0, H2J_TU_PCM, 0, lv, 256, true);
        for (int c = 1; c < 3; c++) {
            for (int i = 0; i < 64; i++) lv[i] = mono_ ? 1 << (s_->bit_depth - 1) : static_cast<int>(vb_.u(s_->bit_depth_c));
            emit(gx / 2, gy / 2, 3, c, 0, H2J_TU_PCM, 0, lv, 64, true);
        }
        m.qp = qp_;
        m.cbp = 0x2F;
        std::memset(m.tc, 16, sizeof(m.tc));
        std::memset(m.tcc, 16, sizeof(m.tcc));
        for (int i = 0; i < 16; i++) m.ipm[i] = 2;
        rec.qp = static_cast<int8_t>(qp_);
        rec.mbflags |= 1;
        return;
    }
    const bool is16 = m.mb_type >= 1 && m.mb_type <= 24;
    if (m.mb_type == 0 && p_->transform_8x8) m.t8x8 = static_cast<int>(vb_.u(1));
    if (m.mb_type == 0) {
        const int n = m.t8x8 ? 4 : 16;
        for (int i = 0; i < n; i++) {
            const int blk = m.t8x8 ? i * 4 : i;
            const int prev = static_cast<int>(vb_.u(1));
            const int rem = prev ? 0 : static_cast<int>(vb_.u(3));
            int nblk;
            const int bx = kBlkX[blk], by = kBlkY[blk];
            Mb* A = nb_blk<AFF>(bx - 1, by, &nblk);
            const int ma = !A ? -1 : (A->mb_type != 0 ? 2 : A->ipm[nblk]);
            Mb* B = nb_blk<AFF>(bx, by - 1, &nblk);
            const int mb = !B ? -1 : (B->mb_type != 0 ? 2 : B->ipm[nblk]);
            const int pm = (ma < 0 || mb < 0) ? 2 : std::min(ma, mb);
            const int mode = prev ? pm : (rem < pm ? rem : rem + 1);
            if (m.t8x8) {
                for (int k = 0; k < 4; k++) m.ipm[blk + k] = static_cast<uint8_t>(mode);
            } else {
                m.ipm[blk] = static_cast<uint8_t>(mode);
            }
        }
    } else {
        for (int i = 0; i < 16; i++) m.ipm[i] = 2;
    }
    if (!mono_) {
        const uint32_t cpm = vb_.ue();
        if (cpm > 3) { err_ = -41; return; }
        m.cpm = static_cast<int>(cpm);
    }
    if (is16) {
        const int t = m.mb_type - 1;
        m.cbp = (((t / 4) % 3) << 4) | (t >= 12 ? 15 : 0);
    } else {
        // Table 9-4 (me(v)): ChromaArrayType 0 maps codeNum 0..15 to luma-only patterns
        static const uint8_t kCbpIntraGray[16] = {15, 0, 7, 11, 13, 14, 3, 5, 10, 12, 1, 2, 4, 8, 6, 9};
        const uint32_t cn = vb_.ue();
        if (cn > (mono_ ? 15u : 47u)) { err_ = -42; return; }
        m.cbp = mono_ ? kCbpIntraGray[cn] : kCbpIntra[cn];
    }
    if ((m.cbp & 15) || (m.cbp >> 4) || is16) {
        const int qpd = vb_.se();
        if (qpd < -(26 + qpbd_ / 2) || qpd > 25 + qpbd_ / 2) { err_ = -43; return; }
        qp_ = ((qp_ + qpd + 52 + 2 * qpbd_) % (52 + qpbd_)) - qpbd_;
    }
    m.qp = qp_;
    rec.qp = static_cast<int8_t>(qp_);
    if (m.t8x8) rec.mbflags |= 2;
    const int qpl = qp_ + qpbd_;
    uint8_t pos[16];
    int lvl[16];
    uint32_t mbe[256];
    int nmb = 0;
    auto entry = [](int p, int v) { return H2J_COEF264(p, v); };
    const uint8_t* z4 = AFF && m.field ? kFld4 : kZz4;  // field MBs: field scans (8.5.6 / 8.5.7)
    const uint8_t* z8 = AFF && m.field ? kFld8 : kZz8;
    if (is16) {
        const int n = cavlc_block(nc_luma<AFF>(0), 16, pos, lvl);
        if (n < 0) { err_ = -44; return; }
        for (int k = 0; k < n; k++) {
            const int r = z4[pos[k]];
            mbe[nmb++] = entry((r >> 2) * 4 * 16 + (r & 3) * 4, lvl[k]);
        }
    }
    for (int b8 = 0; b8 < 4; b8++) {
        const bool coded = (m.cbp >> b8) & 1;
        if (m.t8x8) {
            uint32_t e[64];
            int ne = 0;
            if (coded) {
                for (int i4 = 0; i4 < 4; i4++) {
                    const int blk = b8 * 4 + i4;
                    const int n = cavlc_block(nc_luma<AFF>(blk), 16, pos, lvl);
                    if (n < 0) { err_ = -44; return; }
                    m.tc[blk] = static_cast<uint8_t>(n);
                    for (int k = 0; k < n; k++) e[ne++] = entry(z8[4 * pos[k] + i4], lvl[k]);
                }
            }
            emit_sparse<AFF>(gx + (b8 & 1) * 8, gy + (b8 >> 1) * 8, 3, 0, m.ipm[b8 * 4], qpl, e, ne);
            continue;
        }
        for (int b4 = 0; b4 < 4; b4++) {
            const int blk = b8 * 4 + b4, bx = kBlkX[blk], by = kBlkY[blk];
            uint32_t e[16];
            int ne = 0;
            if (coded) {
                const int n = cavlc_block(nc_luma<AFF>(blk), is16 ? 15 : 16, pos, lvl);
                if (n < 0) { err_ = -44; return; }
                m.tc[blk] = static_cast<uint8_t>(n);
                for (int k = 0; k < n; k++) {
                    if (is16) {
                        const int r = z4[pos[k] + 1];
                        mbe[nmb++] = entry((by * 4 + (r >> 2)) * 16 + bx * 4 + (r & 3), lvl[k]);
                    } else {
                        e[ne++] = entry(z4[pos[k]], lvl[k]);
                    }
                }
            }
            if (!is16) emit_sparse<AFF>(gx + bx * 4, gy + by * 4, 2, 0, m.ipm[blk], qpl, e, ne);
        }
    }
    if (is16) emit_sparse<AFF>(gx, gy, 4, 0, (m.mb_type - 1) % 4, qpl, mbe, nmb);
    uint32_t ce[2][64];
    int nce[2] = {0, 0};
    if (!mono_ && (m.cbp >> 4)) {
        for (int c = 0; c < 2; c++) {
            const int n = cavlc_block(-1, 4, pos, lvl);
            if (n < 0) { err_ = -44; return; }
            for (int k = 0; k < n; k++) ce[c][nce[c]++] = entry((pos[k] >> 1) * 4 * 8 + (pos[k] & 1) * 4, lvl[k]);
        }
    }
    if (!mono_ && (m.cbp >> 4) == 2) {
        for (int c = 0; c < 2; c++)
            for (int b4 = 0; b4 < 4; b4++) {
                const int bx = b4 & 1, by = b4 >> 1;
                const int n = cavlc_block(nc_chroma<AFF>(m, c, b4), 15, pos, lvl);
                if (n < 0) { err_ = -44; return; }
                m.tcc[c][b4] = static_cast<uint8_t>(n);
                for (int k = 0; k < n; k++) {
                    const int r = z4[pos[k] + 1];
                    ce[c][nce[c]++] = entry((by * 4 + (r >> 2)) * 8 + bx * 4 + (r & 3), lvl[k]);
                }
            }
    }
    for (int c = 0; c < 2; c++) {
        const int off = c == 0 ? p_->cqp : p_->cqp2;
        const int qpi = std::max(-qpbd_, std::min(51, qp_ + off));
        emit_sparse<AFF>(gx / 2, gy / 2, 3, 1 + c, m.cpm, chroma_qp_264(qpi) + qpbd_, ce[c], nce[c]);
    }
    if (vb_.overrun()) err_ = -45;
}

int H264Parser::run(const uint8_t* data, size_t size, int threads) {
    std::vector<Nal> nals;
    split_annexb(data, size, nals);
    rbsp_.resize(size + 16);
    bool have = false;
    int first_frame_num = -1, first_idr = -1, fields_seen = 0;
    int nslice = 0;
    std::vector<SliceWork> works;
    for (const Nal& nal : nals) {
        if (nal.n < 1) continue;
        const int nal_ref_idc = (nal.p[0] >> 5) & 3;
        const int type = nal.p[0] & 31;
        const size_t rn = unescape_rbsp(nal.p + 1, nal.n - 1, rbsp_.data());
        BitReader b(rbsp_.data(), rn);
        if (type == 7) {
            if (have) break;
            if (parse_sps(b, sps_) < 0) { job_->message = "unsupported or invalid SPS"; return -2; }
        } else if (type == 8) {
            if (have) break;
            if (parse_pps(b, pps_, sps_) < 0) { job_->message = "unsupported or invalid PPS"; return -3; }
        } else if (type == 1 || type == 5) {
            const uint32_t first_mb_u = b.ue();
            const int slice_type = static_cast<int>(b.ue());
            const uint32_t pps_id = b.ue();
            if (pps_id > 255 || !pps_[pps_id].valid || !sps_[pps_[pps_id].sps_id].valid) {
                job_->message = "slice references a missing parameter set";
                return -4;
            }
            const Pps& p = pps_[pps_id];
            const Sps& s = sps_[p.sps_id];
            const int frame_num = static_cast<int>(b.u(s.log2_max_frame_num));
            // field_pic_flag / bottom_field_flag: a field picture (PAFF).  FFmpeg holds a first field
            // until the second field of the frame arrives ("Wait for second field", h264dec.c) and
            // outputs the interleaved frame; the reference sends one packet (one field: FFmpeg's
            // h264 parser splits fields) and returns false (/root/reference/src/Decoder.cpp:324-360,
            // H2J_STRICT_REFERENCE).  Picture 0 here is the field pair: the first field and the
            // other parity's field of the same frame_num.
            int field_pic = 0, bottom = 0;
            if (!s.frame_mbs_only) {
                field_pic = static_cast<int>(b.u(1));
                if (field_pic) bottom = static_cast<int>(b.u(1));
            }
            // MBAFF: first_mb_in_slice counts pairs; a field: the field's macroblocks
            const int first_mb = first_mb_u < static_cast<uint32_t>(s.mb_w * s.mb_h / (1 + (s.mbaff || field_pic))) ? static_cast<int>(first_mb_u) : -1;
            if (have && !paff_ && (field_pic || first_mb == 0 || frame_num != first_frame_num || (type == 5) != (first_idr == 1))) break;
            if (have && paff_) {
                if (!field_pic || frame_num != first_frame_num) break;
                const bool seen = (fields_seen >> bottom) & 1;
                if (first_mb == 0 ? seen : !seen) break;  // a third field / a slice of an unseen field not at 0
            }
            // FFmpeg h264_slice.c: "first_mb_in_slice overflow" drops the slice; once a slice of
            // picture 0 is collected the picture is still output, so stop there as at a
            // picture boundary, and fail only when nothing of picture 0 was accepted
            if (have && first_mb < 0) break;
            if (first_mb < 0) {
                job_->message = "first_mb_in_slice outside the picture";
                return -6;
            }
            if (slice_type % 5 != 2) {
                // an I field followed by a P / B field (broadcast 1080i) names its cause
                job_->message = have && paff_ ? "PAFF second field is P/B (unsupported: intra field pairs only)"
                                              : "first picture is not intra (P/B slices unsupported)";
                return -5;
            }
            if (type == 5) b.ue();
            if (s.poc_type == 0) {
                b.u(s.log2_max_poc_lsb);
                if (p.bottom_field_pic_order && !field_pic) b.se();
            } else if (s.poc_type == 1 && !s.delta_pic_order_always_zero) {
                b.se();
                if (p.bottom_field_pic_order && !field_pic) b.se();
            }
            if (p.redundant_pic_cnt) b.ue();
            if (nal_ref_idc) {
                if (type == 5) {
                    b.u(1);
                    b.u(1);
                } else if (b.u(1)) {
                    for (int guard = 0; guard < 64; guard++) {
                        const uint32_t op = b.ue();
                        if (op == 0) break;
                        if (op == 1 || op == 3) b.ue();
                        if (op == 2) b.ue();
                        if (op == 3 || op == 6) b.ue();
                        if (op == 4) b.ue();
                    }
                }
            }
            const int qpd = b.se();
            h2j_slice srec{};
            if (p.deblock_ctrl) {
                const uint32_t idc = b.ue();
                if (idc > 2) { job_->message = "disable_deblocking_filter_idc out of range"; return -6; }
                srec.deblock_disabled = static_cast<uint8_t>(idc);
                if (srec.deblock_disabled != 1) {
                    const int a = b.se(), bb = b.se();
                    if (a < -6 || a > 6 || bb < -6 || bb > 6) { job_->message = "deblocking offsets out of range"; return -6; }
                    srec.tc_offset = static_cast<int8_t>(a * 2);
                    srec.beta_offset = static_cast<int8_t>(bb * 2);
                }
            }
            srec.cqp_offset[0] = static_cast<int8_t>(p.cqp);
            srec.cqp_offset[1] = static_cast<int8_t>(p.cqp2);
            // slice identity for the kernels' slice tests: unique over both fields of a pair
            srec.slice_addr_rs = first_mb + bottom * (s.mb_w * s.mb_h / 2);
            if (!have) {
                s_ = &s;
                job_->reorder_delay = s.num_reorder_frames > 0;
                mbw_ = s.mb_w;
                mbh_ = s.mb_h;
                mbaff_ = s.mbaff || field_pic;  // MbaffFrameFlag; a field pair uses the same layout
                paff_ = field_pic;
                job_->field_pair = field_pic != 0;
                qpbd_ = 6 * (s.bit_depth - 8);
                mono_ = s.chroma_format_idc == 0;
                mb_.assign(static_cast<size_t>(mbw_) * mbh_, Mb());
                job_->ctbs.assign(static_cast<size_t>(mbw_) * mbh_, h2j_ctb());
                for (int i = 0; i < mbw_ * mbh_; i++) job_->ctbs[i].ts = static_cast<uint32_t>(i);
                // PAFF: every macroblock of the pair layout is a field MB (h2j_ctb.mbflags bit 3), also
                // the ones a truncated field leaves undecoded, so K0 / K1 / the deblocker map rows
                // alike
                if (paff_)
                    for (auto& c : job_->ctbs) c.mbflags = 8;
                job_->tus.reserve(static_cast<size_t>(mbw_) * mbh_ * 10);
                job_->coefs.reserve(static_cast<size_t>(mbw_) * mbh_ * 64);
                h2j_frame& f = job_->hdr;
                f.codec = H2J_CODEC_H264;
                f.width = mbw_ * 16;
                f.height = mbh_ * 16;
                // decode.c apply_cropping: the left crop as av_frame_apply_cropping aligns it
                const int cl = ff_crop_left(s.crop_l, s.bit_depth > 8 ? 2 : 1);
                if (cl < 0) {
                    job_->message = "left crop FFmpeg's av_frame_apply_cropping rejects (AVERROR_BUG: no frame)";
                    return -6;
                }
                f.crop_x = cl;
                f.crop_y = s.crop_t;
                f.out_w = f.width - cl - s.crop_r;
                f.out_h = f.height - s.crop_t - s.crop_b;
                f.bit_depth = s.bit_depth;
                f.bit_depth_c = s.bit_depth_c;
                f.log2ctb = 4;
                f.ctb_w = mbw_;
                f.ctb_h = mbh_;
                f.mw = f.width / 4;
                f.mh = f.height / 4;
                f.lf_across_tiles = 1;
                f.mbaff = mbaff_;
                if (s.scaling_present || p.scaling_present || p.transform_8x8) {
                    // weight scale tables (raster), used by K1 for every H.264 frame with this flag
                    job_->sl.assign(H2J_SL264_BYTES, 16);
                    for (int c = 0; c < 3; c++)
                        for (int k = 0; k < 16; k++) job_->sl[H2J_SL264_4 + c * 16 + kZz4[k]] = p.sl4[c][k];
                    for (int k = 0; k < 64; k++) job_->sl[H2J_SL264_8 + kZz8[k]] = p.sl8[0][k];
                    f.scaling_list = 1;
                }
                have = true;
                first_frame_num = frame_num;
                first_idr = type == 5;
            }
            p_ = &p;
            if (&s != s_) {  // picture size, bit depth and MBAFF come from the first slice's SPS
                job_->message = "slices of one picture reference different SPSs";
                return -4;
            }
            if (job_->hdr.scaling_list == 0 && (p.transform_8x8 || p.scaling_present || s.scaling_present)) {
                job_->message = "scaling matrices changed inside the picture";
                return -6;
            }
            job_->slices.push_back(srec);
            works.emplace_back();
            SliceWork& w = works.back();
            w.index = nslice;
            w.pps_id = static_cast<int>(pps_id);
            w.first_mb = first_mb;
            w.parity = bottom;
            fields_seen |= field_pic << bottom;
            w.qp = p.init_qp + qpd;
            if (w.qp < -qpbd_ || w.qp > 51) { job_->message = "invalid slice QP"; return -6; }
            w.cabac = p.cabac != 0;
            if (w.cabac) {
                b.align();  // cabac_alignment_one_bit
                const size_t off = b.byte_pos();
                if (off > rn) { job_->message = "truncated slice"; return -6; }
                w.data.assign(rbsp_.begin() + static_cast<long>(off), rbsp_.begin() + static_cast<long>(rn));
                w.nbytes = rn - off;
                w.data.resize(w.nbytes + 8, 0);
            } else {
                // CAVLC: macroblocks until the rbsp_stop_one_bit
                size_t last = rn;
                while (last > 0 && rbsp_[last - 1] == 0) last--;
                if (!last) { job_->message = "empty slice data"; return -6; }
                w.stop_bit = (last - 1) * 8 + 7 - static_cast<size_t>(__builtin_ctz(rbsp_[last - 1]));
                w.data.assign(rbsp_.begin(), rbsp_.begin() + static_cast<long>(rn));
                w.nbytes = rn;
                w.bitpos = b.bit_pos();
                w.data.resize(rn + 8, 0);
            }
            if (++nslice >= 255) { job_->message = "too many slices"; return -8; }
        } else if (type == 9 && have) {
            break;
        }
    }
    if (!have) { job_->message = "no picture found"; return -9; }
    if (paff_ && fields_seen != 3) {  // FFmpeg outputs no frame for a field without its pair
        job_->message = "field picture (PAFF) without the second field of its frame";
        return -3;
    }
    // Slices share nothing for parsing (CABAC / CAVLC restart, neighbours in other slices are
    // unavailable): with threads > 1 they decode side by side, slice 0 into this job, the
    // others into their own jobs, appended in decoding order.
    const int ns = static_cast<int>(works.size());
    if (threads <= 1 || ns <= 1) {
        for (int k = 0; k < ns; k++) {
            const int e = decode_slice(works[k]);
            if (e) return e;
        }
    } else {
        std::vector<FrameJob> part(ns);
        std::vector<std::unique_ptr<H264Parser>> wk(ns);
        for (int k = 1; k < ns; k++) {  // clones first: slice 0 then mutates this parser's state
            part[k].ctbs = job_->ctbs;
            wk[k].reset(new H264Parser(*this, part[k]));
        }
        std::vector<int> rc(ns, 0);
        std::atomic<int> next(1);
        auto work = [&]() {
            for (int k = next++; k < ns; k = next++) rc[k] = wk[k]->decode_slice(works[k]);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < std::min(threads, ns); t++) pool.emplace_back(work);
        rc[0] = decode_slice(works[0]);
        work();
        for (auto& t : pool) t.join();
        for (int k = 1; k < ns; k++)
            if (rc[k]) { job_->message = part[k].message; return rc[k]; }
        if (rc[0]) return rc[0];
        for (int k = 1; k < ns; k++) {
            const uint32_t cbase = static_cast<uint32_t>(job_->coefs.size());
            for (h2j_tu t : part[k].tus) {
                t.coef += cbase;  // (every record carries its position in the coefficient stream)
                job_->tus.push_back(t);
            }
            job_->coefs.insert(job_->coefs.end(), part[k].coefs.begin(), part[k].coefs.end());
            for (size_t m = 0; m < wk[k]->mb_.size(); m++)
                if (wk[k]->mb_[m].slice == k) job_->ctbs[m] = part[k].ctbs[m];
        }
    }
    job_->hdr.nslice = static_cast<uint32_t>(job_->slices.size());
    job_->hdr.topo = (job_->slices.size() != 1 || job_->slices[0].slice_addr_rs != 0) ? 1u : 0u;
    job_->hdr.ntu = static_cast<uint32_t>(job_->tus.size());
    return 0;
}

template <bool AFF>
int H264Parser::mb_loop_cabac(int addr, int nmb) {
    for (;;) {
        if (addr >= nmb) { job_->message = "slice overruns the picture"; return -7; }
        mb_start<AFF>(addr, true);
        decode_mb<AFF>();
        if (err_) { job_->message = "macroblock decode error"; return -7; }
        if (cc_.terminate()) break;
        addr++;
    }
    return 0;
}

template <bool AFF>
int H264Parser::mb_loop_cavlc(int addr, int nmb) {
    for (;;) {
        if (addr >= nmb) { job_->message = "slice overruns the picture"; return -7; }
        mb_start<AFF>(addr, false);
        decode_mb_cavlc<AFF>();
        if (err_) { job_->message = "macroblock decode error"; return -7; }
        if (!vb_.more_rbsp_data(stop_bit_)) break;
        addr++;
    }
    return 0;
}

int H264Parser::decode_slice(const SliceWork& w) {
    p_ = &pps_[w.pps_id];  // this parser's own copy of the parameter sets
    cur_slice_ = w.index;
    qp_ = w.qp;
    prev_qpd_nz_ = 0;
    parity_ = w.parity;
    int addr = w.first_mb * (1 + (mbaff_ && !paff_));  // MBAFF: first_mb_in_slice counts pairs
    const int nmb = paff_ ? mbw_ * mbh_ / 2 : mbw_ * mbh_;
    if (w.cabac) {
        end_ = w.data.data() + w.nbytes;
        cc_.init(w.data.data(), end_);
        for (int i = 0; i < 460; i++) ctx_[i] = cabac_init_word(kInitI[i][0], kInitI[i][1], qp_);
        return mbaff_ ? mb_loop_cabac<true>(addr, nmb) : mb_loop_cabac<false>(addr, nmb);
    } else {
        stop_bit_ = w.stop_bit;
        vb_.init(w.data.data(), w.nbytes, w.bitpos);
        return mbaff_ ? mb_loop_cavlc<true>(addr, nmb) : mb_loop_cavlc<false>(addr, nmb);
    }
}

}  // namespace

int h264_parse_picture(const uint8_t* data, size_t size, FrameJob& job) {
    job.clear();
    std::unique_ptr<H264Parser> p(new H264Parser(job));  // large (parameter-set tables): heap
    const int r = p->run(data, size, job.threads);
    job.error = r;
    return r;
}

}  // namespace h2j
