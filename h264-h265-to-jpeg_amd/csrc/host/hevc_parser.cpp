// HEVC (H.265 Main/Main10, and 4:2:0 range extensions at 8/9/10/12 bits) intra entropy
// decoding on the host.
//
// Replaces the parsing half of FFmpeg's hevc decoder that the reference
// reaches through avcodec_send_packet (/root/reference/src/Decoder.cpp:324):
// VPS/SPS/PPS/slice header (H.265 7.3), CABAC slice data (9.3) including
// SAO syntax, coding quadtree, intra mode derivation (8.4.2/8.4.3), QP
// derivation (8.6.1) and residual_coding.  Instead of reconstructing, it
// emits one h2j_tu per transform block plus the sparse coefficient levels
// (include/h2j_jobs.h); dequantisation, transforms, intra prediction and
// the loop filters run on the GPU.
#include <algorithm>
#include <array>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "bitstream.h"
#include "cabac.h"
#include "job.h"

namespace h2j {
#ifdef H2J_CORO
extern thread_local void (*g_h2j_yield)();  // tools/parse_bench/coro.h experiment
#endif
namespace {

enum {
    C_SAO_MERGE = 0, C_SAO_TYPE = 1, C_SPLIT_CU = 2, C_TQ_BYPASS = 5, C_PART_MODE = 6,
    C_PREV_INTRA = 7, C_CHROMA_MODE = 8, C_SPLIT_TF = 9, C_CBF_LUMA = 12, C_CBF_CHROMA = 14,
    C_TSKIP = 18, C_LAST_X = 20, C_LAST_Y = 38, C_CSBF = 56, C_SIG = 60, C_GT1 = 104,
    C_GT2 = 128, C_QP_DELTA = 134, C_CQO_FLAG = 136, C_CQO_IDX = 137, NUM_CTX = 138
};

// initValue for initType 0 (I slices), H.265 Tables 9-5 .. 9-37
const uint8_t kInitI[NUM_CTX] = {
    153, 200, 139, 141, 157, 154, 184, 184, 63, 153, 138, 138, 111, 141, 94, 138, 182, 154,
    139, 139,
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
    91, 171, 134, 141,
    111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141,
    179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153,
    136, 139, 111, 136, 139, 111, 141, 111,
    140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166,
    182, 140, 227, 122, 197,
    138, 153, 136, 167, 152, 152,
    154, 154,
    154, 154};  // cu_chroma_qp_offset_flag, cu_chroma_qp_offset_idx (Tables 9-34 / 9-35 of H.265 v3)

struct Sps {
    bool valid = false;
    int chroma_format_idc = 0, width = 0, height = 0;
    int conf_l = 0, conf_r = 0, conf_t = 0, conf_b = 0;
    int bit_depth = 8, bit_depth_c = 8, log2_max_poc_lsb = 4;
    int num_reorder_pics = 0;  // sps_max_num_reorder_pics[sps_max_sub_layers_minus1]
    int log2_min_cb = 3, log2_ctb = 4, log2_min_tb = 2, log2_max_tb = 5, max_th_depth_intra = 0;
    int scaling_list_enabled = 0;
    uint8_t sl[4][6][64];
    uint8_t sl_dc[4][6];
    int sao = 0, pcm = 0, pcm_bd = 8, pcm_bd_c = 8, log2_min_pcm = 0, log2_max_pcm = 0, pcm_lf_disabled = 0;
    int num_st_rps = 0;
    int st_num_delta[65];
    int long_term_present = 0, num_lt_sps = 0, temporal_mvp = 0, strong_intra_smoothing = 0;
    int profile_idc = 0;  // general_profile_idc (4: FF_PROFILE_HEVC_REXT)
    // sps_range_extension (H.265 v2 7.3.2.2.2)
    int ts_rotation = 0, ts_context = 0, implicit_rdpcm = 0, explicit_rdpcm = 0, ext_precision = 0;
    int smoothing_disabled = 0, high_prec_offsets = 0, persistent_rice = 0, bypass_alignment = 0;
};

struct Pps {
    bool valid = false;
    int sps_id = 0, dependent_slices = 0, output_flag_present = 0, num_extra_bits = 0, sign_hiding = 0;
    int init_qp = 26, transform_skip = 0, cu_qp_delta = 0, diff_cu_qp_delta_depth = 0;
    int cb_qp_offset = 0, cr_qp_offset = 0, slice_chroma_qp_present = 0, transquant_bypass = 0;
    int tiles = 0, wpp = 0, ntc = 1, ntr = 1, uniform = 1, lf_across_tiles = 1;
    int col_w[64], row_h[64];
    int lf_across_slices = 0, deblock_override = 0, deblock_disabled = 0, beta_offset = 0, tc_offset = 0;
    int sl_present = 0;
    uint8_t sl[4][6][64];
    uint8_t sl_dc[4][6];
    int slice_header_ext = 0;
    // pps_range_extension (7.3.2.3.2), read only for the RExt profile (FFmpeg hevc_ps.c)
    int log2_max_ts = 2, cross_component = 0, cqo_list_enabled = 0, sao_scale_luma = 0, sao_scale_chroma = 0;
    // chroma QP offset lists: entries past chroma_qp_offset_list_len_minus1 stay 0 (FFmpeg's
    // zeroed PPS; its idx parse can reach index 5 whatever the list length)
    int cqo_depth = 0, cqo_len_minus1 = 0, cb_qo[6] = {0, 0, 0, 0, 0, 0}, cr_qo[6] = {0, 0, 0, 0, 0, 0};
};

struct SliceHdr {
    int first_in_pic = 0, dependent = 0, address = 0, slice_addr_rs = 0, pps_id = 0, type = 0;
    int sao_luma = 0, sao_chroma = 0, qp_delta = 0, cb_qp_offset = 0, cr_qp_offset = 0;
    int deblock_disabled = 0, beta_offset = 0, tc_offset = 0, lf_across_slices = 0, slice_qp = 26;
    int cu_chroma_qp_offset_enabled = 0;
    std::vector<uint32_t> entry;  // entry_point_offset_minus1[i] + 1 (bytes, emulation prevention included)
};

const uint8_t kSlIntra[64] = {
    16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18, 17, 18, 18, 17, 18, 21,
    19, 20, 21, 20, 19, 21, 24, 22, 22, 24, 24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29,
    31, 35, 35, 31, 29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115};
const uint8_t kSlInter[64] = {
    16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18, 18, 18, 18, 18, 18, 20,
    20, 20, 20, 20, 20, 20, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28,
    28, 28, 28, 28, 28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91};

void sl_default(uint8_t sl[4][6][64], uint8_t dc[4][6]) {
    for (int m = 0; m < 6; m++) {
        std::memset(sl[0][m], 16, 16);
        for (int s = 1; s < 4; s++) {
            std::memcpy(sl[s][m], m < 3 ? kSlIntra : kSlInter, 64);
            dc[s][m] = 16;
        }
        dc[0][m] = 16;
    }
}

void parse_scaling_list(BitReader& b, uint8_t sl[4][6][64], uint8_t dc[4][6]) {
    for (int sizeId = 0; sizeId < 4; sizeId++)
        for (int m = 0; m < 6; m += (sizeId == 3) ? 3 : 1) {
            int n = sizeId == 0 ? 16 : 64;
            if (!b.u(1)) {
                int delta = static_cast<int>(b.ue());
                if (delta == 0) {
                    if (sizeId == 0) std::memset(sl[0][m], 16, 16);
                    else std::memcpy(sl[sizeId][m], m < 3 ? kSlIntra : kSlInter, 64);
                    dc[sizeId][m] = 16;
                } else {
                    int ref = m - delta * (sizeId == 3 ? 3 : 1);
                    if (ref < 0) ref = 0;
                    std::memcpy(sl[sizeId][m], sl[sizeId][ref], static_cast<size_t>(n));
                    dc[sizeId][m] = dc[sizeId][ref];
                }
            } else {
                int next = 8;
                if (sizeId > 1) {
                    next = b.se() + 8;
                    dc[sizeId][m] = static_cast<uint8_t>(next);
                }
                for (int i = 0; i < n; i++) {
                    next = (next + b.se() + 256) % 256;
                    sl[sizeId][m][i] = static_cast<uint8_t>(next);
                }
                if (sizeId <= 1) dc[sizeId][m] = sl[sizeId][m][0];
            }
        }
}

// profile_tier_level (7.3.3): general_profile_idc, taken from the compatibility flags when it is 0
// (FFmpeg hevc_ps.c decode_profile_tier_level); sub-layer entries skipped
int parse_ptl(BitReader& b, int msl) {
    b.u(3);
    int prof = static_cast<int>(b.u(5));
    for (int j = 0; j < 32; j++)
        if (b.u(1) && prof == 0 && j > 0) prof = j;
    b.u(4); b.u(32); b.u(11); b.u(1); b.u(8);
    int pp[8] = {0}, lp[8] = {0};
    for (int i = 0; i < msl; i++) { pp[i] = static_cast<int>(b.u(1)); lp[i] = static_cast<int>(b.u(1)); }
    if (msl > 0)
        for (int i = msl; i < 8; i++) b.u(2);
    for (int i = 0; i < msl; i++) {
        if (pp[i]) { b.u(32); b.u(32); b.u(24); }
        if (lp[i]) b.u(8);
    }
    return prof;
}

// hrd_parameters (E.2.2) + sub_layer_hrd_parameters (E.2.3), skipped (FFmpeg decode_hrd)
bool skip_hrd(BitReader& b, int max_sub_layers) {
    const int nal = static_cast<int>(b.u(1)), vcl = static_cast<int>(b.u(1));
    int sub_pic = 0;
    if (nal || vcl) {
        sub_pic = static_cast<int>(b.u(1));
        if (sub_pic) b.u(19);
        b.u(8);
        if (sub_pic) b.u(4);
        b.u(15);
    }
    for (int i = 0; i < max_sub_layers; i++) {
        int low_delay = 0;
        uint32_t nb_cpb = 1;
        int fixed = static_cast<int>(b.u(1));
        if (!fixed) fixed = static_cast<int>(b.u(1));
        if (fixed) b.ue();
        else low_delay = static_cast<int>(b.u(1));
        if (!low_delay) {
            nb_cpb = b.ue() + 1;
            if (nb_cpb < 1 || nb_cpb > 32) return false;
        }
        for (int k = 0; k < nal + vcl; k++)
            for (uint32_t j = 0; j < nb_cpb; j++) {
                b.ue(); b.ue();
                if (sub_pic) { b.ue(); b.ue(); }
                b.u(1);
            }
        if (b.overrun()) return false;
    }
    return true;
}

// vui_parameters (E.2.1), skipped: nothing in it changes decoded samples (FFmpeg applies the default
// display window only with its apply_defdispwin option, off by default)
bool skip_vui(BitReader& b, int max_sub_layers) {
    if (b.u(1) && b.u(8) == 255) b.u(32);
    if (b.u(1)) b.u(1);
    if (b.u(1)) {
        b.u(4);
        if (b.u(1)) b.u(24);
    }
    if (b.u(1)) { b.ue(); b.ue(); }
    b.u(3);
    if (b.u(1)) { b.ue(); b.ue(); b.ue(); b.ue(); }
    if (b.u(1)) {
        b.u(32); b.u(32);
        if (b.u(1)) b.ue();
        if (b.u(1) && !skip_hrd(b, max_sub_layers)) return false;
    }
    if (b.u(1)) {
        b.u(3);
        for (int i = 0; i < 5; i++) b.ue();
    }
    return !b.overrun();
}

bool parse_st_rps(BitReader& b, Sps& s, int idx) {
    int inter = 0;
    if (idx != 0) inter = static_cast<int>(b.u(1));
    if (inter) {
        int delta_idx = 1;
        if (idx == s.num_st_rps) delta_idx = static_cast<int>(b.ue()) + 1;
        b.u(1);
        b.ue();
        int ref = idx - delta_idx;
        if (ref < 0) return false;
        int cnt = 0;
        for (int j = 0; j <= s.st_num_delta[ref]; j++) {
            int used = static_cast<int>(b.u(1)), use_delta = 1;
            if (!used) use_delta = static_cast<int>(b.u(1));
            if (used || use_delta) cnt++;
        }
        s.st_num_delta[idx] = cnt;
    } else {
        int neg = static_cast<int>(b.ue()), pos = static_cast<int>(b.ue());
        if (neg > 16 || pos > 16) return false;
        for (int i = 0; i < neg + pos; i++) { b.ue(); b.u(1); }
        s.st_num_delta[idx] = neg + pos;
    }
    return true;
}

int parse_sps(BitReader& b, Sps* tab) {
    b.u(4);
    int msl = static_cast<int>(b.u(3));
    b.u(1);
    const int prof = parse_ptl(b, msl);
    uint32_t id = b.ue();
    if (id > 15) return -1;
    Sps& s = tab[id];
    s = Sps();
    s.profile_idc = prof;
    s.chroma_format_idc = static_cast<int>(b.ue());
    if (s.chroma_format_idc == 3) b.u(1);
    const uint32_t w = b.ue(), h = b.ue();
    if (w == 0 || h == 0 || w > 8192 || h > 8192) return -4;
    s.width = static_cast<int>(w);
    s.height = static_cast<int>(h);
    if (b.u(1)) {
        // conformance window; like FFmpeg (hevc_ps.c "Invalid cropping offsets ... Displaying the
        // whole video surface"), offsets that leave no picture are ignored, not an error
        const uint64_t sw = (s.chroma_format_idc == 1 || s.chroma_format_idc == 2) ? 2 : 1;
        const uint64_t shh = s.chroma_format_idc == 1 ? 2 : 1;
        const uint64_t l = b.ue() * sw, r = b.ue() * sw, t = b.ue() * shh, bo = b.ue() * shh;
        if (l + r < w && t + bo < h) {
            s.conf_l = static_cast<int>(l);
            s.conf_r = static_cast<int>(r);
            s.conf_t = static_cast<int>(t);
            s.conf_b = static_cast<int>(bo);
        }
    }
    // the ue() fields below are range-checked (as FFmpeg's ff_hevc_parse_sps does) before any
    // becomes an int: the syntax allows values up to 2^32 - 2
    const uint32_t bd = b.ue(), bdc = b.ue(), lpl = b.ue();
    if (bd > 4 || bdc > 4 || lpl > 12) return -3;
    s.bit_depth = static_cast<int>(bd) + 8;
    s.bit_depth_c = static_cast<int>(bdc) + 8;
    s.log2_max_poc_lsb = static_cast<int>(lpl) + 4;
    int sub = static_cast<int>(b.u(1));
    for (int i = sub ? 0 : msl; i <= msl; i++) {
        b.ue();
        const uint32_t reorder = b.ue();
        b.ue();
        if (i == msl) s.num_reorder_pics = reorder > 16 ? 16 : static_cast<int>(reorder);
    }
    const uint32_t mcb = b.ue(), dcb = b.ue(), mtb = b.ue(), dtb = b.ue();
    if (mcb > 3 || dcb > 3 || mtb > 3 || dtb > 3) return -3;
    s.log2_min_cb = static_cast<int>(mcb) + 3;
    s.log2_ctb = s.log2_min_cb + static_cast<int>(dcb);
    s.log2_min_tb = static_cast<int>(mtb) + 2;
    s.log2_max_tb = s.log2_min_tb + static_cast<int>(dtb);
    b.ue();
    const uint32_t mthd = b.ue();
    if (mthd > 4) return -3;
    s.max_th_depth_intra = static_cast<int>(mthd);
    s.scaling_list_enabled = static_cast<int>(b.u(1));
    sl_default(s.sl, s.sl_dc);
    if (s.scaling_list_enabled && b.u(1)) parse_scaling_list(b, s.sl, s.sl_dc);
    b.u(1);
    s.sao = static_cast<int>(b.u(1));
    s.pcm = static_cast<int>(b.u(1));
    if (s.pcm) {
        s.pcm_bd = static_cast<int>(b.u(4)) + 1;
        s.pcm_bd_c = static_cast<int>(b.u(4)) + 1;
        const uint32_t mp = b.ue(), dp = b.ue();
        if (mp > 2 || dp > 2) return -3;
        s.log2_min_pcm = static_cast<int>(mp) + 3;
        s.log2_max_pcm = s.log2_min_pcm + static_cast<int>(dp);
        s.pcm_lf_disabled = static_cast<int>(b.u(1));
    }
    s.num_st_rps = static_cast<int>(b.ue());
    if (s.num_st_rps > 64) return -1;
    for (int i = 0; i < s.num_st_rps; i++)
        if (!parse_st_rps(b, s, i)) return -1;
    s.long_term_present = static_cast<int>(b.u(1));
    if (s.long_term_present) {
        const uint32_t nlt = b.ue();
        if (nlt > 32) return -1;
        s.num_lt_sps = static_cast<int>(nlt);
        for (int i = 0; i < s.num_lt_sps; i++) { b.u(s.log2_max_poc_lsb); b.u(1); }
    }
    s.temporal_mvp = static_cast<int>(b.u(1));
    s.strong_intra_smoothing = static_cast<int>(b.u(1));
    if (b.u(1) && !skip_vui(b, msl + 1)) return -1;
    if (b.u(1)) {                                    // sps_extension_present_flag
        const int range = static_cast<int>(b.u(1));  // sps_range_extension_flag
        b.u(7);                                      // multilayer / 3d / scc / 4bits: not read (FFmpeg 4.3)
        if (range) {
            s.ts_rotation = static_cast<int>(b.u(1));
            s.ts_context = static_cast<int>(b.u(1));
            s.implicit_rdpcm = static_cast<int>(b.u(1));
            s.explicit_rdpcm = static_cast<int>(b.u(1));
            s.ext_precision = static_cast<int>(b.u(1));
            s.smoothing_disabled = static_cast<int>(b.u(1));
            s.high_prec_offsets = static_cast<int>(b.u(1));
            s.persistent_rice = static_cast<int>(b.u(1));
            s.bypass_alignment = static_cast<int>(b.u(1));
        }
    }
    if (s.chroma_format_idc != 1) return -2;
    // FFmpeg hevc_ps.c map_pixel_format: 4:2:0 exists at 8, 9, 10 and 12 bits only; luma and
    // chroma depths must match
    if ((s.bit_depth != 8 && s.bit_depth != 9 && s.bit_depth != 10 && s.bit_depth != 12) || s.bit_depth_c != s.bit_depth)
        return -12;
    // extended_precision_processing_flag and cabac_bypass_alignment_enabled_flag: FFmpeg 4.3
    // (hevc_ps.c) logs "... not yet implemented" and decodes as if both were 0; so does this parser
    if (s.log2_ctb > 6 || s.log2_ctb < 4 || s.log2_max_tb > 5) return -3;
    // FFmpeg hevc_ps.c: "Invalid value for log2_min_tb_size", "Invalid coded frame dimensions",
    // "max transform block size out of range", "max_transform_hierarchy_depth_intra out of range",
    // "PCM bit depth ... is greater than normal bit depth"
    if (s.log2_min_tb >= s.log2_min_cb || s.log2_min_cb > s.log2_ctb || s.log2_max_tb > s.log2_ctb) return -3;
    if (s.max_th_depth_intra > s.log2_ctb - s.log2_min_tb) return -3;
    if ((s.width & ((1 << s.log2_min_cb) - 1)) || (s.height & ((1 << s.log2_min_cb) - 1))) return -4;
    if (s.pcm && (s.pcm_bd > s.bit_depth || s.pcm_bd_c > s.bit_depth_c || s.log2_max_pcm > std::min(s.log2_ctb, 5)))
        return -3;
    if (b.overrun()) return -1;
    s.valid = true;
    return 0;
}

int parse_pps(BitReader& b, Pps* tab, const Sps* stab) {
    uint32_t id = b.ue();
    if (id > 63) return -1;
    Pps& p = tab[id];
    p = Pps();
    const uint32_t sps_id = b.ue();
    if (sps_id > 15 || !stab[sps_id].valid) return -1;  // FFmpeg: "SPS %u does not exist"
    const Sps& sps = stab[sps_id];
    p.sps_id = static_cast<int>(sps_id);
    p.dependent_slices = static_cast<int>(b.u(1));
    p.output_flag_present = static_cast<int>(b.u(1));
    p.num_extra_bits = static_cast<int>(b.u(3));
    p.sign_hiding = static_cast<int>(b.u(1));
    b.u(1);
    b.ue();
    b.ue();
    p.init_qp = 26 + b.se();
    if (p.init_qp < -24 || p.init_qp > 51) return -1;
    b.u(1);  // constrained_intra_pred (no effect in all-intra pictures)
    p.transform_skip = static_cast<int>(b.u(1));
    p.cu_qp_delta = static_cast<int>(b.u(1));
    if (p.cu_qp_delta) {
        const uint32_t dd = b.ue();
        if (dd > 3) return -1;
        p.diff_cu_qp_delta_depth = static_cast<int>(dd);
    }
    p.cb_qp_offset = b.se();
    p.cr_qp_offset = b.se();
    if (p.cb_qp_offset < -12 || p.cb_qp_offset > 12 || p.cr_qp_offset < -12 || p.cr_qp_offset > 12) return -1;
    p.slice_chroma_qp_present = static_cast<int>(b.u(1));
    b.u(1);
    b.u(1);
    p.transquant_bypass = static_cast<int>(b.u(1));
    p.tiles = static_cast<int>(b.u(1));
    p.wpp = static_cast<int>(b.u(1));
    if (p.tiles) {
        const uint32_t ntc = b.ue(), ntr = b.ue();
        if (ntc > 63 || ntr > 63) return -1;
        p.ntc = static_cast<int>(ntc) + 1;
        p.ntr = static_cast<int>(ntr) + 1;
        p.uniform = static_cast<int>(b.u(1));
        if (!p.uniform) {  // sizes in CTBs; their sums are checked against the picture in setup_tiles
            for (int i = 0; i < p.ntc - 1; i++) {
                const uint32_t v = b.ue();
                if (v >= 512) return -1;
                p.col_w[i] = static_cast<int>(v) + 1;
            }
            for (int i = 0; i < p.ntr - 1; i++) {
                const uint32_t v = b.ue();
                if (v >= 512) return -1;
                p.row_h[i] = static_cast<int>(v) + 1;
            }
        }
        p.lf_across_tiles = static_cast<int>(b.u(1));
    }
    p.lf_across_slices = static_cast<int>(b.u(1));
    if (b.u(1)) {
        p.deblock_override = static_cast<int>(b.u(1));
        p.deblock_disabled = static_cast<int>(b.u(1));
        if (!p.deblock_disabled) {
            const int bo = b.se(), to = b.se();
            if (bo < -6 || bo > 6 || to < -6 || to > 6) return -1;
            p.beta_offset = bo * 2;
            p.tc_offset = to * 2;
        }
    }
    p.sl_present = static_cast<int>(b.u(1));
    if (p.sl_present) {
        sl_default(p.sl, p.sl_dc);
        parse_scaling_list(b, p.sl, p.sl_dc);
    }
    b.u(1);
    b.ue();
    p.slice_header_ext = static_cast<int>(b.u(1));
    if (b.u(1)) {                                    // pps_extension_present_flag
        const int range = static_cast<int>(b.u(1));  // pps_range_extension_flag
        b.u(7);
        if (range && sps.profile_idc == 4) {         // FFmpeg reads it for FF_PROFILE_HEVC_REXT only
            if (p.transform_skip) {
                const uint32_t v = b.ue();
                if (v > 3) return -1;
                p.log2_max_ts = static_cast<int>(v) + 2;
            }
            p.cross_component = static_cast<int>(b.u(1));  // 4:4:4 only: no effect on 4:2:0
            p.cqo_list_enabled = static_cast<int>(b.u(1));
            if (p.cqo_list_enabled) {
                // FFmpeg 4.3 hevc_ps.c: depth unchecked, "chroma_qp_offset_list_len_minus1 shall be in
                // the range [0, 5]", list entries unchecked (only logged): they are clamped here to a
                // range whose sum with any QP still saturates as FFmpeg's unclamped int sum does
                p.cqo_depth = static_cast<int>(std::min<uint32_t>(b.ue(), 64u));
                const uint32_t len = b.ue();
                if (len > 5) return -1;
                p.cqo_len_minus1 = static_cast<int>(len);
                for (uint32_t i = 0; i <= len; i++) {
                    p.cb_qo[i] = std::max(-128, std::min(128, b.se()));
                    p.cr_qo[i] = std::max(-128, std::min(128, b.se()));
                }
            }
            const uint32_t sl = b.ue(), sc = b.ue();
            const uint32_t lim = sps.bit_depth > 10 ? static_cast<uint32_t>(sps.bit_depth - 10) : 0u;
            if (sl > lim || sc > lim) return -1;
            p.sao_scale_luma = static_cast<int>(sl);
            p.sao_scale_chroma = static_cast<int>(sc);
        }
    }
    if (b.overrun()) return -1;
    p.valid = true;
    return 0;
}

uint8_t g_scan_diag[4][64][2], g_scan_hor[4][64][2], g_scan_ver[4][64][2];
uint8_t g_scan_inv[3][4][64];  // [scanIdx][log2 size][y * size + x] -> scan position
// [scanIdx][log2 TB size - 2][n]: raster offset (y * TB size + x) of 4x4 scan position n inside a
// sub-block, so a coefficient's position is the sub-block's corner offset plus one table entry
uint16_t g_scan_off[3][4][16];
uint8_t g_diag_pos4[16];  // raster (y*4+x) of 4x4 diag scan
uint8_t g_diag_pos8[64];
// context index (C_SIG-relative) of sig_coeff_flag (9.3.4.2.5):
// [chroma][log2n-2][scanIdx][prevCsbf][subblock != 0][scan pos in subblock]
uint8_t g_sigctx[2][4][3][4][2][16];
bool g_scans_ready = false;

void init_scans() {
    if (g_scans_ready) return;
    for (int l = 0; l < 4; l++) {
        int bs = 1 << l, i = 0, x = 0, y = 0;
        while (i < bs * bs) {
            while (y >= 0) {
                if (x < bs && y < bs) {
                    g_scan_diag[l][i][0] = static_cast<uint8_t>(x);
                    g_scan_diag[l][i][1] = static_cast<uint8_t>(y);
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
                g_scan_hor[l][i][0] = static_cast<uint8_t>(x);
                g_scan_hor[l][i][1] = static_cast<uint8_t>(y);
            }
        i = 0;
        for (x = 0; x < bs; x++)
            for (y = 0; y < bs; y++, i++) {
                g_scan_ver[l][i][0] = static_cast<uint8_t>(x);
                g_scan_ver[l][i][1] = static_cast<uint8_t>(y);
            }
    }
    for (int si = 0; si < 3; si++)
        for (int l = 0; l < 4; l++) {
            const uint8_t(*sc)[64][2] = si == 0 ? g_scan_diag : (si == 1 ? g_scan_hor : g_scan_ver);
            for (int i = 0; i < (1 << (2 * l)); i++)
                g_scan_inv[si][l][sc[l][i][1] * (1 << l) + sc[l][i][0]] = static_cast<uint8_t>(i);
        }
    for (int c = 0; c < 2; c++)
        for (int lsb = 0; lsb < 4; lsb++)
            for (int si = 0; si < 3; si++)
                for (int pc = 0; pc < 4; pc++)
                    for (int sb = 0; sb < 2; sb++)
                        for (int nn = 0; nn < 16; nn++) {
                            const uint8_t(*sc)[64][2] = si == 0 ? g_scan_diag : (si == 1 ? g_scan_hor : g_scan_ver);
                            const int log2n = lsb + 2, xp = sc[2][nn][0], yp = sc[2][nn][1];
                            int sigCtx;
                            if (log2n == 2) {
                                static const uint8_t m[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
                                sigCtx = m[(yp << 2) + xp];
                            } else if (!sb && xp + yp == 0) {
                                sigCtx = 0;
                            } else {
                                if (pc == 0) sigCtx = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
                                else if (pc == 1) sigCtx = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
                                else if (pc == 2) sigCtx = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
                                else sigCtx = 2;
                                if (c == 0) {
                                    if (sb) sigCtx += 3;
                                    sigCtx += (log2n == 3) ? ((si == 0) ? 9 : 15) : 21;
                                } else {
                                    sigCtx += (log2n == 3) ? 9 : 12;
                                }
                            }
                            g_sigctx[c][lsb][si][pc][sb][nn] = static_cast<uint8_t>(C_SIG + (c == 0 ? sigCtx : 27 + sigCtx));
                        }
    for (int si = 0; si < 3; si++) {
        const uint8_t(*sc)[64][2] = si == 0 ? g_scan_diag : (si == 1 ? g_scan_hor : g_scan_ver);
        for (int l = 0; l < 4; l++)
            for (int i = 0; i < 16; i++) g_scan_off[si][l][i] = static_cast<uint16_t>(sc[2][i][1] * (4 << l) + sc[2][i][0]);
    }
    for (int i = 0; i < 16; i++) g_diag_pos4[i] = static_cast<uint8_t>(g_scan_diag[2][i][1] * 4 + g_scan_diag[2][i][0]);
    for (int i = 0; i < 64; i++) g_diag_pos8[i] = static_cast<uint8_t>(g_scan_diag[3][i][1] * 8 + g_scan_diag[3][i][0]);
    g_scans_ready = true;
}

int chroma_qp_table(int qpi) {
    static const int t[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    return t[qpi - 30];
}

class HevcParser {
public:
    explicit HevcParser(FrameJob& job) : job_(&job), ctbs_(&job.ctbs) {}
    // a worker for one slice group of the same picture: the picture state (parameter sets,
    // geometry, maps, slice headers) copied, its own outputs
    HevcParser(const HevcParser& proto, FrameJob& job) : HevcParser(proto) {
        job_ = &job;
        ctbs_ = &job.ctbs;
        bind_maps();
    }
    // a worker for the CTB rows of one WPP slice: the picture maps and CTB records are the
    // prototype's (rows write disjoint parts; a row reads the row above only behind its
    // progress counter), the TB records its own
    HevcParser(const HevcParser& proto, bool share_maps) : HevcParser(proto) {
        (void)share_maps;
        ctbs_ = proto.ctbs_;
    }
    int run(const uint8_t* data, size_t size, int threads);

private:
    HevcParser(const HevcParser&) = default;
    FrameJob* job_;
    std::vector<h2j_ctb>* ctbs_;  // CTB records (SAO parameters; read back by sao_merge_left/up)
    Sps sps_[16];
    Pps pps_[64];
    const Sps* s_ = nullptr;
    const Pps* p_ = nullptr;
    std::vector<SliceHdr> sh_;
    std::vector<uint8_t> rbsp_;
    std::vector<uint8_t> slice_data_;
    // picture geometry
    int W = 0, H = 0, log2ctb = 0, ctbs = 0, ctbW = 0, ctbH = 0, nctb = 0, mw = 0, mh = 0;
    int qpbd = 0;
    // maps (4x4 granularity): storage, and the pointers decoding uses (own storage, or the
    // prototype's for WPP row workers)
    std::vector<int8_t> qp_store_;
    std::vector<uint8_t> ipm_store_, ctd_store_;
    std::vector<int> addr_store_, slice_store_;
    int8_t* qp_ = nullptr;
    uint8_t *ipm_ = nullptr, *ctd_ = nullptr;
    int *ctb_addr_rs_ = nullptr, *ctb_slice_ = nullptr;
    void bind_maps() {
        qp_ = qp_store_.data();
        ipm_ = ipm_store_.data();
        ctd_ = ctd_store_.data();
        ctb_addr_rs_ = addr_store_.data();
        ctb_slice_ = slice_store_.data();
    }
    std::vector<int> rs2ts_, ts2rs_, tile_id_, col_bd_;
    // slice decode state
    const SliceHdr* cur_ = nullptr;
    int cur_idx_ = 0;
    Cabac cc_;
    const uint8_t* end_ = nullptr;
    CabacState ctx_[NUM_CTX], ctx_wpp_[NUM_CTX], ctx_ds_[NUM_CTX];
    // StatCoeff (RExt persistent_rice_adaptation, 9.3.2.2): initialised, stored and synchronised
    // together with the context variables (FFmpeg cabac_init_state / save_states / load_states)
    int stat_[4] = {0, 0, 0, 0}, stat_wpp_[4] = {0, 0, 0, 0}, stat_ds_[4] = {0, 0, 0, 0};
    bool rext_ = false;  // a range-extension residual tool is on (residual<true>)
    bool have_ds_ = false;
    int qp_y_ = 0, qg_pred_ = 0, qpd_val_ = 0, last_cu_qp_ = 0;
    bool is_qpd_coded_ = false, first_qg_ = true;
    // chroma QP offsets (H.265 v2 7.3.8.10 / 9.3.4.2): IsCuChromaQpOffsetCoded, CuQpOffsetCb / Cr
    bool cqo_coded_ = false;
    int cu_qo_cb_ = 0, cu_qo_cr_ = 0;
    int cu_bypass_ = 0;
    int cu_tu_begin_ = 0;
    int err_ = 0;

    int parse_slice_header(BitReader& b, int nal_type, SliceHdr& sh, const SliceHdr* prev);
    bool setup_picture();
    bool setup_tiles();
    int decode_slice_data(int shi, const uint8_t* p, const uint8_t* end);
    struct WppRows;
    int decode_wpp_row(int shi, int row, const uint8_t* p, const uint8_t* end, WppRows& w);
    int run_wpp(const std::vector<uint8_t>& seg, const std::vector<uint32_t>& sub, int threads);
    int decode_tile(int shi, int ts0, int ts1, bool last, const uint8_t* p, const uint8_t* end);
    int run_tiles(const std::vector<uint8_t>& seg, const std::vector<uint32_t>& sub, int threads);
    void merge_parts(const std::vector<FrameJob>& part);
    void ctb_start_contexts(int rs, int ts, bool first);
    void init_contexts(int qp) {
        for (int i = 0; i < NUM_CTX; i++) {
            int iv = kInitI[i];
            ctx_[i] = cabac_init_word((iv >> 4) * 5 - 45, ((iv & 15) << 3) - 16, qp);
        }
        std::memset(stat_, 0, sizeof(stat_));
    }
    bool same_region(int xc, int yc, int xn, int yn) const {
        if (xn < 0 || yn < 0 || xn >= W || yn >= H) return false;
        if (((xn ^ xc) | (yn ^ yc)) >> log2ctb == 0) return true;  // inside the current CTB
        int cn = (yn >> log2ctb) * ctbW + (xn >> log2ctb);
        int cc = (yc >> log2ctb) * ctbW + (xc >> log2ctb);
        if (tile_id_[rs2ts_[cn]] != tile_id_[rs2ts_[cc]] || ctb_slice_[cn] < 0) return false;
        return ctb_addr_rs_[cn] == ctb_addr_rs_[cc];
    }
    void qg_start(int xq, int yq);
    void parse_sao(int rx, int ry);
    void coding_quadtree(int x0, int y0, int log2cb, int depth);
    void coding_unit(int x0, int y0, int log2cb);
    void transform_tree(int x0, int y0, int xb, int yb, int log2n, int depth, int blk, int max_depth,
                        int intra_split, int pcb, int pcr, int cm, int cux, int cuy, int log2cb);
    void transform_unit(int x0, int y0, int xb, int yb, int log2n, int blk, int cbf_l, int cbf_cb,
                        int cbf_cr, int cm, int cux, int cuy, int log2cb);
    template <bool RExt>
    void residual(int log2n, int c, int mode, h2j_tu& tu);
    void emit_tu(int x, int y, int log2n, int c, int mode, uint8_t flags, bool cbf, int pred_mode_for_scan);
    void split_ctb_records(size_t first);
    std::vector<h2j_tu> chroma_tmp_;
    uint8_t edge_flags(int x0, int y0) const;
    void pcm_sample(int x0, int y0, int log2cb);
    // (x + 52 + 2 * QpBdOffset) mod (52 + QpBdOffset) of 8.6.1: one conditional subtraction for
    // every in-range CuQpDeltaVal, the division only for out-of-range values
    int qp_wrap(int x) const {
        const int m = 52 + qpbd;
        if (static_cast<unsigned>(x) < static_cast<unsigned>(2 * m)) return x >= m ? x - m : x;
        return x % m;
    }
    // 4x4-granularity maps: rows of 1-16 entries as fixed-size stores (a memset call per row
    // was a visible share of the quadtree's time)
    static void fill_rows(uint8_t* p, int stride, int rows, int w, uint8_t v) {
        const uint64_t v8 = 0x0101010101010101ull * v;
        for (int y = 0; y < rows; y++, p += stride) {
            if (w == 2) std::memcpy(p, &v8, 2);
            else if (w == 4) std::memcpy(p, &v8, 4);
            else if (w == 8) std::memcpy(p, &v8, 8);
            else if (w == 16) { std::memcpy(p, &v8, 8); std::memcpy(p + 8, &v8, 8); }
            else std::memset(p, v, static_cast<size_t>(w));
        }
    }
    void set_map(uint8_t* m, int x0, int y0, int n, uint8_t v) {
        int ye = std::min((y0 + n) >> 2, mh), xe = std::min((x0 + n) >> 2, mw);
        fill_rows(&m[(y0 >> 2) * mw + (x0 >> 2)], mw, ye - (y0 >> 2), xe - (x0 >> 2), v);
    }
    void set_qp(int x0, int y0, int n, int qp) {
        int ye = std::min((y0 + n) >> 2, mh), xe = std::min((x0 + n) >> 2, mw);
        fill_rows(reinterpret_cast<uint8_t*>(&qp_[(y0 >> 2) * mw + (x0 >> 2)]), mw, ye - (y0 >> 2), xe - (x0 >> 2),
                  static_cast<uint8_t>(qp & 0xFF));
    }
    __attribute__((always_inline)) int dec(int ctx) { return cc_.decision(ctx_[ctx]); }  // (inline: box CPU hevc1080 3.40 -> 3.34 ms, r04u)
};

int HevcParser::parse_slice_header(BitReader& b, int nal_type, SliceHdr& sh, const SliceHdr* prev) {
    sh = SliceHdr();
    sh.first_in_pic = static_cast<int>(b.u(1));
    if (nal_type >= 16 && nal_type <= 23) b.u(1);
    const uint32_t pps_id = b.ue();
    if (pps_id > 63 || !pps_[pps_id].valid) return -1;
    sh.pps_id = static_cast<int>(pps_id);
    const Pps& p = pps_[sh.pps_id];
    if (p.sps_id > 15 || !sps_[p.sps_id].valid) return -1;
    const Sps& s = sps_[p.sps_id];
    if (!sh.first_in_pic) {
        if (p.dependent_slices) sh.dependent = static_cast<int>(b.u(1));
        int cs = 1 << s.log2_ctb;
        int n = ((s.width + cs - 1) / cs) * ((s.height + cs - 1) / cs);
        sh.address = static_cast<int>(b.u(ceil_log2(n)));
        if (sh.address >= n) return -1;
    }
    if (sh.dependent) {
        if (!prev) return -1;
        int addr = sh.address, first = sh.first_in_pic;
        sh = *prev;
        sh.address = addr;
        sh.dependent = 1;
        sh.first_in_pic = first;
    } else {
        sh.slice_addr_rs = sh.address;
        for (int i = 0; i < p.num_extra_bits; i++) b.u(1);
        sh.type = static_cast<int>(b.ue());
        if (p.output_flag_present) b.u(1);
        if (nal_type != 19 && nal_type != 20) {
            b.u(s.log2_max_poc_lsb);
            int sps_flag = static_cast<int>(b.u(1));
            if (!sps_flag) {
                Sps tmp = s;
                if (!parse_st_rps(b, tmp, s.num_st_rps)) return -1;
            } else if (s.num_st_rps > 1) {
                b.u(ceil_log2(s.num_st_rps));
            }
            if (s.long_term_present) {
                uint32_t nsps = 0;
                if (s.num_lt_sps > 0) nsps = b.ue();
                const uint32_t npics = b.ue();
                if (nsps > static_cast<uint32_t>(s.num_lt_sps) || npics > 32) return -1;
                for (uint32_t i = 0; i < nsps + npics; i++) {
                    if (i < nsps) {
                        if (s.num_lt_sps > 1) b.u(ceil_log2(s.num_lt_sps));
                    } else {
                        b.u(s.log2_max_poc_lsb);
                        b.u(1);
                    }
                    if (b.u(1)) b.ue();
                }
            }
            if (s.temporal_mvp) b.u(1);
        }
        if (s.sao) {
            sh.sao_luma = static_cast<int>(b.u(1));
            sh.sao_chroma = static_cast<int>(b.u(1));
        }
        if (sh.type != 2) return -2;
        sh.qp_delta = b.se();
        if (p.slice_chroma_qp_present) {
            sh.cb_qp_offset = b.se();
            sh.cr_qp_offset = b.se();
            if (sh.cb_qp_offset < -12 || sh.cb_qp_offset > 12 || sh.cr_qp_offset < -12 || sh.cr_qp_offset > 12 ||
                p.cb_qp_offset + sh.cb_qp_offset < -12 || p.cb_qp_offset + sh.cb_qp_offset > 12 ||
                p.cr_qp_offset + sh.cr_qp_offset < -12 || p.cr_qp_offset + sh.cr_qp_offset > 12)
                return -1;
        }
        if (p.cqo_list_enabled) sh.cu_chroma_qp_offset_enabled = static_cast<int>(b.u(1));
        int override_ = 0;
        if (p.deblock_override) override_ = static_cast<int>(b.u(1));
        sh.deblock_disabled = p.deblock_disabled;
        sh.beta_offset = p.beta_offset;
        sh.tc_offset = p.tc_offset;
        if (override_) {
            sh.deblock_disabled = static_cast<int>(b.u(1));
            if (!sh.deblock_disabled) {
                const int bo = b.se(), to = b.se();
                if (bo < -6 || bo > 6 || to < -6 || to > 6) return -1;
                sh.beta_offset = bo * 2;
                sh.tc_offset = to * 2;
            }
        }
        sh.lf_across_slices = p.lf_across_slices;
        if (p.lf_across_slices && (sh.sao_luma || sh.sao_chroma || !sh.deblock_disabled))
            sh.lf_across_slices = static_cast<int>(b.u(1));
        sh.slice_qp = p.init_qp + sh.qp_delta;
        if (sh.slice_qp < -6 * (s.bit_depth - 8) || sh.slice_qp > 51) return -1;
    }
    if (p.tiles || p.wpp) {
        const uint32_t ne = b.ue();
        const int cs = 1 << s.log2_ctb;
        if (ne >= static_cast<uint32_t>(((s.width + cs - 1) / cs) * ((s.height + cs - 1) / cs))) return -1;
        if (ne > 0) {
            const uint32_t len = b.ue() + 1;
            if (len > 32) return -1;
            for (uint32_t i = 0; i < ne; i++) sh.entry.push_back(b.u(static_cast<int>(len)) + 1u);
        }
    }
    if (p.slice_header_ext) {
        const uint32_t len = b.ue();
        if (len > 256) return -1;
        for (uint32_t i = 0; i < len; i++) b.u(8);
    }
    b.u(1);
    b.align();
    return b.overrun() ? -1 : 0;
}

bool HevcParser::setup_picture() {
    W = s_->width;
    H = s_->height;
    log2ctb = s_->log2_ctb;
    ctbs = 1 << log2ctb;
    ctbW = (W + ctbs - 1) >> log2ctb;
    ctbH = (H + ctbs - 1) >> log2ctb;
    nctb = ctbW * ctbH;
    mw = (W + 3) >> 2;
    mh = (H + 3) >> 2;
    qpbd = 6 * (s_->bit_depth - 8);
    qp_store_.assign(static_cast<size_t>(mw) * mh, 0);
    ipm_store_.assign(static_cast<size_t>(mw) * mh, 1);
    ctd_store_.assign(static_cast<size_t>(mw) * mh, 0);
    addr_store_.assign(nctb, -1);
    slice_store_.assign(nctb, -1);
    bind_maps();
    rs2ts_.assign(nctb, 0);
    ts2rs_.assign(nctb, 0);
    tile_id_.assign(nctb, 0);
    if (!setup_tiles()) return false;
    job_->ctbs.assign(nctb, h2j_ctb());
    for (int rs = 0; rs < nctb; rs++) {
        job_->ctbs[rs].ts = static_cast<uint32_t>(rs2ts_[rs]);
        job_->ctbs[rs].tile = static_cast<uint16_t>(tile_id_[rs2ts_[rs]]);
    }
    job_->tus.reserve(static_cast<size_t>(W) * H / 24);
    job_->coefs.reserve(static_cast<size_t>(W) * H / 8);
    h2j_frame& f = job_->hdr;
    f.codec = H2J_CODEC_HEVC;
    f.width = W;
    f.height = H;
    // decode.c apply_cropping: the left offset as av_frame_apply_cropping aligns it (4:2:0
    // conformance offsets are even, which never hits its AVERROR_BUG case)
    const int cl = ff_crop_left(s_->conf_l, s_->bit_depth > 8 ? 2 : 1);
    f.crop_x = cl;
    f.crop_y = s_->conf_t;
    f.out_w = W - cl - s_->conf_r;
    f.out_h = H - s_->conf_t - s_->conf_b;
    f.bit_depth = s_->bit_depth;
    f.bit_depth_c = s_->bit_depth_c;
    f.log2ctb = log2ctb;
    f.ctb_w = ctbW;
    f.ctb_h = ctbH;
    f.strong_smoothing = s_->strong_intra_smoothing | (s_->smoothing_disabled ? H2J_NO_INTRA_SMOOTHING : 0);
    f.rext = (s_->implicit_rdpcm ? H2J_REXT_RDPCM : 0) | (s_->ts_rotation ? H2J_REXT_TS_ROT : 0);
    rext_ = s_->persistent_rice || s_->ts_context || s_->implicit_rdpcm || p_->log2_max_ts > 2;
    f.sao_enabled = s_->sao;
    f.lf_across_tiles = p_->lf_across_tiles;
    f.cb_qp_offset = p_->cb_qp_offset;
    f.cr_qp_offset = p_->cr_qp_offset;
    f.mw = mw;
    f.mh = mh;
    if (s_->scaling_list_enabled) {
        // ScalingFactor tables (7.4.5): [sizeId][matrixId(c)][y*n+x]
        const uint8_t(*sl)[6][64] = p_->sl_present ? p_->sl : s_->sl;
        const uint8_t(*dc)[6] = p_->sl_present ? p_->sl_dc : s_->sl_dc;
        job_->sl.assign(H2J_SL_BYTES, 16);
        for (int c = 0; c < 3; c++)
            for (int i = 0; i < 16; i++) job_->sl[H2J_SL_S0 + c * 16 + g_diag_pos4[i]] = sl[0][c][i];
        for (int c = 0; c < 3; c++)
            for (int i = 0; i < 64; i++) job_->sl[H2J_SL_S1 + c * 64 + g_diag_pos8[i]] = sl[1][c][i];
        for (int c = 0; c < 3; c++) {
            uint8_t* t = &job_->sl[H2J_SL_S2 + c * 256];
            for (int y = 0; y < 16; y++)
                for (int x = 0; x < 16; x++) {
                    int k = 0;
                    while (g_diag_pos8[k] != (y / 2) * 8 + x / 2) k++;
                    t[y * 16 + x] = sl[2][c][k];
                }
            t[0] = dc[2][c];
        }
        uint8_t* t = &job_->sl[H2J_SL_S3];
        for (int y = 0; y < 32; y++)
            for (int x = 0; x < 32; x++) {
                int k = 0;
                while (g_diag_pos8[k] != (y / 4) * 8 + x / 4) k++;
                t[y * 32 + x] = sl[3][0][k];
            }
        t[0] = dc[3][0];
        f.scaling_list = 1;
    }
    return true;
}

bool HevcParser::setup_tiles() {
    const Pps& p = *p_;
    if (p.ntc > ctbW || p.ntr > ctbH) return false;  // 7.4.3.3: at most one tile per CTB column / row
    std::vector<int> colw(p.ntc), rowh(p.ntr), cbd(p.ntc + 1), rbd(p.ntr + 1);
    int s = 0;
    for (int i = 0; i < p.ntc; i++) {
        if (p.uniform) colw[i] = ((i + 1) * ctbW) / p.ntc - (i * ctbW) / p.ntc;
        else colw[i] = i < p.ntc - 1 ? p.col_w[i] : ctbW - s;
        s += colw[i];
    }
    s = 0;
    for (int j = 0; j < p.ntr; j++) {
        if (p.uniform) rowh[j] = ((j + 1) * ctbH) / p.ntr - (j * ctbH) / p.ntr;
        else rowh[j] = j < p.ntr - 1 ? p.row_h[j] : ctbH - s;
        s += rowh[j];
    }
    for (int i = 0; i < p.ntc; i++)
        if (colw[i] <= 0) return false;  // explicit column widths past the picture
    for (int j = 0; j < p.ntr; j++)
        if (rowh[j] <= 0) return false;
    cbd[0] = 0;
    for (int i = 0; i < p.ntc; i++) cbd[i + 1] = cbd[i] + colw[i];
    rbd[0] = 0;
    for (int j = 0; j < p.ntr; j++) rbd[j + 1] = rbd[j] + rowh[j];
    for (int rs = 0; rs < nctb; rs++) {
        int tbx = rs % ctbW, tby = rs / ctbW, tx = 0, ty = 0;
        for (int i = 0; i < p.ntc; i++)
            if (tbx >= cbd[i]) tx = i;
        for (int j = 0; j < p.ntr; j++)
            if (tby >= rbd[j]) ty = j;
        int v = 0;
        for (int i = 0; i < tx; i++) v += rowh[ty] * colw[i];
        for (int j = 0; j < ty; j++) v += ctbW * rowh[j];
        v += (tby - rbd[ty]) * colw[tx] + tbx - cbd[tx];
        if (v < 0 || v >= nctb) v = rs;
        rs2ts_[rs] = v;
        ts2rs_[v] = rs;
    }
    int tid = 0;
    for (int j = 0; j < p.ntr; j++)
        for (int i = 0; i < p.ntc; i++, tid++)
            for (int y = rbd[j]; y < rbd[j + 1]; y++)
                for (int x = cbd[i]; x < cbd[i + 1]; x++) tile_id_[rs2ts_[y * ctbW + x]] = tid;
    col_bd_ = cbd;
    return true;
}

void HevcParser::qg_start(int xq, int yq) {
    int prev = first_qg_ ? cur_->slice_qp : last_cu_qp_;
    first_qg_ = false;
    int ctb = (yq >> log2ctb) * ctbW + (xq >> log2ctb);
    int qa = prev, qb = prev;
    if (same_region(xq, yq, xq - 1, yq) && (yq >> log2ctb) * ctbW + ((xq - 1) >> log2ctb) == ctb)
        qa = qp_[(yq >> 2) * mw + ((xq - 1) >> 2)];
    if (same_region(xq, yq, xq, yq - 1) && ((yq - 1) >> log2ctb) * ctbW + (xq >> log2ctb) == ctb)
        qb = qp_[((yq - 1) >> 2) * mw + (xq >> 2)];
    qg_pred_ = (qa + qb + 1) >> 1;
    qpd_val_ = 0;
    is_qpd_coded_ = false;
}

void HevcParser::parse_sao(int rx, int ry) {
    int ctb = ry * ctbW + rx;
    h2j_ctb& r = (*ctbs_)[ctb];
    uint32_t ts = r.ts;
    uint16_t tile = r.tile;
    std::memset(&r, 0, sizeof(r));
    r.ts = ts;
    r.tile = tile;
    r.slice = static_cast<uint8_t>(cur_idx_);
    if (!cur_->sao_luma && !cur_->sao_chroma) return;
    auto copy_from = [&](int src) {
        const h2j_ctb& o = (*ctbs_)[src];
        std::memcpy(r.type, o.type, 3);
        std::memcpy(r.band_pos, o.band_pos, 3);
        std::memcpy(r.eo_class, o.eo_class, 3);
        std::memcpy(r.off, o.off, sizeof(r.off));
    };
    if (rx > 0) {
        int l = ctb - 1;
        if (tile_id_[rs2ts_[l]] == tile_id_[rs2ts_[ctb]] && ctb_slice_[l] >= 0 && ctb_addr_rs_[l] == ctb_addr_rs_[ctb]) {
            if (dec(C_SAO_MERGE)) { copy_from(l); return; }
        }
    }
    if (ry > 0) {
        int u = ctb - ctbW;
        if (tile_id_[rs2ts_[u]] == tile_id_[rs2ts_[ctb]] && ctb_slice_[u] >= 0 && ctb_addr_rs_[u] == ctb_addr_rs_[ctb]) {
            if (dec(C_SAO_MERGE)) { copy_from(u); return; }
        }
    }
    const int bd = s_->bit_depth;
    const int cmax = (1 << ((bd < 10 ? bd : 10) - 5)) - 1;
    for (int c = 0; c < 3; c++) {
        if ((c == 0 && !cur_->sao_luma) || (c > 0 && !cur_->sao_chroma)) continue;
        // SaoOffsetVal = offset << log2OffsetScale: the PPS range extension's log2_sao_offset_scale,
        // 0 without it (FFmpeg hls_sao_param; not v1's bitDepth - Min(bitDepth, 10))
        const int shift = c ? p_->sao_scale_chroma : p_->sao_scale_luma;
        if (c == 2) {
            r.type[2] = r.type[1];
            r.eo_class[2] = r.eo_class[1];
        } else {
            int t = 0;
            if (dec(C_SAO_TYPE)) t = cc_.bypass() ? 2 : 1;
            r.type[c] = static_cast<int8_t>(t);
        }
        if (r.type[c] == 0) continue;
        int a[4];
        for (int i = 0; i < 4; i++) {
            int v = 0;
            while (v < cmax && cc_.bypass()) v++;
            a[i] = v;
        }
        if (r.type[c] == 1) {
            for (int i = 0; i < 4; i++)
                if (a[i] && cc_.bypass()) a[i] = -a[i];
            r.band_pos[c] = static_cast<int8_t>(cc_.bypass_bits(5));
            for (int i = 0; i < 4; i++) r.off[c][i] = static_cast<int16_t>(a[i] * (1 << shift));
        } else {
            r.off[c][0] = static_cast<int16_t>(a[0] << shift);
            r.off[c][1] = static_cast<int16_t>(a[1] << shift);
            r.off[c][2] = static_cast<int16_t>(-(a[2] << shift));
            r.off[c][3] = static_cast<int16_t>(-(a[3] << shift));
            if (c == 0) r.eo_class[0] = static_cast<int8_t>(cc_.bypass_bits(2));
            if (c == 1) r.eo_class[1] = static_cast<int8_t>(cc_.bypass_bits(2));
        }
    }
}

uint8_t HevcParser::edge_flags(int x0, int y0) const {
    if (cur_->deblock_disabled) return 0;
    uint8_t f = 0;
    const int mask = ctbs - 1;
    if ((x0 & 7) == 0 && x0 > 0) {
        bool ok = true;
        if ((x0 & mask) == 0) {
            int cn = (y0 >> log2ctb) * ctbW + ((x0 - 1) >> log2ctb), cc = cn + 1;
            if (!cur_->lf_across_slices && ctb_addr_rs_[cn] != ctb_addr_rs_[cc]) ok = false;
            if (!p_->lf_across_tiles && tile_id_[rs2ts_[cn]] != tile_id_[rs2ts_[cc]]) ok = false;
        }
        if (ok) f |= H2J_TU_EDGE_L;
    }
    if ((y0 & 7) == 0 && y0 > 0) {
        bool ok = true;
        if ((y0 & mask) == 0) {
            int cc = (y0 >> log2ctb) * ctbW + (x0 >> log2ctb), cn = cc - ctbW;
            if (!cur_->lf_across_slices && ctb_addr_rs_[cn] != ctb_addr_rs_[cc]) ok = false;
            if (!p_->lf_across_tiles && tile_id_[rs2ts_[cn]] != tile_id_[rs2ts_[cc]]) ok = false;
        }
        if (ok) f |= H2J_TU_EDGE_T;
    }
    return f;
}

// RExt transform_skip_context_enabled_flag: every significance bin of a transform-skip / bypass
// block uses context 42 (luma) / 16 + 27 (chroma) (9.3.4.2.5)
const uint8_t kSigTs[2][16] = {{C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42,
                                C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42, C_SIG + 42},
                               {C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43,
                                C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43, C_SIG + 43}};

// RExt = false: H.265 v1 residual coding (the hot path, unchanged).  RExt = true adds the range
// extensions' residual tools as FFmpeg 4.3 hevc_cabac.c decodes them: transform skip up to
// log2_max_transform_skip_block_size, transform-skip contexts, sign data hiding off under implicit
// RDPCM, persistent Rice adaptation (StatCoeff init / update, Rice parameter not capped at 4).
template <bool RExt>
void HevcParser::residual(int log2n, int c, int pred_mode, h2j_tu& tu) {
    // hot path: engine state in a local (registers), contexts by pointer,
    // coefficients into a local buffer appended once per TU
    Cabac cc = cc_;
    CabacState* const ctx = ctx_;
    const int n = 1 << log2n;
    if (p_->transform_skip && !cu_bypass_ && log2n <= (RExt ? p_->log2_max_ts : 2) && cc.decision(ctx[C_TSKIP + (c ? 1 : 0)]))
        tu.flags |= H2J_TU_TSKIP;
    const bool tsb = (tu.flags & H2J_TU_TSKIP) != 0 || cu_bypass_;
    const bool ts_ctx = RExt && s_->ts_context && tsb;
    const bool no_sdh = RExt && s_->implicit_rdpcm && (tu.flags & H2J_TU_TSKIP) && (pred_mode == 10 || pred_mode == 26);
    const bool price = RExt && s_->persistent_rice;
    int* const stat = &stat_[2 * (c == 0 ? 1 : 0) + (tsb ? 1 : 0)];
    // last_sig_coeff prefix/suffix
    int off, shift;
    if (c == 0) {
        off = 3 * (log2n - 2) + ((log2n - 1) >> 2);
        shift = (log2n + 1) >> 2;
    } else {
        off = 15;
        shift = log2n - 2;
    }
    const int maxp = (log2n << 1) - 1;
    // unary prefixes; bins k >> shift share a context (the word forwarded in a register, as in
    // the significance loop below)
    auto last_prefix = [&](CabacState* lc) __attribute__((always_inline)) {
        int k = 0, pk = 0;
        CabacState pw = lc[0];
        while (k < maxp) {
            const int ci = k >> shift;
            const CabacState lw = lc[ci];
            lc[pk] = pw;
            CabacState w = ci == pk ? pw : lw;
            const int b = cc.decision(w);
            pw = w;
            pk = ci;
            if (!b) break;
            k++;
        }
        lc[pk] = pw;
        return k;
    };
    int lx = last_prefix(ctx + C_LAST_X + off);
    int ly = last_prefix(ctx + C_LAST_Y + off);
    if (lx > 3) {
        int nb = (lx >> 1) - 1;
        lx = (1 << nb) * (2 + (lx & 1)) + static_cast<int>(cc.bypass_bits(nb));
    }
    if (ly > 3) {
        int nb = (ly >> 1) - 1;
        ly = (1 << nb) * (2 + (ly & 1)) + static_cast<int>(cc.bypass_bits(nb));
    }
    int scanIdx = 0;
    if (log2n == 2 || (log2n == 3 && c == 0)) {
        if (pred_mode >= 6 && pred_mode <= 14) scanIdx = 2;
        else if (pred_mode >= 22 && pred_mode <= 30) scanIdx = 1;
    }
    if (scanIdx == 2) std::swap(lx, ly);
    if (lx >= n || ly >= n) { err_ = -20; cc_ = cc; return; }
    const uint8_t(*sc)[64][2] = scanIdx == 0 ? g_scan_diag : (scanIdx == 1 ? g_scan_hor : g_scan_ver);
    const int lsb = log2n - 2;
    // locate last position in scan order
    const int lastSub = g_scan_inv[scanIdx][lsb][((ly >> 2) << lsb) + (lx >> 2)];
    const int lastPos = g_scan_inv[scanIdx][2][((ly & 3) << 2) + (lx & 3)];
    uint8_t csbf[8][8];
    std::memset(csbf, 0, sizeof(csbf));
    int greater1_ctx = 1;
    const bool sdh = p_->sign_hiding != 0;
    const int sbw = 1 << lsb;
    uint32_t out[32 * 32];
    int nout = 0;
    const uint16_t* const posTab = g_scan_off[scanIdx][lsb];
    const uint8_t(*const sigtab)[2][16] = g_sigctx[c ? 1 : 0][lsb][scanIdx];
    CabacState* const gt1ctx = ctx + C_GT1 + (c ? 16 : 0);
    for (int i = lastSub; i >= 0; i--) {
#ifdef H2J_CORO_SB
        if (i < lastSub && g_h2j_yield) g_h2j_yield();
#endif
        const int xs = sc[lsb][i][0], ys = sc[lsb][i][1];
        bool infer_dc = false;
        if (i < lastSub && i > 0) {
            int csr = (xs + 1 < sbw) ? csbf[xs + 1][ys] : 0;
            int csb = (ys + 1 < sbw) ? csbf[xs][ys + 1] : 0;
            csbf[xs][ys] = static_cast<uint8_t>(cc.decision(ctx[C_CSBF + (csr | csb) + (c ? 2 : 0)]));
            infer_dc = true;
        } else {
            csbf[xs][ys] = 1;
        }
        unsigned sigmask = 0;  // bit nn
        int nstart = 15;
        if (i == lastSub) {
            nstart = lastPos - 1;
            sigmask = 1u << lastPos;
        }
        if (csbf[xs][ys]) {
            int prevCsbf = 0;
            if (xs + 1 < sbw) prevCsbf |= csbf[xs + 1][ys];
            if (ys + 1 < sbw) prevCsbf |= csbf[xs][ys + 1] << 1;
            const uint8_t* sig = ts_ctx ? kSigTs[c ? 1 : 0] : sigtab[prevCsbf][(xs | ys) ? 1 : 0];
            // bins feed the mask arithmetically (no data-dependent branch per bin).  Consecutive
            // positions often share a context: the word of the previous bin's context stays in a
            // register and is taken by a select when the next bin uses it again, and only the
            // previous context's word is stored each bin -- a store and reload of the word the
            // next bin needs would put store-to-load forwarding on the decision chain
            unsigned got = 0;
            if (nstart > 0) {
                int pidx = sig[nstart];
                CabacState pw = ctx[pidx];
                got = static_cast<unsigned>(cc.decision(pw)) << nstart;
                for (int nn = nstart - 1; nn > 0; nn--) {
                    const int idx = sig[nn];
                    const CabacState lw = ctx[idx];
                    ctx[pidx] = pw;
                    CabacState w = idx == pidx ? pw : lw;
                    got |= static_cast<unsigned>(cc.decision(w)) << nn;
                    pw = w;
                    pidx = idx;
                }
                ctx[pidx] = pw;
            }
            sigmask |= got;
            infer_dc = infer_dc && got == 0;
            if (nstart >= 0) {
                if (!infer_dc) {
                    if (cc.decision(ctx[sig[0]])) sigmask |= 1u;
                } else {
                    sigmask |= 1u;  // nn == 0 inferred
                }
            }
        }
        if (!sigmask) continue;
        // greater1 / greater2
        int ctxSet = (i == 0 || c > 0) ? 0 : 2;
        if (greater1_ctx == 0) ctxSet++;
        greater1_ctx = 1;
        unsigned g1mask = 0;
        int numG1 = 0, lastG1 = -1;
        unsigned m_uncoded = 0;  // significant positions past the first eight (no greater1 bin)
        const int lastSig = 31 - __builtin_clz(sigmask), firstSig = __builtin_ctz(sigmask);
        CabacState* const g1c = gt1ctx + ctxSet * 4;
        {
            // greater1Ctx runs 1, 2, 3, 3, ... until a bin is 1 and is 0 from then on, so the
            // context of bin k is known before bin k - 1 resolves except for that one switch:
            // the four words stay in registers (a load indexed by the previous outcome, plus a
            // store / reload when the context repeats, sat on the decision chain)
            CabacState w0 = g1c[0], w1 = g1c[1], w2 = g1c[2], w3 = g1c[3];
            unsigned seen = 0, m = sigmask;
            auto bin = [&](CabacState& slot) __attribute__((always_inline)) {
                const int nn = 31 - __builtin_clz(m);
                m &= ~(1u << nn);
                CabacState w = seen ? w0 : slot;
                const unsigned d = static_cast<unsigned>(cc.decision(w));
                if (seen) w0 = w;
                else slot = w;
                seen |= d;
                g1mask |= d << nn;
                numG1++;
            };
            if (m) bin(w1);
            if (m) bin(w2);
            while (m && numG1 < 8) bin(w3);
            g1c[0] = w0;
            g1c[1] = w1;
            g1c[2] = w2;
            g1c[3] = w3;
            m_uncoded = m;
            greater1_ctx = seen ? 0 : 1;  // only "== 0" matters (ctxSet of the next sub-block)
        }
        if (g1mask) lastG1 = 31 - __builtin_clz(g1mask);
        const bool hidden = !cu_bypass_ && !no_sdh && (lastSig - firstSig > 3);
        int g2 = 0;
        if (lastG1 != -1) g2 = cc.decision(ctx[C_GT2 + ctxSet + (c ? 4 : 0)]);
        const unsigned signed_mask = (sdh && hidden) ? (sigmask & ~(1u << firstSig)) : sigmask;
        // all sign bins at once; bin i (MSB first) belongs to the i-th highest position, so the
        // output loop below (highest position first) takes them from the top of qs
        const int ns = __builtin_popcount(signed_mask);
        const uint32_t q = ns > 1 ? cc.bypass_batch(ns) : (ns ? static_cast<uint32_t>(cc.bypass()) : 0u);
        uint32_t qs = ns ? q << (32 - ns) : 0u;
        // positions that carry coeff_abs_level_remaining (baseLevel reached its cap): greater1
        // set (greater2 set for the one position that has it) among the first eight, and every
        // position past them (left in m by the greater1 loop).  Decoding them in their own loop
        // keeps the per-coefficient "escape or not" branch off the output loop.
        unsigned esc = g1mask | m_uncoded;
        if (lastG1 >= 0 && !g2) esc &= ~(1u << lastG1);
        int remv[16] = {};
        int rice = price ? *stat / 4 : 0;
        bool stat_done = false;
        for (unsigned e = esc; e;) {
            const int nn = 31 - __builtin_clz(e);
            e &= ~(1u << nn);
            const int baseL = 1 + ((g1mask >> nn) & 1) + (nn == lastG1 ? g2 : 0);
            {
                // coeff_abs_level_remaining: unary prefix + suffix, usually both inside one
                // 20-bin peek (one division instead of a bin loop with a mispredicted exit)
                constexpr int kPeek = 20;
                const uint32_t q = cc.bypass_peek(kPeek);
                const uint32_t inv = ~q << (32 - kPeek);
                int prefix = inv ? __builtin_clz(inv) : kPeek;
                int rem = -1;
                if (prefix < kPeek) {
                    const int slen = prefix < 3 ? rice : prefix - 3 + rice, total = prefix + 1 + slen;
                    if (total <= kPeek) {
                        const uint32_t top = q >> (kPeek - total);
                        cc.bypass_skip(total, top);
                        const int suf = static_cast<int>(top & ((1u << slen) - 1u));
                        rem = prefix < 3 ? (prefix << rice) + suf : (((1 << (prefix - 3)) + 2) << rice) + suf;
                    }
                }
                if (rem < 0) {
                    prefix = 0;
                    while (prefix < 32 && cc.bypass()) prefix++;
                    if (prefix < 3) rem = (prefix << rice) + static_cast<int>(cc.bypass_bits(rice));
                    else {
                        int pm3 = prefix - 3;
                        if (pm3 + rice > 30) { err_ = -21; cc_ = cc; return; }
                        rem = (((1 << pm3) + 2) << rice) + static_cast<int>(cc.bypass_bits(pm3 + rice));
                    }
                }
                remv[nn] = rem;
                if (baseL + rem > 3 * (1 << rice)) rice = price ? rice + 1 : (rice < 4 ? rice + 1 : 4);
                if (price && !stat_done) {  // StatCoeff update from the sub-block's first remaining level
                    const int ri = *stat / 4;
                    if (rem >= (3 << ri)) ++*stat;
                    else if (2 * rem < (1 << ri) && *stat > 0) --*stat;
                    stat_done = true;
                }
            }
        }
        // sign data hiding: the lowest position (processed last) flips when the level sum is odd
        const int flip_last = (sdh && hidden) ? 1 : 0;
        const int sb_off = ((ys << 2) << log2n) + (xs << 2);
        int sumAbs = 0;
        for (unsigned mm = sigmask; mm;) {
            const int nn = 31 - __builtin_clz(mm);
            mm &= ~(1u << nn);
            const int lvl = 1 + ((g1mask >> nn) & 1) + (nn == lastG1 ? g2 : 0) + remv[nn];
            sumAbs += lvl;
            const int neg = static_cast<int>(qs >> 31) ^ (mm == 0 ? (flip_last & sumAbs) : 0);
            qs <<= 1;
            int v = neg ? -lvl : lvl;
            if (v > 32767) v = 32767;
            if (v < -32768) v = -32768;
            out[nout++] = (static_cast<uint32_t>(sb_off + posTab[nn]) << 16) | static_cast<uint16_t>(v);
        }
    }
    cc_ = cc;
    const uint32_t base = static_cast<uint32_t>(job_->coefs.size());
    job_->coefs.insert(job_->coefs.end(), out, out + nout);
    tu.coef = base - job_->hdr.coef;
    tu.ncoef = static_cast<uint16_t>(nout);
    tu.flags |= H2J_TU_CBF;
}

void HevcParser::split_ctb_records(size_t first) {
    std::vector<h2j_tu>& v = job_->tus;
    chroma_tmp_.clear();
    size_t w = first;
    for (size_t i = first; i < v.size(); i++) {
        if (v[i].c == 0) v[w++] = v[i];
        else chroma_tmp_.push_back(v[i]);
    }
    std::copy(chroma_tmp_.begin(), chroma_tmp_.end(), v.begin() + static_cast<long>(w));
}

void HevcParser::emit_tu(int x, int y, int log2n, int c, int mode, uint8_t flags, bool cbf, int) {
    // built in place: a local record filled field by field and then copied into the vector made
    // the copy's 16-byte load wait for the narrow stores (store-to-load forwarding fails)
    job_->tus.emplace_back();
    h2j_tu& tu = job_->tus.back();
    tu.x = static_cast<uint16_t>(x);
    tu.y = static_cast<uint16_t>(y);
    tu.log2n = static_cast<uint8_t>(log2n);
    tu.c = static_cast<uint8_t>(c);
    tu.mode = static_cast<uint8_t>(mode);
    tu.flags = flags;
    tu.qp = 0;
    tu.qpy = 0;
    tu.ncoef = 0;
    tu.coef = 0;
    if (cbf) {
#ifdef H2J_CORO
        if (g_h2j_yield) g_h2j_yield();
#endif
        if (rext_) residual<true>(log2n, c, mode, tu);
        else residual<false>(log2n, c, mode, tu);
    }
}

void HevcParser::transform_unit(int x0, int y0, int xb, int yb, int log2n, int blk, int cbf_l, int cbf_cb,
                                int cbf_cr, int cm, int cux, int cuy, int log2cb) {
    if ((cbf_l || cbf_cb || cbf_cr) && p_->cu_qp_delta && !is_qpd_coded_) {
        int v = 0;
        if (dec(C_QP_DELTA)) {
            v = 1;
            while (v < 5 && dec(C_QP_DELTA + 1)) v++;
            if (v == 5) {
                int k = 0;
                while (k < 32 && cc_.bypass()) k++;
                if (k > 30) { err_ = -22; return; }
                v += ((1 << k) - 1) + static_cast<int>(cc_.bypass_bits(k));
            }
        }
        if (v && cc_.bypass()) v = -v;
        is_qpd_coded_ = true;
        qpd_val_ = v;
        qp_y_ = qp_wrap(qg_pred_ + v + 52 + 2 * qpbd) - qpbd;
        set_qp(cux, cuy, 1 << log2cb, qp_y_);
    }
    // FFmpeg 4.3 hls_transform_unit: once per chroma QP offset group, at the first TU with a chroma
    // cbf in a CU without transquant bypass; ff_hevc_cu_chroma_qp_offset_idx reads the index as a
    // truncated unary code with cMax FFMAX(5, len_minus1) = 5 (the spec's cMax is len_minus1: the two
    // agree unless a stream codes idx == len_minus1 < 5), and only when len_minus1 > 0
    if ((cbf_cb || cbf_cr) && cur_->cu_chroma_qp_offset_enabled && !cu_bypass_ && !cqo_coded_) {
        int idx = -1;
        if (dec(C_CQO_FLAG)) {
            idx = 0;
            if (p_->cqo_len_minus1 > 0)
                while (idx < 5 && dec(C_CQO_IDX)) idx++;
        }
        cu_qo_cb_ = idx < 0 ? 0 : p_->cb_qo[idx];
        cu_qo_cr_ = idx < 0 ? 0 : p_->cr_qo[idx];
        cqo_coded_ = true;
    }
    const int lmode = ipm_[(y0 >> 2) * mw + (x0 >> 2)];
    uint8_t fl = edge_flags(x0, y0);
    if (cu_bypass_) fl |= H2J_TU_BYPASS | H2J_TU_NOFILT;
    uint8_t lfl = fl;
    if (log2n == 2) lfl |= H2J_TU_DST;
    emit_tu(x0, y0, log2n, 0, lmode, lfl, cbf_l != 0, lmode);
    if ((job_->tus.back().flags & (H2J_TU_TSKIP | H2J_TU_BYPASS)) != 0) job_->tus.back().flags &= ~H2J_TU_DST;
    if (err_) return;
    uint8_t cfl = cu_bypass_ ? (H2J_TU_BYPASS | H2J_TU_NOFILT) : 0;
    if (log2n > 2) {
        emit_tu(x0 >> 1, y0 >> 1, log2n - 1, 1, cm, cfl, cbf_cb != 0, cm);
        if (err_) return;
        emit_tu(x0 >> 1, y0 >> 1, log2n - 1, 2, cm, cfl, cbf_cr != 0, cm);
    } else if (blk == 3) {
        emit_tu(xb >> 1, yb >> 1, 2, 1, cm, cfl, cbf_cb != 0, cm);
        if (err_) return;
        emit_tu(xb >> 1, yb >> 1, 2, 2, cm, cfl, cbf_cr != 0, cm);
    }
}

void HevcParser::transform_tree(int x0, int y0, int xb, int yb, int log2n, int depth, int blk, int max_depth,
                                int intra_split, int pcb, int pcr, int cm, int cux, int cuy, int log2cb) {
    if (err_) return;
    int split;
    if (log2n <= s_->log2_max_tb && log2n > s_->log2_min_tb && depth < max_depth && !(intra_split && depth == 0))
        split = dec(C_SPLIT_TF + 5 - log2n);
    else
        split = log2n > s_->log2_max_tb || (intra_split && depth == 0);
    int cbf_cb = 0, cbf_cr = 0;
    if (log2n > 2) {
        if (depth == 0 || pcb) cbf_cb = dec(C_CBF_CHROMA + depth);
        if (depth == 0 || pcr) cbf_cr = dec(C_CBF_CHROMA + depth);
    } else {
        cbf_cb = pcb;
        cbf_cr = pcr;
    }
    if (split) {
        if (log2n <= 2) { err_ = -23; return; }
        int h = 1 << (log2n - 1);
        transform_tree(x0, y0, x0, y0, log2n - 1, depth + 1, 0, max_depth, intra_split, cbf_cb, cbf_cr, cm, cux, cuy, log2cb);
        transform_tree(x0 + h, y0, x0, y0, log2n - 1, depth + 1, 1, max_depth, intra_split, cbf_cb, cbf_cr, cm, cux, cuy, log2cb);
        transform_tree(x0, y0 + h, x0, y0, log2n - 1, depth + 1, 2, max_depth, intra_split, cbf_cb, cbf_cr, cm, cux, cuy, log2cb);
        transform_tree(x0 + h, y0 + h, x0, y0, log2n - 1, depth + 1, 3, max_depth, intra_split, cbf_cb, cbf_cr, cm, cux, cuy, log2cb);
    } else {
        int cbf_l = dec(C_CBF_LUMA + (depth == 0 ? 1 : 0));
        transform_unit(x0, y0, xb, yb, log2n, blk, cbf_l, cbf_cb, cbf_cr, cm, cux, cuy, log2cb);
    }
}

void HevcParser::pcm_sample(int x0, int y0, int log2cb) {
    const uint8_t* p = cc_.aligned_pos();
    BitReader b(p, static_cast<size_t>(end_ - p));
    const int n = 1 << log2cb;
    const int bd = s_->bit_depth;
    uint8_t fl = edge_flags(x0, y0) | H2J_TU_PCM | H2J_TU_CBF;
    if (s_->pcm_lf_disabled) fl |= H2J_TU_NOFILT;
    for (int c = 0; c < 3; c++) {
        const int cn = c ? n / 2 : n;
        h2j_tu tu;
        tu.x = static_cast<uint16_t>(c ? x0 / 2 : x0);
        tu.y = static_cast<uint16_t>(c ? y0 / 2 : y0);
        // PCM blocks can be 64x64 luma; split into <=32x32 records
        const int sub = cn > 32 ? 32 : cn;
        for (int sy = 0; sy < cn; sy += sub)
            for (int sx = 0; sx < cn; sx += sub) {
                h2j_tu t = tu;
                t.x = static_cast<uint16_t>(tu.x + sx);
                t.y = static_cast<uint16_t>(tu.y + sy);
                t.log2n = static_cast<uint8_t>(sub == 32 ? 5 : (sub == 16 ? 4 : (sub == 8 ? 3 : 2)));
                t.c = static_cast<uint8_t>(c);
                t.mode = 1;
                t.flags = c == 0 ? fl : static_cast<uint8_t>(H2J_TU_PCM | H2J_TU_CBF | (fl & H2J_TU_NOFILT));
                if (c == 0 && (sx || sy)) {
                    t.flags = static_cast<uint8_t>((t.flags & ~(H2J_TU_EDGE_L | H2J_TU_EDGE_T)) |
                                                   (edge_flags(x0 + sx, y0 + sy) & ((sx ? 0 : H2J_TU_EDGE_L) | (sy ? 0 : H2J_TU_EDGE_T))));
                }
                t.qp = 0;
                t.qpy = 0;
                t.coef = static_cast<uint32_t>(job_->coefs.size()) - job_->hdr.coef;
                t.ncoef = static_cast<uint16_t>(sub * sub);
                job_->tus.push_back(t);
                for (int k = 0; k < sub * sub; k++) job_->coefs.push_back(0);
            }
    }
    // samples are stored in raster order of the whole CU per component: fill
    // the records just pushed in bitstream order
    size_t tu_end = job_->tus.size();
    int recs_y = (n > 32) ? 4 : 1;
    size_t first = tu_end - static_cast<size_t>(recs_y + 2);
    for (int c = 0; c < 3; c++) {
        const int cn = c ? n / 2 : n;
        const int pbd = c ? s_->pcm_bd_c : s_->pcm_bd;
        const int sub = cn > 32 ? 32 : cn;
        for (int y = 0; y < cn; y++)
            for (int x = 0; x < cn; x++) {
                int v = static_cast<int>(b.u(pbd)) << (bd - pbd);
                size_t rec = first + (c == 0 ? static_cast<size_t>((y / sub) * (cn / sub) + x / sub) : static_cast<size_t>(recs_y + c - 1));
                const h2j_tu& t = job_->tus[rec];
                int pos = (y % sub) * sub + (x % sub);
                job_->coefs[job_->hdr.coef + t.coef + pos] = (static_cast<uint32_t>(pos) << 16) | static_cast<uint16_t>(v);
            }
    }
    cc_.init(p + b.byte_pos(), end_);
}

void HevcParser::coding_unit(int x0, int y0, int log2cb) {
    const int n = 1 << log2cb;
    cu_tu_begin_ = static_cast<int>(job_->tus.size());
    cu_bypass_ = 0;
    if (p_->transquant_bypass) cu_bypass_ = dec(C_TQ_BYPASS);
    int part_nxn = 0;
    if (log2cb == s_->log2_min_cb) part_nxn = !dec(C_PART_MODE);
    qp_y_ = qp_wrap(qg_pred_ + qpd_val_ + 52 + 2 * qpbd) - qpbd;
    set_qp(x0, y0, n, qp_y_);
    int pcm = 0;
    if (!part_nxn && s_->pcm && log2cb >= s_->log2_min_pcm && log2cb <= s_->log2_max_pcm) pcm = cc_.terminate();
    if (pcm) {
        set_map(ipm_, x0, y0, n, 1);
        pcm_sample(x0, y0, log2cb);
    } else {
        const int np = part_nxn ? 4 : 1, pb = part_nxn ? n / 2 : n;
        int prev[4], mpm[4] = {0, 0, 0, 0}, rem[4] = {0, 0, 0, 0};
        for (int i = 0; i < np; i++) prev[i] = dec(C_PREV_INTRA);
        for (int i = 0; i < np; i++) {
            if (prev[i]) {
                if (cc_.bypass()) mpm[i] = cc_.bypass() ? 2 : 1;
            } else {
                rem[i] = static_cast<int>(cc_.bypass_bits(5));
            }
        }
        for (int i = 0; i < np; i++) {
            const int xp = x0 + (i & 1) * pb, yp = y0 + (i >> 1) * pb;
            int ca = 1, cb = 1;
            if (same_region(xp, yp, xp - 1, yp)) ca = ipm_[(yp >> 2) * mw + ((xp - 1) >> 2)];
            if (same_region(xp, yp, xp, yp - 1) && ((yp - 1) >> log2ctb) == (yp >> log2ctb))
                cb = ipm_[((yp - 1) >> 2) * mw + (xp >> 2)];
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
                if (cand[0] > cand[1]) std::swap(cand[0], cand[1]);
                if (cand[0] > cand[2]) std::swap(cand[0], cand[2]);
                if (cand[1] > cand[2]) std::swap(cand[1], cand[2]);
                mode = rem[i];
                for (int k = 0; k < 3; k++)
                    if (mode >= cand[k]) mode++;
            }
            set_map(ipm_, xp, yp, pb, static_cast<uint8_t>(mode));
        }
        int icpm = 4;
        if (dec(C_CHROMA_MODE)) icpm = static_cast<int>(cc_.bypass_bits(2));
        const int lm = ipm_[(y0 >> 2) * mw + (x0 >> 2)];
        int cm;
        if (icpm == 4) cm = lm;
        else {
            static const int cmodes[4] = {0, 26, 10, 1};
            cm = cmodes[icpm] == lm ? 34 : cmodes[icpm];
        }
        transform_tree(x0, y0, x0, y0, log2cb, 0, 0, s_->max_th_depth_intra + part_nxn, part_nxn, 0, 0, cm, x0, y0, log2cb);
    }
    // patch the CU's QP into its transform blocks (QpY is final now; so are CuQpOffsetCb / Cr for
    // every chroma block with a residual: the offsets are coded before the CU's first chroma cbf)
    const int qpy = qp_y_ + qpbd;
    int qpc[2];
    for (int k = 0; k < 2; k++) {
        int off = k == 0 ? p_->cb_qp_offset + cur_->cb_qp_offset + cu_qo_cb_
                         : p_->cr_qp_offset + cur_->cr_qp_offset + cu_qo_cr_;
        int qpi = qp_y_ + off;
        if (qpi < -qpbd) qpi = -qpbd;
        if (qpi > 57) qpi = 57;
        qpc[k] = chroma_qp_table(qpi) + qpbd;
    }
    for (size_t t = static_cast<size_t>(cu_tu_begin_); t < job_->tus.size(); t++) {
        h2j_tu& tu = job_->tus[t];
        tu.qpy = static_cast<int8_t>(qp_y_);
        tu.qp = static_cast<int8_t>(tu.c == 0 ? qpy : qpc[tu.c - 1]);
    }
    last_cu_qp_ = qp_y_;
}

void HevcParser::coding_quadtree(int x0, int y0, int log2cb, int depth) {
    if (err_) return;
    const int n = 1 << log2cb;
    int split;
    if (x0 + n <= W && y0 + n <= H && log2cb > s_->log2_min_cb) {
        int inc = 0;
        if (same_region(x0, y0, x0 - 1, y0) && ctd_[(y0 >> 2) * mw + ((x0 - 1) >> 2)] > depth) inc++;
        if (same_region(x0, y0, x0, y0 - 1) && ctd_[((y0 - 1) >> 2) * mw + (x0 >> 2)] > depth) inc++;
        split = dec(C_SPLIT_CU + inc);
    } else {
        split = log2cb > s_->log2_min_cb;
    }
    if ((p_->cu_qp_delta && log2cb >= log2ctb - p_->diff_cu_qp_delta_depth) || (!p_->cu_qp_delta && log2cb == log2ctb))
        qg_start(x0, y0);
    if (cur_->cu_chroma_qp_offset_enabled && log2cb >= log2ctb - p_->cqo_depth) cqo_coded_ = false;
    if (split) {
        const int h = n >> 1;
        coding_quadtree(x0, y0, log2cb - 1, depth + 1);
        if (x0 + h < W) coding_quadtree(x0 + h, y0, log2cb - 1, depth + 1);
        if (y0 + h < H) coding_quadtree(x0, y0 + h, log2cb - 1, depth + 1);
        if (x0 + h < W && y0 + h < H) coding_quadtree(x0 + h, y0 + h, log2cb - 1, depth + 1);
    } else {
        set_map(ctd_, x0, y0, n, static_cast<uint8_t>(depth));
        coding_unit(x0, y0, log2cb);
    }
}

void HevcParser::ctb_start_contexts(int rs, int ts, bool first) {
    const int rx = rs % ctbW;
    const int x0 = rx << log2ctb, y0 = (rs / ctbW) << log2ctb;
    const bool tile_start = ts == 0 || tile_id_[ts] != tile_id_[ts - 1];
    bool row_start = false;
    if (p_->wpp)
        for (size_t i = 0; i + 1 < col_bd_.size(); i++)
            if (rx == col_bd_[i]) row_start = true;
    if (!(first || tile_start || row_start)) return;
    if (tile_start) {
        init_contexts(cur_->slice_qp);
    } else if (row_start) {
        const int xr = x0 + ctbs, yr = y0 - ctbs;
        if (xr < W && yr >= 0 && same_region(x0, y0, xr, yr)) {
            std::memcpy(ctx_, ctx_wpp_, sizeof(ctx_));
            std::memcpy(stat_, stat_wpp_, sizeof(stat_));
        } else {
            init_contexts(cur_->slice_qp);
        }
    } else if (cur_->dependent && have_ds_) {
        std::memcpy(ctx_, ctx_ds_, sizeof(ctx_));
        std::memcpy(stat_, stat_ds_, sizeof(stat_));
    } else {
        init_contexts(cur_->slice_qp);
    }
    // qPY_PREV = SliceQpY for the first QG of a tile / of a CTB row under WPP (8.6.1), also
    // when qg_start runs again for a QG smaller than the CTB
    if (tile_start || row_start) {
        first_qg_ = true;
        last_cu_qp_ = cur_->slice_qp;
    }
}

int HevcParser::decode_slice_data(int shi, const uint8_t* p, const uint8_t* end) {
    const SliceHdr& sh = sh_[shi];
    cur_ = &sh;
    cur_idx_ = shi;
    end_ = end;
    cc_.init(p, end);
    int rs = sh.address, ts = rs2ts_[rs];
    if (!sh.dependent) {
        first_qg_ = true;
        last_cu_qp_ = sh.slice_qp;
        cu_qo_cb_ = cu_qo_cr_ = 0;
    }
    bool first = true;
    for (;;) {
        const int rx = rs % ctbW, ry = rs / ctbW;
        ctb_slice_[rs] = shi;
        ctb_addr_rs_[rs] = sh.slice_addr_rs;
        ctb_start_contexts(rs, ts, first);
        first = false;
        parse_sao(rx, ry);
        const size_t first_tu = job_->tus.size();
        coding_quadtree(rx << log2ctb, ry << log2ctb, log2ctb, 0);
        if (err_) return err_;
        // the CTB's luma TBs first, then its chroma TBs, each in z-scan order: the GPU
        // reconstructs the luma and the chroma chains in separate workgroups
        split_ctb_records(first_tu);
        int endf = cc_.terminate();
        if (p_->wpp) {
            for (size_t i = 0; i + 1 < col_bd_.size(); i++)
                if (rx == col_bd_[i] + 1 && col_bd_[i] + 1 < col_bd_[i + 1]) {
                    std::memcpy(ctx_wpp_, ctx_, sizeof(ctx_));
                    std::memcpy(stat_wpp_, stat_, sizeof(stat_));
                }
        }
        ts++;
        if (endf) break;
        if (ts >= nctb) return -30;
        const int nrs = ts2rs_[ts];
        const bool new_tile = tile_id_[ts] != tile_id_[ts - 1];
        bool new_row = false;
        if (p_->wpp)
            for (size_t i = 0; i + 1 < col_bd_.size(); i++)
                if (nrs % ctbW == col_bd_[i]) new_row = true;
        if (new_tile || new_row) {
            cc_.terminate();
            cc_.init(cc_.aligned_pos(), end);
        }
        rs = nrs;
    }
    std::memcpy(ctx_ds_, ctx_, sizeof(ctx_));
    std::memcpy(stat_ds_, stat_, sizeof(stat_));
    have_ds_ = true;
    return 0;
}

// WPP (entropy_coding_sync) rows of one slice decoded side by side: row r may parse CTB x
// once row r-1 has finished CTB x+1 (its contexts after CTB 1 seed row r, 9.3.1 / 9.3.2.4;
// split-flag, availability and SAO-merge neighbours lie at most one CTB up and to the right).
struct HevcParser::WppRows {
    std::unique_ptr<std::atomic<int>[]> done;      // per row: CTBs finished
    std::vector<std::array<CabacState, NUM_CTX>> ctx;  // per row: contexts after its 2nd CTB
    std::vector<std::array<int, 4>> stat;              // per row: StatCoeff after its 2nd CTB
    std::atomic<bool> failed{false};
};

int HevcParser::decode_wpp_row(int shi, int row, const uint8_t* p, const uint8_t* end, WppRows& w) {
    const SliceHdr& sh = sh_[shi];
    cur_ = &sh;
    cur_idx_ = shi;
    end_ = end;
    cc_.init(p, end);
    first_qg_ = true;  // qPY_PREV = SliceQpY at a WPP row start (8.6.1)
    last_cu_qp_ = sh.slice_qp;
    cu_qo_cb_ = cu_qo_cr_ = 0;  // a chroma QP offset group never spans CTBs: the value never carries
    for (int rx = 0; rx < ctbW; rx++) {
        const int rs = row * ctbW + rx;
        if (row > 0) {
            const int need = std::min(rx + 2, ctbW);
            for (int spin = 0; w.done[row - 1].load(std::memory_order_acquire) < need; spin++) {
                if (w.failed.load(std::memory_order_relaxed)) return -31;
                if (spin > 64) std::this_thread::yield();
            }
        }
        ctb_slice_[rs] = shi;
        ctb_addr_rs_[rs] = sh.slice_addr_rs;
        if (rx == 0) {
            if (row > 0 && ctbW > 1) {
                std::memcpy(ctx_, w.ctx[row - 1].data(), sizeof(ctx_));
                std::memcpy(stat_, w.stat[row - 1].data(), sizeof(stat_));
            } else {
                init_contexts(sh.slice_qp);
            }
        }
        parse_sao(rx, row);
        const size_t first_tu = job_->tus.size();
        coding_quadtree(rx << log2ctb, row << log2ctb, log2ctb, 0);
        if (err_) return err_;
        split_ctb_records(first_tu);
        const int endf = cc_.terminate();
        if (rx == 1) {
            std::memcpy(w.ctx[row].data(), ctx_, sizeof(ctx_));
            std::memcpy(w.stat[row].data(), stat_, sizeof(stat_));
        }
        w.done[row].store(rx + 1, std::memory_order_release);
        if (endf != (row == ctbH - 1 && rx == ctbW - 1)) return -30;
    }
    return 0;
}

// seg: the slice's data; sub: each row's substream start in it (from the entry points)
int HevcParser::run_wpp(const std::vector<uint8_t>& seg, const std::vector<uint32_t>& sub, int threads) {
    WppRows w;
    w.done.reset(new std::atomic<int>[ctbH]);
    for (int r = 0; r < ctbH; r++) w.done[r].store(0);
    w.ctx.resize(ctbH);
    w.stat.resize(ctbH);
    std::vector<FrameJob> part(ctbH);
    const int nt = std::min(threads, ctbH);
    std::vector<std::unique_ptr<HevcParser>> wk(nt);
    for (int t = 0; t < nt; t++) {
        wk[t].reset(new HevcParser(*this, true));
        wk[t]->p_ = &wk[t]->pps_[sh_[0].pps_id];
        wk[t]->s_ = &wk[t]->sps_[wk[t]->p_->sps_id];
    }
    const uint8_t* end = seg.data() + (seg.size() - 8);
    std::vector<int> rc(ctbH, 0);
    std::atomic<int> next(0);
    // rows are claimed in order, so every row waited on is already being decoded
    auto work = [&](HevcParser& P) {
        for (int r = next++; r < ctbH; r = next++) {
            P.job_ = &part[r];
            P.err_ = 0;
            rc[r] = P.decode_wpp_row(0, r, seg.data() + sub[r], end, w);
            if (rc[r] < 0) {
                w.failed.store(true);
                w.done[r].store(ctbW, std::memory_order_release);
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work, std::ref(*wk[t]));
    work(*wk[0]);
    for (auto& t : pool) t.join();
    for (int r = 0; r < ctbH; r++)
        if (rc[r] < 0) return rc[r];
    merge_parts(part);
    return 0;
}

// records of the parts appended in decoding order
void HevcParser::merge_parts(const std::vector<FrameJob>& part) {
    for (const FrameJob& pj : part) {
        const uint32_t cbase = static_cast<uint32_t>(job_->coefs.size());
        for (h2j_tu t : pj.tus) {
            if (t.ncoef) t.coef += cbase;  // (records without coefficients keep coef 0)
            job_->tus.push_back(t);
        }
        job_->coefs.insert(job_->coefs.end(), pj.coefs.begin(), pj.coefs.end());
    }
}

// One tile of a slice (CTBs ts0..ts1-1 in tile scan): no parsing dependency on any other
// tile (contexts initialised at the tile start, neighbours across tiles unavailable, 6.4.1).
int HevcParser::decode_tile(int shi, int ts0, int ts1, bool last, const uint8_t* p, const uint8_t* end) {
    const SliceHdr& sh = sh_[shi];
    cur_ = &sh;
    cur_idx_ = shi;
    end_ = end;
    cc_.init(p, end);
    init_contexts(sh.slice_qp);
    first_qg_ = true;
    last_cu_qp_ = sh.slice_qp;
    cu_qo_cb_ = cu_qo_cr_ = 0;
    for (int ts = ts0; ts < ts1; ts++) {
        const int rs = ts2rs_[ts];
        parse_sao(rs % ctbW, rs / ctbW);
        const size_t first_tu = job_->tus.size();
        coding_quadtree((rs % ctbW) << log2ctb, (rs / ctbW) << log2ctb, log2ctb, 0);
        if (err_) return err_;
        split_ctb_records(first_tu);
        if (cc_.terminate() != (last && ts == ts1 - 1)) return -30;
    }
    return 0;
}

// A single slice split into tiles (no WPP): its tiles in parallel from the entry points.
int HevcParser::run_tiles(const std::vector<uint8_t>& seg, const std::vector<uint32_t>& sub, int threads) {
    const int nt = static_cast<int>(sub.size());
    std::vector<int> t0(nt + 1, nctb);
    for (int ts = 0, t = 0; ts < nctb; ts++)
        if (ts == 0 || tile_id_[ts] != tile_id_[ts - 1]) t0[t++] = ts;
    // the slice covers the picture: its CTB ownership is known up front (deblocking-edge
    // flags compare slice addresses across tile borders)
    for (int rs = 0; rs < nctb; rs++) {
        ctb_slice_[rs] = 0;
        ctb_addr_rs_[rs] = sh_[0].slice_addr_rs;
    }
    std::vector<FrameJob> part(nt);
    const int nw = std::min(threads, nt);
    std::vector<std::unique_ptr<HevcParser>> wk(nw);
    for (int w = 0; w < nw; w++) {
        wk[w].reset(new HevcParser(*this, true));
        wk[w]->p_ = &wk[w]->pps_[sh_[0].pps_id];
        wk[w]->s_ = &wk[w]->sps_[wk[w]->p_->sps_id];
    }
    const uint8_t* end = seg.data() + (seg.size() - 8);
    std::vector<int> rc(nt, 0);
    std::atomic<int> next(0);
    auto work = [&](HevcParser& P) {
        for (int t = next++; t < nt; t = next++) {
            P.job_ = &part[t];
            P.err_ = 0;
            rc[t] = P.decode_tile(0, t0[t], t0[t + 1], t == nt - 1, seg.data() + sub[t], end);
        }
    };
    std::vector<std::thread> pool;
    for (int w = 1; w < nw; w++) pool.emplace_back(work, std::ref(*wk[w]));
    work(*wk[0]);
    for (auto& t : pool) t.join();
    for (int t = 0; t < nt; t++)
        if (rc[t] < 0) return rc[t];
    merge_parts(part);
    return 0;
}

int HevcParser::run(const uint8_t* data, size_t size, int threads) {
    init_scans();
    std::vector<Nal> nals;
    split_annexb(data, size, nals);
    rbsp_.resize(size + 16);
    bool have_pic = false;
    const SliceHdr* prev = nullptr;
    sh_.reserve(256);
    std::vector<std::vector<uint8_t>> seg;  // per slice segment: its slice data (+8 zero bytes)
    std::vector<std::vector<uint32_t>> seg_sub;  // per slice segment: substream starts in it
    for (const Nal& nal : nals) {
        if (nal.n < 2) continue;
        const int type = (nal.p[0] >> 1) & 63;
        const size_t rn = unescape_rbsp(nal.p + 2, nal.n - 2, rbsp_.data());
        BitReader b(rbsp_.data(), rn);
        if (type == 33) {
            if (have_pic) break;
            const int e = parse_sps(b, sps_);
            if (e < 0) {
                job_->message = e == -12 ? "unsupported bit depth (FFmpeg 4.3 has no HEVC 4:2:0 format at it)"
                                         : "unsupported or invalid SPS";
                return -2;
            }
        } else if (type == 34) {
            if (have_pic) break;
            if (parse_pps(b, pps_, sps_) < 0) { job_->message = "invalid PPS"; return -3; }
        } else if (type <= 21) {
            if (type >= 10 && type <= 15) continue;
            const int first = (rbsp_[0] >> 7) & 1;
            if (first && have_pic) break;
            if (!first && !have_pic) continue;
            if (sh_.size() >= 255) { job_->message = "too many slices"; return -4; }
            sh_.push_back(SliceHdr());
            SliceHdr& sh = sh_.back();
            int r = parse_slice_header(b, type, sh, prev);
            if (r < 0) {
                job_->message = r == -2 ? "non-intra first picture (P/B slices) unsupported" : "invalid slice header";
                return r == -2 ? -5 : -6;
            }
            if (!have_pic) {
                p_ = &pps_[sh.pps_id];
                s_ = &sps_[p_->sps_id];
                if (!setup_picture()) { job_->message = "invalid tile grid"; return -6; }
                job_->reorder_delay = s_->num_reorder_pics > 0;
                have_pic = true;
            }
            // all slice segments of a picture use one PPS (7.4.7.1; FFmpeg: "PPS changed between
            // slices"): tiles, entry points and the SAO / deblocking layout come from it
            if (&pps_[sh.pps_id] != p_) { job_->message = "PPS change inside picture"; return -6; }
            if (&sps_[p_->sps_id] != s_) { job_->message = "SPS change inside picture"; return -6; }
            // slice data: the RBSP after the header, kept for the decode pass
            const size_t off = b.byte_pos();
            if (off > rn) { job_->message = "truncated slice"; return -6; }
            seg.emplace_back(rbsp_.begin() + static_cast<long>(off), rbsp_.begin() + static_cast<long>(rn));
            seg.back().resize(seg.back().size() + 8, 0);
            seg_sub.emplace_back();
            if (!sh.entry.empty()) {
                // entry points count escaped bytes: map them into the unescaped slice data
                const uint8_t* src = nal.p + 2;
                std::vector<size_t> epb;  // escaped positions of emulation-prevention bytes
                int zeros = 0;
                for (size_t i = 0; i < nal.n - 2; i++) {
                    if (zeros >= 2 && src[i] == 3) {
                        epb.push_back(i);
                        zeros = 0;
                        continue;
                    }
                    zeros = src[i] == 0 ? zeros + 1 : 0;
                }
                size_t e = off, j = 0;
                while (j < epb.size() && epb[j] <= e) { e++; j++; }
                std::vector<uint32_t>& su = seg_sub.back();
                su.push_back(0);
                for (uint32_t len : sh.entry) {
                    e += len;
                    while (j < epb.size() && epb[j] < e) j++;
                    const size_t u = e - j - off;
                    if (u >= rn - off) { su.clear(); break; }  // inconsistent: decode sequentially
                    su.push_back(static_cast<uint32_t>(u));
                }
            }
            h2j_slice rec{};
            rec.beta_offset = static_cast<int8_t>(sh.beta_offset);
            rec.tc_offset = static_cast<int8_t>(sh.tc_offset);
            rec.sao_luma = static_cast<uint8_t>(sh.sao_luma);
            rec.sao_chroma = static_cast<uint8_t>(sh.sao_chroma);
            rec.lf_across_slices = static_cast<uint8_t>(sh.lf_across_slices);
            rec.deblock_disabled = static_cast<uint8_t>(sh.deblock_disabled);
            rec.slice_addr_rs = sh.slice_addr_rs;
            job_->slices.push_back(rec);
            prev = &sh_.back();
        } else if (type == 35 && have_pic) {
            break;
        }
    }
    if (!have_pic) { job_->message = "no picture found"; return -8; }
    // Slice groups: an independent slice segment and the dependent segments that continue it.
    // Groups share nothing for parsing (CABAC restarts, neighbours in other slices are
    // unavailable, 6.4.1), so with threads > 1 they decode side by side: group 0 into this
    // job, the others into their own jobs, appended in decoding order.
    std::vector<int> gs;
    for (size_t i = 0; i < sh_.size(); i++)
        if (i == 0 || !sh_[i].dependent) gs.push_back(static_cast<int>(i));
    gs.push_back(static_cast<int>(sh_.size()));
    const int ng = static_cast<int>(gs.size()) - 1;
    auto decode_group = [&](HevcParser& P, int g) -> int {
        for (int i = gs[g]; i < gs[g + 1]; i++) {
            const std::vector<uint8_t>& d = seg[i];
            P.p_ = &P.pps_[P.sh_[i].pps_id];  // this parser's own copies of the parameter sets
            P.s_ = &P.sps_[P.p_->sps_id];
            const int e = P.decode_slice_data(i, d.data(), d.data() + (d.size() - 8));
            if (e < 0) return e;
        }
        return 0;
    };
    if (threads > 1 && ng == 1 && sh_.size() == 1 && p_->wpp && !p_->tiles && sh_[0].address == 0 && ctbH > 1 &&
        seg_sub[0].size() == static_cast<size_t>(ctbH)) {
        // one WPP slice (the usual single-slice x265 picture): its CTB rows in parallel
        if (run_wpp(seg[0], seg_sub[0], threads) < 0) { job_->message = "slice data decode error"; return -7; }
    } else if (threads > 1 && ng == 1 && sh_.size() == 1 && p_->tiles && !p_->wpp && sh_[0].address == 0 &&
               !seg_sub[0].empty() && seg_sub[0].size() == static_cast<size_t>(tile_id_[nctb - 1] + 1)) {
        // one slice of several tiles: the tiles in parallel
        if (run_tiles(seg[0], seg_sub[0], threads) < 0) { job_->message = "slice data decode error"; return -7; }
    } else if (threads <= 1 || ng <= 1) {
        for (int g = 0; g < ng; g++)
            if (decode_group(*this, g) < 0) { job_->message = "slice data decode error"; return -7; }
    } else {
        std::vector<FrameJob> part(ng);
        std::vector<std::unique_ptr<HevcParser>> wk(ng);
        for (int g = 1; g < ng; g++) {  // clones first: group 0 then mutates this parser's maps
            part[g].ctbs = job_->ctbs;
            wk[g].reset(new HevcParser(*this, part[g]));
        }
        std::vector<int> rc(ng, 0);
        std::atomic<int> next(1);
        auto work = [&]() {
            for (int g = next++; g < ng; g = next++) rc[g] = decode_group(*wk[g], g);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < std::min(threads, ng); t++) pool.emplace_back(work);
        rc[0] = decode_group(*this, 0);
        work();
        for (auto& t : pool) t.join();
        for (int g = 0; g < ng; g++)
            if (rc[g] < 0) { job_->message = "slice data decode error"; return -7; }
        for (int g = 1; g < ng; g++) {
            const uint32_t cbase = static_cast<uint32_t>(job_->coefs.size());
            for (h2j_tu t : part[g].tus) {
                if (t.ncoef) t.coef += cbase;  // (records without coefficients keep coef 0)
                job_->tus.push_back(t);
            }
            job_->coefs.insert(job_->coefs.end(), part[g].coefs.begin(), part[g].coefs.end());
            for (int rs = 0; rs < nctb; rs++)
                if (wk[g]->ctb_slice_[rs] >= gs[g] && wk[g]->ctb_slice_[rs] < gs[g + 1]) job_->ctbs[rs] = part[g].ctbs[rs];
        }
    }
    job_->hdr.nslice = static_cast<uint32_t>(job_->slices.size());
    {
        bool multi = job_->slices.size() != 1 || job_->slices[0].slice_addr_rs != 0;
        for (size_t i = 0; i < tile_id_.size() && !multi; i++) multi = tile_id_[i] != 0;
        job_->hdr.topo = multi ? 1u : 0u;
    }
    job_->hdr.ntu = static_cast<uint32_t>(job_->tus.size());
    return 0;
}

}  // namespace

int hevc_parse_picture(const uint8_t* data, size_t size, FrameJob& job) {
    job.clear();
    std::unique_ptr<HevcParser> p(new HevcParser(job));  // large (parameter-set tables): heap
    int r = p->run(data, size, job.threads);
    job.error = r;
    return r;
}

}  // namespace h2j
