// MI355X (gfx950, CDNA4, wave64) pixel pipeline for the H.264/H.265 still -> JPEG hot path.
// Hand-written HIP; integer work only (no MFMA: 4-32-point fixed transforms and filters,
// latency / HBM bound).  Stages, one launch each per chunk of pictures:
//
//   K0 h2j_k0_prep<codec>   one lane per transform-block record: availability masks, CTB /
//                           MB record ranges, deblocking maps, PCM samples; dequantisation +
//                           inverse DCT/DST batched by TB size (lane = TB column, then row)
//                           into the int16 residual plane (H.265 8.6.2-8.6.4, H.264 8.5)
//   K1 h2j_k1_recon_*       intra prediction + residual add along the dependency chains:
//                           HEVC picture pool (a 16-wave workgroup reconstructs up to 4
//                           pictures; waves take CTB-row jobs -- a picture's luma or Cb/Cr
//                           chain -- from an LDS queue, rows run as a wavefront, 32x32
//                           quadrant windows in LDS prefetched by LDS-DMA); H.264 one workgroup
//                           per picture or 16-MB-row band, MB-row wavefront in LDS windows
//                           (H.265 8.4.4.2, H.264 8.3)
//   K2 h2j_k2_deblock*      HEVC: one thread per 4-line edge segment, V then H pass;
//                           H.264: MB-row wavefront in LDS windows, banded like K1
//                           (H.265 8.7.2, H.264 8.7)
//   K3 h2j_k3_sao           one workgroup per CTB (Y, Cb, Cr), all loads issued up front, LDS tiles + border (H.265 8.7.3)
//   K4 h2j_k4_*             FFmpeg mjpeg forward path as restated in SURVEY.md Appendix A:
//                           pad, MB variance -> rate control -> AP-922 FDCT -> 16-bit
//                           quantiser -> zigzag, then per-table symbol histograms
//   (K5, optimal Huffman tables + bitstream emission, lives in h2j_entropy.hip)
//
// Reference call sites replaced: /root/reference/src/Decoder.cpp:324,342
// (avcodec_send_packet / avcodec_receive_frame) and /root/reference/src/Encoder.cpp:250
// (avcodec_send_frame, mjpeg).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <mutex>
#include <utility>
#include <vector>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "h2j_gpu.h"
#include "grid.h"
#include "jpeg_tile.h"

#define DEVI __device__ __forceinline__

namespace {

// ---------------------------------------------------------------- helpers
DEVI int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

struct FV {  // frame view
    const h2j_frame* f;
    uint8_t* arena;
    const h2j_ctb* ctbs;
    const h2j_slice* slices;
};

template <typename Pel>
DEVI Pel* plane(const h2j_frame& f, uint8_t* arena, uint64_t base, int c) {
    return reinterpret_cast<Pel*>(arena + base) + f.pic_off[c];
}

// 6.4.1 z-scan availability (luma coordinates)
DEVI bool avail(const h2j_frame& f, const h2j_ctb* ctbs, const h2j_slice* slices, int xc, int yc, int xn,
                int yn) {
    if (xn < 0 || yn < 0 || xn >= f.width || yn >= f.height) return false;
    const int l2 = f.log2ctb;
    const int cn = (yn >> l2) * f.ctb_w + (xn >> l2);
    const int cc = (yc >> l2) * f.ctb_w + (xc >> l2);
    if (cn == cc) {
        const int m = (1 << l2) - 1;
        int ax = (xn & m) >> 2, ay = (yn & m) >> 2, bx = (xc & m) >> 2, by = (yc & m) >> 2;
        int za = 0, zb = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            za |= (((ax >> i) & 1) << (2 * i)) | (((ay >> i) & 1) << (2 * i + 1));
            zb |= (((bx >> i) & 1) << (2 * i)) | (((by >> i) & 1) << (2 * i + 1));
        }
        return za <= zb;
    }
    const h2j_ctb& A = ctbs[cn];
    const h2j_ctb& B = ctbs[cc];
    if (A.ts > B.ts) return false;
    if (slices[A.slice].slice_addr_rs != slices[B.slice].slice_addr_rs) return false;
    return A.tile == B.tile;
}

// HEVC 32x32 inverse transform matrix entries from the 33 distinct cosines
__constant__ int kLevelScale[6] = {40, 45, 51, 57, 64, 72};
// the 32x32 HEVC DCT matrix (8.6.4.2, transMatrix), built at compile time from the 33 cosines
// above; an N-point transform uses rows j * 32 / N (packed into kDctPk below).
struct DctMat {
    int v[32][32];
};
constexpr DctMat make_dct32() {
    constexpr int c[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                           61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
    DctMat t{};
    for (int m = 0; m < 32; m++)
        for (int k = 0; k < 32; k++) {
            int a = ((2 * k + 1) * m) & 127;
            if (a > 64) a = 128 - a;
            t.v[m][k] = a > 32 ? -c[64 - a] : c[a];
        }
    return t;
}

// Paired-input layout of the batched HEVC inverse transforms (hevc_residual_group): the inputs
// j of one N-point pass sit as int16 pairs in dwords, ordered the way the even/odd decomposition
// consumes them -- slots [0, N/8): rows 0 mod 8 with 4 mod 8 (EE), [N/8, N/4): 2 mod 8 with 6
// mod 8 (EO), [N/4, N/2): 1 mod 4 with 3 mod 4 (O); N = 4: (0, 1), (2, 3) -- so one
// v_dot2c_i32_i16 (2 multiply-adds) consumes a dword against a packed pair of matrix entries.
template <int N>
__host__ __device__ constexpr int k0_pslot(int j) {
    return N == 4 ? (j >> 1)
           : (j & 1) ? N / 4 + (j >> 2)
           : (j & 3) == 0 ? (j >> 3)
                          : N / 8 + (j >> 3);
}
template <int N>
__host__ __device__ constexpr int k0_phalf(int j) {
    return N == 4 ? (j & 1) : (j & 1) ? ((j >> 1) & 1) : ((j >> 2) & 1);
}
// packed matrix entries (c(j0, i) in the low half, c(j1, i) in the high half) of slot s, output
// i, for N = 4 << L (c = the rows of transMatrix an N-point transform uses); DST 4x4 apart
struct DctPk {
    int v[4][16][16];
    int dst[2][4];
};
constexpr DctPk make_dct_pk() {
    DctPk t{};
    const DctMat m = make_dct32();
    for (int L = 0; L < 4; L++) {
        const int N = 4 << L, sh = 3 - L;
        for (int s = 0; s < N / 2; s++) {
            int j0 = 0, j1 = 0;
            if (N == 4) { j0 = 2 * s; j1 = j0 + 1; }
            else if (s < N / 8) { j0 = 8 * s; j1 = j0 + 4; }
            else if (s < N / 4) { j0 = 8 * (s - N / 8) + 2; j1 = j0 + 4; }
            else { j0 = 4 * (s - N / 4) + 1; j1 = j0 + 2; }
            for (int i = 0; i < 16 && i < N; i++)
                t.v[L][s][i] = static_cast<int>((static_cast<unsigned>(m.v[j0 << sh][i]) & 0xFFFFu) |
                                                (static_cast<unsigned>(m.v[j1 << sh][i]) << 16));
        }
    }
    constexpr int d[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
    for (int s = 0; s < 2; s++)
        for (int i = 0; i < 4; i++)
            t.dst[s][i] = static_cast<int>((static_cast<unsigned>(d[2 * s][i]) & 0xFFFFu) |
                                           (static_cast<unsigned>(d[2 * s + 1][i]) << 16));
    return t;
}
__constant__ DctPk kDctPk = make_dct_pk();
typedef short s16x2 __attribute__((ext_vector_type(2)));
// acc + lo(a) * lo(b) + hi(a) * hi(b), int16 halves, int32 accumulation (v_dot2c_i32_i16)
__device__ __forceinline__ int dot2(int a, int b, int acc) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), acc, false);
}

// ---------------------------------------------------------------- K1: H.264
// H.264 8.3 (intra prediction), 8.5 (scaling + transforms).  Records: luma
// log2n 2 (I4x4), 3 (I8x8), 4 (I16x16, DC levels at (4i,4j)); chroma log2n 3
// (DC levels at (4i,4j)); PCM.  Macroblocks are the "CTB" records (log2ctb 4).
__constant__ int kNorm4[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
__constant__ int kNorm8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                                     {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};

// m (= qP % 6) is uniform: the table row is read with scalar loads, the
// position class is selected per lane
DEVI int h264_norm4(int m, int i, int j) {
    const int n0 = kNorm4[m][0], n1 = kNorm4[m][1], n2 = kNorm4[m][2];
    return (!(i & 1) && !(j & 1)) ? n0 : (((i & 1) && (j & 1)) ? n1 : n2);
}
DEVI int h264_norm8(int m, int i, int j) {
    const int n0 = kNorm8[m][0], n1 = kNorm8[m][1], n2 = kNorm8[m][2], n3 = kNorm8[m][3], n4 = kNorm8[m][4],
              n5 = kNorm8[m][5];
    if (!(i & 3) && !(j & 3)) return n0;
    if ((i & 1) && (j & 1)) return n1;
    if ((i & 3) == 2 && (j & 3) == 2) return n2;
    if ((!(i & 3) && (j & 1)) || ((i & 1) && !(j & 3))) return n3;
    if ((!(i & 3) && (j & 3) == 2) || ((i & 3) == 2 && !(j & 3))) return n4;
    return n5;
}
DEVI int h264_scale4(int lvl, int ls, int qp) {
    return qp >= 24 ? (lvl * ls) << (qp / 6 - 4) : (lvl * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
}
DEVI int h264_scale8(int lvl, int ls, int qp) {
    return qp >= 36 ? (lvl * ls) << (qp / 6 - 6) : (lvl * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
}

DEVI bool h264_avail(const h2j_frame& f, const h2j_ctb* mbs, const h2j_slice* slices, int xc, int yc, int xn, int yn) {
    if (xn < 0 || yn < 0 || xn >= f.width || yn >= f.height) return false;
    const int cn = (yn >> 4) * f.ctb_w + (xn >> 4), cc = (yc >> 4) * f.ctb_w + (xc >> 4);
    if (cn == cc) {
        const int ax = (xn & 15) >> 2, ay = (yn & 15) >> 2, bx = (xc & 15) >> 2, by = (yc & 15) >> 2;
        const int za = (ax & 1) | ((ay & 1) << 1) | ((ax & 2) << 1) | ((ay & 2) << 2);
        const int zb = (bx & 1) | ((by & 1) << 1) | ((bx & 2) << 1) | ((by & 2) << 2);
        return za < zb;
    }
    if (cn > cc) return false;
    const h2j_ctb& A = mbs[cn];
    if (!(A.mbflags & 4)) return false;
    return slices[A.slice].slice_addr_rs == slices[mbs[cc].slice].slice_addr_rs;
}

// 4x4 / 8x8 directional prediction; T[-1] / L[-1] = corner
DEVI int h264_pred_nxn(int mode, int x, int y, int n, const int* T, const int* L, int dcv) {
    switch (mode) {
    case 0: return T[x];
    case 1: return L[y];
    case 2: return dcv;
    case 3:
        if (x == n - 1 && y == n - 1) return (T[2 * n - 2] + 3 * T[2 * n - 1] + 2) >> 2;
        return (T[x + y] + 2 * T[x + y + 1] + T[x + y + 2] + 2) >> 2;
    case 4:
        if (x > y) return (T[x - y - 2] + 2 * T[x - y - 1] + T[x - y] + 2) >> 2;
        if (x < y) return (L[y - x - 2] + 2 * L[y - x - 1] + L[y - x] + 2) >> 2;
        return (T[0] + 2 * T[-1] + L[0] + 2) >> 2;
    case 5: {
        const int z = 2 * x - y;
        if (z >= 0 && !(z & 1)) return (T[x - (y >> 1) - 1] + T[x - (y >> 1)] + 1) >> 1;
        if (z >= 0) return (T[x - (y >> 1) - 2] + 2 * T[x - (y >> 1) - 1] + T[x - (y >> 1)] + 2) >> 2;
        if (z == -1) return (L[0] + 2 * T[-1] + T[0] + 2) >> 2;
        if (n == 4) return (L[y - 1] + 2 * L[y - 2] + L[y - 3] + 2) >> 2;
        return (L[y - 2 * x - 1] + 2 * L[y - 2 * x - 2] + L[y - 2 * x - 3] + 2) >> 2;
    }
    case 6: {
        const int z = 2 * y - x;
        if (z >= 0 && !(z & 1)) return (L[y - (x >> 1) - 1] + L[y - (x >> 1)] + 1) >> 1;
        if (z >= 0) return (L[y - (x >> 1) - 2] + 2 * L[y - (x >> 1) - 1] + L[y - (x >> 1)] + 2) >> 2;
        if (z == -1) return (L[0] + 2 * T[-1] + T[0] + 2) >> 2;
        if (n == 4) return (T[x - 1] + 2 * T[x - 2] + T[x - 3] + 2) >> 2;
        return (T[x - 2 * y - 1] + 2 * T[x - 2 * y - 2] + T[x - 2 * y - 3] + 2) >> 2;
    }
    case 7: {
        const int i = x + (y >> 1);
        return !(y & 1) ? (T[i] + T[i + 1] + 1) >> 1 : (T[i] + 2 * T[i + 1] + T[i + 2] + 2) >> 2;
    }
    default: {
        const int z = x + 2 * y, lim = 2 * n - 3;
        if (z > lim) return L[n - 1];
        if (z == lim) return (L[n - 2] + 3 * L[n - 1] + 2) >> 2;
        const int i = y + (x >> 1);
        return !(z & 1) ? (L[i] + L[i + 1] + 1) >> 1 : (L[i] + 2 * L[i + 1] + L[i + 2] + 2) >> 2;
    }
    }
}

// ---------------------------------------------------------------- K0: per-TU preparation
// Everything about a transform block that does not depend on reconstructed
// neighbour samples, for every TU of the batch in parallel: the reference
// availability mask, the CTB -> TU range, the HEVC deblocking maps, PCM
// samples, and the residual (dequantisation + inverse transform) into an
// int16 plane.  K1 then only walks the serial prediction chain.
constexpr int kK0Tus = 62;  // H.264 TUs per K0 wave (records held one per lane)
// lanes kTus and kTus + 1 hold the neighbour records of a wave's range (h2j_k0_prep)
static_assert(kK0Tus >= 1 && kK0Tus <= 62, "K0 records per wave: 62 at most");
constexpr int kK0TusHevc = 62;  // HEVC: 62 records + the two neighbours of the range in lanes 62, 63
constexpr int kK1WavesWide = 16;  // HEVC K1, launches of <= 128 pictures: waves per group (one group per CU)
constexpr int kAvcWaves = 16;  // waves of the MBAFF / mixed-batch K1 workgroups (macroblock rows in flight)
// H.264 K1 (h2j_k1_recon_h264): 8-wave workgroups, two per CU (LDS), so one picture's last row
// round -- rows left over after the waves' full rounds -- overlaps the other workgroup's work
constexpr int kAvcK1Waves = 8;

struct K0Lds {    // H.264
    int blk[32 * 32];  // up to 4 Intra16x16 MBs' levels ([G][16][16], h264_i16_group)
    int tmp[512];      // row-pass output: at most 8 8x8 / 16 4x4 blocks ([G][N][N])
    int dc[16];
};                     // 6.2 KB: 5 waves per SIMD (the 95-VGPR limit) instead of 4.5 (LDS)
// HEVC: the column pass's output (int16 rows padded to N + 2, bank-conflict-free
// transposition) overlays the dequantised coefficients it was computed from (every lane holds
// its column's sums in registers across a wave barrier): 4.3 KB instead of 8.5 KB per wave, so
// the VGPR limit (6 waves per SIMD at 79 VGPRs), not LDS (4.5), bounds the occupancy
struct K0LdsHevc {
    union {
        int blk[32 * 32];
        int tmp[32 * 34];
    };
};


// Wave-wide integer sum with DPP row shifts + row broadcasts (no LDS trip);
// call with all 64 lanes active.
DEVI int wave_sum_dpp(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return __builtin_amdgcn_readlane(x, 63);
}

// lanes of one wave exchanging data through LDS
DEVI void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Device-side failure flags of a picture (h2j_jstat.dev_error): a wait that never completes flags
// its picture and gives up instead of hanging the GPU.
enum : uint32_t {
    kDevErrK1Band = 1u,       // H.264 K1: band hand-off (global flag) timed out
    kDevErrDbBand = 2u,       // H.264 deblocking: band hand-off timed out
    kDevErrK1Row = 4u,        // HEVC K1: row progress word (LDS) timed out
    kDevErrK1Row264 = 8u,     // H.264 K1: row progress word timed out
    kDevErrDbRow264 = 16u,    // H.264 deblocking: row progress word timed out
};
DEVI uint32_t* dev_error_word(uint8_t* arena, const h2j_frame& f) {
    return reinterpret_cast<uint32_t*>(arena + (static_cast<uint64_t>(f.jstat) + offsetof(h2j_jstat, dev_error)));
}
// Wait (s_sleep polling, workgroup scope, acquire) until the LDS progress word reaches `need`.
// Legitimate waits end within one picture's reconstruction (milliseconds); after 2^24 polls
// (~0.4 s) the picture is flagged with `bit` and the wait returns ~0u, so every later wait of the
// row passes and the workgroup drains.
DEVI uint32_t wait_progress(const uint32_t* word, uint32_t need, uint32_t* err, uint32_t bit) {
    uint32_t seen, it = 0;
    while ((seen = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < need) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1u << 24)) {
            if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            seen = ~0u;
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return seen;
}

// Optional K1 cycle accounting (build with -DH2J_PROF: `make prof`), read via h2j_gpu_prof().
#ifdef H2J_PROF
__device__ unsigned long long g_prof[16];
#define PROF_T() __builtin_amdgcn_s_memtime()
// Accumulators per wave in LDS, added to by lane 0 (r02 kept 16 64-bit accumulators in registers:
// that build of the pool kernel, already at its register limit with SGPR spills, never finished)
#define PROF_DECL                                                                                  \
    __shared__ unsigned long long prof_acc_[16][16];                                               \
    unsigned long long* const pacc_ = prof_acc_[threadIdx.x >> 6];                                 \
    if ((threadIdx.x & 63) < 16) pacc_[threadIdx.x & 63] = 0;                                      \
    unsigned long long pt0 = PROF_T(), pt1;                                                        \
    const unsigned long long prt0 = __builtin_amdgcn_s_memrealtime(), pmt0 = pt0
#define PROF_ADD(i, v) do { if ((threadIdx.x & 63) == 0) pacc_[i] += (v); } while (0)
#define PROF_LAP(i) do { pt1 = PROF_T(); PROF_ADD(i, pt1 - pt0); pt0 = pt1; } while (0)
#define PROF_LAPK(k) do { pt1 = PROF_T(); PROF_ADD(8 + ((k) < 7 ? (k) : 7), pt1 - pt0); pt0 = pt1; } while (0)
#define PROF_FLUSH() do { PROF_ADD(4, __builtin_amdgcn_s_memrealtime() - prt0); PROF_ADD(7, PROF_T() - pmt0); \
    if ((threadIdx.x & 63) < 16) atomicAdd(&g_prof[threadIdx.x & 63], pacc_[threadIdx.x & 63]); } while (0)
#else
#define PROF_DECL
#define PROF_ADD(i, v)
#define PROF_LAP(i)
#define PROF_LAPK(k)
#define PROF_FLUSH()
#endif
// H.264: the counters go to the deblocking pair kernel (default) or, with -DH2J_PROF_AVCK1, to K1
#if defined(H2J_PROF) && defined(H2J_PROF_AVCK1)
#define AVP_DECL PROF_DECL
#define AVP_LAP(i) PROF_LAP(i)
#define AVP_LAPK(k) PROF_LAPK(k)
#define AVP_ADD(i, v) PROF_ADD(i, v)
#define AVP_FLUSH() PROF_FLUSH()
#define DBP_DECL
#define DBP_LAP(i)
#define DBP_LAPK(k)
#define DBP_ADD(i, v)
#define DBP_FLUSH()
#else
#define AVP_DECL
#define AVP_LAP(i)
#define AVP_LAPK(k)
#define AVP_ADD(i, v)
#define AVP_FLUSH()
#define DBP_DECL PROF_DECL
#define DBP_LAP(i) PROF_LAP(i)
#define DBP_LAPK(k) PROF_LAPK(k)
#define DBP_ADD(i, v) PROF_ADD(i, v)
#define DBP_FLUSH() PROF_FLUSH()
#endif

// uniform values into scalar registers; records held one per lane, read with readlane
DEVI uint32_t ufl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
DEVI uint64_t ufl64(uint64_t v) {
    return (static_cast<uint64_t>(ufl(static_cast<uint32_t>(v >> 32))) << 32) | ufl(static_cast<uint32_t>(v));
}

// a record at a wave-uniform address, read as dwords into scalar registers (byte fields would
// otherwise be re-read with per-lane byte loads at every use)
template <typename T>
DEVI T uload(const T* p) {
    static_assert(sizeof(T) % 4 == 0 && alignof(T) >= 4, "dword-aligned records only");
    uint32_t w[sizeof(T) / 4];
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int k = 0; k < static_cast<int>(sizeof(T) / 4); k++) w[k] = ufl(q[k]);
    T t;
    memcpy(&t, w, sizeof(T));
    return t;
}

DEVI h2j_tu tu_from_lanes(const uint4& r, int l) {
    uint32_t w[4];
    w[0] = __builtin_amdgcn_readlane(r.x, l);
    w[1] = __builtin_amdgcn_readlane(r.y, l);
    w[2] = __builtin_amdgcn_readlane(r.z, l);
    w[3] = __builtin_amdgcn_readlane(r.w, l);
    h2j_tu t;
    memcpy(&t, w, sizeof(t));
    return t;
}

DEVI uint64_t mask_from_lanes(const uint2& m, int l) {
    return static_cast<uint64_t>(__builtin_amdgcn_readlane(m.x, l)) |
           (static_cast<uint64_t>(__builtin_amdgcn_readlane(m.y, l)) << 32);
}


// HEVC dequantisation (8.6.2-8.6.3) + transform skip / bypass (8.6.4) of one TB
// into R (int16, stride rst); regular transforms: hevc_residual_group.
struct K0F {  // frame fields K0 uses, in scalar registers (see FU)
    int bd, bdc, slist, log2ctb, ctb_w, width, height, mw, topo, rext;
    uint32_t sl;
};
// 24-bit signed multiply (v_mul_i32_i24, full rate; v_mul_lo_u32 is quarter rate) for index
// arithmetic whose operands fit 24 bits (sample / block coordinates, strides, small factors)
DEVI int m24(int a, int b) { return __mul24(a, b); }

// Sample (x, y) of component c in the tiled HEVC residual planes (h2j_res_q, include/h2j_gpu.h);
// rows of a tile are 1 << h2j_res_q(log2ctb, c) elements apart.
DEVI int16_t* hevc_res_at(int16_t* res, int width, int height, int log2ctb, int c, int x, int y) {
    const int q = h2j_res_q(log2ctb, c), qm = (1 << q) - 1;
    const int wc = c ? width >> 1 : width;
    long long base = 0;
    if (c) {
        base = h2j_res_plane(width, height, h2j_res_q(log2ctb, 0));
        if (c == 2) base += h2j_res_plane(width >> 1, height >> 1, q);
    }
    const long long tile = static_cast<long long>(y >> q) * h2j_res_tiles(wc, q) + (x >> q);
    return res + base + (tile << (2 * q)) + ((y & qm) << q) + (x & qm);
}
// Sample (x, y) of component c in the H.264 residual, tiled by macroblock: MB m (raster order)
// holds its 16x16 luma, then 8x8 Cb, 8x8 Cr residual, 384 int16 (768 B) back to back, so K1
// fetches an MB as one contiguous piece (h264_rows).  Rows of a block are 16 (luma) / 8 (chroma)
// elements apart.
DEVI int16_t* h264_res_at(int16_t* res, int mbw, int c, int x, int y) {
    // (24-bit multiplies and a 32-bit byte offset from the uniform base: r05)
    const int o = c == 0 ? m24(m24(y >> 4, mbw) + (x >> 4), 384) + ((y & 15) << 4) + (x & 15)
                         : m24(m24(y >> 3, mbw) + (x >> 3), 384) + 256 + (c - 1) * 64 + ((y & 7) << 3) + (x & 7);
    return reinterpret_cast<int16_t*>(reinterpret_cast<uint8_t*>(res) + static_cast<uint32_t>(o) * 2u);
}
// H.264 MBAFF frames keep TU records and MB records in the macroblock grid (grid row = 2 * pair row
// + bottom); a field macroblock's row r is picture row 2 * r + bottom of its pair (h2j_ctb.mbflags
// bit 3).  Picture row of grid row y (component c: 16 / 8 rows per MB).
DEVI int h264_mbaff_row(const h2j_ctb* C, int mbw, int c, int x, int y) {
    const int sh = c ? 3 : 4, vy = y >> sh, r = y & ((1 << sh) - 1);
    const bool fld = (C[vy * mbw + (x >> sh)].mbflags & 8) != 0;
    return fld ? (((vy >> 1) << (sh + 1)) + 2 * r + (vy & 1)) : y;
}
DEVI void hevc_residual(const K0F& f, const h2j_tu& tu, const h2j_coef* CO, uint32_t co0, const uint8_t* sl,
                        int16_t* R, int rst, K0LdsHevc& s) {
    const int lane = threadIdx.x;
    const int c = tu.c, log2n = tu.log2n, n = 1 << log2n, nn = n * n;
    const int bd = c ? f.bdc : f.bd;
    const uint8_t flags = tu.flags;
    for (int i = lane; i < nn; i += 64) s.blk[i] = 0;
    wave_sync();
    const bool bypass = (flags & H2J_TU_BYPASS) != 0;
    const int qp = tu.qp;
    const int bdShift = bd + log2n - 5;
    const int ls = kLevelScale[qp % 6] << (qp / 6);
    const uint8_t* slt = nullptr;
    if (f.slist && !((flags & H2J_TU_TSKIP) && n > 4)) {
        const int soff = log2n == 2 ? 0 + c * 16 : (log2n == 3 ? 48 + c * 64 : (log2n == 4 ? 240 + c * 256 : 1008));
        slt = sl + f.sl + soff;
    }
    for (int e = lane; e < tu.ncoef; e += 64) {
        const uint32_t en = e < 64 ? co0 : CO[tu.coef + e];  // first 64 entries prefetched
        const int pos = static_cast<int>(en >> 16);
        const int lvl = static_cast<int16_t>(en & 0xFFFF);
        int d;
        if (bypass) {
            d = lvl;
        } else {
            const int m = slt ? slt[pos] : 16;
            long long v = static_cast<long long>(lvl) * m * ls;
            v = (v + (1ll << (bdShift - 1))) >> bdShift;
            d = static_cast<int>(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
        }
        s.blk[pos] = d;
    }
    wave_sync();
    if (!bypass) {  // transform skip (regular transforms run batched: hevc_residual_group)
        if ((f.rext & H2J_REXT_TS_ROT) && n == 4) {  // RExt rotation: r[x][y] = d[3-x][3-y]
            const int v = lane < 16 ? s.blk[15 - lane] : 0;
            wave_sync();
            if (lane < 16) s.blk[lane] = v;
            wave_sync();
        }
        // tsShift = 5 + log2n then bdShift = 20 - bitDepth (RExt 8.6.4.2): one shift by
        // 15 - bitDepth - log2n, left (int16 wrap) when negative, as FFmpeg's dequant()
        const int sh = 15 - bd - log2n;
        for (int i = lane; i < nn; i += 64)
            s.blk[i] = sh > 0 ? (s.blk[i] + (1 << (sh - 1))) >> sh : static_cast<int16_t>(s.blk[i] * (1 << -sh));
    }
    wave_sync();
    if ((f.rext & H2J_REXT_RDPCM) && (tu.mode == 10 || tu.mode == 26)) {
        // RExt implicit RDPCM (transform skip and bypass): the residual accumulates down the
        // columns (mode 26) / along the rows (mode 10), int16 as FFmpeg's coefficient buffer
        const bool vert = tu.mode == 26;
        if (lane < n) {
            int acc = 0;
            for (int k = 0; k < n; k++) {
                const int i = vert ? k * n + lane : lane * n + k;
                acc = static_cast<int16_t>(acc + s.blk[i]);
                s.blk[i] = acc;
            }
        }
        wave_sync();
    }
    for (int i = lane; i < nn; i += 64) R[(i >> log2n) * rst + (i & (n - 1))] = static_cast<int16_t>(s.blk[i]);
    wave_sync();
}

// HEVC dequantisation + inverse DCT/DST (8.6.2-8.6.4) of up to 64 / N same-size TBs of one wave
// at once: lane = (TB slot, column) in the column pass, (TB slot, row) in the row pass, so no lane
// idles on small TBs.  Each lane keeps its N partial sums in registers and walks the non-zero
// input rows / columns (bounded by the group's largest coefficient position); the matrix row of a
// step is uniform (scalar loads).  The intermediate goes through LDS (int16), the result straight
// to the residual plane.  `gm`: record lanes of the group's G TBs (slot g = g-th set bit).
// TS: 4x4 transform-skip TBs (no rotation / RDPCM in the picture), 16 per pass: the dequantised
// level shifted by tsShift + bdShift (8.6.4.2) is the residual.  Bypass TBs and the other
// transform-skip TBs are not batched (hevc_residual).
template <int LOG2N, bool TS = false>
DEVI void hevc_residual_group(const K0F& f, const uint4& rec, uint64_t gm, int G, const h2j_coef* CO,
                              const uint8_t* sl, int16_t* res, K0LdsHevc& s) {
    static_assert(!TS || LOG2N == 2, "batched transform skip: 4x4 TBs only");
    constexpr int N = 1 << LOG2N, NN = N * N;
    constexpr int P = N + 2, NP = N * P;  // tmp row stride (int16): odd dword stride across lanes
    const int lane = threadIdx.x;
    int16_t* blk = reinterpret_cast<int16_t*>(s.blk);  // [G][N/2 slots][N columns][2] dequantised coefficients
    int16_t* tmp = reinterpret_cast<int16_t*>(s.tmp);  // [G][N rows][P] after the column pass, columns paired
    for (int i = lane * 8; i < G * NN; i += 512) *reinterpret_cast<uint4*>(blk + i) = make_uint4(0, 0, 0, 0);
    wave_sync();
    int mx = 0, my = 0;
    {
        // the group's coefficients in one round: lane = (TB g of the group, sub-lane), 64 / Gmax
        // sub-lanes per TB, each taking entries sub, sub + LPT, ... -- every load of the group is in
        // flight at once (r06: a loop over the G TBs waited out one global-load latency per TB; the
        // 150 KB configs[1] pictures carry ~16k 4x4 TBs with residual each)
        constexpr int LPT = N;          // lanes per TB: the group holds 64 / N TBs of N x N
        constexpr int GMAX = 64 / LPT;
        constexpr int EPL = NN / LPT;   // entries per lane (a TB has at most NN)
        constexpr int CH = EPL < 4 ? EPL : 4;  // loads in flight per lane and round (K0 runs at 72 VGPRs)
        const int g = lane / LPT, sub = lane % LPT;
        uint64_t mg = gm;
        for (int i = 0; i < g && i < GMAX; i++) mg &= mg - 1;
        const int kg = mg ? __ffsll(static_cast<long long>(mg)) - 1 : 0;
        const bool live = g < G;
        const uint32_t w1 = __shfl(rec.y, kg, 64), w2 = __shfl(rec.z, kg, 64), w3 = __shfl(rec.w, kg, 64);
        uint32_t wq[4] = {0u, w1, w2, w3};
        h2j_tu tu;
        memcpy(&tu, wq, sizeof(tu));
        const int c = tu.c, bd = c ? f.bdc : f.bd, qp = tu.qp;
        const int bdShift = bd + LOG2N - 5;
        const long long ls = static_cast<long long>(kLevelScale[qp % 6] << (qp / 6));
        const uint8_t* slt = f.slist ? sl + f.sl + (LOG2N == 2 ? c * 16 : LOG2N == 3 ? 48 + c * 64 : LOG2N == 4 ? 240 + c * 256 : 1008)
                                     : nullptr;
        const int nco = live ? static_cast<int>(tu.ncoef) : 0;
        int ncm = nco;  // the group's largest entry count: rounds past it load nothing
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ncm = max(ncm, __shfl_xor(ncm, o, 64));
        const int rounds = (ufl(ncm) + LPT - 1) / LPT;
        for (int r0 = 0; r0 < rounds; r0 += CH) {
            uint32_t en[CH];
#pragma unroll
            for (int j = 0; j < CH; j++) {
                const int e = sub + (r0 + j) * LPT;
                en[j] = e < nco ? CO[tu.coef + e] : 0u;
            }
#pragma unroll
            for (int j = 0; j < CH; j++) {
                if (sub + (r0 + j) * LPT >= nco) continue;
                const int pos = static_cast<int>(en[j] >> 16);
                const int lvl = static_cast<int16_t>(en[j] & 0xFFFF);
                const int m = slt ? slt[pos] : 16;
                long long v = static_cast<long long>(lvl) * m * ls;
                v = (v + (1ll << (bdShift - 1))) >> bdShift;
                const int d = static_cast<int>(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
                if constexpr (TS) {  // tsShift = 5 + log2n, bdShift = 20 - bitDepth: one right shift (>= 1 up to 12 bits)
                    const int sh = 15 - bd - LOG2N;
                    blk[g * NN + pos] = static_cast<int16_t>((d + (1 << (sh - 1))) >> sh);
                } else {
                    const int jr = pos >> LOG2N, xc = pos & (N - 1);
                    blk[g * NN + 2 * (k0_pslot<N>(jr) * N + xc) + k0_phalf<N>(jr)] = static_cast<int16_t>(d);
                    mx = max(mx, pos & (N - 1));
                    my = max(my, pos >> LOG2N);
                }
            }
        }
    }
    if constexpr (TS) {  // rows straight from LDS: lane = (TB, row)
        wave_sync();
        const int g = lane >> LOG2N, q = lane & (N - 1);
        uint64_t ml = gm;
        for (int i = 0; i < g && i < G - 1; i++) ml &= ml - 1;
        const int k = __ffsll(static_cast<long long>(ml)) - 1;
        // (shuffles with every lane active: a bpermute from a lane outside the exec mask reads garbage)
        const uint32_t w0 = __shfl(rec.x, k, 64), w1 = __shfl(rec.y, k, 64), w2 = __shfl(rec.z, k, 64);
        uint32_t wq[4] = {w0, w1, w2, 0};
        h2j_tu mine;
        memcpy(&mine, wq, sizeof(mine));
        if (g < G) {
            int16_t* R = hevc_res_at(res, f.width, f.height, f.log2ctb, mine.c, mine.x, mine.y) + (q << h2j_res_q(f.log2ctb, mine.c));
            *reinterpret_cast<uint2*>(R) = *reinterpret_cast<const uint2*>(blk + g * NN + q * N);
        }
        wave_sync();
        return;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mx = max(mx, __shfl_xor(mx, o, 64));
        my = max(my, __shfl_xor(my, o, 64));
    }
    const int mxx = ufl(mx), myy = ufl(my);
    wave_sync();
    // this lane's TB: its record lives in lane k of `rec`
    const int g = lane >> LOG2N, q = lane & (N - 1);
    const bool act = g < G;
    uint64_t ml = gm;
    for (int i = 0; i < g && i < G - 1; i++) ml &= ml - 1;
    const int k = __ffsll(static_cast<long long>(ml)) - 1;
    const uint32_t w0 = __shfl(rec.x, k, 64), w1 = __shfl(rec.y, k, 64), w2 = __shfl(rec.z, k, 64);
    uint32_t wq[4] = {w0, w1, w2, 0};
    h2j_tu mine;
    memcpy(&mine, wq, sizeof(mine));
    const bool dst = LOG2N == 2 && (mine.flags & H2J_TU_DST) != 0;
    // One pass of the N-point inverse transform over inputs 0..jmax: acc[i] = sum_j M[j][i] * in(j),
    // the inputs read as paired dwords (k0_pslot) and consumed two per v_dot2c_i32_i16.  DCT rows
    // are even / odd symmetric (M[j][N-1-i] = (-1)^j M[j][i]), so for N >= 8 the even and odd
    // input rows each feed N/2 partial sums: E[i] +/- O[i], and the even half splits once more
    // into rows 0 mod 4 (EE) and 2 mod 4 (EO).  Slots past jmax hold zeros, so a slot whose first
    // input is <= jmax is taken whole.
    constexpr int L = LOG2N - 2;
    auto pass = [&](int jmax, auto inpair, int (&acc)[N]) __attribute__((always_inline)) {
        if constexpr (N >= 8) {
            int E[N / 2], O[N / 2], EE[N / 4], EO[N / 4];
#pragma unroll
            for (int i = 0; i < N / 2; i++) O[i] = 0;
#pragma unroll
            for (int i = 0; i < N / 4; i++) EE[i] = EO[i] = 0;
            for (int ps = 0; ps < N / 8 && 8 * ps <= jmax; ps++) {
                const int v = inpair(ps);
#pragma unroll
                for (int i = 0; i < N / 4; i++) EE[i] = dot2(kDctPk.v[L][ps][i], v, EE[i]);
            }
            for (int ps = 0; ps < N / 8 && 8 * ps + 2 <= jmax; ps++) {
                const int v = inpair(N / 8 + ps);
#pragma unroll
                for (int i = 0; i < N / 4; i++) EO[i] = dot2(kDctPk.v[L][N / 8 + ps][i], v, EO[i]);
            }
#pragma unroll
            for (int i = 0; i < N / 4; i++) {
                E[i] = EE[i] + EO[i];
                E[N / 2 - 1 - i] = EE[i] - EO[i];
            }
            for (int ps = 0; ps < N / 4 && 4 * ps + 1 <= jmax; ps++) {
                const int v = inpair(N / 4 + ps);
#pragma unroll
                for (int i = 0; i < N / 2; i++) O[i] = dot2(kDctPk.v[L][N / 4 + ps][i], v, O[i]);
            }
#pragma unroll
            for (int i = 0; i < N / 2; i++) {
                acc[i] = E[i] + O[i];
                acc[N - 1 - i] = E[i] - O[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < N; i++) acc[i] = 0;
            for (int ps = 0; ps < 2 && 2 * ps <= jmax; ps++) {
                const int v = inpair(ps);
#pragma unroll
                for (int i = 0; i < N; i++) acc[i] = dot2(dst ? kDctPk.dst[ps][i] : kDctPk.v[0][ps][i], v, acc[i]);
            }
        }
    };
    const int* blk32 = reinterpret_cast<const int*>(blk);
    const int* tmp32 = reinterpret_cast<const int*>(tmp);
    const int qcol = 2 * k0_pslot<N>(q) + k0_phalf<N>(q);  // this lane's column in the paired tmp rows
    {  // columns: tmp[y][x] = clip16((sum_j M[j][y] * d[j][x] + 64) >> 7)
        int acc[N];
        if (act) pass(myy, [&](int ps) { return blk32[g * (NN / 2) + ps * N + q]; }, acc);
        wave_sync();  // tmp overlays blk (K0LdsHevc): every column has been read
        if (act) {
#pragma unroll
            for (int i = 0; i < N; i++) tmp[g * NP + i * P + qcol] = static_cast<int16_t>(clip3(-32768, 32767, (acc[i] + 64) >> 7));
        }
    }
    wave_sync();
    if (act) {  // rows: r[y][x] = (sum_j M[j][x] * tmp[y][j] + rnd) >> (20 - bitDepth)
        int acc[N];
        pass(mxx, [&](int ps) { return tmp32[(g * NP + q * P) / 2 + ps]; }, acc);
        const int bdS = 20 - (mine.c ? f.bdc : f.bd);
        const int c = mine.c;
        int16_t* R = hevc_res_at(res, f.width, f.height, f.log2ctb, c, mine.x, mine.y) + (q << h2j_res_q(f.log2ctb, c));
        uint32_t packed[N / 2];
#pragma unroll
        for (int i = 0; i < N / 2; i++) {
            const int a = (acc[2 * i] + (1 << (bdS - 1))) >> bdS, b = (acc[2 * i + 1] + (1 << (bdS - 1))) >> bdS;
            packed[i] = (static_cast<uint32_t>(a) & 0xFFFF) | (static_cast<uint32_t>(b) << 16);
        }
        if (N == 4) {
            *reinterpret_cast<uint2*>(R) = make_uint2(packed[0], packed[1]);
        } else {
#pragma unroll
            for (int i = 0; i < N / 8; i++)
                reinterpret_cast<uint4*>(R)[i] = make_uint4(packed[4 * i], packed[4 * i + 1], packed[4 * i + 2], packed[4 * i + 3]);
        }
    }
    wave_sync();
}

// H.264 scaling (8.5.9, 8.5.10-8.5.12 DC transforms) + 4x4 / 8x8 inverse
// transforms (8.5.12.2, 8.5.13) of one record into R.
// 8-point H.264 inverse transform butterfly (8.5.13.2), one row or column
DEVI void h264_idct8_1d(const int (&d)[8], int (&o)[8]) {
    const int a0 = d[0] + d[4], a4 = d[0] - d[4], a2 = (d[2] >> 1) - d[6], a6 = d[2] + (d[6] >> 1);
    const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
    const int a1 = -d[3] + d[5] - d[7] - (d[7] >> 1), a3 = d[1] + d[7] - d[3] - (d[3] >> 1);
    const int a5 = -d[1] + d[7] + d[5] + (d[5] >> 1), a7 = d[3] + d[5] + d[1] + (d[1] >> 1);
    const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
    o[0] = b0 + b7; o[1] = b2 + b5; o[2] = b4 + b3; o[3] = b6 + b1;
    o[4] = b6 - b1; o[5] = b4 - b3; o[6] = b2 - b5; o[7] = b0 - b7;
}

DEVI void h264_residual(const K0F& f, const h2j_tu& tu, const h2j_coef* CO, uint32_t co0, const uint8_t* sl,
                        int16_t* R, int rst, K0Lds& s) {
    const int lane = threadIdx.x;
    const int c = tu.c, log2n = tu.log2n, n = 1 << log2n, nn = n * n;
    const int qp = tu.qp, qm = qp % 6;
    const bool i16 = c == 0 && log2n == 4;
    const bool chroma = c > 0;
    for (int i = lane; i < nn; i += 64) s.blk[i] = 0;
    wave_sync();
    for (int e = lane; e < tu.ncoef; e += 64) {
        const uint32_t en = e < 64 ? co0 : CO[tu.coef + e];
        s.blk[en >> 24] = static_cast<int>(en << 8) >> 8;  // H2J_COEF264: 24-bit level
    }
    wave_sync();
    if (tu.flags & H2J_TU_BYPASS) {
        // TransformBypassModeFlag: the residual is the levels (DC levels included, at (4i, 4j));
        // vertical / horizontal intra predictions accumulate it down the columns / along the
        // rows of the whole block (8.5.15), one lane per column / row
        const bool dv = tu.flags & H2J_TU_DPCM_V, dh = tu.flags & H2J_TU_DPCM_H;
        if ((dv || dh) && lane < n) {
            int acc = 0;
            for (int k = 0; k < n; k++) {
                const int i = dv ? k * n + lane : lane * n + k;
                acc += s.blk[i];
                s.blk[i] = acc;
            }
        }
        wave_sync();
        for (int i = lane; i < nn; i += 64) R[(i >> log2n) * rst + (i & (n - 1))] = static_cast<int16_t>(s.blk[i]);
        wave_sync();
        return;
    }
    const uint8_t* w4 = f.slist ? sl + f.sl + c * 16 : nullptr;
    if (i16 || chroma) {
        // DC transform (Hadamard 4x4 / 2x2) on the levels at (4i, 4j)
        const int nb = n >> 2;  // blocks per side: 4 (luma) / 2 (chroma)
        if (lane < nb * nb) {
            const int r = lane / nb, q = lane % nb;
            int acc = 0;
            for (int i = 0; i < nb; i++)
                for (int j = 0; j < nb; j++) {
                    const int hr = nb == 4 ? ((r == 0 || (r == 1 && i < 2) || (r == 2 && (i == 0 || i == 3)) || (r == 3 && !(i & 1))) ? 1 : -1)
                                           : ((r == 0 || i == 0) ? 1 : -1);
                    const int hc = nb == 4 ? ((q == 0 || (q == 1 && j < 2) || (q == 2 && (j == 0 || j == 3)) || (q == 3 && !(j & 1))) ? 1 : -1)
                                           : ((q == 0 || j == 0) ? 1 : -1);
                    acc += hr * hc * s.blk[(i * 4) * n + j * 4];
                }
            const int ls0 = (w4 ? w4[0] : 16) * kNorm4[qm][0];
            int v;
            if (nb == 4) v = qp >= 36 ? (acc * ls0) << (qp / 6 - 6) : (acc * ls0 + (1 << (5 - qp / 6))) >> (6 - qp / 6);
            else v = ((acc * ls0) << (qp / 6)) >> 5;
            s.dc[lane] = v;
        }
        wave_sync();
        for (int i = lane; i < nn; i += 64) {
            const int y = i >> log2n, x = i & (n - 1);
            const int by = y >> 2, bx = x >> 2, ry = y & 3, rx = x & 3;
            if (ry == 0 && rx == 0) s.blk[i] = s.dc[by * (n >> 2) + bx];
            else s.blk[i] = h264_scale4(s.blk[i], (w4 ? w4[ry * 4 + rx] : 16) * h264_norm4(qm, ry, rx), qp);
        }
    } else if (log2n == 2) {
        for (int i = lane; i < 16; i += 64)
            s.blk[i] = h264_scale4(s.blk[i], (w4 ? w4[i] : 16) * h264_norm4(qm, i >> 2, i & 3), qp);
    } else {
        const uint8_t* w8 = f.slist ? sl + f.sl + 48 : nullptr;
        for (int i = lane; i < 64; i += 64)
            s.blk[i] = h264_scale8(s.blk[i], (w8 ? w8[i] : 16) * h264_norm8(qm, i >> 3, i & 7), qp);
    }
    wave_sync();
    if (log2n == 3 && !chroma) {
        // 8x8 inverse transform: rows (lanes 0..7) then columns
        for (int pass = 0; pass < 2; pass++) {
            if (lane < 8) {
                int d[8], o[8];
                for (int k = 0; k < 8; k++) d[k] = pass == 0 ? s.blk[lane * 8 + k] : s.tmp[k * 8 + lane];
                h264_idct8_1d(d, o);
                if (pass == 0) for (int k = 0; k < 8; k++) s.tmp[lane * 8 + k] = o[k];
                else for (int k = 0; k < 8; k++) s.blk[k * 8 + lane] = (o[k] + 32) >> 6;
            }
            wave_sync();
        }
    } else {
        // 4x4 inverse transforms of all 4x4 blocks: lane = block * 4 + row/col
        const int nb = n >> 2, nblk = nb * nb;
        for (int pass = 0; pass < 2; pass++) {
            for (int id = lane; id < nblk * 4; id += 64) {
                const int b = id >> 2, k = id & 3;
                const int bx = (b % nb) * 4, by = (b / nb) * 4;
                int d0, d1, d2, d3;
                if (pass == 0) {
                    const int* r = &s.blk[(by + k) * n + bx];
                    d0 = r[0]; d1 = r[1]; d2 = r[2]; d3 = r[3];
                } else {
                    d0 = s.tmp[(by + 0) * n + bx + k]; d1 = s.tmp[(by + 1) * n + bx + k];
                    d2 = s.tmp[(by + 2) * n + bx + k]; d3 = s.tmp[(by + 3) * n + bx + k];
                }
                const int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
                if (pass == 0) {
                    int* o = &s.tmp[(by + k) * n + bx];
                    o[0] = e0 + e3; o[1] = e1 + e2; o[2] = e1 - e2; o[3] = e0 - e3;
                } else {
                    s.blk[(by + 0) * n + bx + k] = (e0 + e3 + 32) >> 6;
                    s.blk[(by + 1) * n + bx + k] = (e1 + e2 + 32) >> 6;
                    s.blk[(by + 2) * n + bx + k] = (e1 - e2 + 32) >> 6;
                    s.blk[(by + 3) * n + bx + k] = (e0 - e3 + 32) >> 6;
                }
            }
            wave_sync();
        }
    }
    for (int i = lane; i < nn; i += 64) R[(i >> log2n) * rst + (i & (n - 1))] = static_cast<int16_t>(s.blk[i]);
    wave_sync();
}

// H.264 luma 4x4 / 8x8 residuals without a DC transform (I4x4, I8x8 TBs), 64 / N TBs per pass
// like hevc_residual_group: lane = (TB, row) dequantises its row and runs the row butterfly in
// registers, then lane = (TB, column) the column butterfly; one packed store per row.  Same
// arithmetic as h264_residual (8.5.12, 8.5.13): int intermediates, (x + 32) >> 6 at the end.
template <int LOG2N>
DEVI void h264_residual_group(const K0F& f, const uint4& rec, uint64_t gm, int G, const h2j_coef* CO,
                              const uint8_t* sl, int16_t* res, int mbw, K0Lds& s) {
    constexpr int N = 1 << LOG2N, NN = N * N, GMAX = 64 / N;
    const int lane = threadIdx.x;
    int* blk = s.blk;  // [G][N][N] levels, then the final residual
    int* tmp = s.tmp;  // [G][N][N] after the row pass
    for (int i = lane; i < G * NN; i += 64) blk[i] = 0;
    // coefficient entries of all TBs of the group first (independent loads), then the scatter
    uint32_t en[GMAX];
    int ncf[GMAX];
    {
        uint64_t mm = gm;
#pragma unroll
        for (int g = 0; g < GMAX; g++) {
            en[g] = 0;
            ncf[g] = 0;
            if (g < G) {
                const int kg = __ffsll(static_cast<long long>(mm)) - 1;
                mm &= mm - 1;
                const h2j_tu tu = tu_from_lanes(rec, kg);
                ncf[g] = tu.ncoef;
                if (lane < tu.ncoef) en[g] = CO[tu.coef + lane];
            }
        }
    }
    wave_sync();
#pragma unroll
    for (int g = 0; g < GMAX; g++)
        if (lane < ncf[g]) blk[g * NN + static_cast<int>(en[g] >> 24)] = static_cast<int>(en[g] << 8) >> 8;
    wave_sync();
    const int g = lane >> LOG2N, q = lane & (N - 1);
    const bool act = g < G;
    uint64_t ml = gm;
    for (int i = 0; i < g && i < G - 1; i++) ml &= ml - 1;
    const int k = __ffsll(static_cast<long long>(ml)) - 1;
    const uint32_t w0 = __shfl(rec.x, k, 64), w1 = __shfl(rec.y, k, 64), w2 = __shfl(rec.z, k, 64);
    uint32_t wq[4] = {w0, w1, w2, 0};
    h2j_tu mine;
    memcpy(&mine, wq, sizeof(mine));
    const int qp = mine.qp, qm = qp % 6;
    if (act) {  // dequantise row q, row butterfly
        const uint8_t* w = f.slist ? sl + f.sl + (LOG2N == 2 ? 0 : 48) : nullptr;
        int d[N];
#pragma unroll
        for (int x = 0; x < N; x++) {
            const int i = q * N + x;
            const int lvl = blk[g * NN + i];
            d[x] = LOG2N == 2 ? h264_scale4(lvl, (w ? w[i] : 16) * h264_norm4(qm, q, x), qp)
                              : h264_scale8(lvl, (w ? w[i] : 16) * h264_norm8(qm, q, x), qp);
        }
        int o[N];
        if constexpr (LOG2N == 2) {
            const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
            o[0] = e0 + e3; o[1] = e1 + e2; o[2] = e1 - e2; o[3] = e0 - e3;
        } else {
            h264_idct8_1d(d, o);
        }
#pragma unroll
        for (int x = 0; x < N; x++) tmp[g * NN + q * N + x] = o[x];
    }
    wave_sync();
    if (act) {  // column q
        int d[N], o[N];
#pragma unroll
        for (int y = 0; y < N; y++) d[y] = tmp[g * NN + y * N + q];
        if constexpr (LOG2N == 2) {
            const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
            o[0] = e0 + e3; o[1] = e1 + e2; o[2] = e1 - e2; o[3] = e0 - e3;
        } else {
            h264_idct8_1d(d, o);
        }
#pragma unroll
        for (int y = 0; y < N; y++) blk[g * NN + y * N + q] = (o[y] + 32) >> 6;
    }
    wave_sync();
    if (act) {  // row q of the residual: one packed store
        int16_t* R = h264_res_at(res, mbw, 0, mine.x, mine.y) + q * 16;
        uint32_t packed[N / 2];
#pragma unroll
        for (int i = 0; i < N / 2; i++)
            packed[i] = (static_cast<uint32_t>(blk[g * NN + q * N + 2 * i]) & 0xFFFF) |
                        (static_cast<uint32_t>(blk[g * NN + q * N + 2 * i + 1]) << 16);
        if constexpr (N == 4) *reinterpret_cast<uint2*>(R) = make_uint2(packed[0], packed[1]);
        else *reinterpret_cast<uint4*>(R) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
    }
    wave_sync();
}

// H.264 chroma 8x8 residuals (4:2:0: 2x2 DC Hadamard + four 4x4 blocks), four TBs per pass:
// lane = (TB g, block b, row / column k).  Same arithmetic as the chroma branch of
// h264_residual (8.5.11: DC ((f * LevelScale4x4(0,0)) << (qP / 6)) >> 5; 8.5.12 AC scaling).
DEVI void h264_chroma_group(const K0F& f, const uint4& rec, uint64_t gm, int G, const h2j_coef* CO,
                            const uint8_t* sl, int16_t* res, int mbw, K0Lds& s) {
    const int lane = threadIdx.x;
    int* blk = s.blk;  // [G][8][8] levels, then the final residual
    int* tmp = s.tmp;  // [G][8][8] after the row pass
    for (int i = lane; i < G * 64; i += 64) blk[i] = 0;
    uint32_t en[4];
    int ncf[4];
    {
        uint64_t mm = gm;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            en[g] = 0;
            ncf[g] = 0;
            if (g < G) {
                const int kg = __ffsll(static_cast<long long>(mm)) - 1;
                mm &= mm - 1;
                const h2j_tu tu = tu_from_lanes(rec, kg);
                ncf[g] = tu.ncoef;
                if (lane < tu.ncoef) en[g] = CO[tu.coef + lane];
            }
        }
    }
    wave_sync();
#pragma unroll
    for (int g = 0; g < 4; g++)
        if (lane < ncf[g]) blk[g * 64 + static_cast<int>(en[g] >> 24)] = static_cast<int>(en[g] << 8) >> 8;
    wave_sync();
    const int g = lane >> 4, b = (lane >> 2) & 3, k = lane & 3;
    const bool act = g < G;
    uint64_t ml = gm;
    for (int i = 0; i < g && i < G - 1; i++) ml &= ml - 1;
    const int kr = __ffsll(static_cast<long long>(ml)) - 1;
    const uint32_t w0 = __shfl(rec.x, kr, 64), w1 = __shfl(rec.y, kr, 64), w2 = __shfl(rec.z, kr, 64);
    uint32_t wq[4] = {w0, w1, w2, 0};
    h2j_tu mine;
    memcpy(&mine, wq, sizeof(mine));
    const int qp = mine.qp, qm = qp % 6;
    const uint8_t* w4 = f.slist ? sl + f.sl + mine.c * 16 : nullptr;
    int* B = blk + g * 64;
    const int bx = (b & 1) * 4, by = (b >> 1) * 4;
    if (act && (lane & 15) < 4) {  // 2x2 DC Hadamard: output (r, q) = lane & 3
        const int r = (lane >> 1) & 1, q = lane & 1;
        const int a = B[0], bb = B[4], c = B[32], d = B[36];
        const int acc = a + (q ? -bb : bb) + (r ? -c : c) + ((r ^ q) ? -d : d);
        const int ls0 = (w4 ? w4[0] : 16) * kNorm4[qm][0];
        s.dc[g * 4 + (lane & 3)] = ((acc * ls0) << (qp / 6)) >> 5;
    }
    wave_sync();
    if (act) {  // row k of block b: AC scaling (DC from the Hadamard), row butterfly
        int d[4];
#pragma unroll
        for (int x = 0; x < 4; x++) {
            const int i = (by + k) * 8 + bx + x;
            d[x] = (k == 0 && x == 0) ? s.dc[g * 4 + b]
                                      : h264_scale4(B[i], (w4 ? w4[k * 4 + x] : 16) * h264_norm4(qm, k, x), qp);
        }
        const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        int* o = tmp + g * 64 + (by + k) * 8 + bx;
        o[0] = e0 + e3; o[1] = e1 + e2; o[2] = e1 - e2; o[3] = e0 - e3;
    }
    wave_sync();
    if (act) {  // column k of block b
        const int* t = tmp + g * 64 + by * 8 + bx + k;
        const int d0 = t[0], d1 = t[8], d2 = t[16], d3 = t[24];
        const int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
        int* o = B + by * 8 + bx + k;
        o[0] = (e0 + e3 + 32) >> 6; o[8] = (e1 + e2 + 32) >> 6; o[16] = (e1 - e2 + 32) >> 6; o[24] = (e0 - e3 + 32) >> 6;
    }
    wave_sync();
    if (act) {  // row k of block b of the residual: 4 samples, one 8-byte store
        const int* v = B + (by + k) * 8 + bx;
        int16_t* R = h264_res_at(res, mbw, mine.c, mine.x + bx, mine.y + by + k);
        *reinterpret_cast<uint2*>(R) = make_uint2((static_cast<uint32_t>(v[0]) & 0xFFFF) | (static_cast<uint32_t>(v[1]) << 16),
                                                  (static_cast<uint32_t>(v[2]) & 0xFFFF) | (static_cast<uint32_t>(v[3]) << 16));
    }
    wave_sync();
}

// H.264 Intra16x16 luma residuals (4x4 DC Hadamard + sixteen 4x4 blocks), four TBs per pass:
// lane = (TB g, 4x4 block), the block's scaling and both butterfly passes in registers (no LDS
// round trip between the passes).  Same arithmetic as the i16 branch of h264_residual (8.5.10,
// 8.5.12).
DEVI void h264_i16_group(const K0F& f, const uint4& rec, uint64_t gm, int G, const h2j_coef* CO,
                         const uint8_t* sl, int16_t* res, int mbw, K0Lds& s) {
    const int lane = threadIdx.x;
    int* blk = s.blk;  // [G][16][16] levels
    for (int i = lane; i < G * 256; i += 64) blk[i] = 0;
    wave_sync();
    {
        uint64_t mm = gm;
        for (int g = 0; g < G; g++) {
            const int kg = __ffsll(static_cast<long long>(mm)) - 1;
            mm &= mm - 1;
            const h2j_tu tu = tu_from_lanes(rec, kg);
            uint32_t en[4];
#pragma unroll
            for (int j = 0; j < 4; j++) en[j] = lane + 64 * j < tu.ncoef ? CO[tu.coef + lane + 64 * j] : 0u;
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (lane + 64 * j < tu.ncoef) blk[g * 256 + static_cast<int>(en[j] >> 24)] = static_cast<int>(en[j] << 8) >> 8;
        }
    }
    wave_sync();
    const int g = lane >> 4, b = lane & 15, bx = b & 3, by = b >> 2;
    // this lane's record, fetched with every lane active (ds_bpermute reads nothing from an
    // inactive source lane, and the record may sit in any of the wave's lanes)
    uint64_t ml = gm;
    for (int i = 0; i < g && i < G - 1; i++) ml &= ml - 1;
    const int kr = __ffsll(static_cast<long long>(ml)) - 1;
    const uint32_t w0 = __shfl(rec.x, kr, 64), w1 = __shfl(rec.y, kr, 64), w2 = __shfl(rec.z, kr, 64);
    if (g < G) {
        uint32_t wq[4] = {w0, w1, w2, 0};
        h2j_tu mine;
        memcpy(&mine, wq, sizeof(mine));
        const int qp = mine.qp, qm = qp % 6;
        const uint8_t* w4 = f.slist ? sl + f.sl : nullptr;
        const int* B = blk + g * 256;
        // DC Hadamard output (by, bx) = this block's DC
        int acc = 0;
    #pragma unroll
        for (int i = 0; i < 4; i++) {
            const int hr = (by == 0 || (by == 1 && i < 2) || (by == 2 && (i == 0 || i == 3)) || (by == 3 && !(i & 1))) ? 1 : -1;
    #pragma unroll
            for (int j = 0; j < 4; j++) {
                const int hc = (bx == 0 || (bx == 1 && j < 2) || (bx == 2 && (j == 0 || j == 3)) || (bx == 3 && !(j & 1))) ? 1 : -1;
                acc += hr * hc * B[(i * 4) * 16 + j * 4];
            }
        }
        const int ls0 = (w4 ? w4[0] : 16) * kNorm4[qm][0];
        const int dcv = qp >= 36 ? (acc * ls0) << (qp / 6 - 6) : (acc * ls0 + (1 << (5 - qp / 6))) >> (6 - qp / 6);
        int v[4][4];
    #pragma unroll
        for (int r = 0; r < 4; r++)
    #pragma unroll
            for (int x = 0; x < 4; x++)
                v[r][x] = (r == 0 && x == 0) ? dcv
                                             : h264_scale4(B[(by * 4 + r) * 16 + bx * 4 + x],
                                                           (w4 ? w4[r * 4 + x] : 16) * h264_norm4(qm, r, x), qp);
    #pragma unroll
        for (int r = 0; r < 4; r++) {  // rows
            const int e0 = v[r][0] + v[r][2], e1 = v[r][0] - v[r][2], e2 = (v[r][1] >> 1) - v[r][3], e3 = v[r][1] + (v[r][3] >> 1);
            v[r][0] = e0 + e3; v[r][1] = e1 + e2; v[r][2] = e1 - e2; v[r][3] = e0 - e3;
        }
    #pragma unroll
        for (int x = 0; x < 4; x++) {  // columns
            const int e0 = v[0][x] + v[2][x], e1 = v[0][x] - v[2][x], e2 = (v[1][x] >> 1) - v[3][x], e3 = v[1][x] + (v[3][x] >> 1);
            v[0][x] = (e0 + e3 + 32) >> 6; v[1][x] = (e1 + e2 + 32) >> 6; v[2][x] = (e1 - e2 + 32) >> 6; v[3][x] = (e0 - e3 + 32) >> 6;
        }
        int16_t* R = h264_res_at(res, mbw, 0, mine.x + bx * 4, mine.y + by * 4);
    #pragma unroll
        for (int r = 0; r < 4; r++)
            *reinterpret_cast<uint2*>(R + r * 16) = make_uint2((static_cast<uint32_t>(v[r][0]) & 0xFFFF) | (static_cast<uint32_t>(v[r][1]) << 16),
                                                                (static_cast<uint32_t>(v[r][2]) & 0xFFFF) | (static_cast<uint32_t>(v[r][3]) << 16));
    }  // g < G
    wave_sync();
}

// position of a 4x4 block inside its CTB in z-scan order (6.5.2)
DEVI int zorder4(int ax, int ay) {
    int z = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) z |= (((ax >> i) & 1) << (2 * i)) | (((ay >> i) & 1) << (2 * i + 1));
    return z;
}

// One kernel per codec (HEVC: batched transforms, more records per wave; each gets its own
// register budget), each skipping the other codec's pictures.
template <bool HEVC>
__global__ void __launch_bounds__(64, 7) h2j_k0_prep(const h2j_frame* frames, const h2j_tu* tus, const h2j_coef* coefs,
                                                 const h2j_ctb* ctbs, const h2j_slice* slices, const uint8_t* sl,
                                                 uint8_t* arena) {
    const GridPos gp = xcd_grid_pos();
    constexpr int kTus = HEVC ? kK0TusHevc : kK0Tus;
    __shared__ typename std::conditional<HEVC, K0LdsHevc, K0Lds>::type s;
    const h2j_frame& fr = frames[gp.y];
    if ((ufl(fr.codec) == H2J_CODEC_HEVC) != HEVC) return;
    const uint32_t ntu = ufl(fr.ntu);
    const uint32_t t0 = gp.x * kTus;
    if (t0 >= ntu) return;
    const int lane = threadIdx.x;
    constexpr bool hevc = HEVC;
    K0F f;
    f.bd = ufl(fr.bit_depth);
    f.bdc = ufl(fr.bit_depth_c);
    f.slist = ufl(fr.scaling_list);
    f.sl = ufl(fr.sl);
    f.log2ctb = ufl(fr.log2ctb);
    f.ctb_w = ufl(fr.ctb_w);
    f.width = ufl(fr.width);
    f.height = ufl(fr.height);
    f.mw = ufl(fr.mw);
    f.topo = ufl(fr.topo);
    f.rext = ufl(fr.rext);
    const h2j_ctb* C = ctbs + ufl(fr.ctb);
    const h2j_slice* S = slices + ufl(fr.slice);
    const h2j_tu* T = tus + ufl(fr.tu);
    const h2j_coef* CO = coefs + ufl(fr.coef);
    uint64_t* masks = reinterpret_cast<uint64_t*>(arena + ufl64(fr.aux));
    uint32_t* rng = reinterpret_cast<uint32_t*>(arena + ufl64(fr.ctbrng));
    uint8_t* fmap = arena + ufl64(fr.maps);
    int8_t* qmap = reinterpret_cast<int8_t*>(fmap + static_cast<size_t>(f.mw) * ufl(fr.mh));
    uint8_t* pic = arena + ufl64(fr.pic);
    int16_t* res = reinterpret_cast<int16_t*>(arena + ufl64(fr.res));
    const int st0 = ufl(fr.pic_stride[0]), st1 = ufl(fr.pic_stride[1]);
    const int off1 = ufl(fr.pic_off[1]), off2 = ufl(fr.pic_off[2]);
    // this workgroup's records (lane k: record t0 + k) and the two neighbours of the range
    const uint32_t t1 = min(ntu, t0 + kTus);
    const int nrec = static_cast<int>(t1 - t0);
    uint4 rec = make_uint4(0, 0, 0, 0);
    {
        int ri = static_cast<int>(t0) + lane;
        if (lane == kTus) ri = static_cast<int>(t0) - 1;
        if (lane == kTus + 1) ri = static_cast<int>(t1);
        if (lane <= kTus + 1 && ri >= 0 && ri < static_cast<int>(ntu)) rec = reinterpret_cast<const uint4*>(T)[ri];
    }
    // (the HEVC matrices are constants: kDctPk; transform-skip and bypass TBs use none)
    wave_sync();
    auto ctb_of_tu = [&](const h2j_tu& tu) __attribute__((always_inline)) {
        const int sh = tu.c ? 1 : 0;
        return ((tu.y << sh) >> f.log2ctb) * f.ctb_w + ((tu.x << sh) >> f.log2ctb);
    };
    const int prev_cb = t0 > 0 ? ctb_of_tu(tu_from_lanes(rec, kTus)) : -1;
    const int prev_c = t0 > 0 ? tu_from_lanes(rec, kTus).c : 0;
    const int next_cb = t1 < ntu ? ctb_of_tu(tu_from_lanes(rec, kTus + 1)) : -1;
    // coefficient entries of the current TU (lane e < 64), prefetched one TU ahead
    auto fetch_co = [&](const h2j_tu& v) __attribute__((always_inline)) -> uint32_t {
        const uint32_t e = min(static_cast<uint32_t>(lane), max(static_cast<uint32_t>(v.ncoef), 1u) - 1);
        return v.ncoef ? CO[v.coef + e] : 0u;
    };
    // ---- per-record metadata, one lane per record: CTB ranges, deblocking maps (HEVC luma),
    // availability masks.  (The neighbours of the range sit in lanes kTus, kTus + 1.)
    h2j_tu own;
    {
        uint32_t w4[4] = {rec.x, rec.y, rec.z, rec.w};
        memcpy(&own, w4, sizeof(own));
    }
    const bool mine = lane < nrec;
    {
        const int oc = own.c, on = 1 << own.log2n, oshc = oc ? 1 : 0;
        const int ox0 = own.x, oy0 = own.y, oxl = ox0 << oshc, oyl = oy0 << oshc;
        const int ocb = (oyl >> f.log2ctb) * f.ctb_w + (oxl >> f.log2ctb);
        const int lcb = __shfl(ocb, lane > 0 ? lane - 1 : 0, 64), lcc = __shfl(oc, lane > 0 ? lane - 1 : 0, 64);
        const int rcb = __shfl(ocb, lane < 63 ? lane + 1 : 63, 64);
        const int pcb = lane == 0 ? prev_cb : lcb, pc = lane == 0 ? prev_c : lcc;
        const int ncb = lane == nrec - 1 ? next_cb : rcb;
        if (mine) {
            const uint32_t t = t0 + lane;
            if (pcb != ocb) rng[4 * ocb] = t;
            if (ncb != ocb) rng[4 * ocb + 2] = t + 1;
            // first chroma record of the CTB (HEVC records are luma first, then chroma)
            if (oc > 0 && (pcb != ocb || pc == 0)) rng[4 * ocb + 1] = t;
            const uint8_t flags = own.flags;
            if (hevc && oc == 0) {  // deblocking maps (luma TBs): a row of the TB's nb 4x4 units per store
                // (r06: byte stores per unit, nb * nb <= 64 steps with a division each on every lane
                // of a wave holding one 32x32 TB); rows stored whole when the map rows keep the
                // TB's alignment (mw a multiple of 8, as at 1080p), else in 1-byte pieces
                const int nb = on >> 2;
                const int pc = (f.mw & 7) == 0 ? nb : 1;  // bytes per store
                const uint32_t base = (flags & H2J_TU_NOFILT) ? 0x04040404u : 0u;
                const uint32_t qv = 0x01010101u * static_cast<uint8_t>(own.qpy);
                for (int by = 0; by < nb; by++) {
                    const uint32_t rowv = base | (by == 0 && (flags & H2J_TU_EDGE_T) ? 0x02020202u : 0u);
                    for (int bx = 0; bx < nb; bx += pc) {
                        const int idx = ((oy0 >> 2) + by) * f.mw + (ox0 >> 2) + bx;
                        const uint32_t fv = rowv | (bx == 0 && (flags & H2J_TU_EDGE_L) ? 1u : 0u);
                        if (pc == 8) {
                            *reinterpret_cast<uint2*>(fmap + idx) = make_uint2(fv, rowv);
                            *reinterpret_cast<uint2*>(qmap + idx) = make_uint2(qv, qv);
                        } else if (pc == 4) {
                            *reinterpret_cast<uint32_t*>(fmap + idx) = fv;
                            *reinterpret_cast<uint32_t*>(qmap + idx) = qv;
                        } else if (pc == 2) {
                            *reinterpret_cast<uint16_t*>(fmap + idx) = static_cast<uint16_t>(fv);
                            *reinterpret_cast<uint16_t*>(qmap + idx) = static_cast<uint16_t>(qv);
                        } else {
                            fmap[idx] = static_cast<uint8_t>(fv);
                            qmap[idx] = static_cast<int8_t>(qv);
                        }
                    }
                }
            }
            // reference availability mask; without several slices / tiles it is pure
            // geometry: inside the picture and earlier in decoding (z-scan / raster) order
            uint64_t mask = 0;
            if (!(flags & H2J_TU_PCM)) {
                if (hevc) {
                    const int u = oc ? 2 : 4, nu = (2 * on) / u;
                    const int l2 = f.log2ctb, m = (1 << l2) - 1;
                    const int zc = zorder4((oxl & m) >> 2, (oyl & m) >> 2);
                    if (f.topo) {  // slices / tiles: every unit by the full rule
                        for (int q = 0; q <= 2 * nu; q++) {
                            int xn, yn;
                            if (q < nu) { xn = ox0 - 1; yn = oy0 + 2 * on - 1 - q * u; }
                            else if (q == nu) { xn = ox0 - 1; yn = oy0 - 1; }
                            else { xn = ox0 + (q - nu - 1) * u; yn = oy0 - 1; }
                            mask |= static_cast<uint64_t>(avail(fr, C, S, oxl, oyl, xn << oshc, yn << oshc)) << q;
                        }
                    } else {
                        // geometry alone, in closed form (r06: the per-unit loop ran 2nu + 1 <= 33
                        // steps on every lane of a wave holding one 32x32 luma / 16x16 chroma TB).
                        // The left and upper halves and the corner neighbour an aligned TB from
                        // blocks that precede it; the below-left / above-right halves each lie in
                        // one aligned block of the TB's size, before the TB in z-order / CTB order
                        // entirely or not at all: test its first unit, then cut at the picture edge.
                        auto geo = [&](int xn, int yn) __attribute__((always_inline)) {
                            const int xnl = xn << oshc, ynl = yn << oshc;
                            if (xnl < 0 || ynl < 0 || xnl >= f.width || ynl >= f.height) return false;
                            const int cn = (ynl >> l2) * f.ctb_w + (xnl >> l2);
                            return cn == ocb ? zorder4((xnl & m) >> 2, (ynl & m) >> 2) <= zc : cn < ocb;
                        };
                        const int nh = nu >> 1, Wc = f.width >> oshc, Hc = f.height >> oshc;
                        const uint64_t half = (1ull << nh) - 1;
                        if (ox0 > 0) mask |= half << nh;
                        if (ox0 > 0 && oy0 > 0) mask |= 1ull << nu;
                        if (oy0 > 0) mask |= half << (nu + 1);
                        if (geo(ox0 - 1, oy0 + on + u - 1)) {
                            const int fit = min(nh, (Hc - oy0 - on) / u);
                            mask |= ((1ull << fit) - 1) << (nh - fit);
                        }
                        if (geo(ox0 + on, oy0 - 1)) {
                            const int fit = min(nh, (Wc - ox0 - on + u - 1) / u);
                            mask |= ((1ull << fit) - 1) << (nu + nh + 1);
                        }
                    }
                } else if (ufl(fr.mbaff)) {  // MBAFF: 6.4.12.2 availability computed by the host parser
                    mask = static_cast<uint64_t>(static_cast<uint8_t>(own.qpy) & 15u);
                } else {
                    const bool nxn = oc == 0 && own.log2n <= 3;
                    for (int q = 0; q < 4; q++) {
                        int xn = oxl, yn = oyl;
                        bool use = true;
                        if (q == 0) yn = oyl - 1;
                        else if (q == 1) xn = oxl - 1;
                        else if (q == 2) { xn = oxl - 1; yn = oyl - 1; }
                        else { xn = oxl + on; yn = oyl - 1; use = nxn; }
                        bool a = false;
                        if (use) {
                            if (f.topo) {
                                a = h264_avail(fr, C, S, oxl, oyl, xn, yn);
                            } else if (xn >= 0 && yn >= 0 && xn < f.width && yn < f.height) {
                                const int cn = (yn >> 4) * f.ctb_w + (xn >> 4), cc = (oyl >> 4) * f.ctb_w + (oxl >> 4);
                                if (cn == cc) {
                                    const int ax = (xn & 15) >> 2, ay = (yn & 15) >> 2, bx = (oxl & 15) >> 2, by = (oyl & 15) >> 2;
                                    a = ((ax & 1) | ((ay & 1) << 1) | ((ax & 2) << 1) | ((ay & 2) << 2)) <
                                        ((bx & 1) | ((by & 1) << 1) | ((bx & 2) << 1) | ((by & 2) << 2));
                                } else {
                                    a = cn < cc;
                                }
                            }
                        }
                        mask |= static_cast<uint64_t>(a) << q;
                    }
                }
            }
            masks[t] = mask;
        }
    }
    // ---- records with per-record work, one after another: PCM samples, H.264 residuals, HEVC
    // transform-skip / bypass residuals (regular HEVC transforms run batched below).  H.264:
    // the next such record's coefficients prefetched one record ahead.
    // H.264 luma 4x4 / 8x8 (no DC transform) run batched below, like the regular HEVC transforms
    const bool grp264 = !hevc && mine && (own.flags & H2J_TU_CBF) && !(own.flags & (H2J_TU_PCM | H2J_TU_BYPASS)) &&
                        own.c == 0 && own.log2n <= 3;
    // ... and the chroma 8x8 TBs, four per pass
    const bool grp264c = !hevc && mine && (own.flags & H2J_TU_CBF) && !(own.flags & (H2J_TU_PCM | H2J_TU_BYPASS)) &&
                         own.c > 0 && own.log2n == 3;
    // ... and the Intra16x16 luma TBs, four per pass
    const bool grp264i = !hevc && mine && (own.flags & H2J_TU_CBF) && !(own.flags & (H2J_TU_PCM | H2J_TU_BYPASS)) &&
                         own.c == 0 && own.log2n == 4;
    // ... and HEVC 4x4 transform-skip TBs of pictures without rotation / implicit RDPCM, 16 per pass
    const bool grpts = hevc && mine && (own.flags & H2J_TU_CBF) && (own.flags & H2J_TU_TSKIP) &&
                       !(own.flags & (H2J_TU_PCM | H2J_TU_BYPASS)) && own.log2n == 2 &&
                       !(f.rext & (H2J_REXT_TS_ROT | H2J_REXT_RDPCM));
    uint64_t work = __ballot(mine && !grp264 && !grp264c && !grp264i && !grpts && ((own.flags & H2J_TU_PCM) ||
                                      ((own.flags & H2J_TU_CBF) && (!hevc || (own.flags & (H2J_TU_TSKIP | H2J_TU_BYPASS))))));
    uint32_t nco = (!hevc && work) ? fetch_co(tu_from_lanes(rec, __ffsll(static_cast<long long>(work)) - 1)) : 0u;
    while (work) {
        const int k = __ffsll(static_cast<long long>(work)) - 1;
        work &= work - 1;
        const h2j_tu tu = tu_from_lanes(rec, k);
        uint32_t co0 = nco;
        if (!hevc && work) nco = fetch_co(tu_from_lanes(rec, __ffsll(static_cast<long long>(work)) - 1));
        if (hevc) co0 = fetch_co(tu);
        const int c = tu.c, log2n = tu.log2n, n = 1 << log2n;
        const int x0 = tu.x, y0 = tu.y;
        const uint8_t flags = tu.flags;
        const int stc = c ? st1 : st0;
        const int offc = c == 0 ? 0 : (c == 1 ? off1 : off2);
        if (flags & H2J_TU_PCM) {
            const bool mbaff = !hevc && ufl(fr.mbaff);  // MBAFF: field MBs' rows interleave (h264_mbaff_row)
            if (f.bd == 8) {
                uint8_t* P = pic + offc;
                for (int e = lane; e < tu.ncoef; e += 64) {
                    const uint32_t en = e < 64 ? co0 : CO[tu.coef + e];
                    const int pos = static_cast<int>(en >> 16);
                    const int yy = y0 + (pos >> log2n), row = mbaff ? h264_mbaff_row(C, f.ctb_w, c, x0, yy) : yy;
                    P[row * stc + x0 + (pos & (n - 1))] = static_cast<uint8_t>(en & 0xFF);
                }
            } else {
                uint16_t* P = reinterpret_cast<uint16_t*>(pic) + offc;
                for (int e = lane; e < tu.ncoef; e += 64) {
                    const uint32_t en = e < 64 ? co0 : CO[tu.coef + e];
                    const int pos = static_cast<int>(en >> 16);
                    const int yy = y0 + (pos >> log2n), row = mbaff ? h264_mbaff_row(C, f.ctb_w, c, x0, yy) : yy;
                    P[row * stc + x0 + (pos & (n - 1))] = static_cast<uint16_t>(en & 0xFFFF);
                }
            }
            continue;
        }
        if constexpr (HEVC)  // R: the TB's origin in its tile, rows 1 << h2j_res_q apart
            hevc_residual(f, tu, CO, co0, sl, hevc_res_at(res, f.width, f.height, f.log2ctb, c, x0, y0),
                          1 << h2j_res_q(f.log2ctb, c), s);
        else h264_residual(f, tu, CO, co0, sl, h264_res_at(res, f.ctb_w, c, x0, y0), c ? 8 : 16, s);
    }
    if constexpr (!HEVC) {  // H.264 luma 4x4 / 8x8 residuals, 16 / 8 same-size TBs per pass
#pragma unroll
        for (int l2 = 2; l2 <= 3; l2++) {
            uint64_t m = __ballot(grp264 && own.log2n == l2);
            const int G = 64 >> l2;
            while (m) {
                uint64_t gm = 0;
                int cnt = 0;
                while (m && cnt < G) {
                    gm |= m & (0 - m);
                    m &= m - 1;
                    cnt++;
                }
                if (l2 == 2) h264_residual_group<2>(f, rec, gm, cnt, CO, sl, res, f.ctb_w, s);
                else h264_residual_group<3>(f, rec, gm, cnt, CO, sl, res, f.ctb_w, s);
            }
        }
        uint64_t m = __ballot(grp264c);
        while (m) {
            uint64_t gm = 0;
            int cnt = 0;
            while (m && cnt < 4) {
                gm |= m & (0 - m);
                m &= m - 1;
                cnt++;
            }
            h264_chroma_group(f, rec, gm, cnt, CO, sl, res, f.ctb_w, s);
        }
        m = __ballot(grp264i);
        while (m) {
            uint64_t gm = 0;
            int cnt = 0;
            while (m && cnt < 4) {
                gm |= m & (0 - m);
                m &= m - 1;
                cnt++;
            }
            h264_i16_group(f, rec, gm, cnt, CO, sl, res, f.ctb_w, s);
        }
    }
    if constexpr (HEVC) {  // HEVC residuals, 64 / N same-size TBs per pass
        const bool batch = lane < nrec && (own.flags & H2J_TU_CBF) && !(own.flags & (H2J_TU_PCM | H2J_TU_TSKIP | H2J_TU_BYPASS));
#pragma unroll
        for (int l2 = 2; l2 <= 5; l2++) {
            uint64_t m = __ballot(batch && own.log2n == l2);
            const int G = 64 >> l2;  // 16, 8, 4, 2 TBs per pass
            while (m) {
                uint64_t gm = 0;  // the next (up to) G TBs of this size
                int cnt = 0;
                while (m && cnt < G) {
                    gm |= m & (0 - m);
                    m &= m - 1;
                    cnt++;
                }
                switch (l2) {
                    case 2: hevc_residual_group<2>(f, rec, gm, cnt, CO, sl, res, s); break;
                    case 3: hevc_residual_group<3>(f, rec, gm, cnt, CO, sl, res, s); break;
                    case 4: hevc_residual_group<4>(f, rec, gm, cnt, CO, sl, res, s); break;
                    default: hevc_residual_group<5>(f, rec, gm, cnt, CO, sl, res, s); break;
                }
            }
        }
        uint64_t m = __ballot(grpts);
        while (m) {
            uint64_t gm = 0;
            int cnt = 0;
            while (m && cnt < 16) {
                gm |= m & (0 - m);
                m &= m - 1;
                cnt++;
            }
            hevc_residual_group<2, true>(f, rec, gm, cnt, CO, sl, res, s);
        }
    }
}

// ---------------------------------------------------------------- K1: intra prediction chain
// One workgroup per picture, kK1Waves waves; wave w reconstructs CTB rows
// w, w + kK1Waves, ...  CTB (x, r) starts once row r-1 has finished CTBs
// 0..x+1 (its left / top-left / top / top-right neighbours: everything intra
// prediction can reference), tracked by row-tagged progress counters in LDS.
// Inside a CTB the wave walks the TUs in decoding order: reference gather
// with K0's availability mask, substitution / filtering, prediction, + K0's
// residual, clip, store.  (H.265 8.4.4.2; H.264 8.3)
struct K1WaveLds {  // HEVC reference arrays (4n + 1 <= 129 samples)
    int16_t sub[132];
    int16_t ref[132];
};

// Asynchronous global -> LDS copies (LDS-DMA): lane i's bytes land at lds + i * size, with no
// VGPR destination.  M0 carries the wave-uniform LDS byte address (set and restored inside the
// statement, the compiler reserves M0).  Issued as asm, so the compiler does not track them:
// every use of the data waits vmcnt(0) explicitly (lds_dma_wait).
DEVI void lds_dma16(const void* g, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
DEVI void lds_dma4(const void* g, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
DEVI void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
DEVI void lds_reads_done() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
DEVI uint32_t lds_addr(const void* p) {
    return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)));
}

// H.264: one macroblock plus its top line and left column, per wave.
// Window coordinates: (x - mb_x + 1, y - mb_y + 1); row 0 is the line
// above (luma incl. the 8 top-right samples), column 0 the left column.
constexpr int kH4MaxTus = 24;
struct alignas(16) H4In {  // one MB's inputs, filled by LDS-DMA while the previous MB runs
    h2j_tu tus[kH4MaxTus];                       // records (16 B each: one dwordx4 per lane)
    uint32_t mlo[kH4MaxTus], mhi[kH4MaxTus];     // availability masks, low / high dwords
    int16_t ry[16][16];                          // K0 residual: luma, then (contiguous) chroma
    int16_t rc[2][8][8];
    DEVI uint64_t mask(int t) const { return static_cast<uint64_t>(mlo[t]) | (static_cast<uint64_t>(mhi[t]) << 32); }
};
static_assert(offsetof(H4In, rc) == offsetof(H4In, ry) + 512 && offsetof(H4In, ry) % 16 == 0,
              "one 48-lane dwordx4 DMA fills ry then rc");
struct alignas(16) H4WaveLds {
    H4In in[2];     // ping-pong: the MB being reconstructed / the next one
    alignas(16) uint8_t stage[3 * 16 * 64];  // reconstructed MBs (Pel): luma [16][16 G] + chroma [2][8][8 G], G = 8 MBs at 8 bits, 4 above
    uint16_t wy[17][25];
    uint16_t wc[2][9][9];
    int top[40];    // top[0] = corner, top[1 + i] = p[i, -1]
    int left[20];   // left[0] = corner, left[1 + i] = p[-1, i]
    int ftop[40], fleft[20];
};


// One H.264 prediction block (I4x4 / I8x8 / I16x16 / chroma) inside the
// wave's macroblock window; all sample traffic is LDS.
DEVI void h264_predict_tu(const h2j_tu& tu, uint64_t mask, int mbx, int mby, int bd, H4WaveLds& s, const H4In& in,
                           int lane) {
    const int c = tu.c, log2n = tu.log2n, n = 1 << log2n, nn = n * n;
    const int ox = c ? tu.x - mbx * 8 : tu.x - mbx * 16;   // block origin inside the macroblock
    const int oy = c ? tu.y - mby * 8 : tu.y - mby * 16;
    const int maxv = (1 << bd) - 1;
    const bool cbf = (tu.flags & H2J_TU_CBF) != 0;
    const bool chroma = c > 0;
    const bool nxn = c == 0 && log2n <= 3;
    const int ntop = nxn ? 2 * n : n;
    // window accessors (dx, dy relative to the block origin; -1 = neighbour)
#define WIN(dx, dy) (chroma ? s.wc[c - 1][oy + (dy) + 1][ox + (dx) + 1] : s.wy[oy + (dy) + 1][ox + (dx) + 1])
    // mask bits: 0 top, 1 left, 2 corner, 3 top-right
    const int fl = static_cast<int>(mask & 15);
    if (c == 0 && log2n == 4) {
        // Intra 16x16 (8.3.3): lane = (column x, rows 4g .. 4g + 3); references straight from the
        // window (unavailable ones read as 0, as the reference arrays below hold them), DC and the
        // plane gradients as wave sums -- no reference arrays, one LDS round trip fewer
        const int mode = tu.mode;
        const bool at = fl & 1, al = fl & 2, ad = fl & 4;
        const int x = lane & 15, y0 = (lane >> 4) * 4;
        const int tx = at ? s.wy[0][1 + x] : 0;
        // per sample: pv = (mode 3) clip((base + cc y) >> 5), else sel ? left : uni  (uni: DC or top)
        int uni = tx, base = 0, cc = 0;
        if (mode == 2) {
            const int part = lane < 16 ? tx : (lane < 32 && al ? s.wy[1 + (lane - 16)][0] : 0);
            const int sum = wave_sum_dpp(part);
            uni = (at && al) ? (sum + 16) >> 5 : ((at || al) ? (sum + 8) >> 4 : 1 << (bd - 1));
        } else if (mode == 3) {
            // H = sum (k + 1)(p[8 + k, -1] - p[6 - k, -1]), V likewise down the left column; the
            // k = 7 terms reach the corner p[-1, -1]
            const int k = lane & 7;
            const bool vl = lane >= 8;
            const int pbi = 7 - k;  // window index of p[6 - k] (0: the corner)
            const int pa = vl ? (al ? s.wy[9 + k][0] : 0) : (at ? s.wy[0][9 + k] : 0);
            const int pb = pbi == 0 ? (ad ? s.wy[0][0] : 0) : (vl ? (al ? s.wy[pbi][0] : 0) : (at ? s.wy[0][pbi] : 0));
            const int term = lane < 16 ? (k + 1) * (pa - pb) : 0;
            const int H = wave_sum_dpp(lane < 8 ? term : 0), V = wave_sum_dpp(vl ? term : 0);
            const int a = 16 * ((al ? s.wy[16][0] : 0) + (at ? s.wy[0][16] : 0));
            const int b = (5 * H + 32) >> 6;
            cc = (5 * V + 32) >> 6;
            base = a + b * (x - 7) - 7 * cc + 16;
        }
#pragma unroll 1
        for (int y = y0; y < y0 + 4; y++) {
            int pv = mode == 1 ? (al ? s.wy[1 + y][0] : 0) : uni;
            if (mode == 3) pv = clip3(0, maxv, (base + cc * y) >> 5);
            const int r = cbf ? in.ry[y][x] : 0;
            s.wy[1 + y][1 + x] = static_cast<uint16_t>(clip3(0, maxv, pv + r));
        }
        wave_sync();
        return;
    }
    for (int i = lane; i <= ntop; i += 64) {
        int v = 0;
        if (i == 0) v = (fl & 4) ? WIN(-1, -1) : 0;
        else if (i - 1 < n) v = (fl & 1) ? WIN(i - 1, -1) : 0;
        else v = (fl & 8) ? WIN(i - 1, -1) : ((fl & 1) ? WIN(n - 1, -1) : 0);
        s.top[i] = v;
    }
    for (int i = lane; i <= n; i += 64) s.left[i] = i == 0 ? ((fl & 4) ? WIN(-1, -1) : 0) : ((fl & 2) ? WIN(-1, i - 1) : 0);
    wave_sync();
    const int mode = tu.mode;
    const int* TT = s.top + 1;
    const int* LL = s.left + 1;
    if (nxn && log2n == 3) {
        // 8.3.2.2.1 reference sample filtering
        const bool at = fl & 1, al = fl & 2, ad = fl & 4;
        for (int i = lane; i <= 16; i += 64) {
            int v = 0;
            if (i == 0) {
                const int C = s.top[0];
                if (!ad) v = C;
                else if (at && al) v = (TT[0] + 2 * C + LL[0] + 2) >> 2;
                else if (at) v = (3 * C + TT[0] + 2) >> 2;
                else if (al) v = (3 * C + LL[0] + 2) >> 2;
                else v = C;
            } else if (at) {
                const int x = i - 1;
                if (x == 0) v = ad ? (s.top[0] + 2 * TT[0] + TT[1] + 2) >> 2 : (3 * TT[0] + TT[1] + 2) >> 2;
                else if (x == 15) v = (TT[14] + 3 * TT[15] + 2) >> 2;
                else v = (TT[x - 1] + 2 * TT[x] + TT[x + 1] + 2) >> 2;
            }
            s.ftop[i] = v;
        }
        for (int i = lane; i < 8; i += 64) {
            int v = 0;
            if (al) {
                if (i == 0) v = ad ? (s.top[0] + 2 * LL[0] + LL[1] + 2) >> 2 : (3 * LL[0] + LL[1] + 2) >> 2;
                else if (i == 7) v = (LL[6] + 3 * LL[7] + 2) >> 2;
                else v = (LL[i - 1] + 2 * LL[i] + LL[i + 1] + 2) >> 2;
            }
            s.fleft[i + 1] = v;
        }
        wave_sync();
        if (lane == 0) s.fleft[0] = s.ftop[0];
        wave_sync();
        TT = s.ftop + 1;
        LL = s.fleft + 1;
    }
    // DC value (luma DC mode 2 only; DPP sum, every lane active: mode is uniform)
    int dcv = 0;
    if (!chroma && mode == 2) {
        const bool at = fl & 1, al = fl & 2;
        int part = 0;
        for (int i = lane; i < n; i += 64) part += (at ? TT[i] : 0) + (al ? LL[i] : 0);
        const int sum = wave_sum_dpp(part);
        if (at && al) dcv = (sum + n) >> (log2n + 1);
        else if (at || al) dcv = (sum + (n >> 1)) >> log2n;
        else dcv = 1 << (bd - 1);
    }
#pragma unroll 1
    for (int i = lane; i < nn; i += 64) {
        const int x = i & (n - 1), y = i >> log2n;
        const int r = cbf ? (chroma ? in.rc[c - 1][oy + y][ox + x] : in.ry[oy + y][ox + x]) : 0;
        int pv;
        if (nxn) {
            pv = h264_pred_nxn(mode, x, y, n, TT, LL, dcv);
        } else if (!chroma) {  // 16x16
            if (mode == 0) pv = TT[x];
            else if (mode == 1) pv = LL[y];
            else if (mode == 2) pv = dcv;
            else {
                int H = 0, V = 0;
                for (int k = 0; k < 8; k++) {
                    H += (k + 1) * (TT[8 + k] - TT[6 - k]);
                    V += (k + 1) * (LL[8 + k] - LL[6 - k]);
                }
                const int a = 16 * (LL[15] + TT[15]), b = (5 * H + 32) >> 6, cc = (5 * V + 32) >> 6;
                pv = clip3(0, maxv, (a + b * (x - 7) + cc * (y - 7) + 16) >> 5);
            }
        } else {  // chroma 8x8 (mode: 0 DC, 1 horizontal, 2 vertical, 3 plane)
            if (mode == 1) pv = LL[y];
            else if (mode == 2) pv = TT[x];
            else if (mode == 3) {
                int H = 0, V = 0;
                for (int k = 0; k < 4; k++) {
                    H += (k + 1) * (TT[4 + k] - TT[2 - k]);
                    V += (k + 1) * (LL[4 + k] - LL[2 - k]);
                }
                const int a = 16 * (LL[7] + TT[7]), b = (34 * H + 32) >> 6, cc = (34 * V + 32) >> 6;
                pv = clip3(0, maxv, (a + b * (x - 3) + cc * (y - 3) + 16) >> 5);
            } else {
                const bool at = fl & 1, al = fl & 2;
                const int bx = x >> 2, by = y >> 2;
                int st4 = 0, sl4 = 0;
                for (int k = 0; k < 4; k++) { st4 += TT[bx * 4 + k]; sl4 += LL[by * 4 + k]; }
                if (bx == by) pv = (at && al) ? (st4 + sl4 + 4) >> 3 : (at ? (st4 + 2) >> 2 : (al ? (sl4 + 2) >> 2 : 1 << (bd - 1)));
                else if (bx) pv = at ? (st4 + 2) >> 2 : (al ? (sl4 + 2) >> 2 : 1 << (bd - 1));
                else pv = al ? (sl4 + 2) >> 2 : (at ? (st4 + 2) >> 2 : 1 << (bd - 1));
            }
        }
        WIN(x, y) = static_cast<uint16_t>(clip3(0, maxv, pv + r));
    }
#undef WIN
    wave_sync();
}

// The Cb and Cr blocks of one macroblock (8x8 each at 4:2:0; same mode and availability) in
// one pass: Cb's references in top / left, Cr's in ftop / fleft (the 8x8 luma filter buffers,
// unused by chroma), both predicted + reconstructed per lane (8.3.4).
DEVI void h264_predict_chroma_pair(const h2j_tu& tb, const h2j_tu& tr, uint64_t mask, int bd, H4WaveLds& s,
                                   const H4In& in, int lane) {
    // lane = (y, x) of both 8x8 blocks; references read straight from the window (unavailable ones
    // as 0), the DC quarter sums and the plane gradients by cross-lane adds -- no reference arrays
    const int maxv = (1 << bd) - 1;
    const bool cbf_b = (tb.flags & H2J_TU_CBF) != 0, cbf_r = (tr.flags & H2J_TU_CBF) != 0;
    const int fl = static_cast<int>(mask & 15);  // bits: 0 top, 1 left, 2 corner
    const bool at = fl & 1, al = fl & 2, ad = fl & 4;
    const int mode = tb.mode;
    const int x = lane & 7, y = lane >> 3;
    int pv[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int tx = at ? s.wc[c][0][1 + x] : 0, ly = al ? s.wc[c][1 + y][0] : 0;
        if (mode == 1) {
            pv[c] = ly;
        } else if (mode == 2) {
            pv[c] = tx;
        } else if (mode == 3) {
            // lanes 0-3: H terms (k + 1)(p[4 + k, -1] - p[2 - k, -1]), lanes 8-11: V terms (k = 3: the corner)
            const int k = lane & 3;
            const bool vl = (lane & 8) != 0;
            const int pa = vl ? (al ? s.wc[c][5 + k][0] : 0) : (at ? s.wc[c][0][5 + k] : 0);
            const int pbi = 3 - k;
            const int pb = pbi == 0 ? (ad ? s.wc[c][0][0] : 0) : (vl ? (al ? s.wc[c][pbi][0] : 0) : (at ? s.wc[c][0][pbi] : 0));
            const int term = (lane & 0x34) == 0 ? (k + 1) * (pa - pb) : 0;  // lanes 0-3 and 8-11
            const int H = wave_sum_dpp(vl ? 0 : term), V = wave_sum_dpp(vl ? term : 0);
            const int a = 16 * ((al ? s.wc[c][8][0] : 0) + (at ? s.wc[c][0][8] : 0));
            const int b = (34 * H + 32) >> 6, cc = (34 * V + 32) >> 6;
            pv[c] = clip3(0, maxv, (a + b * (x - 3) + cc * (y - 3) + 16) >> 5);
        } else {
            // DC per 4x4 quarter: lanes 0-7 hold p[x, -1], lanes 8-15 p[-1, x - 8]; after row_shr 1
            // and 2 adds lane i holds a[i] + a[i-1] + a[i-2] + a[i-3], so lanes 3, 7, 11, 15 hold the
            // four quarter sums
            int v = lane < 8 ? tx : (lane < 16 ? (al ? s.wc[c][1 + (lane - 8)][0] : 0) : 0);
            v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
            v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
            const int t0 = __builtin_amdgcn_readlane(v, 3), t1 = __builtin_amdgcn_readlane(v, 7);
            const int l0 = __builtin_amdgcn_readlane(v, 11), l1 = __builtin_amdgcn_readlane(v, 15);
            const int bx = x >> 2, by = y >> 2;
            const int st4 = bx ? t1 : t0, sl4 = by ? l1 : l0;
            const int half = 1 << (bd - 1);
            int d;
            if (bx == by) d = (at && al) ? (st4 + sl4 + 4) >> 3 : (at ? (st4 + 2) >> 2 : (al ? (sl4 + 2) >> 2 : half));
            else if (bx) d = at ? (st4 + 2) >> 2 : (al ? (sl4 + 2) >> 2 : half);
            else d = al ? (sl4 + 2) >> 2 : (at ? (st4 + 2) >> 2 : half);
            pv[c] = d;
        }
    }
    const int rb = cbf_b ? in.rc[0][y][x] : 0, rr = cbf_r ? in.rc[1][y][x] : 0;
    s.wc[0][y + 1][x + 1] = static_cast<uint16_t>(clip3(0, maxv, pv[0] + rb));
    s.wc[1][y + 1][x + 1] = static_cast<uint16_t>(clip3(0, maxv, pv[1] + rr));
    wave_sync();
}

// H.264 macroblock rows.  Per MB: the records, availability masks and K0 residual, fetched by
// LDS-DMA into the wave's other H4In buffer while the previous MB runs (in raster order the next
// MB's records start where this MB's end; no registers are held across the MB), the line above
// from a per-picture LDS line buffer (each row leaves its unfiltered bottom samples there; the
// top-left corner is carried), the prediction chain in the LDS window, one store of the MB.
template <typename Pel, int NW>
DEVI void h264_rows(const h2j_frame& f, const h2j_tu* T, uint8_t* arena, H4WaveLds& s, uint32_t* prog,
                    uint16_t* line, int band, int nbands) {
    const int w = threadIdx.x >> 6;
    // lane: laundered at every macroblock (below) so the compiler recomputes the lane-dependent
    // LDS / global addresses inside the loop instead of hoisting dozens of them into registers that
    // then spill -- each scratch reload is a vmcnt(0), which also waits for the next MB's LDS-DMA
    int lane = threadIdx.x & 63;
    const uint64_t* masks = reinterpret_cast<const uint64_t*>(arena + ufl64(f.aux));
    const uint32_t* rng = reinterpret_cast<const uint32_t*>(arena + ufl64(f.ctbrng));
    constexpr int kSlots = 2 * NW;
    const int mbw = ufl(f.ctb_w), mbh = ufl(f.ctb_h);
    const int W = ufl(f.width), Wc = W >> 1;
    const int bdy = ufl(f.bit_depth), bdc = ufl(f.bit_depth_c);
    const int sty = ufl(f.pic_stride[0]), stc = ufl(f.pic_stride[1]);
    Pel* PY = reinterpret_cast<Pel*>(arena + ufl64(f.pic));
    Pel* PC[2] = {PY + ufl(f.pic_off[1]), PY + ufl(f.pic_off[2])};
    const int16_t* RY = reinterpret_cast<const int16_t*>(arena + ufl64(f.res));  // MB tiles (h264_res_at)
    uint16_t* LY = line;            // [W]: bottom luma row of the MB row above
    uint16_t* LC = line + W;        // [2][Wc]
    const uint32_t ntot = ufl(f.ntu);
    AVP_DECL;
    // this workgroup's rows: one band of NW MB rows (one per wave; tall pictures run on several
    // workgroups: 16-row bands in the merged launch, 8-row ones in h2j_k1_recon_h264) or,
    // unbanded, rows w, w + NW, ...
    const int rbeg = band * NW, rend = nbands > 1 ? min(mbh, rbeg + NW) : mbh;
    // band hand-off: per-row progress words (4th word of the row's first CTB range, zeroed) and
    // the boundary rows, both accessed with agent-scope atomics (coherent across CUs / XCDs)
    const uint64_t o_flag = ufl64(f.ctbrng) + 12, o_xl = ufl64(f.xline);
    if (rbeg + w >= rend) return;
    const uint32_t* masks32 = reinterpret_cast<const uint32_t*>(masks);
    // records (lanes 0..23, dwordx4), mask halves (dword each) and residual (the MB's 768-B tile,
    // lanes 0..47 16 B each: ry and rc are contiguous in H4In as in the tile) of MB (mx, my)
    auto in_recs = [&](uint32_t a, H4In& d) __attribute__((always_inline)) {
        if (lane < kH4MaxTus) {
            const uint32_t ri = min(a + static_cast<uint32_t>(lane), max(ntot, 1u) - 1);
            lds_dma16(T + ri, lds_addr(d.tus));
            lds_dma4(masks32 + 2 * ri, lds_addr(d.mlo));
            lds_dma4(masks32 + 2 * ri + 1, lds_addr(d.mhi));
        }
    };
    auto in_fetch = [&](int mx, int my, uint32_t a, H4In& d) __attribute__((always_inline)) {
        in_recs(a, d);
        if (lane < 48) lds_dma16(RY + static_cast<size_t>(my * mbw + mx) * 384 + lane * 8, lds_addr(d.ry));
    };
    int cur = 0;
    uint32_t pre_a = rng[4 * ((rbeg + w) * mbw)];  // first record the prefetch assumed
    in_fetch(0, rbeg + w, pre_a, s.in[0]);
    uint16_t cy_corner = 0, cc_corner[2] = {0, 0};  // carried top-left samples (luma, Cb, Cr)
    // A staged 4-MB group goes out as 64-sample luma / 32-sample chroma rows (whole 64-byte segments
    // at 8 bits).  Its stores are issued in the next MB's window step, after that MB's inputs have
    // been waited for: issued at the end of the group's last MB they sat in the vmcnt(0) wait for
    // the next MB's LDS-DMA (one counter for loads and stores).
    // Groups are 8 MBs at 8 bits (128-byte luma / 64-byte chroma rows: whole lines -- 32-byte
    // halves of a line written at different times left K1's WRITE at 1.39x the picture, r04m) and
    // 4 MBs at 16 bits (the staging tile holds either)
    constexpr int G = sizeof(Pel) == 1 ? 8 : 4, LW = 16 * G, CW = 8 * G;  // MBs per group, row widths
    constexpr int SS = 16 / static_cast<int>(sizeof(Pel));                 // samples per 16-byte piece
    int fl_g0 = -1, fl_n = 0, fl_gy = 0, fl_cy = 0;
    auto flush = [&]() __attribute__((always_inline)) {
        if (fl_g0 < 0) return;
        const Pel* SY = reinterpret_cast<const Pel*>(s.stage);
        const Pel* SC = SY + 16 * LW;  // [2][8][CW]
        {  // luma: lane = (row, 2 pieces of 16 bytes)
            const int r = lane >> 2;
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int sp = (lane & 3) * 2 + k;
                if (sp * SS < fl_n * 16)
                    *reinterpret_cast<uint4*>(PY + (fl_gy + r) * sty + fl_g0 * 16 + sp * SS) =
                        *reinterpret_cast<const uint4*>(SY + r * LW + sp * SS);
            }
        }
        {  // chroma: lane = (component, row, 16-byte piece: 2 MBs at 8 bits, 1 at 16)
            constexpr int MPS = SS / 8;  // MBs per piece
            const int c = lane >> 5, cr = (lane >> 2) & 7, sg = lane & 3;
            const Pel* src = SC + (c * 8 + cr) * CW + sg * SS;
            Pel* dst = PC[c] + (fl_cy + cr) * stc + fl_g0 * 8 + sg * SS;
            if (sg * MPS + MPS <= fl_n) {
                if (sizeof(Pel) == 2 || (stc & 15) == 0) {
                    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
                } else {  // 8-byte-aligned chroma rows (width an odd multiple of 16)
                    reinterpret_cast<uint2*>(dst)[0] = reinterpret_cast<const uint2*>(src)[0];
                    reinterpret_cast<uint2*>(dst)[1] = reinterpret_cast<const uint2*>(src)[1];
                }
            } else if (sg * MPS < fl_n) {  // 8 bits: a group's odd last MB
                *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(src);
            }
        }
        fl_g0 = -1;
    };
    for (int row = rbeg + w; row < rend; row += NW) {
        uint32_t* above = prog + (row + kSlots - 1) % kSlots;
        uint32_t* mine = prog + row % kSlots;
        uint32_t seen = 0;
        const bool from_band = nbands > 1 && band > 0 && row == rbeg;             // line above from the band above
        const bool to_band = nbands > 1 && band < nbands - 1 && row == rend - 1;  // bottom row to the band below
        // boundary b (between bands b and b + 1): W dwords = 2W uint16 (luma W, then Cb, Cr Wc each)
        const uint64_t o_xin = o_xl + 4ull * (band - 1) * W, o_xout = o_xl + 4ull * band * W;
        const int gy = row * 16, cy = row * 8;
        for (int mx = 0; mx < mbw; mx++) {
            asm volatile("" : "+v"(lane));
            const int gx = mx * 16, cx = mx * 8;
            const int cb = row * mbw + mx;
            const uint4 rg = reinterpret_cast<const uint4*>(rng)[cb];
            const uint32_t a = rg.x, ntu = min(rg.z - rg.x, static_cast<uint32_t>(kH4MaxTus));
            // the wave's next MB and its first record (loaded here, with rg: a load still in flight
            // when the prefetch DMA is issued makes the compiler wait vmcnt(0) -- for the DMA too --
            // at its first use)
            int nx = mx + 1, ny = row;
            uint32_t na = rg.z;
            if (nx == mbw) {
                nx = 0;
                ny += NW;
                na = ny < mbh ? rng[4 * (ny * mbw)] : 0;
            }
            if (from_band) {  // the row above belongs to another workgroup: bounded wait on its global word
                const uint32_t need = static_cast<uint32_t>(min(mx + 2, mbw));
                if (seen < need) {
                    uint32_t it = 0;
                    uint32_t* fl = reinterpret_cast<uint32_t*>(arena + o_flag) + 4 * ((row - 1) * mbw);
                    while ((seen = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < need) {
                        __builtin_amdgcn_s_sleep(2);
                        if (++it > (1u << 22)) {  // never expected: flag the picture, do not hang the GPU
                            if (lane == 0) __hip_atomic_fetch_or(dev_error_word(arena, f), kDevErrK1Band, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            seen = static_cast<uint32_t>(mbw);
                            break;
                        }
                    }
                }
            } else if (row > rbeg || (row > 0 && nbands <= 1)) {
                const uint32_t need = (static_cast<uint32_t>(row) << 16) | static_cast<uint32_t>(min(mx + 2, mbw));
                if (seen < need) seen = wait_progress(above, need, dev_error_word(arena, f), kDevErrK1Row264);
            }
            AVP_LAP(0);
            // ---- window: the DMA'd inputs, line above from LDS, left column carried
            H4In& in = s.in[cur];
            lds_dma_wait();
            asm volatile("" ::"v"(na));  // its load retired here, with the DMA wait
            if (pre_a != a) {  // an MB without records before this one: reload the records
                lds_reads_done();
                in_recs(a, in);
                lds_dma_wait();
            }
            flush();  // the previous group's rows (staged and synced at the end of the previous MB)
            if (from_band) {  // boundary row of the band above (uint16 pairs in dwords, agent-scope loads)
                int x = -1, e = 0;
                if (lane < 25) { x = gx - 1 + lane; e = x; }
                else if (lane < 43) { const int k = lane - 25, c = k / 9; x = cx - 1 + k % 9; e = W + c * Wc + x; }
                const bool ok = x >= 0 && (lane < 25 ? x < W : x < Wc);
                const uint32_t d = ok ? __hip_atomic_load(reinterpret_cast<const uint32_t*>(arena + o_xin) + (e >> 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                const uint16_t v = ok ? static_cast<uint16_t>((e & 1) ? (d >> 16) : (d & 0xFFFF)) : 0;
                if (lane < 25) s.wy[0][lane] = v;
                else if (lane < 43) { const int k = lane - 25; s.wc[k / 9][0][k % 9] = v; }
            } else if (lane < 25) {  // luma x = gx - 1 .. gx + 23
                const int x = gx - 1 + lane;
                uint16_t v = 0;
                if (row > 0 && x >= 0 && x < W) v = lane == 0 ? cy_corner : LY[x];
                s.wy[0][lane] = v;
            } else if (lane < 43) {
                const int k = lane - 25, c = k / 9, i = k % 9, x = cx - 1 + i;
                uint16_t v = 0;
                if (row > 0 && x >= 0 && x < Wc) v = i == 0 ? (c ? cc_corner[1] : cc_corner[0]) : LC[c * Wc + x];
                s.wc[c][0][i] = v;
            }
            if (mx == 0) {  // left of the picture: never available
                if (lane < 16) s.wy[lane + 1][0] = 0;
                else if (lane < 32) s.wc[(lane - 16) >> 3][((lane - 16) & 7) + 1][0] = 0;
            }
            {  // prefetch the wave's next MB (its records follow this MB's in raster order)
                if (ny < mbh) {
                    lds_reads_done();  // the other buffer's last reader, the previous MB, has finished
                    in_fetch(nx, ny, na, s.in[cur ^ 1]);
                    pre_a = na;
                }
            }
            wave_sync();
            // the next MB's top-left corners = this MB's top line end (about to be overwritten)
            cy_corner = s.wy[0][16];
            cc_corner[0] = s.wc[0][0][8];
            cc_corner[1] = s.wc[1][0][8];
            const bool pcm = ntu > 0 && (in.tus[0].flags & H2J_TU_PCM);
            AVP_LAP(1);
            AVP_ADD(6, 1);
            AVP_ADD(5, ntu);
            if (pcm) {  // samples written by K0: pull them into the window
                for (int i = lane; i < 256; i += 64) s.wy[(i >> 4) + 1][(i & 15) + 1] = PY[(gy + (i >> 4)) * sty + gx + (i & 15)];
                for (int i = lane; i < 128; i += 64) {
                    const int c = i >> 6, k = i & 63;
                    s.wc[c][(k >> 3) + 1][(k & 7) + 1] = PC[c][(cy + (k >> 3)) * stc + cx + (k & 7)];
                }
                wave_sync();
            } else {
                for (uint32_t t = 0; t < ntu; t++) {
                    const h2j_tu tu = in.tus[t];
                    if (tu.c == 1 && tu.log2n == 3 && t + 1 < ntu && in.tus[t + 1].c == 2 && in.tus[t + 1].log2n == 3) {  // Cb + Cr in one pass
                        h264_predict_chroma_pair(tu, in.tus[t + 1], in.mask(t), bdc, s, in, lane);
                        AVP_LAPK(6);
                        t++;
                        continue;
                    }
                    h264_predict_tu(tu, in.mask(t), mx, row, tu.c ? bdc : bdy, s, in, lane);
                    // 8: 4x4, 9: 8x8, 10: 16x16 (+ 3 when the mode is DC), 14: lone chroma
                    AVP_LAPK(tu.c ? 6 : tu.log2n - 2 + (tu.mode == 2 ? 3 : 0));
                }
            }
            AVP_LAP(2);
            // ---- stage the macroblock in the wave's 4-MB-wide staging rows; every 4th MB (and the
            // row's last) the group goes out as 64-sample luma / 32-sample chroma rows, whole
            // 64-byte segments at 8 bits instead of 16-byte pieces per MB (a PCM MB's samples,
            // already in the picture, are rewritten unchanged)
            {
                Pel* SY = reinterpret_cast<Pel*>(s.stage);
                Pel* SC = SY + 16 * LW;  // [2][8][CW]
                const int r = lane >> 2, c4 = (lane & 3) * 4, sx = (mx % G) * 16;
#pragma unroll
                for (int k = 0; k < 4; k++) SY[r * LW + sx + c4 + k] = static_cast<Pel>(s.wy[r + 1][c4 + 1 + k]);
                const int c = lane >> 5, kk = lane & 31, rr = kk >> 2, c2 = (kk & 3) * 2, scx = (mx % G) * 8;
                SC[(c * 8 + rr) * CW + scx + c2] = static_cast<Pel>(s.wc[c][rr + 1][c2 + 1]);
                SC[(c * 8 + rr) * CW + scx + c2 + 1] = static_cast<Pel>(s.wc[c][rr + 1][c2 + 2]);
            }
            // a complete group is stored in the next MB's window step
            if (mx % G == G - 1 || mx == mbw - 1) {
                fl_g0 = mx - mx % G;
                fl_n = mx - fl_g0 + 1;
                fl_gy = gy;
                fl_cy = cy;
            }
            // bottom row for the MB row below; right column becomes the next MB's left column
            if (to_band) {  // hand the bottom row to the band below: data, wait for completion, then progress
                if (lane < 16) {
                    int e0, v0, v1;
                    if (lane < 8) { e0 = gx + 2 * lane; v0 = s.wy[16][2 * lane + 1]; v1 = s.wy[16][2 * lane + 2]; }
                    else { const int c = (lane - 8) >> 2, i = ((lane - 8) & 3) * 2; e0 = W + c * Wc + cx + i;
                           v0 = s.wc[c][8][i + 1]; v1 = s.wc[c][8][i + 2]; }
                    __hip_atomic_store(reinterpret_cast<uint32_t*>(arena + o_xout) + (e0 >> 1), static_cast<uint32_t>(v0) | (static_cast<uint32_t>(v1) << 16),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the boundary stores have completed
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0)
                    __hip_atomic_store(reinterpret_cast<uint32_t*>(arena + o_flag) + 4 * (row * mbw), static_cast<uint32_t>(mx + 1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            } else if (row + 1 < mbh) {
                if (lane < 16) LY[gx + lane] = s.wy[16][lane + 1];
                else if (lane < 32) {
                    const int c = (lane - 16) >> 3, i = (lane - 16) & 7;
                    LC[c * Wc + cx + i] = s.wc[c][8][i + 1];
                }
            }
            if (lane < 16) s.wy[lane + 1][0] = s.wy[lane + 1][16];
            else if (lane < 32) {
                const int c = (lane - 16) >> 3, i = ((lane - 16) & 7) + 1;
                s.wc[c][i][0] = s.wc[c][i][8];
            }
            wave_sync();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0)
                __hip_atomic_store(mine, ((static_cast<uint32_t>(row) + 1) << 16) | static_cast<uint32_t>(mx + 1),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            cur ^= 1;
            AVP_LAP(3);
        }
    }
    flush();  // the wave's last group (synced at the end of its last MB)
    AVP_FLUSH();
}

// H.264 K1 for MBAFF frames (h2j_frame.mbaff): macroblock pairs, wave w walking pair rows w, w + 16,
// ... (a pair needs the pair row above finished through the pair to its right, as h264_rows needs
// the MB row above).  Per MB (top, then bottom of the pair) the window is filled from the picture
// itself, in the MB's own field / frame view: row r of a field MB is picture row 2 r + bottom of
// the pair, its row -1 the picture row two above its first row; a frame MB's rows are consecutive.
// With the 6.4.12.2 neighbour rules those are exactly the samples intra prediction reads (the
// availability masks come from the host parser).  The MB is reconstructed in the window by the
// progressive TB code and stored to its picture rows.  Samples pass between MBs / waves through
// global memory: release / acquire fences around the progress words and between MBs.
template <typename Pel>
DEVI void h264_rows_mbaff(const h2j_frame& f, const h2j_tu* T, const h2j_ctb* C, uint8_t* arena, H4WaveLds& s,
                          uint32_t* prog) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t* masks = reinterpret_cast<const uint64_t*>(arena + ufl64(f.aux));
    const uint32_t* masks32 = reinterpret_cast<const uint32_t*>(masks);
    const uint32_t* rng = reinterpret_cast<const uint32_t*>(arena + ufl64(f.ctbrng));
    constexpr int kSlots = 2 * kAvcWaves;
    const int mbw = ufl(f.ctb_w), npr = ufl(f.ctb_h) >> 1;
    const int W = ufl(f.width), Wc = W >> 1;
    const int bdy = ufl(f.bit_depth), bdc = ufl(f.bit_depth_c);
    const int sty = ufl(f.pic_stride[0]), stc = ufl(f.pic_stride[1]);
    Pel* PY = reinterpret_cast<Pel*>(arena + ufl64(f.pic));
    Pel* PC[2] = {PY + ufl(f.pic_off[1]), PY + ufl(f.pic_off[2])};
    const int16_t* RY = reinterpret_cast<const int16_t*>(arena + ufl64(f.res));
    const uint32_t ntot = ufl(f.ntu);
    H4In& in = s.in[0];
    for (int pr = w; pr < npr; pr += kAvcWaves) {
        uint32_t* above = prog + (pr + kSlots - 1) % kSlots;
        uint32_t* mine = prog + pr % kSlots;
        uint32_t seen = 0;
        const int Y0 = pr * 32, Yc0 = pr * 16;
        for (int x = 0; x < mbw; x++) {
            if (pr > 0) {
                const uint32_t need = (static_cast<uint32_t>(pr) << 16) | static_cast<uint32_t>(min(x + 2, mbw));
                if (seen < need) seen = wait_progress(above, need, dev_error_word(arena, f), kDevErrK1Row264);
            }
            const bool fld = (C[(2 * pr) * mbw + x].mbflags & 8) != 0;
            for (int bot = 0; bot < 2; bot++) {
                const int vy = 2 * pr + bot, cb = vy * mbw + x;
                const uint4 rg = reinterpret_cast<const uint4*>(rng)[cb];
                const uint32_t a = rg.x, ntu = min(rg.z - rg.x, static_cast<uint32_t>(kH4MaxTus));
                // records, masks and the MB's residual tile (h264_res_at) into the window's inputs
                lds_reads_done();
                if (lane < kH4MaxTus) {
                    const uint32_t ri = min(a + static_cast<uint32_t>(lane), max(ntot, 1u) - 1);
                    lds_dma16(T + ri, lds_addr(in.tus));
                    lds_dma4(masks32 + 2 * ri, lds_addr(in.mlo));
                    lds_dma4(masks32 + 2 * ri + 1, lds_addr(in.mhi));
                }
                if (lane < 48) lds_dma16(RY + static_cast<size_t>(cb) * 384 + lane * 8, lds_addr(in.ry));
                // picture rows of this MB's rows -1 .. 15 (luma) / -1 .. 7 (chroma)
                auto yrow = [&](int r) { return fld ? Y0 + 2 * r + bot : Y0 + 16 * bot + r; };
                auto crow = [&](int r) { return fld ? Yc0 + 2 * r + bot : Yc0 + 8 * bot + r; };
                const int ya = fld ? Y0 + bot - 2 : yrow(-1), ca = fld ? Yc0 + bot - 2 : crow(-1);
                if (lane < 25) {  // luma row -1, x = -1 .. 23
                    const int xx = x * 16 - 1 + lane;
                    s.wy[0][lane] = (ya >= 0 && xx >= 0 && xx < W) ? static_cast<uint16_t>(PY[ya * sty + xx]) : 0;
                } else if (lane < 43) {  // chroma row -1, x = -1 .. 7
                    const int k = lane - 25, c = k / 9, i = k % 9, xx = x * 8 - 1 + i;
                    s.wc[c][0][i] = (ca >= 0 && xx >= 0 && xx < Wc) ? static_cast<uint16_t>(PC[c][ca * stc + xx]) : 0;
                }
                if (lane < 16) {  // left column
                    s.wy[lane + 1][0] = x > 0 ? static_cast<uint16_t>(PY[yrow(lane) * sty + x * 16 - 1]) : 0;
                } else if (lane < 32) {
                    const int c = (lane - 16) >> 3, r = (lane - 16) & 7;
                    s.wc[c][r + 1][0] = x > 0 ? static_cast<uint16_t>(PC[c][crow(r) * stc + x * 8 - 1]) : 0;
                }
                lds_dma_wait();
                wave_sync();
                const bool pcm = ntu > 0 && (in.tus[0].flags & H2J_TU_PCM);
                if (pcm) {  // samples written by K0 (at this MB's picture rows)
                    for (int i = lane; i < 256; i += 64) s.wy[(i >> 4) + 1][(i & 15) + 1] = PY[yrow(i >> 4) * sty + x * 16 + (i & 15)];
                    for (int i = lane; i < 128; i += 64) {
                        const int c = i >> 6, k = i & 63;
                        s.wc[c][(k >> 3) + 1][(k & 7) + 1] = PC[c][crow(k >> 3) * stc + x * 8 + (k & 7)];
                    }
                    wave_sync();
                } else {
                    for (uint32_t t = 0; t < ntu; t++) {
                        const h2j_tu tu = in.tus[t];
                        if (tu.c == 1 && tu.log2n == 3 && t + 1 < ntu && in.tus[t + 1].c == 2 && in.tus[t + 1].log2n == 3) {
                            h264_predict_chroma_pair(tu, in.tus[t + 1], in.mask(t), bdc, s, in, lane);
                            t++;
                            continue;
                        }
                        h264_predict_tu(tu, in.mask(t), x, vy, tu.c ? bdc : bdy, s, in, lane);
                    }
                }
                // the MB's rows to the picture: luma lane = (row, 4 samples), chroma lane = (comp, row, 2 x 2 samples)
                {
                    const int r = lane >> 2, q = (lane & 3) * 4;
                    Pel* d = PY + yrow(r) * sty + x * 16 + q;
#pragma unroll
                    for (int k = 0; k < 4; k++) d[k] = static_cast<Pel>(s.wy[r + 1][q + 1 + k]);
                    const int c = lane >> 5, rr = (lane >> 2) & 7, qq = (lane & 3) * 2;
                    Pel* e = PC[c] + crow(rr) * stc + x * 8 + qq;
                    e[0] = static_cast<Pel>(s.wc[c][rr + 1][qq + 1]);
                    e[1] = static_cast<Pel>(s.wc[c][rr + 1][qq + 2]);
                }
                // the next MB of this wave reads these samples back from the picture
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                wave_sync();
            }
            if (lane == 0)
                __hip_atomic_store(mine, ((static_cast<uint32_t>(pr) + 1) << 16) | static_cast<uint32_t>(x + 1),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// HEVC K1.  Per picture, two workgroups run side by side: group 0 walks the
// luma TB chain, group 1 the Cb/Cr chains (intra prediction never crosses
// components, H.265 8.4.4.2.1), halving the dependent chain each one walks.
// Wave w of a group reconstructs CTB rows w, w + kK1Waves, ... one 32x32
// quadrant (16x16 chroma) at a time — the z-scan visits quadrants in order and
// no TB is larger than 32x32 — in a small int16 LDS window, so a group needs
// ~36 KB of LDS and several pictures share a CU.  The quadrant's K0 residual
// is prefetched into registers one quadrant ahead and dropped into the window
// when the quadrant starts; every TB reads its residual and writes its
// reconstruction in place (a TB only reads neighbours that are already
// reconstructed, so the two never alias).  Neighbours come from LDS only: the
// line above from a per-group line buffer (each CTB row leaves its bottom line
// there), the rest from carries (previous CTB's right column, the top
// quadrants' bottom rows, the left quadrant's right column, the next CTB's
// top-left corner).  TU records stream in 64-record batches held one per lane
// (readlane).  HBM is touched only by the prefetches and the quadrant stores.
// Frame fields the K1 loops use, read once into scalar registers.  Reading
// them through the h2j_frame reference inside the loops made the compiler
// re-load them from global memory after every fence, each time waiting for
// every outstanding load and store of the wave (vmcnt(0)).  Per-component
// values are selected, never indexed, so nothing lands in scratch.
// (pointers stay `arena + uniform offset`, so the compiler keeps them global
// and emits global_load, not flat_load — flat ops would also hold lgkmcnt)
struct FU {
    int width, height, log2ctb, ctb_w, ctb_h, bd, bdc, strong, sty, stc;
    uint8_t* pic;     // plane 0 base (bytes); planes 1/2 at off1/off2 elements
    int16_t* res;     // residual planes, tiled by quadrant (hevc_res_at)
    int off1, off2;
    uint32_t* derr;   // the picture's h2j_jstat.dev_error
    DEVI int st(int c) const { return c ? stc : sty; }
    DEVI int off(int c) const { return c == 0 ? 0 : (c == 1 ? off1 : off2); }
    template <typename Pel>
    DEVI Pel* plane(int c) const { return reinterpret_cast<Pel*>(pic) + off(c); }
};
DEVI FU make_fu(const h2j_frame& f, uint8_t* arena) {
    FU u;
    u.width = ufl(f.width);
    u.height = ufl(f.height);
    u.log2ctb = ufl(f.log2ctb);
    u.ctb_w = ufl(f.ctb_w);
    u.ctb_h = ufl(f.ctb_h);
    u.bd = ufl(f.bit_depth);
    u.bdc = ufl(f.bit_depth_c);
    u.strong = ufl(f.strong_smoothing);
    u.sty = ufl(f.pic_stride[0]);
    u.stc = ufl(f.pic_stride[1]);
    u.off1 = ufl(f.pic_off[1]);
    u.off2 = ufl(f.pic_off[2]);
    u.pic = arena + ufl64(f.pic);
    u.res = reinterpret_cast<int16_t*>(arena + ufl64(f.res));
    u.derr = dev_error_word(arena, f);
    return u;
}

struct QComp {              // one component's carried neighbours (quadrant size Qc <= 32, CTB size Sc <= 64)
    int16_t top[68];        // y = -1: x = -1 .. 2Qc-1 (index x + 1)
    int16_t left[64];       // x = -1: y = 0 .. 2Qc-1
    int16_t prevR[2][64];   // right column of the previous CTB (double-buffered by CTB parity)
    int16_t qbot[64];       // bottom rows of the top quadrant row (TL | TR)
    int16_t qright[32];     // right column of the left quadrant (TL for TR, BL for BR)
    int16_t corner, pad;    // top-left sample of the next CTB
};
struct QWave {
    int16_t body[2][32 * 32];  // quadrant windows (ping-pong): luma | Cb at 0 and Cr at 256 (16x16 each)
    QComp cs[2];            // luma: cs[0]; chroma: Cb cs[0], Cr cs[1]
    K1WaveLds k;
};
// dynamic LDS of one K1 group: QWave[kK1Waves], prog[2 * kK1Waves], line[2 * max width] (int16)
__host__ __device__ constexpr size_t k1_fixed_lds(int waves) { return sizeof(QWave) * waves + 2 * waves * sizeof(uint32_t); }


// intraPredAngle / invAngle (H.265 Tables 8-4, 8-5) from the mode with scalar
// arithmetic on packed constants (no memory round trip per TB):
// d = m - 26 (vertical) or 10 - m (horizontal), angle = sign(d) * mag[|d|].  (m24 -- see its
// definition -- multiplies a sample (<= 16 bits) or a window / angle index by a small factor.)
// Both from k = |d| with no compare chain (r05: resolving invAngle by comparing the angle against
// its eight values compiled to ~40 scalar instructions and branches per angular TB).
struct HevcAng {
    int angle, inv;  // inv: only used for angle < 0, -round(8192 / |angle|)
};
DEVI HevcAng hevc_ang(int m) {
    const int d = m >= 18 ? m - 26 : 10 - m;
    const int k = d < 0 ? -d : d;
    const int mag = k == 8 ? 32 : static_cast<int>((0x1A15110D09050200ull >> (8 * k)) & 0xFF);
    // |invAngle| for k = 1..8: 4096, 1638, 910, 630 | 482, 390, 315, 256 (k = 0: unused)
    const int km = (k - 1) & 3;
    const uint64_t tab = k <= 4 ? 0x0276038E06661000ull : 0x0100013B018601E2ull;
    const int v = static_cast<int>((tab >> (16 * km)) & 0xFFFF);
    return HevcAng{d < 0 ? -mag : mag, -v};
}


// One HEVC TB predicted + reconstructed inside the wave's CTB window
// (H.265 8.4.4.2.2 substitution, 8.4.4.2.3 filtering, 8.4.4.2.4-6 planar / DC /
// angular).  Reference index k: 0 .. 2n-1 = p(-1, 2n-1-k), 2n = p(-1,-1),
// 2n+1 .. 4n = p(k-2n-1, -1).  Each lane first resolves which sample its
// (possibly substituted) reference comes from using only the availability
// ballots, then reads it with one LDS load.
// One copy per TB size 1 << LN (compile-time sizes fold the index arithmetic; LN < 0: any
// size, from tu.log2n).
template <int LN>
DEVI void hevc_predict_tb(const FU& u, const h2j_tu& tu, uint64_t mask, int ox, int oy, int S, int16_t* body,
                          int topo, int lefto, K1WaveLds& s, int lane) {
    const int c = tu.c, log2n = LN >= 0 ? LN : tu.log2n, n = 1 << log2n, nn = n * n;
    const int bd = c ? u.bdc : u.bd;
    const int maxv = (1 << bd) - 1;
    const bool cbf = (tu.flags & H2J_TU_CBF) != 0;
    const int L = 4 * n + 1;
    const int ush = c ? 1 : 2, nu = (2 * n) >> ush;
    const int nch = (L + 63) >> 6;  // 1 (n <= 8 luma / n <= 8 chroma), 2 (n = 16), 3 (n = 32)
    // availability ballots (unit = 4 luma / 2 chroma samples; bit nu = corner)
    unsigned long long m[3] = {0, 0, 0};
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        if (ch < nch) {
            const int k = lane + 64 * ch;
            const int unit = k < 2 * n ? (k >> ush) : nu + ((k - 2 * n + (1 << ush) - 1) >> ush);
            const bool a = k < L && ((mask >> unit) & 1ull);
            m[ch] = __ballot(a);
        }
    }
    const bool any = (m[0] | m[1] | m[2]) != 0;
    // substitution (8.4.4.2.2): sample k takes the last available index <= k, or the
    // first available one; per chunk the "nothing below in this chunk" case is uniform
    const int first = m[0] ? __ffsll(static_cast<long long>(m[0])) - 1
                           : (m[1] ? 64 + __ffsll(static_cast<long long>(m[1])) - 1 : 128);
    const int last0 = m[0] ? 63 - __clzll(m[0]) : first;
    const int fb[3] = {first, last0, m[1] ? 127 - __clzll(m[1]) : last0};
    // neighbour sample -> element index relative to `body` (topo / lefto: the element offsets of
    // the carried top / left arrays from it)
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    int dcpart = 0, v0 = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        if (ch < nch) {
            const int k = lane + 64 * ch;
            const unsigned long long le = m[ch] & upto;
            const int j = le ? 64 * ch + 63 - static_cast<int>(__clzll(le)) : fb[ch];
            const int xn = j > 2 * n ? ox + (j - 2 * n - 1) : ox - 1;
            const int yn = j < 2 * n ? oy + (2 * n - 1 - j) : oy - 1;
            const int idx = yn < 0 ? topo + xn + 1 : (xn < 0 ? lefto + yn : m24(yn, S) + xn);
            const int raw = body[idx];  // unconditional: idx stays inside the wave's window
            const int v = any ? raw : (1 << (bd - 1));
            if (ch == 0) v0 = v;
            if (nch > 1) s.sub[k < L ? k : 131] = static_cast<int16_t>(v);
            // DC: p(-1, 0..n-1) = k in [n, 2n), p(0..n-1, -1) = k in [2n+1, 3n]
            dcpart += (k >= n && k <= 3 * n && k != 2 * n) ? v : 0;
        }
    }
    const int mode = tu.mode;
    bool filt = false;
    if (c == 0 && mode != 1 && n != 4 && !(u.strong & H2J_NO_INTRA_SMOOTHING)) {
        const int d26 = abs(mode - 26), d10 = abs(mode - 10);
        const int md = d26 < d10 ? d26 : d10;
        const int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
        filt = mode == 0 || md > thr;
    }
    int dc = 0;
    if (mode == 1) dc = (wave_sum_dpp(dcpart) + n) >> (log2n + 1);
    const int edge = c == 0 && n < 32;  // DC / pure horizontal / pure vertical boundary smoothing
    if (nch == 1) {
        // L <= 64 (n <= 8 luma, chroma <= 8): lane k keeps reference k in a register; the
        // filter and the prediction read neighbours by ds_bpermute (__shfl) instead of an LDS
        // write, a barrier and LDS reads.  Only luma 8x8 is ever filtered here (no strong filter).
        int r = v0;
        if (filt) {
            const int vl = __shfl(v0, lane - 1, 64), vr = __shfl(v0, lane + 1, 64);
            r = (lane == 0 || lane == 4 * n) ? v0 : (vl + 2 * v0 + vr + 2) >> 2;
        }
        const int i = lane, x = i & (n - 1), y = i >> log2n;
        int pv;
        if (mode == 0) {
            const int tr = __builtin_amdgcn_readlane(r, 3 * n + 1), bl = __builtin_amdgcn_readlane(r, n - 1);
            const int left = __shfl(r, 2 * n - 1 - y, 64), above = __shfl(r, 2 * n + 1 + x, 64);
            pv = (m24(n - 1 - x, left) + m24(x + 1, tr) + m24(n - 1 - y, above) + m24(y + 1, bl) + n) >> (log2n + 1);
        } else if (mode == 1) {
            const int above = __shfl(r, 2 * n + 1 + x, 64), left = __shfl(r, 2 * n - 1 - y, 64);
            // edge samples by selects (lane-divergent branches cost exec-mask scalar work)
            const int pc = (left + 2 * dc + above + 2) >> 2, pt = (above + 3 * dc + 2) >> 2, pl = (left + 3 * dc + 2) >> 2;
            const int pe = x == 0 ? (y == 0 ? pc : pl) : pt;
            pv = edge && (x == 0 || y == 0) ? pe : dc;
        } else {
            const HevcAng ang = hevc_ang(mode);
            const int angle = ang.angle, inv = ang.inv;
            const bool vert = mode >= 18;
            const int sgn = vert ? 1 : -1;
            const bool bnd = edge && (mode == 26 || mode == 10);
            const int a = vert ? y : x, b = vert ? x : y;
            const int pos = m24(a + 1, angle), idx = pos >> 5, fr = pos & 31;
            const int k1 = b + idx + 1, k2 = k1 + 1;
            const int o1 = k1 >= 0 ? k1 : -((m24(k1, inv) + 128) >> 8);
            const int o2 = k2 >= 0 ? k2 : -((m24(k2, inv) + 128) >> 8);
            const int r1 = __shfl(r, 2 * n + (vert ? o1 : -o1), 64), r2 = __shfl(r, 2 * n + (vert ? o2 : -o2), 64);
            pv = (m24(32 - fr, r1) + m24(fr, r2) + 16) >> 5;
            if (bnd) {
                const int side = __shfl(r, 2 * n + (vert ? -(a + 1) : a + 1), 64);
                const int e = clip3(0, maxv, __builtin_amdgcn_readlane(r, 2 * n + sgn) +
                                                 ((side - __builtin_amdgcn_readlane(r, 2 * n)) >> 1));
                pv = b == 0 ? e : pv;
            }
        }
        if (i < nn) {
            int16_t* d = body + m24(oy + y, S) + ox + x;
            *d = static_cast<int16_t>(clip3(0, maxv, pv + (cbf ? *d : 0)));
        }
        wave_sync();
        return;
    }
    wave_sync();
    if (filt) {
        const int corner = s.sub[2 * n];
        const bool strong = (u.strong & 1) && n == 32 &&
                            abs(corner + s.sub[4 * n] - 2 * s.sub[3 * n]) < (1 << (bd - 5)) &&
                            abs(corner + s.sub[0] - 2 * s.sub[n]) < (1 << (bd - 5));
        if (strong) {
            const int bl = s.sub[0], tr = s.sub[4 * n];
#pragma unroll
            for (int it = 0; it < nch; it++) {  // uniform trip count (lane-strided loops juggle exec)
                const int k = lane + 64 * it;
                if (k >= L) break;
                int v;
                if (k == 0 || k == 4 * n || k == 2 * n) v = s.sub[k];
                else if (k < 2 * n) { const int y = 2 * n - 1 - k; v = (m24(63 - y, corner) + m24(y + 1, bl) + 32) >> 6; }
                else { const int x = k - 2 * n - 1; v = (m24(63 - x, corner) + m24(x + 1, tr) + 32) >> 6; }
                s.ref[k] = v;
            }
        } else {
#pragma unroll
            for (int it = 0; it < nch; it++) {
                const int k = lane + 64 * it;
                if (k >= L) break;
                const int v = (k == 0 || k == 4 * n) ? s.sub[k] : (s.sub[k - 1] + 2 * s.sub[k] + s.sub[k + 1] + 2) >> 2;
                s.ref[k] = v;
            }
        }
        wave_sync();
    }
    // p(-1,y) = R[2n-1-y], p(x,-1) = R[2n+1+x], p(-1,-1) = R[2n]
    const int16_t* R = filt ? s.ref : s.sub;
    // four horizontally adjacent samples per lane (n >= 16): the residual quad read and the
    // reconstructed quad written as one 8-byte window access each, the index arithmetic done
    // once per quad (TB origins and window rows are multiples of 4 samples, so the quad is 8-byte
    // aligned)
    const int qsh = log2n - 2, nq4 = nn >> 2;
    auto put4 = [&](int x, int y, int p0, int p1, int p2, int p3) __attribute__((always_inline)) {
        uint2* d = reinterpret_cast<uint2*>(body + m24(oy + y, S) + ox + x);
        int r0 = 0, r1 = 0, r2 = 0, r3 = 0;
        if (cbf) {
            const uint2 rr = *d;
            r0 = static_cast<int>(rr.x << 16) >> 16;
            r1 = static_cast<int>(rr.x) >> 16;
            r2 = static_cast<int>(rr.y << 16) >> 16;
            r3 = static_cast<int>(rr.y) >> 16;
        }
        *d = make_uint2(static_cast<uint32_t>(clip3(0, maxv, p0 + r0) | (clip3(0, maxv, p1 + r1) << 16)),
                        static_cast<uint32_t>(clip3(0, maxv, p2 + r2) | (clip3(0, maxv, p3 + r3) << 16)));
    };
    if (mode == 0) {
        const int tr = R[3 * n + 1], bl = R[n - 1];
        #pragma unroll 1
        for (int it = 0; it < (nq4 >> 6); it++) {  // n >= 16 here: nq4 a multiple of 64
            const int i = lane + 64 * it;
            const int x = (i & ((n >> 2) - 1)) * 4, y = i >> qsh;
            const int ly = R[2 * n - 1 - y];
            const int base = m24(y + 1, bl) + n, wy = n - 1 - y, dd = tr - ly;
            const int a0 = m24(n - 1 - x, ly) + m24(x + 1, tr) + base;
            put4(x, y, (a0 + m24(wy, R[2 * n + 1 + x])) >> (log2n + 1), (a0 + dd + m24(wy, R[2 * n + 2 + x])) >> (log2n + 1),
                 (a0 + 2 * dd + m24(wy, R[2 * n + 3 + x])) >> (log2n + 1), (a0 + 3 * dd + m24(wy, R[2 * n + 4 + x])) >> (log2n + 1));
        }
    } else if (mode == 1) {
        #pragma unroll 1
        for (int it = 0; it < (nq4 >> 6); it++) {  // n >= 16 here: nq4 a multiple of 64
            const int i = lane + 64 * it;
            const int x = (i & ((n >> 2) - 1)) * 4, y = i >> qsh;
            int p0 = dc, p1 = dc, p2 = dc, p3 = dc;
            if (edge) {  // uniform; the edge samples by selects
                const bool top = y == 0, lft = x == 0;
                const int t0 = R[2 * n + 1 + x], c0 = (R[2 * n - 1] + 2 * dc + t0 + 2) >> 2;
                const int l0 = (R[2 * n - 1 - y] + 3 * dc + 2) >> 2;
                p0 = top ? (lft ? c0 : (t0 + 3 * dc + 2) >> 2) : (lft ? l0 : dc);
                p1 = top ? (R[2 * n + 2 + x] + 3 * dc + 2) >> 2 : dc;
                p2 = top ? (R[2 * n + 3 + x] + 3 * dc + 2) >> 2 : dc;
                p3 = top ? (R[2 * n + 4 + x] + 3 * dc + 2) >> 2 : dc;
            }
            put4(x, y, p0, p1, p2, p3);
        }
    } else {
        const HevcAng ang = hevc_ang(mode);
        const int angle = ang.angle, inv = ang.inv;
        const bool vert = mode >= 18;
        // vertical: main = top row (refV(k) = R[2n + k], k < 0 projected from the left column);
        // horizontal: main = left column (refH(k) = R[2n - k], k < 0 projected from the top row)
        const int sgn = vert ? 1 : -1;
        const bool bnd = edge && (mode == 26 || mode == 10);
        // the main reference extended to negative positions once per TB (8.4.4.2.6: ref[k] for
        // k < 0 projects onto the side reference through invAngle), M[n + k] for k = -n .. 2n + 1, in
        // the reference array R is not: the sample loop then reads entries with no projection
        int16_t* M = filt ? s.sub : s.ref;
#pragma unroll
        for (int it = 0; it < (3 * n + 2 + 63) / 64; it++) {
            const int k = lane + 64 * it;
            if (k >= 3 * n + 2) break;
            const int kk = k - n;
            const int o = kk >= 0 ? kk : -((m24(kk, inv) + 128) >> 8);
            // (entry 2n + 1 is only ever read with weight 0 -- clamped into R)
            M[k] = R[clip3(0, 4 * n, 2 * n + sgn * o)];
        }
        wave_sync();
        auto lerp = [](int fr, int a, int b) __attribute__((always_inline)) { return (m24(32 - fr, a) + m24(fr, b) + 16) >> 5; };
        if (vert) {  // the quad shares its row, so its position along the angle: five entries
            #pragma unroll 1
            for (int it = 0; it < (nq4 >> 6); it++) {  // n >= 16 here: nq4 a multiple of 64
            const int i = lane + 64 * it;
                const int x = (i & ((n >> 2) - 1)) * 4, y = i >> qsh;
                const int pos = m24(y + 1, angle), fr = pos & 31;
                const int k1 = n + x + (pos >> 5) + 1;
                const int m0 = M[k1], m1 = M[k1 + 1], m2 = M[k1 + 2], m3 = M[k1 + 3], m4 = M[k1 + 4];
                int p0 = lerp(fr, m0, m1);
                if (bnd && x == 0) p0 = clip3(0, maxv, R[2 * n + 1] + ((R[2 * n - (y + 1)] - R[2 * n]) >> 1));
                put4(x, y, p0, lerp(fr, m1, m2), lerp(fr, m2, m3), lerp(fr, m3, m4));
            }
        } else {
            #pragma unroll 1
            for (int it = 0; it < (nq4 >> 6); it++) {  // n >= 16 here: nq4 a multiple of 64
            const int i = lane + 64 * it;
                const int x = (i & ((n >> 2) - 1)) * 4, y = i >> qsh;
                int p[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int pos = m24(x + q + 1, angle), k = n + y + (pos >> 5) + 1;
                    p[q] = lerp(pos & 31, M[k], M[k + 1]);
                    if (bnd && y == 0) p[q] = clip3(0, maxv, R[2 * n - 1] + ((R[2 * n + x + q + 1] - R[2 * n]) >> 1));
                }
                put4(x, y, p[0], p[1], p[2], p[3]);
            }
        }
    }
    wave_sync();
}

// A Cb TB and the Cr TB at the same place (n <= 8: at most 33 references) in one pass: both
// components share geometry, availability and the intra mode (chroma is never filtered, no
// boundary smoothing), so the substitution indices, the reference gathers and the prediction
// indices are computed once and applied to two register sets (lane k: Cb and Cr reference k).
template <int LN>  // TB size 1 << LN (2 or 3), compile-time
DEVI void hevc_predict_chroma_pair(const FU& u, const h2j_tu& tb, bool cbf_cr, uint64_t mask, int ox, int oy,
                                   int S, int16_t* bcb, int16_t* bcr, int top_cb, int left_cb, int top_cr, int left_cr,
                                   int lane) {
    constexpr int log2n = LN, n = 1 << log2n, nn = n * n;
    const int maxv = (1 << u.bdc) - 1;
    const bool cbf_cb = (tb.flags & H2J_TU_CBF) != 0;
    const int L = 4 * n + 1, nu = n;  // unit = 2 chroma samples
    const int k = lane;
    const int unit = k < 2 * n ? (k >> 1) : nu + ((k - 2 * n + 1) >> 1);
    const unsigned long long m = __ballot(k < L && ((mask >> unit) & 1ull));
    const bool any = m != 0;
    const int first = m ? __ffsll(static_cast<long long>(m)) - 1 : 0;
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const unsigned long long le = m & upto;
    const int j = le ? 63 - static_cast<int>(__clzll(le)) : first;
    const int xn = j > 2 * n ? ox + (j - 2 * n - 1) : ox - 1;
    const int yn = j < 2 * n ? oy + (2 * n - 1 - j) : oy - 1;
    const int in = m24(yn, S) + xn;
    const int icb = yn < 0 ? top_cb + xn + 1 : (xn < 0 ? left_cb + yn : in);
    const int icr = yn < 0 ? top_cr + xn + 1 : (xn < 0 ? left_cr + yn : in);
    const int half = 1 << (u.bdc - 1);
    const int rb = any ? bcb[icb] : half, rr = any ? bcr[icr] : half;
    const int mode = tb.mode;
    int dcb = 0, dcr = 0;
    if (mode == 1) {
        const bool dk = k >= n && k <= 3 * n && k != 2 * n;
        dcb = (wave_sum_dpp(dk ? rb : 0) + n) >> (log2n + 1);
        dcr = (wave_sum_dpp(dk ? rr : 0) + n) >> (log2n + 1);
    }
    const int i = lane, x = i & (n - 1), y = i >> log2n;
    int pb, pr;
    if (mode == 0) {
        const int trb = __builtin_amdgcn_readlane(rb, 3 * n + 1), blb = __builtin_amdgcn_readlane(rb, n - 1);
        const int trr = __builtin_amdgcn_readlane(rr, 3 * n + 1), blr = __builtin_amdgcn_readlane(rr, n - 1);
        const int il = 2 * n - 1 - y, ia = 2 * n + 1 + x;
        const int lb = __shfl(rb, il, 64), ab = __shfl(rb, ia, 64), lr = __shfl(rr, il, 64), ar = __shfl(rr, ia, 64);
        pb = (m24(n - 1 - x, lb) + m24(x + 1, trb) + m24(n - 1 - y, ab) + m24(y + 1, blb) + n) >> (log2n + 1);
        pr = (m24(n - 1 - x, lr) + m24(x + 1, trr) + m24(n - 1 - y, ar) + m24(y + 1, blr) + n) >> (log2n + 1);
    } else if (mode == 1) {
        pb = dcb;
        pr = dcr;
    } else {
        const HevcAng ang = hevc_ang(mode);
        const int angle = ang.angle, inv = ang.inv;
        const bool vert = mode >= 18;
        const int a = vert ? y : x, b = vert ? x : y;
        const int pos = m24(a + 1, angle), idx = pos >> 5, fr = pos & 31;
        const int k1 = b + idx + 1, k2 = k1 + 1;
        const int o1 = k1 >= 0 ? k1 : -((m24(k1, inv) + 128) >> 8);
        const int o2 = k2 >= 0 ? k2 : -((m24(k2, inv) + 128) >> 8);
        const int i1 = 2 * n + (vert ? o1 : -o1), i2 = 2 * n + (vert ? o2 : -o2);
        pb = (m24(32 - fr, __shfl(rb, i1, 64)) + m24(fr, __shfl(rb, i2, 64)) + 16) >> 5;
        pr = (m24(32 - fr, __shfl(rr, i1, 64)) + m24(fr, __shfl(rr, i2, 64)) + 16) >> 5;
    }
    if (i < nn) {
        int16_t* db = bcb + m24(oy + y, S) + ox + x;
        int16_t* dr = bcr + m24(oy + y, S) + ox + x;
        *db = static_cast<int16_t>(clip3(0, maxv, pb + (cbf_cb ? *db : 0)));
        *dr = static_cast<int16_t>(clip3(0, maxv, pr + (cbf_cr ? *dr : 0)));
    }
    wave_sync();
}

// The Cb and Cr 16x16 TBs at the same place in one pass (the chroma quadrant of a 64x64 CTB):
// availability, substitution indices and prediction indices computed once, the sample work done
// for both components.  Cb references in s.sub, Cr in s.ref (chroma is never filtered, no
// boundary smoothing), the angular modes' extended main references after them (from index 66).
DEVI void hevc_predict_chroma_pair16(const FU& u, const h2j_tu& tb, bool cbf_cr, uint64_t mask, int ox, int oy, int S,
                                     int16_t* bcb, int16_t* bcr, int top_cb, int left_cb, int top_cr, int left_cr,
                                     K1WaveLds& s, int lane) {
    constexpr int log2n = 4, n = 16, L = 4 * n + 1, nu = n, nh = n * n / 2;  // unit = 2 chroma samples
    const int maxv = (1 << u.bdc) - 1;
    const bool cbf_cb = (tb.flags & H2J_TU_CBF) != 0;
    unsigned long long m[2];
#pragma unroll
    for (int ch = 0; ch < 2; ch++) {
        const int k = lane + 64 * ch;
        const int unit = k < 2 * n ? (k >> 1) : nu + ((k - 2 * n + 1) >> 1);
        m[ch] = __ballot(k < L && ((mask >> unit) & 1ull));
    }
    const bool any = (m[0] | m[1]) != 0;
    const int first = m[0] ? __ffsll(static_cast<long long>(m[0])) - 1
                           : (m[1] ? 64 + __ffsll(static_cast<long long>(m[1])) - 1 : 128);
    const int fb[2] = {first, m[0] ? 63 - __clzll(m[0]) : first};
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int half = 1 << (u.bdc - 1);
    int dsb = 0, dsr = 0;
#pragma unroll
    for (int ch = 0; ch < 2; ch++) {
        const int k = lane + 64 * ch;
        const unsigned long long le = m[ch] & upto;
        const int j = le ? 64 * ch + 63 - static_cast<int>(__clzll(le)) : fb[ch];
        const int xn = j > 2 * n ? ox + (j - 2 * n - 1) : ox - 1;
        const int yn = j < 2 * n ? oy + (2 * n - 1 - j) : oy - 1;
        const int in = m24(yn, S) + xn;
        const int icb = yn < 0 ? top_cb + xn + 1 : (xn < 0 ? left_cb + yn : in);
        const int icr = yn < 0 ? top_cr + xn + 1 : (xn < 0 ? left_cr + yn : in);
        const int vb = any ? bcb[icb] : half, vr = any ? bcr[icr] : half;
        s.sub[k < L ? k : 131] = static_cast<int16_t>(vb);
        s.ref[k < L ? k : 131] = static_cast<int16_t>(vr);
        const bool dk = k >= n && k <= 3 * n && k != 2 * n;
        dsb += dk ? vb : 0;
        dsr += dk ? vr : 0;
    }
    const int mode = tb.mode;
    wave_sync();
    const int16_t* Rb = s.sub;
    const int16_t* Rr = s.ref;
    auto put2 = [&](int x, int y, int b0, int b1, int r0, int r1) __attribute__((always_inline)) {
        const int o = m24(oy + y, S) + ox + x;
        int* db = reinterpret_cast<int*>(bcb + o);
        int* dr = reinterpret_cast<int*>(bcr + o);
        int rb0 = 0, rb1 = 0, rr0 = 0, rr1 = 0;
        if (cbf_cb) { const int v = *db; rb0 = (v << 16) >> 16; rb1 = v >> 16; }
        if (cbf_cr) { const int v = *dr; rr0 = (v << 16) >> 16; rr1 = v >> 16; }
        *db = clip3(0, maxv, b0 + rb0) | (clip3(0, maxv, b1 + rb1) << 16);
        *dr = clip3(0, maxv, r0 + rr0) | (clip3(0, maxv, r1 + rr1) << 16);
    };
    if (mode == 0) {
        const int trb = Rb[3 * n + 1], blb = Rb[n - 1], trr = Rr[3 * n + 1], blr = Rr[n - 1];
        for (int it = 0; it < nh / 64; it++) {  // uniform trip count
            const int i = lane + 64 * it;
            const int x = (i & 7) * 2, y = i >> 3, wy = n - 1 - y;
            const int lb = Rb[2 * n - 1 - y], lr = Rr[2 * n - 1 - y];
            const int bb = m24(y + 1, blb) + n, br = m24(y + 1, blr) + n;
            const int a0b = m24(n - 1 - x, lb) + m24(x + 1, trb), a0r = m24(n - 1 - x, lr) + m24(x + 1, trr);
            put2(x, y, (a0b + m24(wy, Rb[2 * n + 1 + x]) + bb) >> (log2n + 1),
                 (a0b - lb + trb + m24(wy, Rb[2 * n + 2 + x]) + bb) >> (log2n + 1),
                 (a0r + m24(wy, Rr[2 * n + 1 + x]) + br) >> (log2n + 1),
                 (a0r - lr + trr + m24(wy, Rr[2 * n + 2 + x]) + br) >> (log2n + 1));
        }
    } else if (mode == 1) {
        const int dcb = (wave_sum_dpp(dsb) + n) >> (log2n + 1), dcr = (wave_sum_dpp(dsr) + n) >> (log2n + 1);
        for (int it = 0; it < nh / 64; it++) put2(((lane + 64 * it) & 7) * 2, (lane + 64 * it) >> 3, dcb, dcb, dcr, dcr);
    } else {
        const HevcAng ang = hevc_ang(mode);
        const int angle = ang.angle, inv = ang.inv;
        const bool vert = mode >= 18;
        const int sgn = vert ? 1 : -1;
        int16_t* Mb = s.sub + 66;  // M[n + k], k = -n .. 2n + 1 (as hevc_predict_tb)
        int16_t* Mr = s.ref + 66;
        if (lane < 3 * n + 2) {
            const int kk = lane - n;
            const int o = kk >= 0 ? kk : -((m24(kk, inv) + 128) >> 8);
            const int ix = clip3(0, 4 * n, 2 * n + sgn * o);
            Mb[lane] = Rb[ix];
            Mr[lane] = Rr[ix];
        }
        wave_sync();
        for (int it = 0; it < nh / 64; it++) {  // uniform trip count
            const int i = lane + 64 * it;
            const int x = (i & 7) * 2, y = i >> 3;
            if (vert) {
                const int pos = m24(y + 1, angle), fr = pos & 31, k1 = n + x + (pos >> 5) + 1;
                const int b0 = Mb[k1], b1 = Mb[k1 + 1], b2 = Mb[k1 + 2];
                const int r0 = Mr[k1], r1 = Mr[k1 + 1], r2 = Mr[k1 + 2];
                put2(x, y, (m24(32 - fr, b0) + m24(fr, b1) + 16) >> 5, (m24(32 - fr, b1) + m24(fr, b2) + 16) >> 5,
                     (m24(32 - fr, r0) + m24(fr, r1) + 16) >> 5, (m24(32 - fr, r1) + m24(fr, r2) + 16) >> 5);
            } else {
                const int pos0 = m24(x + 1, angle), pos1 = pos0 + angle;
                const int f0 = pos0 & 31, f1 = pos1 & 31;
                const int k0 = n + y + (pos0 >> 5) + 1, k1 = n + y + (pos1 >> 5) + 1;
                put2(x, y, (m24(32 - f0, Mb[k0]) + m24(f0, Mb[k0 + 1]) + 16) >> 5,
                     (m24(32 - f1, Mb[k1]) + m24(f1, Mb[k1 + 1]) + 16) >> 5,
                     (m24(32 - f0, Mr[k0]) + m24(f0, Mr[k0 + 1]) + 16) >> 5,
                     (m24(32 - f1, Mr[k1]) + m24(f1, Mr[k1 + 1]) + 16) >> 5);
            }
        }
    }
    wave_sync();
}

// K0 residual of one quadrant -> a quadrant window in LDS by LDS-DMA (no registers held while
// it is in flight).  The residual planes are tiled by quadrant (h2j_res_q): the quadrant is one
// contiguous tile, copied in 16-B pieces (luma: Qc x Qc row-major; chroma: Cb at element 0 and
// Cr at 256, Qc x Qc each).  Tiles past the picture's right / bottom edge exist in full, so no
// lane needs a bounds test; their samples outside the picture are never written by K0 (stale
// arena bytes) and never read by reconstruction: every TB lies inside the coded picture, because
// the parser rejects widths / heights that are not a multiple of MinCbSize (hevc_parser.cpp,
// vector m_hevc_width_not_mincb) and the coding quadtree splits implicitly at the picture edge
// (7.3.8.4), so every CB -- and with it every TB -- ends inside the picture.
DEVI void hevc_qres_dma(const FU& u, int grp, int X0, int Y0, int Qc, int16_t* body, int lane) {
    const int chunks = (Qc * Qc) >> 3;  // 16-B pieces of one plane's tile
    if (grp == 0) {
        const int16_t* R = hevc_res_at(u.res, u.width, u.height, u.log2ctb, 0, X0, Y0);
#pragma unroll
        for (int j = 0; j < 2; j++) {
            if (64 * j < chunks && lane + 64 * j < chunks) lds_dma16(R + (lane + 64 * j) * 8, lds_addr(body + 512 * j));
        }
    } else {
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const int16_t* R = hevc_res_at(u.res, u.width, u.height, u.log2ctb, 1 + c, X0, Y0);
            if (lane < chunks) lds_dma16(R + lane * 8, lds_addr(body + 256 * c));
        }
    }
}

// One CTB row `row` of one component group (grp 0: luma; grp 1: Cb and Cr) of a picture, by one
// wave: CTBs left to right, each in z-order quadrants (skipping quadrants outside the picture).
// `above` / `mine`: the progress words of the row above / this row ((row + 1) << 16 | quadrants
// done, quadrant granularity); `line`: the group's bottom-line buffer (row r writes the line
// row r + 1 reads).
template <typename Pel>
DEVI void hevc_row(const FU& u, const h2j_tu* T, const uint64_t* masks, const uint32_t* rng, int grp, QWave& w,
                   const uint32_t* above, uint32_t* mine, int16_t* line, const int row, Pel* stg) {
    const int lane = threadIdx.x & 63;
    const int shc = grp ? 1 : 0;                 // component subsampling of this group
    const int CS = 1 << u.log2ctb;               // luma CTB size
    const int Sc = CS >> shc;                    // CTB size in this group's components
    const int Q = CS == 64 ? 32 : CS;            // luma quadrant size
    const int Qc = Q >> shc;
    const int nqs = CS / Q;                      // quadrants per side (2 or 1)
    const int nq = nqs * nqs;                    // quadrants per CTB (units of the row progress words)
    const int Wc = u.width >> shc, Hc = u.height >> shc;
    const int ncomp = grp ? 2 : 1;
    PROF_DECL;
    auto q_inside = [&](int cx, int q) __attribute__((always_inline)) {
        return cx * Sc + (q & 1) * Qc < Wc && row * Sc + (q >> 1) * Qc < Hc;
    };
    auto q_next = [&](int& cx, int& q) __attribute__((always_inline)) {  // next quadrant of the row inside the picture
        do {
            if (++q == nq) {
                q = 0;
                ++cx;
            }
        } while (cx < u.ctb_w && !q_inside(cx, q));
    };
    int cur = 0;  // quadrant window in use (the other one is being filled for the next quadrant)
    hevc_qres_dma(u, grp, 0, row * Sc, Qc, w.body[0], lane);
    lds_dma_wait();
    // this group's record range of a CTB: luma [first, first chroma), chroma [first chroma, end)
    auto grange = [&](int cbi, uint32_t& ra, uint32_t& rb) __attribute__((always_inline)) {
        const uint4 r = reinterpret_cast<const uint4*>(rng)[cbi];
        const uint32_t mid = (r.y > r.x && r.y <= r.z) ? r.y : r.z;
        ra = grp ? mid : r.x;
        rb = grp ? r.z : mid;
    };
    uint32_t na, nb;
    grange(row * u.ctb_w, na, nb);
    {
        uint32_t seen = 0;
        const bool below = row + 1 < u.ctb_h;
        for (int cx = 0; cx < u.ctb_w; cx++) {
            const int CX0 = cx * Sc, CY0 = row * Sc;
            const int pin = cx & 1, pprev = pin ^ 1;   // prevR slot written by this CTB / read from the previous
            // this CTB's record range + first batch (prefetched); prefetch the next CTB's
            const uint32_t a = na, b = nb;
            uint32_t t = a, tb = a;
            // (r06: the first record batch is loaded here, not prefetched a CTB ahead: six VGPRs held
            // across the whole CTB had the pool kernel spill 25 VGPRs, 8 without them)
            uint4 rec = reinterpret_cast<const uint4*>(T)[min(a + lane, max(b, 1u) - 1)];
            uint2 msk = reinterpret_cast<const uint2*>(masks)[min(a + lane, max(b, 1u) - 1)];
            if (cx + 1 < u.ctb_w) grange(row * u.ctb_w + cx + 1, na, nb);
            for (int q = 0; q < nq; q++) {
                if (!q_inside(cx, q)) continue;
                const int qx = q & 1, qy = q >> 1;
                const int X0 = CX0 + qx * Qc, Y0 = CY0 + qy * Qc;
                {  // prefetch the row's next quadrant's residual into the other window (its last
                   // reader, the previous quadrant's store, has finished reading it)
                    int nc = cx, nqi = q;
                    q_next(nc, nqi);
                    lds_reads_done();
                    if (nc < u.ctb_w)
                        hevc_qres_dma(u, grp, nc * Sc + (nqi & 1) * Qc, row * Sc + (nqi >> 1) * Qc, Qc, w.body[cur ^ 1], lane);
                }
                // top quadrants need the row above (progress counts its quadrants, nq per CTB):
                // the left one up to this CTB, the right one also the next CTB's bottom-left
                // quadrant (whose top line is the right one's above-right reference)
                if (row > 0 && qy == 0) {
                    int cnt = nq * (cx + 1);
                    if (qx == nqs - 1 && cx + 1 < u.ctb_w) cnt += nqs == 2 ? 3 : 1;
                    const uint32_t need = (static_cast<uint32_t>(row) << 16) | static_cast<uint32_t>(cnt);
                    if (seen < need) seen = wait_progress(above, need, u.derr, kDevErrK1Row);
                }
                PROF_LAP(0);
                // neighbour arrays of the quadrant: one pass, lane = x of the line above and y of
                // the column on the left, lane 0 also the top-left corner; sources picked by
                // uniform element offsets from the start of the group's LDS, one unconditional
                // load each, all loads of both components issued before the first write
                {
                    int16_t* base = reinterpret_cast<int16_t*>(&w);
                    int16_t tv[2], lv[2], cv[2];
                    bool ta[2], la[2], cz[2];
#pragma unroll
                    for (int ci = 0; ci < 2; ci++) {
                        if (ci >= ncomp) break;
                        QComp& C = w.cs[ci];
                        const int o_line = static_cast<int>(line + ci * (Wc + 64) - base);
                        const int o_qbot = static_cast<int>(C.qbot - base);
                        const int o_prev = static_cast<int>(C.prevR[pprev] - base);
                        const int o_qr = static_cast<int>(C.qright - base);
                        const int o_cor = static_cast<int>(&C.corner - base);
                        const int x = lane, y = lane;
                        int to, lo, co;
                        if (qy == 0) { ta[ci] = row > 0 && X0 + x < Wc; to = o_line + X0 + x; }
                        else { ta[ci] = qx * Qc + x < 2 * Qc; to = o_qbot + qx * Qc + x; }
                        if (qx == 0) { la[ci] = cx > 0 && qy * Qc + y < Sc; lo = o_prev + qy * Qc + y; }
                        else { la[ci] = y < Qc; lo = o_qr + y; }
                        if (qy == 0) { cz[ci] = !(row > 0 && X0 > 0); co = qx == 0 ? o_cor : o_line + X0 - 1; }
                        else { cz[ci] = qx == 0 && cx == 0; co = qx == 0 ? o_prev + Qc - 1 : o_qbot + Qc - 1; }
                        tv[ci] = base[ta[ci] ? to : o_qbot];
                        lv[ci] = base[la[ci] ? lo : o_qbot];
                        cv[ci] = base[cz[ci] ? o_qbot : co];
                    }
#pragma unroll
                    for (int ci = 0; ci < 2; ci++) {
                        if (ci >= ncomp) break;
                        QComp& C = w.cs[ci];
                        if (lane < 2 * Qc) {
                            C.top[lane + 1] = ta[ci] ? tv[ci] : int16_t(0);
                            C.left[lane] = la[ci] ? lv[ci] : int16_t(0);
                        }
                        if (lane == 0) C.top[0] = cz[ci] ? int16_t(0) : cv[ci];
                    }
                }
                wave_sync();
                PROF_LAP(1);
                // this group's TBs of quadrant q (records are in z-scan order)
                while (t < b) {
                    if (t - tb >= 64) {  // next 64-record batch
                        tb = t;
                        rec = reinterpret_cast<const uint4*>(T)[min(t + lane, b - 1)];
                        msk = reinterpret_cast<const uint2*>(masks)[min(t + lane, b - 1)];
                    }
                    const int l = static_cast<int>(t - tb);
                    const h2j_tu tu = tu_from_lanes(rec, l);
                    const int c = tu.c;
                    const int ox = tu.x - X0, oy = tu.y - Y0;
                    if (ox >= Qc || oy >= Qc) break;  // first TB of a later quadrant
                    const int ci = c == 2 ? 1 : 0;
                    int16_t* body = w.body[cur] + ci * 256;
                    // element offsets of the carried top / left arrays of component ci from the
                    // window of component cj, from the layout (scalar; pointer differences of the
                    // generic LDS pointers cost a shared-aperture conversion each)
                    auto nbo = [&](int cj, int ci2, bool left) __attribute__((always_inline)) {
                        return static_cast<int>((offsetof(QWave, cs) + static_cast<size_t>(ci2) * sizeof(QComp) +
                                                 (left ? offsetof(QComp, left) : offsetof(QComp, top)) -
                                                 offsetof(QWave, body) - static_cast<size_t>(cur) * sizeof(w.body[0]) -
                                                 static_cast<size_t>(cj) * 512) / 2);
                    };
                    if (c == 1 && tu.log2n <= 4 && l + 1 < 64 && t + 1 < b && !(tu.flags & H2J_TU_PCM)) {
                        // Cb TB followed by the Cr TB at the same place: one pass for both
                        const h2j_tu tr = tu_from_lanes(rec, l + 1);
                        if (tr.c == 2 && tr.x == tu.x && tr.y == tu.y && tr.log2n == tu.log2n && !(tr.flags & H2J_TU_PCM)) {
                            if (tu.log2n == 4)
                                hevc_predict_chroma_pair16(u, tu, (tr.flags & H2J_TU_CBF) != 0, mask_from_lanes(msk, l), ox, oy, Qc,
                                                           body, w.body[cur] + 256, nbo(0, 0, false), nbo(0, 0, true),
                                                           nbo(1, 1, false), nbo(1, 1, true), w.k, lane);
                            else if (tu.log2n == 2)
                                hevc_predict_chroma_pair<2>(u, tu, (tr.flags & H2J_TU_CBF) != 0, mask_from_lanes(msk, l), ox, oy, Qc,
                                                            body, w.body[cur] + 256, nbo(0, 0, false), nbo(0, 0, true),
                                                            nbo(1, 1, false), nbo(1, 1, true), lane);
                            else
                                hevc_predict_chroma_pair<3>(u, tu, (tr.flags & H2J_TU_CBF) != 0, mask_from_lanes(msk, l), ox, oy, Qc,
                                                            body, w.body[cur] + 256, nbo(0, 0, false), nbo(0, 0, true),
                                                            nbo(1, 1, false), nbo(1, 1, true), lane);
                            PROF_ADD(5, 2);
                            PROF_LAPK(tu.log2n - 2 + 4);
                            t += 2;
                            continue;
                        }
                    }
                    if (tu.flags & H2J_TU_PCM) {  // samples written by K0: pull that block into the window
                        const int n = 1 << tu.log2n;
                        const Pel* P = u.plane<Pel>(c);
                        for (int i = lane; i < n * n; i += 64)
                            body[(oy + i / n) * Qc + ox + (i % n)] =
                                static_cast<int16_t>(P[(tu.y + i / n) * u.st(c) + tu.x + (i % n)]);
                        wave_sync();
                    } else {
                        if (tu.log2n == 2)
                            hevc_predict_tb<2>(u, tu, mask_from_lanes(msk, l), ox, oy, Qc, body, nbo(ci, ci, false), nbo(ci, ci, true), w.k, lane);
                        else if (tu.log2n == 3)
                            hevc_predict_tb<3>(u, tu, mask_from_lanes(msk, l), ox, oy, Qc, body, nbo(ci, ci, false), nbo(ci, ci, true), w.k, lane);
                        else if (tu.log2n == 4)
                            hevc_predict_tb<4>(u, tu, mask_from_lanes(msk, l), ox, oy, Qc, body, nbo(ci, ci, false), nbo(ci, ci, true), w.k, lane);
                        else  // 32x32 (TB sizes are 4..32)
                            hevc_predict_tb<5>(u, tu, mask_from_lanes(msk, l), ox, oy, Qc, body, nbo(ci, ci, false), nbo(ci, ci, true), w.k, lane);
                    }
                    PROF_ADD(5, 1);
                    PROF_LAPK(tu.log2n - 2 + (c ? 4 : 0));
                    t++;
                }
                // store the quadrant and update the carries; the next quadrant's window has
                // landed by now (issued a whole quadrant ago), retire it before the stores
                lds_dma_wait();
                const int wq = min(Qc, Wc - X0), hq = min(Qc, Hc - Y0);
                const int lq = __builtin_ctz(static_cast<unsigned>(Qc)) - 2;  // log2 of 4-sample steps per row
                // quadrant pairs (TL | TR, BL | BR) leave as whole CTB-wide rows (64 B of 8-bit luma
                // instead of two 32-B halves, 32 B of chroma instead of 16): a left quadrant whose
                // right neighbour lies inside the picture is parked in `stg` (the wave's staging
                // tile, samples packed as Pel) and stored with it
                const bool pair = stg != nullptr && nqs == 2;
                const bool park = pair && qx == 0 && X0 + Qc < Wc;
                const bool joined = pair && qx == 1;
                for (int ci = 0; ci < ncomp; ci++) {
                    const int c = grp ? ci + 1 : 0;
                    QComp& C = w.cs[ci];
                    const int16_t* body = w.body[cur] + ci * 256;
                    Pel* P = u.plane<Pel>(c);
                    const int st = u.st(c);
                    auto pack4 = [&](const int16_t* src) __attribute__((always_inline)) {
                        const uint2 v = *reinterpret_cast<const uint2*>(src);
                        return sizeof(Pel) == 1 ? make_uint2((v.x & 0xFF) | ((v.x >> 8) & 0xFF00) | ((v.y & 0xFF) << 16) | ((v.y >> 16) << 24), 0u)
                                                : v;
                    };
                    auto put4 = [&](Pel* d, uint2 v) __attribute__((always_inline)) {
                        if (sizeof(Pel) == 1) *reinterpret_cast<uint32_t*>(d) = v.x;
                        else *reinterpret_cast<uint2*>(d) = v;
                    };
                    // quadrants 16 or 32 samples wide and whole inside the picture: one 16-byte
                    // store per lane step -- 16 samples at 8 bits (four window dwords packed by
                    // v_perm), 8 at 16 bits -- instead of 4 samples
                    constexpr int SC = 16 / static_cast<int>(sizeof(Pel));  // samples per 16-byte chunk
                    const bool wide = Qc >= 16 && wq == Qc && ((st | u.off(c)) & (SC - 1)) == 0;
                    auto pack16 = [&](const int16_t* src) __attribute__((always_inline)) {
                        const uint2* q = reinterpret_cast<const uint2*>(src);
                        if (sizeof(Pel) == 2) {
                            const uint2 a = q[0], b = q[1];
                            return make_uint4(a.x, a.y, b.x, b.y);
                        }
                        const uint2 a = q[0], b = q[1], c2 = q[2], d = q[3];
                        return make_uint4(__builtin_amdgcn_perm(a.y, a.x, 0x06040200u), __builtin_amdgcn_perm(b.y, b.x, 0x06040200u),
                                          __builtin_amdgcn_perm(c2.y, c2.x, 0x06040200u), __builtin_amdgcn_perm(d.y, d.x, 0x06040200u));
                    };
                    const int lc = __builtin_ctz(static_cast<unsigned>(Qc / SC));  // log2 of chunks per quadrant row
                    if (wide && park) {
                        Pel* sg = stg + ci * 256;
                        for (int i = lane; i < (hq << lc); i += 64) {
                            const int y = i >> lc, x = (i & ((1 << lc) - 1)) * SC;
                            *reinterpret_cast<uint4*>(sg + y * Qc + x) = pack16(body + y * Qc + x);
                        }
                    } else if (wide && joined) {
                        const Pel* sg = stg + ci * 256;
                        Pel* D = P + (Y0 * st + X0 - Qc);
                        for (int i = lane; i < (hq << (lc + 1)); i += 64) {
                            const int y = i >> (lc + 1), x = (i & ((2 << lc) - 1)) * SC;
                            const uint4 v = x < Qc ? *reinterpret_cast<const uint4*>(sg + y * Qc + x) : pack16(body + y * Qc + x - Qc);
                            *reinterpret_cast<uint4*>(D + y * st + x) = v;
                        }
                    } else if (wide) {
                        Pel* D = P + (Y0 * st + X0);
                        for (int i = lane; i < (hq << lc); i += 64) {
                            const int y = i >> lc, x = (i & ((1 << lc) - 1)) * SC;
                            *reinterpret_cast<uint4*>(D + y * st + x) = pack16(body + y * Qc + x);
                        }
                    } else if (park) {  // Qc x hq samples into the staging tile (rows of Qc, Cb at 0, Cr at 256)
                        Pel* sg = stg + ci * 256;
                        for (int i = lane; i < (hq << lq); i += 64) {
                            const int y = i >> lq, x = (i & ((1 << lq) - 1)) * 4;
                            put4(sg + (y << (lq + 2)) + x, pack4(body + (y << (lq + 2)) + x));
                        }
                    } else if (joined) {  // rows of 2Qc: the parked left quadrant, then this one
                        const Pel* sg = stg + ci * 256;
                        const int l2 = lq + 1;  // log2 of 4-sample steps per joined row
                        for (int i = lane; i < (hq << l2); i += 64) {
                            const int y = i >> l2, x = (i & ((1 << l2) - 1)) * 4;
                            if (x >= Qc + wq) continue;
                            uint2 v;
                            if (x < Qc) {
                                const Pel* q = sg + (y << (lq + 2)) + x;
                                v = sizeof(Pel) == 1 ? make_uint2(*reinterpret_cast<const uint32_t*>(q), 0u)
                                                     : *reinterpret_cast<const uint2*>(q);
                            } else {
                                v = pack4(body + (y << (lq + 2)) + x - Qc);
                            }
                            put4(P + (Y0 + y) * st + X0 - Qc + x, v);
                        }
                    } else {
                        // 4 samples per lane step (component widths are multiples of 4); rows of
                        // the window beyond the picture's right edge masked
                        for (int i = lane; i < (hq << lq); i += 64) {
                            const int y = i >> lq, x = (i & ((1 << lq) - 1)) * 4;
                            if (x >= wq) continue;
                            put4(P + (Y0 + y) * st + X0 + x, pack4(body + (y << (lq + 2)) + x));
                        }
                    }
                    // carries: the bottom row (line for the CTB row below, qbot for the bottom
                    // quadrants) and the right column (qright for the right quadrant, prevR for
                    // the next CTB), each read once
                    const int k = lane & (Qc - 1);
                    const int16_t bv = body[(Qc - 1) * Qc + k];
                    const int16_t rv = body[k * Qc + Qc - 1];
                    const int16_t tq = C.top[Qc];
                    if (lane < Qc) {
                        if (qy == nqs - 1 && below && lane < wq) line[ci * (Wc + 64) + X0 + lane] = bv;
                        if (qy == 0 && nqs == 2) C.qbot[qx * Qc + lane] = bv;
                        if (qx == 0 && nqs == 2) C.qright[lane] = rv;
                        if (qx == nqs - 1) C.prevR[pin][qy * Qc + lane] = rv;
                    }
                    if (qx == nqs - 1 && qy == 0 && lane == 0) C.corner = tq;
                }
                wave_sync();
                cur ^= 1;
                PROF_LAP(3);
                if (nqs == 2 && q == 2 && below) {  // bottom-left quadrant: its bottom line is in `line`
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0)
                        __hip_atomic_store(mine, ((static_cast<uint32_t>(row) + 1) << 16) | static_cast<uint32_t>(nq * cx + 3),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            PROF_ADD(6, 1);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0)
                __hip_atomic_store(mine, ((static_cast<uint32_t>(row) + 1) << 16) | static_cast<uint32_t>(nq * (cx + 1)),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    PROF_FLUSH();
}

// Static row assignment (the <= 128-picture "wide" launches and the mixed-batch kernel): wave wv
// of a W_-wave group walks rows wv, wv + W_, ...; progress words in 2 * W_ row-tagged slots.
template <typename Pel>
DEVI void hevc_rows(const h2j_frame& f, const h2j_tu* T, uint8_t* arena, int grp, QWave* W, uint32_t* prog,
                    int16_t* line, int wv, const int W_) {
    const FU u = make_fu(f, arena);
    const uint64_t* masks = reinterpret_cast<const uint64_t*>(arena + ufl64(f.aux));
    const uint32_t* rng = reinterpret_cast<const uint32_t*>(arena + ufl64(f.ctbrng));
    const int kSlots = 2 * W_;
    for (int row = wv; row < u.ctb_h; row += W_)
        hevc_row<Pel>(u, T, masks, rng, grp, W[wv], prog + (row + kSlots - 1) % kSlots, prog + row % kSlots, line, row,
                      static_cast<Pel*>(nullptr));
}


// Separate kernels per codec so each gets its own register budget; a mixed
// batch launches both and each skips the other codec's pictures.
// grid (pictures, 2): blockIdx.y = 0 luma chain, 1 chroma chains.
template <typename Pel, int W_>
__global__ void __launch_bounds__(64 * W_, 4) h2j_k1_recon_hevc(const h2j_frame* frames, const h2j_tu* tus,
                                                            uint8_t* arena) {
    extern __shared__ __align__(16) uint8_t k1lds[];
    QWave* W = reinterpret_cast<QWave*>(k1lds);
    uint32_t* prog = reinterpret_cast<uint32_t*>(k1lds + sizeof(QWave) * W_);
    int16_t* line = reinterpret_cast<int16_t*>(k1lds + k1_fixed_lds(W_));
    const h2j_frame& f = frames[blockIdx.x];
    if (f.codec != H2J_CODEC_HEVC || (f.bit_depth > 8) != (sizeof(Pel) == 2)) return;
    if (threadIdx.x < 2 * W_) prog[threadIdx.x] = 0;
    __syncthreads();
    hevc_rows<Pel>(f, tus + ufl(f.tu), arena, static_cast<int>(blockIdx.y), W, prog, line,
                       static_cast<int>(threadIdx.x >> 6), W_);
}

// grid = h2j_gpu_batch.k1wgs8: workgroup -> (picture, band of kAvcK1Waves rows) from the host's
// map (band-major, so a band only ever waits on an earlier workgroup)
__global__ void __launch_bounds__(64 * kAvcK1Waves, 4) h2j_k1_recon_h264(const h2j_frame* frames, const h2j_tu* tus,
                                                                    const h2j_ctb* ctbs, uint8_t* arena, const uint32_t* map) {
    extern __shared__ __align__(16) uint8_t h4lds[];
    H4WaveLds* wl = reinterpret_cast<H4WaveLds*>(h4lds);
    uint32_t* prog = reinterpret_cast<uint32_t*>(h4lds + sizeof(H4WaveLds) * kAvcK1Waves);
    uint16_t* line = reinterpret_cast<uint16_t*>(h4lds + sizeof(H4WaveLds) * kAvcK1Waves + 2 * kAvcK1Waves * 4);
    const uint32_t me = map[blockIdx.x];
    const h2j_frame& f = frames[me >> 8];
    const int band = static_cast<int>(me & 0xFF);
    if (f.codec != H2J_CODEC_H264) return;
    const int nbands = ufl(f.k1bands) > 1 ? (static_cast<int>(ufl(f.ctb_h)) + kAvcK1Waves - 1) / kAvcK1Waves : 1;
    if (threadIdx.x < 2 * kAvcK1Waves) prog[threadIdx.x] = 0;
    __syncthreads();
    H4WaveLds& s = wl[threadIdx.x >> 6];
    const h2j_tu* T = tus + ufl(f.tu);
    if (ufl(f.mbaff)) return;  // h2j_k1_recon_h264_mbaff
    if (f.bit_depth == 8) h264_rows<uint8_t, kAvcK1Waves>(f, T, arena, s, prog, line, band, nbands);
    else h264_rows<uint16_t, kAvcK1Waves>(f, T, arena, s, prog, line, band, nbands);
}

// MBAFF frames (h2j_frame.mbaff) in a kernel of their own, so the progressive kernel keeps its
// register allocation; same (picture, band) map, other pictures return at once.
__global__ void __launch_bounds__(64 * kAvcWaves) h2j_k1_recon_h264_mbaff(const h2j_frame* frames, const h2j_tu* tus,
                                                                        const h2j_ctb* ctbs, uint8_t* arena,
                                                                        const uint32_t* map) {
    extern __shared__ __align__(16) uint8_t h4lds[];
    H4WaveLds* wl = reinterpret_cast<H4WaveLds*>(h4lds);
    uint32_t* prog = reinterpret_cast<uint32_t*>(h4lds + sizeof(H4WaveLds) * kAvcWaves);
    const h2j_frame& f = frames[map[blockIdx.x] >> 8];
    if (f.codec != H2J_CODEC_H264 || !ufl(f.mbaff)) return;
    if (threadIdx.x < 2 * kAvcWaves) prog[threadIdx.x] = 0;
    __syncthreads();
    H4WaveLds& s = wl[threadIdx.x >> 6];
    const h2j_tu* T = tus + ufl(f.tu);
    if (f.bit_depth == 8) h264_rows_mbaff<uint8_t>(f, T, ctbs + ufl(f.ctb), arena, s, prog);
    else h264_rows_mbaff<uint16_t>(f, T, ctbs + ufl(f.ctb), arena, s, prog);
}

// K1 HEVC, picture pool: one 16-wave workgroup reconstructs P pictures.  Its waves take CTB-row
// jobs from one LDS queue ordered row by row and, inside a row index, the pictures' luma rows
// before their chroma rows (row 0: P0 luma, P1 luma, ..., P0 chroma, ...): a wave that finishes a row takes the
// next row of either component group and either picture.  Rows of one (picture, group) chain
// through progress words as in hevc_rows; a job only ever waits on an earlier job, which some
// wave is running or has finished, so the queue cannot deadlock.  Against one picture per
// workgroup with a fixed 9 luma / 7 chroma split (r01) no wave idles through a
// second row round, and one picture's wavefront start-up overlaps the other's tail.
// LDS: QWave[16] | progress words [P][2][maxrows] | queue word (+3 pad) | lines [P][lstride]
// (luma bottom line at 0, Cb / Cr lines at lchroma).
constexpr int kPoolWaves = 16;
__host__ __device__ constexpr size_t k1_pool_lds(int P, int maxrows, int lstride) {
    return sizeof(QWave) * kPoolWaves + (static_cast<size_t>(P) * 2 * maxrows + 4) * 4 +
           static_cast<size_t>(P) * lstride * 2;
}
// + per wave a staging tile of 32 x 32 samples (quadrant pairs stored as whole CTB-wide rows)
__host__ __device__ constexpr size_t k1_pool_stage_lds(int pel_bytes) {
    return static_cast<size_t>(kPoolWaves) * 32 * 32 * pel_bytes;
}
// The pool's job loop over pictures fi0 .. fi0 + P - 1 (those below `nframes`) in `lds` (see
// k1_pool_lds); every thread of the 16-wave workgroup calls it.
// `staged`: the LDS also holds the staging tiles (k1_pool_stage_lds, after k1_pool_lds rounded to 16 B).
template <typename Pel>
DEVI void hevc_pool_jobs(const h2j_frame* frames, const h2j_tu* tus, uint8_t* arena, int fi0, int nframes, int P,
                         int maxrows, int lstride, int lchroma, uint8_t* lds, bool staged) {
    QWave* W = reinterpret_cast<QWave*>(lds);
    uint32_t* prog = reinterpret_cast<uint32_t*>(lds + sizeof(QWave) * kPoolWaves);
    const int nprog = P * 2 * maxrows;
    uint32_t* queue = prog + nprog;
    int16_t* lines = reinterpret_cast<int16_t*>(queue + 4);
    for (int i = static_cast<int>(threadIdx.x); i < nprog + 4; i += 64 * kPoolWaves) prog[i] = 0;
    __syncthreads();
    const int lane = static_cast<int>(threadIdx.x & 63), wv = static_cast<int>(threadIdx.x >> 6);
    const uint32_t njobs = static_cast<uint32_t>(nprog);
    Pel* stg = staged ? reinterpret_cast<Pel*>(lds + ((k1_pool_lds(P, maxrows, lstride) + 15) & ~size_t(15))) + wv * 1024
                      : static_cast<Pel*>(nullptr);
    for (;;) {
        uint32_t j = 0;
        if (lane == 0) j = __hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        j = ufl(static_cast<uint32_t>(__shfl(static_cast<int>(j), 0, 64)));
        if (j >= njobs) break;
        // a row index's luma rows of the P pictures, then their chroma rows (the longer luma
        // chains start first; same-box 9.28 -> 9.18 ms per 1024 hevc1080 pictures against
        // luma / chroma alternating per picture)
        const int row = static_cast<int>(j) / (2 * P), rem = static_cast<int>(j) - row * 2 * P;
        const int grp = rem >= P ? 1 : 0, p = rem - grp * P;
        const int fi = fi0 + p;
        if (fi >= nframes) continue;
        const h2j_frame& f = frames[fi];
        if (ufl(f.codec) != H2J_CODEC_HEVC || (ufl(f.bit_depth) > 8) != (sizeof(Pel) == 2)) continue;
        const FU u = make_fu(f, arena);
        if (row >= u.ctb_h) continue;
        const h2j_tu* T = tus + ufl(f.tu);
        const uint64_t* masks = reinterpret_cast<const uint64_t*>(arena + ufl64(f.aux));
        const uint32_t* rng = reinterpret_cast<const uint32_t*>(arena + ufl64(f.ctbrng));
        uint32_t* pr = prog + (p * 2 + grp) * maxrows;
        int16_t* line = lines + p * lstride + (grp ? lchroma : 0);
        if (grp == 0) hevc_row<Pel>(u, T, masks, rng, 0, W[wv], pr + (row ? row - 1 : 0), pr + row, line, row, stg);
        else hevc_row<Pel>(u, T, masks, rng, 1, W[wv], pr + (row ? row - 1 : 0), pr + row, line, row, stg);
    }
}
template <typename Pel>
__global__ void __launch_bounds__(64 * kPoolWaves) h2j_k1_recon_hevc_pool(const h2j_frame* frames, const h2j_tu* tus,
                                                                        uint8_t* arena, int nframes, int P, int maxrows,
                                                                        int lstride, int lchroma, int staged) {
    extern __shared__ __align__(16) uint8_t k1lds[];
    hevc_pool_jobs<Pel>(frames, tus, arena, static_cast<int>(blockIdx.x) * P, nframes, P, maxrows, lstride, lchroma, k1lds,
                        staged != 0);
}

// K1 for batches mixing HEVC 8-bit, HEVC high bit depth and H.264 pictures (configs[4]): one
// launch instead of three back-to-back ones, so the pictures' chains run side by side (each
// launch alone is one long chain per picture and leaves most of the GPU idle).  Workgroups of
// 16 waves: an HEVC picture's luma group (waves 0-7) and chroma group (waves 8-15) share one
// workgroup; an H.264 workgroup is one band as in h2j_k1_recon_h264.  Tall HEVC pictures (the
// longest chains of such a batch) instead get one 16-wave workgroup per component group, twice
// the rows in flight.  `map`: the host's list, longest chains first; bit 31 marks HEVC entries,
// bit 30 a 16-wave group (bit 0: 0 luma, 1 chroma).
__global__ void __launch_bounds__(64 * kAvcWaves) h2j_k1_recon_any(const h2j_frame* frames, const h2j_tu* tus,
                                                                 const h2j_ctb* ctbs, uint8_t* arena, const uint32_t* map) {
    extern __shared__ __align__(16) uint8_t anylds[];
    const uint32_t me = map[blockIdx.x];
    const h2j_frame& f = frames[(me >> 8) & 0x3FFFFFu];
    const h2j_tu* T = tus + ufl(f.tu);
    if ((me & 0xC0000000u) == 0xC0000000u) {  // one 16-wave HEVC group
        const int grp = static_cast<int>(me & 1);
        QWave* W = reinterpret_cast<QWave*>(anylds);
        uint32_t* prog = reinterpret_cast<uint32_t*>(anylds + sizeof(QWave) * kK1WavesWide);
        int16_t* line = reinterpret_cast<int16_t*>(anylds + k1_fixed_lds(kK1WavesWide));
        if (threadIdx.x < 2 * kK1WavesWide) prog[threadIdx.x] = 0;
        __syncthreads();
        const int wv = static_cast<int>(threadIdx.x >> 6);
        if (ufl(f.bit_depth) == 8 && ufl(f.bit_depth_c) == 8) hevc_rows<uint8_t>(f, T, arena, grp, W, prog, line, wv, kK1WavesWide);
        else hevc_rows<uint16_t>(f, T, arena, grp, W, prog, line, wv, kK1WavesWide);
    } else if (me & 0x80000000u) {  // one HEVC picture: the pool's job loop over its rows (P = 1)
        const int fi = static_cast<int>((me >> 8) & 0x3FFFFFu);
        const int w = static_cast<int>(ufl(f.width)), rows = static_cast<int>(ufl(f.ctb_h));
        if (ufl(f.bit_depth) == 8 && ufl(f.bit_depth_c) == 8)
            hevc_pool_jobs<uint8_t>(frames, tus, arena, fi, fi + 1, 1, rows, 2 * w + 192, w + 64, anylds, false);
        else
            hevc_pool_jobs<uint16_t>(frames, tus, arena, fi, fi + 1, 1, rows, 2 * w + 192, w + 64, anylds, false);
    } else {
        H4WaveLds* wl = reinterpret_cast<H4WaveLds*>(anylds);
        uint32_t* prog = reinterpret_cast<uint32_t*>(anylds + sizeof(H4WaveLds) * kAvcWaves);
        uint16_t* line = reinterpret_cast<uint16_t*>(anylds + sizeof(H4WaveLds) * kAvcWaves + 2 * kAvcWaves * 4);
        const int band = static_cast<int>(me & 0xFF);
        const int nbands = ufl(f.k1bands);
            if (threadIdx.x < 2 * kAvcWaves) prog[threadIdx.x] = 0;
            __syncthreads();
        H4WaveLds& s = wl[threadIdx.x >> 6];
        if (ufl(f.mbaff)) return;  // h2j_k1_recon_h264_mbaff
        if (f.bit_depth == 8) h264_rows<uint8_t, kAvcWaves>(f, T, arena, s, prog, line, band, nbands);
        else h264_rows<uint16_t, kAvcWaves>(f, T, arena, s, prog, line, band, nbands);
    }
}

// ---------------------------------------------------------------- K2: deblocking
__constant__ uint8_t kBeta[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                  34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
__constant__ uint8_t kTc[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,  1,  1,  1,  1,  1, 1,
                                2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

__constant__ int kChromaQp265[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
DEVI int chroma_qp_tab(int qpi) { return qpi < 30 ? qpi : (qpi > 43 ? qpi - 6 : kChromaQp265[qpi - 30]); }

// 4 samples at p (4-sample aligned) <-> ints; one dword (8-bit) / two (16-bit) per access
template <typename Pel>
DEVI void ld4(const Pel* p, int (&v)[4]) {
    if (sizeof(Pel) == 1) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
        v[0] = w & 0xFF; v[1] = (w >> 8) & 0xFF; v[2] = (w >> 16) & 0xFF; v[3] = w >> 24;
    } else {
        const uint2 w = *reinterpret_cast<const uint2*>(p);
        v[0] = w.x & 0xFFFF; v[1] = w.x >> 16; v[2] = w.y & 0xFFFF; v[3] = w.y >> 16;
    }
}
template <typename Pel>
DEVI void st4(Pel* p, const int (&v)[4]) {
    if (sizeof(Pel) == 1) {
        *reinterpret_cast<uint32_t*>(p) = static_cast<uint32_t>(v[0]) | (static_cast<uint32_t>(v[1]) << 8) |
                                          (static_cast<uint32_t>(v[2]) << 16) | (static_cast<uint32_t>(v[3]) << 24);
    } else {
        *reinterpret_cast<uint2*>(p) = make_uint2(static_cast<uint32_t>(v[0]) | (static_cast<uint32_t>(v[1]) << 16),
                                                  static_cast<uint32_t>(v[2]) | (static_cast<uint32_t>(v[3]) << 16));
    }
}

// One 4-line luma edge segment (8.7.2.5.3 decisions, 8.7.2.5.7 filters).  Edges lie on the 8x8
// grid, so the 8-sample window across an edge (4 on each side) is 4-sample aligned and the
// windows of different edges of one pass never overlap: each line is read and written back as
// whole 4-sample words (vertical edges: 2 words per line; horizontal edges: one word per row
// of 4 lines).  P[k][i] / Q[k][i]: line k, distance i from the edge.
// a sample of a plane by a 32-bit element offset from its (uniform) base: the global access then
// takes the saddr form, no 64-bit address arithmetic per access (r05)
template <typename Pel>
DEVI Pel* at32(Pel* base, int off) {
    return reinterpret_cast<Pel*>(reinterpret_cast<uint8_t*>(base) + static_cast<uint32_t>(off) * static_cast<uint32_t>(sizeof(Pel)));
}
template <typename Pel>
DEVI const Pel* at32(const Pel* base, int off) {
    return reinterpret_cast<const Pel*>(reinterpret_cast<const uint8_t*>(base) + static_cast<uint32_t>(off) * static_cast<uint32_t>(sizeof(Pel)));
}
template <typename Pel>
DEVI void hevc_luma_edge(const h2j_frame& f, Pel* pl, int st, const uint8_t* fmap, const int8_t* qmap,
                         const h2j_slice& sl, bool vert, int xe, int ye) {
    const int xp = vert ? xe - 1 : xe, yp = vert ? ye : ye - 1;
    const int qpq = qmap[m24(ye >> 2, f.mw) + (xe >> 2)], qpp = qmap[m24(yp >> 2, f.mw) + (xp >> 2)];
    const int qpl = (qpq + qpp + 1) >> 1;
    const int bd = f.bit_depth;
    const int beta = kBeta[clip3(0, 51, qpl + sl.beta_offset)] * (1 << (bd - 8));
    const int tc = kTc[clip3(0, 53, qpl + 2 + sl.tc_offset)] * (1 << (bd - 8));
    const int maxv = (1 << bd) - 1;
    int P[4][4], Q[4][4];
    if (vert) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            int a[4], c[4];
            ld4(at32(pl, m24(ye + k, st) + xe - 4), a);
            ld4(at32(pl, m24(ye + k, st) + xe), c);
#pragma unroll
            for (int i = 0; i < 4; i++) { P[k][i] = a[3 - i]; Q[k][i] = c[i]; }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int a[4], c[4];
            ld4(at32(pl, m24(ye - 1 - i, st) + xe), a);
            ld4(at32(pl, m24(ye + i, st) + xe), c);
#pragma unroll
            for (int k = 0; k < 4; k++) { P[k][i] = a[k]; Q[k][i] = c[k]; }
        }
    }
    const int dp0 = abs(P[0][2] - 2 * P[0][1] + P[0][0]), dp3 = abs(P[3][2] - 2 * P[3][1] + P[3][0]);
    const int dq0 = abs(Q[0][2] - 2 * Q[0][1] + Q[0][0]), dq3 = abs(Q[3][2] - 2 * Q[3][1] + Q[3][0]);
    const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3;
    if (dpq0 + dpq3 >= beta) return;
    const bool s0 = (2 * dpq0 < (beta >> 2)) && (abs(P[0][3] - P[0][0]) + abs(Q[0][0] - Q[0][3]) < (beta >> 3)) &&
                    (abs(P[0][0] - Q[0][0]) < ((5 * tc + 1) >> 1));
    const bool s3 = (2 * dpq3 < (beta >> 2)) && (abs(P[3][3] - P[3][0]) + abs(Q[3][0] - Q[3][3]) < (beta >> 3)) &&
                    (abs(P[3][0] - Q[3][0]) < ((5 * tc + 1) >> 1));
    const bool dEp = dp < ((beta + (beta >> 1)) >> 3);
    const bool dEq = dq < ((beta + (beta >> 1)) >> 3);
    const bool nfp = fmap[m24(yp >> 2, f.mw) + (xp >> 2)] & 4;
    const bool nfq = fmap[m24(ye >> 2, f.mw) + (xe >> 2)] & 4;
    int NP[4][4], NQ[4][4];  // filtered lines (unfiltered samples keep their value)
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int p0 = P[k][0], p1 = P[k][1], p2 = P[k][2], p3 = P[k][3];
        const int q0 = Q[k][0], q1 = Q[k][1], q2 = Q[k][2], q3 = Q[k][3];
#pragma unroll
        for (int i = 0; i < 4; i++) { NP[k][i] = P[k][i]; NQ[k][i] = Q[k][i]; }
        if (s0 && s3) {
            if (!nfp) {
                NP[k][0] = clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
                NP[k][1] = clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2);
                NP[k][2] = clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
            }
            if (!nfq) {
                NQ[k][0] = clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
                NQ[k][1] = clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2);
                NQ[k][2] = clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3);
            }
        } else {
            int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (abs(delta) < tc * 10) {
                delta = clip3(-tc, tc, delta);
                if (!nfp) NP[k][0] = clip3(0, maxv, p0 + delta);
                if (!nfq) NQ[k][0] = clip3(0, maxv, q0 - delta);
                if (dEp && !nfp) NP[k][1] = clip3(0, maxv, p1 + clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1));
                if (dEq && !nfq) NQ[k][1] = clip3(0, maxv, q1 + clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1));
            }
        }
    }
    if (vert) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int a[4] = {NP[k][3], NP[k][2], NP[k][1], NP[k][0]};
            if (!nfp) st4(at32(pl, m24(ye + k, st) + xe - 4), a);
            if (!nfq) st4(at32(pl, m24(ye + k, st) + xe), NQ[k]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 3; i++) {  // rows at distance 3 are never modified
            const int a[4] = {NP[0][i], NP[1][i], NP[2][i], NP[3][i]};
            const int c[4] = {NQ[0][i], NQ[1][i], NQ[2][i], NQ[3][i]};
            if (!nfp) st4(at32(pl, m24(ye - 1 - i, st) + xe), a);
            if (!nfq) st4(at32(pl, m24(ye + i, st) + xe), c);
        }
    }
}

// One 4-line chroma edge segment (8.7.2.5.5) on the 8x8 chroma grid, whole 4-sample words as
// for luma (vertical edges: the words at xc - 4 and xc of each line; horizontal: rows yc - 2 ..
// yc + 1 at xc).
template <typename Pel>
DEVI void hevc_chroma_edge(const h2j_frame& f, Pel* pl, int st, int pw, int ph, const uint8_t* fmap,
                           const int8_t* qmap, const h2j_slice& sl, int cqpoff, bool vert, int xc, int yc) {
    const int xl = xc * 2, yl = yc * 2;
    const int xp = vert ? xl - 1 : xl, yp = vert ? yl : yl - 1;
    const int qpq = qmap[m24(yl >> 2, f.mw) + (xl >> 2)], qpp = qmap[m24(yp >> 2, f.mw) + (xp >> 2)];
    const int qpc = chroma_qp_tab(((qpq + qpp + 1) >> 1) + cqpoff);
    const int bd = f.bit_depth_c;
    const int tc = kTc[clip3(0, 53, qpc + 2 + sl.tc_offset)] * (1 << (bd - 8));
    const int maxv = (1 << bd) - 1;
    const bool nfp = fmap[m24(yp >> 2, f.mw) + (xp >> 2)] & 4;
    const bool nfq = fmap[m24(yl >> 2, f.mw) + (xl >> 2)] & 4;
    if (vert) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (yc + k >= ph) break;
            const int ro = m24(yc + k, st) + xc;
            int a[4], c[4];
            ld4(at32(pl, ro - 4), a);
            ld4(at32(pl, ro), c);
            const int p0 = a[3], p1 = a[2], q0 = c[0], q1 = c[1];
            const int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
            a[3] = clip3(0, maxv, p0 + delta);
            c[0] = clip3(0, maxv, q0 - delta);
            if (!nfp) st4(at32(pl, ro - 4), a);
            if (!nfq) st4(at32(pl, ro), c);
        }
    } else {
        int r[4][4];  // rows yc - 2 .. yc + 1, columns xc .. xc + 3 (chroma widths are multiples of 4)
#pragma unroll
        for (int j = 0; j < 4; j++) ld4(at32(pl, m24(yc - 2 + j, st) + xc), r[j]);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int p1 = r[0][k], p0 = r[1][k], q0 = r[2][k], q1 = r[3][k];
            const int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
            r[1][k] = clip3(0, maxv, p0 + delta);
            r[2][k] = clip3(0, maxv, q0 - delta);
        }
        if (!nfp) st4(at32(pl, m24(yc - 1, st) + xc), r[1]);
        if (!nfq) st4(at32(pl, m24(yc, st) + xc), r[2]);
    }
}

template <typename Pel>
DEVI void deblock_thread(const h2j_frame& f, const h2j_ctb* ctbs, const h2j_slice* slices, uint8_t* arena,
                         bool vert, int x4, int y4) {
    const int idx = m24(y4, f.mw) + x4;
    const uint8_t* fmap = arena + f.maps;
    const int8_t* qmap = reinterpret_cast<const int8_t*>(fmap + static_cast<size_t>(f.mw) * f.mh);
    const uint8_t fl = fmap[idx];
    if (!(fl & (vert ? 1 : 2))) return;
    const int xe = x4 * 4, ye = y4 * 4;
    auto run = [&](const h2j_slice& sl) __attribute__((always_inline)) {
        hevc_luma_edge<Pel>(f, plane<Pel>(f, arena, f.pic, 0), f.pic_stride[0], fmap, qmap, sl, vert, xe, ye);
        // chroma edges lie on the 16-luma grid; one chroma segment = 8 luma lines
        if ((vert ? (xe & 15) == 0 && (ye & 7) == 0 : (ye & 15) == 0 && (xe & 7) == 0)) {
            const int pw = f.width >> 1, ph = f.height >> 1;
            hevc_chroma_edge<Pel>(f, plane<Pel>(f, arena, f.pic, 1), f.pic_stride[1], pw, ph, fmap, qmap, sl,
                                  f.cb_qp_offset, vert, xe >> 1, ye >> 1);
            hevc_chroma_edge<Pel>(f, plane<Pel>(f, arena, f.pic, 2), f.pic_stride[2], pw, ph, fmap, qmap, sl,
                                  f.cr_qp_offset, vert, xe >> 1, ye >> 1);
        }
    };
    // one slice from CTB 0 and one tile (frame.topo 0): the picture's first slice, a uniform
    // (scalar) load, instead of two dependent per-thread loads (the CTB record, then its slice)
    if (f.topo) run(slices[ctbs[(ye >> f.log2ctb) * f.ctb_w + (xe >> f.log2ctb)].slice]);
    else run(slices[0]);
}

__global__ void __launch_bounds__(256, 8) h2j_k2_deblock(const h2j_frame* __restrict__ frames,
                                                     const h2j_ctb* __restrict__ ctbs,
                                                     const h2j_slice* __restrict__ slices, uint8_t* __restrict__ arena,
                                                     int vert) {
    const h2j_frame& f = frames[blockIdx.y];
    if (f.codec != H2J_CODEC_HEVC) return;
    // threads only on the 8x8 edge grid of the pass: even 4x4 columns (vertical edges) or even
    // 4x4 rows (horizontal edges) -- one thread per 4x4 block left half the lanes of every
    // vertical-pass wave idle and half the horizontal-pass waves empty
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    int x4, y4;
    if (vert) {
        const int mw2 = (f.mw + 1) >> 1;
        if (idx >= mw2 * f.mh) return;
        y4 = idx / mw2;
        x4 = (idx - y4 * mw2) * 2;
    } else {
        const int mh2 = (f.mh + 1) >> 1;
        if (idx >= f.mw * mh2) return;
        const int r = idx / f.mw;
        x4 = idx - r * f.mw;
        y4 = r * 2;
    }
    const h2j_ctb* C = ctbs + f.ctb;
    const h2j_slice* S = slices + f.slice;
    if (f.bit_depth == 8) deblock_thread<uint8_t>(f, C, S, arena, vert != 0, x4, y4);
    else deblock_thread<uint16_t>(f, C, S, arena, vert != 0, x4, y4);
}


// ---------------------------------------------------------------- K2': H.264 deblocking
// H.264 8.7 filters macroblock by macroblock (vertical edges, then
// horizontal edges) and each macroblock sees the samples already filtered by
// its left / top / top-right neighbours, so it is not edge-parallel like
// HEVC.  One workgroup per picture walks the anti-diagonals d = mx + 2*my
// (all dependencies of an MB lie on earlier diagonals); 16 lanes per MB,
// one lane per line across each edge phase.
__constant__ int kAlpha264[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   4,   4,
                                      5,  6,  7,  8,  9,  10, 12, 13, 15, 17, 20, 22, 25,  28,  32,  36,  40,  45,
                                      50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
__constant__ int kBeta264[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  2,  2,
                                     2,  3,  3,  3,  3,  4,  4,  4,  6,  6,  7,  7,  8,  8,  9,  9,  10, 10,
                                     11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
__constant__ int kTc0_264[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1},
    {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4},
    {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11},
    {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

__constant__ int kChromaQp264[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

// H.264 edge filter (8.7.2.3-8.7.2.4) on a line held in registers, for a lane that holds either a
// luma line or a chroma line (`chroma`), so luma and chroma lanes run one instruction stream: chroma (8.7.2.3-8.7.2.4 with chromaEdgeFlag = 1) is the
// luma filter with ap / aq < beta forced false -- tc = tc0 + 1, p1 / q1 untouched for bS < 4, the
// 3-tap p0 / q0 form for bS 4 -- and only p1..q1 of it matter.  v: 20 samples, the edge between
// v[E - 1] and v[E]; `on` false leaves the line as is.  Selects only (lanes diverge on data).
// Every sample of v is in [0, 65535] (loaded from uint16, and the filters' outputs stay between
// their inputs), so |a - b| is one v_sad_u16 (the high halves are zero); the clips below all have
// lo <= hi, where clip3 is one v_med3_i32 (the compiler emits min + max for runtime bounds).
DEVI int db_absd(int a, int b) {
    return static_cast<int>(__builtin_amdgcn_sad_u16(static_cast<uint32_t>(a), static_cast<uint32_t>(b), 0u));
}
DEVI int db_clip(int lo, int hi, int v) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(lo), "v"(hi));
    return r;
}
template <int E>
DEVI void h264_filt_line(int (&v)[20], bool on, int bs, int alpha, int beta, int tc0, int maxv, bool chroma) {
    const int p0 = v[E - 1], p1 = v[E - 2], p2 = v[E - 3], q0 = v[E], q1 = v[E + 1], q2 = v[E + 2];
    const int d0 = db_absd(p0, q0);
    const bool f = on && d0 < alpha && db_absd(p1, p0) < beta && db_absd(q1, q0) < beta;
    const bool apb = !chroma && db_absd(p2, p0) < beta, aqb = !chroma && db_absd(q2, q0) < beta;
    if (bs < 4) {
        const int tc = chroma ? tc0 + 1 : tc0 + apb + aqb;
        const int dl = db_clip(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
        const int avg = (p0 + q0 + 1) >> 1;
        const int np1 = apb ? p1 + db_clip(-tc0, tc0, (p2 + avg - (p1 * 2)) >> 1) : p1;
        const int nq1 = aqb ? q1 + db_clip(-tc0, tc0, (q2 + avg - (q1 * 2)) >> 1) : q1;
        v[E - 1] = f ? db_clip(0, maxv, p0 + dl) : p0;
        v[E] = f ? db_clip(0, maxv, q0 - dl) : q0;
        v[E - 2] = f ? np1 : p1;
        v[E + 1] = f ? nq1 : q1;
    } else {
        const int p3 = v[E - 4], q3 = v[E + 3];
        const bool sm = d0 < ((alpha >> 2) + 2);
        const bool sp = apb && sm, sq = aqb && sm;
        const int np0 = sp ? (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3 : (2 * p1 + p0 + q1 + 2) >> 2;
        const int np1 = sp ? (p2 + p1 + p0 + q0 + 2) >> 2 : p1;
        const int np2 = sp ? (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3 : p2;
        const int nq0 = sq ? (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3 : (2 * q1 + q0 + p1 + 2) >> 2;
        const int nq1 = sq ? (p0 + q0 + q1 + q2 + 2) >> 2 : q1;
        const int nq2 = sq ? (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3 : q2;
        v[E - 1] = f ? np0 : p0;
        v[E - 2] = f ? np1 : p1;
        v[E - 3] = f ? np2 : p2;
        v[E] = f ? nq0 : q0;
        v[E + 1] = f ? nq1 : q1;
        v[E + 2] = f ? nq2 : q2;
    }
}

// H.264 K2 (8.7) window of one MB: MB (x, y) starts once row y-1 has finished MBs 0..x+1 (its
// top edge reads and modifies row y-1's bottom rows, which MB (x+1, y-1)'s left edge modifies
// too).  The MB is filtered inside an LDS window (the MB, 4 luma / 2 chroma rows above it, 4 / 2
// columns left of it); the rows above come from a per-picture line buffer that every row leaves
// behind, the columns on the left are carried from the previous MB.  After the 8 luma + 4 chroma
// edge passes the window is written back once.
// r05: the staging is Pel-typed (luma 4, chroma 8 MBs wide at 8 bits) and the previous MB is kept
// in it rather than in a copy, so an 8-bit window is 3.7 KB: with the 8-bit LDS line buffer (6 bytes
// per column) two 8-wave workgroups of the 8-bit kernel share a CU (4 waves per SIMD, where one
// 104 KB workgroup left 2)
constexpr int kDbGL = 4;  // luma staging group (MBs): 64-byte rows at 8 bits
template <typename Pel>
constexpr int kDbGC = sizeof(Pel) == 1 ? 8 : 4;  // chroma staging group: 64-byte rows
template <typename Pel>
struct alignas(16) DbWin {
    uint16_t y[20][20];     // luma: (row, col) = (y + 4, x + 4) relative to the MB
    // chroma: (y + 2, x + 2); rows of 12 (2 unused): the filter's dword / sample loads of the chroma
    // lines then fall on banks the luma lines leave free more often (modelled 54 -> 48 LDS cycles
    // per MB for the edge loads)
    uint16_t c[2][10][12];
    // final samples staged and written as whole rows: rows 12..15 of the MBs above (luma
    // [4][16 GL], chroma [2][2][8 GC]) and rows of this row's MBs (luma [16][16 GL], chroma
    // [2][8][8 GC])
    alignas(16) Pel sa[4 * 16 * kDbGL + 2 * 2 * 8 * kDbGC<Pel>];
    alignas(16) Pel sb[16 * 16 * kDbGL + 2 * 8 * 8 * kDbGC<Pel>];
};
// n (4, 8 or 16) Pel between 16-byte-aligned LDS staging and the picture
template <typename Pel, int N>
DEVI void db264_copy(Pel* dst, const Pel* src) {
    constexpr int B = N * static_cast<int>(sizeof(Pel));
    if constexpr (B == 4) *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(src);
    else if constexpr (B == 8) *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(src);
    else {
#pragma unroll
        for (int k = 0; k < B / 16; k++) reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
    }
}

// Deblocking parameters of one MB and of its top neighbour, loaded one MB ahead with VECTOR
// loads (lane 0/1: the MB's dwords 2 and 9, lane 2/3: the top MB's): scalar loads would be
// waited with lgkmcnt(0), which also drains every LDS access in between (the old form cost
// ~2k cycles per MB).  Fields: slice = byte 9, qp = byte 36, mbflags = byte 37.
static_assert(offsetof(h2j_ctb, slice) == 9 && offsetof(h2j_ctb, qp) == 36 && offsetof(h2j_ctb, mbflags) == 37 &&
                  sizeof(h2j_ctb) % 4 == 0,
              "h2j_ctb layout assumed by db264_info_raw");
DEVI uint32_t db264_info_raw(const h2j_ctb* mbs, int mbw, int mx, int my, int lane) {
    const int top = my > 0 ? m24(my - 1, mbw) + mx : m24(my, mbw) + mx;
    const int idx = (lane & 2) ? top : m24(my, mbw) + mx;
    return reinterpret_cast<const uint32_t*>(mbs + idx)[(lane & 1) ? 9 : 2];
}
// LDS copies of the H.264 deblocking tables (per-lane lookups, no scalar-load chains)
constexpr int kDbSlices = 64;  // slices cached in LDS; more are read from global memory
static_assert(sizeof(h2j_slice) % 4 == 0, "slice records are copied to LDS as dwords");
struct DbTables {
    int alpha[52], beta[52], tc0[52];  // tc0: bS 3 column (intra internal edges)
    int cqp[22];                       // chroma QP map above 29
    h2j_slice sl[kDbSlices];
};

// ---- H.264 K2, two macroblock rows per wave (fill the wave).  A workgroup of
// kDbPairWaves waves deblocks a picture (or a 16-row band of a tall one); wave w takes the row
// pairs (2p, 2p + 1), p = w, w + kDbPairWaves, ...: lanes 0-31 (half 0) walk row 2p, lanes 32-63
// (half 1) walk row 2p + 1 kDbLag MBs behind.  h264_db_rows left lanes 32-63 idle through the
// line filter (32 lines per MB: 16 luma, 8 + 8 chroma); here they filter the second row's MB in
// the same instructions, and the data movement around the filter moves each MB with 32 lanes
// instead of 64 (the same instructions per MB).  Dependencies are those of h264_db_rows: MB
// (x, y) needs row y - 1 finished through MB x + 1 -- inside a wave by the lag (half 0 has
// finished x + kDbLag MBs when half 1 starts MB x), across waves by the progress word of row
// 2p - 1.  The halves share the picture's line buffer: at one step they touch disjoint MB
// columns of it (half 0 columns s - 1 and s, half 1 columns s - 3 and s - 2).  Pictures wider
// than the LDS line buffer allows (line_w) keep it in global memory, in the picture's residual
// region (K1's input, dead once K1 has run).
constexpr int kDbPairWaves = 8;
constexpr int kDbLag = 2;
constexpr int kDbPairSlots = 4 * kDbPairWaves;  // progress words: 2 rows in flight per wave, twice over
static_assert(sizeof(h2j_slice) == 12 && offsetof(h2j_slice, slice_addr_rs) == 8 &&
                  offsetof(h2j_slice, deblock_disabled) == 5 && offsetof(h2j_slice, cqp_offset) == 6,
              "slice dwords assumed by h264_db_pairs");
template <typename Pel>
struct DbPrefetch2 {  // one MB per half: 8 luma + 4 chroma samples per lane, as loaded
    typename std::conditional<sizeof(Pel) == 1, uint2, uint4>::type y;
    typename std::conditional<sizeof(Pel) == 1, uint32_t, uint2>::type c;
};
template <typename Pel>
DEVI void db264_fetch2(const uint8_t* PB, uint32_t oc0, uint32_t oc1, int sty, int stc, int mx, int my, DbPrefetch2<Pel>& r, int hl) {
    using TY = decltype(r.y);
    using TC = decltype(r.c);
    constexpr uint32_t B = sizeof(Pel);
    r.y = *reinterpret_cast<const TY*>(PB + static_cast<uint32_t>(m24(my * 16 + (hl >> 1), sty) + mx * 16 + (hl & 1) * 8) * B);
    const int k = hl & 15;
    r.c = *reinterpret_cast<const TC*>(PB + ((hl >> 4) ? oc1 : oc0) + static_cast<uint32_t>(m24(my * 8 + (k >> 1), stc) + mx * 8 + (k & 1) * 4) * B);
}
// 4 uint16 window samples (two dwords) as 4 Pel of the picture / staging
DEVI uint32_t db_pk8(uint2 v) { return __builtin_amdgcn_perm(v.y, v.x, 0x06040200u); }
template <typename Pel>
DEVI void db_st4(Pel* d, uint2 v) {
    if constexpr (sizeof(Pel) == 1) *reinterpret_cast<uint32_t*>(d) = db_pk8(v);
    else *reinterpret_cast<uint2*>(d) = v;
}
template <typename Pel>
DEVI void db_st8(Pel* d, uint2 a, uint2 b) {
    if constexpr (sizeof(Pel) == 1) *reinterpret_cast<uint2*>(d) = make_uint2(db_pk8(a), db_pk8(b));
    else *reinterpret_cast<uint4*>(d) = make_uint4(a.x, a.y, b.x, b.y);
}
DEVI uint2 db_ld4a8(const uint16_t* p) { return *reinterpret_cast<const uint2*>(p); }  // 8-byte aligned
DEVI uint2 db_ld4a4(const uint16_t* p) {                                              // 4-byte aligned
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    return make_uint2(q[0], q[1]);
}
DEVI uint32_t db_u16pair(const uint16_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
DEVI void db_put_u16pair(uint16_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
// two line-buffer samples as a window pair (low half the first): uint16 lines as they are, the
// 8-bit kernel's LDS line widened / narrowed by byte permutes
DEVI uint32_t db_line2(const uint16_t* p) { return db_u16pair(p); }
DEVI uint32_t db_line2(const uint8_t* p) {
    return __builtin_amdgcn_perm(0u, static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(p)), 0x0c010c00u);
}
DEVI void db_put_line2(uint16_t* p, uint32_t v) { db_put_u16pair(p, v); }
DEVI void db_put_line2(uint8_t* p, uint32_t v) {
    *reinterpret_cast<uint16_t*>(p) = static_cast<uint16_t>(__builtin_amdgcn_perm(0u, v, 0x0c0c0200u));
}

// Line: the line buffer's sample type (GLine: uint16 in global memory; else Pel, in LDS)
template <typename Pel, bool GLine, typename Line>
DEVI void h264_db_pairs(const h2j_frame& f, const h2j_ctb* mbs, const h2j_slice* slices, uint8_t* arena, DbWin<Pel>* W,
                        uint32_t* prog, Line* line, int band, int nbands, const DbTables& TB) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, hl = lane & 31;
    DbWin<Pel>& w = W[2 * wv + h];
    const int mbw = ufl(f.ctb_w), mbh = ufl(f.ctb_h), width = ufl(f.width);
    const int bd = ufl(f.bit_depth), bdc = ufl(f.bit_depth_c);
    const int sty = ufl(f.pic_stride[0]), stc = ufl(f.pic_stride[1]);
    // picture addresses as the uniform base plus a 32-bit byte offset (the saddr form of the global
    // accesses: no 64-bit address arithmetic per access)
    uint8_t* const PB = arena + ufl64(f.pic);
    const uint32_t oc0 = ufl(f.pic_off[1]) * static_cast<uint32_t>(sizeof(Pel));
    const uint32_t oc1 = ufl(f.pic_off[2]) * static_cast<uint32_t>(sizeof(Pel));
    auto py_at = [&](int o) __attribute__((always_inline)) {
        return reinterpret_cast<Pel*>(PB + static_cast<uint32_t>(o) * static_cast<uint32_t>(sizeof(Pel)));
    };
    auto pc_at = [&](int c, int o) __attribute__((always_inline)) {
        return reinterpret_cast<Pel*>(PB + (c ? oc1 : oc0) + static_cast<uint32_t>(o) * static_cast<uint32_t>(sizeof(Pel)));
    };
    Line* LY = line;              // [4][width]: rows 12..15 of the MB row above
    Line* LC = line + 4 * width;  // [2 comps][2 rows][width / 2]: chroma rows 6..7
    const int cw = width >> 1;
    const int rbeg = band * 16, rend = nbands > 1 ? min(mbh, rbeg + 16) : mbh;
    const int npairs = (rend - rbeg + 1) >> 1;
    const uint64_t o_flag = ufl64(f.ctbrng) + 12, o_xl = ufl64(f.xline);
    if (wv >= npairs) return;
    const int hl_ln = hl;
    DBP_DECL;
    // filter lanes of a half: 0-15 luma lines, 16-23 Cb, 24-31 Cr
    const bool luma_lane = hl < 16, chroma = !luma_lane;
    const int cc = (hl >> 3) & 1, ck = hl & 7;
    const int maxv = chroma ? (1 << bdc) - 1 : (1 << bd) - 1;
    const int tsh = chroma ? bdc - 8 : bd - 8, clo = -6 * (bdc - 8);
    DbPrefetch2<Pel> pf;
    uint32_t ninfo = 0;
    {
        const int r = rbeg + 2 * wv + h;
        if (r < rend) {
            db264_fetch2<Pel>(PB, oc0, oc1, sty, stc, 0, r, pf, hl);
            ninfo = db264_info_raw(mbs, mbw, 0, r, hl);
        }
    }
    int lmf = 0, lqp = 0, lsaddr = -1;  // left neighbour (previous MB of the half's row)
    for (int p = wv; p < npairs; p += kDbPairWaves) {
        const int r0 = rbeg + 2 * p;
        const bool two = r0 + 1 < rend;
        const int row = r0 + h;
        const bool hv = h == 0 || two;
        const int nsteps = two ? mbw + kDbLag : mbw;
        const bool from_band = nbands > 1 && band > 0 && p == 0;  // half 0's row is the band's first
        const bool fb = from_band && h == 0;
        const bool to_band = nbands > 1 && band < nbands - 1 && row == rend - 1;
        const uint64_t o_xin = o_xl + 12ull * (band - 1) * width, o_xout = o_xl + 12ull * band * width;
        uint32_t* above = prog + (r0 + kDbPairSlots - 1) % kDbPairSlots;  // row r0 - 1
        uint32_t* mine = prog + (r0 + 1) % kDbPairSlots;                  // row r0 + 1 (half 1)
        uint32_t seen = 0;
        for (int s = 0; s < nsteps; s++) {
            const int mx = s - kDbLag * h;
            const bool live = hv && mx >= 0 && mx < mbw;
            // half 0's MB s needs row r0 - 1 through MB s + 1 (half 1's row is covered by the lag)
            if (s < mbw) {
                if (from_band) {
                    const uint32_t need = static_cast<uint32_t>(mbw + min(s + 2, mbw));
                    if (seen < need) {
                        uint32_t it = 0;
                        uint32_t* fl = reinterpret_cast<uint32_t*>(arena + o_flag) + 4 * ((r0 - 1) * mbw);
                        while ((seen = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < need) {
                            __builtin_amdgcn_s_sleep(2);
                            if (++it > (1u << 22)) {  // never expected: flag the picture, do not hang the GPU
                                if (lane == 0) __hip_atomic_fetch_or(dev_error_word(arena, f), kDevErrDbBand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                seen = 2u * mbw;
                                break;
                            }
                        }
                    }
                } else if (r0 > rbeg || (r0 > 0 && nbands <= 1)) {
                    const uint32_t need = (static_cast<uint32_t>(r0) << 16) | static_cast<uint32_t>(min(s + 2, mbw));
                    if (seen < need) seen = wait_progress(above, need, dev_error_word(arena, f), kDevErrDbRow264);
                }
            }
            DBP_LAP(0);
            // this MB's parameters (loaded one MB ahead) are taken before the next MB's loads are
            // issued: consumed after them, the compiler's vmcnt wait for them covered those loads too
            const uint32_t cur = ninfo;
            asm volatile("" ::"v"(cur));  // (the copy's wait here, not where ninfo's register is reloaded)
            if (live) {
                // the lane index laundered per MB in the window and write-back sections: the
                // compiler then recomputes their lane-dependent LDS / global addresses there
                // instead of keeping dozens of them live across the MB loop (r05: 208 -> 110
                // VGPRs, 4 waves per SIMD; laundering the filter sections too measured slower)
                int hl = hl_ln;
                asm volatile("" : "+v"(hl));
                // window: the MB body (prefetched), the rows above (line buffer), left columns carried
                {
                    uint16_t* d = &w.y[(hl >> 1) + 4][(hl & 1) * 8 + 4];  // 8-byte aligned
                    if constexpr (sizeof(Pel) == 1) {
                        *reinterpret_cast<uint2*>(d) = make_uint2(__builtin_amdgcn_perm(0u, pf.y.x, 0x0c010c00u), __builtin_amdgcn_perm(0u, pf.y.x, 0x0c030c02u));
                        *reinterpret_cast<uint2*>(d + 4) = make_uint2(__builtin_amdgcn_perm(0u, pf.y.y, 0x0c010c00u), __builtin_amdgcn_perm(0u, pf.y.y, 0x0c030c02u));
                    } else {
                        *reinterpret_cast<uint2*>(d) = make_uint2(pf.y.x, pf.y.y);
                        *reinterpret_cast<uint2*>(d + 4) = make_uint2(pf.y.z, pf.y.w);
                    }
                    const int k = hl & 15;
                    uint16_t* e = &w.c[hl >> 4][(k >> 1) + 2][(k & 1) * 4 + 2];  // 4-byte aligned
                    if constexpr (sizeof(Pel) == 1) {
                        db_put_u16pair(e, __builtin_amdgcn_perm(0u, pf.c, 0x0c010c00u));
                        db_put_u16pair(e + 2, __builtin_amdgcn_perm(0u, pf.c, 0x0c030c02u));
                    } else {
                        db_put_u16pair(e, pf.c.x);
                        db_put_u16pair(e + 2, pf.c.y);
                    }
                }
                if (fb) {
                    const uint16_t* X = reinterpret_cast<const uint16_t*>(arena + o_xin);
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int e = hl * 2 + j, tr = e >> 4, tc = e & 15;
                        w.y[tr][tc + 4] = __hip_atomic_load(X + tr * width + mx * 16 + tc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    const int c2 = hl >> 4, cr = (hl >> 3) & 1, k2 = hl & 7;
                    w.c[c2][cr][k2 + 2] = __hip_atomic_load(X + 4 * width + (c2 * 2 + cr) * cw + mx * 8 + k2,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if (row > 0) {
                    const int tr = hl >> 3, tc = (hl & 7) * 2;  // 4 rows x 16 luma columns, 2 per lane
                    db_put_u16pair(&w.y[tr][tc + 4], db_line2(LY + m24(tr, width) + mx * 16 + tc));
                    const int c2 = hl >> 4, cr = (hl >> 3) & 1, k2 = hl & 7;  // 2 comps x 2 rows x 8 columns
                    w.c[c2][cr][k2 + 2] = static_cast<uint16_t>(LC[m24(c2 * 2 + cr, cw) + mx * 8 + k2]);
                }
                // prefetch the half's next MB (its next row: two pairs on) and its parameters
                int nx = mx + 1, ny = row;
                if (nx == mbw) { nx = 0; ny += 2 * kDbPairWaves; }
                if (ny < mbh) {
                    db264_fetch2<Pel>(PB, oc0, oc1, sty, stc, nx, ny, pf, hl);
                    ninfo = db264_info_raw(mbs, mbw, nx, ny, hl);
                }
            }
            wave_sync();
            DBP_LAP(1);
            auto pick = [&](int k) __attribute__((always_inline)) {
                const uint32_t a = __builtin_amdgcn_readlane(cur, k), b = __builtin_amdgcn_readlane(cur, 32 + k);
                return h ? b : a;
            };
            const uint32_t i0 = pick(0), i1 = pick(1), i2 = pick(2), i3 = pick(3);
            const int mf = static_cast<int>((i1 >> 8) & 0xFF), mqp = static_cast<int8_t>(i1 & 0xFF);
            const int csl = static_cast<int>((i0 >> 8) & 0xFF), tsl = static_cast<int>((i2 >> 8) & 0xFF);
            const int tmf = row > 0 ? static_cast<int>((i3 >> 8) & 0xFF) : 0, tqp = static_cast<int8_t>(i3 & 0xFF);
            // the slice's dwords {beta, tc, sao, sao}, {lf, dd, cqp0, cqp1}, {first MB}
            uint32_t s0, s1, s2, ts2 = ~0u;
            const uint32_t* TBS = reinterpret_cast<const uint32_t*>(TB.sl);
            const uint32_t* GS = reinterpret_cast<const uint32_t*>(slices);
            // (slices past the LDS copy: global loads, waited inside their branch -- a wait at the
            // merged first use would also wait for the next MB's prefetch loads)
            if (csl < kDbSlices) { s0 = TBS[3 * csl]; s1 = TBS[3 * csl + 1]; s2 = TBS[3 * csl + 2]; }
            else { s0 = GS[3 * csl]; s1 = GS[3 * csl + 1]; s2 = GS[3 * csl + 2]; asm volatile("" ::"v"(s0), "v"(s1), "v"(s2)); }
            if (row > 0) {
                if (tsl < kDbSlices) ts2 = TBS[3 * tsl + 2];
                else { ts2 = GS[3 * tsl + 2]; asm volatile("" ::"v"(ts2)); }
            }
            const int dd = static_cast<int>((s1 >> 8) & 0xFF);
            const int beo = static_cast<int8_t>(s0 & 0xFF), tco = static_cast<int8_t>((s0 >> 8) & 0xFF);
            const int cq0 = static_cast<int8_t>((s1 >> 16) & 0xFF), cq1 = static_cast<int8_t>(s1 >> 24);
            const int saddr = static_cast<int>(s2), tsaddr = static_cast<int>(ts2);
            DBP_LAP(2);
            if (live && (mf & 4) && dd != 1) {
                // thresholds of the lane's component, per lane (no cross-lane traffic): the left and
                // top MB edges and the internal edges (8.7.2.2; chroma QPs through Table 8-15)
                const int qm = (mf & 1) ? 0 : mqp, ql = (lmf & 1) ? 0 : lqp, qt = (tmf & 1) ? 0 : tqp;
                const int off = cc ? cq1 : cq0;
                auto cqp = [&](int q) __attribute__((always_inline)) {
                    const int a = clip3(clo, 51, q + off);
                    const int m = a < 30 ? a : TB.cqp[max(a - 30, 0)];
                    return chroma ? m : q;
                };
                const int qmc = cqp(qm), qlc = cqp(ql), qtc = cqp(qt);
                const int qaL = (qlc + qmc + 1) >> 1, qaT = (qtc + qmc + 1) >> 1;
                const int iaL = clip3(0, 51, qaL + tco), ibL = clip3(0, 51, qaL + beo);
                const int iaT = clip3(0, 51, qaT + tco), ibT = clip3(0, 51, qaT + beo);
                const int iaI = clip3(0, 51, qmc + tco), ibI = clip3(0, 51, qmc + beo);
                const int aL = TB.alpha[iaL] << tsh, bL = TB.beta[ibL] << tsh;
                const int aT = TB.alpha[iaT] << tsh, bT = TB.beta[ibT] << tsh;
                const int aI = TB.alpha[iaI] << tsh, bI = TB.beta[ibI] << tsh, tI = TB.tc0[iaI] << tsh;
                const bool t8 = (mf & 2) != 0;
                for (int dir = 0; dir < 2; dir++) {  // 0: vertical edges, 1: horizontal edges
                    const bool vert = dir == 0;
                    const int nmf = vert ? (mx > 0 ? lmf : 0) : tmf;
                    bool mb_edge = (nmf & 4) != 0;
                    if (mb_edge && dd == 2 && (vert ? lsaddr : tsaddr) != saddr) mb_edge = false;
                    const int aM = vert ? aL : aT, bM = vert ? bL : bT;
                    // the line of this lane, as in h264_db_rows (chroma at v[2..11])
                    const int stp = vert ? 1 : (luma_lane ? 20 : 12);
                    const uint16_t* base = luma_lane ? (vert ? &w.y[hl + 4][0] : &w.y[0][hl + 4])
                                                     : (vert ? &w.c[cc][ck + 2][0] : &w.c[cc][0][ck + 2]) - 2 * stp;
                    int v[20];
                    // vertical edges: the lane's line is a window row, 4-byte aligned (luma rows 40 B,
                    // chroma rows 24 B from column -2): ten dword loads / stores instead of twenty
                    // / eighteen 16-bit ones (r04m: LDS bank conflicts were 68 % of LDS cycles)
                    if (vert) {
                        const uint32_t* b32 = reinterpret_cast<const uint32_t*>(base);
#pragma unroll
                        for (int d = 0; d < 10; d++) {
                            const uint32_t u = b32[d];
                            v[2 * d] = static_cast<int>(u & 0xFFFFu);
                            v[2 * d + 1] = static_cast<int>(u >> 16);
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < 20; i++) v[i] = base[i * stp];
                    }
                    h264_filt_line<4>(v, mb_edge, 4, aM, bM, 0, maxv, chroma);
                    h264_filt_line<8>(v, chroma || !t8, 3, aI, bI, tI, maxv, chroma);
                    h264_filt_line<12>(v, luma_lane, 3, aI, bI, tI, maxv, chroma);
                    h264_filt_line<16>(v, luma_lane && !t8, 3, aI, bI, tI, maxv, chroma);
                    uint16_t* dst = const_cast<uint16_t*>(base);
                    if (vert) {  // luma: the whole row (v[0], v[19] unchanged); chroma: its row, v[2..11]
                        uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
                        for (int d = 0; d < 10; d++)
                            if (luma_lane || (d >= 1 && d <= 5))
                                d32[d] = static_cast<uint32_t>(v[2 * d]) | (static_cast<uint32_t>(v[2 * d + 1]) << 16);
                    } else {
#pragma unroll
                        for (int i = 1; i < 19; i++)
                            if (luma_lane || (i >= 3 && i <= 8)) dst[i * stp] = static_cast<uint16_t>(v[i]);
                    }
                    wave_sync();
                    DBP_LAPK(dir * 4);
                }
            }
            if (live) {
                int hl = hl_ln;
                asm volatile("" : "+v"(hl));
                lmf = mf;
                lqp = mqp;
                lsaddr = saddr;
                // write back (the rules of h264_db_rows): rows 12..15 of MB (x, y - 1), rows of
                // MB (x - 1, y), and on the row's last MB its own rows.  Staged kDbGL (luma) /
                // kDbGC (chroma) MBs wide so every flush writes rows of 64 bytes or more (r05:
                // 32-byte chroma pieces made the L2 fetch each line they touch, FETCH 1.3x -> 5x the
                // picture).  An MB's samples go to the staging as soon as the MB is done; the next
                // MB's left edge then rewrites the columns it changed (luma 12..15, chroma 7).
                constexpr int GL = kDbGL, GC = kDbGC<Pel>, LW = 16 * GL, CW = 8 * GC;
                constexpr int SS = 16 / static_cast<int>(sizeof(Pel));  // samples per 16-byte piece
                const bool last_row = row == mbh - 1, last = mx == mbw - 1;
                const int nr = last_row ? 16 : 12, ncr = last_row ? 8 : 6;
                Pel* SA = w.sa;  // luma [4][LW] | chroma [2][2][CW]
                Pel* SB = w.sb;  // luma [16][LW] | chroma [2][8][CW]
                Pel* const SAc = SA + 4 * LW;
                Pel* const SBc = SB + 16 * LW;
                // 16-byte chroma pieces: one store when the row is 16-byte aligned (at 8 bits the
                // chroma width may be an odd multiple of 8)
                auto cput16 = [&](Pel* d, const Pel* q) __attribute__((always_inline)) {
                    if (sizeof(Pel) == 2 || (stc & 15) == 0) {
                        db264_copy<Pel, SS>(d, q);
                    } else {
                        db264_copy<Pel, 8>(d, q);
                        db264_copy<Pel, 8>(d + 8, q + 8);
                    }
                };
                if (row > 0) {
                    if (hl < 16) {
                        const int tr = hl >> 2, c4 = (hl & 3) * 4;
                        db_st4<Pel>(SA + tr * LW + (mx % GL) * 16 + c4, db_ld4a8(&w.y[tr][c4 + 4]));
                    } else if (hl < 24) {  // chroma rows 6..7
                        const int k = hl - 16, c2 = k >> 2, cr = (k >> 1) & 1, c4 = (k & 1) * 4;
                        db_st4<Pel>(SAc + (c2 * 2 + cr) * CW + (mx % GC) * 8 + c4, db_ld4a4(&w.c[c2][cr][c4 + 2]));
                    }
                    const bool fl = mx % GL == GL - 1 || last, fc = mx % GC == GC - 1 || last;
                    if (fl || fc) wave_sync();
                    if (fl) {  // the group's luma rows 12..15: 4 rows x LW / SS pieces of 16 bytes
                        const int g0 = mx - mx % GL, nmb = mx - g0 + 1;
                        const int tr = hl >> 3, sg = hl & 7;
                        if (sg * SS < nmb * 16) db264_copy<Pel, SS>(py_at(m24(row * 16 - 4 + tr, sty) + g0 * 16 + sg * SS), SA + tr * LW + sg * SS);
                    }
                    if (fc) {  // chroma rows 6..7: 2 comps x 2 rows x 8 pieces of 8 bytes
                        constexpr int S8 = 8 / static_cast<int>(sizeof(Pel));
                        const int g0 = mx - mx % GC, nmb = mx - g0 + 1;
                        const int c2 = hl >> 4, cr = (hl >> 3) & 1, cs = hl & 7;
                        if (cs * S8 < nmb * 8)
                            db264_copy<Pel, S8>(pc_at(c2, m24(row * 8 - 2 + cr, stc) + g0 * 8 + cs * S8), SAc + (c2 * 2 + cr) * CW + cs * S8);
                    }
                }
                auto flush_bl = [&](int g0, int nmb) __attribute__((always_inline)) {
                    // luma: 16 rows x LW / SS pieces of 16 bytes, piece e = hl + 32 k
                    constexpr int PR = LW / SS;
#pragma unroll
                    for (int k = 0; k < 16 * PR / 32; k++) {
                        const int e = hl + 32 * k, r = e / PR, sp = e % PR;
                        if (r < nr && sp * SS < nmb * 16) db264_copy<Pel, SS>(py_at(m24(row * 16 + r, sty) + g0 * 16 + sp * SS), SB + r * LW + sp * SS);
                    }
                };
                auto flush_bc = [&](int g0, int nmb) __attribute__((always_inline)) {
                    // chroma: 2 comps x 8 rows x 4 pieces of 16 bytes (CW is 64 bytes at either size)
                    static_assert(CW == 4 * SS, "chroma staging rows of four 16-byte pieces");
#pragma unroll
                    for (int k = 0; k < 2; k++) {
                        const int e = hl + 32 * k, c2 = e >> 5, cr = (e >> 2) & 7, sg = e & 3;
                        if (cr < ncr) {
                            Pel* d = pc_at(c2, m24(row * 8 + cr, stc) + g0 * 8 + sg * SS);
                            const Pel* q = SBc + (c2 * 8 + cr) * CW + sg * SS;
                            if ((sg + 1) * SS <= nmb * 8) cput16(d, q);
                            else if (sg * SS < nmb * 8) db264_copy<Pel, 8>(d, q);  // 8 bits: an odd last MB
                        }
                    }
                };
                if (mx > 0) {  // the previous MB's columns the left edge just finished
                    const int px = mx - 1;
                    if (hl < 16) {
                        db_st4<Pel>(SB + hl * LW + (px % GL) * 16 + 12, db_ld4a8(&w.y[hl + 4][0]));
                    } else {
                        const int k = hl - 16, c2 = k >> 3, cr = k & 7;
                        SBc[(c2 * 8 + cr) * CW + (px % GC) * 8 + 7] = static_cast<Pel>(w.c[c2][cr + 2][1]);
                    }
                    const bool fl = px % GL == GL - 1, fc = px % GC == GC - 1;
                    if (fl || fc) wave_sync();
                    if (fl) flush_bl(px - (GL - 1), GL);
                    if (fc) flush_bc(px - (GC - 1), GC);
                }
                {  // this MB's rows into the staging (in-order LDS: after the flush's reads above)
                    const int r = hl >> 1, c8 = (hl & 1) * 8;
                    db_st8<Pel>(SB + r * LW + (mx % GL) * 16 + c8, db_ld4a8(&w.y[r + 4][c8 + 4]), db_ld4a8(&w.y[r + 4][c8 + 8]));
                    const int c2 = hl >> 4, k = hl & 15, cr = k >> 1, c4 = (k & 1) * 4;
                    db_st4<Pel>(SBc + (c2 * 8 + cr) * CW + (mx % GC) * 8 + c4, db_ld4a4(&w.c[c2][cr + 2][c4 + 2]));
                }
                if (last) {  // the row's last MB: its rows are final now
                    wave_sync();
                    flush_bl(mx - mx % GL, mx % GL + 1);
                    flush_bc(mx - mx % GC, mx % GC + 1);
                }
                // line buffer for the row below: the MB's bottom rows (columns final so far) and the
                // previous MB's last columns, which this MB's left edge has just finished
                if (to_band) {  // into the boundary buffer of the band below
                    uint16_t* X = reinterpret_cast<uint16_t*>(arena + o_xout);
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int e = hl + 32 * j, tr = e >> 4, tc = e & 15;
                        if (tc < 12 || last)
                            __hip_atomic_store(X + tr * width + mx * 16 + tc, w.y[tr + 16][tc + 4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (mx > 0 && hl < 16) {
                        const int tr = hl >> 2, tc = hl & 3;
                        __hip_atomic_store(X + tr * width + mx * 16 - 4 + tc, w.y[tr + 16][tc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    {
                        const int c2 = hl >> 4, cr = (hl >> 3) & 1, k2 = hl & 7;
                        uint16_t* XC = X + 4 * width + (c2 * 2 + cr) * cw + mx * 8;
                        if (k2 < 6 || last)
                            __hip_atomic_store(XC + k2, w.c[c2][cr + 8][k2 + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (mx > 0 && k2 < 2)
                            __hip_atomic_store(XC - 2 + k2, w.c[c2][cr + 8][k2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): picture and boundary stores have completed
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (hl == 0)
                        __hip_atomic_store(reinterpret_cast<uint32_t*>(arena + o_flag) + 4 * (row * mbw),
                                           static_cast<uint32_t>(mbw + mx + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if (row + 1 < mbh) {
                    {
                        const int tr = hl >> 3, tc = (hl & 7) * 2;  // rows 12..15 of this MB, 2 per lane
                        if (tc < 12 || last) db_put_line2(LY + m24(tr, width) + mx * 16 + tc, db_u16pair(&w.y[tr + 16][tc + 4]));
                    }
                    if (mx > 0 && hl < 8) {
                        const int tr = hl >> 1, tc = (hl & 1) * 2;
                        db_put_line2(LY + m24(tr, width) + mx * 16 - 4 + tc, db_u16pair(&w.y[tr + 16][tc]));
                    }
                    const int c2 = hl >> 4, cr = (hl >> 3) & 1, k2 = hl & 7;  // chroma rows 6..7
                    if (k2 < 6 || last) LC[m24(c2 * 2 + cr, cw) + mx * 8 + k2] = static_cast<Line>(w.c[c2][cr + 8][k2 + 2]);
                    if (mx > 0 && k2 < 2) LC[m24(c2 * 2 + cr, cw) + mx * 8 - 2 + k2] = static_cast<Line>(w.c[c2][cr + 8][k2]);
                }
                wave_sync();
                {  // carry the last columns into the next MB's left strip
                    const int r = hl >> 1, k2 = (hl & 1) * 2;
                    db_put_u16pair(&w.y[r + 4][k2], db_u16pair(&w.y[r + 4][k2 + 16]));
                    const int c2 = hl >> 4, r2 = (hl >> 1) & 7, k = hl & 1;
                    w.c[c2][r2 + 2][k] = w.c[c2][r2 + 2][k + 8];
                }
                if constexpr (GLine) __builtin_amdgcn_s_waitcnt(0x0F70);  // global line buffer stores done
                wave_sync();
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0 && two && s >= kDbLag)
                __hip_atomic_store(mine, ((static_cast<uint32_t>(r0) + 2) << 16) | static_cast<uint32_t>(s - kDbLag + 1),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            DBP_LAP(3);
            DBP_ADD(6, 1 + (two && s >= kDbLag && s - kDbLag < mbw ? 1 : 0) - (s < mbw ? 0 : 1));
        }
    }
    DBP_FLUSH();
}

// line_w: the widest picture whose line buffer the launch's LDS holds (wider: global memory)
// ---- H.264 K2 for MBAFF frames (8.7 with MbaffFrameFlag 1; FFmpeg h264_loopfilter.c behind
// /root/reference/src/Decoder.cpp:324), on the picture in global memory.  Wave w walks pair rows
// w, w + kDbPairWaves, ...; a pair starts once the pair row above has finished through the pair to
// its right (its top edges read and change rows that pair's left edge changes).  Per MB (top, then
// bottom) in 8.7 order: luma vertical edges, luma horizontal edges, chroma vertical, chroma
// horizontal, one lane per line.  Geometry as in the oracle: vertical edges run along picture rows
// (the p side of a left MB edge is the left pair's MB holding that picture row); horizontal edges
// step through the MB's own rows (field MB: every other picture row) and its top MB edge reaches
// up the same way; a frame top MB under a field pair filters its top edge twice, once per field
// (bS 3).  All-intra bS: 4 on vertical MB edges and on horizontal MB edges between two frame MBs,
// else 3.
template <typename Pel>
DEVI void db264_mbaff_line(Pel* q, int step, int bs, int alpha, int beta, int tc0, bool chroma, int maxv) {
    const int p0 = q[-step], p1 = q[-2 * step], q0 = q[0], q1 = q[step];
    if (!(abs(p0 - q0) < alpha && abs(p1 - p0) < beta && abs(q1 - q0) < beta)) return;
    if (chroma) {
        if (bs < 4) {
            const int tc = tc0 + 1, dl = clip3(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
            q[-step] = static_cast<Pel>(clip3(0, maxv, p0 + dl));
            q[0] = static_cast<Pel>(clip3(0, maxv, q0 - dl));
        } else {
            q[-step] = static_cast<Pel>((2 * p1 + p0 + q1 + 2) >> 2);
            q[0] = static_cast<Pel>((2 * q1 + q0 + p1 + 2) >> 2);
        }
        return;
    }
    const int p2 = q[-3 * step], q2 = q[2 * step];
    const int ap = abs(p2 - p0), aq = abs(q2 - q0);
    if (bs < 4) {
        const int tc = tc0 + (ap < beta) + (aq < beta), dl = clip3(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
        q[-step] = static_cast<Pel>(clip3(0, maxv, p0 + dl));
        q[0] = static_cast<Pel>(clip3(0, maxv, q0 - dl));
        if (ap < beta) q[-2 * step] = static_cast<Pel>(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 * 2)) >> 1));
        if (aq < beta) q[step] = static_cast<Pel>(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 * 2)) >> 1));
        return;
    }
    const int p3 = q[-4 * step], q3 = q[3 * step];
    const bool strong = abs(p0 - q0) < ((alpha >> 2) + 2);
    if (ap < beta && strong) {
        q[-step] = static_cast<Pel>((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
        q[-2 * step] = static_cast<Pel>((p2 + p1 + p0 + q0 + 2) >> 2);
        q[-3 * step] = static_cast<Pel>((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
    } else {
        q[-step] = static_cast<Pel>((2 * p1 + p0 + q1 + 2) >> 2);
    }
    if (aq < beta && strong) {
        q[0] = static_cast<Pel>((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
        q[step] = static_cast<Pel>((p0 + q0 + q1 + q2 + 2) >> 2);
        q[2 * step] = static_cast<Pel>((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
    } else {
        q[0] = static_cast<Pel>((2 * q1 + q0 + p1 + 2) >> 2);
    }
}

template <typename Pel>
DEVI void h264_db_mbaff(const h2j_frame& f, const h2j_ctb* C, const h2j_slice* SL, uint8_t* arena, uint32_t* prog) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int kSlots = 2 * kDbPairWaves;
    const int mbw = ufl(f.ctb_w), npr = ufl(f.ctb_h) >> 1;
    const int bdy = ufl(f.bit_depth), bdc = ufl(f.bit_depth_c), qpbdc = 6 * (bdc - 8);
    const int sty = ufl(f.pic_stride[0]), stc = ufl(f.pic_stride[1]);
    Pel* PL[3] = {reinterpret_cast<Pel*>(arena + ufl64(f.pic)), nullptr, nullptr};
    PL[1] = PL[0] + ufl(f.pic_off[1]);
    PL[2] = PL[0] + ufl(f.pic_off[2]);
    auto qpf = [&](const h2j_ctb& m) { return (m.mbflags & 1) ? 0 : static_cast<int>(m.qp); };  // I_PCM: 0
    auto cqp = [&](int qpy, int off) {
        const int qi = clip3(-qpbdc, 51, qpy + off);
        return qi < 30 ? qi : kChromaQp264[qi - 30];
    };
    for (int pr = w; pr < npr; pr += kDbPairWaves) {
        uint32_t* above = prog + (pr + kSlots - 1) % kSlots;
        uint32_t* mine = prog + pr % kSlots;
        uint32_t seen = 0;
        for (int x = 0; x < mbw; x++) {
            if (pr > 0) {
                const uint32_t need = (static_cast<uint32_t>(pr) << 16) | static_cast<uint32_t>(min(x + 2, mbw));
                if (seen < need) seen = wait_progress(above, need, dev_error_word(arena, f), kDevErrDbRow264);
            }
            for (int bot = 0; bot < 2; bot++) {
                const h2j_ctb m = C[(2 * pr + bot) * mbw + x];
                if (!(m.mbflags & 4)) continue;  // not decoded
                const h2j_slice sl = SL[m.slice];
                if (sl.deblock_disabled == 1) continue;
                const bool fld = (m.mbflags & 8) != 0, t8 = (m.mbflags & 2) != 0;
                // slice tests on the neighbour of a field MB's own parity (a PAFF pair's fields are
                // separate slices; an MBAFF pair's MBs share one)
                const int par = fld ? bot : 0;
                bool left = x > 0;
                if (left) {
                    const h2j_ctb& L = C[(2 * pr + par) * mbw + x - 1];
                    left = (L.mbflags & 4) && !(sl.deblock_disabled == 2 && SL[L.slice].slice_addr_rs != sl.slice_addr_rs);
                }
                bool top;
                if (!fld && bot) top = true;  // the pair's internal edge
                else if (pr == 0) top = false;
                else {
                    const h2j_ctb& B = C[(2 * pr - 2 + par) * mbw + x];
                    top = (B.mbflags & 4) && !(sl.deblock_disabled == 2 && SL[B.slice].slice_addr_rs != sl.slice_addr_rs);
                }
                const bool above_fld = pr > 0 && (C[(2 * pr - 2) * mbw + x].mbflags & 8);
                for (int c = 0; c < 3; c += (c == 0 ? 1 : 2)) {  // luma, then both chroma components per pass
                    const int S = c ? 8 : 16, Y0 = pr * 2 * S;
                    const int bd = c ? bdc : bdy, maxv = (1 << bd) - 1;
                    // this lane's component and line
                    const int cc = c ? 1 + (lane >> 3) : 0, k = c ? (lane & 7) : lane;
                    const bool act = lane < 16;
                    const int st = cc ? stc : sty;
                    Pel* P0 = PL[cc];
                    const int off = cc == 1 ? sl.cqp_offset[0] : sl.cqp_offset[1];
                    auto row = [&](int r) { return fld ? Y0 + 2 * r + bot : Y0 + S * bot + r; };
                    auto edge = [&](Pel* q, int step, int bs, const h2j_ctb& Pm) __attribute__((always_inline)) {
                        const int qa = cc ? (cqp(qpf(Pm), off) + cqp(qpf(m), off) + 1) >> 1 : (qpf(Pm) + qpf(m) + 1) >> 1;
                        const int ia = clip3(0, 51, qa + sl.tc_offset), ib = clip3(0, 51, qa + sl.beta_offset);
                        const int alpha = kAlpha264[ia] << (bd - 8), beta = kBeta264[ib] << (bd - 8);
                        const int tc0 = bs < 4 ? kTc0_264[ia][bs - 1] << (bd - 8) : 0;
                        db264_mbaff_line<Pel>(q, step, bs, alpha, beta, tc0, cc != 0, maxv);
                    };
                    auto sync = [&]() __attribute__((always_inline)) {  // this pass's stores before the next pass's loads
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                        wave_sync();
                    };
                    for (int e = 0; e < S; e += 4) {  // vertical edges
                        if (!c && (e == 4 || e == 12) && t8) continue;
                        if (e == 0 && !left) continue;
                        if (act) {
                            const int Y = row(k);
                            const h2j_ctb* Pm = &m;
                            if (e == 0) {
                                const bool lf = (C[(2 * pr) * mbw + x - 1].mbflags & 8) != 0;
                                const int r = Y - Y0, lb = lf ? (r & 1) : (r >= S ? 1 : 0);
                                Pm = &C[(2 * pr + lb) * mbw + x - 1];
                            }
                            edge(P0 + Y * st + x * S + e, 1, e == 0 ? 4 : 3, *Pm);
                        }
                        sync();
                    }
                    for (int e = 0; e < S; e += 4) {  // horizontal edges
                        if (!c && (e == 4 || e == 12) && t8) continue;
                        if (e == 0 && !top) continue;
                        const int Yq = row(e);
                        if (e == 0 && !fld && !bot && above_fld) {  // twice, once per field of the pair above
                            for (int j = 0; j < 2; j++) {
                                if (act) edge(P0 + (Yq + j) * st + x * S + k, 2 * st, 3, C[(2 * pr - 2 + j) * mbw + x]);
                                sync();
                            }
                            continue;
                        }
                        if (act) {
                            const h2j_ctb* Pm = &m;
                            int bs = 3;
                            if (e == 0) {
                                if (!fld && bot) {
                                    Pm = &C[(2 * pr) * mbw + x];
                                } else {
                                    const int r = Yq - (fld ? 2 : 1) - (Y0 - 2 * S), ab = above_fld ? (r & 1) : (r >= S ? 1 : 0);
                                    Pm = &C[(2 * pr - 2 + ab) * mbw + x];
                                }
                                bs = (!fld && !(Pm->mbflags & 8)) ? 4 : 3;
                            }
                            edge(P0 + Yq * st + x * S + k, fld ? 2 * st : st, bs, *Pm);
                        }
                        sync();
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0)
                __hip_atomic_store(mine, ((static_cast<uint32_t>(pr) + 1) << 16) | static_cast<uint32_t>(x + 1),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// One kernel per sample type (its window and LDS line sizes differ: the 8-bit one fits two
// workgroups per CU) and one for MBAFF frames (no windows: its LDS is the progress words); each
// skips the pictures of the others.  Launched for the kinds present (h2j_gpu_batch.h264_pels).
// kWide: the pictures wider than the launch's LDS line (line_w) with their line buffer in global
// memory; the LDS-line launch sizes its line for two workgroups per CU at 8 bits, so a batch with
// 4K pictures does not drop every picture's deblocking to one workgroup per CU.
template <typename Pel, bool kWide>
__global__ void __launch_bounds__(64 * kDbPairWaves) h2j_k2_deblock264p(const h2j_frame* frames, const h2j_ctb* ctbs,
                                                                      const h2j_slice* slices, uint8_t* arena,
                                                                      const uint32_t* map, int line_w) {
    // LDS: windows (two per wave) | progress | tables | line buffer (h2j_gpu_deblock)
    extern __shared__ __align__(16) uint8_t dblds[];
    DbWin<Pel>* W = reinterpret_cast<DbWin<Pel>*>(dblds);
    uint32_t* prog = reinterpret_cast<uint32_t*>(dblds + sizeof(DbWin<Pel>) * 2 * kDbPairWaves);
    DbTables& TB = *reinterpret_cast<DbTables*>(dblds + sizeof(DbWin<Pel>) * 2 * kDbPairWaves + kDbPairSlots * 4);
    Pel* line = reinterpret_cast<Pel*>(reinterpret_cast<uint8_t*>(&TB) + sizeof(DbTables));
    const uint32_t me = map[blockIdx.x];  // same (picture, band) map as K1
    const h2j_frame& f = frames[me >> 8];
    const int band = static_cast<int>(me & 0xFF);
    if (f.codec != H2J_CODEC_H264 || ufl(f.mbaff) || (ufl(f.bit_depth) == 8) != (sizeof(Pel) == 1)) return;
    if ((static_cast<int>(ufl(f.width)) > line_w) != kWide) return;  // the other launch's picture
    const int nbands = ufl(f.k1bands);
    const h2j_ctb* C = ctbs + f.ctb;
    const h2j_slice* S = slices + f.slice;
    const int t = threadIdx.x;
    if (t < kDbPairSlots) prog[t] = 0;
    if (t < 52) {
        TB.alpha[t] = kAlpha264[t];
        TB.beta[t] = kBeta264[t];
        TB.tc0[t] = kTc0_264[t][2];
    }
    if (t < 22) TB.cqp[t] = kChromaQp264[t];
    const int nsl = min(static_cast<int>(ufl(f.nslice)), kDbSlices);
    if (t < nsl * static_cast<int>(sizeof(h2j_slice) / 4))
        reinterpret_cast<uint32_t*>(TB.sl)[t] = reinterpret_cast<const uint32_t*>(S)[t];
    __syncthreads();
    if constexpr (!kWide) {
        h264_db_pairs<Pel, false>(f, C, S, arena, W, prog, line, band, nbands, TB);
    } else {  // one line buffer per band in the picture's residual region (12 bytes per column)
        uint16_t* gl = reinterpret_cast<uint16_t*>(arena + ufl64(f.res)) + static_cast<size_t>(band) * 6 * ufl(f.width);
        h264_db_pairs<Pel, true>(f, C, S, arena, W, prog, gl, band, nbands, TB);
    }
}

// MBAFF frames (one workgroup per picture: h2j_frame.k1bands 1)
__global__ void __launch_bounds__(64 * kDbPairWaves) h2j_k2_deblock264m(const h2j_frame* frames, const h2j_ctb* ctbs,
                                                                      const h2j_slice* slices, uint8_t* arena,
                                                                      const uint32_t* map) {
    __shared__ uint32_t prog[kDbPairSlots];
    const h2j_frame& f = frames[map[blockIdx.x] >> 8];
    if (f.codec != H2J_CODEC_H264 || !ufl(f.mbaff)) return;
    const h2j_ctb* C = ctbs + f.ctb;
    const h2j_slice* S = slices + f.slice;
    if (threadIdx.x < kDbPairSlots) prog[threadIdx.x] = 0;
    __syncthreads();
    if (ufl(f.bit_depth) == 8) h264_db_mbaff<uint8_t>(f, C, S, arena, prog);
    else h264_db_mbaff<uint16_t>(f, C, S, arena, prog);
}

// ---------------------------------------------------------------- K3: SAO
// K3 SAO (H.265 8.7.3): one 256-thread workgroup per CTB, all three components.  Every load of
// the CTB is issued before the first LDS write (the deblocked samples of Y, Cb and Cr plus a
// one-sample border, 4 samples per load; the border columns; the per-4x4 "loop filters off"
// flags), so a workgroup waits for HBM once instead of once per loop iteration.  Samples are
// staged as int16 (-1 = outside the picture) in LDS tiles whose interior starts at column 4
// (8-byte aligned rows).  The CTB's SAO parameters and the usability of its 8 neighbour CTBs
// across slice / tile boundaries are resolved once; each thread then filters 4 horizontally
// adjacent samples per step and writes them with one store.  Pictures without SAO alias
// pic2 = pic and are skipped (the host lays them out that way).
constexpr int kSaoTsY = 72, kSaoTsC = 40;  // LDS tile row strides (int16): 4 + 64 + 4, 4 + 32 + 4
struct SaoLds {
    int16_t y[66 * kSaoTsY];
    int16_t c[2][34 * kSaoTsC];
    uint8_t keep[256];  // per 4x4 luma block of the CTB: pcm / transquant bypass with loop filters off
    uint32_t nbm;       // usable neighbour CTBs (sao_stage_store)
    unsigned long long var[16];  // K4a's per-MB sums of the CTB's final luma: (sum << 32) | sum of squares
};

// K4a's macroblock variances (the JPEG rate control input) are summed by K3 from the SAO output
// it holds in registers, when the output's 16x16 MB grid is aligned with the CTB grid; K4a then
// skips the picture (one full read of the final picture less).
DEVI bool sao_sums_variance(const h2j_frame& f, int fold) { return fold && h2j_sao_folds_variance(f); }

template <typename Pel>
DEVI uint2 sao_load4(const Pel* p) {  // 4 samples -> 4 int16 halves of a uint2
    if (sizeof(Pel) == 1) {
        const uint32_t v = *reinterpret_cast<const uint32_t*>(p);
        return make_uint2((v & 0xFFu) | ((v & 0xFF00u) << 8), ((v >> 16) & 0xFFu) | ((v >> 8) & 0xFF0000u));
    }
    return *reinterpret_cast<const uint2*>(p);
}

// geometry of component c of a CTB
struct SaoGeo {
    int S, x0, y0, w, h, pw, ph, lq, ts;  // lq: log2 of 4-sample chunks per CTB row; ts: tile stride
};
DEVI SaoGeo sao_geo(const h2j_frame& f, int ctb, int c) {
    const int sh = c ? 1 : 0;
    const int l2 = f.log2ctb, CS = 1 << l2;
    const int cxi = ctb % f.ctb_w, cyi = ctb / f.ctb_w;
    SaoGeo g;
    g.S = CS >> sh;
    g.x0 = (cxi * CS) >> sh;
    g.y0 = (cyi * CS) >> sh;
    g.pw = f.width >> sh;
    g.ph = f.height >> sh;
    g.w = min(g.S, g.pw - g.x0);
    g.h = min(g.S, g.ph - g.y0);
    g.lq = l2 - 2 - sh;
    g.ts = c ? kSaoTsC : kSaoTsY;
    return g;
}

// stage loads of component c: interior chunks (rows -1 .. h of the CTB) and the two border
// columns, held in registers until every load of the CTB is in flight
template <typename Pel, int NI>
DEVI void sao_stage_load(const h2j_frame& f, uint8_t* arena, const SaoGeo& g, int c, uint2 (&iv)[NI], int16_t& bv) {
    const int tid = threadIdx.x;
    const Pel* P = plane<Pel>(f, arena, f.pic, c);
    const int st = f.pic_stride[c];
#pragma unroll
    for (int k = 0; k < NI; k++) {
        const int i = tid + 256 * k, r = i >> g.lq, ch = i & ((1 << g.lq) - 1);
        const int y = g.y0 + r - 1, x = g.x0 + 4 * ch;
        iv[k] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        if (r < g.h + 2 && 4 * ch < g.w && y >= 0 && y < g.ph) iv[k] = sao_load4(at32(P, m24(y, st) + x));
    }
    const int r = tid >> 1, x = (tid & 1) ? g.x0 + g.w : g.x0 - 1, y = g.y0 + r - 1;
    bv = -1;
    if (r < g.h + 2 && x >= 0 && x < g.pw && y >= 0 && y < g.ph) bv = static_cast<int16_t>(*at32(P, m24(y, st) + x));
}
template <int NI>
DEVI void sao_stage_store(const SaoGeo& g, int16_t* T, const uint2 (&iv)[NI], int16_t bv) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < NI; k++) {
        const int i = tid + 256 * k, r = i >> g.lq, ch = i & ((1 << g.lq) - 1);
        if (r < g.h + 2) *reinterpret_cast<uint2*>(T + r * g.ts + 4 + 4 * ch) = iv[k];
    }
    const int r = tid >> 1;
    if (r < g.h + 2) T[r * g.ts + ((tid & 1) ? 4 + g.w : 3)] = bv;
}
// The staged rows -1 and h and the border columns belong to the 8 neighbour CTBs; samples of a
// neighbour that may not be used across a slice / tile boundary (bit (dy + 1) * 3 + dx + 1 of
// nbm clear) are overwritten with -1, like samples outside the picture (8.7.3.2: the edge
// offset then leaves the sample unmodified).  Only CTBs at such boundaries take this pass.
DEVI void sao_stage_mask(const SaoGeo& g, int16_t* T, uint32_t nbm) {
    const int tid = threadIdx.x;
    auto usable = [&](int r, int dx) __attribute__((always_inline)) {
        const int dy = r == 0 ? -1 : (r == g.h + 1 ? 1 : 0);
        return ((nbm >> ((dy + 1) * 3 + dx + 1)) & 1u) != 0;
    };
    if (tid < 2 * g.w) {  // rows -1 and h
        const int r = tid < g.w ? 0 : g.h + 1, x = tid < g.w ? tid : tid - g.w;
        if (!usable(r, 0)) T[r * g.ts + 4 + x] = -1;
    }
    const int r = tid >> 1, dx = (tid & 1) ? 1 : -1;
    if (r < g.h + 2 && !usable(r, dx)) T[r * g.ts + ((tid & 1) ? 4 + g.w : 3)] = -1;
}

// filter component c (uniform: its SAO parameters sit in scalar registers)
template <typename Pel>
DEVI void sao_filter(const h2j_frame& f, uint8_t* arena, const SaoGeo& g, int c, const h2j_ctb& cc, bool on,
                     const int16_t* T, const SaoLds& L, unsigned long long* vacc = nullptr) {
    const int tid = threadIdx.x;
    Pel* D = plane<Pel>(f, arena, f.pic2, c);
    const int st = f.pic_stride[c];
    const int type = on ? cc.type[c] : 0;
    const int bd = c ? f.bit_depth_c : f.bit_depth;
    const int maxv = (1 << bd) - 1;
    const int cls = cc.eo_class[c], band = cc.band_pos[c];
    const int o0 = cc.off[c][0], o1 = cc.off[c][1], o2 = cc.off[c][2], o3 = cc.off[c][3];
    const int hx = cls == 0 ? -1 : (cls == 1 ? 0 : (cls == 2 ? -1 : 1));
    const int vy = cls == 0 ? 0 : -1;
    const int sh = c ? 1 : 0, l2b = f.log2ctb - 2;
    const int ts = g.ts;
    // |SaoOffsetVal| <= 31 without range extensions: the packed forms below; else the select form
    const bool packed = max(max(abs(o0), abs(o1)), max(abs(o2), abs(o3))) <= 31;
    const int da = vy * ts + hx;  // element offset of neighbour a (b is at -da)
    // packed forms (r06): two samples per instruction as int16 halves (v_pk_* ops); the offset of a
    // sample picked by v_perm_b32 from a byte table of offset + 64 (high byte of each half 0x00),
    // edge index (sa + sb) & 7 = 6, 7, 0, 1, 2 for edgeIdx 0..4, band index min(band delta, 4)
    const auto b64 = [](int v) { return static_cast<uint32_t>(v + 64) & 0xFFu; };
    const uint32_t eo_lo = 64u | (b64(o2) << 8) | (b64(o3) << 16), eo_hi = (b64(o0) << 16) | (b64(o1) << 24);
    const uint32_t bo_lo = b64(o0) | (b64(o1) << 8) | (b64(o2) << 16) | (b64(o3) << 24), bo_hi = 64u;
    const s16x2 k64 = {64, 64}, kmax = {static_cast<short>(maxv), static_cast<short>(maxv)}, kzero = {0, 0};
    const auto h2 = [](uint32_t v) { return __builtin_bit_cast(s16x2, v); };
    const auto u2 = [](s16x2 v) { return __builtin_bit_cast(uint32_t, v); };
    const auto apply = [&](uint32_t v, uint32_t t) __attribute__((always_inline)) {  // clip(v + t - 64)
        const s16x2 r = h2(v) + h2(t) - k64;
        return u2(__builtin_elementwise_min(__builtin_elementwise_max(r, kzero), kmax));
    };
    // (the sign clamps and the sentinel shift as v_pk_max/min/ashr by asm: the compiler turns the
    // C form into per-half compares and selects)
    const auto sgn2 = [](uint32_t d) __attribute__((always_inline)) {  // clamp(d, -1, 1) per int16 half
        uint32_t r;
        asm("v_pk_max_i16 %0, %1, %2\n\tv_pk_min_i16 %0, %0, %3" : "=&v"(r) : "v"(d), "s"(0xFFFFFFFFu), "s"(0x00010001u));
        return r;
    };
    const auto eo2 = [&](uint32_t v, uint32_t a, uint32_t b) __attribute__((always_inline)) {
        const uint32_t sa = sgn2(u2(h2(v) - h2(a))), sb = sgn2(u2(h2(v) - h2(b)));
        const uint32_t t = __builtin_amdgcn_perm(eo_hi, eo_lo, (u2(h2(sa) + h2(sb)) & 0x00070007u) | 0x0C000C00u);
        uint32_t inv;  // 0xFFFF in a half whose a or b is -1 (unusable): that sample keeps v
        asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(inv) : "s"(0x000F000Fu), "v"(a | b));
        return (inv & v) | (~inv & apply(v, t));
    };
    const auto bo2 = [&](uint32_t v) __attribute__((always_inline)) {
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const u16x2 d = __builtin_bit_cast(u16x2, u2((h2(v) >> static_cast<short>(bd - 5)) - h2(0x00010001u * static_cast<uint32_t>(band))) & 0x001F001Fu);
        const u16x2 four = {4, 4};
        const uint32_t bi = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(d, four));
        return apply(v, __builtin_amdgcn_perm(bo_hi, bo_lo, bi | 0x0C000C00u));
    };
    for (int i = tid; i < (g.h << g.lq); i += 256) {
        const int y = i >> g.lq, x = (i & ((1 << g.lq) - 1)) * 4;
        if (x >= g.w) continue;
        const uint2 vv = *reinterpret_cast<const uint2*>(T + (y + 1) * ts + 4 + x);
        // samples of pcm (loop filter off) / transquant-bypass blocks stay untouched
        const bool keep = type == 0 || L.keep[(((y << sh) >> 2) << l2b) + ((x << sh) >> 2)] != 0;
        uint32_t px, py;  // the four output samples as int16 pairs
        if (type == 2 && packed) {  // edge offset, packed
            const int16_t* C0 = T + (y + 1) * ts + 4 + x;
            uint2 av, bv;
            __builtin_memcpy(&av, C0 + da, 8);
            __builtin_memcpy(&bv, C0 - da, 8);
            px = eo2(vv.x, av.x, bv.x);
            py = eo2(vv.y, av.y, bv.y);
            if (keep) { px = vv.x; py = vv.y; }
        } else if (type == 1 && packed) {  // band offset, packed
            px = bo2(vv.x);
            py = bo2(vv.y);
            if (keep) { px = vv.x; py = vv.y; }
        } else {
            const int v[4] = {static_cast<int>(vv.x & 0xFFFF), static_cast<int>(vv.x >> 16), static_cast<int>(vv.y & 0xFFFF),
                              static_cast<int>(vv.y >> 16)};
            int o[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                int sel = -1;  // offset index 0..3, -1 none
                if (type == 1) {
                    const int b = ((v[k] >> (bd - 5)) - band) & 31;
                    sel = b < 4 ? b : -1;
                } else if (type == 2) {
                    const int xa = x + k + hx, ya = y + vy, xb = x + k - hx, yb = y - vy;
                    const int a = T[(ya + 1) * ts + 4 + xa], bb = T[(yb + 1) * ts + 4 + xb];
                    if (a >= 0 && bb >= 0) {
                        const int e = 2 + ((v[k] > a) - (v[k] < a)) + ((v[k] > bb) - (v[k] < bb));
                        // edgeIdx 0, 1, 2, 3, 4 -> category 1, 2, 0, 3, 4 -> offset index 0, 1, -, 2, 3
                        sel = e == 0 ? 0 : (e == 1 ? 1 : (e == 2 ? -1 : e - 1));
                    }
                }
                const int off = sel == 0 ? o0 : (sel == 1 ? o1 : (sel == 2 ? o2 : (sel == 3 ? o3 : 0)));
                o[k] = keep ? v[k] : clip3(0, maxv, v[k] + off);
            }
            px = static_cast<uint32_t>(o[0]) | (static_cast<uint32_t>(o[1]) << 16);
            py = static_cast<uint32_t>(o[2]) | (static_cast<uint32_t>(o[3]) << 16);
        }
        if (vacc) {  // luma of a sao_sums_variance picture: K4a's sums, per MB of the CTB
            // output rows below the picture repeat its last row (jpeg_sample), so that row counts
            // for them too; rows / columns outside the output (above / left of the crop window too) count 0
            const int oy = g.y0 + y - f.crop_y, ox = g.x0 + x - f.crop_x, last = f.out_h - 1;
            const unsigned wgt = (oy < 0 || ox < 0 || ox >= f.out_w) ? 0u : (oy < last ? 1u : (oy == last ? 16u - (last & 15) : 0u));
            if (wgt) {
                unsigned s4 = 0, n4 = 0;
                if (bd == 8) {  // sums and squares of the int16 pairs by v_dot2
                    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
                    const u16x2 ux = __builtin_bit_cast(u16x2, px), uy = __builtin_bit_cast(u16x2, py), one = {1, 1};
                    s4 = __builtin_amdgcn_udot2(uy, one, __builtin_amdgcn_udot2(ux, one, 0u, false), false);
                    n4 = __builtin_amdgcn_udot2(uy, uy, __builtin_amdgcn_udot2(ux, ux, 0u, false), false);
                } else {
                    const int o[4] = {static_cast<int>(px & 0xFFFF), static_cast<int>(px >> 16), static_cast<int>(py & 0xFFFF),
                                      static_cast<int>(py >> 16)};
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const unsigned u = min(static_cast<unsigned>(o[k] + (1 << (bd - 9))) >> (bd - 8), 255u);
                        s4 += u;
                        n4 += u * u;
                    }
                }
                atomicAdd(&vacc[((y >> 4) << (f.log2ctb - 4)) + (x >> 4)],
                          (static_cast<unsigned long long>(s4 * wgt) << 32) | (n4 * wgt));
            }
        }
        Pel* d = at32(D, m24(g.y0 + y, st) + g.x0 + x);
        if (sizeof(Pel) == 1) *reinterpret_cast<uint32_t*>(d) = __builtin_amdgcn_perm(py, px, 0x06040200u);
        else *reinterpret_cast<uint2*>(d) = make_uint2(px, py);
    }
}

// staged loads of one CTB (registers), written to LDS once the previous CTB is filtered
struct SaoRegs {
    uint2 iy[5], ib[2], ir[2];  // (66 x 16) and 2 x (34 x 8) 4-sample chunks over 256 threads
    int16_t by, bb, br;
    uint8_t kf;
};
template <typename Pel>
DEVI void sao_load(const h2j_frame& f, uint8_t* arena, int ctb, SaoRegs& R) {
    const int tid = threadIdx.x;
    const SaoGeo gy = sao_geo(f, ctb, 0), gb = sao_geo(f, ctb, 1), gr = sao_geo(f, ctb, 2);
    sao_stage_load<Pel>(f, arena, gy, 0, R.iy, R.by);
    sao_stage_load<Pel>(f, arena, gb, 1, R.ib, R.bb);
    sao_stage_load<Pel>(f, arena, gr, 2, R.ir, R.br);
    R.kf = 0;
    const int lb = f.log2ctb - 2, bY = tid >> lb, bX = tid & ((1 << lb) - 1);
    const int gyy = (gy.y0 >> 2) + bY, gxx = (gy.x0 >> 2) + bX;
    if (bY < (1 << lb) && gxx < f.mw && gyy < f.mh) R.kf = arena[f.maps + static_cast<size_t>(gyy) * f.mw + gxx] & 4;
}

// usability of neighbour CTB (dx, dy) = (k % 3 - 1, k / 3 - 1) of CTB (cx, row) for SAO across
// slice / tile boundaries (8.7.3.2); outside the picture counts as usable (those samples are
// staged as -1 anyway)
DEVI bool sao_nb_ok(const h2j_frame& f, const h2j_ctb* C, const h2j_slice* SL, int cx, int row, int k) {
    const int dx = k % 3 - 1, dy = k / 3 - 1;
    const int nx = cx + dx, ny = row + dy;
    if (nx < 0 || ny < 0 || nx >= f.ctb_w || ny >= f.ctb_h || (dx == 0 && dy == 0)) return true;
    const h2j_ctb& cc = C[row * f.ctb_w + cx];
    const h2j_ctb& nc = C[ny * f.ctb_w + nx];
    const h2j_slice& sc = SL[cc.slice];
    const h2j_slice& sn = SL[nc.slice];
    bool ok = true;
    if (sn.slice_addr_rs != sc.slice_addr_rs) {
        if (nc.ts < cc.ts && !sc.lf_across_slices) ok = false;
        if (cc.ts < nc.ts && !sn.lf_across_slices) ok = false;
    }
    if (!f.lf_across_tiles && nc.tile != cc.tile) ok = false;
    return ok;
}

// one CTB (Y, Cb, Cr) per workgroup
template <typename Pel>
DEVI void sao_ctb(const h2j_frame& f, const h2j_ctb* C, const h2j_slice* SL, uint8_t* arena, int ctb, SaoLds& L, int fold) {
    const int tid = threadIdx.x;
    const int cx = ctb % f.ctb_w, row = ctb / f.ctb_w;
    const h2j_ctb cc = uload(C + ctb);
    const h2j_slice sc = uload(SL + cc.slice);
    const bool onY = cc.type[0] != 0 && sc.sao_luma, onC = sc.sao_chroma;
    const bool onCb = onC && cc.type[1] != 0, onCr = onC && cc.type[2] != 0;
    const bool eo = (onY && cc.type[0] == 2) || (onCb && cc.type[1] == 2) || (onCr && cc.type[2] == 2);
    const SaoGeo gy = sao_geo(f, ctb, 0), gb = sao_geo(f, ctb, 1), gr = sao_geo(f, ctb, 2);
    // 1. every load of the CTB in flight at once
    SaoRegs R;
    sao_load<Pel>(f, arena, ctb, R);
    // one slice from CTB 0 and one tile (frame.topo 0): every neighbour CTB is usable, no record loads
    const bool nok = !eo || tid >= 9 || !f.topo || sao_nb_ok(f, C, SL, cx, row, tid);
    // 2. LDS
    if (tid < 64) {
        const uint64_t m = __ballot(tid < 9 && nok);
        if (tid == 0) L.nbm = static_cast<uint32_t>(m & 0x1FFu);
    }
    sao_stage_store(gy, L.y, R.iy, R.by);
    sao_stage_store(gb, L.c[0], R.ib, R.bb);
    sao_stage_store(gr, L.c[1], R.ir, R.br);
    L.keep[tid] = R.kf;
    const bool var = sao_sums_variance(f, fold);
    if (tid < 16) L.var[tid] = 0;
    __syncthreads();
    const uint32_t nbm = L.nbm;
    if (nbm != 0x1FFu) {
        sao_stage_mask(gy, L.y, nbm);
        sao_stage_mask(gb, L.c[0], nbm);
        sao_stage_mask(gr, L.c[1], nbm);
        __syncthreads();
    }
    // 3. filter and store, one component at a time
    sao_filter<Pel>(f, arena, gy, 0, cc, onY, L.y, L, var ? L.var : nullptr);
    sao_filter<Pel>(f, arena, gb, 1, cc, onCb, L.c[0], L);
    sao_filter<Pel>(f, arena, gr, 2, cc, onCr, L.c[1], L);
    if (var) {  // the CTB's MBs inside the output: K4a's formula, one atomic per CTB
        __syncthreads();
        if (tid < 64) {
            const int l2m = f.log2ctb - 4;
            unsigned long long t = 0;
            if (tid < (1 << (2 * l2m))) {
                const int oy0 = gy.y0 - f.crop_y + ((tid >> l2m) << 4), ox0 = gy.x0 - f.crop_x + ((tid & ((1 << l2m) - 1)) << 4);
                if (oy0 >= 0 && oy0 < f.out_h && ox0 >= 0 && ox0 < f.out_w) {
                    const unsigned long long a = L.var[tid];
                    const unsigned sm = static_cast<unsigned>(a >> 32), n = static_cast<unsigned>(a);
                    t = (n - ((sm * sm) >> 8) + 500 + 128) >> 8;
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
            if (tid == 0 && t) {
                h2j_jstat* js = reinterpret_cast<h2j_jstat*>(arena + f.jstat);
                atomicAdd(reinterpret_cast<unsigned long long*>(&js->var_sum), t);
            }
        }
    }
}

// grid (CTBs of the largest picture at the smallest CTB size, pictures)
// (256, 8): at least 8 waves per SIMD -- the compiler keeps the kernel to 78 SGPRs (35 of them
// spilled to VGPR lanes) instead of 104, which had held it to 7 (hevc1080 per 1024 pictures
// 4.18 -> 3.53 ms)
__global__ void __launch_bounds__(256, 8) h2j_k3_sao(const h2j_frame* __restrict__ frames,
                                                 const h2j_ctb* __restrict__ ctbs,
                                                 const h2j_slice* __restrict__ slices, uint8_t* __restrict__ arena,
                                                 int fold, const uint32_t* __restrict__ ymap) {
    const GridPos gp = xcd_grid_pos();
    __shared__ SaoLds L;
    const h2j_frame& f = frames[ymap[gp.y]];  // gp.y: picture of this launch's CTB-count class
    if (f.codec != H2J_CODEC_HEVC || f.pic2 == f.pic) return;
    const int ctb = gp.x;
    if (ctb >= f.ctb_w * f.ctb_h) return;
    const h2j_ctb* C = ctbs + f.ctb;
    const h2j_slice* S = slices + f.slice;
    if (f.bit_depth == 8) sao_ctb<uint8_t>(f, C, S, arena, ctb, L, fold);
    else sao_ctb<uint16_t>(f, C, S, arena, ctb, L, fold);
}

// ---------------------------------------------------------------- K4: JPEG
template <typename Pel>
DEVI int jpeg_sample(const h2j_frame& f, const uint8_t* arena, int c, int x, int y) {
    const int shc = c ? 1 : 0;
    const int pw = f.out_w >> shc, ph = f.out_h >> shc;
    x = x < pw ? x : pw - 1;
    y = y < ph ? y : ph - 1;
    const Pel* p = reinterpret_cast<const Pel*>(arena + f.pic2) + f.pic_off[c];
    int v = p[(y + (f.crop_y >> shc)) * f.pic_stride[c] + x + (f.crop_x >> shc)];
    const int bd = c ? f.bit_depth_c : f.bit_depth;
    if (bd > 8) {
        v = (v + (1 << (bd - 9))) >> (bd - 8);
        v = v > 255 ? 255 : v;
    }
    return v;
}


// 16 lanes per macroblock, one 16-sample row each (4 dword loads at 8 bits inside the picture,
// jpeg_sample's clamped path at the edges / above 8 bits); the row sums meet by DPP row shifts.
DEVI unsigned row16_sum(unsigned x) {  // inclusive prefix over each 16-lane row: lane 15 = total
    x += static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xf, 0xf, false));
    x += static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xf, 0xf, false));
    x += static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xf, 0xf, false));
    x += static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xf, 0xf, false));
    return x;
}
__global__ void __launch_bounds__(256) h2j_k4a_variance(const h2j_frame* __restrict__ frames, uint8_t* __restrict__ arena, int fold) {
    const h2j_frame& f = frames[blockIdx.y];
    if (sao_sums_variance(f, fold)) return;  // K3 has summed this picture's MB variances
    const int mbw = (f.out_w + 15) >> 4, mbh = (f.out_h + 15) >> 4;
    const int mb = blockIdx.x * 16 + static_cast<int>(threadIdx.x >> 4), r = threadIdx.x & 15;
    unsigned s = 0, n = 0;
    const bool live = mb < mbw * mbh;
    if (live) {
        const int mx = mb % mbw, my = mb / mbw;
        const bool inside = mx * 16 + 15 < f.out_w && (f.crop_x & 3) == 0;
        const int y = min(my * 16 + r, f.out_h - 1);
        if (inside && f.bit_depth == 8) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(arena + f.pic2 + f.pic_off[0] +
                                                                  static_cast<size_t>(y + f.crop_y) * f.pic_stride[0] +
                                                                  mx * 16 + f.crop_x);
#pragma unroll
            for (int k = 0; k < 4; k++) {  // 4 samples per v_dot4_u32_u8: the sum and the sum of squares
                const uint32_t w = p[k];
                s = __builtin_amdgcn_udot4(w, 0x01010101u, s, false);
                n = __builtin_amdgcn_udot4(w, w, n, false);
            }
        } else if (inside && f.bit_depth > 8) {  // 16-bit samples, converted as jpeg_sample does
            const uint2* p = reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(arena + f.pic2) + f.pic_off[0] +
                                                            static_cast<size_t>(y + f.crop_y) * f.pic_stride[0] +
                                                            mx * 16 + f.crop_x);
            const int bd = f.bit_depth;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint2 w = p[k];
                const uint32_t h[4] = {w.x & 0xFFFF, w.x >> 16, w.y & 0xFFFF, w.y >> 16};
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const unsigned v = min((h[b] + (1u << (bd - 9))) >> (bd - 8), 255u);
                    s += v;
                    n += v * v;
                }
            }
        } else {
            for (int i = 0; i < 16; i++) {
                const unsigned v = static_cast<unsigned>(f.bit_depth == 8 ? jpeg_sample<uint8_t>(f, arena, 0, mx * 16 + i, my * 16 + r)
                                                                          : jpeg_sample<uint16_t>(f, arena, 0, mx * 16 + i, my * 16 + r));
                s += v;
                n += v * v;
            }
        }
    }
    s = row16_sum(s);
    n = row16_sum(n);
    __shared__ long long part[16];
    if (r == 15) part[threadIdx.x >> 4] = live ? static_cast<long long>((n - ((s * s) >> 8) + 500 + 128) >> 8) : 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int k = 0; k < 16; k++) t += part[k];
        if (t) {
            h2j_jstat* js = reinterpret_cast<h2j_jstat*>(arena + f.jstat);
            atomicAdd(reinterpret_cast<unsigned long long*>(&js->var_sum), static_cast<unsigned long long>(t));
        }
    }
}

__constant__ uint8_t kMpeg1Intra[64] = {
    8,  16, 19, 22, 26, 27, 29, 34, 16, 16, 22, 24, 27, 29, 34, 37, 19, 22, 26, 27, 29, 34,
    34, 38, 22, 22, 26, 27, 29, 34, 37, 40, 22, 26, 27, 29, 32, 35, 40, 48, 26, 27, 29, 32,
    35, 40, 48, 58, 26, 27, 29, 34, 38, 46, 56, 69, 27, 29, 35, 38, 46, 56, 69, 83};
__constant__ uint8_t kZigzag[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Rate control of FFmpeg's one-pass RC for frame 0; IEEE
// double with correctly rounded sqrt/div and no contraction, as on the host.
__global__ void __launch_bounds__(64) h2j_k4b_ratecontrol(const h2j_frame* frames, uint8_t* arena) {
#pragma clang fp contract(off)
    const h2j_frame& f = frames[blockIdx.x];
    h2j_jstat* js = reinterpret_cast<h2j_jstat*>(arena + f.jstat);
    __shared__ int qs_sh;
    if (threadIdx.x == 0) {
        const double qp2l = 118.0, qs = 2.0 * 118.0;
        const long long V = js->var_sum;
        const int T = static_cast<int>(qp2l * 7.0 * __dsqrt_rn(static_cast<double>(V)) / qs);
        const double bits = __dsqrt_rn(static_cast<double>(T) * qs) + 1.0;
        double q = qs * static_cast<double>(T + 1) / (bits > 0.9 ? bits : 0.9);
        q = 0.8 * q;
        q = (0.0005 + q) / 1.0005;
        q = q < 189.0 ? 189.0 : (q > 2926.0 ? 2926.0 : q);
        const int lambda = static_cast<int>(q + 0.5);
        int qscale = (lambda * 139 + 128 * 64) >> 14;
        qscale = qscale < 2 ? 2 : (qscale > 31 ? 31 : qscale);
        js->qscale = qscale;
        js->lambda = lambda;
        qs_sh = qscale;
    }
    __syncthreads();
    const int qscale = qs_sh;
    const int i = threadIdx.x;
    int M = i == 0 ? 8 : ((kMpeg1Intra[i] * qscale) >> 3);
    M = M > 255 ? 255 : M;
    int q = (2 << 16) / (16 * M);
    if (q == 0 || q == 128 * 256) q = 128 * 256 - 1;
    js->dqt[i] = static_cast<uint8_t>(M);
    js->q16[i] = static_cast<uint16_t>(q);
    js->b16[i] = static_cast<uint16_t>((96 * 256 + (q >> 1)) / q);
}

DEVI int16_t sat16(int v) { return static_cast<int16_t>(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }
DEVI int16_t mulhi16(int a, int c) { return static_cast<int16_t>((a * c) >> 16); }

// AP-922 FDCT (ff_fdct_sse2) restated in SURVEY.md A.4, on one 8x8 block
DEVI void fdct_ap922(int16_t* b) {
    int16_t t[64];
#pragma unroll
    for (int x = 0; x < 8; x++) {
        const int x0 = b[x], x1 = b[8 + x], x2 = b[16 + x], x3 = b[24 + x], x4 = b[32 + x], x5 = b[40 + x],
                  x6 = b[48 + x], x7 = b[56 + x];
        const int16_t t0 = sat16(sat16(x0 + x7) * 8), t1 = sat16(sat16(x1 + x6) * 8);
        const int16_t t2 = sat16(sat16(x2 + x5) * 8), t3 = sat16(sat16(x3 + x4) * 8);
        const int16_t tp03 = sat16(t0 + t3), tm03 = sat16(t0 - t3), tp12 = sat16(t1 + t2), tm12 = sat16(t1 - t2);
        t[x] = sat16(tp03 + tp12);
        t[32 + x] = sat16(tp03 - tp12);
        t[16 + x] = static_cast<int16_t>(sat16(tm03 + mulhi16(tm12, 27146)) | 1);
        t[48 + x] = static_cast<int16_t>(sat16(mulhi16(tm03, 27146) - tm12) | 1);
        const int16_t d16 = sat16(sat16(x1 - x6) * 16), d25 = sat16(sat16(x2 - x5) * 16);
        const int16_t tp65 = static_cast<int16_t>(mulhi16(sat16(d16 + d25), 23170) | 1);
        const int16_t tm65 = mulhi16(sat16(d16 - d25), 23170);
        const int16_t t4 = sat16(sat16(x3 - x4) * 8), t7 = sat16(sat16(x0 - x7) * 8);
        const int16_t tp465 = sat16(t4 + tm65), tm465 = sat16(t4 - tm65);
        const int16_t tp765 = sat16(t7 + tp65), tm765 = sat16(t7 - tp65);
        t[8 + x] = static_cast<int16_t>(sat16(tp765 + mulhi16(tp465, 13036)) | 1);
        t[56 + x] = sat16(mulhi16(tp765, 13036) - tp465);
        t[24 + x] = sat16(tm765 - sat16(mulhi16(tm465, -21746) + tm465));
        t[40 + x] = sat16(sat16(mulhi16(tm765, -21746) + tm765) + tm465);
    }
    const int kRow[4][7] = {{22725, 21407, 19266, 16384, 12873, 8867, 4520},
                            {31521, 29692, 26722, 22725, 17855, 12299, 6270},
                            {29692, 27969, 25172, 21407, 16819, 11585, 5906},
                            {26722, 25172, 22654, 19266, 15137, 10426, 5315}};
    const int kSel[8] = {0, 1, 2, 3, 0, 3, 2, 1};
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const int* cc = kRow[kSel[r]];
        const int C1 = cc[0], C2 = cc[1], C3 = cc[2], C4 = cc[3], C5 = cc[4], C6 = cc[5], C7 = cc[6];
        const int16_t* x = t + r * 8;
        const int s0 = sat16(x[0] + x[7]), s1 = sat16(x[1] + x[6]), s2 = sat16(x[2] + x[5]), s3 = sat16(x[3] + x[4]);
        const int d0 = sat16(x[0] - x[7]), d1 = sat16(x[1] - x[6]), d2 = sat16(x[2] - x[5]), d3 = sat16(x[3] - x[4]);
        int Y[8];
        Y[0] = C4 * s0 + C4 * s1 + C4 * s2 + C4 * s3;
        Y[4] = C4 * s0 - C4 * s1 - C4 * s2 + C4 * s3;
        Y[2] = C2 * s0 + C6 * s1 - C6 * s2 - C2 * s3;
        Y[6] = C6 * s0 - C2 * s1 + C2 * s2 - C6 * s3;
        Y[1] = C1 * d0 + C3 * d1 + C5 * d2 + C7 * d3;
        Y[3] = C3 * d0 - C7 * d1 - C1 * d2 - C5 * d3;
        Y[5] = C5 * d0 - C1 * d1 + C7 * d2 + C3 * d3;
        Y[7] = C7 * d0 - C5 * d1 + C3 * d2 - C1 * d3;
#pragma unroll
        for (int k = 0; k < 8; k++) b[r * 8 + k] = sat16((Y[k] + 65536) >> 17);
    }
}

// The same AP-922 FDCT on column pairs (r06): P[r][m] holds samples (row r, columns 2m and 2m + 1) as
// int16 halves, so the column pass runs two columns per v_pk_* instruction and its output is already
// the row pass's pairs; the row pass's 32 multiply-adds are 16 v_dot2 (int32 accumulation, as the
// scalar form).  The saturations of the scalar form never act for samples in [0, 255] (every sample
// K4 reads is): the largest intermediate is 32640 (checked against fdct_ap922 on 4 M random and
// extreme 0 / 255 blocks, tools/diag/fdct_pk_check.cpp), so plain wrapping int16 arithmetic is exact.
DEVI s16x2 fd_h2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
DEVI uint32_t fd_u(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
DEVI s16x2 fd_mh(s16x2 a, int c) {  // (a * c) >> 16 per half: two products, their high halves by one v_perm
    const int lo = static_cast<int>(a.x) * c, hi = static_cast<int>(a.y) * c;
    return fd_h2(__builtin_amdgcn_perm(static_cast<uint32_t>(hi), static_cast<uint32_t>(lo), 0x07060302u));
}
DEVI void fdct_ap922_pk(const uint32_t (&P)[8][4], int16_t (&b)[64]) {
    const s16x2 one = {1, 1};
    s16x2 T[8][4];  // column pass output, same pair layout: T[row][m]
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const s16x2 x0 = fd_h2(P[0][m]), x1 = fd_h2(P[1][m]), x2 = fd_h2(P[2][m]), x3 = fd_h2(P[3][m]);
        const s16x2 x4 = fd_h2(P[4][m]), x5 = fd_h2(P[5][m]), x6 = fd_h2(P[6][m]), x7 = fd_h2(P[7][m]);
        const s16x2 t0 = (x0 + x7) << 3, t1 = (x1 + x6) << 3, t2 = (x2 + x5) << 3, t3 = (x3 + x4) << 3;
        const s16x2 tp03 = t0 + t3, tm03 = t0 - t3, tp12 = t1 + t2, tm12 = t1 - t2;
        T[0][m] = tp03 + tp12;
        T[4][m] = tp03 - tp12;
        T[2][m] = (tm03 + fd_mh(tm12, 27146)) | one;
        T[6][m] = (fd_mh(tm03, 27146) - tm12) | one;
        const s16x2 d16 = (x1 - x6) << 4, d25 = (x2 - x5) << 4;
        const s16x2 tp65 = fd_mh(d16 + d25, 23170) | one, tm65 = fd_mh(d16 - d25, 23170);
        const s16x2 t4 = (x3 - x4) << 3, t7 = (x0 - x7) << 3;
        const s16x2 tp465 = t4 + tm65, tm465 = t4 - tm65, tp765 = t7 + tp65, tm765 = t7 - tp65;
        T[1][m] = (tp765 + fd_mh(tp465, 13036)) | one;
        T[7][m] = fd_mh(tp765, 13036) - tp465;
        T[3][m] = tm765 - (fd_mh(tm465, -21746) + tm465);
        T[5][m] = (fd_mh(tm765, -21746) + tm765) + tm465;
    }
    constexpr short kRow[4][7] = {{22725, 21407, 19266, 16384, 12873, 8867, 4520},
                                  {31521, 29692, 26722, 22725, 17855, 12299, 6270},
                                  {29692, 27969, 25172, 21407, 16819, 11585, 5906},
                                  {26722, 25172, 22654, 19266, 15137, 10426, 5315}};
    constexpr int kSel[8] = {0, 1, 2, 3, 0, 3, 2, 1};
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const short* cc = kRow[kSel[r]];
        const short C1 = cc[0], C2 = cc[1], C3 = cc[2], C4 = cc[3], C5 = cc[4], C6 = cc[5], C7 = cc[6];
        const uint32_t u67 = fd_u(T[r][3]), u45 = fd_u(T[r][2]);
        const s16x2 x76 = fd_h2((u67 >> 16) | (u67 << 16)), x54 = fd_h2((u45 >> 16) | (u45 << 16));
        const s16x2 s01 = T[r][0] + x76, s23 = T[r][1] + x54, d01 = T[r][0] - x76, d23 = T[r][1] - x54;
        auto dt = [](s16x2 a, short p, short q, s16x2 c, short u, short v) __attribute__((always_inline)) {
            // (the output rounding's + 65536 as the accumulator's start)
            return __builtin_amdgcn_sdot2(c, s16x2{u, v}, __builtin_amdgcn_sdot2(a, s16x2{p, q}, 65536, false), false);
        };
        int Y[8];
        Y[0] = dt(s01, C4, C4, s23, C4, C4);
        Y[4] = dt(s01, C4, static_cast<short>(-C4), s23, static_cast<short>(-C4), C4);
        Y[2] = dt(s01, C2, C6, s23, static_cast<short>(-C6), static_cast<short>(-C2));
        Y[6] = dt(s01, C6, static_cast<short>(-C2), s23, C2, static_cast<short>(-C6));
        Y[1] = dt(d01, C1, C3, d23, C5, C7);
        Y[3] = dt(d01, C3, static_cast<short>(-C7), d23, static_cast<short>(-C1), static_cast<short>(-C5));
        Y[5] = dt(d01, C5, static_cast<short>(-C1), d23, C7, C3);
        Y[7] = dt(d01, C7, static_cast<short>(-C5), d23, C3, static_cast<short>(-C1));
#pragma unroll
        for (int k = 0; k < 8; k++) b[r * 8 + k] = static_cast<int16_t>(Y[k] >> 17);
    }
}

template <typename Pel>
DEVI void jpeg_block(const h2j_frame& f, uint8_t* arena, int bi) {
    const int mbw = (f.out_w + 15) >> 4;
    const int mcu = bi / 6, b = bi % 6;
    const int mx = mcu % mbw, my = mcu / mbw;
    int c, x0, y0;
    if (b < 4) { c = 0; x0 = mx * 16 + (b & 1) * 8; y0 = my * 16 + (b >> 1) * 8; }
    else { c = b - 3; x0 = mx * 8; y0 = my * 8; }
    int16_t blk[64];
#pragma unroll
    for (int j = 0; j < 8; j++)
#pragma unroll
        for (int i = 0; i < 8; i++) blk[j * 8 + i] = static_cast<int16_t>(jpeg_sample<Pel>(f, arena, c, x0 + i, y0 + j));
    fdct_ap922(blk);
    const h2j_jstat* js = reinterpret_cast<const h2j_jstat*>(arena + f.jstat);
    int16_t out[64];
    out[0] = static_cast<int16_t>(((blk[0] >> 2) + 8) / 16);
#pragma unroll
    for (int k = 1; k < 64; k++) {
        const int i = kZigzag[k];
        const int X = blk[i];
        const unsigned a = static_cast<unsigned>(X < 0 ? -X : X);
        unsigned tt = a + js->b16[i];
        tt = tt > 65535u ? 65535u : tt;
        int L = static_cast<int>((tt * js->q16[i]) >> 16);
        L = L > 1023 ? 1023 : L;
        out[k] = static_cast<int16_t>(X < 0 ? -L : L);
    }
    int16_t* dst = reinterpret_cast<int16_t*>(arena + f.jcoef) + static_cast<size_t>(bi) * 64;
#pragma unroll
    for (int k = 0; k < 64; k += 8) {
        int4 v;
        v.x = (static_cast<uint16_t>(out[k]) | (static_cast<uint32_t>(static_cast<uint16_t>(out[k + 1])) << 16));
        v.y = (static_cast<uint16_t>(out[k + 2]) | (static_cast<uint32_t>(static_cast<uint16_t>(out[k + 3])) << 16));
        v.z = (static_cast<uint16_t>(out[k + 4]) | (static_cast<uint32_t>(static_cast<uint16_t>(out[k + 5])) << 16));
        v.w = (static_cast<uint16_t>(out[k + 6]) | (static_cast<uint32_t>(static_cast<uint16_t>(out[k + 7])) << 16));
        *reinterpret_cast<int4*>(dst + k) = v;
    }
}

// ---- K4c, symbol form (the production path).  One workgroup = one 256-block tile of a
// frame; a lane computes its block's FDCT + quantiser as jpeg_block, then, instead of the dense
// int16 plane, writes the block's JPEG symbols: its quantised DC (int16) and the AC symbols in
// emission order -- ZRL / run-size symbols with their magnitude bits, EOB -- one uint32 each
// (bits 0-7 symbol, 8-11 magnitude bit count, 12-27 magnitude bits), stored symbol-major
// ([k][lane]: the readers in h2j_entropy.hip load symbol k of 64 blocks with one coalesced load).
// The AC symbol histograms (the optimal Huffman tables' input) are counted here in LDS, so the
// coefficients are never re-read: K5b / K5d consume the ~4 B per symbol instead of 128 B per
// block.  Tile layout (kJTileBytes, jpeg_tile.h conventions shared with h2j_entropy.hip):
// [kJSymMax][256] uint32 | count[256] uint8 | dc[256] int16.
template <typename Pel>
DEVI void jpeg_block_coefs(const h2j_frame& f, const uint8_t* arena, int bi, int16_t (&out)[64]) {
    const int mbw = (f.out_w + 15) >> 4;
    const int mcu = bi / 6, b = bi % 6;
    const int mx = mcu % mbw, my = mcu / mbw;
    int c, x0, y0;
    if (b < 4) { c = 0; x0 = mx * 16 + (b & 1) * 8; y0 = my * 16 + (b >> 1) * 8; }
    else { c = b - 3; x0 = mx * 8; y0 = my * 8; }
    uint32_t P[8][4];  // row j, columns (2m, 2m + 1) as int16 halves (fdct_ap922_pk)
    const int shc = c ? 1 : 0;
    const int pw = f.out_w >> shc, ph = f.out_h >> shc;
    const int cx = f.crop_x >> shc, cy = f.crop_y >> shc;
    if (sizeof(Pel) == 1 && x0 + 8 <= pw && y0 + 8 <= ph && ((cx + x0) & 7) == 0 && (f.pic_stride[c] & 7) == 0) {
        // the block lies inside the picture: eight 8-byte row loads, bytes to int16 pairs by v_perm
        const uint8_t* p = arena + f.pic2 + f.pic_off[c] + static_cast<size_t>(cy + y0) * f.pic_stride[c] + cx + x0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint2 v = *reinterpret_cast<const uint2*>(p + static_cast<size_t>(j) * f.pic_stride[c]);
            P[j][0] = __builtin_amdgcn_perm(0u, v.x, 0x0C010C00u);
            P[j][1] = __builtin_amdgcn_perm(0u, v.x, 0x0C030C02u);
            P[j][2] = __builtin_amdgcn_perm(0u, v.y, 0x0C010C00u);
            P[j][3] = __builtin_amdgcn_perm(0u, v.y, 0x0C030C02u);
        }
    } else if (sizeof(Pel) == 2 && x0 + 8 <= pw && y0 + 8 <= ph && ((cx + x0) & 7) == 0 && (f.pic_stride[c] & 7) == 0) {
        // 16-bit samples inside the picture: eight 16-byte row loads, converted as jpeg_sample does
        const uint16_t* p = reinterpret_cast<const uint16_t*>(arena + f.pic2) + f.pic_off[c] +
                            static_cast<size_t>(cy + y0) * f.pic_stride[c] + cx + x0;
        const int bd = c ? f.bit_depth_c : f.bit_depth;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint4 v = *reinterpret_cast<const uint4*>(p + static_cast<size_t>(j) * f.pic_stride[c]);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int m = 0; m < 4; m++) {
                uint32_t u0 = w[m] & 0xFFFFu, u1 = w[m] >> 16;
                if (bd > 8) {
                    u0 = min((u0 + (1u << (bd - 9))) >> (bd - 8), 255u);
                    u1 = min((u1 + (1u << (bd - 9))) >> (bd - 8), 255u);
                }
                P[j][m] = u0 | (u1 << 16);
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
#pragma unroll
            for (int m = 0; m < 4; m++)
                P[j][m] = static_cast<uint32_t>(jpeg_sample<Pel>(f, arena, c, x0 + 2 * m, y0 + j)) |
                          (static_cast<uint32_t>(jpeg_sample<Pel>(f, arena, c, x0 + 2 * m + 1, y0 + j)) << 16);
    }
    int16_t blk[64];
    fdct_ap922_pk(P, blk);
    const h2j_jstat* js = reinterpret_cast<const h2j_jstat*>(arena + f.jstat);
    out[0] = static_cast<int16_t>(((blk[0] >> 2) + 8) / 16);
#pragma unroll
    for (int k = 1; k < 64; k++) {
        const int i = kZigzag[k];
        const int X = blk[i];
        const unsigned a = static_cast<unsigned>(X < 0 ? -X : X);
        unsigned tt = a + js->b16[i];
        tt = tt > 65535u ? 65535u : tt;
        int L = static_cast<int>((tt * js->q16[i]) >> 16);
        L = L > 1023 ? 1023 : L;
        out[k] = static_cast<int16_t>(X < 0 ? -L : L);
    }
}

DEVI int jnbits(int v) {
    const unsigned a = static_cast<unsigned>(v < 0 ? -v : v);
    return a ? 32 - __clz(a) : 0;
}

__global__ void __launch_bounds__(256) h2j_k4c_fdct_sym(const h2j_frame* frames, uint8_t* arena) {
    const GridPos gp = xcd_grid_pos();
    __shared__ unsigned hist[2][256];
    const h2j_frame& f = frames[gp.y];
    const int nblk = ((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4) * 6;
    const int b0 = gp.x * 256;
    if (b0 >= nblk) return;
    for (int i = threadIdx.x; i < 512; i += 256) (&hist[0][0])[i] = 0;
    __syncthreads();
    const int t = threadIdx.x, bi = b0 + t;
    uint8_t* tile = arena + f.jcoef + static_cast<size_t>(gp.x) * kJTileBytes;
    uint32_t* sym = reinterpret_cast<uint32_t*>(tile);
    bool eob = false;
    if (bi < nblk) {
        int16_t out[64];
        if (f.bit_depth == 8) jpeg_block_coefs<uint8_t>(f, arena, bi, out);
        else jpeg_block_coefs<uint16_t>(f, arena, bi, out);
        const int tab = (bi % 6) < 4 ? 0 : 1;
        int n = 0, prev = 0;
#pragma unroll
        for (int k = 1; k < 64; k++) {
            const int v = out[k];
            if (v) {
                int run = k - prev - 1;
                prev = k;
                for (; run >= 16; run -= 16) {
                    sym[n++ * 256 + t] = 0xF0u;
                    atomicAdd(&hist[tab][0xF0], 1u);
                }
                const int nb = jnbits(v);
                const int s2 = (run << 4) | nb;
                const uint32_t mag = static_cast<uint32_t>(v < 0 ? v - 1 : v) & ((1u << nb) - 1u);
                sym[n++ * 256 + t] = static_cast<uint32_t>(s2) | (static_cast<uint32_t>(nb) << 8) | (mag << 12);
                atomicAdd(&hist[tab][s2], 1u);
            }
        }
        eob = prev < 63;
        if (eob) sym[n++ * 256 + t] = 0u;  // EOB
        tile[kJCntOff + t] = static_cast<uint8_t>(n);
        reinterpret_cast<int16_t*>(tile + kJDcOff)[t] = out[0];
    }
    {  // EOB counts per wave and table: one LDS atomic each instead of one per block (same bin)
        const int tab = ((b0 + t) % 6) < 4 ? 0 : 1;
        const unsigned long long e0 = __ballot(eob && tab == 0), e1 = __ballot(eob && tab == 1);
        if ((t & 63) == 0) {
            if (e0) atomicAdd(&hist[0][0], static_cast<unsigned>(__popcll(e0)));
            if (e1) atomicAdd(&hist[1][0], static_cast<unsigned>(__popcll(e1)));
        }
    }
    __syncthreads();
    h2j_jstat* js = reinterpret_cast<h2j_jstat*>(arena + f.jstat);
    for (int i = threadIdx.x; i < 512; i += 256) {
        const unsigned v = (&hist[0][0])[i];
        if (v) atomicAdd(&js->hist[2 + (i >> 8)][i & 255], v);
    }
}

__global__ void __launch_bounds__(256) h2j_k4c_fdct_quant(const h2j_frame* frames, uint8_t* arena) {
    const h2j_frame& f = frames[blockIdx.y];
    const int nblk = ((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4) * 6;
    const int bi = blockIdx.x * blockDim.x + threadIdx.x;
    if (bi >= nblk) return;
    if (f.bit_depth == 8) jpeg_block<uint8_t>(f, arena, bi);
    else jpeg_block<uint16_t>(f, arena, bi);
}


}  // namespace

namespace h2jgpu {
thread_local char g_err[256] = {0};

int check(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -static_cast<int>(e) - 1000;
}
}  // namespace h2jgpu
using h2jgpu::check;
using h2jgpu::g_err;

// ---------------------------------------------------------------- C ABI
extern "C" {

const char* h2j_gpu_last_error(void) { return g_err; }

int h2j_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
int h2j_gpu_set_device(int device) { return check(hipSetDevice(device), "hipSetDevice"); }
int h2j_gpu_pci_bus_id(int device, char* buf, int len) {
    return check(hipDeviceGetPCIBusId(buf, len, device), "hipDeviceGetPCIBusId");
}
void* h2j_gpu_malloc(size_t bytes) {
    void* p = nullptr;
    if (check(hipMalloc(&p, bytes), "hipMalloc")) return nullptr;
    return p;
}
int h2j_gpu_free(void* p) { return check(hipFree(p), "hipFree"); }
int h2j_gpu_mem_info(size_t* free_bytes, size_t* total_bytes) {
    return check(hipMemGetInfo(free_bytes, total_bytes), "hipMemGetInfo");
}
void* h2j_gpu_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (check(hipHostMalloc(&p, bytes, hipHostMallocDefault), "hipHostMalloc")) return nullptr;
    return p;
}
int h2j_gpu_host_free(void* p) { return check(hipHostFree(p), "hipHostFree"); }
void* h2j_gpu_stream_create(void) {
    hipStream_t s = nullptr;
    if (check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate")) return nullptr;
    return s;
}
int h2j_gpu_stream_destroy(void* s) { return check(hipStreamDestroy(static_cast<hipStream_t>(s)), "hipStreamDestroy"); }
// hipStreamSynchronize (HIP yields while it waits: the host CPU use of the bench is the
// same as with blocking waits).  H2J_SYNC=block waits on a blocking-sync event instead.
int h2j_gpu_stream_sync(void* s) {
    static const bool spin = [] {
        const char* e = std::getenv("H2J_SYNC");
        return !(e && std::strcmp(e, "block") == 0);
    }();
    hipStream_t st = static_cast<hipStream_t>(s);
    if (spin) return check(hipStreamSynchronize(st), "hipStreamSynchronize");
    hipEvent_t ev = nullptr;
    int r = check(hipEventCreateWithFlags(&ev, hipEventBlockingSync | hipEventDisableTiming), "hipEventCreateWithFlags");
    if (r) return r;
    r = check(hipEventRecord(ev, st), "hipEventRecord");
    if (!r) r = check(hipEventSynchronize(ev), "hipEventSynchronize");
    (void)hipEventDestroy(ev);
    return r;
}
int h2j_gpu_memcpy_h2d(void* dst, const void* src, size_t n, void* s) {
    return check(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, static_cast<hipStream_t>(s)), "hipMemcpyH2D");
}
int h2j_gpu_memcpy_d2h(void* dst, const void* src, size_t n, void* s) {
    return check(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, static_cast<hipStream_t>(s)), "hipMemcpyD2H");
}
int h2j_gpu_memset(void* dst, int v, size_t n, void* s) {
    return check(hipMemsetAsync(dst, v, n, static_cast<hipStream_t>(s)), "hipMemsetAsync");
}
void* h2j_gpu_event_create(void) {
    hipEvent_t e = nullptr;
    if (check(hipEventCreate(&e), "hipEventCreate")) return nullptr;
    return e;
}
int h2j_gpu_event_destroy(void* e) { return check(hipEventDestroy(static_cast<hipEvent_t>(e)), "hipEventDestroy"); }
int h2j_gpu_event_record(void* e, void* s) {
    return check(hipEventRecord(static_cast<hipEvent_t>(e), static_cast<hipStream_t>(s)), "hipEventRecord");
}
int h2j_gpu_stream_wait_event(void* s, void* e) {
    return check(hipStreamWaitEvent(static_cast<hipStream_t>(s), static_cast<hipEvent_t>(e), 0), "hipStreamWaitEvent");
}
float h2j_gpu_event_elapsed_ms(void* a, void* b) {
    float ms = -1.f;
    if (check(hipEventElapsedTime(&ms, static_cast<hipEvent_t>(a), static_cast<hipEvent_t>(b)), "hipEventElapsedTime"))
        return -1.f;
    return ms;
}

int h2j_gpu_prep(const h2j_gpu_batch* b, void* stream) {
    if (!b || b->nframes <= 0) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (b->max_ntu <= 0) return 0;
    if (b->has_hevc) {
        const int waves = (b->max_ntu + kK0TusHevc - 1) / kK0TusHevc;
        hipLaunchKernelGGL(h2j_k0_prep<true>, dim3(waves, b->nframes), dim3(64), 0, s, b->frames, b->tus, b->coefs,
                           b->ctbs, b->slices, b->sl, b->arena);
        const int r = check(hipGetLastError(), "h2j_k0_prep<hevc>");
        if (r) return r;
    }
    if (b->has_h264) {
        const int waves = (b->max_ntu + kK0Tus - 1) / kK0Tus;
        hipLaunchKernelGGL(h2j_k0_prep<false>, dim3(waves, b->nframes), dim3(64), 0, s, b->frames, b->tus, b->coefs,
                           b->ctbs, b->slices, b->sl, b->arena);
        return check(hipGetLastError(), "h2j_k0_prep<h264>");
    }
    return 0;
}

// K1 cycle accounting (only in -DH2J_PROF builds): copies 16 counters, optionally resets them.
int h2j_gpu_prof(unsigned long long* out, int n, int reset) {
#ifdef H2J_PROF
    unsigned long long h[16] = {0};
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prof), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < n && i < 16; i++) out[i] = h[i];
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
#else
    (void)out; (void)n; (void)reset;
    return -1;
#endif
}

// companion stream + fork / join events of a chunk stream (created on first use, kept)
struct AuxStream {
    hipStream_t s2 = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
static AuxStream* aux_stream(hipStream_t s) {
    static std::mutex mu;
    static std::vector<std::pair<hipStream_t, AuxStream*>> all;
    std::lock_guard<std::mutex> lk(mu);
    for (auto& e : all)
        if (e.first == s) return e.second;
    AuxStream* a = new AuxStream();
    if (hipStreamCreateWithFlags(&a->s2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&a->fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&a->join, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        delete a;
        return nullptr;
    }
    all.emplace_back(s, a);
    return a;
}

static int predict_main(const h2j_gpu_batch* b, void* stream) {
    if (!b || b->nframes <= 0) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // two workgroups per HEVC picture (luma, chroma).  Up to 128 pictures every group gets a CU
    // of its own and runs kK1WavesWide waves (rows in flight); beyond that two groups share
    // a CU and run kK1Waves each (VGPR-bound occupancy).
    const bool wide = b->nframes <= 128;
    const int pels = b->hevc_pels;  // bit 0: 8-bit HEVC pictures, bit 1: high bit depth
    const int kinds = ((pels & 1) ? 1 : 0) + ((pels & 2) ? 1 : 0) + (b->has_h264 && b->k1wgs > 0 ? 1 : 0);
    const size_t lds264 = sizeof(H4WaveLds) * kAvcK1Waves + 2 * kAvcK1Waves * 4 + 4 * static_cast<size_t>(b->max_w);
    const size_t lds264any = sizeof(H4WaveLds) * kAvcWaves + 2 * kAvcWaves * 4 + 4 * static_cast<size_t>(b->max_w);
    static bool attr = false;
    if (!attr) {
        const void* fns[] = {reinterpret_cast<const void*>(h2j_k1_recon_hevc<uint8_t, kK1WavesWide>),
                             reinterpret_cast<const void*>(h2j_k1_recon_hevc<uint16_t, kK1WavesWide>),
                             reinterpret_cast<const void*>(h2j_k1_recon_h264),
                             reinterpret_cast<const void*>(h2j_k1_recon_any),
                             reinterpret_cast<const void*>(h2j_k1_recon_hevc_pool<uint8_t>),
                             reinterpret_cast<const void*>(h2j_k1_recon_hevc_pool<uint16_t>)};
        for (const void* fn : fns) {  // dynamic LDS up to 160 KB minus the kernel's static LDS
            hipFuncAttributes fa{};
            const size_t st = hipFuncGetAttributes(&fa, fn) == hipSuccess ? fa.sharedSizeBytes : 0;
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(160 * 1024 - st));
        }
        (void)hipGetLastError();  // attribute calls must not leave an error for the launch checks
        attr = true;
    }
    constexpr int pool_p = 4;  // max pictures per pool workgroup
    const size_t line_bytes = 2 * (static_cast<size_t>(b->max_w) + 64) * sizeof(int16_t);
    const size_t wbytes = k1_fixed_lds(kK1WavesWide) + line_bytes;
    // merged launch: an HEVC picture workgroup runs the pool's job loop with P = 1 (hevc_pool_jobs)
    const size_t pool1 = k1_pool_lds(1, (b->max_h + 15) / 16, 2 * b->max_w + 192);
    const size_t lds_any = std::max(std::max(pool1, lds264any), wbytes);
    // one launch for every kind of picture (unless the widest picture's line buffers would not
    // fit one workgroup's LDS: then the per-kind launches below)
    if (!wide && kinds >= 2 && b->k1all && b->k1all_n > 0 && lds_any <= 160 * 1024) {
        AuxStream* ax2 = (b->has_h264 && b->k1wgs8 > 0 && b->k1hevc_n > 0) ? aux_stream(s) : nullptr;
        if (!ax2) {
            hipLaunchKernelGGL(h2j_k1_recon_any, dim3(b->k1all_n), dim3(64 * kAvcWaves), lds_any, s, b->frames, b->tus,
                               b->ctbs, b->arena, b->k1all);
            return check(hipGetLastError(), "h2j_k1_recon_any");
        }
        // the HEVC pictures' merged launch and the H.264 pictures' own launch (8-wave workgroups, two
        // per CU, 8-row bands) side by side on two streams (r06: 18.45 -> 17.72 ms per 1024 configs[4]
        // pictures against every kind in h2j_k1_recon_any, profiles/r06_ab_runs.txt)
        (void)hipEventRecord(ax2->fork, s);
        (void)hipStreamWaitEvent(ax2->s2, ax2->fork, 0);
        hipLaunchKernelGGL(h2j_k1_recon_h264, dim3(b->k1wgs8), dim3(64 * kAvcK1Waves), lds264, ax2->s2, b->frames, b->tus,
                           b->ctbs, b->arena, b->k1map8);
        const int r2 = check(hipGetLastError(), "h2j_k1_recon_h264");
        (void)hipEventRecord(ax2->join, ax2->s2);
        const size_t lds_hev = std::max(pool1, wbytes);
        hipLaunchKernelGGL(h2j_k1_recon_any, dim3(b->k1hevc_n), dim3(64 * kAvcWaves), lds_hev, s, b->frames, b->tus,
                           b->ctbs, b->arena, b->k1hevc);
        const int r1 = check(hipGetLastError(), "h2j_k1_recon_any");
        (void)hipStreamWaitEvent(s, ax2->join, 0);
        return r1 ? r1 : r2;
    }
    // per-kind launches: H.264 on a companion stream forked from (and joined back into) the
    // chunk's stream, so its workgroups fill the CUs the HEVC launches leave idle
    AuxStream* ax = (b->has_hevc && b->has_h264 && b->k1wgs > 0) ? aux_stream(s) : nullptr;
    if (ax) {
        (void)hipEventRecord(ax->fork, s);
        (void)hipStreamWaitEvent(ax->s2, ax->fork, 0);
        hipLaunchKernelGGL(h2j_k1_recon_h264, dim3(b->k1wgs8), dim3(64 * kAvcK1Waves), lds264, ax->s2, b->frames, b->tus,
                           b->ctbs, b->arena, b->k1map8);
        const int r = check(hipGetLastError(), "h2j_k1_recon_h264");
        (void)hipEventRecord(ax->join, ax->s2);
        if (r) {
            (void)hipStreamWaitEvent(s, ax->join, 0);
            return r;
        }
    }
    if (b->has_hevc) {
        const bool p8 = pels == 0 || (pels & 1), p16 = pels == 0 || (pels & 2);
        if (wide) {
            const size_t lds = wbytes;
            const dim3 grid(b->nframes, 2), block(64 * kK1WavesWide);
            if (p8) hipLaunchKernelGGL((h2j_k1_recon_hevc<uint8_t, kK1WavesWide>), grid, block, lds, s, b->frames, b->tus, b->arena);
            if (p16) hipLaunchKernelGGL((h2j_k1_recon_hevc<uint16_t, kK1WavesWide>), grid, block, lds, s, b->frames, b->tus, b->arena);
        } else {
            // pictures per pool workgroup: at least 256 workgroups (one per CU) per launch, as
            // many pictures each as fit (LDS: one set of line buffers + progress words per picture)
            const int maxrows = (b->max_h + 15) / 16;
            const int lstride = 2 * b->max_w + 192, lchroma = b->max_w + 64;
            // LDS: the pool's layout + the staging tiles (k1_pool_stage_lds) of the launch's sample size
            auto pool_lds = [&](int P, int pel) {
                return ((k1_pool_lds(P, maxrows, lstride) + 15) & ~size_t(15)) + k1_pool_stage_lds(pel);
            };
            for (int pel = 1; pel <= 2; pel++) {
                if (!(pel == 1 ? p8 : p16)) continue;
                int P = std::max(1, std::min(pool_p, b->nframes / 256));  // never fewer than 256 workgroups
                while (P > 1 && pool_lds(P, pel) > 160 * 1024) P--;
                const size_t lds = pool_lds(P, pel);
                if (lds > 160 * 1024) {
                    snprintf(g_err, sizeof(g_err), "h2j_k1_recon_hevc_pool: %zu B of LDS per workgroup (max 160 KB)", lds);
                    return -1;
                }
                const dim3 grid((b->nframes + P - 1) / P), block(64 * kPoolWaves);
                if (pel == 1) hipLaunchKernelGGL(h2j_k1_recon_hevc_pool<uint8_t>, grid, block, lds, s, b->frames, b->tus, b->arena,
                                                 b->nframes, P, maxrows, lstride, lchroma, 1);
                else hipLaunchKernelGGL(h2j_k1_recon_hevc_pool<uint16_t>, grid, block, lds, s, b->frames, b->tus, b->arena,
                                        b->nframes, P, maxrows, lstride, lchroma, 1);
            }
        }
        int r = check(hipGetLastError(), "h2j_k1_recon_hevc");
        if (ax) (void)hipStreamWaitEvent(s, ax->join, 0);
        if (r) return r;
    }
    if (b->has_h264 && !ax) {
        // dynamic LDS: per-wave windows, progress counters, line buffer (luma + 2 chroma, uint16)
        if (b->k1wgs > 0)
            hipLaunchKernelGGL(h2j_k1_recon_h264, dim3(b->k1wgs8), dim3(64 * kAvcK1Waves), lds264, s, b->frames, b->tus,
                               b->ctbs, b->arena, b->k1map8);
        return check(hipGetLastError(), "h2j_k1_recon_h264");
    }
    return 0;
}

// K1 for MBAFF H.264 pictures, after the other K1 launches of the batch (h2j_gpu_predict)
static int predict_mbaff(const h2j_gpu_batch* b, hipStream_t s) {
    if (!b->has_mbaff || b->k1wgs <= 0) return 0;
    static bool attr = false;
    if (!attr) {
        const void* fn = reinterpret_cast<const void*>(h2j_k1_recon_h264_mbaff);
        hipFuncAttributes fa{};
        const size_t st = hipFuncGetAttributes(&fa, fn) == hipSuccess ? fa.sharedSizeBytes : 0;
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(160 * 1024 - st));
        (void)hipGetLastError();
        attr = true;
    }
    const size_t lds = sizeof(H4WaveLds) * kAvcWaves + 2 * kAvcWaves * 4;
    hipLaunchKernelGGL(h2j_k1_recon_h264_mbaff, dim3(b->k1wgs), dim3(64 * kAvcWaves), lds, s, b->frames, b->tus, b->ctbs,
                       b->arena, b->k1map);
    return check(hipGetLastError(), "h2j_k1_recon_h264_mbaff");
}

int h2j_gpu_predict(const h2j_gpu_batch* b, void* stream) {
    const int r = predict_main(b, stream);
    return (r || !b) ? r : predict_mbaff(b, static_cast<hipStream_t>(stream));
}

int h2j_gpu_recon(const h2j_gpu_batch* b, void* stream) {
    const int r = h2j_gpu_prep(b, stream);
    return r ? r : h2j_gpu_predict(b, stream);
}

int h2j_gpu_deblock(const h2j_gpu_batch* b, void* stream) {
    if (!b || b->nframes <= 0) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (b->has_hevc) {
        const int mw = (b->max_w + 3) >> 2, mh = (b->max_h + 3) >> 2;  // 4x4 grid of the largest picture
        const dim3 gv((((mw + 1) >> 1) * mh + 255) / 256, b->nframes), gh((mw * ((mh + 1) >> 1) + 255) / 256, b->nframes);
        hipLaunchKernelGGL(h2j_k2_deblock, gv, dim3(256), 0, s, b->frames, b->ctbs, b->slices, b->arena, 1);
        int r = check(hipGetLastError(), "h2j_k2_deblock(v)");
        if (r) return r;
        hipLaunchKernelGGL(h2j_k2_deblock, gh, dim3(256), 0, s, b->frames, b->ctbs, b->slices, b->arena, 0);
        r = check(hipGetLastError(), "h2j_k2_deblock(h)");
        if (r) return r;
    }
    if (!b->has_h264 || b->k1wgs <= 0) return 0;
    // dynamic LDS: windows, progress, tables and a line buffer (6 samples per column) of the batch's
    // widest picture up to line_w: at 8 bits the width that keeps two workgroups per CU (80 KB),
    // at 16 bits what fits the CU's 160 KB.  Wider pictures: a second launch, line in global memory.
    auto launch = [&](auto pel, const void* fn, const void* fn_wide, const char* name) -> int {
        using Pel = decltype(pel);
        static size_t cap[2] = {0, 0};  // LDS budget minus the kernel's static LDS
        size_t& c = cap[sizeof(Pel) - 1];
        const size_t fixed = sizeof(DbWin<Pel>) * 2 * kDbPairWaves + kDbPairSlots * 4 + sizeof(DbTables);
        if (!c) {
            hipFuncAttributes fa{};
            const size_t st = hipFuncGetAttributes(&fa, fn) == hipSuccess ? fa.sharedSizeBytes : 0;
            c = (sizeof(Pel) == 1 ? 80 : 160) * 1024 - st;
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(160 * 1024 - st));
            (void)hipFuncSetAttribute(fn_wide, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(fixed));
            (void)hipGetLastError();
        }
        const int line_w = std::min(b->max_w, static_cast<int>((c - fixed) / (6 * sizeof(Pel))) & ~15);
        // the wide pictures (long banded chains) on the companion stream, started first and
        // running beside the LDS-line launch instead of after its tail
        const bool wide = b->max_w > line_w;
        AuxStream* ax = wide ? aux_stream(s) : nullptr;
        if (ax) {
            (void)hipEventRecord(ax->fork, s);
            (void)hipStreamWaitEvent(ax->s2, ax->fork, 0);
        }
        if (wide) {
            hipLaunchKernelGGL((h2j_k2_deblock264p<Pel, true>), dim3(b->k1wgs), dim3(64 * kDbPairWaves), fixed,
                               ax ? ax->s2 : s, b->frames, b->ctbs, b->slices, b->arena, b->k1map, line_w);
            const int rw = check(hipGetLastError(), name);
            if (ax) (void)hipEventRecord(ax->join, ax->s2);
            if (rw) {
                if (ax) (void)hipStreamWaitEvent(s, ax->join, 0);
                return rw;
            }
        }
        hipLaunchKernelGGL((h2j_k2_deblock264p<Pel, false>), dim3(b->k1wgs), dim3(64 * kDbPairWaves),
                           fixed + 6 * sizeof(Pel) * static_cast<size_t>(line_w), s, b->frames, b->ctbs, b->slices,
                           b->arena, b->k1map, line_w);
        const int rc = check(hipGetLastError(), name);
        if (ax) (void)hipStreamWaitEvent(s, ax->join, 0);
        return rc;
    };
    int r = 0;
    if (b->h264_pels & 1)
        r = launch(uint8_t{}, reinterpret_cast<const void*>(h2j_k2_deblock264p<uint8_t, false>),
                   reinterpret_cast<const void*>(h2j_k2_deblock264p<uint8_t, true>), "h2j_k2_deblock264p<u8>");
    if (!r && (b->h264_pels & 2))
        r = launch(uint16_t{}, reinterpret_cast<const void*>(h2j_k2_deblock264p<uint16_t, false>),
                   reinterpret_cast<const void*>(h2j_k2_deblock264p<uint16_t, true>), "h2j_k2_deblock264p<u16>");
    if (!r && b->has_mbaff) {
        hipLaunchKernelGGL(h2j_k2_deblock264m, dim3(b->k1wgs), dim3(64 * kDbPairWaves), 0, s, b->frames, b->ctbs,
                           b->slices, b->arena, b->k1map);
        r = check(hipGetLastError(), "h2j_k2_deblock264m");
    }
    return r;
}

int h2j_gpu_sao(const h2j_gpu_batch* b, void* stream) {
    if (!b || b->nframes <= 0 || !b->has_hevc) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // one launch per CTB-count class (h2j_gpu_batch.sao_map): grid = the class's largest CTB count
    // x its pictures, so a mixed batch's small pictures do not run the 4K grid's empty workgroups
    for (int g = 0; g < b->sao_groups && g < H2J_SAO_GROUPS; g++) {
        if (b->sao_count[g] <= 0 || b->sao_ctbs[g] <= 0) continue;
        dim3 grid(static_cast<unsigned>(b->sao_ctbs[g]), static_cast<unsigned>(b->sao_count[g]));
        hipLaunchKernelGGL(h2j_k3_sao, grid, dim3(256), 0, s, b->frames, b->ctbs, b->slices, b->arena, 1,
                           b->sao_map + b->sao_first[g]);
        if (int rc = check(hipGetLastError(), "h2j_k3_sao")) return rc;
    }
    return 0;
}

int h2j_gpu_jpeg(const h2j_gpu_batch* b, void* stream) {
    if (!b || b->nframes <= 0) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int mbs = b->max_mcu;
    if (b->k4a_frames > 0) {  // none: K3 has summed every picture's MB variances
        hipLaunchKernelGGL(h2j_k4a_variance, dim3((mbs + 15) / 16, b->nframes), dim3(256), 0, s, b->frames, b->arena, 1);
        const int r = check(hipGetLastError(), "h2j_k4a_variance");
        if (r) return r;
    }
    int r = 0;
    hipLaunchKernelGGL(h2j_k4b_ratecontrol, dim3(b->nframes), dim3(64), 0, s, b->frames, b->arena);
    r = check(hipGetLastError(), "h2j_k4b_ratecontrol");
    if (r) return r;
    const int nblk = mbs * 6;
    if (b->jpeg_dense) {  // inspection path (h2j_engine_jpeg_coeffs): the dense int16 plane
        hipLaunchKernelGGL(h2j_k4c_fdct_quant, dim3((nblk + 255) / 256, b->nframes), dim3(256), 0, s, b->frames, b->arena);
        return check(hipGetLastError(), "h2j_k4c_fdct_quant");
    }
    hipLaunchKernelGGL(h2j_k4c_fdct_sym, dim3((nblk + 255) / 256, b->nframes), dim3(256), 0, s, b->frames, b->arena);
    r = check(hipGetLastError(), "h2j_k4c_fdct_sym");
    if (r) return r;
    return h2j_gpu_histogram(b, stream);  // DC histograms
}

}  // extern "C"
