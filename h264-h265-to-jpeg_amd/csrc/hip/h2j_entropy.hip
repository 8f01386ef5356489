// MI355X (gfx950) JPEG entropy stage: symbol histograms, FFmpeg-exact optimal
// Huffman tables and baseline-JPEG bit emission, all on the GPU, so only the
// entropy-coded payload (~1/30 of the coefficient bytes) crosses PCIe.
//
//   (K4c h2j_k4c_fdct_sym, h2j_kernels.hip, writes each block's quantised DC and
//   its AC symbols -- run/size + magnitude bits -- and counts the AC histograms)
//   K4e h2j_k4e_dc_hist    — per 256-block tile: DC differences from the tiles'
//                            DC arrays, LDS histogram, one global atomic per
//                            (tile, category)
//   K5a h2j_k5a_tables     — one workgroup per (frame, table): AV_QSORT +
//                            package-merge (max length 16) restated without
//                            item lists (per-level probability arrays + leaf
//                            prefix counts), then the length sort and canonical
//                            code assignment of mjpegenc_huffman.c
//   K5b h2j_k5b_tile_bits  — bits per 256-block tile, from the symbol stream
//   K5c h2j_k5c_scan       — per-frame tile offsets, payload sizes, then the
//                            batch-level segment offsets (one workgroup)
//   K5z h2j_k5z_zero       — clears the used part of the segment pool
//   K5d h2j_k5d_emit       — per lane one block: workgroup scan of block bit
//                            counts, MSB-first words from the symbol stream,
//                            atomicOr only on the two words a block can share
//                            with its neighbours
//
// Byte stuffing (0xFF -> 0xFF 0x00) is left to the host, which copies the
// payload into the JPEG container anyway.  Reference semantics: FFmpeg
// mjpegenc_common.c / mjpegenc_huffman.c as restated in SURVEY.md Appendix A
// (A.6) and oracle/jpeg_ref.c; the host restatement is
// csrc/host/jpeg_writer.cpp.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <cstdio>

#include "h2j_gpu.h"
#include "grid.h"
#include "jpeg_tile.h"

#define DEVI __device__ __forceinline__

namespace {

constexpr int kTile = 256;      // blocks per workgroup

DEVI int nbits16(int v) {
    const unsigned a = static_cast<unsigned>(v < 0 ? -v : v);
    return a ? 32 - __clz(a) : 0;
}

DEVI int nblocks(const h2j_frame& f) { return ((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4) * 6; }

// quantised DC of block bi (the tiles' DC arrays) and its DPCM predictor (MCU order Y0 Y1 Y2 Y3
// Cb Cr, FFmpeg's last_dc = 128 at the scan start)
DEVI int dc_of(const uint8_t* base, int bi) {
    return reinterpret_cast<const int16_t*>(base + static_cast<size_t>(bi >> 8) * kJTileBytes + kJDcOff)[bi & 255];
}
DEVI int prev_dc(const uint8_t* base, int bi) {
    const int mcu = bi / 6, b = bi - mcu * 6;
    int pb;
    if (b < 4) pb = b > 0 ? bi - 1 : (mcu > 0 ? bi - 3 : -1);
    else pb = mcu > 0 ? bi - 6 : -1;
    return pb < 0 ? 128 : dc_of(base, pb);
}

// ---------------------------------------------------------------- K4e
__global__ void __launch_bounds__(kTile) h2j_k4e_dc_hist(const h2j_frame* frames, uint8_t* arena) {
    __shared__ unsigned hist[2][16];
    const h2j_frame& f = frames[blockIdx.y];
    const int nblk = nblocks(f);
    const int b0 = blockIdx.x * kTile;
    if (b0 >= nblk) return;
    if (threadIdx.x < 32) (&hist[0][0])[threadIdx.x] = 0;
    __syncthreads();
    const uint8_t* base = arena + f.jcoef;
    const int bi = b0 + threadIdx.x;
    if (bi < nblk) atomicAdd(&hist[(bi % 6) < 4 ? 0 : 1][nbits16(dc_of(base, bi) - prev_dc(base, bi))], 1u);
    __syncthreads();
    h2j_jstat* js = reinterpret_cast<h2j_jstat*>(arena + f.jstat);
    if (threadIdx.x < 32) {
        const unsigned v = (&hist[0][0])[threadIdx.x];
        if (v) atomicAdd(&js->hist[threadIdx.x >> 4][threadIdx.x & 15], v);
    }
}

// ---------------------------------------------------------------- K5a
struct HuffLds {
    uint64_t leaf[16][9];     // bit m of level t: item m of list t is a leaf (cumulative counts
                              // by popcount; 1 KB instead of a 16 KB count table)
    int pv[260], pp[260];     // leaves (symbol, count), sorted by AV_QSORT
    union {                   // three phases that never overlap in time:
        unsigned hist[256];   // the table's symbol counts, staged by all lanes (until the leaves
                              // are collected)
        int P[2][520];        // item probabilities of the previous / current package-merge list
        struct {
            int hc[256], hl[256];  // (symbol, length) pairs, once the code lengths are known
        };
    };
    int nlist[17];
    int nb[260];              // code length per symbol
    int stk[64][2];
};
// ~9 KB: the 16 tables a CU gets (4 per picture over 1024 pictures on 256 CUs) all fit its
// 160 KB of LDS at once, so this latency-bound serial kernel runs them in one round
static_assert(sizeof(HuffLds) <= 10 * 1024, "K5a LDS per table");

// libavutil/qsort.h AV_QSORT on index range [0, num) (unstable: tie order
// must be FFmpeg's own, so this is a literal restatement, run by one lane).
template <typename Cmp, typename Swp>
DEVI void av_qsort_dev(int num, Cmp cmp, Swp swp, int (*stk)[2]) {
    if (num <= 0) return;
    int sp = 1;
    stk[0][0] = 0;
    stk[0][1] = num - 1;
    while (sp) {
        --sp;
        int start = stk[sp][0], end = stk[sp][1];
        while (start < end) {
            if (start < end - 1) {
                int checksort = 0;
                int right = end - 2, left = start + 1, mid = start + ((end - start) >> 1);
                if (cmp(start, end) > 0) {
                    if (cmp(end, mid) > 0) swp(start, mid);
                    else swp(start, end);
                } else {
                    if (cmp(start, mid) > 0) swp(start, mid);
                    else checksort = 1;
                }
                if (cmp(mid, end) > 0) {
                    swp(mid, end);
                    checksort = 0;
                }
                if (start == end - 2) break;
                swp(end - 1, mid);
                while (left <= right) {
                    while (left <= right && cmp(left, end - 1) < 0) left++;
                    while (left <= right && cmp(right, end - 1) > 0) right--;
                    if (left <= right) {
                        swp(left, right);
                        left++;
                        right--;
                    }
                }
                swp(end - 1, left);
                if (checksort && (mid == left - 1 || mid == left)) {
                    mid = start;
                    while (mid < end && cmp(mid, mid + 1) <= 0) mid++;
                    if (mid == end) break;
                }
                if (end - left < left - start) {
                    stk[sp][0] = start;
                    stk[sp][1] = right;
                    sp++;
                    start = left + 1;
                } else {
                    stk[sp][0] = left + 1;
                    stk[sp][1] = end;
                    sp++;
                    end = right;
                }
            } else {
                if (cmp(start, end) > 0) swp(start, end);
                break;
            }
        }
    }
}

__global__ void __launch_bounds__(64) h2j_k5a_tables(const h2j_frame* frames, uint8_t* arena) {
    __shared__ HuffLds s;
    const h2j_frame& f = frames[blockIdx.y];
    h2j_jstat* js = reinterpret_cast<h2j_jstat*>(arena + f.jstat);
    const int t = blockIdx.x;
    // the counts through LDS (one wide pass by every lane; a serial loop of global loads
    // would wait for each of them)
    for (int i = threadIdx.x; i < 256; i += 64) {
        s.hist[i] = js->hist[t][i];
        js->len[t][i] = 0;  // by every lane; lane 0 writes the used entries below (same wave:
        js->code[t][i] = 0; // its later stores to these addresses land after these)
    }
    __syncthreads();
    if (threadIdx.x != 0) return;  // serial by construction (AV_QSORT tie order)
    int nval = 0;
    for (int i = 0; i < 256; i++) {
        const unsigned c = s.hist[i];
        if (c) {
            s.pv[nval] = i;
            s.pp[nval] = static_cast<int>(c);
            nval++;
        }
    }
    s.pv[nval] = 256;
    s.pp[nval] = 0;
    const int size = nval + 1;
    av_qsort_dev(
        size, [&](int a, int b) { return s.pp[a] - s.pp[b]; },
        [&](int a, int b) {
            int x = s.pv[a]; s.pv[a] = s.pv[b]; s.pv[b] = x;
            x = s.pp[a]; s.pp[a] = s.pp[b]; s.pp[b] = x;
        },
        s.stk);
    // package-merge, 16 levels + the final pairing round (i not reset).  The next two leaf
    // weights and the next two pair sums ride in registers (INT_MAX once a list is used up), so
    // a step's leaf-or-pair decision compares registers and the loads it needs were issued a
    // step earlier: one lane walking LDS waited a round trip per step before.
    int np = 0, cur = 0, i = 0;
    for (int lvl = 0; lvl <= 16; lvl++) {
        int* Pc = s.P[cur];
        const int* Pp = s.P[cur ^ 1];
        int j = 0, n = 0;
        uint64_t word = 0;  // leaf bits of the current 64 items
        if (lvl < 16) i = 0;
        const int npv = np;
        auto ldleaf = [&](int k) { return k < size ? s.pp[k] : INT_MAX; };
        auto ldpair = [&](int k) { return k + 1 < npv ? Pp[k] + Pp[k + 1] : INT_MAX; };
        int l0 = ldleaf(i), l1 = ldleaf(i + 1), q0 = ldpair(j), q1 = ldpair(j + 2);
        while (i < size || j + 1 < np) {
            // = i < size && (j + 1 >= np || pp[i] < Pp[j] + Pp[j + 1]): weights stay far below INT_MAX
            const bool leaf = l0 < q0;
            if (leaf) {
                Pc[n] = l0;
                i++;
                l0 = l1;
                l1 = ldleaf(i + 1);
            } else {
                Pc[n] = q0;
                j += 2;
                q0 = q1;
                q1 = ldpair(j + 2);
            }
            if (lvl < 16) {
                word |= static_cast<uint64_t>(leaf) << (n & 63);
                if ((n & 63) == 63) {
                    s.leaf[lvl][n >> 6] = word;
                    word = 0;
                }
            }
            n++;
        }
        if (lvl < 16 && (n & 63)) s.leaf[lvl][n >> 6] = word;
        s.nlist[lvl] = n;
        np = n;
        cur ^= 1;
    }
    for (int k = 0; k < 257; k++) s.nb[k] = 0;
    {
        const int mn = size - 1 < s.nlist[16] ? size - 1 : s.nlist[16];
        int m = 2 * mn;
        for (int lvl = 15; lvl >= 0 && m > 0; lvl--) {
            int lv = 0;  // leaves among the first m items of list lvl
            for (int wd = 0; wd < (m >> 6); wd++) lv += __popcll(s.leaf[lvl][wd]);
            if (m & 63) lv += __popcll(s.leaf[lvl][m >> 6] & ((1ull << (m & 63)) - 1ull));
            for (int k = 0; k < lv; k++) s.nb[s.pv[k]]++;
            m = 2 * (m - lv);
        }
    }
    int nd = 0;
    for (int k = 0; k < 256; k++)
        if (s.nb[k] > 0) {
            s.hc[nd] = k;
            s.hl[nd] = s.nb[k];
            nd++;
        }
    av_qsort_dev(
        nval, [&](int a, int b) { return s.hl[a] - s.hl[b]; },
        [&](int a, int b) {
            int x = s.hc[a]; s.hc[a] = s.hc[b]; s.hc[b] = x;
            x = s.hl[a]; s.hl[a] = s.hl[b]; s.hl[b] = x;
        },
        s.stk);
    // codes per length counted in registers / LDS, not by read-modify-writes of global memory
    int bits[17];
#pragma unroll
    for (int l = 0; l <= 16; l++) bits[l] = 0;
    for (int k = 0; k < nval; k++) {
        const int l = s.hl[k];
#pragma unroll
        for (int q = 1; q <= 16; q++) bits[q] += l == q ? 1 : 0;
        js->val[t][k] = static_cast<uint8_t>(s.hc[k]);
    }
    for (int k = 0; k < 20; k++) js->bits[t][k] = k <= 16 ? static_cast<uint8_t>(bits[k]) : 0;
    js->nval[t] = static_cast<uint32_t>(nval);
    int c = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        for (int q = 0; q < bits[l]; q++, k++) {
            js->code[t][s.hc[k]] = static_cast<uint16_t>(c++);
            js->len[t][s.hc[k]] = static_cast<uint8_t>(l);
        }
        c <<= 1;
    }
}

// ---------------------------------------------------------------- K5b / K5d shared
struct CodeLds {
    uint8_t len[4][256];
    uint16_t code[4][256];
};

DEVI void load_codes(const h2j_jstat* js, CodeLds& c, bool with_codes) {
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        (&c.len[0][0])[i] = (&js->len[0][0])[i];
        if (with_codes) (&c.code[0][0])[i] = (&js->code[0][0])[i];
    }
}

// bits of block t of a tile: DC code + magnitude, then the AC symbols' codes + magnitudes
DEVI uint32_t block_bits(const CodeLds& c, const uint32_t* sym, int cnt, int t, int dc_diff, int tab) {
    const int nd = nbits16(dc_diff);
    uint32_t bits = c.len[tab][nd] + nd;
    const uint8_t* al = c.len[2 + tab];
    for (int k = 0; k < cnt; k += 8) {  // 8 symbol loads in flight per lane
        uint32_t w[8];
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = k + j < cnt ? sym[(k + j) * kTile + t] : 0u;
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (k + j < cnt) bits += al[w[j] & 0xFF] + ((w[j] >> 8) & 15);
    }
    return bits;
}

// 256-thread workgroup exclusive scan (4 waves of 64)
DEVI uint32_t wg_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
    for (int k = 0; k < kTile / 64; k++) {
        if (k < w) base += sh[k];
        total += sh[k];
    }
    __syncthreads();
    return base + x - v;
}

// ---------------------------------------------------------------- K5b
__global__ void __launch_bounds__(kTile) h2j_k5b_tile_bits(const h2j_frame* frames, uint8_t* arena,
                                                           uint32_t* tile_bits, int max_tiles) {
    const GridPos gp = xcd_grid_pos();
    __shared__ CodeLds cl;
    __shared__ uint32_t sh[kTile / 64];
    const h2j_frame& f = frames[gp.y];
    const int nblk = nblocks(f);
    const int b0 = gp.x * kTile;
    if (b0 >= nblk) return;
    const int nb = min(kTile, nblk - b0);
    const h2j_jstat* js = reinterpret_cast<const h2j_jstat*>(arena + f.jstat);
    const uint8_t* base = arena + f.jcoef;
    const uint8_t* tile = base + static_cast<size_t>(gp.x) * kJTileBytes;
    load_codes(js, cl, false);
    __syncthreads();
    uint32_t bits = 0;
    const int t = threadIdx.x;
    if (t < nb) {
        const int bi = b0 + t;
        bits = block_bits(cl, reinterpret_cast<const uint32_t*>(tile), tile[kJCntOff + t], t,
                          dc_of(base, bi) - prev_dc(base, bi), (bi % 6) < 4 ? 0 : 1);
    }
    uint32_t total;
    wg_excl_scan(bits, sh, total);
    if (threadIdx.x == 0) tile_bits[static_cast<size_t>(gp.y) * max_tiles + gp.x] = total;
}

// ---------------------------------------------------------------- K5c
// grid (nframes): exclusive scan of the frame's tile bit counts in place.
__global__ void __launch_bounds__(kTile) h2j_k5c_scan_tiles(const h2j_frame* frames, uint8_t* arena,
                                                            uint32_t* tile_bits, int max_tiles) {
    __shared__ uint32_t sh[kTile / 64];
    const h2j_frame& f = frames[blockIdx.x];
    const int ntiles = (nblocks(f) + kTile - 1) / kTile;
    uint32_t* tb = tile_bits + static_cast<size_t>(blockIdx.x) * max_tiles;
    uint32_t carry = 0;
    for (int t0 = 0; t0 < ntiles; t0 += kTile) {
        const int t = t0 + threadIdx.x;
        const uint32_t v = t < ntiles ? tb[t] : 0;
        uint32_t total;
        const uint32_t ex = wg_excl_scan(v, sh, total);
        if (t < ntiles) tb[t] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) {
        h2j_jstat* js = reinterpret_cast<h2j_jstat*>(arena + f.jstat);
        js->nbits = carry;
        js->nbytes = (carry + 7) >> 3;
    }
}

// one workgroup: segment offsets of all frames (16-byte aligned) + pool total
__global__ void __launch_bounds__(kTile) h2j_k5c_scan_frames(const h2j_frame* frames, int nframes, uint8_t* arena,
                                                             uint64_t seg_cap, uint64_t* seg_total) {
    __shared__ uint32_t sh[kTile / 64];
    uint64_t carry = 0;
    for (int k0 = 0; k0 < nframes; k0 += kTile) {
        const int k = k0 + threadIdx.x;
        h2j_jstat* js = k < nframes ? reinterpret_cast<h2j_jstat*>(arena + frames[k].jstat) : nullptr;
        // sizes in 16-byte units keep the 32-bit scan exact for any batch
        const uint32_t v = js ? (js->nbytes + 15) >> 4 : 0;
        uint32_t total;
        const uint32_t ex = wg_excl_scan(v, sh, total);
        if (js) {
            const uint64_t off = (carry + ex) << 4;
            js->seg_off = off + (static_cast<uint64_t>(v) << 4) <= seg_cap ? off : ~0ull;
        }
        carry += total;
    }
    if (threadIdx.x == 0) *seg_total = carry << 4 <= seg_cap ? carry << 4 : seg_cap;
}

// ---------------------------------------------------------------- K5z
__global__ void __launch_bounds__(256) h2j_k5z_zero(uint8_t* seg, const uint64_t* seg_total) {
    const uint64_t n = *seg_total >> 4;
    uint4* p = reinterpret_cast<uint4*>(seg);
    const uint4 z = make_uint4(0, 0, 0, 0);
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) p[i] = z;
}

// ---------------------------------------------------------------- K5d
// MSB-first bit writer of one block into 32-bit big-endian words; the block's first word and
// its last partial word may be shared with the neighbouring blocks (OR), the others are its own.
// kLds: words of the workgroup's LDS image of its tile (index word - w0), else global words.
template <bool kLds>
struct BitSink {
    uint32_t* out;
    uint32_t word, w0;
    uint64_t acc;
    int nacc;
    bool first;

    DEVI void store(uint32_t w, bool atomic) {
        const uint32_t be = __builtin_bswap32(w);
        uint32_t* p = out + (kLds ? word - w0 : word);
        if (atomic) atomicOr(p, be);
        else *p = be;
        word++;
    }
    DEVI void put(uint32_t v, int n) {
        acc = (acc << n) | v;
        nacc += n;
        if (nacc >= 32) {
            nacc -= 32;
            store(static_cast<uint32_t>(acc >> nacc), first);
            first = false;
        }
    }
    DEVI void finish() {
        if (nacc > 0) store(static_cast<uint32_t>(acc << (32 - nacc)), true);
    }
};

// A tile's payload is assembled in LDS when it fits (the usual case: a few hundred bytes per
// 256 blocks): the blocks' shared boundary words meet in LDS atomics, and the tile goes out as
// whole-word stores, only its first and last word by global atomics (shared with the
// neighbouring tiles).  Larger tiles write straight to global memory as before.
// 8 KB: with the 3 KB code tables a 256-thread workgroup holds 11 KB, so 8 of them (the wave
// limit) share a CU; a 32 KB image allowed 4, and the kernel waited on its symbol loads with half
// the waves (per 1024 pictures: hevc1080 1.53 -> 0.94 ms, 4K Main10 2.0 -> 0.9 ms)
constexpr int kEmitWords = 2048;

template <bool kLds>
DEVI void emit_block(uint32_t* out, uint32_t w0, uint32_t bit0, uint32_t bits, const CodeLds& cl, const uint32_t* sym,
                     int cnt, int t, int diff, int tab, bool last_block) {
    BitSink<kLds> s;
    s.out = out;
    s.w0 = w0;
    s.word = bit0 >> 5;
    s.acc = 0;
    s.nacc = bit0 & 31;
    s.first = true;
    const int nd = nbits16(diff);
    s.put(cl.code[tab][nd], cl.len[tab][nd]);
    if (nd) s.put(static_cast<uint32_t>(diff < 0 ? diff - 1 : diff) & ((1u << nd) - 1u), nd);
    const uint8_t* al = cl.len[2 + tab];
    const uint16_t* ac = cl.code[2 + tab];
    for (int k = 0; k < cnt; k++) {
        const uint32_t w = sym[k * kTile + t];
        const int sv = static_cast<int>(w & 0xFF), n = static_cast<int>((w >> 8) & 15);
        s.put(ac[sv], al[sv]);
        if (n) s.put(w >> 12, n);
    }
    if (last_block) {
        const int pad = (8 - static_cast<int>((bit0 + bits) & 7)) & 7;  // FFmpeg: pad with 1-bits
        if (pad) s.put((1u << pad) - 1u, pad);
    }
    s.finish();
}

// emit_words: tiles whose payload spans more words take the global-memory path (kEmitWords;
// H2J_EMIT_GLOBAL=1 passes 0, every tile on the global path: coverage of that path in tests)
__global__ void __launch_bounds__(kTile) h2j_k5d_emit(const h2j_frame* frames, uint8_t* arena,
                                                      const uint32_t* tile_bits, int max_tiles, uint8_t* seg,
                                                      int emit_words) {
    const GridPos gp = xcd_grid_pos();
    __shared__ CodeLds cl;
    __shared__ uint32_t sh[kTile / 64];
    __shared__ uint32_t img[kEmitWords];
    const h2j_frame& f = frames[gp.y];
    const int nblk = nblocks(f);
    const int b0 = gp.x * kTile;
    if (b0 >= nblk) return;
    const h2j_jstat* js = reinterpret_cast<const h2j_jstat*>(arena + f.jstat);
    if (js->seg_off == ~0ull) return;  // pool overflow: host reports the frame as failed
    const int nb = min(kTile, nblk - b0);
    const uint8_t* base = arena + f.jcoef;
    const uint8_t* tile = base + static_cast<size_t>(gp.x) * kJTileBytes;
    const uint32_t* sym = reinterpret_cast<const uint32_t*>(tile);
    load_codes(js, cl, true);
    __syncthreads();
    const int t = threadIdx.x;
    const bool mine = t < nb;
    const int bi = b0 + t;
    const int tab = (bi % 6) < 4 ? 0 : 1;
    int diff = 0, cnt = 0;
    uint32_t bits = 0;
    if (mine) {
        diff = dc_of(base, bi) - prev_dc(base, bi);
        cnt = tile[kJCntOff + t];
        bits = block_bits(cl, sym, cnt, t, diff, tab);
    }
    uint32_t total;
    const uint32_t ex = wg_excl_scan(bits, sh, total);
    const uint32_t tile0 = tile_bits[static_cast<size_t>(gp.y) * max_tiles + gp.x];
    const uint32_t bit0 = tile0 + ex;
    uint32_t* out = reinterpret_cast<uint32_t*>(seg + js->seg_off);
    const uint32_t w_lo = tile0 >> 5, w_hi = (tile0 + total + 31) >> 5;
    const int nw = static_cast<int>(w_hi - w_lo);
    if (nw > emit_words) {  // rare: straight to global memory
        if (mine) emit_block<false>(out, 0, bit0, bits, cl, sym, cnt, t, diff, tab, bi == nblk - 1);
        return;
    }
    for (int i = t; i < nw; i += kTile) img[i] = 0;
    __syncthreads();
    if (mine) emit_block<true>(img, w_lo, bit0, bits, cl, sym, cnt, t, diff, tab, bi == nblk - 1);
    __syncthreads();
    for (int i = t; i < nw; i += kTile) {
        const uint32_t v = img[i];
        if (i == 0 || i == nw - 1) {
            if (v) atomicOr(out + w_lo + i, v);
        } else {
            out[w_lo + i] = v;
        }
    }
}

}  // namespace

namespace h2jgpu {  // defined in h2j_kernels.hip: one error slot for the whole C ABI
extern thread_local char g_err[256];
int check(hipError_t e, const char* what);
}  // namespace h2jgpu
using h2jgpu::check;
using h2jgpu::g_err;

extern "C" {

int h2j_gpu_histogram(const h2j_gpu_batch* b, void* stream) {
    if (!b || b->nframes <= 0) return 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int tiles = (b->max_mcu * 6 + kTile - 1) / kTile;
    hipLaunchKernelGGL(h2j_k4e_dc_hist, dim3(tiles, b->nframes), dim3(kTile), 0, s, b->frames, b->arena);
    return check(hipGetLastError(), "h2j_k4e_dc_hist");
}

int h2j_gpu_entropy(const h2j_gpu_batch* b, void* stream) {
    if (!b || b->nframes <= 0) return 0;
    if (!b->seg || !b->tile_bits || !b->seg_total) {
        snprintf(g_err, sizeof(g_err), "h2j_gpu_entropy: segment pool / scratch not set");
        return -1;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int tiles = (b->max_mcu * 6 + kTile - 1) / kTile;
    hipLaunchKernelGGL(h2j_k5a_tables, dim3(4, b->nframes), dim3(64), 0, s, b->frames, b->arena);
    int r = check(hipGetLastError(), "h2j_k5a_tables");
    if (r) return r;
    hipLaunchKernelGGL(h2j_k5b_tile_bits, dim3(tiles, b->nframes), dim3(kTile), 0, s, b->frames, b->arena,
                       b->tile_bits, tiles);
    if ((r = check(hipGetLastError(), "h2j_k5b_tile_bits"))) return r;
    hipLaunchKernelGGL(h2j_k5c_scan_tiles, dim3(b->nframes), dim3(kTile), 0, s, b->frames, b->arena, b->tile_bits,
                       tiles);
    if ((r = check(hipGetLastError(), "h2j_k5c_scan_tiles"))) return r;
    hipLaunchKernelGGL(h2j_k5c_scan_frames, dim3(1), dim3(kTile), 0, s, b->frames, b->nframes, b->arena, b->seg_cap,
                       b->seg_total);
    if ((r = check(hipGetLastError(), "h2j_k5c_scan_frames"))) return r;
    hipLaunchKernelGGL(h2j_k5z_zero, dim3(1024), dim3(256), 0, s, b->seg, b->seg_total);
    if ((r = check(hipGetLastError(), "h2j_k5z_zero"))) return r;
    const char* eg = std::getenv("H2J_EMIT_GLOBAL");  // read per launch: tests switch it inside one process
    const int emit_words = (eg && eg[0] == '1') ? 0 : kEmitWords;
    hipLaunchKernelGGL(h2j_k5d_emit, dim3(tiles, b->nframes), dim3(kTile), 0, s, b->frames, b->arena, b->tile_bits,
                       tiles, b->seg, emit_words);
    return check(hipGetLastError(), "h2j_k5d_emit");
}

}  // extern "C"
