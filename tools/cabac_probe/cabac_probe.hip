// GPU arithmetic-decoder probe ("entropy decoding on the GPU"): how fast one wave
// runs the CABAC decision chain (H.265 9.3.4.3.2) on gfx950, to size a device-side entropy stage
// against the host threads that set the end-to-end number today.
//
// Every stream decodes N context-coded bins from real HEVC slice bytes (tests/golden/bench) with a
// data-dependent context pattern (64 contexts; the index depends on the bin position and on the
// previous bin, like the significance / greater1 loops).  Three placements of the decoder:
//   S  one stream per wave, everything wave-uniform: engine state in SGPRs (SALU), contexts and
//      next-state tables in LDS (uniform ds_read + readfirstlane)
//   R  one stream per wave, contexts and next-state tables held in VGPR lanes (v_readlane /
//      v_writelane with the context index in an SGPR), engine state in SGPRs
//   V  64 streams per wave, one per lane (the lock-step bound: a real parser would diverge)
// The host decodes the same streams with the same step function and checks every checksum.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../h264-h265-to-jpeg_amd/csrc/host \
//       cabac_probe.hip ../../h264-h265-to-jpeg_amd/csrc/host/cabac_tables.cpp -o cabac_probe
//   ./cabac_probe ../../tests/golden/bench/*.h265
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "cabac.h"

#define HD __host__ __device__ __forceinline__

namespace {

constexpr int kCtx = 64;
constexpr int kBins = 100000;

struct Eng {
    uint32_t value, range;
    int bits;
    uint32_t pos;  // next 16-bit half of the stream (words hold two, big-endian order)
};

HD uint32_t clz32(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __clz(x);
#else
    return __builtin_clz(x);
#endif
}

HD void eng_init(Eng& e, const uint32_t* w, uint32_t pos) {
    e.value = w[pos >> 1];
    e.pos = pos + 2;
    e.range = 510;
    e.bits = 23;
}

// One context-coded bin.  The context is (lps4, st): lps4 holds rangeTabLps[pStateIdx][0..3] as
// bytes, st = (pStateIdx << 1) | valMps; nm* / nl* are the context after an MPS / LPS bin, looked
// up by the caller from st (off the dependent chain).  32-bit window: value = offset << bits |
// look-ahead, refilled 16 bits at a time when bits goes negative (value < 2^31 throughout).
HD int step(Eng& e, uint32_t& lps4, uint32_t& st, uint32_t nml, uint32_t nms, uint32_t nll, uint32_t nls,
            const uint32_t* w) {
    const uint32_t lps = (lps4 >> ((e.range >> 3) & 24)) & 0xffu;
    const uint32_t rmps = e.range - lps;
    const uint32_t scaled = rmps << e.bits;
    const uint32_t msh = (rmps >> 8) ^ 1u;
    const uint32_t lsh = clz32(lps) - 23u;
    const bool L = e.value >= scaled;
    const int bin = static_cast<int>((st & 1u) ^ (L ? 1u : 0u));
    e.value = L ? e.value - scaled : e.value;
    e.range = L ? lps << lsh : rmps << msh;
    e.bits -= static_cast<int>(L ? lsh : msh);
    lps4 = L ? nll : nml;
    st = L ? nls : nms;
    if (e.bits < 0) {
        const uint32_t word = w[e.pos >> 1];
        const uint32_t h = (e.pos & 1u) ? (word & 0xffffu) : (word >> 16);
        e.value = (e.value << 16) | h;
        e.bits += 16;
        e.pos++;
    }
    return bin;
}

HD int ctx_index(int i, int prev) {
    // significance-map-like: runs of positions sharing a context, the previous bin selects a pair
    const int pat = (i & 15) < 10 ? 0 : ((i & 15) < 15 ? 1 : 2);
    return ((i >> 4) & 7) * 8 + pat * 2 + prev;
}

// tables: [0] lps4 after MPS, [1] st after MPS, [2] lps4 after LPS, [3] st after LPS; [4] lps4 of st
struct Tabs {
    uint32_t t[5][128];
};

Tabs make_tabs() {
    Tabs T;
    for (int s = 0; s < 128; s++) {
        const int p = s >> 1, m = s & 1;
        auto lps4 = [](int ps) {
            return static_cast<uint32_t>(h2j::kCabacLps[ps][0]) | (static_cast<uint32_t>(h2j::kCabacLps[ps][1]) << 8) |
                   (static_cast<uint32_t>(h2j::kCabacLps[ps][2]) << 16) | (static_cast<uint32_t>(h2j::kCabacLps[ps][3]) << 24);
        };
        const int pm = std::min(p + 1, 62);
        const int pl = h2j::kCabacTransLps[p];
        const int ml = p == 0 ? 1 - m : m;
        T.t[0][s] = lps4(pm);
        T.t[1][s] = static_cast<uint32_t>((pm << 1) | m);
        T.t[2][s] = lps4(pl);
        T.t[3][s] = static_cast<uint32_t>((pl << 1) | ml);
        T.t[4][s] = lps4(p);
    }
    return T;
}

HD uint32_t init_st(int k) { return static_cast<uint32_t>(((20 + (k * 7) % 40) << 1) | (k & 1)); }

// ---- S: one stream per wave, uniform state, LDS contexts ----
__global__ __launch_bounds__(64) void k_s(const uint32_t* __restrict__ w, const uint32_t* __restrict__ start,
                                         const Tabs* __restrict__ tabs, uint32_t* __restrict__ out, int nbins) {
    __shared__ uint32_t T[4][128];
    __shared__ uint32_t cl[kCtx], cs[kCtx];
    for (int i = threadIdx.x; i < 4 * 128; i += 64) T[i >> 7][i & 127] = tabs->t[i >> 7][i & 127];
    for (int k = threadIdx.x; k < kCtx; k += 64) {
        cs[k] = init_st(k);
        cl[k] = tabs->t[4][init_st(k)];
    }
    __syncthreads();
    Eng e;
    eng_init(e, w, start[blockIdx.x]);
    uint32_t sum = 0;
    int prev = 0;
    for (int i = 0; i < nbins; i++) {
        const int k = ctx_index(i, prev);
        uint32_t l4 = cl[k], st = cs[k];
        const int b = step(e, l4, st, T[0][st], T[1][st], T[2][st], T[3][st], w);
        cl[k] = l4;
        cs[k] = st;
        sum = sum * 3u + static_cast<uint32_t>(b);
        prev = b;
    }
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = sum;
        out[2 * blockIdx.x + 1] = e.pos;
    }
}

// ---- R: one stream per wave, contexts and tables in VGPR lanes ----
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ uint32_t wl(uint32_t val, uint32_t lane, uint32_t v) {
    // gfx9: one SGPR per VALU instruction from the constant bus, so the lane select goes in M0
    asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(val), "s"(lane) : "m0");
    return v;
}

__global__ __launch_bounds__(64) void k_r(const uint32_t* __restrict__ w, const uint32_t* __restrict__ start,
                                         const Tabs* __restrict__ tabs, uint32_t* __restrict__ out, int nbins) {
    const int ln = threadIdx.x;
    // next-state tables: entry s in lane s & 63 of the register for s >> 6
    uint32_t t[4][2];
    for (int j = 0; j < 4; j++) {
        t[j][0] = tabs->t[j][ln];
        t[j][1] = tabs->t[j][64 + ln];
    }
    uint32_t vcs = init_st(ln);
    uint32_t vcl = tabs->t[4][vcs];
    Eng e;
    eng_init(e, w, start[blockIdx.x]);
    uint32_t sum = 0;
    int prev = 0;
    for (int i = 0; i < nbins; i++) {
        const uint32_t k = static_cast<uint32_t>(ctx_index(i, prev));
        uint32_t l4 = rl(vcl, k), st = rl(vcs, k);
        const uint32_t hi = st >> 6, lo = st & 63u;
        const uint32_t nml = hi ? rl(t[0][1], lo) : rl(t[0][0], lo);
        const uint32_t nms = hi ? rl(t[1][1], lo) : rl(t[1][0], lo);
        const uint32_t nll = hi ? rl(t[2][1], lo) : rl(t[2][0], lo);
        const uint32_t nls = hi ? rl(t[3][1], lo) : rl(t[3][0], lo);
        const int b = step(e, l4, st, nml, nms, nll, nls, w);
        vcl = wl(l4, k, vcl);
        vcs = wl(st, k, vcs);
        sum = sum * 3u + static_cast<uint32_t>(b);
        prev = b;
    }
    if (ln == 0) {
        out[2 * blockIdx.x] = sum;
        out[2 * blockIdx.x + 1] = e.pos;
    }
}

// ---- V: one stream per lane ----
__global__ __launch_bounds__(64) void k_v(const uint32_t* __restrict__ w, const uint32_t* __restrict__ start,
                                         const Tabs* __restrict__ tabs, uint32_t* __restrict__ out, int nbins) {
    __shared__ uint32_t T[4][128];
    __shared__ uint32_t cl[kCtx][64], cs[kCtx][64];
    const int ln = threadIdx.x;
    for (int i = ln; i < 4 * 128; i += 64) T[i >> 7][i & 127] = tabs->t[i >> 7][i & 127];
    for (int k = 0; k < kCtx; k++) {
        cs[k][ln] = init_st(k);
        cl[k][ln] = tabs->t[4][init_st(k)];
    }
    __syncthreads();
    const int sid = blockIdx.x * 64 + ln;
    Eng e;
    eng_init(e, w, start[sid]);
    uint32_t sum = 0;
    int prev = 0;
    for (int i = 0; i < nbins; i++) {
        const int k = ctx_index(i, prev);
        uint32_t l4 = cl[k][ln], st = cs[k][ln];
        const int b = step(e, l4, st, T[0][st], T[1][st], T[2][st], T[3][st], w);
        cl[k][ln] = l4;
        cs[k][ln] = st;
        sum = sum * 3u + static_cast<uint32_t>(b);
        prev = b;
    }
    out[2 * sid] = sum;
    out[2 * sid + 1] = e.pos;
}

void host_decode(const uint32_t* w, uint32_t start, const Tabs& T, int nbins, uint32_t& sum_out, uint32_t& pos_out) {
    uint32_t cl[kCtx], cs[kCtx];
    for (int k = 0; k < kCtx; k++) {
        cs[k] = init_st(k);
        cl[k] = T.t[4][cs[k]];
    }
    Eng e;
    eng_init(e, w, start);
    uint32_t sum = 0;
    int prev = 0;
    for (int i = 0; i < nbins; i++) {
        const int k = ctx_index(i, prev);
        uint32_t l4 = cl[k], st = cs[k];
        const int b = step(e, l4, st, T.t[0][st], T.t[1][st], T.t[2][st], T.t[3][st], w);
        cl[k] = l4;
        cs[k] = st;
        sum = sum * 3u + static_cast<uint32_t>(b);
        prev = b;
    }
    sum_out = sum;
    pos_out = e.pos;
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t err_ = (x);                                                       \
        if (err_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

}  // namespace

int main(int argc, char** argv) {
    std::vector<uint8_t> bytes;
    for (int a = 1; a < argc; a++) {
        FILE* f = std::fopen(argv[a], "rb");
        if (!f) continue;
        uint8_t buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) bytes.insert(bytes.end(), buf, buf + n);
        std::fclose(f);
    }
    if (bytes.size() < (1u << 20)) {
        std::fprintf(stderr, "need >= 1 MB of stream bytes\n");
        return 2;
    }
    std::vector<uint32_t> words(bytes.size() / 4);
    for (size_t i = 0; i < words.size(); i++)
        words[i] = (static_cast<uint32_t>(bytes[4 * i]) << 24) | (static_cast<uint32_t>(bytes[4 * i + 1]) << 16) |
                   (static_cast<uint32_t>(bytes[4 * i + 2]) << 8) | bytes[4 * i + 3];
    const Tabs T = make_tabs();
    // 100k bins consume < 64k halves (measured max ~ 9k words); stream starts spread over the data
    const uint32_t span = static_cast<uint32_t>(words.size() - 40000) * 2u;
    const int max_streams = 4096 * 64;
    std::vector<uint32_t> start(max_streams);
    for (int s = 0; s < max_streams; s++) start[s] = static_cast<uint32_t>((static_cast<uint64_t>(s) * 7919u * 2u) % span);

    uint32_t *dw, *dstart, *dout;
    Tabs* dtabs;
    CK(hipMalloc(&dw, words.size() * 4));
    CK(hipMalloc(&dstart, start.size() * 4));
    CK(hipMalloc(&dout, static_cast<size_t>(max_streams) * 8));
    CK(hipMalloc(&dtabs, sizeof(Tabs)));
    CK(hipMemcpy(dw, words.data(), words.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dstart, start.data(), start.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtabs, &T, sizeof(Tabs), hipMemcpyHostToDevice));

    // host reference for the checked streams, and the host's own ns per bin (one thread)
    const int nchk = 1024;
    std::vector<uint32_t> ref(2 * nchk);
    const auto h0 = std::chrono::steady_clock::now();
    for (int s = 0; s < nchk; s++) host_decode(words.data(), start[s], T, kBins, ref[2 * s], ref[2 * s + 1]);
    const double host_ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - h0).count() /
                           (static_cast<double>(nchk) * kBins);
    std::printf("host one thread: %.2f ns/bin (same step function)\n", host_ns);

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint32_t> out(2 * static_cast<size_t>(max_streams));
    const char* names = "SRV";
    for (int v = 0; v < 3; v++) {
        for (int waves : {256, 1024, 2048, 4096}) {
            if (v == 2 && waves > 1024) continue;
            const int streams = v == 2 ? waves * 64 : waves;
            float best = 1e30f;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipEventRecord(e0));
                if (v == 0) k_s<<<waves, 64>>>(dw, dstart, dtabs, dout, kBins);
                if (v == 1) k_r<<<waves, 64>>>(dw, dstart, dtabs, dout, kBins);
                if (v == 2) k_v<<<waves, 64>>>(dw, dstart, dtabs, dout, kBins);
                CK(hipGetLastError());
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            CK(hipMemcpy(out.data(), dout, static_cast<size_t>(streams) * 8, hipMemcpyDeviceToHost));
            int bad = 0;
            for (int s = 0; s < std::min(streams, nchk); s++)
                if (out[2 * s] != ref[2 * s] || out[2 * s + 1] != ref[2 * s + 1]) bad++;
            const double bins = static_cast<double>(streams) * kBins;
            std::printf("%c waves %5d streams %6d: %8.3f ms  %7.2f ns/bin per stream  %6.2f Gbin/s  mismatches %d\n",
                        names[v], waves, streams, best, best * 1e6 / kBins, bins / (best * 1e6), bad);
        }
    }
    return 0;
}
