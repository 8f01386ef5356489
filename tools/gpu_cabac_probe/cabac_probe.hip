// Feasibility probe for DESIGN §9.1 (entropy decode on the GPU): how fast one wave runs a CABAC
// context-coded decision chain, and how many such chains the chip runs at once.  Each workgroup
// (one wave) decodes `nbins` context-coded bins from its own byte stream with the H.265 9.3.4.3.2
// arithmetic (the spec's rangeTabLps and transIdx tables), 64 contexts in LDS, the context of bin
// k chosen from bin k-1 (a dependent chain, like the significance / greater1 syntax).  Wave-uniform
// control flow: the engine state lives in scalar registers, the stream is read through scalar loads.
// Not product code: the parse stays on the host.
//   hipcc --offload-arch=gfx950 -O3 -o cabac_probe cabac_probe.hip && ./cabac_probe STREAM.h265
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__constant__ unsigned char kLps[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158},  {90, 110, 130, 150},
    {85, 104, 123, 142},  {81, 99, 117, 135},   {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},
    {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},     {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},     {41, 50, 59, 69},
    {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},     {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},
    {23, 28, 33, 39},     {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},     {14, 18, 21, 24},
    {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},     {12, 14, 17, 20},     {11, 14, 16, 19},
    {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},      {9, 11, 12, 14},
    {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
__constant__ unsigned char kNextLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                           13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                           24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                           33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

__global__ void __launch_bounds__(64) probe(const unsigned* __restrict__ words, size_t stride_words, int nbins,
                                            unsigned* out) {
    __shared__ unsigned char cs[64];  // context: (pStateIdx << 1) | valMps
    __shared__ unsigned char lpsT[64][4], nxT[64];  // the tables in LDS (byte loads cannot go through the scalar unit)
    const int lane = threadIdx.x;
    cs[lane] = static_cast<unsigned char>((((lane * 7) % 40) << 1) | (lane & 1));
    for (int q = 0; q < 4; q++) lpsT[lane][q] = kLps[lane][q];
    nxT[lane] = kNextLps[lane];
    __syncthreads();
    // the stream as big-endian 32-bit words, read through uniform (scalar) loads one word ahead
    const unsigned* W = words + static_cast<size_t>(blockIdx.x % 64) * stride_words;
    unsigned wcur = __builtin_bswap32(W[0]), wnext = __builtin_bswap32(W[1]);
    int wpos = 2, wbits = 32;
    auto byte = [&]() __attribute__((always_inline)) {
        const unsigned b = wcur >> 24;
        wcur <<= 8;
        wbits -= 8;
        if (wbits == 0) {
            wcur = wnext;
            wnext = __builtin_bswap32(W[wpos++]);
            wbits = 32;
        }
        return b;
    };
    unsigned range = 510, value = (byte() << 16) | (byte() << 8) | byte();
    int bits = 15;  // look-ahead bits below the 9-bit offset window
    unsigned ctx = 0, acc = 0;
    for (int k = 0; k < nbins; k++) {
        if (bits < 8) {
            value = (value << 8) | byte();
            bits += 8;
        }
        const unsigned c = __builtin_amdgcn_readfirstlane(cs[ctx]);
        const unsigned s = c >> 1, m = c & 1;
        const unsigned lps = __builtin_amdgcn_readfirstlane(lpsT[s][(range >> 6) & 3]);
        range -= lps;
        const unsigned scaled = range << bits;
        unsigned bin, nc;
        if (value < scaled) {  // MPS
            bin = m;
            nc = ((s < 62 ? s + 1 : 62) << 1) | m;
            if (range < 256) {
                range <<= 1;
                bits--;
            }
        } else {  // LPS
            value -= scaled;
            bin = m ^ 1u;
            nc = (static_cast<unsigned>(nxT[s]) << 1) | (s == 0 ? m ^ 1u : m);
            const int n = __builtin_clz(lps) - 23;  // renormalise the 9-bit range
            range = lps << n;
            bits -= n;
        }
        cs[ctx] = static_cast<unsigned char>(nc);
        acc = acc * 31u + bin;
        ctx = ((ctx << 1) | bin) & 63u;
    }
    if (lane == 0) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    std::vector<unsigned char> buf;
    if (argc > 1) {
        FILE* f = std::fopen(argv[1], "rb");
        if (!f) return 1;
        unsigned char tmp[65536];
        size_t n;
        while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
        std::fclose(f);
    }
    if (buf.size() < 4096) { buf.resize(1 << 20); for (size_t i = 0; i < buf.size(); i++) buf[i] = static_cast<unsigned char>((i * 2654435761u) >> 13); }
    const size_t len = (buf.size() + 3) / 4 * 4 + 64;
    buf.resize(len);
    std::vector<unsigned char> rep(len * 64);
    for (int i = 0; i < 64; i++) for (size_t j = 0; j < len; j++) rep[i * len + j] = buf[(j + i * 977) % len];
    unsigned char* d;
    unsigned* o;
    CHECK(hipMalloc(&d, rep.size()));
    CHECK(hipMalloc(&o, 65536 * sizeof(unsigned)));
    CHECK(hipMemcpy(d, rep.data(), rep.size(), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int nbins = 200000;
    hipLaunchKernelGGL(probe, dim3(64), dim3(64), 0, 0, reinterpret_cast<const unsigned*>(d), len / 4, 1000, o);  // warm-up
    CHECK(hipDeviceSynchronize());
    std::printf("waves  ms      ns/bin/wave  Gbins/s (all waves)\n");
    for (int waves : {1, 256, 1024, 2048, 4096, 8192}) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(probe, dim3(waves), dim3(64), 0, 0, reinterpret_cast<const unsigned*>(d), len / 4, nbins, o);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        std::printf("%5d  %7.2f  %8.1f  %8.3f\n", waves, ms, ms * 1e6 / nbins, static_cast<double>(waves) * nbins / (ms * 1e-3) / 1e9);
        std::fflush(stdout);
    }
    unsigned h = 0;
    CHECK(hipMemcpy(&h, o, 4, hipMemcpyDeviceToHost));
    std::printf("checksum %08x\n", h);
    return 0;
}
