// D2H copy rate probe (profiles/r05_4k_d2h.md): hipMemcpyAsync device -> pinned host of N MB,
// first copy into a fresh pinned buffer and repeats, timed with HIP events.
//   hipcc -O2 d2h_probe.cpp -o d2h_probe && ./d2h_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

static float copy_ms(void* dst, const void* src, size_t n, hipStream_t s, hipEvent_t a, hipEvent_t b) {
    hipEventRecord(a, s);
    hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const size_t sizes[] = {8u << 20, 32u << 20, 64u << 20, 128u << 20, 256u << 20};
    void* d = nullptr;
    if (hipMalloc(&d, 256u << 20) != hipSuccess) return 1;
    hipMemset(d, 1, 256u << 20);
    for (size_t n : sizes) {
        void* h = nullptr;
        if (hipHostMalloc(&h, n, hipHostMallocDefault) != hipSuccess) return 2;
        const float f0 = copy_ms(h, d, n, s, a, b);
        float best = 1e9f, worst = 0;
        for (int r = 0; r < 5; r++) {
            const float t = copy_ms(h, d, n, s, a, b);
            best = t < best ? t : best;
            worst = t > worst ? t : worst;
        }
        // the same after the host has read the buffer (pages touched by the CPU)
        volatile unsigned sum = 0;
        for (size_t i = 0; i < n; i += 4096) sum += static_cast<unsigned char*>(h)[i];
        const float f2 = copy_ms(h, d, n, s, a, b);
        std::printf("%4zu MB: first %.2f ms (%.1f GB/s), repeat best %.2f (%.1f GB/s) worst %.2f, after host read %.2f (%.1f GB/s)\n",
                    n >> 20, f0, n / f0 / 1e6, best, n / best / 1e6, worst, f2, n / f2 / 1e6);
        hipHostFree(h);
    }
    hipFree(d);
    return 0;
}
