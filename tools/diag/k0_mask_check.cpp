// HEVC K0 availability masks (r06): the closed form h2j_k0_prep uses for pictures without slices /
// tiles (h2j_kernels.hip, "geometry alone, in closed form") against the per-unit loop it replaced,
// on every aligned TB position of 8..200 x 8..136 pictures at CTB 16 / 32 / 64, luma and chroma.
//   g++ -O2 -o /tmp/k0_mask_check tools/diag/k0_mask_check.cpp && /tmp/k0_mask_check
// (r06n: 971658 cases, 0 mismatches)
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
using namespace std;
static int zorder4(int ax, int ay) { int z = 0; for (int b = 0; b < 5; b++) z |= ((ax >> b) & 1) << (2 * b) | ((ay >> b) & 1) << (2 * b + 1); return z; }
struct F { int log2ctb, ctb_w, width, height; };
static uint64_t old_mask(const F& f, int ox0, int oy0, int log2n, int oc) {
    const int on = 1 << log2n, oshc = oc ? 1 : 0, oxl = ox0 << oshc, oyl = oy0 << oshc;
    const int ocb = (oyl >> f.log2ctb) * f.ctb_w + (oxl >> f.log2ctb);
    uint64_t mask = 0;
    const int u = oc ? 2 : 4, nu = (2 * on) / u;
    const int l2 = f.log2ctb, m = (1 << l2) - 1;
    const int zc = zorder4((oxl & m) >> 2, (oyl & m) >> 2);
    for (int q = 0; q <= 2 * nu; q++) {
        int xn, yn;
        if (q < nu) { xn = ox0 - 1; yn = oy0 + 2 * on - 1 - q * u; }
        else if (q == nu) { xn = ox0 - 1; yn = oy0 - 1; }
        else { xn = ox0 + (q - nu - 1) * u; yn = oy0 - 1; }
        const int xnl = xn << oshc, ynl = yn << oshc;
        bool a = false;
        if (xnl >= 0 && ynl >= 0 && xnl < f.width && ynl < f.height) {
            const int cn = (ynl >> l2) * f.ctb_w + (xnl >> l2);
            a = cn == ocb ? zorder4((xnl & m) >> 2, (ynl & m) >> 2) <= zc : cn < ocb;
        }
        mask |= static_cast<uint64_t>(a) << q;
    }
    return mask;
}
static uint64_t new_mask(const F& f, int ox0, int oy0, int log2n, int oc) {
    const int on = 1 << log2n, oshc = oc ? 1 : 0, oxl = ox0 << oshc, oyl = oy0 << oshc;
    const int ocb = (oyl >> f.log2ctb) * f.ctb_w + (oxl >> f.log2ctb);
    uint64_t mask = 0;
    const int u = oc ? 2 : 4, nu = (2 * on) / u;
    const int l2 = f.log2ctb, m = (1 << l2) - 1;
    const int zc = zorder4((oxl & m) >> 2, (oyl & m) >> 2);
    auto geo = [&](int xn, int yn) {
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
    if (geo(ox0 - 1, oy0 + on + u - 1)) { const int fit = min(nh, (Hc - oy0 - on) / u); mask |= ((1ull << fit) - 1) << (nh - fit); }
    if (geo(ox0 + on, oy0 - 1)) { const int fit = min(nh, (Wc - ox0 - on + u - 1) / u); mask |= ((1ull << fit) - 1) << (nu + nh + 1); }
    return mask;
}
int main() {
    long n = 0, bad = 0;
    for (int l2c = 4; l2c <= 6; l2c++)
    for (int W = 8; W <= 200; W += 8) for (int H = 8; H <= 136; H += 8) {
        F f{l2c, (W + (1 << l2c) - 1) >> l2c, W, H};
        for (int c = 0; c < 2; c++) for (int log2n = 2; log2n <= 5; log2n++) {
            const int on = 1 << log2n, sh = c;
            if ((on << sh) > (1 << l2c)) continue;
            if (c && log2n == 5) continue;
            for (int y = 0; y + on <= (H >> sh); y += on) for (int x = 0; x + on <= (W >> sh); x += on) {
                n++;
                uint64_t a = old_mask(f, x, y, log2n, c), b = new_mask(f, x, y, log2n, c);
                if (a != b) { if (bad++ < 10) printf("ctb %d W %d H %d c %d n %d (%d,%d): %llx vs %llx\n", l2c, W, H, c, on, x, y, (unsigned long long)a, (unsigned long long)b); }
            }
        }
    }
    printf("%ld cases, %ld mismatches\n", n, bad);
}
