// K4c packed FDCT (r06): the column-pair restatement fdct_ap922_pk uses (wrapping int16 halves, rows by dot2)
// against the saturating AP-922 scalar form (fdct_ap922) on 4 M random and extreme 0 / 255 blocks.
//   g++ -O2 -o /tmp/fdct_pk_check tools/diag/fdct_pk_check.cpp && /tmp/fdct_pk_check   (r06: 0 mismatches, max 32640)
// host check: packed-pair restatement (wrapping int16, no saturation, dot2 rows) == AP922 scalar with saturation, inputs 0..255
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <random>
static int16_t sat16(int v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }
static int16_t mulhi16(int a, int c) { return (int16_t)((a * c) >> 16); }
static void ref(int16_t* b) {
    int16_t t[64];
    for (int x = 0; x < 8; x++) {
        const int x0 = b[x], x1 = b[8 + x], x2 = b[16 + x], x3 = b[24 + x], x4 = b[32 + x], x5 = b[40 + x], x6 = b[48 + x], x7 = b[56 + x];
        const int16_t t0 = sat16(sat16(x0 + x7) * 8), t1 = sat16(sat16(x1 + x6) * 8);
        const int16_t t2 = sat16(sat16(x2 + x5) * 8), t3 = sat16(sat16(x3 + x4) * 8);
        const int16_t tp03 = sat16(t0 + t3), tm03 = sat16(t0 - t3), tp12 = sat16(t1 + t2), tm12 = sat16(t1 - t2);
        t[x] = sat16(tp03 + tp12);
        t[32 + x] = sat16(tp03 - tp12);
        t[16 + x] = (int16_t)(sat16(tm03 + mulhi16(tm12, 27146)) | 1);
        t[48 + x] = (int16_t)(sat16(mulhi16(tm03, 27146) - tm12) | 1);
        const int16_t d16 = sat16(sat16(x1 - x6) * 16), d25 = sat16(sat16(x2 - x5) * 16);
        const int16_t tp65 = (int16_t)(mulhi16(sat16(d16 + d25), 23170) | 1);
        const int16_t tm65 = mulhi16(sat16(d16 - d25), 23170);
        const int16_t t4 = sat16(sat16(x3 - x4) * 8), t7 = sat16(sat16(x0 - x7) * 8);
        const int16_t tp465 = sat16(t4 + tm65), tm465 = sat16(t4 - tm65);
        const int16_t tp765 = sat16(t7 + tp65), tm765 = sat16(t7 - tp65);
        t[8 + x] = (int16_t)(sat16(tp765 + mulhi16(tp465, 13036)) | 1);
        t[56 + x] = sat16(mulhi16(tp765, 13036) - tp465);
        t[24 + x] = sat16(tm765 - sat16(mulhi16(tm465, -21746) + tm465));
        t[40 + x] = sat16(sat16(mulhi16(tm765, -21746) + tm765) + tm465);
    }
    const int kRow[4][7] = {{22725, 21407, 19266, 16384, 12873, 8867, 4520}, {31521, 29692, 26722, 22725, 17855, 12299, 6270},
                            {29692, 27969, 25172, 21407, 16819, 11585, 5906}, {26722, 25172, 22654, 19266, 15137, 10426, 5315}};
    const int kSel[8] = {0, 1, 2, 3, 0, 3, 2, 1};
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
        for (int k = 0; k < 8; k++) b[r * 8 + k] = sat16((Y[k] + 65536) >> 17);
    }
}
// the packed form: wrapping int16 halves, mulhi per half, rows by dot2 (int32 accumulate)
static int16_t w16(int v) { return (int16_t)(uint16_t)(v & 0xFFFF); }
static int16_t mh(int16_t a, int c) { return (int16_t)(((int)a * c) >> 16); }
static int dot2(int16_t a0, int16_t a1, int16_t b0, int16_t b1, int acc) { return acc + a0 * b0 + a1 * b1; }
static long long maxabs = 0;
static int16_t W(int v) { if (llabs(v) > maxabs) maxabs = llabs(v); return w16(v); }
static void pk(int16_t* b) {
    int16_t t[64];
    for (int x = 0; x < 8; x++) {
        const int16_t x0 = b[x], x1 = b[8 + x], x2 = b[16 + x], x3 = b[24 + x], x4 = b[32 + x], x5 = b[40 + x], x6 = b[48 + x], x7 = b[56 + x];
        const int16_t t0 = W(W(x0 + x7) << 3), t1 = W(W(x1 + x6) << 3), t2 = W(W(x2 + x5) << 3), t3 = W(W(x3 + x4) << 3);
        const int16_t tp03 = W(t0 + t3), tm03 = W(t0 - t3), tp12 = W(t1 + t2), tm12 = W(t1 - t2);
        t[x] = W(tp03 + tp12);
        t[32 + x] = W(tp03 - tp12);
        t[16 + x] = W(W(tm03 + mh(tm12, 27146)) | 1);
        t[48 + x] = W(W(mh(tm03, 27146) - tm12) | 1);
        const int16_t d16 = W(W(x1 - x6) << 4), d25 = W(W(x2 - x5) << 4);
        const int16_t tp65 = W(mh(W(d16 + d25), 23170) | 1), tm65 = mh(W(d16 - d25), 23170);
        const int16_t t4 = W(W(x3 - x4) << 3), t7 = W(W(x0 - x7) << 3);
        const int16_t tp465 = W(t4 + tm65), tm465 = W(t4 - tm65), tp765 = W(t7 + tp65), tm765 = W(t7 - tp65);
        t[8 + x] = W(W(tp765 + mh(tp465, 13036)) | 1);
        t[56 + x] = W(mh(tp765, 13036) - tp465);
        t[24 + x] = W(tm765 - W(mh(tm465, -21746) + tm465));
        t[40 + x] = W(W(mh(tm765, -21746) + tm765) + tm465);
    }
    const int kRow[4][7] = {{22725, 21407, 19266, 16384, 12873, 8867, 4520}, {31521, 29692, 26722, 22725, 17855, 12299, 6270},
                            {29692, 27969, 25172, 21407, 16819, 11585, 5906}, {26722, 25172, 22654, 19266, 15137, 10426, 5315}};
    const int kSel[8] = {0, 1, 2, 3, 0, 3, 2, 1};
    for (int r = 0; r < 8; r++) {
        const int* cc = kRow[kSel[r]];
        const int16_t C1 = cc[0], C2 = cc[1], C3 = cc[2], C4 = cc[3], C5 = cc[4], C6 = cc[5], C7 = cc[6];
        const int16_t* x = t + r * 8;
        const int16_t s0 = W(x[0] + x[7]), s1 = W(x[1] + x[6]), s2 = W(x[2] + x[5]), s3 = W(x[3] + x[4]);
        const int16_t d0 = W(x[0] - x[7]), d1 = W(x[1] - x[6]), d2 = W(x[2] - x[5]), d3 = W(x[3] - x[4]);
        int Y[8];
        Y[0] = dot2(s2, s3, C4, C4, dot2(s0, s1, C4, C4, 0));
        Y[4] = dot2(s2, s3, (int16_t)-C4, C4, dot2(s0, s1, C4, (int16_t)-C4, 0));
        Y[2] = dot2(s2, s3, (int16_t)-C6, (int16_t)-C2, dot2(s0, s1, C2, C6, 0));
        Y[6] = dot2(s2, s3, C2, (int16_t)-C6, dot2(s0, s1, C6, (int16_t)-C2, 0));
        Y[1] = dot2(d2, d3, C5, C7, dot2(d0, d1, C1, C3, 0));
        Y[3] = dot2(d2, d3, (int16_t)-C1, (int16_t)-C5, dot2(d0, d1, C3, (int16_t)-C7, 0));
        Y[5] = dot2(d2, d3, C7, C3, dot2(d0, d1, C5, (int16_t)-C1, 0));
        Y[7] = dot2(d2, d3, C3, (int16_t)-C1, dot2(d0, d1, C7, (int16_t)-C5, 0));
        for (int k = 0; k < 8; k++) b[r * 8 + k] = W((Y[k] + 65536) >> 17);
    }
}
int main() {
    std::mt19937 g(7);
    long bad = 0;
    for (long it = 0; it < 4000000; it++) {
        int16_t a[64], c[64];
        const int mode = it % 4;
        for (int i = 0; i < 64; i++) {
            int v = mode == 0 ? g() % 256 : mode == 1 ? (g() & 1) * 255 : mode == 2 ? ((g() % 4) == 0 ? 255 : 0) : (g() % 2 ? 255 - (g() % 8) : g() % 8);
            a[i] = c[i] = (int16_t)v;
        }
        ref(a); pk(c);
        for (int i = 0; i < 64; i++) if (a[i] != c[i]) { if (bad++ < 5) printf("mismatch it %ld i %d %d %d\n", it, i, a[i], c[i]); break; }
    }
    // every 0/255 column pattern in a fixed row pattern sweep
    printf("mismatches %ld, max |intermediate| %lld\n", bad, maxabs);
}
