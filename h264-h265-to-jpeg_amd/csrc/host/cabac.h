// Context-adaptive binary arithmetic decoder (H.264 9.3.3.2 / H.265 9.3.4.3)
// for the host entropy threads.
#pragma once
#include <cstdint>

namespace h2j {

#ifdef H2J_CABAC_COUNT  // diagnostics (tools/parse_bench): bins decoded by this thread
extern thread_local unsigned long long g_bins_ctx, g_bins_byp;
#define H2J_COUNT(v, n) (v += (n))
#else
#define H2J_COUNT(v, n) ((void)0)
#endif

// Tables are internal to the library: hidden, so the -fPIC code reaches them RIP-relative and not
// through a GOT load that held a register in the bin loops.
#pragma GCC visibility push(hidden)
extern const uint8_t kCabacLps[64][4];
extern const uint8_t kCabacTransLps[64];
extern const uint8_t kCabacRenorm[32];
// next context state ((pStateIdx << 1) | valMps) after an MPS / LPS bin
extern const uint16_t kCabacNextMps[128];
extern const uint16_t kCabacNextLps[128];
// rangeTabLps by (state, range >> 6): [(pStateIdx << 1) | valMps][8], columns 4..7 used
extern const uint8_t kCabacLpsByState[128][8];
// A context variable as one 64-bit word: bits 0-31 hold rangeTabLps[pStateIdx][0..3] (one byte per
// range quarter, (range >> 6) & 3), bits 32-38 the state (pStateIdx << 1) | valMps.  The LPS range
// of a bin is then a shift of a register by the range, not a table load after it.
typedef uint64_t CabacState;
// word of each state, and the word after an MPS / LPS bin
extern const uint64_t kCabacWord[128];

extern const uint64_t kCabacNextMpsW[128];
extern const uint64_t kCabacNextLpsW[128];
#pragma GCC visibility pop


inline uint8_t cabac_init_state(int m, int n, int qp) {
    if (qp < 0) qp = 0;
    if (qp > 51) qp = 51;
    int pre = ((m * qp) >> 4) + n;
    if (pre < 1) pre = 1;
    if (pre > 126) pre = 126;
    int mps = pre <= 63 ? 0 : 1;
    int st = mps ? pre - 64 : 63 - pre;
    return static_cast<uint8_t>((st << 1) | mps);
}
inline CabacState cabac_init_word(int m, int n, int qp) { return kCabacWord[cabac_init_state(m, n, qp)]; }

// Branch-free on the MPS/LPS decision: the offset lives at the top of a
// 64-bit window (value = offset << bits | look-ahead), renormalisation is a
// count-leading-zeros shift of the range and a decrement of `bits`, and the
// window is refilled 32 bits at a time.
//
// kInlineRefill: the 32-bit refill inline at every bin (HEVC parser, `Cabac`) or one out-of-line
// call (H.264 parser, `CabacOutlineRefill`).  Inline, a decoder copied into a local (the residual
// loops) never has its address taken: GCC had kept the HEVC engine's range / offset / bits in the
// stack frame, storing them after every bin and reloading them after context stores (box CPU
// r04pb: HEVC bench parse -2.3 %, 149 KB set -3.5 %); the clang-built H.264 parser measured
// 1.7 % slower with it (larger hot loops) and keeps the call.
template <bool kInlineRefill>
class CabacT {
public:
    void init(const uint8_t* p, const uint8_t* end) {
        cur_ = p;
        end_ = end;
        range_ = 510;
        value_ = 0;
        for (int i = 0; i < 4; i++) value_ = (value_ << 8) | (cur_ < end_ ? *cur_++ : 0u);
        bits_ = 32 - 9;
    }
    // The MPS/LPS outcome as conditional moves, never a branch: context-coded bins are one dependency
    // chain, and a mispredicted branch per bin costs more than the selects (measured on the GPU
    // box's host CPU, tools/gpu_parse_ab.sh: the branch form for skewed contexts was 2.5-6 % slower
    // end to end).  Both outcomes' renormalised ranges are ready when the compare resolves (rLPS
    // shifted by its leading zeros; rMPS = range - rLPS >= 128 shifted by 0 or 1), so the chain
    // per bin is range -> byte shift of the context word -> subtract -> scale -> compare -> cmov.
    __attribute__((always_inline)) inline int decision(CabacState& ctx) {
        H2J_COUNT(g_bins_ctx, 1);
        const uint64_t w = ctx;
        const unsigned st = static_cast<unsigned>(w >> 32);
        const uint32_t lps = static_cast<uint32_t>(w >> ((range_ >> 3) & 24)) & 0xffu;
        const uint32_t rmps = range_ - lps;
        const uint64_t scaled = static_cast<uint64_t>(rmps) << bits_;
        const uint32_t msh = (rmps >> 8) ^ 1u;
        uint32_t r = rmps << msh, sh = msh;
        const uint32_t lsh = static_cast<uint32_t>(__builtin_clz(lps)) - 23u;
        const uint32_t lr = lps << lsh;
        // next state words from two loads that depend only on the state (issued early), then a
        // select: a load indexed by the outcome would sit on the chain of a context used twice
        uint64_t nx = kCabacNextMpsW[st];
        const uint64_t nl = kCabacNextLpsW[st];
        uint64_t v = value_;
        const uint64_t vl = value_ - scaled;
        uint32_t is_lps = 0;
#if defined(__x86_64__)
        // one compare, then conditional moves (the compiler turns a C select of these into a
        // branch, mispredicted on every LPS bin)
        __asm__("cmpq %[sc], %[v]\n\t"
                "cmovaeq %[vl], %[v]\n\t"
                "cmovael %[lr], %[r]\n\t"
                "cmovael %[ls], %[sh]\n\t"
                "cmovaeq %[nl], %[nx]\n\t"
                "setae %b[il]"
                : [v] "+r"(v), [r] "+r"(r), [sh] "+r"(sh), [nx] "+r"(nx), [il] "+q"(is_lps)
                : [sc] "r"(scaled), [vl] "r"(vl), [lr] "r"(lr), [ls] "r"(lsh), [nl] "r"(nl)
                : "cc");
#else
        // portable form (other targets): the same selects in C
        is_lps = v >= scaled ? 1u : 0u;
        v = is_lps ? vl : v;
        r = is_lps ? lr : r;
        sh = is_lps ? lsh : sh;
        nx = is_lps ? nl : nx;
#endif
        value_ = v;
        range_ = r;
        bits_ -= static_cast<int>(sh);
        ctx = nx;
        if (bits_ < 0) refill();
        return static_cast<int>((st & 1) ^ is_lps);
    }
    __attribute__((always_inline)) int bypass_b() {
        H2J_COUNT(g_bins_byp, 1);
        if (--bits_ < 0) refill();
        const uint64_t scaled = static_cast<uint64_t>(range_) << bits_;
        const bool one = value_ >= scaled;
        value_ -= one ? scaled : 0;
        return one;
    }
    // k (1..24) bypass bins at once, first bin in the MSB.  Decoding bypass bins
    // (9.3.4.3.4) is long division of the offset, extended by one look-ahead bit
    // per bin, by the range: the bins are the k-bit quotient, the new offset the
    // remainder.
    __attribute__((always_inline)) uint32_t bypass_batch_b(int k) {
        H2J_COUNT(g_bins_byp, k);
        if (bits_ < k) refill();
        const int sh = bits_ - k;
        const uint64_t v = value_ >> sh;
        const uint32_t q = static_cast<uint32_t>(v / range_);
        value_ -= (static_cast<uint64_t>(q) * range_) << sh;
        bits_ = sh;
        return q;
    }
    // The next k (1..24) bypass bins without consuming them (MSB first) ...
    __attribute__((always_inline)) uint32_t bypass_peek_b(int k) {
        if (bits_ < k) refill();
        return static_cast<uint32_t>((value_ >> (bits_ - k)) / range_);
    }
    // ... and consuming the first n of them, whose value (the top n bits of the peek) is top:
    // the quotient's leading bits are the quotient of the truncated dividend
    __attribute__((always_inline)) void bypass_skip_b(int n, uint32_t top) {
        H2J_COUNT(g_bins_byp, n);
        const int sh = bits_ - n;
        value_ -= (static_cast<uint64_t>(top) * range_) << sh;
        bits_ = sh;
    }
    __attribute__((always_inline)) uint32_t bypass_bits_b(int n) {
        if (n <= 2) {
            uint32_t v = 0;
            for (int i = 0; i < n; i++) v = (v << 1) | static_cast<uint32_t>(bypass());
            return v;
        }
        if (n <= 24) return bypass_batch(n);
        const uint32_t hi = bypass_batch(n - 16);
        return (hi << 16) | bypass_batch(16);
    }
    __attribute__((always_inline)) int terminate_b() {
        range_ -= 2;
        const uint64_t scaled = static_cast<uint64_t>(range_) << bits_;
        if (value_ >= scaled) return 1;
        if (range_ < 256) {
            range_ <<= 1;
            if (--bits_ < 0) refill();
        }
        return 0;
    }
    // public entry points: forced inline for the HEVC engine, the compiler's choice for H.264's
    // (forcing them there measured 1.7 % slower, r04pb3)
    __attribute__((always_inline)) int bypass() { return kInlineRefill ? bypass_b() : bypass_o(); }
    int bypass_o() { return bypass_b(); }
    __attribute__((always_inline)) uint32_t bypass_batch(int k) { return kInlineRefill ? bypass_batch_b(k) : bypass_batch_o(k); }
    uint32_t bypass_batch_o(int k) { return bypass_batch_b(k); }
    __attribute__((always_inline)) uint32_t bypass_peek(int k) { return kInlineRefill ? bypass_peek_b(k) : bypass_peek_o(k); }
    uint32_t bypass_peek_o(int k) { return bypass_peek_b(k); }
    __attribute__((always_inline)) void bypass_skip(int n, uint32_t top) { kInlineRefill ? bypass_skip_b(n, top) : bypass_skip_o(n, top); }
    void bypass_skip_o(int n, uint32_t top) { bypass_skip_b(n, top); }
    __attribute__((always_inline)) uint32_t bypass_bits(int n) { return kInlineRefill ? bypass_bits_b(n) : bypass_bits_o(n); }
    uint32_t bypass_bits_o(int n) { return bypass_bits_b(n); }
    __attribute__((always_inline)) int terminate() { return kInlineRefill ? terminate_b() : terminate_o(); }
    int terminate_o() { return terminate_b(); }
    // After terminate() returned 1 the arithmetic decoder (9.3.4.3.5) has
    // consumed exactly through the flush's final '1' bit; the next
    // byte-aligned syntax (pcm_sample, next substream) starts at the first
    // byte boundary after it.
    const uint8_t* aligned_pos() const { return cur_ - (bits_ >> 3); }

private:
    __attribute__((always_inline)) void refill() {
        if (kInlineRefill) refill_word();
        else refill_o();
    }
    void refill_o() {
        uint32_t w;
        if (end_ - cur_ >= 4) {
            w = (static_cast<uint32_t>(cur_[0]) << 24) | (static_cast<uint32_t>(cur_[1]) << 16) |
                (static_cast<uint32_t>(cur_[2]) << 8) | cur_[3];
            cur_ += 4;
        } else {
            w = 0;
            for (int i = 0; i < 4; i++) w = (w << 8) | (cur_ < end_ ? *cur_++ : 0u);
        }
        value_ = (value_ << 32) | w;
        bits_ += 32;
    }
    __attribute__((always_inline)) void refill_word() {
        uint32_t w;
        if (__builtin_expect(end_ - cur_ >= 4, 1)) {
            w = (static_cast<uint32_t>(cur_[0]) << 24) | (static_cast<uint32_t>(cur_[1]) << 16) |
                (static_cast<uint32_t>(cur_[2]) << 8) | cur_[3];
            cur_ += 4;
        } else {
            w = tail_word(cur_, end_);
            cur_ = end_ > cur_ ? end_ : cur_;
        }
        value_ = (value_ << 32) | w;
        bits_ += 32;
    }
    // the bytes left before end (fewer than four), zero-padded, as a big-endian word
    __attribute__((noinline)) static uint32_t tail_word(const uint8_t* cur, const uint8_t* end) {
        uint32_t w = 0;
        for (int i = 0; i < 4; i++) w = (w << 8) | (cur < end ? *cur++ : 0u);
        return w;
    }
    const uint8_t* cur_ = nullptr;
    const uint8_t* end_ = nullptr;
    uint64_t value_ = 0;
    uint32_t range_ = 510;
    int bits_ = 0;
};
typedef CabacT<true> Cabac;
typedef CabacT<false> CabacOutlineRefill;

}  // namespace h2j
