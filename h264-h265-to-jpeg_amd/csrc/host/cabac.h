// Context-adaptive binary arithmetic decoder (H.264 9.3.3.2 / H.265 9.3.4.3)
// for the host entropy threads.  Byte-wise refill with a 16-bit value
// register holding the 9-bit offset plus 7 look-ahead bits, so the common
// MPS path is one compare and no bitstream access.
#pragma once
#include <cstdint>

namespace h2j {

extern const uint8_t kCabacLps[64][4];
extern const uint8_t kCabacTransLps[64];
extern const uint8_t kCabacRenorm[32];

struct CabacCtx {
    uint8_t state;  // (pStateIdx << 1) | valMps
};

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

class Cabac {
public:
    void init(const uint8_t* p, const uint8_t* end) {
        cur_ = p;
        end_ = end;
        range_ = 510;
        bits_needed_ = 8;
        value_ = 0;
        if (cur_ < end_) { value_ = static_cast<uint32_t>(*cur_++) << 8; bits_needed_ -= 8; }
        if (cur_ < end_) { value_ |= *cur_++; bits_needed_ -= 8; }
    }
    inline int decision(uint8_t& ctx) {
        int s = ctx >> 1;
        int mps = ctx & 1;
        uint32_t lps = kCabacLps[s][(range_ >> 6) - 4];
        range_ -= lps;
        uint32_t scaled = range_ << 7;
        if (value_ < scaled) {
            ctx = static_cast<uint8_t>(((s + (s < 62)) << 1) | mps);
            if (scaled < (256u << 7)) {
                range_ = scaled >> 6;
                value_ <<= 1;
                if (++bits_needed_ == 0) {
                    bits_needed_ = -8;
                    if (cur_ < end_) value_ |= *cur_++;
                }
            }
            return mps;
        }
        value_ -= scaled;
        int nb = kCabacRenorm[lps >> 3];
        value_ <<= nb;
        range_ = lps << nb;
        int bin = !mps;
        if (s == 0) mps = !mps;
        ctx = static_cast<uint8_t>((kCabacTransLps[s] << 1) | mps);
        bits_needed_ += nb;
        if (bits_needed_ >= 0) {
            if (cur_ < end_) value_ |= static_cast<uint32_t>(*cur_++) << bits_needed_;
            bits_needed_ -= 8;
        }
        return bin;
    }
    inline int bypass() {
        value_ <<= 1;
        if (++bits_needed_ >= 0) {
            bits_needed_ = -8;
            if (cur_ < end_) value_ |= *cur_++;
        }
        uint32_t scaled = range_ << 7;
        if (value_ >= scaled) {
            value_ -= scaled;
            return 1;
        }
        return 0;
    }
    inline uint32_t bypass_bits(int n) {
        uint32_t v = 0;
        for (int i = 0; i < n; i++) v = (v << 1) | static_cast<uint32_t>(bypass());
        return v;
    }
    inline int terminate() {
        range_ -= 2;
        uint32_t scaled = range_ << 7;
        if (value_ >= scaled) return 1;
        if (scaled < (256u << 7)) {
            range_ = scaled >> 6;
            value_ <<= 1;
            if (++bits_needed_ == 0) {
                bits_needed_ = -8;
                if (cur_ < end_) value_ |= *cur_++;
            }
        }
        return 0;
    }
    // After terminate() returned 1 the arithmetic decoder has consumed
    // exactly through the flush's final '1' bit; the next byte-aligned
    // syntax (pcm_sample, next substream) starts at cur_.
    const uint8_t* aligned_pos() const { return cur_; }
    bool overrun() const { return cur_ >= end_ && bits_needed_ > -8 + 0 && false; }

private:
    const uint8_t* cur_ = nullptr;
    const uint8_t* end_ = nullptr;
    uint32_t range_ = 510;
    uint32_t value_ = 0;
    int bits_needed_ = 0;
};

}  // namespace h2j
