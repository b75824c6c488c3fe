// Bit-level readers of the native front-end: NAL unit extraction, RBSP bit reader
// (u(n), ue(v), se(v)) and the CABAC arithmetic decoding engine (H.265 9.3.4.3).
//
// Replaces the reference's BitStreamBuffer (decoder/bsb.py:6-176: search_start_code,
// read_bits, u, ue, se) and the engine half of decoder/cabac.py (Cabac.decode_decision,
// decode_bypass, decode_terminate, renormalization_process: cabac.py:219-293).  The
// reference reads the byte stream bit by bit through Python calls; here a NAL unit is
// first turned into its RBSP (emulation_prevention_three_byte removed) and the engine
// keeps up to 31 look-ahead bits below ivlOffset in a 64-bit word, refilled 4 bytes at a time.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace p265fe {

struct BitstreamError : std::runtime_error {
    explicit BitstreamError(const std::string& s) : std::runtime_error(s) {}
};
struct Unsupported : std::runtime_error {
    explicit Unsupported(const std::string& s) : std::runtime_error(s) {}
};

[[noreturn]] inline void bs_fail(const char* what) { throw BitstreamError(what); }

// One NAL unit of an Annex-B byte stream: header fields + RBSP bytes.
struct Nal {
    int type = 0, layer_id = 0, temporal_id = 0;
    std::vector<uint8_t> rbsp;   // payload after the 2-byte header, emulation prevention removed
};

// Split an Annex-B byte stream at start codes (0x000001 / 0x00000001), dropping
// trailing_zero_8bits, and convert each NAL unit payload to RBSP (7.3.1.1, 7.4.2).  Zero bytes are
// found with memchr and the bytes between emulation_prevention_three_bytes are block-copied (the
// split runs on one thread ahead of the parallel slice-data parse).
inline std::vector<Nal> split_nals(const uint8_t* d, size_t n) {
    std::vector<Nal> out;
    // first k >= from with d[k..k+2] == 00 00 01 (n if none)
    auto find_sc = [&](size_t from) -> size_t {
        size_t k = from;
        while (k + 2 < n) {
            const void* z = std::memchr(d + k, 0, n - 2 - k);
            if (!z) return n;
            k = (size_t)(static_cast<const uint8_t*>(z) - d);
            if (d[k + 1] == 0 && d[k + 2] == 1) return k;
            ++k;
        }
        return n;
    };
    size_t i = find_sc(0);
    while (i < n) {
        size_t start = i + 3;
        size_t next = find_sc(start);
        size_t end = next;
        while (end > start && d[end - 1] == 0) --end;   // zero_byte of the next start code / trailing zeros
        if (end - start >= 2) {
            Nal nal;
            uint16_t h = (uint16_t)((d[start] << 8) | d[start + 1]);
            if (h & 0x8000) bs_fail("forbidden_zero_bit set");
            nal.type = (h >> 9) & 63;
            nal.layer_id = (h >> 3) & 63;
            nal.temporal_id = (int)(h & 7) - 1;
            if (nal.temporal_id < 0) bs_fail("nuh_temporal_id_plus1 == 0");
            nal.rbsp.resize(end - start - 2);
            uint8_t* o = nal.rbsp.data();
            size_t k = start + 2;
            while (k < end) {
                // next 00 00 03 at p >= k (a removed 03 resets the zero count: the search restarts after it)
                size_t p = k;
                size_t cut = end;
                while (p + 2 < end) {
                    const void* z = std::memchr(d + p, 0, end - 2 - p);
                    if (!z) break;
                    p = (size_t)(static_cast<const uint8_t*>(z) - d);
                    if (d[p + 1] == 0 && d[p + 2] == 3) { cut = p + 2; break; }
                    ++p;
                }
                std::memcpy(o, d + k, cut - k);                   // up to (not including) the 03
                o += cut - k;
                k = cut < end ? cut + 1 : end;
            }
            nal.rbsp.resize((size_t)(o - nal.rbsp.data()));
            out.push_back(std::move(nal));
        }
        i = next;
    }
    return out;
}

// MSB-first bit reader over an RBSP (u(n), ue(v), se(v): 7.2, 9.2).
class BitReader {
public:
    BitReader(const uint8_t* p, size_t n, size_t bitpos = 0) : p_(p), n_(n), pos_(bitpos) {}
    uint32_t u(int bits) {
        uint32_t v = 0;
        for (int k = 0; k < bits; ++k) v = (v << 1) | bit();
        return v;
    }
    uint32_t bit() {
        if (pos_ >= n_ * 8) bs_fail("read past end of RBSP");
        uint32_t b = (p_[pos_ >> 3] >> (7 - (pos_ & 7))) & 1;
        ++pos_;
        return b;
    }
    uint32_t ue() {
        int lz = 0;
        while (!bit()) {
            if (++lz > 31) bs_fail("ue(v) too long");
        }
        if (lz == 0) return 0;
        uint64_t v = ((uint64_t)1 << lz) - 1 + u(lz);
        if (v > 0xFFFFFFFEull) bs_fail("ue(v) overflow");
        return (uint32_t)v;
    }
    int32_t se() {
        uint32_t k = ue();
        return (k & 1) ? (int32_t)((k + 1) >> 1) : -(int32_t)(k >> 1);
    }
    bool flag() { return bit() != 0; }
    void skip(size_t bits) { pos_ += bits; if (pos_ > n_ * 8) bs_fail("skip past end of RBSP"); }
    bool byte_aligned() const { return (pos_ & 7) == 0; }
    size_t pos() const { return pos_; }
    size_t size_bits() const { return n_ * 8; }
    // byte_alignment(): alignment_bit_equal_to_one + zero bits (7.3.2.11)
    void byte_alignment() {
        if (bit() != 1) bs_fail("alignment_bit_equal_to_one != 1");
        while (!byte_aligned())
            if (bit() != 0) bs_fail("alignment_bit_equal_to_zero != 0");
    }
    // more_rbsp_data() (7.2): anything before the rbsp_stop_one_bit?
    bool more_rbsp_data() const {
        size_t last = n_;
        while (last > 0 && p_[last - 1] == 0) --last;
        if (last == 0) return false;
        uint8_t b = p_[last - 1];
        int tz = 0;
        while (!((b >> tz) & 1)) ++tz;
        size_t stop = (last - 1) * 8 + (7 - tz);   // bit index of rbsp_stop_one_bit
        return pos_ < stop;
    }

private:
    const uint8_t* p_;
    size_t n_;
    size_t pos_;
};

// ---------------------------------------------------------------------------------
// CABAC arithmetic decoding engine (9.3.4.3).  Context state = (pStateIdx << 1) | valMps, kept in a
// uint16_t (not a char type) so that state writes cannot alias the engine's registers.
// ---------------------------------------------------------------------------------
extern const uint8_t kLpsTable[64][4];      // rangeTabLps (Table 9-46; cabac.py:66-132)
extern const uint8_t kNextStateMps[64];     // transIdxMps (Table 9-47; cabac.py:134-143)
extern const uint8_t kNextStateLps[64];     // transIdxLps (cabac.py:145-154)
// both transitions of a context state word (pStateIdx << 1 | valMps), by "the bin was the LPS":
// kTransTable[s][0] = MPS transition, [s][1] = LPS transition (incl. the valMps flip at state 0)
extern const uint8_t kTransTable[128][2];

// The engine with ivlOffset kept at bits 39..47 of a 64-bit word and up to 31 look-ahead bits below it,
// refilled 4 bytes at a time (one refill branch per ~32 stream bits; measured against the byte-refill
// 32-bit form on the box: one thread 46.6 k -> 51.1 k CTU/s, 16 threads 608 k -> 643 k).  Next stream bit
// position: 7 + bits_needed_; a refill (bits_needed_ >= 24 after a shift of at most 8) puts the next
// big-endian word at bits [bits_needed_ - 24, bits_needed_ + 8).
class Cabac {
public:
    // Start (or restart) the engine at byte `byte_pos` of the RBSP (9.3.2.5: ivlCurrRange = 510,
    // ivlOffset = read_bits(9)).
    void start(const uint8_t* rbsp, size_t n, size_t byte_pos) {
        base_ = rbsp;
        end_ = rbsp + n;
        cur_ = rbsp + (byte_pos < n ? byte_pos : n);
        range_ = 510;
        value_ = 0;
        bits_needed_ = 40;
        refill();
        // 9.3.2.5: a conforming bitstream never starts with ivlOffset 510 or 511 (>= ivlCurrRange); every
        // bin after it keeps ivlOffset < ivlCurrRange, which bypass_bits' quotient (< 2^k) relies on
        if ((value_ >> kShift) >= 510) bs_fail("CABAC ivlOffset 510 / 511 at initialisation");
    }
    // Branch-free bin decoding: MPS and LPS outcomes computed together and selected (the
    // MPS / LPS branch of 9.3.4.3.2 mispredicts about as often as the LPS occurs); one shared
    // renormalization (an MPS range is >= 128, so it shifts by at most 1, as 9.3.4.3.3 does).
    inline int decision(uint16_t& ctx) {
        const uint32_t s = ctx;
        // the state's four rangeTabLps entries as one word (loaded off the range chain), the entry picked by a
        // shift of (range >> 6) & 3 bytes: the range -> lps step is two ALU ops instead of a dependent load
        uint32_t row;
        std::memcpy(&row, kLpsTable[s >> 1], 4);
        const uint32_t lps = (row >> ((range_ >> 3) & 24u)) & 0xffu;
        const uint32_t rmps = range_ - lps;
        const uint64_t scaled = (uint64_t)rmps << kShift;
        const uint32_t is_lps = value_ >= scaled ? 1u : 0u;
        value_ -= scaled & (0ull - is_lps);
        const uint32_t r = is_lps ? lps : rmps;
        ctx = kTransTable[s][is_lps];
        const int nb = renorm_bits(r);
        range_ = r << nb;
        value_ <<= nb;
        bits_needed_ += nb;
        if (bits_needed_ >= 24) refill();
        return (int)((s & 1u) ^ is_lps);
    }
    inline int bypass() {
        value_ <<= 1;
        if (++bits_needed_ >= 24) refill();
        const uint64_t scaled = (uint64_t)range_ << kShift;
        const uint32_t b = value_ >= scaled ? 1u : 0u;
        value_ -= scaled & (0ull - b);
        return (int)b;
    }
    // n bypass bins (9.3.4.3.4) at once, up to 8 per step: shifting k bits in and dividing by the
    // scaled range is the same binary long division the bin-by-bin compare / subtract performs
    // (the scaled range has kShift zero low bits, so the quotient is (value >> kShift) / range)
    inline uint32_t bypass_bits(int n) {
        uint32_t v = 0;
        while (n > 0) {
            const int k = n < 8 ? n : 8;
            value_ <<= k;
            bits_needed_ += k;
            if (bits_needed_ >= 24) refill();
            const uint32_t q = (uint32_t)(value_ >> kShift) / range_;
            value_ -= (uint64_t)(q * range_) << kShift;
            v = (v << k) | q;
            n -= k;
        }
        return v;
    }
    inline int terminate() {
        range_ -= 2;
        if (value_ >= (uint64_t)range_ << kShift) return 1;     // no renormalization (9.3.4.3.5)
        if (range_ < 256u) {
            range_ <<= 1;
            value_ <<= 1;
            if (++bits_needed_ >= 24) refill();
        }
        return 0;
    }
    // Bit position (in the RBSP) of the spec decoder, which has read 9 bits at start and one
    // per renormalization shift: the bytes fetched minus the look-ahead bits (31 - bits_needed_).
    // After a terminate bin equal to 1 the last bit read is the final '1' written by the encoder
    // flush (rbsp_stop_one_bit / alignment_bit_equal_to_one / the bit before pcm_alignment_zero_bit);
    // the next byte-aligned position follows it.
    size_t bit_pos() const {
        return (size_t)((cur_ - base_) * 8 + bits_needed_ - 31);
    }
    size_t aligned_byte_after_terminate() const { return (bit_pos() + 7) >> 3; }
    bool overrun() const { return bit_pos() > (size_t)(end_ - base_) * 8; }

private:
    static constexpr int kShift = 39;
    static inline int renorm_bits(uint32_t r) {   // shifts to bring r (>= 2) back to >= 256
        return __builtin_clz(r) - 23;
    }
    inline void refill() {
        uint32_t w;
        if (end_ - cur_ >= 4) {
            std::memcpy(&w, cur_, 4);
            w = __builtin_bswap32(w);
        } else {                                  // the RBSP's last bytes, zeros past its end
            w = 0;
            for (int i = 0; i < 4; ++i) w = (w << 8) | (cur_ + i < end_ ? cur_[i] : 0u);
        }
        cur_ += 4;
        value_ |= (uint64_t)w << (bits_needed_ - 24);
        bits_needed_ -= 32;
    }
    const uint8_t* base_ = nullptr;
    const uint8_t* end_ = nullptr;
    const uint8_t* cur_ = nullptr;
    uint32_t range_ = 510;
    uint64_t value_ = 0;
    int bits_needed_ = 0;
};

}  // namespace p265fe
