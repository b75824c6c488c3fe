// SAO-only in-loop filter pass (H.265 8.7.3), one wave per CTB: the batch kernel for CTB 32 / 64
// without deblocking.  (CTB 16 keeps the strip kernel of sao_rows.h, batches with deblocking the
// fused window kernel of loopfilter.h.)  The reference parses the SAO syntax (decoder/sao.py:15-136)
// and never filters.
//
// Why per CTB: a CTB's SaoTypeIdx and SaoEoClass are uniform, so the wave branches once on them and
// each variant does only its own arithmetic -- the vertical class takes its neighbours straight from
// the rows above / below, the others need one v_alignbyte per neighbour -- instead of computing all
// four classes and masking (sao_rows.h, whose 62-dword strips span several CTBs).  Sample layout:
// lane = (row group, 16-byte column): a luma CTB 64 is 4 columns x 16 groups of 4 rows, the Cb and
// Cr CTBs of a chroma wave (SaoTypeIdx and the EO class are shared by Cb and Cr, 7.3.8.3) 2 columns
// x 16 groups of 2 rows in each wave half.  Every lane loads its rows and the one above / below as
// 16-byte loads (all in flight at once), the dwords left / right of its column come from the lanes
// beside it (DPP quad permutes) or, at the CTB's edge, from one extra dword load per row.  4 samples
// per dword are filtered in two packed 16-bit halves: sgn by clamped packed subtraction, the
// SaoOffsetVal table looked up with one v_perm_b32 per half, saturation by packed min.  Which
// samples may change (8.7.3.2: neighbours inside the picture and in CTBs this one may use; PCM /
// bypass samples, pcm_loop_filter_disabled / cu_transquant_bypass) is a per-lane byte mask built
// once per wave from the nine CTU records.  HBM traffic: each sample read once and written once
// (+ one halo row above / below per CTB from L2).  Plane and record addresses come from the
// batch layout (BatchView), so the sample loads and the CTU-record loads are one round trip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "../../include/p265r.h"
#include "intra.h"
#include "loopfilter.h"
#include "sao.h"

namespace p265r {

__device__ __forceinline__ uint32_t pk_sub_i16(uint32_t a, uint32_t b) {
    uint32_t r; asm("v_pk_sub_i16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
// clamp each signed 16-bit half to [-1, 1]
__device__ __forceinline__ uint32_t pk_sgn_i16(uint32_t d) {
    uint32_t r;
    asm("v_pk_max_i16 %0, %1, %2" : "=v"(r) : "v"(d), "v"(0xffffffffu));
    asm("v_pk_min_i16 %0, %1, %2" : "=v"(r) : "v"(r), "v"(0x00010001u));
    return r;
}

// SAO class variants of a wave (wave-uniform): 0..3 edge offset class, 4 band offset, 5 off (copy)
enum { kSaoEo0 = 0, kSaoEo1 = 1, kSaoEo2 = 2, kSaoEo3 = 3, kSaoBo = 4, kSaoCopy = 5 };

template <int L>                      // CtbLog2SizeY 5 or 6
struct SaoCtbShape {
    static constexpr int CW = 1 << L;
    // luma: NC columns of 16 B, NG row groups of R rows (64 lanes)
    static constexpr int NCL = CW / 16, NGL = 64 / NCL, RL = CW / NGL;
    // chroma: per wave half (32 lanes) one of Cb / Cr; NGC groups (<= 32 / NCC) of RC rows
    static constexpr int CWC = CW / 2, NCC = CWC / 16;
    static constexpr int NGC = (32 / NCC) < CWC ? (32 / NCC) : CWC, RC = CWC / NGC;
    static_assert(NCL * NGL == 64 && RL * NGL == CW, "luma layout");
    static_assert(NCC * NGC <= 32 && RC * NGC == CWC, "chroma layout");
};

// byte-wise 0 / 1 -> 0x00 / 0xff (0x80 - 1 per byte never borrows; LLVM turns x * 255 and
// (x << 8) - x into a quarter-rate v_mul_lo_u32)
__device__ __forceinline__ uint32_t bytes_ff(uint32_t b01) { return (0x80808080u - b01) ^ 0x80808080u; }

// 16-bit ok mask (bit i: sample i of the lane's 16 may change) -> 4 dword byte masks
__device__ __forceinline__ void expand_mask(uint32_t m16, uint32_t* d) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t b = ((m16 >> (4 * j)) & 0xfu) * 0x00204081u & 0x01010101u;   // bit k -> byte k (24-bit mul)
        d[j] = bytes_ff(b);
    }
}

// The rows a lane needs, loaded before anything else of the wave (they depend only on the wave's
// position, so their latency overlaps the CTU-record loads): rows y0 - 1 .. y0 + R of its 16-byte
// column (c[0] = the row above), and the dwords left (x - 4) / right (x + 16) of the column in each
// row -- from the neighbouring lanes of its row group (DPP), at the CTB's edge by an extra load.
template <int R, int NC>
struct SaoRows {
    uint32_t c[R + 2][4];
    uint32_t hl[R + 2], hr[R + 2];
    __device__ __forceinline__ void load(const uint8_t* __restrict__ src, int st, int H, int W, int X, int cx, int y0) {
        typedef __attribute__((address_space(1))) uint8_t gu8;
        typedef __attribute__((address_space(1))) uint32_t gu32;
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        const gu8* s = (const gu8*)src;
        const int xl = max(X - 4, 0), xr = min(X + 16, W - 4);
#pragma unroll
        for (int k = 0; k < R + 2; ++k) {
            const int y = min(max(y0 - 1 + k, 0), H - 1);
            const gu8* row = s + __umul24((uint32_t)y, (uint32_t)st);   // y, st < 2^16: exact 32-bit product
            const u4v v = *(const __attribute__((address_space(1))) u4v*)(row + X);
            c[k][0] = v.x; c[k][1] = v.y; c[k][2] = v.z; c[k][3] = v.w;
            // only the CTB's outer columns need the halo dwords; the others take their neighbours'
            hl[k] = cx == 0 ? *(const gu32*)(row + xl) : 0u;
            hr[k] = cx == NC - 1 ? *(const gu32*)(row + xr) : 0u;
        }
    }
    __device__ __forceinline__ void exchange(int cx) {
#pragma unroll
        for (int k = 0; k < R + 2; ++k) {
            if constexpr (NC == 4) {
                const uint32_t l = (uint32_t)__builtin_amdgcn_mov_dpp((int)c[k][3], 0x90, 0xf, 0xf, false);   // quad [0,0,1,2]
                const uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)c[k][0], 0xf9, 0xf, 0xf, false);   // quad [1,2,3,3]
                hl[k] = cx == 0 ? hl[k] : l;
                hr[k] = cx == NC - 1 ? hr[k] : r;
            } else if constexpr (NC == 2) {
                const uint32_t l = (uint32_t)__builtin_amdgcn_mov_dpp((int)c[k][3], 0xa0, 0xf, 0xf, false);   // quad [0,0,2,2]
                const uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)c[k][0], 0xf5, 0xf, 0xf, false);   // quad [1,1,3,3]
                hl[k] = cx == 0 ? hl[k] : l;
                hr[k] = cx == NC - 1 ? hr[k] : r;
            }
        }
    }
};

// Filter and store a lane's R rows (V = variant).  tables: SaoOffsetVal as positive / negative byte
// tables (lo: entries 0..3, hi: 4), badd: band rotation.  m_first / m_mid / m_last: byte masks of
// the lane's first row, middle rows and last row (equal for R = 1).
template <int V, int R, int NC>
__device__ __forceinline__ void sao_ctb_rows(const SaoRows<R, NC>& L, uint8_t* __restrict__ dst, int st, int H,
                                             int X, int y0, bool act, const uint32_t* m_first,
                                             const uint32_t* m_mid, const uint32_t* m_last, uint32_t tp_lo,
                                             uint32_t tp_hi, uint32_t tn_lo, uint32_t tn_hi, uint32_t badd,
                                             const uint8_t* __restrict__ nf, int nf_w, int sub) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    auto split_lo = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c020c00u); };   // bytes 0, 2
    auto split_hi = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c030c01u); };   // bytes 1, 3
    auto join = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x06020400u); };
    // v16 + table[sel16] clipped to [0, 255]; sel16 = entry index per 16-bit half, 0x0c above it
    auto apply16 = [&](uint32_t v16, uint32_t sel16) {
        const uint32_t pos = __builtin_amdgcn_perm(tp_hi, tp_lo, sel16);
        const uint32_t neg = __builtin_amdgcn_perm(tn_hi, tn_lo, sel16);
        return pk_min_u16(pk_subsat_u16(pk_add_u16(v16, pos), neg), 0x00ff00ffu);
    };
    auto edge16 = [&](uint32_t v16, uint32_t a16, uint32_t b16) {    // 2 + sgn(v - a) + sgn(v - b), + 0x0c00
        return pk_add_u16(pk_add_u16(pk_sgn_i16(pk_sub_i16(v16, a16)), pk_sgn_i16(pk_sub_i16(v16, b16))), 0x0c020c02u);
    };
    auto at = [&](int k, int j) -> uint32_t {                        // dword j (-1 .. 4) of loaded row k
        return j < 0 ? L.hl[k] : (j > 3 ? L.hr[k] : L.c[k][j]);
    };
    typedef __attribute__((address_space(1))) uint8_t gu8;
    gu8* d = (gu8*)dst;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int k = r + 1;                  // this row in L.c (row 0 = the row above)
        const int y = y0 + r;
        const uint32_t* m = r == 0 ? m_first : (r == R - 1 ? m_last : m_mid);
        uint32_t nfm[4] = {0u, 0u, 0u, 0u};   // PCM / bypass samples: unchanged
        if (nf) {
            const int ny = (int)__umul24((uint32_t)((min(y, H - 1) << sub) >> 3), (uint32_t)nf_w);
#pragma unroll
            for (int j = 0; j < 4; ++j) nfm[j] = nf[ny + min(((X + 4 * j) << sub) >> 3, nf_w - 1)] ? 0xffffffffu : 0u;
        }
        uint32_t out[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t cur = L.c[k][j];
            if constexpr (V == kSaoCopy) {
                out[j] = cur;
            } else {
                uint32_t sel_lo, sel_hi;
                const uint32_t v_lo = split_lo(cur), v_hi = split_hi(cur);
                if constexpr (V == kSaoBo) {
                    // band offset: entry 1..4 for the four bands from sao_band_position, else 0
                    const uint32_t kk = (((cur >> 3) & 0x1f1f1f1fu) + badd) & 0x1f1f1f1fu;
                    const uint32_t big = (((kk & 0x1c1c1c1cu) + 0x7f7f7f7fu) & 0x80808080u) >> 7;
                    const uint32_t sel = (kk + 0x01010101u) & ~bytes_ff(big);
                    sel_lo = __builtin_amdgcn_perm(0x0c0c0c0cu, sel, 0x04020400u);
                    sel_hi = __builtin_amdgcn_perm(0x0c0c0c0cu, sel, 0x04030401u);
                } else {
                    uint32_t a, b;                                        // neighbours, byte-aligned
                    if constexpr (V == kSaoEo0) {
                        a = __builtin_amdgcn_alignbyte(cur, at(k, j - 1), 3);
                        b = __builtin_amdgcn_alignbyte(at(k, j + 1), cur, 1);
                    } else if constexpr (V == kSaoEo1) {
                        a = L.c[k - 1][j];
                        b = L.c[k + 1][j];
                    } else if constexpr (V == kSaoEo2) {
                        a = __builtin_amdgcn_alignbyte(L.c[k - 1][j], at(k - 1, j - 1), 3);
                        b = __builtin_amdgcn_alignbyte(at(k + 1, j + 1), L.c[k + 1][j], 1);
                    } else {
                        a = __builtin_amdgcn_alignbyte(at(k - 1, j + 1), L.c[k - 1][j], 1);
                        b = __builtin_amdgcn_alignbyte(L.c[k + 1][j], at(k + 1, j - 1), 3);
                    }
                    sel_lo = edge16(v_lo, split_lo(a), split_lo(b));
                    sel_hi = edge16(v_hi, split_hi(a), split_hi(b));
                }
                const uint32_t res = join(apply16(v_lo, sel_lo), apply16(v_hi, sel_hi));
                const uint32_t mk = m[j] & ~nfm[j];
                out[j] = (res & mk) | (cur & ~mk);
            }
        }
        if (act && y < H)
            *(__attribute__((address_space(1))) u4v*)(d + __umul24((uint32_t)y, (uint32_t)st) + X) = u4v{out[0], out[1], out[2], out[3]};
    }
}

// One CTB of a wave: the luma CTB (CHROMA = false) or the Cb + Cr CTBs (CHROMA = true) of CTB rs of
// picture pic.  load() issues every memory access the CTB needs (sample rows, CTU records), filter()
// consumes them, so a wave can put several CTBs' loads in flight before filtering the first.
template <int L, bool CHROMA>
struct SaoCtb {
    using S = SaoCtbShape<L>;
    static constexpr int NC = CHROMA ? S::NCC : S::NCL, NG = CHROMA ? S::NGC : S::NGL, R = CHROMA ? S::RC : S::RL;
    static constexpr int sub = CHROMA ? 1 : 0;
    static constexpr int cs = S::CW >> sub;                        // CTB size in this component
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    SaoRows<R, NC> rows;
    u4v me0, me1, nb[9];
    const uint8_t* nf;
    int rs, bx, by, c, cx, X, y0, W, H, st;
    bool act;
    uint64_t pofs;

    __device__ __forceinline__ void load(const DevPic* __restrict__ pics, const Geo& g, const BatchView& v, int pic,
                                         int rs_, int lane) {
        rs = rs_;
        bx = rs % g.wc; by = rs / g.wc;
        // lane -> (component, column cx, row group ry)
        const int half = CHROMA ? lane >> 5 : 0;
        const int hl = CHROMA ? lane & 31 : lane;
        c = CHROMA ? 1 + half : 0;
        cx = hl % NC;
        const int ry = hl / NC;
        const bool in_layout = ry < NG;
        W = CHROMA ? g.cw : g.w; H = CHROMA ? g.ch : g.h;
        X = bx * cs + 16 * cx;
        y0 = by * cs + R * (in_layout ? ry : 0);
        act = in_layout && X < W;
        st = g.stride[c];
        pofs = (uint64_t)pic * v.pic_bytes + v.plane_off[c];
        // the sample loads depend on the position only: issued first
        rows.load(v.rec0 + pofs, st, H, W, X, cx, y0);
        nf = pics[pic].nofilter;
        const uint32_t* crec = reinterpret_cast<const uint32_t*>(v.ctus0 + (size_t)pic * g.wc * g.hc);
        me0 = *reinterpret_cast<const u4v*>(crec + (size_t)rs * 8);
        me1 = *reinterpret_cast<const u4v*>(crec + (size_t)rs * 8 + 4);
#pragma unroll
        for (int k = 0; k < 9; ++k) {                             // all nine in flight together
            const int nx = min(max(bx + k % 3 - 1, 0), g.wc - 1), ny = min(max(by + k / 3 - 1, 0), g.hc - 1);
            nb[k] = *reinterpret_cast<const u4v*>(crec + (size_t)(ny * g.wc + nx) * 8);
        }
    }

    __device__ __forceinline__ void filter(const Geo& g, const BatchView& v) {
        const int Y0b = by * cs;
        // ---- the CTB's SAO parameters and 8.7.3.2 permissions of its 3x3 neighbourhood (scalar) ----
        uint32_t allow = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int dx = k % 3 - 1, dy = k / 3 - 1;
            const int nx = bx + dx, ny = by + dy;
            if (nx < 0 || ny < 0 || nx >= g.wc || ny >= g.hc) continue;
            const int ro = ny * g.wc + nx;
            const u4v o = nb[k];
            bool ok = true;
            const uint32_t ti = me0.y >> 16, to = o.y >> 16;
            if (o.z != me0.z) {                                   // other slice: the later sample's flag
                const bool o_first = to < ti || (to == ti && ro < rs);
                ok = ((o_first ? me0.w : o.w) & P265R_CTU_LF_ACROSS_SLICES) != 0;
            }
            if (!g.lf_tiles && to != ti) ok = false;
            if (ok) allow |= 1u << k;
        }
        allow = __builtin_amdgcn_readfirstlane(allow);
        auto A = [&](int ay, int ax) { return ((allow >> (ay * 3 + ax)) & 1u) != 0; };
        // record dword 3: flags | SaoTypeIdx[3] << 8; dword 4: class[3] | dbk offsets; 5..7: offsets.
        // Cb and Cr share SaoTypeIdx and the EO class (validated at upload), not the band position
        const int typ = (int)((me0.w >> (8 * (c + 1))) & 0xffu);
        const int cls = (int)((me1.x >> (8 * c)) & 0xffu);
        const int variant = __builtin_amdgcn_readfirstlane(typ == 0 ? kSaoCopy : (typ == 1 ? kSaoBo : (cls & 3)));
        const uint32_t o = c == 0 ? me1.y : (c == 1 ? me1.z : me1.w); // SaoOffsetVal[1..4], signed bytes
        const uint32_t t_lo = typ == 2 ? __builtin_amdgcn_perm(0u, o, 0x020c0100u) : (o << 8);
        const uint32_t t_hi = o >> 24;
        const uint32_t n_lo = (t_lo >> 7) & 0x01010101u, n_hi = (t_hi >> 7) & 0x01010101u;
        const uint32_t tp_lo = t_lo & ~bytes_ff(n_lo), tp_hi = t_hi & ~bytes_ff(n_hi);
        const uint32_t tn_lo = (~t_lo & bytes_ff(n_lo)) + n_lo, tn_hi = (~t_hi & bytes_ff(n_hi)) + n_hi;
        const uint32_t bsh = (uint32_t)((32 - cls) & 31);
        const uint32_t badd = __umul24(bsh, 0x010101u) | bsh << 24;   // (32 - band position) in every byte

        // ---- byte masks: which of the lane's 16 samples may change, per row kind --------------------
        // neighbour (dx, dy) of sample i of row y is usable iff inside the picture and its CTB allowed;
        // only sample 0 / 15 can leave the lane's column, only the CTB's first / last row its rows.
        // Samples at x >= W are stored into the row padding and never read: don't care.
        const int n_in = W - X;                                    // samples of the lane inside the picture
        auto col_bits = [&](int dx, int ay) -> uint32_t {          // A-row ay of the neighbour's CTB
            if (ay < 0) return 0u;                                 // the neighbour's row is outside the picture
            if (dx == 0) return A(ay, 1) ? 0xffffu : 0u;
            if (dx < 0) return (A(ay, 1) ? 0xfffeu : 0u) | ((X > 0 && A(ay, cx == 0 ? 0 : 1)) ? 1u : 0u);
            const uint32_t inner = n_in >= 16 ? 0x7fffu : ((1u << max(n_in - 1, 0)) - 1u);
            return (A(ay, 1) ? inner : 0u) | ((n_in > 16 && A(ay, cx == NC - 1 ? 2 : 1)) ? 0x8000u : 0u);
        };
        const int ylast = min(Y0b + cs, H) - 1;                    // the CTB's last row in the picture
        // A-row of a vertical neighbour of row y: above (dy = -1) / below (dy = +1); -1 = outside
        auto row_a = [&](int y, int dy) -> int {
            if (dy == 0) return 1;
            if (dy < 0) return y == Y0b ? 0 : 1;                   // Y0b == 0: no CTB row above -> A bits 0
            return y == ylast ? (y == H - 1 ? -1 : 2) : 1;
        };
        auto mask16 = [&](int y) -> uint32_t {
            if (variant == kSaoCopy) return 0u;
            if (variant == kSaoBo) return 0xffffu;
            const int dxa = variant == kSaoEo1 ? 0 : (variant == kSaoEo3 ? 1 : -1);
            const int dya = variant == kSaoEo0 ? 0 : -1;
            return col_bits(dxa, row_a(y, dya)) & col_bits(-dxa, row_a(y, -dya));
        };
        uint32_t m_first[4], m_mid[4], m_last[4];
        expand_mask(mask16(y0), m_first);
        expand_mask(R >= 3 ? mask16(y0 + 1) : 0u, m_mid);          // rows 1 .. R-2
        expand_mask(mask16(y0 + R - 1), m_last);
        rows.exchange(cx);
        uint8_t* dst = v.out0 + pofs;
        switch (variant) {
            case kSaoEo0: sao_ctb_rows<kSaoEo0, R, NC>(rows, dst, st, H, X, y0, act, m_first, m_mid, m_last, tp_lo, tp_hi, tn_lo, tn_hi, badd, nf, g.nf_w, sub); break;
            case kSaoEo1: sao_ctb_rows<kSaoEo1, R, NC>(rows, dst, st, H, X, y0, act, m_first, m_mid, m_last, tp_lo, tp_hi, tn_lo, tn_hi, badd, nf, g.nf_w, sub); break;
            case kSaoEo2: sao_ctb_rows<kSaoEo2, R, NC>(rows, dst, st, H, X, y0, act, m_first, m_mid, m_last, tp_lo, tp_hi, tn_lo, tn_hi, badd, nf, g.nf_w, sub); break;
            case kSaoEo3: sao_ctb_rows<kSaoEo3, R, NC>(rows, dst, st, H, X, y0, act, m_first, m_mid, m_last, tp_lo, tp_hi, tn_lo, tn_hi, badd, nf, g.nf_w, sub); break;
            case kSaoBo:  sao_ctb_rows<kSaoBo, R, NC>(rows, dst, st, H, X, y0, act, m_first, m_mid, m_last, tp_lo, tp_hi, tn_lo, tn_hi, badd, nf, g.nf_w, sub); break;
            default:      sao_ctb_rows<kSaoCopy, R, NC>(rows, dst, st, H, X, y0, act, m_first, m_mid, m_last, tp_lo, tp_hi, tn_lo, tn_hi, badd, nf, g.nf_w, sub); break;
        }
    }
};

// CTBs per wave (P265R_SAO_PAIR): 2 = two horizontally adjacent CTBs, both loaded before either is
// filtered (twice the bytes in flight per wave; a luma row pair is one 128-B line)
#ifndef P265R_SAO_PAIR
#define P265R_SAO_PAIR 1
#endif
template <int L, bool CHROMA>
__device__ __forceinline__ void sao_ctb_wave(const DevPic* __restrict__ pics, const Geo& g, const BatchView& v,
                                             int pic, int u, int lane) {
    const int nctb = g.wc * g.hc;
    if constexpr (P265R_SAO_PAIR == 2) {
        SaoCtb<L, CHROMA> a, b;
        const bool two = 2 * u + 1 < nctb;                        // wave-uniform
        a.load(pics, g, v, pic, 2 * u, lane);
        if (two) b.load(pics, g, v, pic, 2 * u + 1, lane);
        a.filter(g, v);
        if (two) b.filter(g, v);
    } else {
        SaoCtb<L, CHROMA> a;
        a.load(pics, g, v, pic, u, lane);
        a.filter(g, v);
    }
}

#ifndef P265R_SAO_WPE
#define P265R_SAO_WPE 4
#endif
template <int L>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(P265R_SAO_WPE))) void sao_ctb_kernel(const DevPic* __restrict__ pics, Geo g, BatchView v, int n_pics) {
    const int lane = threadIdx.x & 63;
    const int per = (g.wc * g.hc + P265R_SAO_PAIR - 1) / P265R_SAO_PAIR;   // waves per component and picture
    const int total = 2 * per * n_pics;
    const int nblk = (total + 3) >> 2;
    const int bunit = xcd_unit(blockIdx.x, nblk);
    const int unit = __builtin_amdgcn_readfirstlane(bunit * 4 + (int)(threadIdx.x >> 6));
    if (bunit >= nblk || unit >= total) return;                   // whole wave (no barriers)
    const int pic = unit / (2 * per);
    const int u = unit - pic * 2 * per;
    if (u >= per) sao_ctb_wave<L, true>(pics, g, v, pic, u - per, lane);
    else sao_ctb_wave<L, false>(pics, g, v, pic, u, lane);
}

}  // namespace p265r
