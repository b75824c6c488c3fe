// SAO-only in-loop filter pass (H.265 8.7.3), CTB 32 / 64 without deblocking: a streaming strip
// kernel with 16 samples per lane.  (CTB 16 keeps sao_rows.h, whose 4-sample lanes never straddle
// an 8-sample chroma CTB; batches with deblocking the fused window kernel of loopfilter.h.)  The
// reference parses the SAO syntax (decoder/sao.py:15-136) and never filters.
//
// One wave = one CTB row of one component over a strip of 62 x 16 samples (lane l: the 16 samples
// at x = 992 s + 16 (l - 1); lanes 0 and 63 only supply the neighbours of lanes 1 and 62).  Every
// row is ONE coalesced 1-KB load per wave instruction (the per-CTB layout of a row group would
// touch 16 half cache lines per instruction, which measured texture-addresser bound); the wave walks
// down its CTB row K rows at a time, the next K rows loaded before the current ones are filtered.
// A lane's 16 samples lie in one CTB (16 | CTB width), so its SaoTypeIdx, class and offsets are
// per-lane constants; the neighbours a, b of edge offset are selected per lane (v_cndmask on the
// class) and byte-aligned with one v_alignbyte each, the dwords beside the lane's column come from
// lanes l -/+ 1 (DPP wave shifts).  4 samples per dword in two packed 16-bit halves: sgn by clamped
// packed subtraction, the SaoOffsetVal table looked up with one v_perm_b32 per half, saturation by
// packed min.  (Measured against a class-uniform one-wave-per-CTB layout -- 16 lanes per row group,
// every load touching 16 half cache lines: texture-addresser bound, 1.09 vs 0.85 ms per 512 1080p
// pictures.)
// HBM traffic per sample: one read (+ 2 halo rows per CTB height) and one write.
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

#ifndef P265R_SAO_WPE
#define P265R_SAO_WPE 6
#endif

#ifndef P265R_SAO_NT
#define P265R_SAO_NT 0                     // A/B: 1 non-temporal output stores, 2 non-temporal loads too
#endif

constexpr int kSao16Strip = 62 * 16;       // output samples per strip
#ifndef P265R_SAO16_CHUNK
#define P265R_SAO16_CHUNK 2
#endif
// rows per load batch: 2 (80 VGPRs, 6 waves per SIMD) rather than 4 (100 VGPRs): 0.74 -> 0.77 ms
// alone, but two SAO waves per SIMD fit beside the W = 8 row kernel of another lane: pipelined
// 46.9-47.1 -> 47.0-48.0 M CTU/s (3 interleaved reps, round 3)
constexpr int kSao16Chunk = P265R_SAO16_CHUNK;

// waves per picture: hc CTB rows x (luma strips + 2 x chroma strips)
__host__ __device__ __forceinline__ int sao16_units(const Geo& g) {
    return g.hc * ((g.w + kSao16Strip - 1) / kSao16Strip + 2 * ((g.cw + kSao16Strip - 1) / kSao16Strip));
}

// grid: 4 waves per block, one wave per (picture, CTB row, component, strip), XCD-aware order
template <int L>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(P265R_SAO_WPE))) void sao_strip16_kernel(
        const DevPic* __restrict__ pics, Geo g, BatchView v, int n_pics) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) uint8_t gu8;
    P265R_BW_PRIO_SET();
    const int lane = threadIdx.x & 63;
    const int per_pic = sao16_units(g);
    const int total = per_pic * n_pics;
    const int nblk = (total + 3) >> 2;
    const int bunit = xcd_unit(blockIdx.x, nblk);
    const int unit = __builtin_amdgcn_readfirstlane(bunit * 4 + (int)(threadIdx.x >> 6));
    if (bunit >= nblk || unit >= total) return;                   // whole wave (no barriers below)
    const int pic = unit / per_pic;
    int u = unit - pic * per_pic;
    const int nsl = (g.w + kSao16Strip - 1) / kSao16Strip, nsc = (g.cw + kSao16Strip - 1) / kSao16Strip;
    // unit order inside a picture: CTB row major, then luma strips, Cb strips, Cr strips
    const int cy = u / (nsl + 2 * nsc);
    u -= cy * (nsl + 2 * nsc);
    int c, sx;
    if (u < nsl) { c = 0; sx = u; }
    else { c = 1 + (u - nsl) / nsc; sx = (u - nsl) % nsc; }
    // CTU records: slots of the context size; a ragged batch's smaller picture uses its own raster
    const uint32_t* crec = reinterpret_cast<const uint32_t*>(v.ctus0 + (size_t)pic * g.wc * g.hc);
    if (P265R_RAGGED && g.ragged) {
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)pics[pic].wh));
        if (cy >= g.hc || sx * kSao16Strip >= (c ? g.cw : g.w)) return;   // whole wave, outside this picture
    }
    const int sub = c ? 1 : 0;
    const int Ls = L - sub, cs = 1 << Ls;
    const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
    const int st = (c ? g.stride[1] : g.stride[0]);
    const uint64_t pofs = (uint64_t)pic * v.pic_bytes + v.plane_off[c];
    const gu8* src = (const gu8*)(v.rec0 + pofs);
    gu8* dst = (gu8*)(v.out0 + pofs);
    const int X = sx * kSao16Strip + 16 * (lane - 1);
    const bool act = lane >= 1 && lane <= 62 && X < W;
    const int Xc = min(max(X, 0), ((W - 1) & ~15));               // every lane reads a valid 16-B column
    const int yb = cy << Ls, ye = min(yb + cs, H);
    const int bx = Xc >> Ls, xb = bx << Ls;
    auto row_ld = [&](int y) {
        const __attribute__((address_space(1))) u4v* p =
            (const __attribute__((address_space(1))) u4v*)(src + __umul24((uint32_t)min(max(y, 0), H - 1), (uint32_t)st) + Xc);
        if constexpr (P265R_SAO_NT >= 2) return __builtin_nontemporal_load(p);
        else return *p;
    };
    // ---- first: the rows of the first chunk (position only) ----------------------------------
    constexpr int K = kSao16Chunk;
    u4v rowv[K + 2], nxt[K];
#pragma unroll
    for (int k = 0; k < K + 2; ++k) rowv[k] = row_ld(yb - 1 + k);

    // ---- this lane's CTB: SAO parameters, 8.7.3.2 permissions of its 3x3 neighbourhood ----------
    const int rs = cy * g.wc + bx;
    u4v nb[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int nx = min(max(bx + k % 3 - 1, 0), g.wc - 1), ny = min(max(cy + k / 3 - 1, 0), g.hc - 1);
        nb[k] = *(const __attribute__((address_space(1))) u4v*)(crec + (size_t)(ny * g.wc + nx) * 8);
    }
    const u4v mt = *(const __attribute__((address_space(1))) u4v*)(crec + (size_t)rs * 8 + 4);
    const uint8_t* nf = pics[pic].nofilter;
    uint32_t allow = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int dx = k % 3 - 1, dy = k / 3 - 1;
        const int nx = bx + dx, ny = cy + dy;
        bool ok = nx >= 0 && ny >= 0 && nx < g.wc && ny < g.hc;
        const uint32_t ti = nb[4].y >> 16, to = nb[k].y >> 16;
        if (ok && nb[k].z != nb[4].z) {                          // other slice: the later sample's slice flag
            const bool o_first = to < ti || (to == ti && ny * g.wc + nx < rs);
            ok = ((o_first ? nb[4].w : nb[k].w) & P265R_CTU_LF_ACROSS_SLICES) != 0;
        }
        if (!g.lf_tiles && to != ti) ok = false;
        if (ok) allow |= 1u << k;
    }
    auto A = [&](int ay, int ax) { return ((allow >> (ay * 3 + ax)) & 1u) != 0; };
    // record dword 3: flags | SaoTypeIdx[3] << 8; dword 4: class[3] | dbk offsets; 5..7: offsets
    const int typ = (int)((nb[4].w >> (8 * (c + 1))) & 0xffu);
    const int cls = (int)((mt.x >> (8 * c)) & 0xffu);
    const uint32_t o = c == 0 ? mt.y : (c == 1 ? mt.z : mt.w);    // SaoOffsetVal[1..4], signed bytes
    const uint32_t t_lo = typ == 2 ? __builtin_amdgcn_perm(0u, o, 0x020c0100u) : (o << 8);
    const uint32_t t_hi = o >> 24;
    const uint32_t n_lo = (t_lo >> 7) & 0x01010101u, n_hi = (t_hi >> 7) & 0x01010101u;
    const uint32_t tp_lo = t_lo & ~bytes_ff(n_lo), tp_hi = t_hi & ~bytes_ff(n_hi);
    const uint32_t tn_lo = (~t_lo & bytes_ff(n_lo)) + n_lo, tn_hi = (~t_hi & bytes_ff(n_hi)) + n_hi;
    const uint32_t bsh = (uint32_t)((32 - cls) & 31);
    const uint32_t badd = __umul24(bsh, 0x010101u) | bsh << 24;   // (32 - band position) in every byte
    const int ecls = typ == 2 ? (cls & 3) : 0;
    const bool c0 = ecls == 0, c3 = ecls == 3;
    // a = alignbyte(a_hi, a_lo, sha), b = alignbyte(b_hi, b_lo, shb) with the sources per class:
    //   class 0: a = (cur j, cur j-1, 3)  b = (cur j+1, cur j, 1);  class 1: a = up j, b = dn j (shift 0)
    //   class 2: a = (up j, up j-1, 3)    b = (dn j+1, dn j, 1);    class 3: a = (up j+1, up j, 1)  b = (dn j, dn j-1, 3)
    const uint32_t sha = ecls == 1 ? 0u : (c3 ? 1u : 3u), shb = ecls == 1 ? 0u : (c3 ? 3u : 1u);
    // the same as sources of one shifted row view: a = alignbyte(V[j + ea], V[j + ea - 1], sha) of
    // V = the a-row (class 0: this row, else the row above), b likewise with eb, the b-row
    const bool ea = ecls == 1 || c3, eb = !c3;

    // ---- byte masks: which of the lane's 16 samples may change, per row kind --------------------
    // neighbour (dx, dy) of sample i of row y is usable iff inside the picture and its CTB allowed;
    // only sample 0 / 15 can leave the lane's CTB column, only the CTB row's first / last row its
    // rows; samples at x >= W are stored into the row padding and never read: don't care
    const int n_in = W - Xc;
    const bool ctb_first = Xc == xb, ctb_last = Xc + 16 == xb + cs;
    auto col_bits = [&](int dx, int ay) -> uint32_t {
        if (ay < 0) return 0u;
        if (dx == 0) return A(ay, 1) ? 0xffffu : 0u;
        if (dx < 0) return (A(ay, 1) ? 0xfffeu : 0u) | ((Xc > 0 && A(ay, ctb_first ? 0 : 1)) ? 1u : 0u);
        const uint32_t inner = n_in >= 16 ? 0x7fffu : ((1u << max(n_in - 1, 0)) - 1u);
        return (A(ay, 1) ? inner : 0u) | ((n_in > 16 && A(ay, ctb_last ? 2 : 1)) ? 0x8000u : 0u);
    };
    const int ylast = ye - 1;
    auto row_a = [&](int y, int dy) -> int {
        if (dy == 0) return 1;
        if (dy < 0) return y == yb ? 0 : 1;
        return y == ylast ? (y == H - 1 ? -1 : 2) : 1;
    };
    auto mask16 = [&](int y) -> uint32_t {
        if (typ == 0) return 0u;
        if (typ == 1) return 0xffffu;
        const int dxa = ecls == 1 ? 0 : (c3 ? 1 : -1);
        const int dya = ecls == 0 ? 0 : -1;
        return col_bits(dxa, row_a(y, dya)) & col_bits(-dxa, row_a(y, -dya));
    };
    uint32_t m_top[4], m_mid[4], m_bot[4];
    expand_mask(mask16(yb), m_top);
    expand_mask(mask16(yb + 1), m_mid);
    expand_mask(mask16(ylast), m_bot);
    const bool meo = typ == 2;

    auto split_lo = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c020c00u); };   // bytes 0, 2
    auto split_hi = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c030c01u); };   // bytes 1, 3
    auto join = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x06020400u); };
    auto apply16 = [&](uint32_t v16, uint32_t sel16) {
        const uint32_t pos = __builtin_amdgcn_perm(tp_hi, tp_lo, sel16);
        const uint32_t neg = __builtin_amdgcn_perm(tn_hi, tn_lo, sel16);
        return pk_min_u16(pk_subsat_u16(pk_add_u16(v16, pos), neg), 0x00ff00ffu);
    };
    auto edge16 = [&](uint32_t v16, uint32_t a16, uint32_t b16) {
        return pk_add_u16(pk_add_u16(pk_sgn_i16(pk_sub_i16(v16, a16)), pk_sgn_i16(pk_sub_i16(v16, b16))), 0x0c020c02u);
    };
    // the dword left of the lane's column (lane l - 1's dword 3) / right of it (lane l + 1's dword 0)
    auto left_of = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x138, 0xf, 0xf, false); };
    auto right_of = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x130, 0xf, 0xf, false); };

    // waves without a band-offset lane skip the band arithmetic (wave-uniform choice)
    auto filter_rows = [&](auto has_bo) {
        constexpr bool HB = decltype(has_bo)::value;
        for (int y0 = yb; y0 < ye; y0 += K) {
            if (y0 + K < ye) {
#pragma unroll
                for (int k = 0; k < K; ++k) nxt[k] = row_ld(y0 + K + k + 1);
            }
            // dwords beside the column, per loaded row
            uint32_t lft[K + 2], rgt[K + 2];
#pragma unroll
            for (int k = 0; k < K + 2; ++k) { lft[k] = left_of(rowv[k].w); rgt[k] = right_of(rowv[k].x); }
            auto dw = [&](int k, int j) -> uint32_t {                // dword j (-1 .. 4) of loaded row k
                return j < 0 ? lft[k] : (j > 3 ? rgt[k] : (j == 0 ? rowv[k].x : (j == 1 ? rowv[k].y : (j == 2 ? rowv[k].z : rowv[k].w))));
            };
#pragma unroll
            for (int r = 0; r < K; ++r) {
                const int y = y0 + r;
                const int k = r + 1;
                uint32_t nfm[4] = {0u, 0u, 0u, 0u};
                if (nf) {
                    const int ny = (int)__umul24((uint32_t)((min(y, H - 1) << sub) >> 3), (uint32_t)g.nf_w);
#pragma unroll
                    for (int j = 0; j < 4; ++j) nfm[j] = nf[ny + min(((Xc + 4 * j) << sub) >> 3, g.nf_w - 1)] ? 0xffffffffu : 0u;
                }
                // plane heights are multiples of 4 samples (host-checked), so a chunk's first row is
                // the only one that can be the CTB row's first, its last the only one that can be the last
                const uint32_t* m = r == 0 ? (y == yb ? m_top : m_mid) : (r == K - 1 ? (y == ylast ? m_bot : m_mid) : m_mid);
                // neighbours per lane class: a from row U (this row for class 0, the row above
                // otherwise), b from row D (this row / the row below), each horizontally shifted
                // by the class's dx: one select per dword of U / D and of their shifted views,
                // shared by the row's four dwords
                uint32_t U[6], D[6], Ua[5], Db[5];
#pragma unroll
                for (int j = -1; j <= 4; ++j) {
                    U[j + 1] = c0 ? dw(k, j) : dw(k - 1, j);
                    D[j + 1] = c0 ? dw(k, j) : dw(k + 1, j);
                }
#pragma unroll
                for (int j = -1; j <= 3; ++j) {
                    Ua[j + 1] = ea ? U[j + 2] : U[j + 1];
                    Db[j + 1] = eb ? D[j + 2] : D[j + 1];
                }
                uint32_t out[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t cur = dw(k, j);
                    const uint32_t a = __builtin_amdgcn_alignbyte(Ua[j + 1], Ua[j], sha);
                    const uint32_t b = __builtin_amdgcn_alignbyte(Db[j + 1], Db[j], shb);
                    const uint32_t v_lo = split_lo(cur), v_hi = split_hi(cur);
                    uint32_t sel_lo = edge16(v_lo, split_lo(a), split_lo(b));
                    uint32_t sel_hi = edge16(v_hi, split_hi(a), split_hi(b));
                    if constexpr (HB) {
                        const uint32_t kk = (((cur >> 3) & 0x1f1f1f1fu) + badd) & 0x1f1f1f1fu;
                        const uint32_t big = (((kk & 0x1c1c1c1cu) + 0x7f7f7f7fu) & 0x80808080u) >> 7;
                        const uint32_t sel = (kk + 0x01010101u) & ~bytes_ff(big);
                        sel_lo = meo ? sel_lo : __builtin_amdgcn_perm(0x0c0c0c0cu, sel, 0x04020400u);
                        sel_hi = meo ? sel_hi : __builtin_amdgcn_perm(0x0c0c0c0cu, sel, 0x04030401u);
                    }
                    const uint32_t res = join(apply16(v_lo, sel_lo), apply16(v_hi, sel_hi));
                    const uint32_t mk = m[j] & ~nfm[j];
                    out[j] = (res & mk) | (cur & ~mk);
                }
                if (act && y < ye) {
                    __attribute__((address_space(1))) u4v* q = (__attribute__((address_space(1))) u4v*)(dst + __umul24((uint32_t)y, (uint32_t)st) + Xc);
                    if constexpr (P265R_SAO_NT >= 1) __builtin_nontemporal_store(u4v{out[0], out[1], out[2], out[3]}, q);
                    else *q = u4v{out[0], out[1], out[2], out[3]};
                }
            }
            rowv[0] = rowv[K];
            rowv[1] = rowv[K + 1];
#pragma unroll
            for (int k = 0; k < K; ++k) rowv[k + 2] = nxt[k];
        }
    };
    if (__ballot(act && typ == 1)) filter_rows(std::integral_constant<bool, true>{});
    else filter_rows(std::integral_constant<bool, false>{});
}

}  // namespace p265r
