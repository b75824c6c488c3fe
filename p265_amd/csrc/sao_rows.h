// SAO-only in-loop filter pass (H.265 8.7.3) for batches without deblocking: a streaming
// kernel, no LDS.  (Batches with deblocking keep the fused deblocking + SAO window kernel of
// loopfilter.h.)  The reference parses the SAO syntax (decoder/sao.py:15-136) and never filters.
//
// One wave = one CTB row of one component over a strip of 62 sample dwords (lane l: the 4-sample
// dword at x = 248 s + 4 (l - 1); lanes 0 and 63 only supply the neighbours of lanes 1 and 62).
// The wave walks down the CTB row 8 output rows at a time: the 10 rows a chunk needs are loaded
// one chunk ahead (one dword per lane and row, a 256-byte coalesced load per row, all in
// flight together), left / right neighbour dwords come from lanes l -/+ 1 by DPP wave shifts,
// 4 samples per dword are filtered with the SWAR arithmetic of loopfilter.h and the dword is
// stored to the output plane.  Each lane's CTB (SaoTypeIdx, class, offsets, the 8.7.3.2
// neighbour permissions) is fixed for the wave.  HBM traffic per sample: one read (+ 2 halo rows
// per CTB height, + 2 / 62 halo columns) and one write.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "../../include/p265r.h"
#include "intra.h"
#include "loopfilter.h"
#include "sao.h"

namespace p265r {

#ifndef P265R_SAO_CHUNK
#define P265R_SAO_CHUNK 8
#endif
constexpr int kSaoRowsChunk = P265R_SAO_CHUNK;   // output rows per load batch

constexpr int kSaoStrip = 248;             // output samples per strip (62 dwords)

// waves per picture: hc CTB rows x (luma strips + 2 x chroma strips)
__host__ __device__ __forceinline__ int sao_rows_units(const Geo& g) {
    return g.hc * ((g.w + kSaoStrip - 1) / kSaoStrip + 2 * ((g.cw + kSaoStrip - 1) / kSaoStrip));
}

// grid: 4 waves per block, one wave per (picture, component, CTB row, strip), XCD-aware order
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void sao_rows_kernel(const DevPic* __restrict__ pics, Geo g, int n_pics) {
    const int lane = threadIdx.x & 63;
    const int per_pic = sao_rows_units(g);
    const int total = per_pic * n_pics;
    const int nblk = (total + 3) >> 2;
    const int bunit = xcd_unit(blockIdx.x, nblk);                 // block -> 4 consecutive units
    // wave-uniform (readfirstlane): everything derived from the unit lives in SGPRs
    const int unit = __builtin_amdgcn_readfirstlane(bunit * 4 + (int)(threadIdx.x >> 6));
    if (bunit >= nblk || unit >= total) return;                   // whole wave (no barriers below)
    const int pic = unit / per_pic;
    int u = unit - pic * per_pic;
    const int nsl = (g.w + kSaoStrip - 1) / kSaoStrip, nsc = (g.cw + kSaoStrip - 1) / kSaoStrip;
    // unit order inside a picture: CTB row major, then luma strips, Cb strips, Cr strips
    const int cy = u / (nsl + 2 * nsc);
    u -= cy * (nsl + 2 * nsc);
    int c, sx;
    if (u < nsl) { c = 0; sx = u; }
    else { c = 1 + (u - nsl) / nsc; sx = (u - nsl) % nsc; }
    typedef __attribute__((address_space(1))) uint8_t gu8;
    typedef __attribute__((address_space(1))) uint32_t gu32;
    const DevPic* P = pics + pic;
    if (P265R_RAGGED && g.ragged) {                                               // this picture's size and CTU raster
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)P->wh));
        if (cy >= g.hc || sx * kSaoStrip >= (c ? g.cw : g.w)) return;   // whole wave, outside this picture
    }
    const int sub = c ? 1 : 0;
    const int Ls = g.ctb_log2 - sub, cs = 1 << Ls;
    const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
    const int st = (c ? g.stride[1] : g.stride[0]);
    const gu8* src = (const gu8*)P->rec[c];
    gu8* dst = (gu8*)P->out[c];
    const int X = sx * kSaoStrip + 4 * (lane - 1);
    const bool act = lane >= 1 && lane <= 62 && X < W;
    const int Xc = min(max(X, 0), W - 4);                         // every lane reads a valid dword
    const int yb = cy << Ls, ye = min(yb + cs, H);
    const int bx = Xc >> Ls, xb = bx << Ls;

    // ---- this lane's CTB: SAO parameters and 8.7.3.2 permissions of its 3x3 neighbourhood ----
    // (the nine records' first 16 B are loaded together; 8.7.3.2 as sao.h sao_allow)
    const gu32* crec = (const gu32*)P->ctus;
    const int rs = cy * g.wc + bx;
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    u4v nb[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int nx = min(max(bx + k % 3 - 1, 0), g.wc - 1), ny = min(max(cy + k / 3 - 1, 0), g.hc - 1);
        nb[k] = *(const __attribute__((address_space(1))) u4v*)(crec + (size_t)(ny * g.wc + nx) * 8);
    }
    const u4v mt = *(const __attribute__((address_space(1))) u4v*)(crec + (size_t)rs * 8 + 4);
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
    auto rok = [&](int rr, int cc) { return ((allow >> (rr * 3 + cc)) & 1u) != 0; };
    // record dword 3: flags | SaoTypeIdx[3] << 8; dword 4: class[3] | dbk offsets; 5..7: offsets
    const int typ = (int)((nb[4].w >> (8 * (c + 1))) & 0xffu);
    const int cls = (int)((mt.x >> (8 * c)) & 0xffu);
    const uint32_t o = c == 0 ? mt.y : (c == 1 ? mt.z : mt.w);    // SaoOffsetVal[1..4], signed bytes
    // 8-entry byte tables (lo: entries 0..3, hi: 4..7) of max(off, 0) and max(-off, 0): EO raw
    // e = 2 + sgn + sgn -> edgeIdx 1, 2, 0, 3, 4; BO slot 1..4 = the four bands, slot 0 = none
    const uint32_t t_lo = typ == 2 ? __builtin_amdgcn_perm(0u, o, 0x020c0100u) : (o << 8);
    const uint32_t t_hi = o >> 24;
    const uint32_t n_lo = (t_lo >> 7) & 0x01010101u, n_hi = (t_hi >> 7) & 0x01010101u;
    const uint32_t tp_lo = t_lo & ~(n_lo * 0xffu), tp_hi = t_hi & ~(n_hi * 0xffu);
    const uint32_t tn_lo = (~t_lo & (n_lo * 0xffu)) + n_lo, tn_hi = (~t_hi & (n_hi * 0xffu)) + n_hi;
    const uint32_t badd = (uint32_t)((32 - cls) & 31) * 0x01010101u;
    const int cl = Xc == xb ? 0 : 1, cr = Xc + 4 == xb + cs ? 2 : 1;
    const bool has_l = Xc > 0, right_in = Xc + 4 < W;
    const gu8* nf = (const gu8*)P->nofilter;
    // Everything per lane below is a bit mask, not a branch: the lanes of a wave span several
    // CTBs of different type / class (the compiler otherwise branches with EXEC juggling per row).
    auto msk = [](bool b) { return b ? 0xffffffffu : 0u; };
    const uint32_t mc0 = msk(cls == 0), mc1 = msk(cls == 1), mc2 = msk(cls == 2), mc3 = msk(cls == 3);
    const uint32_t meo = msk(typ == 2);
    // which samples may change (8.7.3.2: EO neighbours inside the picture and in a CTB this one
    // may use; SaoTypeIdx != 0), per kind of row: rup / rdn = CTB row of the up / down neighbour
    auto okm_of = [&](bool vert, int rup, int rdn) -> uint32_t {
        if (typ == 0) return 0u;
        if (typ == 1) return 0xffffffffu;
        const bool v_ok = vert && rok(rup, 1) && rok(rdn, 1);
        bool mid, first, last;
        if (cls == 0) { mid = true; first = has_l && rok(1, cl); last = right_in && rok(1, cr); }
        else if (cls == 1) { mid = first = last = v_ok; }
        else if (cls == 2) {
            mid = v_ok;
            first = vert && has_l && rok(rup, cl) && rok(rdn, 1);
            last = vert && right_in && rok(rup, 1) && rok(rdn, cr);
        } else {
            mid = v_ok;
            first = vert && has_l && rok(rup, 1) && rok(rdn, cl);
            last = vert && right_in && rok(rup, cr) && rok(rdn, 1);
        }
        return (mid ? 0x00ffff00u : 0u) | (first ? 0xffu : 0u) | (last ? 0xff000000u : 0u);
    };
    const uint32_t ok_top = okm_of(true, 0, 1), ok_mid = okm_of(true, 1, 1), ok_bot = okm_of(true, 1, 2);
    const uint32_t ok_nv = okm_of(false, 1, 1);                   // picture's first / last row

    auto split_lo = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c020c00u); };   // bytes 0, 2
    auto split_hi = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c030c01u); };   // bytes 1, 3
    auto join = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x06020400u); };
    auto apply = [&](uint32_t v, uint32_t sel) {                  // v + table[sel] clipped to [0, 255]
        const uint32_t pos = __builtin_amdgcn_perm(tp_hi, tp_lo, sel);
        const uint32_t neg = __builtin_amdgcn_perm(tn_hi, tn_lo, sel);
        const uint32_t m255 = 0x00ff00ffu;
        const uint32_t rl = pk_min_u16(pk_subsat_u16(pk_add_u16(split_lo(v), split_lo(pos)), split_lo(neg)), m255);
        const uint32_t rh = pk_min_u16(pk_subsat_u16(pk_add_u16(split_hi(v), split_hi(pos)), split_hi(neg)), m255);
        return join(rl, rh);
    };
    auto gt = [&](uint32_t v, uint32_t a) { return pk_min_u16(pk_subsat_u16(v, a), 0x00010001u); };
    auto edge = [&](uint32_t v, uint32_t a, uint32_t b) {      // 2 + sgn(v - a) + sgn(v - b), 16-bit lanes
        return pk_sub_u16(pk_add_u16(pk_add_u16(gt(v, a), gt(v, b)), 0x00020002u), pk_add_u16(gt(a, v), gt(b, v)));
    };

    // dwords left / right of this lane's: lanes l -/+ 1 (DPP wave shifts; lanes 0 / 63 are not output)
    auto left_of = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xf, 0xf, false); };
    auto right_of = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x130, 0xf, 0xf, false); };
    auto row_ld = [&](int y) { return *(const gu32*)(src + (size_t)min(max(y, 0), H - 1) * st + Xc); };
    constexpr int K = kSaoRowsChunk;
    // rows y0 - 1 .. y0 + K of the current chunk; the next chunk's K new rows are loaded before
    // the current chunk is filtered.  A chunk is one basic block (rows past the CTB row are
    // computed and not stored), so the scheduler interleaves its independent rows.
    // waves without a band-offset CTB (about half of them: ~82 % of CTBs are edge-offset) skip the
    // band arithmetic; the choice is wave-uniform
    auto filter_rows = [&](auto has_bo) {
        constexpr bool HB = decltype(has_bo)::value;
        uint32_t rowv[K + 2], nxt[K];
        rowv[0] = row_ld(yb - 1);
        rowv[1] = row_ld(yb);
#pragma unroll
        for (int k = 2; k < K + 2; ++k) rowv[k] = row_ld(yb + k - 1);
        for (int y0 = yb; y0 < ye; y0 += K) {
            if (y0 + K < ye) {
#pragma unroll
                for (int k = 0; k < K; ++k) nxt[k] = row_ld(y0 + K + k + 1);
            }
            uint32_t nfm[K];                                          // PCM / bypass samples: unchanged
#pragma unroll
            for (int k = 0; k < K; ++k) nfm[k] = 0u;
            if (nf) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    nfm[k] = nf[(size_t)((min(y0 + k, H - 1) << sub) >> 3) * g.nf_w + ((Xc << sub) >> 3)] ? 0xffffffffu : 0u;
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int y = y0 + k;
                const uint32_t cur = rowv[k + 1], up = rowv[k], dn = rowv[k + 2];
                const uint32_t lc = left_of(cur), rc = right_of(cur);
                const uint32_t lu = left_of(up), ru_ = right_of(up);
                const uint32_t ld = left_of(dn), rd_ = right_of(dn);
                // edge offset: neighbours a, b of the 4 samples (byte-aligned) per SaoEoClass
                const uint32_t a = (__builtin_amdgcn_alignbyte(cur, lc, 3) & mc0) | (up & mc1) |
                                   (__builtin_amdgcn_alignbyte(up, lu, 3) & mc2) | (__builtin_amdgcn_alignbyte(ru_, up, 1) & mc3);
                const uint32_t b = (__builtin_amdgcn_alignbyte(rc, cur, 1) & mc0) | (dn & mc1) |
                                   (__builtin_amdgcn_alignbyte(rd_, dn, 1) & mc2) | (__builtin_amdgcn_alignbyte(dn, ld, 3) & mc3);
                const uint32_t sel_eo = join(edge(split_lo(cur), split_lo(a), split_lo(b)), edge(split_hi(cur), split_hi(a), split_hi(b)));
                uint32_t sel = sel_eo;
                if constexpr (HB) {
                    // band offset: slot 1..4 for the four bands from sao_band_position, else 0
                    const uint32_t kk = (((cur >> 3) & 0x1f1f1f1fu) + badd) & 0x1f1f1f1fu;
                    const uint32_t big = (((kk & 0x1c1c1c1cu) + 0x7f7f7f7fu) & 0x80808080u) >> 7;
                    const uint32_t sel_bo = (kk + 0x01010101u) & ~((big << 8) - big);
                    sel = (sel_eo & meo) | (sel_bo & ~meo);
                }
                // row kind (wave-uniform): picture's first / last row, CTB's first / last row, other
                const uint32_t okm = ((y == 0 || y + 1 == H) ? ok_nv : (y == yb ? ok_top : (y == yb + cs - 1 ? ok_bot : ok_mid))) & ~nfm[k];
                const uint32_t res = (apply(cur, sel) & okm) | (cur & ~okm);
                if (act && y < ye) *(gu32*)(dst + (size_t)y * st + X) = res;
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
