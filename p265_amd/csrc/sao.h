// SAO phase (H.265 8.7.3): band offset / edge offset per CTB and component.
//
// The reference only parses the SAO syntax (decoder/sao.py:15-136) and never filters
// a sample; this kernel is new.  Input is the pre-SAO (here: pre-deblocking)
// reconstructed picture, output a separate plane, so every CTB is independent:
// one workgroup per (CTB, picture) covering all three components, one thread per
// SEG-sample row segment (SEG = 16; 8 for 16x16 CTBs).  Each thread loads its segment
// and, for edge offset, the rows above/below plus one sample left/right as dwords
// (neighbour re-reads hit L2), classifies its SEG samples in registers and writes one
// 16-B (8-B) store.  HBM traffic per sample: 1 B read + 1 B write.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"

namespace p265r {

__device__ __forceinline__ bool ts_before(const p265r_ctu& a, int ra, const p265r_ctu& b, int rb) {
    // CtbAddrRsToTs[a] < CtbAddrRsToTs[b]; tiles are numbered in tile-scan order
    return a.tile_id < b.tile_id || (a.tile_id == b.tile_id && ra < rb);
}

__device__ __forceinline__ int sgn(int v) { return (v > 0) - (v < 0); }

// may samples of CTB rs use samples of the neighbouring CTB (dx, dy)?  (8.7.3.2)
__device__ __forceinline__ bool sao_allow(const p265r_ctu* ctus, const p265r_ctu& me, int rs, int rx, int ry,
                                          int dx, int dy, const Geo& g) {
    const int nx = rx + dx, ny = ry + dy;
    if (nx < 0 || ny < 0 || nx >= g.wc || ny >= g.hc) return false;
    if (!dx && !dy) return true;
    const int ro = ny * g.wc + nx;
    const p265r_ctu o = ctus[ro];
    bool ok = true;
    if (o.slice_addr != me.slice_addr) {
        // the flag of the slice containing the LATER of the two samples
        ok = ts_before(o, ro, me, rs) ? (me.flags & P265R_CTU_LF_ACROSS_SLICES) != 0
                                      : (o.flags & P265R_CTU_LF_ACROSS_SLICES) != 0;
    }
    if (!g.lf_tiles && o.tile_id != me.tile_id) ok = false;
    return ok;
}

template <int SEG>
__global__ __launch_bounds__(384) void sao_kernel(const DevPic* __restrict__ pics, Geo g) {
    constexpr int NW = SEG / 4;                 // words per segment
    __shared__ uint32_t s_allow;
    const int rs = blockIdx.x;
    const DevPic* P = pics + blockIdx.y;
    const p265r_ctu* ctus = P->ctus;
    const int rx = rs % g.wc, ry = rs / g.wc;
    const p265r_ctu me = ctus[rs];
    const int tid = threadIdx.x;
    if (tid < 64) {
        const bool ok = tid < 9 && sao_allow(ctus, me, rs, rx, ry, tid % 3 - 1, tid / 3 - 1, g);
        const uint32_t bits = (uint32_t)__ballot(ok);
        if (tid == 0) s_allow = bits;
    }
    __syncthreads();
    const uint32_t allow = s_allow;

    // ---- task -> (component, row, segment) ------------------------------------------
    const int ctb_log2 = g.ctb_log2;
    const int cs_l = 1 << ctb_log2;
    constexpr int seg_log = SEG == 16 ? 4 : 3;
    const int nl = (cs_l >> seg_log) * cs_l;                 // luma tasks
    const int nc = ((cs_l >> 1) >> seg_log) * (cs_l >> 1);   // tasks per chroma component
    int c, t;
    if (tid < nl) { c = 0; t = tid; }
    else if (tid < nl + nc) { c = 1; t = tid - nl; }
    else if (tid < nl + 2 * nc) { c = 2; t = tid - nl - nc; }
    else return;
    const int sub = c ? 1 : 0;
    const int cs = cs_l >> sub;
    const int spr_log = (ctb_log2 - sub) - seg_log;          // segments per row (log2)
    const int row = t >> spr_log, col = (t & ((1 << spr_log) - 1)) << seg_log;
    const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
    const int xb = rx * cs, yb = ry * cs;
    const int X = xb + col, Y = yb + row;
    if (X >= W || Y >= H) return;
    const int st = c == 0 ? g.stride[0] : g.stride[1];
    const uint8_t* src = P->rec[c];
    uint8_t* dst = P->out[c];
    const int typ = me.sao_type[c];
    const size_t o = (size_t)Y * st + X;

    uint32_t cur[NW];
    if constexpr (SEG == 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + o);
        cur[0] = v.x; cur[1] = v.y; cur[2] = v.z; cur[3] = v.w;
    } else {
        const uint2 v = *reinterpret_cast<const uint2*>(src + o);
        cur[0] = v.x; cur[1] = v.y;
    }
    uint32_t res[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) res[q] = cur[q];

    if (typ != 0) {
        // samples of PCM / bypass CUs with loop filtering disabled stay unchanged
        uint32_t keep = 0;                           // bit i: sample i not filtered
        if (P->nofilter) {
            const uint8_t* nf = P->nofilter + (size_t)((Y << sub) >> 3) * g.nf_w;
#pragma unroll
            for (int i = 0; i < SEG; i += 4)          // 4 samples never straddle an 8x8 luma block
                if (nf[((X + i) << sub) >> 3]) keep |= 0xfu << i;
        }
        const int o1 = me.sao_offset[c][0], o2 = me.sao_offset[c][1];
        const int o3 = me.sao_offset[c][2], o4 = me.sao_offset[c][3];
        auto offv = [&](int i) { return i == 1 ? o1 : i == 2 ? o2 : i == 3 ? o3 : i == 4 ? o4 : 0; };
        const int cls = me.sao_class[c];
        if (typ == 1) {
            // band offset: bandTable[v >> 3] = k + 1 for bands sao_band_position + k, k < 4
#pragma unroll
            for (int i = 0; i < SEG; ++i) {
                const int v = (cur[i >> 2] >> (8 * (i & 3))) & 0xff;
                const int bi = ((v >> 3) - cls) & 31;
                int r = v;
                if (bi < 4) r = min(max(v + offv(bi + 1), 0), 255);
                if ((keep >> i) & 1u) r = v;
                res[i >> 2] = (res[i >> 2] & ~(0xffu << (8 * (i & 3)))) | ((uint32_t)r << (8 * (i & 3)));
            }
        } else {
            // edge offset: neighbours a = (x+ax, y+ay), b = (x-ax, y-ay)
            const int ax = cls == 1 ? 0 : (cls == 3 ? 1 : -1);
            const int ay = cls == 0 ? 0 : -1;
            // extended rows: word 0 = dword at X-4 (byte 3 = sample X-1), words 1..NW =
            // the segment, word NW+1 = dword at X+SEG (byte 0 = sample X+SEG)
            uint32_t up[NW + 2], mid[NW + 2], dn[NW + 2];
            const bool has_l = X > 0, has_r = X + SEG < W;
            const bool has_u = Y > 0, has_d = Y + 1 < H;
            auto load_row = [&](uint32_t* e, int yy) {
                const uint8_t* p = src + (size_t)yy * st + X;
                if constexpr (SEG == 16) {
                    const uint4 v = *reinterpret_cast<const uint4*>(p);
                    e[1] = v.x; e[2] = v.y; e[3] = v.z; e[4] = v.w;
                } else {
                    const uint2 v = *reinterpret_cast<const uint2*>(p);
                    e[1] = v.x; e[2] = v.y;
                }
                e[0] = has_l ? *reinterpret_cast<const uint32_t*>(p - 4) : 0u;
                e[NW + 1] = has_r ? *reinterpret_cast<const uint32_t*>(p + SEG) : 0u;
            };
#pragma unroll
            for (int q = 0; q < NW; ++q) { mid[q + 1] = cur[q]; up[q + 1] = 0; dn[q + 1] = 0; }
            mid[0] = has_l ? *reinterpret_cast<const uint32_t*>(src + o - 4) : 0u;
            mid[NW + 1] = has_r ? *reinterpret_cast<const uint32_t*>(src + o + SEG) : 0u;
            up[0] = up[NW + 1] = dn[0] = dn[NW + 1] = 0;
            if (ay != 0) {
                if (has_u) load_row(up, Y - 1);
                if (has_d) load_row(dn, Y + 1);
            }
            // neighbour permission by CTB region: row region of y-1 / y+1, column region of x-1 / x+SEG
            const int ru = Y == yb ? 0 : 1, rd = Y == yb + cs - 1 ? 2 : 1;
            const int cl = X == xb ? 0 : 1, cr = X + SEG == xb + cs ? 2 : 1;
            auto region_ok = [&](int rr, int cc) { return (allow >> (rr * 3 + cc)) & 1u; };
            auto byte_at = [&](const uint32_t* e, int j) {        // j = -1 .. SEG
                return (int)((e[(j + 4) >> 2] >> (8 * ((j + 4) & 3))) & 0xff);
            };
#pragma unroll
            for (int i = 0; i < SEG; ++i) {
                const int v = (cur[i >> 2] >> (8 * (i & 3))) & 0xff;
                const int ja = i + ax, jb = i - ax;                 // column offsets (-1..SEG)
                // availability of a (row y+ay) and b (row y-ay)
                const int ca = ja < 0 ? cl : (ja >= SEG ? cr : 1);
                const int cb = jb < 0 ? cl : (jb >= SEG ? cr : 1);
                // (a segment may overhang the picture's right edge: X + j < W per sample)
                const bool xa_in = ja < 0 ? has_l : X + ja < W;
                const bool xb_in = jb < 0 ? has_l : X + jb < W;
                bool ok, okb;
                int a, b;
                if (ay == 0) {
                    ok = xa_in && region_ok(1, ca);
                    okb = xb_in && region_ok(1, cb);
                    a = byte_at(mid, ja); b = byte_at(mid, jb);
                } else {                                            // ay = -1: a above, b below
                    ok = has_u && xa_in && region_ok(ru, ca);
                    okb = has_d && xb_in && region_ok(rd, cb);
                    a = byte_at(up, ja); b = byte_at(dn, jb);
                }
                int r = v;
                if (ok && okb) {
                    int ei = 2 + sgn(v - a) + sgn(v - b);
                    ei = ei == 2 ? 0 : (ei < 2 ? ei + 1 : ei);
                    r = min(max(v + offv(ei), 0), 255);
                }
                if ((keep >> i) & 1u) r = v;
                res[i >> 2] = (res[i >> 2] & ~(0xffu << (8 * (i & 3)))) | ((uint32_t)r << (8 * (i & 3)));
            }
        }
    }
    if constexpr (SEG == 16) *reinterpret_cast<uint4*>(dst + o) = make_uint4(res[0], res[1], res[2], res[3]);
    else *reinterpret_cast<uint2*>(dst + o) = make_uint2(res[0], res[1]);
}

}  // namespace p265r
