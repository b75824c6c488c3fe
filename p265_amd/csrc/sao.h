// SAO phase (H.265 8.7.3): band offset / edge offset per CTB and component.
//
// The reference only parses the SAO syntax (decoder/sao.py:15-136) and never filters
// a sample; this kernel is new.  Input is the pre-SAO (here: pre-deblocking)
// reconstructed picture, output a separate plane, so every CTB is independent:
// one 256-thread workgroup per (CTB, picture), all three components.
// HBM traffic per sample: 1 B read (+ halo re-reads served by L2) + 1 B write.
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

__global__ __launch_bounds__(256) void sao_kernel(const DevPic* __restrict__ pics, Geo g) {
    __shared__ int s_allow[9];           // may a sample of this CTB use a neighbour in CTB (dx,dy)?
    const int rs = blockIdx.x;
    const DevPic P = pics[blockIdx.y];
    const int rx = rs % g.wc, ry = rs / g.wc;
    const p265r_ctu me = P.ctus[rs];
    const int tid = threadIdx.x;
    if (tid < 9) {
        const int dx = tid % 3 - 1, dy = tid / 3 - 1;
        const int nx = rx + dx, ny = ry + dy;
        int ok = 1;
        if (nx < 0 || ny < 0 || nx >= g.wc || ny >= g.hc) ok = 0;
        else if (dx || dy) {
            const int ro = ny * g.wc + nx;
            const p265r_ctu o = P.ctus[ro];
            if (o.slice_addr != me.slice_addr) {
                // 8.7.3.2: the flag of the slice containing the LATER of the two samples
                ok = ts_before(o, ro, me, rs) ? (me.flags & P265R_CTU_LF_ACROSS_SLICES) != 0
                                              : (o.flags & P265R_CTU_LF_ACROSS_SLICES) != 0;
            }
            if (!g.lf_tiles && o.tile_id != me.tile_id) ok = 0;
        }
        s_allow[tid] = ok;
    }
    __syncthreads();
    const int ctb = 1 << g.ctb_log2;
    for (int c = 0; c < 3; ++c) {
        const int sub = c ? 1 : 0;
        const int cs = ctb >> sub;
        const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
        const int xb = rx * cs, yb = ry * cs;
        const int wv = min(cs, W - xb), hv = min(cs, H - yb);
        const uint8_t* src = P.rec[c];
        uint8_t* dst = P.out[c];
        const int st = g.stride[c];
        const int typ = me.sao_type[c];
        const int maxv = (1 << g.bd[c]) - 1;
        const int o1 = me.sao_offset[c][0], o2 = me.sao_offset[c][1];
        const int o3 = me.sao_offset[c][2], o4 = me.sao_offset[c][3];
        // SaoOffsetVal[i], i = 0..4 (register select; no runtime-indexed local array)
        auto offv = [&](int i) { return i == 1 ? o1 : i == 2 ? o2 : i == 3 ? o3 : i == 4 ? o4 : 0; };
        const int shift = g.bd[c] - 5;
        const int cls = me.sao_class[c];
        const int ax = cls == 1 ? 0 : (cls == 3 ? 1 : -1);
        const int ay = cls == 0 ? 0 : -1;
        for (int e = tid; e < wv * hv; e += 256) {
            const int yy = e / wv, xx = e - yy * wv;
            const int X = xb + xx, Y = yb + yy;
            const size_t o = (size_t)Y * st + X;
            const int v = src[o];
            int r = v;
            bool skip = typ == 0;
            if (!skip && P.nofilter) skip = P.nofilter[((Y << sub) >> 3) * g.nf_w + ((X << sub) >> 3)] != 0;
            if (!skip) {
                if (typ == 1) {
                    const int bi = ((v >> shift) - cls) & 31;     // bandTable[v >> bandShift] - 1
                    if (bi < 4) r = min(max(v + offv(bi + 1), 0), maxv);
                } else {
                    const int xa = X + ax, ya = Y + ay, xc = X - ax, yc = Y - ay;
                    bool ok = xa >= 0 && ya >= 0 && xa < W && ya < H && xc >= 0 && yc >= 0 && xc < W && yc < H;
                    if (ok) {
                        const int da = (xa < xb ? 0 : (xa >= xb + cs ? 2 : 1)) + 3 * (ya < yb ? 0 : (ya >= yb + cs ? 2 : 1));
                        const int dc = (xc < xb ? 0 : (xc >= xb + cs ? 2 : 1)) + 3 * (yc < yb ? 0 : (yc >= yb + cs ? 2 : 1));
                        ok = s_allow[da] && s_allow[dc];
                    }
                    if (ok) {
                        int ei = 2 + sgn(v - (int)src[(size_t)ya * st + xa]) + sgn(v - (int)src[(size_t)yc * st + xc]);
                        ei = ei == 2 ? 0 : (ei < 2 ? ei + 1 : ei);
                        r = min(max(v + offv(ei), 0), maxv);
                    }
                }
            }
            dst[o] = (uint8_t)r;
        }
    }
}

}  // namespace p265r
