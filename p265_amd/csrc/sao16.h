// SAO only (8.7.3) for 16-bit samples (BitDepth 9..10, Main 10): a streaming kernel, one thread per
// 8 consecutive samples of one row of one plane (16-B loads and stores), for batches without
// deblocking.  Same arithmetic as the SAO part of loopfilter16.h (band: bandShift = BitDepth - 5;
// edge classes with the 8.7.3.2 neighbour rules: picture edges, slices, tiles; PCM / bypass samples
// untouched), without staging CTB windows in LDS: the rows above and below come straight from the
// reconstruction (L2-resident: consecutive blocks walk consecutive rows of one XCD).
//
// The reference only parses the SAO syntax (decoder/sao.py:15-136, SaoOffsetVal sao.py:174-178); the
// filter rests on the spec restatement (oracle/recon_oracle.py sao_picture).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"
#include "loopfilter.h"
#include "sao.h"

namespace p265r {

// row units per picture in the context's layout: luma rows, then Cb rows, then Cr rows
__host__ __device__ __forceinline__ int sao16_rows(const Geo& g) { return g.h + 2 * g.ch; }

// grid: 8 * ceil(row units * pictures / 8) blocks of 256 threads, one row of one plane per block (XCD-aware
// block order: consecutive rows on one XCD, so the rows above / below are L2 hits); thread t takes the
// 8-sample groups t, t + 256, ... of the row
__global__ __launch_bounds__(256) void sao16_kernel(const DevPic* __restrict__ pics, Geo g, int n_pics) {
    const int upp = sao16_rows(g);
    const int nunits = upp * n_pics;
    const int lu = xcd_unit(blockIdx.x, nunits);
    if (lu >= nunits) return;
    const int pic = __builtin_amdgcn_readfirstlane(lu / upp);
    const int u = __builtin_amdgcn_readfirstlane(lu - pic * upp);
    const int c = u < g.h ? 0 : (u < g.h + g.ch ? 1 : 2);
    const int Y = u < g.h ? u : (u - g.h - (c - 1) * g.ch);
    const DevPic* P = pics + pic;
    Geo pg = g;
    if (P265R_RAGGED && g.ragged) pg = pic_geo(g, P->wh);     // (strides stay the context's)
    const int sub = c ? 1 : 0;
    const int W = c ? pg.cw : pg.w, H = c ? pg.ch : pg.h;
    if (Y >= H) return;
    for (int X0 = (int)threadIdx.x * 8; X0 < W; X0 += 256 * 8) {
        const int ctbl = pg.ctb_log2 - sub, cs = 1 << ctbl;
        const int rx = X0 >> ctbl, ry = Y >> ctbl, rs = ry * pg.wc + rx;
        const p265r_ctu* ctus = P->ctus;
        const p265r_ctu& me = ctus[rs];                             // (its fields are read from memory, indexed by c)
        const int st = c ? g.stride[1] : g.stride[0];
        const uint16_t* in = reinterpret_cast<const uint16_t*>(P->rec[c]);
        uint16_t* out = reinterpret_cast<uint16_t*>(P->out[c]);
        const uint4 cv = *reinterpret_cast<const uint4*>(in + (size_t)Y * st + X0);
        uint32_t w[4] = {cv.x, cv.y, cv.z, cv.w};
        auto smp = [](const uint32_t* ww, int i) { return (int)((ww[i >> 1] >> (16 * (i & 1))) & 0xffffu); };
        const int typ = me.sao_type[c];
        if (typ != 0) {
            const int bd = c ? g.bd[1] : g.bd[0], maxv = (1 << bd) - 1;
            const int cls = me.sao_class[c];
            const uint32_t offw = *reinterpret_cast<const uint32_t*>(&me.sao_offset[c][0]);   // SaoOffsetVal[1..4]
            auto off = [&](int k) { return (int)(int8_t)(offw >> (8 * k)); };
            // PCM / bypass (nofilter, per 8x8 luma block): chroma groups span two luma blocks
            uint32_t nfm = 0;                                          // bit i: sample i untouched
            if (P->nofilter) {
                const int ly = Y << sub, lx = X0 << sub;
                const uint8_t* nf = P->nofilter + (size_t)(ly >> 3) * pg.nf_w;
                if (nf[lx >> 3]) nfm |= c ? 0x0fu : 0xffu;
                if (c && (lx >> 3) + 1 < pg.nf_w && nf[(lx >> 3) + 1]) nfm |= 0xf0u;
            }
            int res[8];
            if (typ == 1) {
    #pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int v = smp(w, i);
                    const int k = ((v >> (bd - 5)) - cls) & 31;       // band slot relative to the position
                    res[i] = k < 4 ? min(max(v + off(k), 0), maxv) : v;
                }
            } else {
                const int ax = cls == 0 ? -1 : (cls == 1 ? 0 : (cls == 2 ? -1 : 1));
                const int ay = cls == 0 ? 0 : -1;
                // neighbour rows (ay = -1: above for a, below for b); each: samples X0 - 1 .. X0 + 8
                uint32_t wa[4] = {0, 0, 0, 0}, wb[4] = {0, 0, 0, 0};
                int la = 0, ra = 0, lbv = 0, rbv = 0;                  // the samples beside the 8 (a row / b row)
                const bool va = Y + ay >= 0, vb = Y - ay < H;          // rows inside the picture
                if (ay != 0) {
                    if (va) {
                        const uint16_t* row = in + (size_t)(Y - 1) * st + X0;
                        const uint4 t = *reinterpret_cast<const uint4*>(row);
                        wa[0] = t.x; wa[1] = t.y; wa[2] = t.z; wa[3] = t.w;
                        if (X0 > 0) la = row[-1];
                        if (X0 + 8 < W) ra = row[8];
                    }
                    if (vb) {
                        const uint16_t* row = in + (size_t)(Y + 1) * st + X0;
                        const uint4 t = *reinterpret_cast<const uint4*>(row);
                        wb[0] = t.x; wb[1] = t.y; wb[2] = t.z; wb[3] = t.w;
                        if (X0 > 0) lbv = row[-1];
                        if (X0 + 8 < W) rbv = row[8];
                    }
                } else {
                    const uint16_t* row = in + (size_t)Y * st + X0;
                    if (X0 > 0) la = lbv = row[-1];
                    if (X0 + 8 < W) ra = rbv = row[8];
    #pragma unroll
                    for (int q = 0; q < 4; ++q) { wa[q] = w[q]; wb[q] = w[q]; }
                }
                // 8.7.3.2 across CTB borders: the 3 x 3 CTB neighbourhood's permissions, only where a
                // neighbour of this group can lie outside its CTB
                const int col0 = X0 & (cs - 1), row0 = Y & (cs - 1);
                uint32_t allow = 1u << 4;                              // (0, 0)
                const bool edge = col0 == 0 || col0 + 8 >= cs || row0 == 0 || row0 == cs - 1;
                if (edge) {
                    for (int k = 0; k < 9; ++k)
                        if (k != 4 && sao_allow(ctus, me, rs, rx, ry, k % 3 - 1, k / 3 - 1, pg)) allow |= 1u << k;
                } else {
                    allow = 0x1ffu;
                }
                auto ok_at = [&](int x, int y) {                       // neighbour sample (x, y) usable?
                    if (x < 0 || x >= W || y < 0 || y >= H) return false;
                    const int dx = (x >> ctbl) - rx, dy = (y >> ctbl) - ry;
                    return ((allow >> ((dy + 1) * 3 + dx + 1)) & 1u) != 0;
                };
    #pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int v = smp(w, i);
                    const int X = X0 + i;
                    // neighbour columns i + ax / i - ax (ax = -1, 0, 1): every candidate at a compile-time
                    // index (no dynamically indexed register array, which would go to scratch)
                    const int am = i == 0 ? la : smp(wa, i > 0 ? i - 1 : 0), a0 = smp(wa, i), ap = i == 7 ? ra : smp(wa, i < 7 ? i + 1 : 7);
                    const int bm = i == 0 ? lbv : smp(wb, i > 0 ? i - 1 : 0), b0 = smp(wb, i), bp = i == 7 ? rbv : smp(wb, i < 7 ? i + 1 : 7);
                    const int a = ax < 0 ? am : (ax == 0 ? a0 : ap);
                    const int b = ax > 0 ? bm : (ax == 0 ? b0 : bp);
                    const bool ok = ok_at(X + ax, Y + ay) && ok_at(X - ax, Y - ay);
                    int e = 2 + (v > a) - (v < a) + (v > b) - (v < b);
                    e = e == 2 ? 0 : (e < 2 ? e + 1 : e);               // edgeIdx 0..4
                    res[i] = (ok && e) ? min(max(v + off(e - 1), 0), maxv) : v;
                }
            }
    #pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i0 = 2 * q, i1 = 2 * q + 1;
                const int r0 = ((nfm >> i0) & 1u) ? smp(w, i0) : res[i0];
                const int r1 = ((nfm >> i1) & 1u) ? smp(w, i1) : res[i1];
                w[q] = (uint32_t)r0 | (uint32_t)r1 << 16;
            }
        }
        *reinterpret_cast<uint4*>(out + (size_t)Y * st + X0) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

}  // namespace p265r
