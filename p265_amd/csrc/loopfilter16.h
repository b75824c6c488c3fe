// In-loop filters of the 16-bit sample path (BitDepth 9..12; Geo::pel16): deblocking (8.7.2)
// + SAO (8.7.3) fused in one pass, as loopfilter.h does for 8-bit samples, with the bit-depth rules:
//   beta = beta' * (1 << (BitDepthY - 8)), tC = tC' * (1 << (BitDepth - 8))   (8.7.2.5.3, 8.7.2.5.5)
//   QpY = Qp'Y - QpBdOffsetY on both sides of an edge (the deblocking map carries Qp'Y, loopfilter.h)
//   bandShift = BitDepth - 5, SaoOffsetVal as recorded (<< (BitDepth - Min(BitDepth, 10)) by the
//   front-end), clipping to (1 << BitDepth) - 1                              (8.7.3.2, 7.4.9.3.2)
// The reference has neither filter (decoder/sao.py:15-136 parses the syntax, sao.py:174-178 derives
// cMax from the bit depth); oracle/recon_oracle.py restates both for every bit depth.
//
// One workgroup per (CTB, picture), XCD-aware order; the CTB plus a 4-sample halo is staged in LDS as
// uint16 samples (luma (S+8)^2, chroma (S/2+8)^2 each), deblocked there (the window is closed under
// deblocking, loopfilter.h), and SAO of the CTB runs from it, one sample per thread and step.  Plain
// per-sample arithmetic: this path is for correctness and coverage of Main 10, not the headline.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"
#include "loopfilter.h"
#include "sao.h"

namespace p265r {

__device__ __forceinline__ void dbk_luma_seg16(int (&P)[4][4], int (&Q)[4][4], int qpp, int qpq, int boff, int toff,
                                               bool nop, bool noq, int bd) {
    const int qpl = (qpq + qpp + 1) >> 1;
    const int beta = dbk_beta(min(max(qpl + 2 * boff, 0), 51)) << (bd - 8);
    const int tc = (int)c_tc_table[min(max(qpl + 2 + 2 * toff, 0), 53)] << (bd - 8);     // bS = 2
    const int maxv = (1 << bd) - 1;
    const int dp0 = abs(P[2][0] - 2 * P[1][0] + P[0][0]), dp3 = abs(P[2][3] - 2 * P[1][3] + P[0][3]);
    const int dq0 = abs(Q[2][0] - 2 * Q[1][0] + Q[0][0]), dq3 = abs(Q[2][3] - 2 * Q[1][3] + Q[0][3]);
    if (dp0 + dq0 + dp3 + dq3 >= beta) return;
    auto dsam = [&](int k, int dpq) {
        return dpq < (beta >> 2) && abs(P[3][k] - P[0][k]) + abs(Q[0][k] - Q[3][k]) < (beta >> 3) &&
               abs(P[0][k] - Q[0][k]) < ((5 * tc + 1) >> 1);
    };
    const bool strong = dsam(0, 2 * (dp0 + dq0)) && dsam(3, 2 * (dp3 + dq3));
    const int side = (beta + (beta >> 1)) >> 3;
    const bool dep = dp0 + dp3 < side, deq = dq0 + dq3 < side;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int p0 = P[0][k], p1 = P[1][k], p2 = P[2][k], p3 = P[3][k];
        const int q0 = Q[0][k], q1 = Q[1][k], q2 = Q[2][k], q3 = Q[3][k];
        if (strong) {
            const int t2 = 2 * tc;
            if (!nop) {
                P[0][k] = min(max((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, p0 - t2), p0 + t2);
                P[1][k] = min(max((p2 + p1 + p0 + q0 + 2) >> 2, p1 - t2), p1 + t2);
                P[2][k] = min(max((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3, p2 - t2), p2 + t2);
            }
            if (!noq) {
                Q[0][k] = min(max((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, q0 - t2), q0 + t2);
                Q[1][k] = min(max((p0 + q0 + q1 + q2 + 2) >> 2, q1 - t2), q1 + t2);
                Q[2][k] = min(max((p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3, q2 - t2), q2 + t2);
            }
        } else {
            int d = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (abs(d) < tc * 10) {
                d = min(max(d, -tc), tc);
                const int th = tc >> 1;
                if (!nop) {
                    P[0][k] = min(max(p0 + d, 0), maxv);
                    if (dep) P[1][k] = min(max(p1 + min(max((((p2 + p0 + 1) >> 1) - p1 + d) >> 1, -th), th), 0), maxv);
                }
                if (!noq) {
                    Q[0][k] = min(max(q0 - d, 0), maxv);
                    if (deq) Q[1][k] = min(max(q1 + min(max((((q2 + q0 + 1) >> 1) - q1 - d) >> 1, -th), th), 0), maxv);
                }
            }
        }
    }
}

// grid (8 * ceil(CTUs * pictures / 8)), 256 threads; planes of uint16_t samples, Geo::stride samples
template <int CTBL, bool DBK>
__global__ __launch_bounds__(256) void loopfilter16_kernel(const DevPic* __restrict__ pics, Geo g, int sao_on, int n_pics) {
    constexpr int S = 1 << CTBL, SC = S / 2;
    constexpr int RL = S + 8, RC = SC + 8;                   // window rows / columns (halo 4)
    constexpr int NB = S / 8 + 2;                             // 8x8 luma blocks per window row (map)
    constexpr int NLE = S / 8 + 1, NCE = SC / 8 + 1;          // edges per direction
    constexpr int WL = RL / 4, WC = RC / 4;                   // 4-line segments per edge
    constexpr int T = 256;
    __shared__ uint16_t s_l[RL * RL];
    __shared__ uint16_t s_c[2][RC * RC];
    __shared__ uint16_t s_map[NB * NB];
    __shared__ uint8_t s_nf[NB * NB];
    __shared__ LfCtu s_ctu[9];
    __shared__ uint32_t s_allow;

    const int n_ctus = g.wc * g.hc;
    const int unit = xcd_unit(blockIdx.x, n_ctus * n_pics);
    if (unit >= n_ctus * n_pics) return;                     // whole workgroup: before any barrier
    const int pic = unit / n_ctus;
    int rs = unit - pic * n_ctus;
    const DevPic* P = pics + pic;
    const p265r_ctu* ctus = P->ctus;
    const int rx = rs % g.wc, ry = rs / g.wc;
    if (P265R_RAGGED && g.ragged) {
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)P->wh));
        if (rx >= g.wc || ry >= g.hc) return;
        rs = ry * g.wc + rx;
    }
    const int x0 = rx * S, y0 = ry * S, xc0 = x0 >> 1, yc0 = y0 >> 1;
    const int tid = threadIdx.x;
    const p265r_ctu me = ctus[rs];
    const int qp_off = 6 * (g.bd[0] - 8);                    // QpBdOffsetY: the map holds Qp'Y

    if (tid < 64) {
        const bool ok = tid < 9 && sao_allow(ctus, me, rs, rx, ry, tid % 3 - 1, tid / 3 - 1, g);
        const uint32_t bits = (uint32_t)__ballot(ok);
        if (tid == 0) s_allow = bits;
        if (DBK && tid < 9) {
            const int nx = rx + tid % 3 - 1, ny = ry + tid / 3 - 1;
            LfCtu e{0xffffffffu, 0xffff, 0, 0};
            if (nx >= 0 && ny >= 0 && nx < g.wc && ny < g.hc) {
                const p265r_ctu& o = ctus[ny * g.wc + nx];
                e = LfCtu{o.slice_addr, o.tile_id, o.flags, o.deblock_offsets};
            }
            s_ctu[tid] = e;
        }
    }
    const int nf_h = (g.h + 7) >> 3;
    for (int i = tid; i < NB * NB; i += T) {
        const int bx = (x0 >> 3) - 1 + i % NB, by = (y0 >> 3) - 1 + i / NB;
        const bool in = bx >= 0 && by >= 0 && bx < g.nf_w && by < nf_h;
        const size_t o = (size_t)by * g.nf_w + bx;
        if (DBK) s_map[i] = in ? reinterpret_cast<const uint16_t*>(P->dbk_map)[o] : 0;
        s_nf[i] = in && P->nofilter ? P->nofilter[o] : 0;
    }
    {
        const uint16_t* src = reinterpret_cast<const uint16_t*>(P->rec[0]);
        for (int i = tid; i < RL * RL; i += T) {
            const int r = i / RL, q = i - r * RL;
            const int gy = y0 - 4 + r, gx = x0 - 4 + q;
            s_l[i] = (gy >= 0 && gy < g.h && gx >= 0 && gx < g.w) ? src[(size_t)gy * g.stride[0] + gx] : 0;
        }
        for (int i = tid; i < 2 * RC * RC; i += T) {
            const int c = i >= RC * RC, k = i - c * RC * RC;
            const int r = k / RC, q = k - r * RC;
            const int gy = yc0 - 4 + r, gx = xc0 - 4 + q;
            const uint16_t* cs = reinterpret_cast<const uint16_t*>(P->rec[1 + c]);
            s_c[c][k] = (gy >= 0 && gy < g.ch && gx >= 0 && gx < g.cw) ? cs[(size_t)gy * g.stride[1] + gx] : 0;
        }
    }
    __syncthreads();

    if constexpr (DBK) {
        auto slot = [&](int x, int y) { return ((y >> CTBL) - ry + 1) * 3 + (x >> CTBL) - rx + 1; };
        auto mblk = [&](int x, int y) { return ((y >> 3) - (y0 >> 3) + 1) * NB + (x >> 3) - (x0 >> 3) + 1; };
        auto edge_offs = [&](int xp, int yp, int xq, int yq) -> int {
            const LfCtu q = s_ctu[slot(xq, yq)];
            if (!(q.flags & P265R_CTU_DEBLOCK)) return -1;
            const LfCtu p = s_ctu[slot(xp, yp)];
            if (!g.lf_tiles && p.tile_id != q.tile_id) return -1;
            if (p.slice_addr != q.slice_addr && !(q.flags & P265R_CTU_LF_ACROSS_SLICES)) return -1;
            return q.offs;
        };
        constexpr int N_DBK = NLE * WL + 2 * NCE * WC;
        for (int dir = 0; dir < 2; ++dir) {                  // 0: vertical edges, 1: horizontal edges
            const int ebit = dir ? DBK16_H : DBK16_V;
            for (int t = tid; t < N_DBK; t += T) {
                if (t < NLE * WL) {
                    const int i = t / WL, j = t % WL;
                    const int ge = (dir ? y0 : x0) + 8 * i, gs = (dir ? x0 : y0) - 4 + 4 * j;
                    const int xq = dir ? gs : ge, yq = dir ? ge : gs;
                    const int xp = dir ? xq : xq - 1, yp = dir ? yq - 1 : yq;
                    if (ge <= 0 || ge >= (dir ? g.h : g.w) || gs < 0 || gs >= (dir ? g.w : g.h)) continue;
                    const int bq = mblk(xq, yq), bp = mblk(xp, yp);
                    const int mq = s_map[bq];
                    if (!(mq & ebit)) continue;
                    const int offs = edge_offs(xp, yp, xq, yq);
                    if (offs < 0) continue;
                    // window sample of P_a / Q_a on line k
                    auto at = [&](int a, int k, bool q) -> uint16_t& {
                        const int e = 8 * i + (q ? 4 + a : 3 - a), l = 4 * j + k;
                        return dir ? s_l[e * RL + l] : s_l[l * RL + e];
                    };
                    int Pm[4][4], Qm[4][4];
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int k = 0; k < 4; ++k) { Pm[a][k] = at(a, k, false); Qm[a][k] = at(a, k, true); }
                    dbk_luma_seg16(Pm, Qm, (s_map[bp] & DBK16_QP) - qp_off, (mq & DBK16_QP) - qp_off, nib4(offs & 15),
                                   nib4(offs >> 4), s_nf[bp] != 0, s_nf[bq] != 0, g.bd[0]);
#pragma unroll
                    for (int a = 0; a < 3; ++a)
#pragma unroll
                        for (int k = 0; k < 4; ++k) { at(a, k, false) = (uint16_t)Pm[a][k]; at(a, k, true) = (uint16_t)Qm[a][k]; }
                } else {
                    const int u = t - NLE * WL;
                    const int c = u / (NCE * WC), v = u % (NCE * WC);
                    const int i = v / WC, j = v % WC;
                    const int ge = (dir ? yc0 : xc0) + 8 * i, gs = (dir ? xc0 : yc0) - 4 + 4 * j;
                    if (ge <= 0 || ge >= (dir ? g.ch : g.cw) || gs < 0 || gs >= (dir ? g.cw : g.ch)) continue;
                    const int xq = (dir ? gs : ge) << 1, yq = (dir ? ge : gs) << 1;
                    const int xp = dir ? xq : xq - 1, yp = dir ? yq - 1 : yq;
                    const int bq = mblk(xq, yq), bp = mblk(xp, yp);
                    const int mq = s_map[bq];
                    if (!(mq & ebit)) continue;
                    const int offs = edge_offs(xp, yp, xq, yq);
                    if (offs < 0) continue;
                    const int qpi = ((((mq & DBK16_QP) - qp_off) + ((s_map[bp] & DBK16_QP) - qp_off) + 1) >> 1) +
                                    (c ? g.cqp[1] : g.cqp[0]);
                    const int tc = (int)c_tc_table[min(max(qpc_table(qpi) + 2 + 2 * nib4(offs >> 4), 0), 53)] << (g.bd[1] - 8);
                    const int maxc = (1 << g.bd[1]) - 1;
                    const bool nop = s_nf[bp] != 0, noq = s_nf[bq] != 0;
                    uint16_t* w = s_c[c];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int l = 4 * j + k, e = 8 * i;
                        uint16_t& p0 = dir ? w[(e + 3) * RC + l] : w[l * RC + e + 3];
                        uint16_t& q0 = dir ? w[(e + 4) * RC + l] : w[l * RC + e + 4];
                        const int p1 = dir ? w[(e + 2) * RC + l] : w[l * RC + e + 2];
                        const int q1 = dir ? w[(e + 5) * RC + l] : w[l * RC + e + 5];
                        const int d = min(max((((int)q0 - (int)p0) * 4 + p1 - q1 + 4) >> 3, -tc), tc);
                        const int np0 = min(max((int)p0 + d, 0), maxc), nq0 = min(max((int)q0 - d, 0), maxc);
                        if (!nop) p0 = (uint16_t)np0;
                        if (!noq) q0 = (uint16_t)nq0;
                    }
                }
            }
            __syncthreads();
        }
    }

    // ---- SAO of the CTB from the (deblocked) window, one sample per thread and step ----
    const uint32_t allow = s_allow;
    constexpr int NL = S * S, NC = SC * SC;
    for (int u = tid; u < NL + 2 * NC; u += T) {
        const int c = u < NL ? 0 : 1 + (u - NL) / NC;
        const int t = u < NL ? u : (u - NL) % NC;
        const int sub = c ? 1 : 0;
        const int cs = S >> sub;
        const int row = t >> (CTBL - sub), col = t & (cs - 1);
        const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
        const int xb = c ? xc0 : x0, yb = c ? yc0 : y0;
        const int X = xb + col, Y = yb + row;
        if (X >= W || Y >= H) continue;
        const uint16_t* win = c ? s_c[c - 1] : s_l;
        const int ws = c ? RC : RL;
        auto smp = [&](int dx, int dy) { return (int)win[(row + 4 + dy) * ws + col + 4 + dx]; };
        const int v = smp(0, 0);
        int r = v;
        const int typ = sao_on ? me.sao_type[c] : 0;
        const int lx = X << sub, ly = Y << sub;
        const bool nf = s_nf[((ly >> 3) - (y0 >> 3) + 1) * NB + (lx >> 3) - (x0 >> 3) + 1] != 0;
        if (typ != 0 && !nf) {
            const int bd = g.bd[c], maxv = (1 << bd) - 1;
            const int cls = me.sao_class[c];
            if (typ == 1) {
                const int k = ((v >> (bd - 5)) - cls) & 31;              // band slot relative to the position
                if (k < 4) r = min(max(v + (int)me.sao_offset[c][k], 0), maxv);
            } else {
                const int ax = cls == 0 ? -1 : (cls == 1 ? 0 : (cls == 2 ? -1 : 1));
                const int ay = cls == 0 ? 0 : -1;
                const int bx = -ax, by = -ay;
                bool ok = X + ax >= 0 && X + ax < W && Y + ay >= 0 && Y + ay < H &&
                          X + bx >= 0 && X + bx < W && Y + by >= 0 && Y + by < H;
                auto reg = [&](int dx, int dy) {
                    const int cx = col + dx < 0 ? 0 : (col + dx >= cs ? 2 : 1);
                    const int cy = row + dy < 0 ? 0 : (row + dy >= cs ? 2 : 1);
                    return ((allow >> (cy * 3 + cx)) & 1u) != 0;
                };
                ok = ok && reg(ax, ay) && reg(bx, by);
                if (ok) {
                    const int a = smp(ax, ay), b = smp(bx, by);
                    int e = 2 + (v > a) - (v < a) + (v > b) - (v < b);
                    e = e == 2 ? 0 : (e < 2 ? e + 1 : e);                 // edgeIdx 0..4
                    if (e) r = min(max(v + (int)me.sao_offset[c][e - 1], 0), maxv);
                }
            }
        }
        reinterpret_cast<uint16_t*>(P->out[c])[(size_t)Y * g.stride[c] + X] = (uint16_t)r;
    }
}

}  // namespace p265r
