// In-loop filter phase: deblocking (H.265 8.7.2) + SAO (8.7.3) fused in one pass.
//
// The reference has neither filter: it parses their syntax (decoder/pps.py:122-131,
// slice.py:170-179, sao.py:15-136) and stops there.  Both kernels here are new.
//
// One workgroup per (CTB, picture).  The workgroup stages the CTB plus a 4-sample halo
// on every side (luma (S+8)^2, each chroma (S/2+8)^2) in LDS.  That window is closed
// under deblocking: every vertical edge x0, x0+8, .., x0+S reads at most 4 samples on
// either side (x0-4 .. x0+S+3) and no edge outside that set modifies a sample inside
// the window (filters reach 3 samples luma / 1 chroma, edges sit 8 apart, the window
// edges are 4 away from the nearest edge); the same holds for rows.  So filtering all
// vertical then all horizontal edges of the window in LDS yields the exact deblocked
// picture on the whole window, and SAO of the CTB (which reads one sample around it)
// then runs from LDS.  HBM traffic per sample: (S+8)^2/S^2 reads (1.27 at CTB 64) + 1
// write; no intermediate deblocked plane exists.
//
// Edge information comes from dbk_map_kernel: one byte per 8x8 luma block,
//   bits 0..5 QpY of its CU, bit 6 its left side is a transform-block edge,
//   bit 7 its top side is a transform-block edge.
// In 4:2:0 intra pictures every TB boundary on the 8x8 grid is an edge with bS = 2
// (8.7.2.4: intra on either side); prediction-block edges of NxN CUs sit at 4-sample
// offsets and never reach the grid.  Every 8x8 block is written by exactly one luma TB:
// the TB covering it if log2 >= 3, else the 4x4 TB at its top-left (blkIdx 0) whose
// block's left/top sides are TB edges by construction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"
#include "sao.h"

namespace p265r {

enum : uint8_t { DBK_V = 0x40, DBK_H = 0x80, DBK_QP = 0x3f };

// Table 8-12 tC' (Q = 0..53); beta' has the closed form used in dbk_beta()
__constant__ uint8_t c_tc_table[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

__device__ __forceinline__ int dbk_beta(int q) {           // beta' for Q = 0..51
    return q < 16 ? 0 : (q <= 28 ? q - 10 : 2 * q - 38);
}
__device__ __forceinline__ int qpc_table(int qpi) {          // Table 8-10, ChromaArrayType 1
    if (qpi < 30) return qpi;
    if (qpi >= 43) return qpi - 6;
    // QpC - 29 for qPi = 30..42 (0,1,2,3,4,4,5,5,6,6,7,7,8), 4 bits each
    constexpr uint64_t t = 0x8776655443210ull;
    return 29 + (int)((t >> (4 * (qpi - 30))) & 15u);
}
__device__ __forceinline__ int nib4(int v) { return (v ^ 8) - 8; }   // 4-bit two's complement

// ---------------------------------------------------------------------------------------
// Edge map: grid (CTUs, pictures), one wave per CTU walks its TBs.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void dbk_map_kernel(const DevPic* __restrict__ pics, Geo g) {
    const DevPic* P = pics + blockIdx.y;
    const p265r_ctu me = P->ctus[blockIdx.x];
    const p265r_tb* tbs = P->tbs + me.tb_begin;
    uint8_t* map = P->dbk_map;
    const int qp_off = 6 * (g.bd[0] - 8);
    for (int t = threadIdx.x; t < me.tb_count; t += 64) {
        const p265r_tb tb = tbs[t];
        if (tb.c_idx != 0) continue;
        const int qpy = (int)tb.qp - qp_off;
        const int bx0 = tb.x >> 3, by0 = tb.y >> 3;
        if (tb.log2_size == 2) {
            if ((tb.x & 7) == 0 && (tb.y & 7) == 0) map[by0 * g.nf_w + bx0] = (uint8_t)(qpy | DBK_V | DBK_H);
            continue;
        }
        const int n8 = 1 << (tb.log2_size - 3);
        for (int j = 0; j < n8; ++j)
            for (int i = 0; i < n8; ++i)
                map[(by0 + j) * g.nf_w + bx0 + i] = (uint8_t)(qpy | (i == 0 ? DBK_V : 0) | (j == 0 ? DBK_H : 0));
    }
}

// ---------------------------------------------------------------------------------------
// Filters on registers.  P[i][k] / Q[i][k]: sample i away from the edge on line k.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void dbk_luma_seg(int (&P)[4][4], int (&Q)[4][4], int qpp, int qpq, int boff, int toff,
                                             bool nop, bool noq) {
    const int qpl = (qpq + qpp + 1) >> 1;
    const int beta = dbk_beta(min(max(qpl + 2 * boff, 0), 51));
    const int tc = c_tc_table[min(max(qpl + 2 + 2 * toff, 0), 53)];          // bS = 2
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
                    P[0][k] = min(max(p0 + d, 0), 255);
                    if (dep) P[1][k] = min(max(p1 + min(max((((p2 + p0 + 1) >> 1) - p1 + d) >> 1, -th), th), 0), 255);
                }
                if (!noq) {
                    Q[0][k] = min(max(q0 - d, 0), 255);
                    if (deq) Q[1][k] = min(max(q1 + min(max((((q2 + q0 + 1) >> 1) - q1 - d) >> 1, -th), th), 0), 255);
                }
            }
        }
    }
}

__device__ __forceinline__ void dbk_chroma_line(int& p0, int p1, int& q0, int q1, int tc, bool nop, bool noq) {
    const int d = min(max((((q0 - p0) * 4) + p1 - q1 + 4) >> 3, -tc), tc);
    const int np0 = min(max(p0 + d, 0), 255), nq0 = min(max(q0 - d, 0), 255);
    if (!nop) p0 = np0;
    if (!noq) q0 = nq0;
}

__device__ __forceinline__ int byte_of(uint32_t w, int b) { return (int)((w >> (8 * b)) & 0xffu); }
__device__ __forceinline__ uint32_t set_byte(uint32_t w, int b, int v) {
    return (w & ~(0xffu << (8 * b))) | ((uint32_t)v << (8 * b));
}

struct LfCtu {                  // the fields of a neighbouring CTU record the filters read
    uint32_t slice_addr;
    uint16_t tile_id;
    uint8_t  flags;
    uint8_t  offs;
};

template <int CTBL> struct LfShape {
    static constexpr int S = 1 << CTBL, SC = S / 2;
    static constexpr int RL = S + 8, RC = SC + 8;          // window sizes (halo 4)
    static constexpr int WL = RL / 4, WC = RC / 4;         // dwords per window row
    static constexpr int NB = S / 8 + 2;                   // 8x8 luma blocks per window row (map)
    static constexpr int UL = 16, UC = SC < 16 ? SC : 16;  // SAO unit widths (samples)
    static constexpr int N_SAO = S * (S / UL) + 2 * SC * (SC / UC);
    static constexpr int NLE = S / 8 + 1, NCE = SC / 8 + 1;   // edges per direction
    static constexpr int N_DBK = NLE * WL + 2 * NCE * WC;     // 4-line segments per direction
    static constexpr int T0 = N_SAO > N_DBK ? N_SAO : N_DBK;
    static constexpr int THREADS = (T0 + 63) / 64 * 64;
};

// grid (CTUs, pictures); DBK: deblock the window first (else the window is the SAO input as is)
template <int CTBL, bool DBK>
__global__ __launch_bounds__(LfShape<CTBL>::THREADS) void loopfilter_kernel(const DevPic* __restrict__ pics, Geo g,
                                                                          int sao_on) {
    using SH = LfShape<CTBL>;
    constexpr int S = SH::S, SC = SH::SC, WL = SH::WL, WC = SH::WC, NB = SH::NB;
    __shared__ uint32_t s_l[SH::RL * WL];
    __shared__ uint32_t s_c[2][SH::RC * WC];
    __shared__ uint8_t s_map[NB * NB];
    __shared__ uint8_t s_nf[NB * NB];
    __shared__ LfCtu s_ctu[9];
    __shared__ uint32_t s_allow;

    const int rs = blockIdx.x;
    const DevPic* P = pics + blockIdx.y;
    const p265r_ctu* ctus = P->ctus;
    const int rx = rs % g.wc, ry = rs / g.wc;
    const int x0 = rx * S, y0 = ry * S, xc0 = x0 >> 1, yc0 = y0 >> 1;
    const int tid = threadIdx.x;
    constexpr int T = SH::THREADS;
    const p265r_ctu me = ctus[rs];

    // ---- CTU neighbourhood, SAO permissions (8.7.3.2), map windows, sample windows ---------------
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
        if (DBK) s_map[i] = in ? P->dbk_map[o] : 0;
        s_nf[i] = in && P->nofilter ? P->nofilter[o] : 0;
    }
    {
        const uint8_t* src = P->rec[0];
        const int st = g.stride[0];
        for (int i = tid; i < SH::RL * WL; i += T) {
            const int gy = y0 - 4 + i / WL, gx = x0 - 4 + 4 * (i % WL);
            s_l[i] = (gy >= 0 && gy < g.h && gx >= 0 && gx < g.w) ? *reinterpret_cast<const uint32_t*>(src + (size_t)gy * st + gx) : 0u;
        }
        for (int i = tid; i < 2 * SH::RC * WC; i += T) {
            const int c = i >= SH::RC * WC, k = i - c * SH::RC * WC;
            const int gy = yc0 - 4 + k / WC, gx = xc0 - 4 + 4 * (k % WC);
            s_c[c][k] = (gy >= 0 && gy < g.ch && gx >= 0 && gx < g.cw)
                            ? *reinterpret_cast<const uint32_t*>(P->rec[1 + c] + (size_t)gy * g.stride[1] + gx) : 0u;
        }
    }
    __syncthreads();

    if constexpr (DBK) {
        // slot of the CTU containing luma (x, y) in the 3x3 neighbourhood
        auto slot = [&](int x, int y) { return ((y >> CTBL) - ry + 1) * 3 + (x >> CTBL) - rx + 1; };
        auto mblk = [&](int x, int y) { return ((y >> 3) - (y0 >> 3) + 1) * NB + (x >> 3) - (x0 >> 3) + 1; };
        // filterEdgeFlag for the edge between luma p0 (xp, yp) and q0 (xq, yq); returns Q's offsets or -1
        auto edge_offs = [&](int xp, int yp, int xq, int yq) -> int {
            const LfCtu q = s_ctu[slot(xq, yq)];
            if (!(q.flags & P265R_CTU_DEBLOCK)) return -1;
            const LfCtu p = s_ctu[slot(xp, yp)];
            if (!g.lf_tiles && p.tile_id != q.tile_id) return -1;
            if (p.slice_addr != q.slice_addr && !(q.flags & P265R_CTU_LF_ACROSS_SLICES)) return -1;
            return q.offs;
        };
        for (int dir = 0; dir < 2; ++dir) {              // 0: vertical edges, 1: horizontal edges
            const uint8_t ebit = dir ? DBK_H : DBK_V;
            for (int t = tid; t < SH::N_DBK; t += T) {
                if (t < SH::NLE * WL) {
                    // ---- luma: edge i, 4-line segment j --------------------------------------------
                    const int i = t / WL, j = t % WL;
                    const int ge = (dir ? y0 : x0) + 8 * i;            // edge coordinate
                    const int gs = (dir ? x0 : y0) - 4 + 4 * j;        // segment start
                    const int xq = dir ? gs : ge, yq = dir ? ge : gs;
                    const int xp = dir ? xq : xq - 1, yp = dir ? yq - 1 : yq;
                    if (ge <= 0 || ge >= (dir ? g.h : g.w) || gs < 0 || gs >= (dir ? g.w : g.h)) continue;
                    const int bq = mblk(xq, yq), bp = mblk(xp, yp);
                    const int mq = s_map[bq];
                    if (!(mq & ebit)) continue;
                    const int offs = edge_offs(xp, yp, xq, yq);
                    if (offs < 0) continue;
                    int Pm[4][4], Qm[4][4];
                    if (!dir) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t lo = s_l[(4 * j + k) * WL + 2 * i], hi = s_l[(4 * j + k) * WL + 2 * i + 1];
#pragma unroll
                            for (int a = 0; a < 4; ++a) { Pm[a][k] = byte_of(lo, 3 - a); Qm[a][k] = byte_of(hi, a); }
                        }
                    } else {
#pragma unroll
                        for (int a = 0; a < 4; ++a) {
                            const uint32_t wp = s_l[(8 * i + 3 - a) * WL + j], wq = s_l[(8 * i + 4 + a) * WL + j];
#pragma unroll
                            for (int k = 0; k < 4; ++k) { Pm[a][k] = byte_of(wp, k); Qm[a][k] = byte_of(wq, k); }
                        }
                    }
                    dbk_luma_seg(Pm, Qm, s_map[bp] & DBK_QP, mq & DBK_QP, nib4(offs & 15), nib4(offs >> 4),
                                 s_nf[bp] != 0, s_nf[bq] != 0);
                    if (!dir) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            uint32_t lo = 0, hi = 0;
#pragma unroll
                            for (int a = 0; a < 4; ++a) { lo |= (uint32_t)Pm[3 - a][k] << (8 * a); hi |= (uint32_t)Qm[a][k] << (8 * a); }
                            s_l[(4 * j + k) * WL + 2 * i] = lo;
                            s_l[(4 * j + k) * WL + 2 * i + 1] = hi;
                        }
                    } else {
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            uint32_t wp = 0, wq = 0;
#pragma unroll
                            for (int k = 0; k < 4; ++k) { wp |= (uint32_t)Pm[a][k] << (8 * k); wq |= (uint32_t)Qm[a][k] << (8 * k); }
                            s_l[(8 * i + 3 - a) * WL + j] = wp;
                            s_l[(8 * i + 4 + a) * WL + j] = wq;
                        }
                    }
                } else {
                    // ---- chroma (4:2:0): edge i every 8 chroma samples, 4-line segment j -------------------
                    const int u = t - SH::NLE * WL;
                    const int c = u / (SH::NCE * WC), v = u % (SH::NCE * WC);
                    const int i = v / WC, j = v % WC;
                    const int ge = (dir ? yc0 : xc0) + 8 * i;
                    const int gs = (dir ? xc0 : yc0) - 4 + 4 * j;
                    if (ge <= 0 || ge >= (dir ? g.ch : g.cw) || gs < 0 || gs >= (dir ? g.cw : g.ch)) continue;
                    const int xq = (dir ? gs : ge) << 1, yq = (dir ? ge : gs) << 1;     // luma position of q0
                    const int xp = dir ? xq : xq - 1, yp = dir ? yq - 1 : yq;
                    const int bq = mblk(xq, yq), bp = mblk(xp, yp);
                    const int mq = s_map[bq];
                    if (!(mq & ebit)) continue;
                    const int offs = edge_offs(xp, yp, xq, yq);
                    if (offs < 0) continue;
                    const int qpi = (((mq & DBK_QP) + (s_map[bp] & DBK_QP) + 1) >> 1) + g.cqp[c];
                    const int tc = c_tc_table[min(max(qpc_table(qpi) + 2 + 2 * nib4(offs >> 4), 0), 53)];
                    const bool nop = s_nf[bp] != 0, noq = s_nf[bq] != 0;
                    uint32_t* w = s_c[c];
                    if (!dir) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            uint32_t lo = w[(4 * j + k) * WC + 2 * i], hi = w[(4 * j + k) * WC + 2 * i + 1];
                            int p0 = byte_of(lo, 3), q0 = byte_of(hi, 0);
                            dbk_chroma_line(p0, byte_of(lo, 2), q0, byte_of(hi, 1), tc, nop, noq);
                            w[(4 * j + k) * WC + 2 * i] = set_byte(lo, 3, p0);
                            w[(4 * j + k) * WC + 2 * i + 1] = set_byte(hi, 0, q0);
                        }
                    } else {
                        const uint32_t w1 = w[(8 * i + 2) * WC + j], w4 = w[(8 * i + 5) * WC + j];
                        uint32_t w2 = w[(8 * i + 3) * WC + j], w3 = w[(8 * i + 4) * WC + j];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            int p0 = byte_of(w2, k), q0 = byte_of(w3, k);
                            dbk_chroma_line(p0, byte_of(w1, k), q0, byte_of(w4, k), tc, nop, noq);
                            w2 = set_byte(w2, k, p0);
                            w3 = set_byte(w3, k, q0);
                        }
                        w[(8 * i + 3) * WC + j] = w2;
                        w[(8 * i + 4) * WC + j] = w3;
                    }
                }
            }
            __syncthreads();
        }
    }

    // ---- SAO of the CTB from the (deblocked) window; one thread per UL / UC-sample row unit ----
    const uint32_t allow = s_allow;
    if (tid >= SH::N_SAO) return;
    int c, t;
    constexpr int NL = S * (S / SH::UL), NC = SC * (SC / SH::UC);
    if (tid < NL) { c = 0; t = tid; }
    else { c = 1 + (tid - NL) / NC; t = (tid - NL) % NC; }
    const int sub = c ? 1 : 0;
    const int U = c ? SH::UC : SH::UL;                 // samples per unit (16 or 8)
    const int NW = U / 4;
    const int cs = S >> sub;
    const int upr = cs / U;
    const int row = t / upr, col = (t % upr) * U;
    const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
    const int xb = c ? xc0 : x0, yb = c ? yc0 : y0;
    const int X = xb + col, Y = yb + row;
    if (X >= W || Y >= H) return;
    const uint32_t* win = c ? s_c[c - 1] : s_l;
    const int wst = c ? WC : WL;
    // window dword (r, d) holds samples (xb - 4 + 4d .. +3, yb - 4 + r)
    const int wr = row + 4, wd = col / 4 + 1;
    uint32_t cur[4], res[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = q < NW ? win[wr * wst + wd + q] : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) res[q] = cur[q];
    const int typ = sao_on ? me.sao_type[c] : 0;
    if (typ != 0) {
        uint32_t keep = 0;
        for (int i = 0; i < U; i += 4) {                 // 4 samples never straddle an 8x8 luma block
            const int lx = (X + i) << sub, ly = Y << sub;
            if (s_nf[((ly >> 3) - (y0 >> 3) + 1) * NB + (lx >> 3) - (x0 >> 3) + 1]) keep |= 0xfu << i;
        }
        const int o1 = me.sao_offset[c][0], o2 = me.sao_offset[c][1];
        const int o3 = me.sao_offset[c][2], o4 = me.sao_offset[c][3];
        auto offv = [&](int i) { return i == 1 ? o1 : i == 2 ? o2 : i == 3 ? o3 : i == 4 ? o4 : 0; };
        const int cls = me.sao_class[c];
        if (typ == 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i >= U) break;
                const int v = byte_of(cur[i >> 2], i & 3);
                const int bi = ((v >> 3) - cls) & 31;
                int r = v;
                if (bi < 4) r = min(max(v + offv(bi + 1), 0), 255);
                if ((keep >> i) & 1u) r = v;
                res[i >> 2] = set_byte(res[i >> 2], i & 3, r);
            }
        } else {
            const int ax = cls == 1 ? 0 : (cls == 3 ? 1 : -1);
            const int ay = cls == 0 ? 0 : -1;
            const bool has_l = X > 0, has_u = Y > 0, has_d = Y + 1 < H;
            const int ru = Y == yb ? 0 : 1, rd = Y == yb + cs - 1 ? 2 : 1;
            const int cl = X == xb ? 0 : 1, cr = X + U == xb + cs ? 2 : 1;
            auto region_ok = [&](int rr, int cc) { return (allow >> (rr * 3 + cc)) & 1u; };
            // sample at unit column j (-1 .. U) of window row r
            auto at = [&](int r, int j) {
                const int d = wd + ((j + 4) >> 2) - 1;
                return byte_of(win[r * wst + d], (j + 4) & 3);
            };
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i >= U) break;
                const int v = byte_of(cur[i >> 2], i & 3);
                const int ja = i + ax, jb = i - ax;
                const int ca = ja < 0 ? cl : (ja >= U ? cr : 1);
                const int cb = jb < 0 ? cl : (jb >= U ? cr : 1);
                const bool xa_in = ja < 0 ? has_l : X + ja < W;
                const bool xb_in = jb < 0 ? has_l : X + jb < W;
                bool ok, okb;
                int a, b;
                if (ay == 0) {
                    ok = xa_in && region_ok(1, ca);
                    okb = xb_in && region_ok(1, cb);
                    a = at(wr, ja); b = at(wr, jb);
                } else {
                    ok = has_u && xa_in && region_ok(ru, ca);
                    okb = has_d && xb_in && region_ok(rd, cb);
                    a = at(wr - 1, ja); b = at(wr + 1, jb);
                }
                int r = v;
                if (ok && okb) {
                    int ei = 2 + sgn(v - a) + sgn(v - b);
                    ei = ei == 2 ? 0 : (ei < 2 ? ei + 1 : ei);
                    r = min(max(v + offv(ei), 0), 255);
                }
                if ((keep >> i) & 1u) r = v;
                res[i >> 2] = set_byte(res[i >> 2], i & 3, r);
            }
        }
    }
    uint8_t* dst = P->out[c] + (size_t)Y * g.stride[c] + X;
    if (NW == 4) *reinterpret_cast<uint4*>(dst) = make_uint4(res[0], res[1], res[2], res[3]);
    else *reinterpret_cast<uint2*>(dst) = make_uint2(res[0], res[1]);
}

}  // namespace p265r
