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
//   bits 0..5 Qp'Y of its CU (= QpY at 8 bits), bit 6 its left side is a transform-block edge,
//   bit 7 its top side is a transform-block edge.  Above 8 bits one uint16 per block: bits 0..7
//   Qp'Y (loopfilter16.h subtracts QpBdOffsetY), bit 8 left edge, bit 9 top edge.
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
// BitDepth > 8 (loopfilter16.h): Qp'Y reaches 51 + 6 * (BitDepth - 8) = 75 at 12 bits, past 6 bits, so the
// map holds uint16 entries there: Qp'Y in the low byte, the edge bits above it.
enum : uint16_t { DBK16_V = 0x100, DBK16_H = 0x200, DBK16_QP = 0xff };

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
template <typename M>        // uint8_t: BitDepth 8 (DBK_*); uint16_t: BitDepth 9..12 (DBK16_*)
__global__ __launch_bounds__(64) void dbk_map_kernel(const DevPic* __restrict__ pics, Geo g) {
    constexpr int EV = sizeof(M) == 1 ? DBK_V : DBK16_V, EH = sizeof(M) == 1 ? DBK_H : DBK16_H;
    const DevPic* P = pics + blockIdx.y;
    if (P265R_RAGGED && g.ragged) {                                              // grid: the context's CTU count
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)P->wh));
        if ((int)blockIdx.x >= g.wc * g.hc) return;
    }
    const p265r_ctu me = P->ctus[blockIdx.x];
    const p265r_tb* tbs = P->tbs + me.tb_begin;
    M* map = reinterpret_cast<M*>(P->dbk_map);
    for (int t = threadIdx.x; t < me.tb_count; t += 64) {
        const p265r_tb tb = tbs[t];
        if (tb.c_idx != 0) continue;
        const int qpy = (int)tb.qp;                  // Qp'Y (0..63 up to BitDepth 10, 0..75 at 12)
        const int bx0 = tb.x >> 3, by0 = tb.y >> 3;
        if (tb.log2_size == 2) {
            if ((tb.x & 7) == 0 && (tb.y & 7) == 0) map[by0 * g.nf_w + bx0] = (M)(qpy | EV | EH);
            continue;
        }
        const int n8 = 1 << (tb.log2_size - 3);
        for (int j = 0; j < n8; ++j)
            for (int i = 0; i < n8; ++i)
                map[(by0 + j) * g.nf_w + bx0 + i] = (M)(qpy | (i == 0 ? EV : 0) | (j == 0 ? EH : 0));
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

// packed unsigned 16-bit ops (two samples per dword); inline asm keeps them packed (the
// compiler otherwise splits clamped / min forms into per-element compares)
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
    uint32_t r; asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b) {
    uint32_t r; asm("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ __forceinline__ uint32_t pk_subsat_u16(uint32_t a, uint32_t b) {       // max(a - b, 0)
    uint32_t r; asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    uint32_t r; asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
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

#ifndef P265R_LF_DBK_THREADS
#define P265R_LF_DBK_THREADS 192
#endif

template <int CTBL> struct LfShape {
    static constexpr int S = 1 << CTBL, SC = S / 2;
    static constexpr int RL = S + 8, RC = SC + 8;          // window rows (halo 4) and used columns
    static constexpr int WL = RL / 4, WC = RC / 4;         // used dwords per window row (4-sample segments)
    // physical window rows start GL / GC samples left of the CTB (load granule: 16 B, 8 B for
    // 8-wide chroma CTBs) so every global load is one aligned 16-B (8-B) access
    static constexpr int GL = 16, GC = SC >= 16 ? 16 : 8;
    static constexpr int PL = (GL + S + 4 + GL - 1) / GL * GL / 4;     // dwords per physical row
    static constexpr int PC = (GC + SC + 4 + GC - 1) / GC * GC / 4;
    static constexpr int DXL = (GL - 4) / 4, DXC = (GC - 4) / 4;      // dword of sample x0 - 4
    static constexpr int NB = S / 8 + 2;                   // 8x8 luma blocks per window row (map)
    static constexpr int UL = 16, UC = SC < 16 ? SC : 16;  // SAO unit widths (samples)
    static constexpr int N_SAO = S * (S / UL) + 2 * SC * (SC / UC);
    static constexpr int NLE = S / 8 + 1, NCE = SC / 8 + 1;   // edges per direction
    static constexpr int N_DBK = NLE * WL + 2 * NCE * WC;     // 4-line segments per direction
    static constexpr int T0 = N_SAO > N_DBK ? N_SAO : N_DBK;
    static constexpr int T1 = (T0 + 63) / 64 * 64;
    // with deblocking, at most three waves per workgroup: smaller workgroups let more CTB windows
    // be in flight per CU (the kernel is bound by load latency, not by issue).  Measured, 1080p
    // CTB 64, 512 pictures: 64 / 128 / 192 / 256 threads -> 3.62 / 2.83 / 2.64 / 3.42 ms.  SAO
    // alone prefers one unit per thread (256: 1.65 ms, 128: 1.73 ms).  Every phase loops over
    // its tasks, so any multiple of 64 is correct.
    static constexpr int threads(bool dbk) { return dbk && T1 > P265R_LF_DBK_THREADS ? P265R_LF_DBK_THREADS : T1; }
};

// grid (CTUs, pictures); DBK: deblock the window first (else the window is the SAO input as is)
// XCD-aware block order: hardware block b runs on XCD b % 8 (observed round-robin,
// MI355X_MICROARCH.md); logical unit (picture, CTB) = (b % 8) * per + b / 8, so each XCD
// walks one contiguous raster range and the halo rows / columns its windows share with
// the neighbouring CTBs are read from its own L2.
__device__ __forceinline__ int xcd_unit(int b, int n_units) {
    const int per = (n_units + 7) >> 3;
    return (b & 7) * per + (b >> 3);
}

// grid (8 * ceil(CTUs * pictures / 8)); DBK: deblock the window first (else the window is
// the SAO input as is)
template <int CTBL, bool DBK>
__global__ __launch_bounds__(LfShape<CTBL>::threads(DBK)) void loopfilter_kernel(const DevPic* __restrict__ pics, Geo g,
                                                                          int sao_on, int n_pics) {
    using SH = LfShape<CTBL>;
    constexpr int S = SH::S, SC = SH::SC, WL = SH::WL, WC = SH::WC, NB = SH::NB;
    constexpr int PL = SH::PL, PC = SH::PC;
    __shared__ __attribute__((aligned(16))) uint32_t s_lphys[SH::RL * PL];
    __shared__ __attribute__((aligned(16))) uint32_t s_cphys[2][SH::RC * PC];
    // logical windows: row r, dword d = samples (x0 - 4 + 4d .. +3, y0 - 4 + r)
    uint32_t* const s_l = s_lphys + SH::DXL;
    auto s_cw = [&](int c) -> uint32_t* { return (c ? s_cphys[1] : s_cphys[0]) + SH::DXC; };
    __shared__ uint8_t s_map[NB * NB];
    __shared__ uint8_t s_nf[NB * NB];
    __shared__ LfCtu s_ctu[9];
    __shared__ uint32_t s_allow;

    const int n_ctus = g.wc * g.hc;
    const int unit = xcd_unit(blockIdx.x, n_ctus * n_pics);
    if (unit >= n_ctus * n_pics) return;                         // whole workgroup: before any barrier
    const int pic = unit / n_ctus;
    int rs = unit - pic * n_ctus;
    const DevPic* P = pics + pic;
    const p265r_ctu* ctus = P->ctus;
    const int rx = rs % g.wc, ry = rs / g.wc;
    if (P265R_RAGGED && g.ragged) {                                              // this picture's size and CTU raster
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)P->wh));
        if (rx >= g.wc || ry >= g.hc) return;                    // whole workgroup: before any barrier
        rs = ry * g.wc + rx;
    }
    const int x0 = rx * S, y0 = ry * S, xc0 = x0 >> 1, yc0 = y0 >> 1;
    const int tid = threadIdx.x;
    constexpr int T = SH::threads(DBK);
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
        // sample windows: aligned 16-B (8-B) loads; bytes right of the picture edge come from
        // the row padding (stride >= 64-aligned width) and are never used
        constexpr int QL = PL / 4;                                 // uint4 per luma row
        const uint8_t* src = P->rec[0];
        const int st = g.stride[0];
        for (int i = tid; i < SH::RL * QL; i += T) {
            const int r = i / QL, q = i - r * QL;
            const int gy = y0 - 4 + r, gx = x0 - SH::GL + 16 * q;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (gy >= 0 && gy < g.h && gx >= 0 && gx < g.w) v = *reinterpret_cast<const uint4*>(src + (size_t)gy * st + gx);
            *reinterpret_cast<uint4*>(&s_lphys[r * PL + 4 * q]) = v;
        }
        constexpr int GCW = SH::GC / 4;                            // dwords per chroma granule
        constexpr int QC = PC / GCW;
        for (int i = tid; i < 2 * SH::RC * QC; i += T) {
            const int c = i >= SH::RC * QC, k = i - c * SH::RC * QC;
            const int r = k / QC, q = k - r * QC;
            const int gy = yc0 - 4 + r, gx = xc0 - SH::GC + SH::GC * q;
            const bool in = gy >= 0 && gy < g.ch && gx >= 0 && gx < g.cw;
            const uint8_t* p = P->rec[1 + c] + (size_t)gy * g.stride[1] + gx;
            if constexpr (GCW == 4) {
                uint4 v = make_uint4(0, 0, 0, 0);
                if (in) v = *reinterpret_cast<const uint4*>(p);
                *reinterpret_cast<uint4*>(&s_cphys[c][r * PC + 4 * q]) = v;
            } else {
                uint2 v = make_uint2(0, 0);
                if (in) v = *reinterpret_cast<const uint2*>(p);
                *reinterpret_cast<uint2*>(&s_cphys[c][r * PC + 2 * q]) = v;
            }
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
                            const uint32_t lo = s_l[(4 * j + k) * PL + 2 * i], hi = s_l[(4 * j + k) * PL + 2 * i + 1];
#pragma unroll
                            for (int a = 0; a < 4; ++a) { Pm[a][k] = byte_of(lo, 3 - a); Qm[a][k] = byte_of(hi, a); }
                        }
                    } else {
#pragma unroll
                        for (int a = 0; a < 4; ++a) {
                            const uint32_t wp = s_l[(8 * i + 3 - a) * PL + j], wq = s_l[(8 * i + 4 + a) * PL + j];
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
                            s_l[(4 * j + k) * PL + 2 * i] = lo;
                            s_l[(4 * j + k) * PL + 2 * i + 1] = hi;
                        }
                    } else {
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            uint32_t wp = 0, wq = 0;
#pragma unroll
                            for (int k = 0; k < 4; ++k) { wp |= (uint32_t)Pm[a][k] << (8 * k); wq |= (uint32_t)Qm[a][k] << (8 * k); }
                            s_l[(8 * i + 3 - a) * PL + j] = wp;
                            s_l[(8 * i + 4 + a) * PL + j] = wq;
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
                    const int qpi = (((mq & DBK_QP) + (s_map[bp] & DBK_QP) + 1) >> 1) + (c ? g.cqp[1] : g.cqp[0]);
                    const int tc = c_tc_table[min(max(qpc_table(qpi) + 2 + 2 * nib4(offs >> 4), 0), 53)];
                    const bool nop = s_nf[bp] != 0, noq = s_nf[bq] != 0;
                    uint32_t* w = s_cw(c);
                    if (!dir) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            uint32_t lo = w[(4 * j + k) * PC + 2 * i], hi = w[(4 * j + k) * PC + 2 * i + 1];
                            int p0 = byte_of(lo, 3), q0 = byte_of(hi, 0);
                            dbk_chroma_line(p0, byte_of(lo, 2), q0, byte_of(hi, 1), tc, nop, noq);
                            w[(4 * j + k) * PC + 2 * i] = set_byte(lo, 3, p0);
                            w[(4 * j + k) * PC + 2 * i + 1] = set_byte(hi, 0, q0);
                        }
                    } else {
                        const uint32_t w1 = w[(8 * i + 2) * PC + j], w4 = w[(8 * i + 5) * PC + j];
                        uint32_t w2 = w[(8 * i + 3) * PC + j], w3 = w[(8 * i + 4) * PC + j];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            int p0 = byte_of(w2, k), q0 = byte_of(w3, k);
                            dbk_chroma_line(p0, byte_of(w1, k), q0, byte_of(w4, k), tc, nop, noq);
                            w2 = set_byte(w2, k, p0);
                            w3 = set_byte(w3, k, q0);
                        }
                        w[(8 * i + 3) * PC + j] = w2;
                        w[(8 * i + 4) * PC + j] = w3;
                    }
                }
            }
            __syncthreads();
        }
    }

    // ---- SAO of the CTB from the (deblocked) window; one UL / UC-sample row unit per task ----
    const uint32_t allow = s_allow;
    for (int u = tid; u < SH::N_SAO; u += T) {
    int c, t;
    constexpr int NL = S * (S / SH::UL), NC = SC * (SC / SH::UC);
    if (u < NL) { c = 0; t = u; }
    else { c = 1 + (u - NL) / NC; t = (u - NL) % NC; }
    const int sub = c ? 1 : 0;
    const int U = c ? SH::UC : SH::UL;                 // samples per unit (16 or 8)
    const int NW = U / 4;
    const int cs = S >> sub;
    const int upr = cs / U;
    const int row = t / upr, col = (t % upr) * U;
    const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
    const int xb = c ? xc0 : x0, yb = c ? yc0 : y0;
    const int X = xb + col, Y = yb + row;
    if (X >= W || Y >= H) continue;
    const uint32_t* win = c ? s_cw(c - 1) : s_l;
    const int wst = c ? PC : PL;
    // window dword (r, d) holds samples (xb - 4 + 4d .. +3, yb - 4 + r)
    const int wr = row + 4, wd = col / 4 + 1;
    uint32_t cur[4], res[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = q < NW ? win[wr * wst + wd + q] : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) res[q] = cur[q];
    const int typ = sao_on ? me.sao_type[c] : 0;
    if (typ != 0) {
        // packed byte arithmetic, 4 samples per dword (SWAR): per sample a table index
        // (edgeIdx or band slot) is built in a byte, the offsets are looked up 4 at a time
        // with v_perm_b32 from 8-byte tables, and v + offset is clipped in 16-bit lanes
        const int cls = me.sao_class[c];
        int tab[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (typ == 2) {        // raw e = 2 + sgn(v - a) + sgn(v - b): edgeIdx 1, 2, 0, 3, 4
            tab[0] = me.sao_offset[c][0]; tab[1] = me.sao_offset[c][1];
            tab[3] = me.sao_offset[c][2]; tab[4] = me.sao_offset[c][3];
        } else {               // slot 1..4 = bands sao_band_position + 0..3, slot 0 = no offset
#pragma unroll
            for (int k = 0; k < 4; ++k) tab[k + 1] = me.sao_offset[c][k];
        }
        uint32_t tp_lo = 0, tp_hi = 0, tn_lo = 0, tn_hi = 0;       // max(off, 0) / max(-off, 0)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tp_lo |= (uint32_t)max(tab[k], 0) << (8 * k);
            tn_lo |= (uint32_t)max(-tab[k], 0) << (8 * k);
            tp_hi |= (uint32_t)max(tab[k + 4], 0) << (8 * k);
            tn_hi |= (uint32_t)max(-tab[k + 4], 0) << (8 * k);
        }
        // which samples of the unit may be changed: neighbours available (EO), not PCM/bypass
        uint32_t okm[4];
        const bool has_l = X > 0, has_u = Y > 0, has_d = Y + 1 < H, right_in = X + U < W;
        const int ru = Y == yb ? 0 : 1, rd = Y == yb + cs - 1 ? 2 : 1;
        const int cl = X == xb ? 0 : 1, cr = X + U == xb + cs ? 2 : 1;
        auto rok = [&](int rr, int cc) { return ((allow >> (rr * 3 + cc)) & 1u) != 0; };
        bool mid = true, first = true, last = true;
        if (typ == 2) {
            const bool vert = has_u && has_d;
            if (cls == 0) { first = has_l && rok(1, cl); last = right_in && rok(1, cr); }
            else if (cls == 1) { mid = first = last = vert && rok(ru, 1) && rok(rd, 1); }
            else if (cls == 2) {
                mid = vert && rok(ru, 1) && rok(rd, 1);
                first = vert && has_l && rok(ru, cl) && rok(rd, 1);
                last = vert && right_in && rok(ru, 1) && rok(rd, cr);
            } else {
                mid = vert && rok(ru, 1) && rok(rd, 1);
                first = vert && has_l && rok(ru, 1) && rok(rd, cl);
                last = vert && right_in && rok(ru, cr) && rok(rd, 1);
            }
        }
        const int ilast = min(U, W - X) - 1;                 // last sample inside the picture
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t m = mid ? 0xffffffffu : 0u;
            if (q == 0) m = first ? (m | 0xffu) : (m & ~0xffu);
            if (q == (ilast >> 2)) {
                const uint32_t b = 0xffu << (8 * (ilast & 3));
                m = last ? (m | b) : (m & ~b);
            }
            // 4 samples never straddle an 8x8 luma block
            const int lx = (X + 4 * q) << sub, ly = Y << sub;
            if (s_nf[((ly >> 3) - (y0 >> 3) + 1) * NB + (lx >> 3) - (x0 >> 3) + 1]) m = 0;
            okm[q] = m;
        }
        auto split_lo = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c020c00u); };   // bytes 0, 2
        auto split_hi = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c030c01u); };   // bytes 1, 3
        auto join = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x06020400u); };
        // v + table[sel] clipped to [0, 255], 4 samples
        auto apply = [&](uint32_t v, uint32_t sel) {
            const uint32_t pos = __builtin_amdgcn_perm(tp_hi, tp_lo, sel);
            const uint32_t neg = __builtin_amdgcn_perm(tn_hi, tn_lo, sel);
            const uint32_t m255 = 0x00ff00ffu;
            const uint32_t rl = pk_min_u16(pk_subsat_u16(pk_add_u16(split_lo(v), split_lo(pos)), split_lo(neg)), m255);
            const uint32_t rh = pk_min_u16(pk_subsat_u16(pk_add_u16(split_hi(v), split_hi(pos)), split_hi(neg)), m255);
            return join(rl, rh);
        };
        if (typ == 1) {
            const uint32_t badd = (uint32_t)((32 - cls) & 31) * 0x01010101u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= NW) break;
                const uint32_t k = (((cur[q] >> 3) & 0x1f1f1f1fu) + badd) & 0x1f1f1f1fu;
                const uint32_t big = (((k & 0x1c1c1c1cu) + 0x7f7f7f7fu) & 0x80808080u) >> 7;
                const uint32_t sel = (k + 0x01010101u) & ~((big << 8) - big);
                res[q] = (apply(cur[q], sel) & okm[q]) | (cur[q] & ~okm[q]);
            }
        } else {
            // rows above / below with one dword either side (window dwords wd-1 .. wd+NW)
            uint32_t up[6], mi[6], dn[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const bool in = q <= NW + 1;
                mi[q] = in ? win[wr * wst + wd - 1 + q] : 0u;
                up[q] = in ? win[(wr - 1) * wst + wd - 1 + q] : 0u;
                dn[q] = in ? win[(wr + 1) * wst + wd - 1 + q] : 0u;
            }
            // 2 + sgn(v - a) + sgn(v - b) in unsigned 16-bit lanes: [v > a] = min(sat(v - a), 1)
            auto gt = [&](uint32_t v, uint32_t a) { return pk_min_u16(pk_subsat_u16(v, a), 0x00010001u); };
            auto edge = [&](uint32_t v, uint32_t a, uint32_t b) {
                return pk_sub_u16(pk_add_u16(pk_add_u16(gt(v, a), gt(v, b)), 0x00020002u), pk_add_u16(gt(a, v), gt(b, v)));
            };
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= NW) break;
                uint32_t a, b;                                 // neighbours of the 4 samples, byte-aligned
                if (cls == 0) { a = __builtin_amdgcn_alignbyte(mi[q + 1], mi[q], 3); b = __builtin_amdgcn_alignbyte(mi[q + 2], mi[q + 1], 1); }
                else if (cls == 1) { a = up[q + 1]; b = dn[q + 1]; }
                else if (cls == 2) { a = __builtin_amdgcn_alignbyte(up[q + 1], up[q], 3); b = __builtin_amdgcn_alignbyte(dn[q + 2], dn[q + 1], 1); }
                else { a = __builtin_amdgcn_alignbyte(up[q + 2], up[q + 1], 1); b = __builtin_amdgcn_alignbyte(dn[q + 1], dn[q], 3); }
                const uint32_t v = cur[q];
                const uint32_t sel = join(edge(split_lo(v), split_lo(a), split_lo(b)), edge(split_hi(v), split_hi(a), split_hi(b)));
                res[q] = (apply(v, sel) & okm[q]) | (v & ~okm[q]);
            }
        }
    }
    uint8_t* dst = P->out[c] + (size_t)Y * (c ? g.stride[1] : g.stride[0]) + X;
    if (NW == 4) *reinterpret_cast<uint4*>(dst) = make_uint4(res[0], res[1], res[2], res[3]);
    else *reinterpret_cast<uint2*>(dst) = make_uint2(res[0], res[1]);
    }
}

}  // namespace p265r
