// Residual phase: scaling (8.6.3) + inverse DCT/DST (8.6.4.2) + bdShift (8.6.2).
//
// Replaces decoder/scaling.py:4-47 and decoder/transform.py:74-109 (the reference's
// 1-D inverse indexes the matrix transposed and samples the wrong axis; this follows
// the spec, checked against oracle/recon_oracle.py:residual_block).
//
// Data layout: the batch's coefficients are re-packed at upload into one int16 pool,
// grouped by job class (luma 4x4 DST, chroma 4x4 DCT, 8x8, 16x16, 32x32, transform
// skip), each TB's N*N levels contiguous in raster [y][x] order.  Each kernel streams
// its class's slab and writes residual samples r[y][x] at the same offsets of a
// separate int16 buffer (clamped to int16, exact for BitDepth <= 15 because the
// reconstruction clips), so a resident batch can be re-run.
// HBM traffic per coefficient: 2 B read + 2 B write; no MFMA (integer butterflies).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "tables.h"

namespace p265r {

#ifndef P265R_RES_NT
#define P265R_RES_NT 0   // A/B: residual stores non-temporal (the row kernel reads them a phase later)
#endif
typedef unsigned int res_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void res_store16(int16_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    if constexpr (P265R_RES_NT) __builtin_nontemporal_store(res_u4{a, b, c, d}, reinterpret_cast<res_u4*>(p));
    else *reinterpret_cast<uint4*>(p) = make_uint4(a, b, c, d);
}

struct ResJob {          // 8 bytes, one per coded TB, in pool order within its class
    uint32_t off;        // int16 offset of the TB in the pool
    uint8_t  qp;         // qP (incl. QpBdOffset)
    uint8_t  flags;      // P265R_TB_*
    uint8_t  log2;
    uint8_t  c_idx;
};

enum ResClass { RC_DST4 = 0, RC_DCT4, RC_DCT8, RC_DCT16, RC_DCT32, RC_TSKIP, RC_NUM };

__device__ __forceinline__ int clamp16(long long v) {
    return v < -32768 ? -32768 : (v > 32767 ? 32767 : (int)v);
}
__device__ __forceinline__ int clamp16i(int v) {
    return v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
}

// d = Clip3(-32768, 32767, (L * 16 * levelScale[qP%6] << (qP/6) + (1 << (bdShift-1))) >> bdShift)
// computed exactly in 32 bits with the shift pair folded: |L| <= 2^15 and 16 * 72 < 2^11 give
// |L * scale| < 2^26 (one 24-bit multiply), and lshift = qP/6 - bdShift <= 8 - 5 = 3 (8-bit video:
// qP <= 51, bdShift >= 5; p265r_create rejects other bit depths), so the shifted product stays
// below 2^29.  (Round 2 widened it to 64 bits: ~10 VALU per coefficient instead of 5.)
struct Dequant {
    int scale, lshift, rshift, rnd;
    __device__ __forceinline__ Dequant(int qp, int bd_shift) {
        const int per = qp / 6;
        // levelScale[qP % 6] = 40, 45, 51, 57, 64, 72 as the bytes of one 64-bit constant (a shift, not a
        // per-lane branch tree: qP differs between a wave's TBs)
        scale = 16 * (int)((0x484039332D28ull >> (8 * (qp - 6 * per))) & 0xffu);
        if (per >= bd_shift) { lshift = per - bd_shift; rshift = 0; rnd = 0; }
        else { lshift = 0; rshift = bd_shift - per; rnd = 1 << (rshift - 1); }
        scale <<= lshift;                 // <= 1152 << 3 < 2^14: still a 24-bit operand (one v_mad_i32_i24)
    }
    __device__ __forceinline__ int operator()(int level) const {
        return clamp16i((__mul24(level, scale) + rnd) >> rshift);
    }
};

// Scaling lists (scaling_list_enabled_flag; decoder/scaling.py:32-44): m[y][x] = the TB's ScalingFactor
// instead of 16, from the context's 2032-byte table (p265r_set_scaling_factors: intra matrices, [y][x] per
// (sizeId, matrixId = cIdx)).  |L * m * levelScale| < 2^31, but the << qP / 6 needs 64 bits.
__host__ __device__ __forceinline__ int sf_offset(int log2, int c_idx) {
    // 4x4 Y/Cb/Cr at 0/16/32, 8x8 at 48/112/176, 16x16 at 240/496/752, 32x32 Y at 1008
    return log2 == 2 ? 16 * c_idx : (log2 == 3 ? 48 + 64 * c_idx : (log2 == 4 ? 240 + 256 * c_idx : 1008));
}
struct DequantM {
    int ls, per, bds;
    __device__ __forceinline__ DequantM(int qp, int bd_shift) {
        per = qp / 6;
        ls = (int)((0x484039332D28ull >> (8 * (qp - 6 * per))) & 0xffu);
        bds = bd_shift;
    }
    __device__ __forceinline__ int operator()(int level, int m) const {
        const long long v = (long long)(level * m * ls) << per;
        return clamp16((v + (1ll << (bds - 1))) >> bds);
    }
};

// ---------------------------------------------------------------------------
// 4x4: one thread per TB, everything in registers.
// ---------------------------------------------------------------------------
template <bool DST>
__device__ __forceinline__ int t4(int j, int i) { return DST ? kDST4[j][i] : kDCT32[j * 8][i]; }

// o[n] = sum_k t4(k, n) * c[k] in butterfly form (same integer sums as the matrix product):
// DST 29/55/74/84 factorisation, DCT even/odd.
template <bool DST>
__device__ __forceinline__ void inv4(const int (&c)[4], int (&o)[4]) {
    if constexpr (DST) {
        static_assert(kDST4[0][0] == 29 && kDST4[0][1] == 55 && kDST4[1][0] == 74 && kDST4[0][3] == 84, "DST matrix");
        const int a = c[0] + c[2], b = c[2] + c[3], d = c[0] - c[3], e = 74 * c[1];
        o[0] = 29 * a + 55 * b + e;
        o[1] = 55 * d - 29 * b + e;
        o[2] = 74 * (c[0] - c[2] + c[3]);
        o[3] = 55 * a + 29 * d - e;
    } else {
        const int e0 = 64 * (c[0] + c[2]), e1 = 64 * (c[0] - c[2]);
        const int o0 = 83 * c[1] + 36 * c[3], o1 = 36 * c[1] - 83 * c[3];
        o[0] = e0 + o0; o[1] = e1 + o1; o[2] = e1 - o1; o[3] = e0 - o0;
    }
}

// A class's TBs are packed back to back in job order (p265r_batch_upload), so TB i of a fixed-size
// class sits at slab + i * N * N: the coefficient loads do not wait for the job record (which
// only supplies qP), one dependent memory round trip less per TB.
template <bool DST, bool SL = false>
__global__ __launch_bounds__(256) void residual4_kernel(const int16_t* __restrict__ pool,
                                                        int16_t* __restrict__ res,
                                                        const ResJob* __restrict__ jobs, int n_jobs,
                                                        int bit_depth, uint32_t slab, const uint8_t* __restrict__ sf) {
    P265R_BW_PRIO_SET();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_jobs) return;
    const ResJob jb = jobs[i];
    const size_t off = (size_t)slab + (size_t)i * 16;
    const int16_t* blk = pool + off;
    int16_t* dst = res + off;
    const uint4 raw0 = *reinterpret_cast<const uint4*>(blk);       // 16 x int16 = 32 B
    const uint4 raw1 = *reinterpret_cast<const uint4*>(blk + 8);
    const uint32_t w[8] = {raw0.x, raw0.y, raw0.z, raw0.w, raw1.x, raw1.y, raw1.z, raw1.w};
    int d[4][4];
    if constexpr (SL) {
        const DequantM dq(jb.qp, bit_depth + 2 - 5);
        const uint4 mw = *reinterpret_cast<const uint4*>(sf + sf_offset(2, jb.c_idx));
        const uint32_t mv[4] = {mw.x, mw.y, mw.z, mw.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int lv = (int)(int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xffff);
            d[k >> 2][k & 3] = dq(lv, (int)((mv[k >> 2] >> (8 * (k & 3))) & 0xffu));
        }
    } else {
        const Dequant dq(jb.qp, bit_depth + 2 - 5);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int lv = (int)(int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xffff);
            d[k >> 2][k & 3] = dq(lv);
        }
    }
    int g[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {            // columns: e[y][x] = sum_j T[j][y] d[j][x]
        const int cin[4] = {d[0][x], d[1][x], d[2][x], d[3][x]};
        int e[4];
        inv4<DST>(cin, e);
#pragma unroll
        for (int y = 0; y < 4; ++y) g[y][x] = clamp16i((e[y] + 64) >> 7);
    }
    const int bd2 = 20 - bit_depth;
    const int rnd2 = 1 << (bd2 - 1);
    uint32_t o[8];
#pragma unroll
    for (int y = 0; y < 4; ++y) {
        int r[4];
        const int rin[4] = {g[y][0], g[y][1], g[y][2], g[y][3]};
        int acc[4];
        inv4<DST>(rin, acc);
#pragma unroll
        for (int x = 0; x < 4; ++x) r[x] = clamp16i((acc[x] + rnd2) >> bd2);
        o[y * 2 + 0] = (uint32_t)(uint16_t)r[0] | ((uint32_t)(uint16_t)r[1] << 16);
        o[y * 2 + 1] = (uint32_t)(uint16_t)r[2] | ((uint32_t)(uint16_t)r[3] << 16);
    }
    res_store16(dst, o[0], o[1], o[2], o[3]);
    res_store16(dst + 8, o[4], o[5], o[6], o[7]);
}

// ---------------------------------------------------------------------------
// One N-point inverse transform, x[n] = sum_k M_N[k][n] c[k] with M_N[k][n] = kDCT32[k*32/N][n],
// as an even/odd butterfly: even rows of the DCT matrix are symmetric (M_N[2k][n] = M_{N/2}[k][n]
// for n < N/2), odd rows antisymmetric, so x[n] = E[n] + O[n] and x[N-1-n] = E[n] - O[n] with E the
// N/2-point transform of the even coefficients.  Same integer sum as the matrix product (exact),
// about N^2/3 instead of N^2 multiply-adds.
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void inv_dct_eo(const int (&c)[N], int (&x)[N]) {
    constexpr int H = N / 2;
    constexpr int S = 32 / N;
    int ce[H], ev[H];
#pragma unroll
    for (int k = 0; k < H; ++k) ce[k] = c[2 * k];
    if constexpr (H == 2) {
        ev[0] = kDCT32[0][0] * ce[0] + kDCT32[16][0] * ce[1];
        ev[1] = kDCT32[0][1] * ce[0] + kDCT32[16][1] * ce[1];
    } else {
        inv_dct_eo<H>(ce, ev);
    }
#pragma unroll
    for (int n = 0; n < H; ++n) {
        int od = 0;
#pragma unroll
        for (int j = 0; j < H; ++j) od += kDCT32[(2 * j + 1) * S][n] * c[2 * j + 1];
        x[n] = ev[n] + od;
        x[N - 1 - n] = ev[n] - od;
    }
}

// The same butterfly with the odd parts as packed 16-bit dot products: every input of either stage is an
// int16 (dequantised coefficients and the stage-1 output are clipped to 16 bits), so two odd coefficients
// pack into one register and one v_dot2c_i32_i16 with a literal pair of matrix entries adds two products
// into the 32-bit sum (exact: |sum| < 2^15 * 90 * 32 < 2^31).  About half the multiply-add instructions of
// inv_dct_eo, the same integer result.
#ifndef P265R_RES_DOT2
#define P265R_RES_DOT2 1
#endif
typedef short res_v2s __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack16(int lo, int hi) {          // (int16) lo | (int16) hi << 16
    return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}
// rnd64: a rounding constant / 64 added to every output for free (folded into the 2-point stage, where every
// output's sum starts: 64 c0 + 64 c1 + rnd = 64 (c0 + c1 + rnd64))
template <int N>
__device__ __forceinline__ void inv_dct_d2(const int (&c)[N], int (&x)[N], int rnd64 = 0) {
    constexpr int H = N / 2;
    constexpr int S = 32 / N;
    int ce[H], ev[H];
#pragma unroll
    for (int k = 0; k < H; ++k) ce[k] = c[2 * k];
    if constexpr (H == 2) {
        static_assert(kDCT32[0][0] == 64 && kDCT32[16][0] == 64 && kDCT32[0][1] == 64 && kDCT32[16][1] == -64, "DCT rows 0 / 16");
        ev[0] = 64 * (ce[0] + ce[1] + rnd64);
        ev[1] = 64 * (ce[0] - ce[1] + rnd64);
    } else {
        inv_dct_d2<H>(ce, ev, rnd64);
    }
    if constexpr (H == 2) {                                      // one odd pair: plain products
#pragma unroll
        for (int n = 0; n < H; ++n) {
            const int od = kDCT32[S][n] * c[1] + kDCT32[3 * S][n] * c[3];
            x[n] = ev[n] + od;
            x[N - 1 - n] = ev[n] - od;
        }
    } else {
        uint32_t p[H / 2];                                       // (c[4j+1], c[4j+3])
#pragma unroll
        for (int j = 0; j < H / 2; ++j) p[j] = pack16(c[4 * j + 1], c[4 * j + 3]);
#pragma unroll
        for (int n = 0; n < H; ++n) {
            int xp = ev[n];                                      // ev + od accumulated in place (no zero init)
#pragma unroll
            for (int j = 0; j < H / 2; ++j) {
                const uint32_t kk = (uint32_t)(uint16_t)(int16_t)kDCT32[(4 * j + 1) * S][n] |
                                    (uint32_t)(uint16_t)(int16_t)kDCT32[(4 * j + 3) * S][n] << 16;
                xp = __builtin_amdgcn_sdot2(__builtin_bit_cast(res_v2s, p[j]), __builtin_bit_cast(res_v2s, kk), xp, false);
            }
            x[n] = xp;
            x[N - 1 - n] = 2 * ev[n] - xp;                       // ev - od
        }
    }
}

// ---------------------------------------------------------------------------
// NxN, N = 8/16/32: N threads per TB (256/N TBs per 256-thread block).
//   load row r (16-B vectors) -> dequant -> LDS [r][c]
//   thread c: column transform (stage 1) + (e+64)>>7 clip -> LDS [k][c]
//   thread r: row transform (stage 2) + bdShift -> 16-B vector stores, in place.
// Matrix entries are compile-time immediates (fully unrolled).
// ---------------------------------------------------------------------------
template <int LOG2, bool SL = false>
__global__ __launch_bounds__(256) void residualN_kernel(const int16_t* __restrict__ pool,
                                                       int16_t* __restrict__ res,
                                                       const ResJob* __restrict__ jobs, int n_jobs,
                                                       int bit_depth_luma, int bit_depth_chroma, uint32_t slab,
                                                       const uint8_t* __restrict__ sf) {
    P265R_BW_PRIO_SET();
    constexpr int N = 1 << LOG2;
    constexpr int TPB = 256 / N;                 // TBs per block
    constexpr int S = N + 2;                     // padded LDS row (odd dword stride)
    __shared__ int16_t tile[TPB][N * S];
    const int local = threadIdx.x / N;
    const int lane = threadIdx.x % N;            // row index (load/store) and column index (stage 1)
    const int job = blockIdx.x * TPB + local;
    const bool active = job < n_jobs;
    int16_t* t = tile[local];
    ResJob jb = active ? jobs[job] : ResJob{0, 0, 0, 0, 0};
    const size_t off = (size_t)slab + (size_t)(active ? job : 0) * (N * N);   // (class slab, job order)
    const int16_t* blk = pool + off;
    int16_t* dst = res + off;
    const int bit_depth = jb.c_idx ? bit_depth_chroma : bit_depth_luma;
    if (active && SL) {
        const DequantM dq(jb.qp, bit_depth + LOG2 - 5);
        const uint8_t* mrow = sf + sf_offset(LOG2, jb.c_idx) + lane * N;      // m[row = lane][..]
#pragma unroll
        for (int v = 0; v < N / 8; ++v) {
            const uint4 raw = *reinterpret_cast<const uint4*>(blk + lane * N + v * 8);
            const uint2 mw = *reinterpret_cast<const uint2*>(mrow + v * 8);
            const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int lv = (int)(int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xffff);
                const int m = (int)((((k < 4) ? mw.x : mw.y) >> (8 * (k & 3))) & 0xffu);
                t[lane * S + v * 8 + k] = (int16_t)dq(lv, m);
            }
        }
    } else if (active) {
        const Dequant dq(jb.qp, bit_depth + LOG2 - 5);
#pragma unroll
        for (int v = 0; v < N / 8; ++v) {
            const uint4 raw = *reinterpret_cast<const uint4*>(blk + lane * N + v * 8);
            const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int lv = (int)(int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xffff);
                t[lane * S + v * 8 + k] = (int16_t)dq(lv);
            }
        }
    }
    __syncthreads();
    if (active) {
        int col[N], e[N];
#pragma unroll
        for (int k = 0; k < N; ++k) col[k] = t[k * S + lane];
#ifdef P265R_RES_NOMATH   // timing experiment only (wrong results): the transform's arithmetic removed
#pragma unroll
        for (int k = 0; k < N; ++k) e[k] = col[k] << 7;
#else
        if constexpr (P265R_RES_DOT2) inv_dct_d2<N>(col, e, 1); else inv_dct_eo<N>(col, e);   // (+64 folded in)
#endif
#pragma unroll
        for (int y = 0; y < N; ++y) t[y * S + lane] = (int16_t)clamp16i((e[y] + (P265R_RES_DOT2 ? 0 : 64)) >> 7);
    }
    __syncthreads();
    if (active) {
        int row[N], xr[N];
#pragma unroll
        for (int k = 0; k < N; ++k) row[k] = t[lane * S + k];
#ifdef P265R_RES_NOMATH
#pragma unroll
        for (int k = 0; k < N; ++k) xr[k] = row[k];
#else
        // (8-bit video: bdShift 12, its rounding 2048 = 64 * 32 folded into the butterfly)
        if constexpr (P265R_RES_DOT2) inv_dct_d2<N>(row, xr, 1 << (19 - bit_depth - 6)); else inv_dct_eo<N>(row, xr);
#endif
        const int bd2 = 20 - bit_depth;
        const int rnd2 = 1 << (bd2 - 1);
#ifdef P265R_RES_PADV     // timing experiment only: P265R_RES_PADV dependent VALU per thread
        {
            uint32_t z = (uint32_t)lane;
#pragma unroll
            for (int q = 0; q < P265R_RES_PADV; ++q) asm volatile("v_add_u32 %0, 1, %0" : "+v"(z));
            asm volatile("" :: "v"(z));
        }
#endif
#pragma unroll
        for (int v = 0; v < N / 8; ++v) {
            uint32_t o[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                int r2[2];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int x = v * 8 + h * 2 + q;
                    r2[q] = clamp16i((xr[x] + (P265R_RES_DOT2 ? 0 : rnd2)) >> bd2);
                }
                o[h] = (uint32_t)(uint16_t)r2[0] | ((uint32_t)(uint16_t)r2[1] << 16);
            }
            res_store16(dst + lane * N + v * 8, o[0], o[1], o[2], o[3]);
        }
    }
}

// ---------------------------------------------------------------------------
// Transform skip (any size): r = (d << tsShift + rnd) >> bdShift, tsShift = 5 + log2.
// One thread per TB (rare: ~0.8 % of luma 4x4 in the sanity.bin mix).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void residual_tskip_kernel(const int16_t* __restrict__ pool,
                                                             int16_t* __restrict__ res,
                                                             const ResJob* __restrict__ jobs, int n_jobs,
                                                             int bit_depth_luma, int bit_depth_chroma,
                                                             const uint8_t* __restrict__ sf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_jobs) return;
    const ResJob jb = jobs[i];
    const int bd = jb.c_idx ? bit_depth_chroma : bit_depth_luma;
    const Dequant dq(jb.qp, bd + jb.log2 - 5);
    const DequantM dqm(jb.qp, bd + jb.log2 - 5);        // scaling lists: m applies to transform skip too (8.6.4.2)
    const uint8_t* m = sf ? sf + sf_offset(jb.log2, jb.c_idx) : nullptr;
    const int ts = 5 + jb.log2;
    const int bd2 = 20 - bd;
    const int n2 = 1 << (2 * jb.log2);
    const int16_t* blk = pool + jb.off;
    int16_t* dst = res + jb.off;
    for (int k = 0; k < n2; ++k) {
        const long long r = (long long)(m ? dqm(blk[k], m[k]) : dq(blk[k])) << ts;
        dst[k] = (int16_t)clamp16((r + (1 << (bd2 - 1))) >> bd2);
    }
}

}  // namespace p265r
