// Intra prediction + reconstruction phase: one wavefront (64 lanes) per CTU.
//
// Replaces the per-CU chain of the reference, Cu.decode_intra -> IntraPu.decode ->
// decode_neighbor / decode_intra_{planar,dc,angular} -> reconstruction
// (decoder/cu.py:595-615, decoder/intra.py:39-305, decoder/reconstruction.py:4-27),
// which fetches every neighbour sample through a tree walk (cu.py:617-632,
// image.py:38-73) and never runs (cu.py:487-488).
//
// Scheduling: intra TBs of a CTU are serial (decode order), and a CTU needs its left,
// top-left, top and top-right CTUs.  The host launches one kernel per anti-diagonal
// step s = cx + 2*cy (2-CTU-lag wavefront) over ALL pictures of the batch, so every
// launch holds (CTUs on the diagonal) x (pictures) independent wavefronts.
//
// Per CTU the wave keeps, in LDS: the CTU's own reconstructed samples (interior),
// the row above it (x = -1 .. 2*CtbSize-1, incl. top-left and top-right CTUs) and the
// column left of it, all loaded once from the picture plane.  Neighbour availability
// (6.4.1) is then decided per reference sample without any table: outside the CTU by
// the CTU-level slice/tile checks, inside it by the z-order (Morton) rank of the 4x4
// block, which is exactly MinTbAddrZs restricted to one CTB (pps.py:246-262).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "../../include/p265r.h"
#include "tables.h"

namespace p265r {

// Intra job record written by intra_prep_kernel (layout: intra_prep.h).
struct IntraJob {                // 24 bytes (intra_prep.h documents the words)
    uint32_t w[6];
};

struct DevPic {                 // per picture, device-resident table
    const p265r_ctu* ctus;
    const p265r_tb*  tbs;       // coef_off rewritten to pool offsets
    uint8_t* rec[3];            // pre-SAO planes (padded stride)
    uint8_t* out[3];            // SAO output planes (== rec when SAO is off)
    const uint8_t* nofilter;    // per 8x8 luma block or nullptr
    IntraJob* jobs;             // same index space as tbs (jobs of a CTU start at tb_begin)
    uint32_t* jcount;           // per CTU four words: luma jobs | chroma jobs << 16 (chroma listed first), the
                                // index of the first job of each list that reads the top-right CTU, the index of
                                // one past the last job in the CTB's bottom-left quadrant, 0 (intra_prep.h)
    uint8_t* dbk_map;           // per 8x8 luma block (loopfilter.h), nullptr without deblocking
    int32_t  pool_rel;          // residual pool element index of coefficient pool element 0 (<= 0)
    uint32_t zero_off;          // residual pool element index of a 256-sample zero block
    uint32_t wh;                // this picture's luma size, width | height << 16 (Geo::ragged batches)
    uint32_t pad_;
};

// Batch-uniform layout of the per-picture arrays (p265r.hip batch_upload places them at fixed
// strides), so a kernel computes a picture's plane and CTU-record addresses without loading its
// DevPic first: one dependent memory round trip less
struct BatchView {
    uint8_t* rec0;              // picture 0's reconstruction planes (Y at plane_off[0])
    uint8_t* out0;              // picture 0's output planes (== rec0 without in-loop filters)
    uint64_t pic_bytes;         // bytes of one picture's three planes
    uint64_t plane_off[3];      // Y, Cb, Cr offsets inside a picture's planes
    const p265r_ctu* ctus0;     // picture 0's CTU records (PicSizeInCtbsY per picture)
    int* err;                   // the batch's sticky error word (bit 0: a row-kernel wait gave up; bit 1: the
                                // prep kernel's half-CTU self-check failed, Geo::tr_check)
};

struct Geo {                    // batch-uniform geometry
    int w, h;                   // luma size
    int cw, ch;                 // chroma size
    int stride[3];
    int ctb_log2, wc, hc;
    int bd[3];
    int strong;
    int lf_tiles;
    int nf_w;                   // nofilter / deblocking map width (ceil(w/8))
    int cqp[2];                 // pps_cb_qp_offset, pps_cr_qp_offset (chroma deblocking)
    int fair;                   // intra_rows_kernel: the workgroup behind its CU partner raises its priority
                                // (P265R_FAIR, default 1)
    int quad;                   // intra_prep_kernel merges 4x4 quads into one job: bit 0 luma, bit 1 chroma;
                                // bit 2 (A/B only): Cb+Cr 8x8 pairs take the general path
                                // (P265R_QUAD, default 3)
    int ragged;                 // some picture of the batch is smaller than w x h (DevPic::wh): kernels
                                // take that picture's size from pic_geo().  Per-picture arrays keep the
                                // context-size slots (CTU records, job counts, maps, planes) -- a
                                // picture's CTU raster and map rows use ITS width in CTUs / 8x8 blocks
    int tr_info;                // intra_prep_kernel: compute the top-right / bottom-left job indices (jcount words 1
                                // and 2) -- set for batches that may run a latency layout (2 pictures per CU or
                                // fewer), whose row kernels read them; the throughput builds never do
    int tr_check;               // P265R_TR_CHECK (tests): the host launches the cross-group row kernel's checking
                                // instance, which poisons the top-right part of a CTU's row-above copy until its
                                // wait and serves the left half of every CTU's bottom line from the half-CTU
                                // publish alone (checks prep's `tr` and `br` deterministically); the prep kernel
                                // checks `br` against the TBs' extents (error word bit 1)
    int pel16;                  // samples are 16-bit (BitDepth 9..12): planes of stride[] samples of 2
                                // bytes, the per-diagonal intra kernel and loopfilter16.h (else uint8_t)
};

// A/B: s_setprio of the bandwidth-phase kernels' waves (residual, prep, SAO), 0 = default
#ifndef P265R_BW_PRIO
#define P265R_BW_PRIO 0
#endif
#if P265R_BW_PRIO > 0
#define P265R_BW_PRIO_SET() __builtin_amdgcn_s_setprio(P265R_BW_PRIO)
#else
#define P265R_BW_PRIO_SET() do { } while (0)
#endif

// ragged-batch support compiled into the kernels (0: A/B only -- a ragged batch then decodes wrongly)
#ifndef P265R_RAGGED
#define P265R_RAGGED 1
#endif

// Geometry of one picture of a ragged batch: its own size, CTU grid and map width; strides and the
// per-picture slot sizes stay the context's (take them from the batch Geo before calling this).
__device__ __forceinline__ Geo pic_geo(Geo g, uint32_t wh) {
    g.w = (int)(wh & 0xffffu);
    g.h = (int)(wh >> 16);
    g.cw = g.w >> 1;
    g.ch = g.h >> 1;
    g.wc = (g.w + (1 << g.ctb_log2) - 1) >> g.ctb_log2;
    g.hc = (g.h + (1 << g.ctb_log2) - 1) >> g.ctb_log2;
    g.nf_w = (g.w + 7) >> 3;
    return g;
}

__constant__ int8_t  c_angle[35];
__constant__ int16_t c_inv_angle[35];
// job word w1 of mode m (intra_prep.h): intraPredAngle (int8) | |invAngle| << 8 (256 for the modes
// without an inverse angle: intra_rows.h ang_inv)
__constant__ uint32_t c_angw[35];
__constant__ uint32_t c_ztab[64];       // avail_ztab_word(s, yu) at 16 s + yu (ref_avail_mask32)

__host__ __device__ __forceinline__ int morton4(int x, int y) {      // 4-bit x, y -> 8-bit z-order
    x = (x | (x << 2)) & 0x33; x = (x | (x << 1)) & 0x55;
    y = (y | (y << 2)) & 0x33; y = (y | (y << 1)) & 0x55;
    return x | (y << 1);
}

__device__ __forceinline__ bool ctu_same_region(const p265r_ctu& a, const p265r_ctu& b) {
    return a.slice_addr == b.slice_addr && a.tile_id == b.tile_id;
}

template <typename T>           // sample type: uint8_t (BitDepth 8) or uint16_t (BitDepth 9..12, Geo::pel16)
struct CtuLdsT {
    T        y[64 * 64];        // interior luma, stride 64
    T        c[2][32 * 32];     // interior chroma, stride 32
    T        ytop[132];         // row y=-1, x = -1 .. 127  (index x+1)
    T        ctop[2][68];       // row y=-1, x = -1 .. 63
    T        yleft[64];         // column x=-1, y = 0 .. 63
    T        cleft[2][32];
    uint16_t ref[2][136];       // linear reference arrays (raw/substituted, filtered)
};

// Availability of the neighbouring sample at CTB-relative LUMA position (xl, yl) for a
// block whose top-left is at CTB-relative luma (xc, yc).  flags: bit0 L, bit1 T, bit2 TL, bit3 TR.
__device__ __forceinline__ bool nb_available(int xl, int yl, int xc, int yc, int x0, int y0,
                                             const Geo& g, int ctb, unsigned flags) {
    if (x0 + xl >= g.w || y0 + yl >= g.h) return false;
    if (yl < 0) {
        if (xl < 0) return flags & 4u;
        if (xl < ctb) return flags & 2u;
        if (xl < 2 * ctb) return flags & 8u;
        return false;
    }
    if (xl < 0) return (yl < ctb) && (flags & 1u);
    if (xl >= ctb || yl >= ctb) return false;
    return morton4(xl >> 2, yl >> 2) < morton4(xc >> 2, yc >> 2);
}

__host__ __device__ __forceinline__ bool nb_available_wh(int xl, int yl, int xc, int yc, int x0, int y0,
                                                int w, int h, int ctb, unsigned flags) {
    if (x0 + xl >= w || y0 + yl >= h) return false;
    if (yl < 0) {
        if (xl < 0) return flags & 4u;
        if (xl < ctb) return flags & 2u;
        if (xl < 2 * ctb) return flags & 8u;
        return false;
    }
    if (xl < 0) return (yl < ctb) && (flags & 1u);
    if (xl >= ctb || yl >= ctb) return false;
    return morton4(xl >> 2, yl >> 2) < morton4(xc >> 2, yc >> 2);
}

// Availability (6.4.1) of the 2L+1 reference units of an intra TB in the linear order of
// 8.4.4.2.2 (bit u; unit = 4 luma samples: left units u < L bottom-up, corner u = L, top
// units u > L left to right), for a TB of n x n samples of component c at component
// position (xr, yr) inside the CTB whose luma origin is (x0, y0).  flags: neighbouring
// CTUs usable (bit0 L, bit1 T, bit2 TL, bit3 TR; same slice and tile).  Equal to
// nb_available_wh() unit by unit (tools/avail_check.hip): the bottom-left units lie in one
// aligned block, so one z-order comparison decides them all, likewise the top-right
// units; only the picture's bottom / right edges cut them unit by unit.
__host__ __device__ __forceinline__ unsigned long long ref_avail_mask(int c, int xr, int yr, int n, int x0, int y0,
                                                                      int w, int h, int ctb, unsigned flags) {
    // straight-line form (selects, no branches): the prep kernel evaluates it on every lane at once
    const int sub = c ? 1 : 0;
    const int xc = xr << sub, yc = yr << sub, nl = n << sub;      // luma, CTB-relative
    const int L = (2 * n) >> (c ? 1 : 2);                         // units per side
    const int half = L >> 1;
    const int zc = morton4(xc >> 2, yc >> 2);
    const bool fl = (flags & 1u) != 0, ft = (flags & 2u) != 0, ftl = (flags & 4u) != 0, ftr = (flags & 8u) != 0;
    // (bitwise & / |: a short-circuit && / || becomes a divergent branch)
    const bool left = (xc > 0) | fl;
    const int zbl = morton4(max(xc - 1, 0) >> 2, min(yc + nl, ctb - 1) >> 2);
    const bool bl = (yc + nl < ctb) & (xc == 0 ? fl : zbl < zc);
    const bool corner = xc > 0 ? ((yc > 0) | ft) : (yc > 0 ? fl : ftl);
    const bool top = (yc > 0) | ft;
    const int ztr = morton4(min(xc + nl, ctb - 1) >> 2, max(yc - 1, 0) >> 2);
    const bool tr = xc + nl < ctb ? (yc > 0 ? ztr < zc : ft) : ((yc == 0) & ftr);
    // bits [lo, hi) for 0 <= lo, hi <= 33 (empty when hi <= lo)
    auto bits = [](int lo, int hi) -> unsigned long long { return ((1ull << hi) - 1ull) & ~((1ull << lo) - 1ull); };
    const int u_min = max(0, (y0 + yc + 2 * nl - h) >> 2);        // units below the picture: u < u_min
    const int j_max = (w - x0 - xc) >> 2;                          // top units inside the picture: j < j_max
    const unsigned long long m_bl = bits(min(u_min, half), half), m_l = bits(half, L), m_c = 1ull << L;
    const unsigned long long m_t = bits(L + 1, L + 1 + half);
    const unsigned long long m_tr = bits(L + 1 + half, L + 1 + max(half, min(L, j_max)));
    return (bl ? m_bl : 0ull) | (left ? m_l : 0ull) | (corner ? m_c : 0ull) | (top ? m_t : 0ull) | (tr ? m_tr : 0ull);
}

// z-order availability of the bottom-left / top-right neighbour unit inside the CTB (the morton
// comparisons of ref_avail_mask), tabulated: word 16 s + yu for TBs of 4 << s luma samples
// (s = 0..3) in unit row yu; bit 2 xu: unit (xu - 1, yu + 2^s) precedes unit (xu, yu) in z-order,
// bit 2 xu + 1: unit (xu + 2^s, yu - 1) does.  Independent of the CTB size: z-order of 4x4 units
// inside any aligned square; the cases at the CTB's edges are decided before the table is read.
__host__ __device__ inline uint32_t avail_ztab_word(int s, int yu) {
    const int su = 1 << s;
    uint32_t w = 0;
    for (int xu = 0; xu < 16; ++xu) {
        const int zc = morton4(xu, yu);
        if (xu > 0 && yu + su < 16 && morton4(xu - 1, yu + su) < zc) w |= 1u << (2 * xu);
        if (yu > 0 && xu + su < 16 && morton4(xu + su, yu - 1) < zc) w |= 1u << (2 * xu + 1);
    }
    return w;
}

// ref_avail_mask in 32-bit pieces: returns units 0..31, bit32 = unit 32 (only a 32-sample luma /
// 16-sample chroma TB has it), with the z-order comparisons read from zw = avail_ztab_word(log2(n
// in luma samples) - 2, yc / 4).  Equal to ref_avail_mask (tools/avail_check.hip, exhaustive).
__host__ __device__ __forceinline__ uint32_t ref_avail_mask32(int c, int xr, int yr, int n, int x0, int y0, int w,
                                                              int h, int ctb, unsigned flags, uint32_t zw,
                                                              uint32_t& bit32) {
    const int sub = c ? 1 : 0;
    const int xc = xr << sub, yc = yr << sub, nl = n << sub;      // luma, CTB-relative
    const int L = nl >> 1, half = L >> 1;                         // units (4 luma samples) per side
    const int xu = (xc >> 2) & 15;
    const bool fl = (flags & 1u) != 0, ft = (flags & 2u) != 0, ftl = (flags & 4u) != 0, ftr = (flags & 8u) != 0;
    const bool left = (xc > 0) | fl;
    const bool bl = (yc + nl < ctb) & (xc == 0 ? fl : ((zw >> (2 * xu)) & 1u) != 0);
    const bool corner = xc > 0 ? ((yc > 0) | ft) : (yc > 0 ? fl : ftl);
    const bool top = (yc > 0) | ft;
    const bool tr = xc + nl < ctb ? (yc > 0 ? ((zw >> (2 * xu + 1)) & 1u) != 0 : ft) : ((yc == 0) & ftr);
    const int u_min = max(0, (y0 + yc + 2 * nl - h) >> 2);        // units below the picture: u < u_min
    const int j_max = (w - x0 - xc) >> 2;                          // top units inside the picture: j < j_max
    auto bits = [](int lo, int wd) -> uint32_t { return ((1u << wd) - 1u) << lo; };   // lo <= 25, wd <= 16
    const uint32_t m_bl = bits(min(u_min, half), max(half - u_min, 0)), m_l = bits(half, half), m_c = 1u << L;
    const uint32_t m_t = bits(L + 1, half);
    const int tr_w = max(min(L, j_max) - half, 0);
    const uint32_t m_tr = bits(L + 1 + half, min(tr_w, 31 - (L + half)));   // the part below bit 32
    bit32 = (tr & (L == 16) & (j_max >= 16)) ? 1u : 0u;
    return (bl ? m_bl : 0u) | (left ? m_l : 0u) | (corner ? m_c : 0u) | (top ? m_t : 0u) | (tr ? m_tr : 0u);
}

// One launch per anti-diagonal step (P265R_SCHEDULE=steps; the only schedule of the 16-bit sample path,
// Main 10: T = uint16_t, planes of Geo::stride samples of 2 bytes).
template <typename T>
__global__ __launch_bounds__(64) void intra_step_kernel(const DevPic* __restrict__ pics,
                                                       const int16_t* __restrict__ pool,
                                                       const int16_t* __restrict__ resid,
                                                       Geo g, int step, int cy_min) {
    __shared__ CtuLdsT<T> L;
    const int lane = threadIdx.x;
    const int cy = cy_min + blockIdx.x;
    const int cx = step - 2 * cy;
    if (cy >= g.hc || cx < 0 || cx >= g.wc) return;
    const DevPic P = pics[blockIdx.y];
    if (P265R_RAGGED && g.ragged) {
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)P.wh));
        if (cy >= g.hc || cx >= g.wc) return;
    }
    const int ctb = 1 << g.ctb_log2;
    const int x0 = cx << g.ctb_log2, y0 = cy << g.ctb_log2;
    const int addr = cy * g.wc + cx;
    const p265r_ctu me = P.ctus[addr];

    unsigned flags = 0;
    if (cx > 0 && ctu_same_region(me, P.ctus[addr - 1])) flags |= 1u;
    if (cy > 0 && ctu_same_region(me, P.ctus[addr - g.wc])) flags |= 2u;
    if (cx > 0 && cy > 0 && ctu_same_region(me, P.ctus[addr - g.wc - 1])) flags |= 4u;
    if (cx + 1 < g.wc && cy > 0 && ctu_same_region(me, P.ctus[addr - g.wc + 1])) flags |= 8u;

    // ---- neighbour rows/columns from the picture planes -------------------------
    for (int c = 0; c < 3; ++c) {
        const int sub = c ? 1 : 0;
        const int cs = ctb >> sub;
        const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
        const int xb = x0 >> sub, yb = y0 >> sub;
        const T* plane = reinterpret_cast<const T*>(P.rec[c]);
        const int st = (c ? g.stride[1] : g.stride[0]);
        T* top = c ? L.ctop[c - 1] : L.ytop;
        T* left = c ? L.cleft[c - 1] : L.yleft;
        for (int e = lane; e <= 2 * cs; e += 64) {
            const int x = e - 1;
            const unsigned need = x < 0 ? 4u : (x < cs ? 2u : 8u);
            if ((flags & need) && xb + x < W) top[e] = plane[(size_t)(yb - 1) * st + xb + x];
        }
        if ((flags & 1u) && lane < cs && yb + lane < H) left[lane] = plane[(size_t)(yb + lane) * st + xb - 1];
    }
    __syncthreads();

    const p265r_tb* tbs = P.tbs + me.tb_begin;
    for (int t = 0; t < (int)me.tb_count; ++t) {
        const p265r_tb tb = tbs[t];
        const int c = tb.c_idx;
        const int sub = c ? 1 : 0;
        const int log2 = tb.log2_size, n = 1 << log2;
        const int cs = ctb >> sub;
        const int xr = tb.x - (x0 >> sub), yr = tb.y - (y0 >> sub);   // CTB-relative, component units
        const int bd = (c ? g.bd[1] : g.bd[0]);
        const int maxv = (1 << bd) - 1;
        T* interior = c ? L.c[c - 1] : L.y;
        const int ist = c ? 32 : 64;
        T* top = c ? L.ctop[c - 1] : L.ytop;
        T* left = c ? L.cleft[c - 1] : L.yleft;

        // samples owned by this lane: S consecutive in raster order of the TB
        const int nn = n * n;
        const int S = nn >= 64 ? (nn >> 6) : 1;
        const bool own = lane * S < nn;
        const int sidx = lane * S;
        const int sy = sidx >> log2, sx = sidx & (n - 1);

        // residual (prefetched before the reference-sample work)
        int res[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) res[i] = 0;
        const bool coded = tb.flags & (P265R_TB_CBF | P265R_TB_PCM);
        if (coded && own) {
            // residuals come from the residual phase, raw levels (bypass / PCM) from the pool
            const int16_t* rp = ((tb.flags & (P265R_TB_BYPASS | P265R_TB_PCM)) ? pool : resid) + tb.coef_off + sidx;
            if (S == 16) {
                const uint4 a = *reinterpret_cast<const uint4*>(rp);
                const uint4 b = *reinterpret_cast<const uint4*>(rp + 8);
                const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                for (int i = 0; i < 16; ++i) res[i] = (int)(int16_t)(w[i >> 1] >> ((i & 1) * 16));
            } else if (S == 4) {
                const uint2 a = *reinterpret_cast<const uint2*>(rp);
                res[0] = (int)(int16_t)(a.x & 0xffff); res[1] = (int)(int16_t)(a.x >> 16);
                res[2] = (int)(int16_t)(a.y & 0xffff); res[3] = (int)(int16_t)(a.y >> 16);
            } else {
                res[0] = rp[0];
            }
        }

        int pred[16];
        if (tb.flags & P265R_TB_PCM) {
#pragma unroll
            for (int i = 0; i < 16; ++i) pred[i] = 0;
        } else {
            // ---- reference samples in linear order k = 0..4n --------------------
            const int nref = 4 * n + 1;
            int val[3];
            bool av[3];
            const int xcl = xr << sub, ycl = yr << sub;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int k = lane + 64 * j;
                val[j] = 0;
                av[j] = false;
                if (k < nref) {
                    const int dx = k < 2 * n ? -1 : (k == 2 * n ? -1 : k - 2 * n - 1);
                    const int dy = k < 2 * n ? 2 * n - 1 - k : -1;
                    const int xn = xr + dx, yn = yr + dy;
                    av[j] = nb_available(xn << sub, yn << sub, xcl, ycl, x0, y0, g, ctb, flags);
                    if (av[j]) {
                        val[j] = yn < 0 ? top[xn + 1] : (xn < 0 ? left[yn] : interior[yn * ist + xn]);
                    }
                    L.ref[0][k] = (uint16_t)val[j];
                }
            }
            const unsigned long long m0 = __ballot(av[0]);
            const unsigned long long m1 = __ballot(av[1]);
            const unsigned long long m2 = __ballot(av[2]);
            __syncthreads();
            // ---- substitution (8.4.4.2.2) -----------------------------------------
            const bool any = (m0 | m1 | m2) != 0ull;
            const int first = m0 ? __ffsll((long long)m0) - 1
                                 : (m1 ? 64 + __ffsll((long long)m1) - 1 : 128 + __ffsll((long long)m2) - 1);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int k = lane + 64 * j;
                if (k < nref && !av[j]) {
                    int src = -1;
                    const unsigned long long mk[3] = {m0, m1, m2};
                    const unsigned long long below = lane ? (mk[j] & ((1ull << lane) - 1ull)) : 0ull;
                    if (below) src = 64 * j + 63 - __clzll((long long)below);
                    else if (j >= 2 && m1) src = 64 + 63 - __clzll((long long)m1);
                    else if (j >= 1 && m0) src = 63 - __clzll((long long)m0);
                    if (src < 0) src = first;
                    val[j] = any ? (int)L.ref[0][src] : (1 << (bd - 1));
                }
            }
            __syncthreads();
            const int mode = tb.pred_mode;
            // ---- filtering (8.4.4.2.3), luma only ---------------------------------
            bool filt = false;
            if (c == 0 && mode != 1 && n != 4) {
                const int dist = min(abs(mode - 26), abs(mode - 10));
                const int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
                filt = dist > thr;
            }
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int k = lane + 64 * j;
                if (k < nref) L.ref[0][k] = (uint16_t)val[j];
            }
            __syncthreads();
            const uint16_t* R = L.ref[0];
            if (filt) {
                const int corner = R[2 * n], bl = R[0], tr = R[4 * n];
                const bool strong = g.strong && n == 32 &&
                                    abs(corner + tr - 2 * (int)R[3 * n]) < (1 << (bd - 5)) &&
                                    abs(corner + bl - 2 * (int)R[n]) < (1 << (bd - 5));
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int k = lane + 64 * j;
                    if (k < nref) {
                        int f;
                        if (k == 0 || k == 4 * n) f = R[k];
                        else if (strong) {
                            f = k == 2 * n ? corner
                              : (k < 2 * n ? ((63 - (2 * n - 1 - k)) * corner + (2 * n - k) * bl + 32) >> 6
                                           : ((63 - (k - 2 * n - 1)) * corner + (k - 2 * n) * tr + 32) >> 6);
                        } else f = (R[k - 1] + 2 * R[k] + R[k + 1] + 2) >> 2;
                        L.ref[1][k] = (uint16_t)f;
                    }
                }
                __syncthreads();
                R = L.ref[1];
            }
            // ---- prediction (8.4.4.2.4-6) -----------------------------------------
            if (mode == 0) {
                const int trs = R[3 * n + 1], bls = R[n - 1];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (i < S) {
                        const int x = sx + i, y = sy;
                        pred[i] = ((n - 1 - x) * R[2 * n - 1 - y] + (x + 1) * trs + (n - 1 - y) * R[2 * n + 1 + x] +
                                   (y + 1) * bls + n) >> (log2 + 1);
                    }
                }
            } else if (mode == 1) {
                int s = 0;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int k = lane + 64 * j;
                    if ((k >= n && k < 2 * n) || (k > 2 * n && k <= 3 * n)) s += val[j];
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                const int dc = (s + n) >> (log2 + 1);
                const bool edge = c == 0 && n < 32;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (i < S) {
                        const int x = sx + i, y = sy;
                        int v = dc;
                        if (edge) {
                            if (x == 0 && y == 0) v = (R[2 * n - 1] + 2 * dc + R[2 * n + 1] + 2) >> 2;
                            else if (y == 0) v = (R[2 * n + 1 + x] + 3 * dc + 2) >> 2;
                            else if (x == 0) v = (R[2 * n - 1 - y] + 3 * dc + 2) >> 2;
                        }
                        pred[i] = v;
                    }
                }
            } else {
                const int ang = c_angle[mode];
                const int inv = c_inv_angle[mode];
                const bool vert = mode >= 18;
                const int dir = vert ? 1 : -1;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (i < S) {
                        const int x = sx + i, y = sy;
                        const int a = vert ? y : x, b = vert ? x : y;
                        const int idx = ((a + 1) * ang) >> 5, fact = ((a + 1) * ang) & 31;
                        const int r0 = b + idx + 1;
                        const int k0 = r0 >= 0 ? 2 * n + dir * r0 : 2 * n - dir * ((r0 * inv + 128) >> 8);
                        int v = R[k0];
                        if (fact) {
                            const int r1 = r0 + 1;
                            const int k1 = r1 >= 0 ? 2 * n + dir * r1 : 2 * n - dir * ((r1 * inv + 128) >> 8);
                            v = ((32 - fact) * v + fact * (int)R[k1] + 16) >> 5;
                        }
                        if (c == 0 && n < 32) {
                            if (mode == 26 && x == 0) v = min(max((int)R[2 * n + 1] + (((int)R[2 * n - 1 - y] - (int)R[2 * n]) >> 1), 0), maxv);
                            if (mode == 10 && y == 0) v = min(max((int)R[2 * n - 1] + (((int)R[2 * n + 1 + x] - (int)R[2 * n]) >> 1), 0), maxv);
                        }
                        pred[i] = v;
                    }
                }
            }
        }
        // ---- reconstruction: Clip1(pred + res) into the CTU's LDS image ------------
        if (own && sizeof(T) == 2) {
            T* dst = interior + (yr + sy) * ist + xr + sx;
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (i < S) dst[i] = (T)min(max(pred[i] + res[i], 0), maxv);
        } else if (own) {
            uint8_t* dst = reinterpret_cast<uint8_t*>(interior + (yr + sy) * ist + xr + sx);
            if (S == 16) {
                uint32_t w[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t v = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        v |= (uint32_t)min(max(pred[q * 4 + b] + res[q * 4 + b], 0), maxv) << (8 * b);
                    w[q] = v;
                }
                *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
            } else if (S == 4) {
                uint32_t v = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) v |= (uint32_t)min(max(pred[b] + res[b], 0), maxv) << (8 * b);
                *reinterpret_cast<uint32_t*>(dst) = v;
            } else {
                dst[0] = (uint8_t)min(max(pred[0] + res[0], 0), maxv);
            }
        }
        (void)cs;
        __syncthreads();
    }

    // ---- write the CTU back to the picture planes (clipped to the picture) -----------
    for (int c = 0; c < 3; ++c) {
        const int sub = c ? 1 : 0;
        const int cs = ctb >> sub;
        const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
        const int xb = x0 >> sub, yb = y0 >> sub;
        const int wv = min(cs, W - xb), hv = min(cs, H - yb);
        const T* src = c ? L.c[c - 1] : L.y;
        const int ist = c ? 32 : 64;
        T* plane = reinterpret_cast<T*>(P.rec[c]);
        const int st = (c ? g.stride[1] : g.stride[0]);
        // 4-sample granules (plane widths are multiples of 4: MinCbSize >= 8): 4 or 8 bytes
        typedef typename std::conditional<sizeof(T) == 1, uint32_t, uint2>::type G4;
        const int gpr = wv >> 2;
        for (int e = lane; e < gpr * hv; e += 64) {
            const int yy = e / gpr, xx = (e - yy * gpr) << 2;
            *reinterpret_cast<G4*>(plane + (size_t)(yb + yy) * st + xb + xx) =
                *reinterpret_cast<const G4*>(src + yy * ist + xx);
        }
    }
}

}  // namespace p265r
