// Intra prediction + reconstruction, CU-local wavefront ("row pipeline") schedule.
//
// One workgroup owns whole pictures: its W waves pull CTU ROWS from an LDS row queue
// (pictures of the workgroup in order, rows top to bottom) and walk each row left to
// right.  Row r may start CTU cx once row r-1 has finished CTU min(cx+2, wc) - the
// 2-CTU lag that makes the left, top-left, top and top-right CTUs available.  The
// queue runs across picture boundaries, so waves never idle at a picture's ramp-down;
// picture slots (line buffers + progress words) are reused only after the slot's
// previous picture has completed every row.
//
// All neighbour data lives in LDS: the row above comes from a per-picture, per-row-
// parity LINE BUFFER (bottom sample row of every finished CTU), the column on the left
// is the wave's own previous CTU.  Nothing is re-read from HBM and no cross-CU
// hand-off exists, so the only synchronisation is one LDS progress word per row
// (workgroup-scope release/acquire).  Per transform block the wave does three LDS
// round trips (gather, substitute+filter, predict+reconstruct) with wave-local
// ordering only; the TB record comes from a VGPR (v_readlane) and its residual was
// fetched while the previous TB was being processed.
//
// Same per-TB arithmetic as intra.h (8.4.4.2.x, 8.6.7); replaces decoder/intra.py:24-305
// and decoder/reconstruction.py:4-27 driven by decoder/cu.py:595-615.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"

extern "C" __device__ int __ockl_wfred_add_i32(int);

namespace p265r {

#define P265R_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const P265R_GLOBAL T* gptr(const T* p) { return (const P265R_GLOBAL T*)p; }
template <typename T>
__device__ __forceinline__ P265R_GLOBAL T* gptr_w(T* p) { return (P265R_GLOBAL T*)p; }
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld16(const void* p) {
    const u32x4_t v = *reinterpret_cast<const P265R_GLOBAL u32x4_t*>(gptr(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
// make every 32-bit word of a (wave-uniform) struct provably uniform: SGPRs, scalar branches
template <typename T>
__device__ __forceinline__ T uniform(const T& v) {
    static_assert(sizeof(T) % 4 == 0, "32-bit granules");
    uint32_t w[sizeof(T) / 4];
    __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w[i] = __builtin_amdgcn_readfirstlane(w[i]);
    T o;
    __builtin_memcpy(&o, w, sizeof(T));
    return o;
}
// copy a POD struct out of global memory with global (not flat) loads
template <typename T>
__device__ __forceinline__ T gload(const T* p) {
    static_assert(sizeof(T) % 8 == 0, "8-byte granules");
    const P265R_GLOBAL u32x2_t* q = reinterpret_cast<const P265R_GLOBAL u32x2_t*>(gptr(p));
    u32x2_t tmp[sizeof(T) / 8];
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 8); ++i) tmp[i] = q[i];
    T v;
    __builtin_memcpy(&v, tmp, sizeof(T));
    return v;
}

struct WaveLds {                 // one wave's private CTU state (6816 B)
    uint8_t  y[64 * 64];         // interior luma, stride 64
    uint8_t  c[2][32 * 32];      // interior chroma, stride 32
    uint8_t  yleft[64];          // right column of the previous CTU of this row
    uint8_t  cleft[2][32];
    uint16_t ref[2][136];        // raw / final linear reference arrays
};

struct RowCtrl {                 // 256 B at the start of dynamic LDS
    int next_row;
    int error;
    int done[32];                // per picture slot: rows completed (monotonic over generations)
    int pad[30];
};
// Dynamic LDS layout: [RowCtrl 256 B][prog: fs x hc ints][W x WaveLds][fs x 2 line buffers]
// prog[slot][cy] = (local picture index & 0xffff) << 16 | CTUs done.

__device__ __forceinline__ void wave_sync() {
    // LDS operations of one wavefront execute in program order; only the compiler
    // must be kept from reordering the cross-lane LDS write -> read pairs.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// index of the value that substitutes linear entry k (8.4.4.2.2), given the
// availability masks of entries 0..63, 64..127, 128 (m0, m1, m2).  -1: none available.
__device__ __forceinline__ int subst_src(int k, unsigned long long m0, unsigned long long m1,
                                         unsigned long long m2) {
    const int j = k >> 6, b = k & 63;
    const unsigned long long mj = j == 0 ? m0 : (j == 1 ? m1 : m2);
    if ((mj >> b) & 1ull) return k;
    const unsigned long long below = b ? (mj & ((1ull << b) - 1ull)) : 0ull;
    if (below) return 64 * j + 63 - __clzll((long long)below);
    if (j >= 2 && m1) return 64 + 63 - __clzll((long long)m1);
    if (j >= 1 && m0) return 63 - __clzll((long long)m0);
    if (m0) return __ffsll((long long)m0) - 1;
    if (m1) return 64 + __ffsll((long long)m1) - 1;
    if (m2) return 128 + __ffsll((long long)m2) - 1;
    return -1;
}

struct CtuCtx {                  // wave-uniform state of the CTU being reconstructed
    int x0, y0, w, h, cw, ctb;
    unsigned flags;              // bit0 L, bit1 T, bit2 TL, bit3 TR available
    int bd_l, bd_c, strong;
};

__device__ __forceinline__ int clip_pel(int v, int maxv) { return min(max(v, 0), maxv); }

// Reconstruct one TB of size 2^LOG2.  tw1 = TB record word 1 (log2 | c | mode | flags),
// (tx, ty) its position; (ra, rb) this lane's residual words (prefetched).
template <int LOG2>
__device__ __forceinline__ void recon_tb(const CtuCtx& X, WaveLds& L, const uint8_t* line_up,
                                        int tx, int ty, int c, int mode, int flags,
                                        uint4 ra, uint4 rb, int lane) {
    constexpr int n = 1 << LOG2;
    constexpr int nn = n * n;
    constexpr int S = nn >= 64 ? nn / 64 : 1;        // samples per lane (raster run)
    constexpr int nref = 4 * n + 1;
    constexpr int NCH = (nref + 63) / 64;
    const int sub = c ? 1 : 0;
    const int xr = tx - (X.x0 >> sub), yr = ty - (X.y0 >> sub);
    const int bd = c ? X.bd_c : X.bd_l;
    const int maxv = (1 << bd) - 1;
    uint8_t* interior = c == 0 ? L.y : (c == 1 ? L.c[0] : L.c[1]);
    const int ist = c ? 32 : 64;
    const uint8_t* top = line_up + (c == 0 ? 0 : (c == 1 ? X.w : X.w + X.cw)) + (X.x0 >> sub);
    const uint8_t* left = c == 0 ? L.yleft : (c == 1 ? L.cleft[0] : L.cleft[1]);
    const bool own = lane * S < nn;
    const int sidx = own ? lane * S : 0;
    const int sy = sidx >> LOG2, sx = sidx & (n - 1);
    // (ra, rb): the two aligned 16-B chunks holding this lane's residual run (see res_addr)
    uint32_t rw[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
    if constexpr (S == 4) {
        const bool hi = sidx & 4;
        rw[0] = hi ? ra.z : ra.x; rw[1] = hi ? ra.w : ra.y;
    } else if constexpr (S == 1) {
        const int e = sidx & 7;
        const uint32_t wd = e < 2 ? ra.x : (e < 4 ? ra.y : (e < 6 ? ra.z : ra.w));
        rw[0] = (e & 1) ? (wd >> 16) : (wd & 0xffffu);
    }
    auto resv = [&](int i) { return (int)(int16_t)(rw[i >> 1] >> ((i & 1) * 16)); };
    uint32_t outw[(S + 3) / 4];
#pragma unroll
    for (int q = 0; q < (S + 3) / 4; ++q) outw[q] = 0;
    auto put = [&](int i, int v) { outw[i >> 2] |= (uint32_t)clip_pel(v + resv(i), maxv) << (8 * (i & 3)); };

    if (flags & P265R_TB_PCM) {
#pragma unroll
        for (int i = 0; i < S; ++i) put(i, 0);
    } else {
        // ---- A: gather raw reference samples + availability (6.4.1) --------------------
        const int xcl = xr << sub, ycl = yr << sub;
        unsigned long long m[3] = {0ull, 0ull, 0ull};
#pragma unroll
        for (int jj = 0; jj < NCH; ++jj) {
            const int k = lane + 64 * jj;
            bool av = false;
            if (k < nref) {
                const int dx = k <= 2 * n ? -1 : k - 2 * n - 1;
                const int dy = k < 2 * n ? 2 * n - 1 - k : -1;
                const int xn = xr + dx, yn = yr + dy;
                av = nb_available_wh(xn << sub, yn << sub, xcl, ycl, X.x0, X.y0, X.w, X.h, X.ctb, X.flags);
                int v = 0;
                if (av) v = yn < 0 ? top[xn] : (xn < 0 ? left[yn] : interior[yn * ist + xn]);
                L.ref[0][k] = (uint16_t)v;
            }
            m[jj] = __ballot(av);
        }
        constexpr unsigned long long full0 = nref >= 64 ? ~0ull : ((1ull << (nref & 63)) - 1ull);
        constexpr unsigned long long full1 = nref >= 128 ? ~0ull : (nref > 64 ? ((1ull << ((nref - 64) & 63)) - 1ull) : 0ull);
        constexpr unsigned long long full2 = nref > 128 ? 1ull : 0ull;
        const bool all = m[0] == full0 && m[1] == full1 && m[2] == full2;
        bool filt = false;
        if (n != 4 && c == 0 && mode != 1) {
            const int dist = min(abs(mode - 26), abs(mode - 10));
            filt = dist > (n == 8 ? 7 : (n == 16 ? 1 : 0));
        }
        wave_sync();
        const uint16_t* R = L.ref[0];
        int dcs = 0;
        if (!all || filt || mode == 1) {
            // ---- B: substitution (8.4.4.2.2) + filtering (8.4.4.2.3) -> ref[1] ------------
            const bool any = (m[0] | m[1] | m[2]) != 0ull;
            const int half = 1 << (bd - 1);
            auto sval = [&](int i) -> int {
                if (all) return (int)L.ref[0][i];
                const int s = subst_src(i, m[0], m[1], m[2]);
                return s < 0 ? half : (int)L.ref[0][s];
            };
            bool strong = false;
            int corner = 0, bl = 0, tr = 0;
            if (n == 32 && filt && X.strong) {
                corner = sval(2 * n); bl = sval(0); tr = sval(4 * n);
                strong = abs(corner + tr - 2 * sval(3 * n)) < (1 << (bd - 5)) &&
                         abs(corner + bl - 2 * sval(n)) < (1 << (bd - 5));
            }
#pragma unroll
            for (int jj = 0; jj < NCH; ++jj) {
                const int k = lane + 64 * jj;
                if (k < nref) {
                    const int sk = any ? sval(k) : half;
                    int f = sk;
                    if (filt && k > 0 && k < 4 * n) {
                        if (strong) {
                            f = k == 2 * n ? corner
                              : (k < 2 * n ? ((63 - (2 * n - 1 - k)) * corner + (2 * n - k) * bl + 32) >> 6
                                           : ((63 - (k - 2 * n - 1)) * corner + (k - 2 * n) * tr + 32) >> 6);
                        } else {
                            f = (sval(k - 1) + 2 * sk + sval(k + 1) + 2) >> 2;
                        }
                    }
                    L.ref[1][k] = (uint16_t)f;
                    if ((k >= n && k < 2 * n) || (k > 2 * n && k <= 3 * n)) dcs += sk;
                }
            }
            wave_sync();
            R = L.ref[1];
        }
        // ---- C: prediction (8.4.4.2.4-6) fused with reconstruction (8.6.7) ----------------
        if (mode == 0) {
            const int trs = R[3 * n + 1], bls = R[n - 1];
            const int ly = R[2 * n - 1 - sy];
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const int x = sx + i;
                put(i, ((n - 1 - x) * ly + (x + 1) * trs + (n - 1 - sy) * R[2 * n + 1 + x] + (sy + 1) * bls + n) >> (LOG2 + 1));
            }
        } else if (mode == 1) {
            const int dc = (__ockl_wfred_add_i32(dcs) + n) >> (LOG2 + 1);
            const bool edge = c == 0 && n < 32;
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const int x = sx + i;
                int v = dc;
                if (edge) {
                    if (x == 0 && sy == 0) v = (R[2 * n - 1] + 2 * dc + R[2 * n + 1] + 2) >> 2;
                    else if (sy == 0) v = (R[2 * n + 1 + x] + 3 * dc + 2) >> 2;
                    else if (x == 0) v = (R[2 * n - 1 - sy] + 3 * dc + 2) >> 2;
                }
                put(i, v);
            }
        } else if (mode >= 18) {                                    // vertical family
            const int ang = c_angle[mode];
            const int inv = c_inv_angle[mode];
            const int idx = ((sy + 1) * ang) >> 5, fact = ((sy + 1) * ang) & 31;
            auto refk = [&](int r) { return r >= 0 ? 2 * n + r : 2 * n - ((r * inv + 128) >> 8); };
            const bool bflt = mode == 26 && c == 0 && n < 32;
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const int x = sx + i;
                const int r0 = x + idx + 1;
                int v = R[refk(r0)];
                if (fact) v = ((32 - fact) * v + fact * (int)R[refk(r0 + 1)] + 16) >> 5;
                if (bflt && x == 0) v = clip_pel((int)R[2 * n + 1] + (((int)R[2 * n - 1 - sy] - (int)R[2 * n]) >> 1), maxv);
                put(i, v);
            }
        } else {                                                    // horizontal family
            const int ang = c_angle[mode];
            const int inv = c_inv_angle[mode];
            auto refk = [&](int r) { return r >= 0 ? 2 * n - r : 2 * n + ((r * inv + 128) >> 8); };
            const bool bflt = mode == 10 && c == 0 && n < 32 && sy == 0;
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const int x = sx + i;
                const int idx = ((x + 1) * ang) >> 5, fact = ((x + 1) * ang) & 31;
                const int r0 = sy + idx + 1;
                int v = R[refk(r0)];
                if (fact) v = ((32 - fact) * v + fact * (int)R[refk(r0 + 1)] + 16) >> 5;
                if (bflt) v = clip_pel((int)R[2 * n - 1] + (((int)R[2 * n + 1 + x] - (int)R[2 * n]) >> 1), maxv);
                put(i, v);
            }
        }
    }
    if (own) {
        uint8_t* dst = interior + (yr + sy) * ist + xr + sx;
        if constexpr (S == 16) *reinterpret_cast<uint4*>(dst) = make_uint4(outw[0], outw[1], outw[2], outw[3]);
        else if constexpr (S == 4) *reinterpret_cast<uint32_t*>(dst) = outw[0];
        else dst[0] = (uint8_t)outw[0];
    }
    wave_sync();
}

template <int W>
__global__ __launch_bounds__(64 * W) void intra_rows_kernel(const DevPic* __restrict__ pics,
                                                           const int16_t* __restrict__ pool,
                                                           const int16_t* __restrict__ resid,
                                                           Geo g, int n_pics, int fs_count,
                                                           int* __restrict__ err_flag,
                                                           int* __restrict__ dbg) {
    // debug trace (P265R_DEBUG_SYNC=1): host-mapped words, one per wave
#if defined(P265R_DBG_NOTRACE)
#define P265R_TRACE(code) do { } while (0)
#else
#define P265R_TRACE(code) do { if (dbg && lane == 0) __hip_atomic_store(dbg + blockIdx.x * W + wave, (code), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#endif
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    RowCtrl& ctl = *reinterpret_cast<RowCtrl*>(smem);
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int prog_bytes = (fs_count * g.hc * 4 + 15) & ~15;
    int* prog = reinterpret_cast<int*>(smem + 256);
    WaveLds& L = reinterpret_cast<WaveLds*>(smem + 256 + prog_bytes)[wave];
    const int line_bytes = g.w + 2 * g.cw;            // Y | Cb | Cr bottom sample rows
    unsigned char* lines = smem + 256 + prog_bytes + W * sizeof(WaveLds);

    if (threadIdx.x == 0) { ctl.next_row = 0; ctl.error = 0; }
    if (threadIdx.x < 32) ctl.done[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < fs_count * g.hc; i += 64 * W) prog[i] = -1;
    __syncthreads();

    const int G = gridDim.x;
    const int b = blockIdx.x;
    const int n_my = b < n_pics ? (n_pics - b + G - 1) / G : 0;
    const int rows_total = n_my * g.hc;
    const int ctb = 1 << g.ctb_log2;
    // bounded spin-wait on an LDS word; false = gave up (error published, caller bails out).
    // Every condition is made wave-uniform (readfirstlane) so the loops are scalar loops.
    long long t_wait = 0;
    const long long t_begin = __builtin_amdgcn_s_memtime();
    auto wait_until = [&](auto ready) -> bool {
        const long long t0 = __builtin_amdgcn_s_memtime();
        for (int spins = 0; spins < (1 << 24); ++spins) {
            if (spins == 0 && __builtin_amdgcn_readfirstlane((int)ready())) return true;
            if (__builtin_amdgcn_readfirstlane((int)ready())) { t_wait += __builtin_amdgcn_s_memtime() - t0; return true; }
            if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&ctl.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
                return false;
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(&ctl.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   // all lanes, same value
        atomicOr(err_flag, 1);
        return false;                                       // never hang the GPU
    };
    bool failed = false;

    P265R_TRACE(1);
    for (;;) {
        // row queue: the whole wave executes the atomic (no lane-0 branch inside the loop);
        // only lane 0 contributes, so the wave takes exactly one row
        int r = __hip_atomic_fetch_add(&ctl.next_row, lane == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        r = __builtin_amdgcn_readfirstlane(r);
        if (r >= rows_total || failed) break;
        P265R_TRACE(2 | (r << 8));
        const int j = r / g.hc, cy = r - j * g.hc;
        const int slot = j % fs_count, gen = j / fs_count;
        const DevPic P = uniform(gload(pics + b + j * G));
        // picture slot reuse: every row of picture j waits until picture j - fs_count (the
        // slot's previous occupant) has completed all its rows; those rows were dequeued
        // earlier and are held by running waves, so this wait always ends.
        if (!wait_until([&] {
                return __hip_atomic_load(&ctl.done[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= gen * g.hc;
            })) { failed = true; break; }
        P265R_TRACE(3 | (r << 8));
        unsigned char* line_cur = lines + (size_t)(slot * 2 + (cy & 1)) * line_bytes;
        const unsigned char* line_up = lines + (size_t)(slot * 2 + ((cy & 1) ^ 1)) * line_bytes;
        int* my_prog = &prog[slot * g.hc + cy];
        const int* up_prog = &prog[slot * g.hc + (cy > 0 ? cy - 1 : 0)];
        const int tag = (j & 0xffff) << 16;
        __hip_atomic_store(my_prog, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const p265r_ctu* ctus = P.ctus;

        for (int cx = 0; cx < g.wc; ++cx) {
            // ---- wait for the row above (2-CTU lag) -------------------------------------
            if (cy > 0) {
                const int need = min(cx + 2, g.wc);
                if (!wait_until([&] {
                        const int v = __hip_atomic_load(up_prog, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        return (v & 0xffff0000) == tag && (v & 0xffff) >= need;
                    })) { failed = true; break; }
            }
            P265R_TRACE(4 | (cx << 8) | (r << 16));
            CtuCtx X;
            X.x0 = cx << g.ctb_log2; X.y0 = cy << g.ctb_log2;
            X.w = g.w; X.h = g.h; X.cw = g.cw; X.ctb = ctb;
            X.bd_l = g.bd[0]; X.bd_c = g.bd[1]; X.strong = g.strong;
            const int addr = cy * g.wc + cx;
            // the CTU and its four causal neighbours: five independent loads, one wait
            const p265r_ctu me = uniform(gload(ctus + addr));
            const p265r_ctu nl = uniform(gload(ctus + (cx > 0 ? addr - 1 : addr)));
            const p265r_ctu nt_ = uniform(gload(ctus + (cy > 0 ? addr - g.wc : addr)));
            const p265r_ctu ntl = uniform(gload(ctus + (cx > 0 && cy > 0 ? addr - g.wc - 1 : addr)));
            const p265r_ctu ntr = uniform(gload(ctus + (cx + 1 < g.wc && cy > 0 ? addr - g.wc + 1 : addr)));
            unsigned flags = 0;
            if (cx > 0 && ctu_same_region(me, nl)) flags |= 1u;
            if (cy > 0 && ctu_same_region(me, nt_)) flags |= 2u;
            if (cx > 0 && cy > 0 && ctu_same_region(me, ntl)) flags |= 4u;
            if (cx + 1 < g.wc && cy > 0 && ctu_same_region(me, ntr)) flags |= 8u;
            X.flags = flags;

            const int nt = me.tb_count;
            const uint4* trec = reinterpret_cast<const uint4*>(P.tbs + me.tb_begin);
            uint4 rec = make_uint4(0, 0, 0, 0);
            if (lane < nt) rec = ld16(trec + lane);

            // residual of TB t: always two aligned 16-B loads per lane (fixed shape, so the
            // compiler's vmcnt bookkeeping stays exact; pools are padded by 64 B), issued
            // while TB t-1 is processed.  TB offsets are multiples of 16 elements.
            auto res_addr = [&](uint32_t w1, uint32_t off) {
                const int lg = (int)(w1 & 0xff), fl = (int)(w1 >> 24);
                const int nn = 1 << (2 * lg);
                const int S = nn >= 64 ? (nn >> 6) : 1;
                const int sidx = lane * S < nn ? lane * S : 0;
                const int16_t* base = (fl & (P265R_TB_BYPASS | P265R_TB_PCM)) ? pool : resid;
                return reinterpret_cast<const uint4*>(base + off + (sidx & ~7));
            };
            uint32_t w0n = 0, w1n = 0, w3n = 0;
            uint4 ra = make_uint4(0, 0, 0, 0), rb = ra;
            if (nt) {
                w0n = __builtin_amdgcn_readlane(rec.x, 0);
                w1n = __builtin_amdgcn_readlane(rec.y, 0);
                w3n = __builtin_amdgcn_readlane(rec.w, 0);
                const uint4* a = res_addr(w1n, w3n);
                ra = ld16(a); rb = ld16(a + 1);
            }
            for (int t = 0; t < nt; ++t) {
                const uint32_t w0 = w0n, w1 = w1n;
                const uint4 ca = ra, cb = rb;
                const bool coded = (w1 >> 24) & (P265R_TB_CBF | P265R_TB_PCM);
                if (t + 1 < nt) {
                    const int l = (t + 1) & 63;
                    if (l == 0) {
                        if (t + 1 + lane < nt) rec = ld16(trec + t + 1 + lane);
                        else rec = make_uint4(0, 0, 0, 0);
                    }
                    w0n = __builtin_amdgcn_readlane(rec.x, l);
                    w1n = __builtin_amdgcn_readlane(rec.y, l);
                    w3n = __builtin_amdgcn_readlane(rec.w, l);
                    const uint4* a = res_addr(w1n, w3n);
                    ra = ld16(a); rb = ld16(a + 1);
                }
                const uint4 za = coded ? ca : make_uint4(0, 0, 0, 0);
                const uint4 zb = coded ? cb : make_uint4(0, 0, 0, 0);
                const int tx = (int)(w0 & 0xffff), ty = (int)(w0 >> 16);
                const int lg = (int)(w1 & 0xff), c = (int)((w1 >> 8) & 0xff);
                const int mode = (int)((w1 >> 16) & 0xff), fl = (int)(w1 >> 24);
                switch (lg) {
                    case 2: recon_tb<2>(X, L, line_up, tx, ty, c, mode, fl, za, zb, lane); break;
                    case 3: recon_tb<3>(X, L, line_up, tx, ty, c, mode, fl, za, zb, lane); break;
                    case 4: recon_tb<4>(X, L, line_up, tx, ty, c, mode, fl, za, zb, lane); break;
                    default: recon_tb<5>(X, L, line_up, tx, ty, c, mode, fl, za, zb, lane); break;
                }
            }

            P265R_TRACE(5 | (cx << 8) | (r << 16));
            // ---- publish the CTU: planes (HBM), bottom line (LDS), right column (LDS) ----------
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int sub = c ? 1 : 0;
                const int cs = ctb >> sub;
                const int Wd = c ? g.cw : g.w, Ht = c ? g.ch : g.h;
                const int xb = X.x0 >> sub, yb = X.y0 >> sub;
                const int wv = min(cs, Wd - xb), hv = min(cs, Ht - yb);
                const uint8_t* src = c == 0 ? L.y : (c == 1 ? L.c[0] : L.c[1]);
                const int ist = c ? 32 : 64;
                P265R_GLOBAL uint8_t* plane = gptr_w(P.rec[c]);
                const int st = g.stride[c];
                const int gpr = wv >> 2;
                for (int e = lane; e < gpr * hv; e += 64) {
                    const int yy = e / gpr, xx = (e - yy * gpr) << 2;
                    *reinterpret_cast<P265R_GLOBAL uint32_t*>(plane + (size_t)(yb + yy) * st + xb + xx) =
                        *reinterpret_cast<const uint32_t*>(src + yy * ist + xx);
                }
                unsigned char* lc = line_cur + (c == 0 ? 0 : (c == 1 ? g.w : g.w + g.cw)) + xb;
                if (lane < wv) lc[lane] = src[(hv - 1) * ist + lane];
                uint8_t* lf = c == 0 ? L.yleft : (c == 1 ? L.cleft[0] : L.cleft[1]);
                if (lane < hv) lf[lane] = src[lane * ist + wv - 1];
            }
            __hip_atomic_store(my_prog, tag | (cx + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            wave_sync();
        }
        if (failed) break;
        __hip_atomic_fetch_add(&ctl.done[slot], lane == 0 ? 1 : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        P265R_TRACE(6 | (r << 8));
    }
    P265R_TRACE(7);
    if (dbg) {   // debug statistics: [total cycles, cycles in dependency waits] per wave
        const long long t_all = __builtin_amdgcn_s_memtime() - t_begin;
        const int slotw = gridDim.x * W + 2 * (blockIdx.x * W + wave);
        __hip_atomic_store(dbg + slotw, (int)(t_all >> 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dbg + slotw + 1, (int)(t_wait >> 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // all stores of this wave are issued before it ends (compiler barrier)
    asm volatile("" ::: "memory");
}

}  // namespace p265r
