// Intra prediction + reconstruction, CU-local wavefront ("row pipeline") schedule.
//
// One workgroup owns whole pictures: its W waves pull CTU ROW UNITS from an LDS row queue
// (pictures of the workgroup in order, rows top to bottom; every CTU row is two units, the
// luma chain and the chroma (Cb + Cr) chain, which 4:2:0 intra prediction never couples)
// and walk each unit left to right.  Row r may start CTU cx once row r-1 has finished CTU min(cx+2, wc) - the
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
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"
#include "intra_prep.h"

namespace p265r {

// s_sleep argument between two polls of a row-kernel dependency wait
#ifndef P265R_SPIN_SLEEP
#define P265R_SPIN_SLEEP 8
#endif

// SGPR bases of the job loop (LDS base, angle tables, Cb line) behind opaque s_mov copies per job (1, A/B),
// or left to the compiler (0: round 5, with 24-B job records, 5.26-5.27 vs 5.30 ms per pipelined step)
#ifndef P265R_OPAQUE_S
#define P265R_OPAQUE_S 0
#endif

// intraPredAngle 0 (modes 10 / 26) as plain copies in the fast paths (0 = the generic angular code)
#ifndef P265R_HV_FAST
#define P265R_HV_FAST 1
#endif

#ifdef P265R_ISA_MARK                    // tools/isa.sh: comment markers in the device assembly
#define P265R_MARK(x) asm volatile("; MARK " x)
#else
#define P265R_MARK(x) do { } while (0)
#endif
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
__device__ __forceinline__ uint2 ld8(const void* p) {
    const u32x2_t v = *reinterpret_cast<const P265R_GLOBAL u32x2_t*>(gptr(p));
    return make_uint2(v.x, v.y);
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

// generic pointer to the LDS byte at 32-bit LDS address a
__device__ __forceinline__ void* lds_ptr(uint32_t a) {
    return (void*)(__attribute__((address_space(3))) void*)(uintptr_t)a;
}
// LDS-typed pointers straight from a 32-bit LDS address: no generic round trip, so no
// null-pointer remapping (v_cmp + v_cndmask per cast) in the fast paths
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ lds_u8* lds8(uint32_t a) { return (lds_u8*)(uintptr_t)a; }
__device__ __forceinline__ lds_u32* lds32(uint32_t a) { return (lds_u32*)(uintptr_t)a; }
// sample T (uint8_t, uint16_t for BitDepth 9..10, int16_t for 11..12) at SAMPLE address s (byte address s * sizeof(T)): the
// job functions compute their LDS addresses in sample units, so one formula serves both sample sizes
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T* ldsT(uint32_t s) {
    return (__attribute__((address_space(3))) T*)(uintptr_t)(s * (uint32_t)sizeof(T));
}

// Packed Cb | Cr << 16 arithmetic of the chroma jobs: w x both halves.  8-bit samples packed at 16-bit
// spacing stay below 2^24, so one v_mul_u32_u24 weighs both; 10-bit ones do not, and take the packed
// 16-bit multiply (every weighted sum of the chroma predictors stays below 2^16 per half at 10 bits too)
template <typename T>
__device__ __forceinline__ uint32_t pmul(uint32_t w, uint32_t packed) {
    if constexpr (sizeof(T) == 1) {
        return __umul24(w, packed);
    } else {
        uint32_t r;
        asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(w * 0x00010001u), "v"(packed));
        return r;
    }
}

// Packed angular interpolation ((32 - f) a + f b + 16) >> 5 of a Cb | Cr pair (wa + wb = 32).  BitDepth 11-12
// (sample type int16_t, the row kernel's tag for them) passes 16 bits per half (32 x 4095), so each sample is
// split into 6-bit halves a = 64 ah + al: the result is 2 (wa ah + wb bh) + ((wa al + wb bl + 16) >> 5)
// exactly (64 X is a multiple of 32), every partial sum below 2^12 per half.
template <typename T>
__device__ __forceinline__ uint32_t pang(uint32_t wa, uint32_t a, uint32_t wb, uint32_t b) {
    if constexpr (std::is_same<T, int16_t>::value) {
        const uint32_t hi = pmul<T>(wa, (a >> 6) & 0x003f003fu) + pmul<T>(wb, (b >> 6) & 0x003f003fu);
        const uint32_t lo = pmul<T>(wa, a & 0x003f003fu) + pmul<T>(wb, b & 0x003f003fu) + 0x00100010u;
        return (hi << 1) + ((lo >> 5) & 0x003f003fu);
    } else {
        return ((pmul<T>(wa, a) + pmul<T>(wb, b) + 0x00100010u) >> 5) & 0x07ff07ffu;
    }
}

// Signed 24-bit product (both |operands| < 2^23): the projected-reference index r * invAngle
// (8.4.4.2.6), which LLVM otherwise widens to a quarter-rate v_mul_lo_u32 once it knows both
// factors are negative.  b is wave-uniform (invAngle of the job's mode) and goes in an SGPR.
__device__ __forceinline__ int mul_i24(int a, int b) {
    int r;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "s"(b), "v"(a));
    return r;
}

// Angular reference index (8.4.4.2.6) in the linear order of 8.4.4.2.2 (left column reversed at
// 0..2n-1, corner 2n, top row 2n+1..4n) of projection position r:
//   idx = 2n + s * (r >= 0 ? r : -((r * invAngle + 128) >> 8)),  s = +1 vertical, -1 horizontal.
// With nr = -r and ia = |invAngle| (>= 256 for every negative intraPredAngle; 256 stands in for
// the modes without one, ang_inv), the bracket equals -max(nr, (nr * ia + 128) >> 8) for EVERY r
// (r >= 0: the product rounds to <= -r; r < 0: it rounds to >= |r|), so the index needs no
// per-lane select on the sign of r: idx = 2n + ns * max(...), ns = -s (wave-uniform).
template <int TWO_N>
__device__ __forceinline__ int ang_ref(int nr, int ia, int ns) {
    const int q = (mul_i24(nr, ia) + 128) >> 8;
    int r;   // TWO_N + ns * max(nr, q) in one v_mad_i32_i24 (LLVM widens ns * x to v_mul_lo_u32: |ns| = 1)
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "s"(ns), "v"(max(nr, q)), "i"(TWO_N));
    return r;
}
// |invAngle| of job word w1 / angtab bits [8,21), 256 for the modes without an inverse angle
__device__ __forceinline__ int ang_inv(uint32_t angw) {
    return (int)((angw >> 8) & 0x1fffu);      // the angle tables store 256 for the modes without one
}

// AngTab4: the 4x4 angular table in LDS (35 modes x 16 samples, one dword each; modes 0 / 1 zero).
// Entry of mode m, sample (x, y) of a 4x4 block: byte 0 / 1 = 4 x the linear reference index of
// the two samples 8.4.4.2.6 interpolates (ds_bpermute byte addresses), byte 2 = iFact, byte 3 =
// 32 - iFact.  Quad stages read their sample's entry with the stage's gather, so an angular stage
// costs two bpermutes and the weighting instead of the projection arithmetic.
// AngTab8 (P265R_ANGTAB8): the same for 8x8 blocks (35 x 64 dwords), read by the fast luma 8x8
// and Cb+Cr 8x8 jobs.
#ifndef P265R_ANGTAB8
#define P265R_ANGTAB8 1
#endif
constexpr int kAngTab4Bytes = 35 * 16 * 4;
constexpr int kAngTab8Bytes = P265R_ANGTAB8 ? 35 * 64 * 4 : 0;
constexpr int kAngTabBytes = kAngTab4Bytes + kAngTab8Bytes;
template <int LOG2>
__device__ __forceinline__ uint32_t angtab_entry(int m, int p) {
    constexpr int n = 1 << LOG2;
    if (m < 2) return 0u;
    const int x = p & (n - 1), y = p >> LOG2;
    const int ang = c_angle[m];
    const int ia = c_inv_angle[m] ? -(int)c_inv_angle[m] : 256;
    const bool vert = m >= 18;
    const int ns = vert ? -1 : 1;
    const int along = vert ? y : x, across = vert ? x : y;
    const int pa = (along + 1) * ang;
    const int idx = pa >> 5, fact = pa & 31;
    const int nr0 = -1 - across - idx;
    auto ref = [&](int nr) { return 2 * n + ns * max(nr, (nr * ia + 128) >> 8); };   // ang_ref<2n>
    const uint32_t a = (uint32_t)(ref(nr0) * 4) & 0xffu, b = (uint32_t)(ref(nr0 - 1) * 4) & 0xffu;
    return a | b << 8 | (uint32_t)fact << 16 | (uint32_t)(32 - fact) << 24;
}

template <typename T>            // sample type: uint8_t (BitDepth 8), uint16_t (9..10), int16_t (11..12: a tag, pang)
struct WaveLdsT {                // one wave's private CTU state (4564 B at 8 bits): a wave holds one row
    T        ref[2][136];        // unit at a time, luma OR chroma, so their areas overlap
    union {                      // ref: raw / final linear reference arrays
        struct {
            T y[64 * 64];                // interior luma, stride 64
            T yleft[64];                 // right column of the previous CTU of this row
            T ytop[sizeof(T) == 1 ? 132 : 136];   // XG: the row above, [4 + x] for x = -4 .. 2 CTB - 1
                                                  // (16-bit: padded so consecutive waves stay 16-B aligned)
        };
        struct {
            T c[2][32 * 32];             // interior chroma, stride 32
            T cleft[2][32];
            T ctop[2][68];               // XG: per plane as ytop
        };
    };
};
using WaveLds = WaveLdsT<uint8_t>;
// timing experiment (wrong output): every residual load of the row kernel inside one 8-KB window
#ifdef P265R_RES_FAKE
#define P265R_RI(x) ((x) & 4095)
#else
#define P265R_RI(x) (x)
#endif
#ifndef P265R_XG_SLEEP
#define P265R_XG_SLEEP 8                 // s_sleep between the cross-group kernel's progress polls (A/B knob)
#endif
#ifndef P265R_XG_PRE
#define P265R_XG_PRE 0                   // XG: the next CTU's first residual fetched at the publish (A/B knob)
#endif
#ifndef P265R_PIPE_PRIO
#define P265R_PIPE_PRIO 0                // A/B: s_setprio of the pipelined (W = 8) row kernel's waves
#endif
#ifndef P265R_LATE_REC
#define P265R_LATE_REC 0                 // 1: the next job's record read after the job (A/B: slower)
#endif
#ifndef P265R_QUAD_COMPOSED
#define P265R_QUAD_COMPOSED 0            // A/B: composed quad-stage references in the cross-group kernel (quad_stage_c):
                                         // parity green, C5 intra 2.11-2.14 -> 2.31-2.34 ms (3 reps): not kept
#endif
#ifndef P265R_TR_DEFER
#define P265R_TR_DEFER 1                 // 0: wait for the top-right CTU before the CTU starts (A/B knob)
#endif
// job word w0 addresses a TB origin as yr * 64 + xr (luma) or 4096 + yr * 32 + xr (chroma,
// intra_prep.h); WaveLds sample of that origin = w0 offset + kOrg[chroma] (sample units: bytes at 8 bits)
template <typename T> constexpr uint32_t kOrgLT = (uint32_t)(offsetof(WaveLdsT<T>, y) / sizeof(T));
template <typename T> constexpr uint32_t kOrgCT = (uint32_t)(offsetof(WaveLdsT<T>, c) / sizeof(T)) - 4096u;
template <typename T> constexpr uint32_t kRefT = (uint32_t)(offsetof(WaveLdsT<T>, ref) / sizeof(T));
template <typename T> constexpr uint32_t kYLeftT = (uint32_t)(offsetof(WaveLdsT<T>, yleft) / sizeof(T));
template <typename T> constexpr uint32_t kCLeftT = (uint32_t)(offsetof(WaveLdsT<T>, cleft) / sizeof(T));
constexpr uint32_t kOrgL = kOrgLT<uint8_t>;
constexpr uint32_t kOrgC = kOrgCT<uint8_t>;

struct RowCtrl {                 // 256 B at the start of dynamic LDS
    int next_row;
    int error;
    int done[32];                // per picture slot: rows completed (monotonic over generations)
    int cu_slot;                 // this workgroup's per-CU slot (Geo::fair) and its rank there
    int cu_rank;
    int pad[28];
};

// Fair sharing of a CU between the row kernel's workgroups (Geo::fair).  Two workgroups share
// each CU; the SIMDs arbitrate vector issue by priority, then age, so the older one runs ahead
// and finishes ~25 % earlier (measured: 11.9 vs 14.9 M cycles per 1080p picture), leaving the CU
// half empty for the younger one's tail.  Each workgroup takes a rank in its CU's slot (one
// atomic add at start; slot = XCC id x 128 + CU / SH / SE id), publishes the rows it has
// dequeued, and at every row start runs at priority 1 while it is behind its partner.
constexpr int kRowCuSlots = 2048;
struct RowCuSlot { int count; int prog[3]; };
// Dynamic LDS layout: [RowCtrl 256 B][prog: fs x hc ints][W x WaveLds][fs x 2 line buffers][AngTab4][AngTab8]
// prog[slot][cy] = (local picture index & 0xffff) << 16 | CTUs done.

__device__ __forceinline__ void wave_sync() {
    // LDS operations of one wavefront execute in program order; only the compiler
    // must be kept from reordering the cross-lane LDS write -> read pairs.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int clip_pel(int v, int maxv) { return min(max(v, 0), maxv); }

// lane l <- lane l - 1 / lane l + 1 of the whole wave (DPP wave_shr:1 / wave_shl:1; the end lane keeps
// its own value): a one-lane shift without the LDS crossbar round trip of a ds_bpermute
__device__ __forceinline__ int wave_from_prev(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int wave_from_next(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xf, 0xf, false); }

// sum of v over the 32-lane half of the wave (PAIR) or the whole wave; NR = how many 16-lane
// rows from the start of each half can hold non-zero values (1, 2 or 4: fewer lane reads)
template <bool PAIR, int NR = 4>
__device__ __forceinline__ int wave_sum(int v, int half) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);    // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true);   // row_half_mirror
    v += __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true);   // row_mirror: every lane holds its row's sum
    auto rl = [&](int l) { return __builtin_amdgcn_readlane(v, l); };
    if constexpr (NR == 1) {
        return PAIR ? (half ? rl(32) : rl(0)) : rl(0);
    } else if constexpr (NR == 2) {
        return PAIR ? (half ? rl(32) + rl(48) : rl(0) + rl(16)) : rl(0) + rl(16);
    } else {
        const int s0 = rl(0) + rl(16);
        const int s1 = rl(32) + rl(48);
        return PAIR ? (half ? s1 : s0) : s0 + s1;
    }
}

// Reconstruct one intra job of size 2^LOG2: a luma TB (PAIR = false, 64 lanes) or the
// Cb/Cr TBs of one TU (PAIR = true, lanes 0-31 Cb, 32-63 Cr).  (w0, w1, w2) = job words
// (intra_prep.h), (ra, rb) = this lane's prefetched residual chunks, line_top = the
// row above the CTU for this lane's component, at the CTU's first column.
//
// Reference samples (8.4.4.2.2) are gathered straight from the LDS copies of the
// neighbourhood (CTU interior, left column, line buffer), every lane reading the sample
// that substitutes its entry (availability comes precomputed per 4-luma-sample unit),
// so substitution costs no extra round trip; luma filtering (8.4.4.2.3) adds one.
template <int LOG2, bool PAIR, typename T = uint8_t>
__device__ __forceinline__ void recon_job(WaveLdsT<T>& L, const T* line_top, uint32_t w0, uint32_t w1,
                                          uint32_t w2, uint4 ra, uint4 rb, int lane, int maxv = 255) {
    constexpr int n = 1 << LOG2;
    constexpr int nn = n * n;
    constexpr int LANES = PAIR ? 32 : 64;
    constexpr int S = nn >= LANES ? nn / LANES : 1;       // samples per lane (raster run)
    constexpr int nref = 4 * n + 1;
    constexpr int NCH = (nref + LANES - 1) / LANES;
    constexpr int US = PAIR ? 1 : 2;                      // log2 availability unit (samples)
    constexpr int NU = (2 * n) >> US;                     // units per side
    constexpr int SPW = 4 / (int)sizeof(T);               // samples per 32-bit word
    const int half_v = (maxv + 1) >> 1;                   // 1 << (BitDepth - 1): no reference available
    const int hl = PAIR ? (lane & 31) : lane;
    const int half = PAIR ? (lane >> 5) : 0;
    const int ofs = (int)(w0 & 0x1fffu);
    const int xr = PAIR ? ((ofs - 4096) & 31) : (ofs & 63);
    const int yr = PAIR ? ((ofs - 4096) >> 5) : (ofs >> 6);
    constexpr int ist = PAIR ? 32 : 64;
    T* const org = reinterpret_cast<T*>(&L) + (PAIR ? kOrgCT<T> : kOrgLT<T>) + ofs + half * 1024;   // TB origin
    const T* const lcol = (PAIR ? L.cleft[half] : L.yleft) + yr;
    const int mode = (int)((w0 >> 17) & 63u);
    const bool own = hl * S < nn && (!PAIR || ((w0 >> (15 + half)) & 1u));
    const int sidx = hl * S < nn ? hl * S : 0;
    const int sy = sidx >> LOG2, sx = sidx & (n - 1);
    const bool coded = (w0 >> (28 + half)) & 1u;
    if (!coded) { ra = make_uint4(0, 0, 0, 0); rb = ra; }
    uint32_t rw[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
    if constexpr (S == 4) {
        const bool hi = sidx & 4;
        rw[0] = hi ? ra.z : ra.x; rw[1] = hi ? ra.w : ra.y;
    } else if constexpr (S == 2) {
        const int e = (sidx & 7) >> 1;
        rw[0] = e == 0 ? ra.x : (e == 1 ? ra.y : (e == 2 ? ra.z : ra.w));
    } else if constexpr (S == 1) {
        const int e = sidx & 7;
        const uint32_t wd = e < 2 ? ra.x : (e < 4 ? ra.y : (e < 6 ? ra.z : ra.w));
        rw[0] = (e & 1) ? (wd >> 16) : (wd & 0xffffu);
    }
    auto resv = [&](int i) { return (int)(int16_t)(rw[i >> 1] >> ((i & 1) * 16)); };
    uint32_t outw[(S + SPW - 1) / SPW];
#pragma unroll
    for (int q = 0; q < (S + SPW - 1) / SPW; ++q) outw[q] = 0;
    auto put = [&](int i, int v) {
        outw[i / SPW] |= (uint32_t)clip_pel(v + resv(i), maxv) << (8 * (int)sizeof(T) * (i % SPW));
    };

    if (w0 & J_PCM) {
#pragma unroll
        for (int i = 0; i < S; ++i) put(i, 0);
    } else {
        // ---- gather (+ substitution) --------------------------------------------------
        const int filt = PAIR ? 0 : (int)((w0 >> 24) & 3u);
        T* const R0 = PAIR ? L.ref[half] : L.ref[0];
        T* const RF = (PAIR || !filt) ? R0 : L.ref[1];
        // sources: left column (entries 0..2n-1), corner (2n), top row (2n+1..4n)
        const T* const lbase = xr == 0 ? lcol : org - 1;
        const int lstep = xr == 0 ? 1 : ist;
        const T* const tbase = yr == 0 ? line_top + xr : org - ist;
        const T* const cptr = yr == 0 ? line_top + xr - 1 : (xr == 0 ? lcol - 1 : org - ist - 1);
        const unsigned long long m = (unsigned long long)w2 | ((unsigned long long)((w1 >> 21) & 1u) << 32);
        const bool all = w0 & J_ALL, none = w0 & J_NONE;
        int dcs = 0;
#pragma unroll
        for (int jj = 0; jj < NCH; ++jj) {
            const int k = hl + LANES * jj;
            if (jj + 1 < NCH || k < nref) {
                int s = k;
                if (!all) {
                    const int u = k < 2 * n ? (k >> US) : (k == 2 * n ? NU : NU + 1 + ((k - 2 * n - 1) >> US));
                    const unsigned long long below = m & ((1ull << u) - 1ull);
                    // both substitution candidates computed, then selected (no divergent branch)
                    const int ub = 63 - __clzll((long long)(below | 1ull));   // nearest available unit below
                    const int sb = ub < NU ? (ub << US) + (1 << US) - 1 : (ub == NU ? 2 * n : 2 * n + ((ub - NU) << US));
                    const int uf = __ffsll((long long)m) - 1;                 // first available unit
                    const int sf = uf < NU ? (uf << US) : (uf == NU ? 2 * n : 2 * n + 1 + ((uf - NU - 1) << US));
                    s = ((m >> u) & 1ull) ? k : (below ? sb : sf);
                }
                const T* src = s < 2 * n ? lbase + (2 * n - 1 - s) * lstep : (s == 2 * n ? cptr : tbase + (s - 2 * n - 1));
                const int v = none ? half_v : (int)*src;
                R0[k] = (T)v;
                if ((k >= n && k < 2 * n) || (k > 2 * n && k <= 3 * n)) dcs += v;
            }
        }
        wave_sync();
        if (!PAIR && filt) {
            // ---- filtering (8.4.4.2.3): [1 2 1], or strong bi-linear for 32x32 -----------
            bool strong = false;
            int corner = 0, bl = 0, tr = 0;
            if (n == 32 && filt == 2) {
                corner = R0[2 * n]; bl = R0[0]; tr = R0[4 * n];
                const int thr = (maxv + 1) >> 5;                  // 1 << (BitDepth - 5)
                strong = abs(corner + tr - 2 * (int)R0[3 * n]) < thr && abs(corner + bl - 2 * (int)R0[n]) < thr;
            }
#pragma unroll
            for (int jj = 0; jj < NCH; ++jj) {
                const int k = lane + 64 * jj;
                if (jj + 1 < NCH || k < nref) {
                    int f = R0[k];
                    if (k > 0 && k < 4 * n) {
                        if (strong) {
                            // (24-bit multiplies: every factor < 2^8; v_mul_lo_u32 is quarter rate)
                            f = k == 2 * n ? corner
                              : (k < 2 * n ? (__mul24(63 - (2 * n - 1 - k), corner) + __mul24(2 * n - k, bl) + 32) >> 6
                                           : (__mul24(63 - (k - 2 * n - 1), corner) + __mul24(k - 2 * n, tr) + 32) >> 6);
                        } else {
                            f = ((int)R0[k - 1] + 2 * f + (int)R0[k + 1] + 2) >> 2;
                        }
                    }
                    RF[k] = (T)f;
                }
            }
            wave_sync();
        }
        const T* const R = RF;
        // ---- prediction (8.4.4.2.4-6) fused with reconstruction (8.6.7) ---------------
        if (mode == 0) {
            const int trs = R[3 * n + 1], bls = R[n - 1];
            const int ly = R[2 * n - 1 - sy];
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const int x = sx + i;
                put(i, (__mul24(n - 1 - x, ly) + __mul24(x + 1, trs) + __mul24(n - 1 - sy, (int)R[2 * n + 1 + x]) +
                        __mul24(sy + 1, bls) + n) >> (LOG2 + 1));
            }
        } else if (mode == 1) {
            const int dc = (wave_sum<PAIR>(dcs, half) + n) >> (LOG2 + 1);
            constexpr bool edge = !PAIR && n < 32;
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
        } else {
            const int ang = (int)(int8_t)(w1 & 0xffu);
            const int ia = ang_inv(w1);
            if (mode >= 18) {                                        // vertical family
                const int pa = __mul24(sy + 1, ang);
                const int idx = pa >> 5, fact = pa & 31;
                auto refk = [&](int r) { return ang_ref<2 * n>(-r, ia, -1); };
                const bool bflt = !PAIR && n < 32 && mode == 26;
#pragma unroll
                for (int i = 0; i < S; ++i) {
                    const int x = sx + i;
                    const int r0 = x + idx + 1;
                    int v = R[refk(r0)];
                    v = (__mul24(32 - fact, v) + __mul24(fact, (int)R[refk(r0 + 1)]) + 16) >> 5;   // fact = 0: v
                    if (bflt && x == 0) v = clip_pel((int)R[2 * n + 1] + (((int)R[2 * n - 1 - sy] - (int)R[2 * n]) >> 1), maxv);
                    put(i, v);
                }
            } else {                                                 // horizontal family
                auto refk = [&](int r) { return ang_ref<2 * n>(-r, ia, 1); };
                const bool bflt = !PAIR && n < 32 && mode == 10 && sy == 0;
#pragma unroll
                for (int i = 0; i < S; ++i) {
                    const int x = sx + i;
                    const int pa = __mul24(x + 1, ang);
                    const int idx = pa >> 5, fact = pa & 31;
                    const int r0 = sy + idx + 1;
                    int v = R[refk(r0)];
                    v = (__mul24(32 - fact, v) + __mul24(fact, (int)R[refk(r0 + 1)]) + 16) >> 5;   // fact = 0: v
                    if (bflt) v = clip_pel((int)R[2 * n - 1] + (((int)R[2 * n + 1 + x] - (int)R[2 * n]) >> 1), maxv);
                    put(i, v);
                }
            }
        }
    }
    if (own) {
        T* dst = org + sy * ist + sx;
        constexpr int NB = S * (int)sizeof(T);                 // bytes per lane, naturally aligned
        if constexpr (NB == 32) {
            reinterpret_cast<uint4*>(dst)[0] = make_uint4(outw[0], outw[1], outw[2], outw[3]);
            reinterpret_cast<uint4*>(dst)[1] = make_uint4(outw[4], outw[5], outw[6], outw[7]);
        }
        else if constexpr (NB == 16) *reinterpret_cast<uint4*>(dst) = make_uint4(outw[0], outw[1], outw[2], outw[3]);
        else if constexpr (NB == 8) *reinterpret_cast<uint2*>(dst) = make_uint2(outw[0], outw[1]);
        else if constexpr (NB == 4) *reinterpret_cast<uint32_t*>(dst) = outw[0];
        else if constexpr (NB == 2) *reinterpret_cast<uint16_t*>(dst) = (uint16_t)outw[0];
        else dst[0] = (T)outw[0];
    }
    wave_sync();
}

// Prediction (8.4.4.2.4-6) of sample (x, y) of a fast job: lane k of v holds reference
// sample k of this lane's half (linear order of 8.4.4.2.2, substituted, filtered);
// angw = intraPredAngle (int8, bits 0..7) | |invAngle| << 8 (job word w1's layout; 256 without one).
// TAB: angw is instead this lane's entry of the workgroup's 4x4 angular table (AngTab4: both
// reference indices and the weights, no projection arithmetic); modes 10 / 26 are told by number.
template <int LOG2, bool PAIR, bool TAB = false>
__device__ __forceinline__ int fast_pred(int mode, uint32_t angw, int v, int x, int y, int k, int hl, int half,
                                         int maxv = 255) {
    constexpr int n = 1 << LOG2;
    const int base = half * 32;                                  // first reference lane of this half
    auto ref = [&](int i) { return __builtin_amdgcn_ds_bpermute((base + i) << 2, v); };
    auto uref = [&](int i) {                                     // reference i of this lane's half, uniform per half
        if constexpr (PAIR) {
            const int c0 = __builtin_amdgcn_readlane(v, i), c1 = __builtin_amdgcn_readlane(v, i + 32);
            return half ? c1 : c0;
        } else {
            return __builtin_amdgcn_readlane(v, i);
        }
    };
    int pred;
    // angular modes first (the most frequent path tests one condition: modes 2..34)
    if (mode >= 2) {
        if (P265R_HV_FAST && (TAB ? (mode & ~16) == 10 : (angw & 0xffu) == 0u)) {
            // modes 10 / 26 (intraPredAngle 0): a copy of the column left / the row above, plus the
            // luma boundary smoothing of 8.4.4.2.6 (fast jobs are n < 32) - no projection arithmetic
            const bool vert = mode >= 18;
            pred = ref(vert ? 2 * n + 1 + x : 2 * n - 1 - y);
            if (!PAIR) {
                const int b = ref(vert ? 2 * n - 1 - y : 2 * n + 1 + x);
                const int edge = clip_pel(uref(vert ? 2 * n + 1 : 2 * n - 1) + ((b - uref(2 * n)) >> 1), maxv);
                pred = (vert ? x : y) == 0 ? edge : pred;
            }
        } else if (TAB) {
            const int a = __builtin_amdgcn_ds_bpermute((int)(angw & 0xffu), v);
            const int b = __builtin_amdgcn_ds_bpermute((int)((angw >> 8) & 0xffu), v);
            pred = (__mul24((int)(angw >> 24), a) + __mul24((int)((angw >> 16) & 0xffu), b) + 16) >> 5;
        } else {
            const int ang = (int)(int8_t)(angw & 0xffu);
            const int ia = ang_inv(angw);
            const bool vert = mode >= 18;
            const int ns = vert ? -1 : 1;
            const int along = vert ? y : x, across = vert ? x : y;   // projection row / position on it
            const int pa = __mul24(along + 1, ang);
            const int idx = pa >> 5, fact = pa & 31;
            const int nr0 = -1 - across - idx;                       // -(iIdx + across + 1)
            const bool bflt = !P265R_HV_FAST && !PAIR && (mode == 26 || mode == 10);   // HV_FAST: copies above
            const int k1 = ang_ref<2 * n>(nr0 - 1, ia, ns);          // computed unconditionally: a select, no branch
            const int i1 = bflt ? (vert ? 2 * n - 1 - y : 2 * n + 1 + x) : k1;
            const int a = ref(ang_ref<2 * n>(nr0, ia, ns)), b = ref(i1);
            pred = (__mul24(32 - fact, a) + __mul24(fact, b) + 16) >> 5;   // = a when iFact = 0 (b then unused)
            if (bflt) {                                              // modes 26 / 10, luma: boundary smoothing
                const int edge = clip_pel(uref(vert ? 2 * n + 1 : 2 * n - 1) + ((b - uref(2 * n)) >> 1), maxv);
                pred = (vert ? x : y) == 0 ? edge : pred;
            }
        }
    } else if (mode == 0) {
        const int lft = ref(2 * n - 1 - y), top = ref(2 * n + 1 + x);
        pred = (__mul24(n - 1 - x, lft) + __mul24(x + 1, uref(3 * n + 1)) + __mul24(n - 1 - y, top) +
                __mul24(y + 1, uref(n - 1)) + n) >> (LOG2 + 1);
    } else {
        const bool in = (k >= n && k < 2 * n) || (k > 2 * n && k <= 3 * n);
        // luma: the edge samples' bpermutes go out first, their latency under the DPP reduction
        const int lft = PAIR ? 0 : ref(2 * n - 1 - y), top = PAIR ? 0 : ref(2 * n + 1 + x);
        const int dc = (wave_sum<PAIR, (LOG2 == 2 ? 1 : (LOG2 == 3 ? 2 : 4))>((hl <= 4 * n && in) ? v : 0, half) + n) >> (LOG2 + 1);
        if (PAIR) {
            pred = dc;
        } else {                                                 // luma n < 32: edge smoothing
            // (lft + 2dc + top + 2) >> 2 at (0,0); one-sided (3dc + side + 2) >> 2 on row 0 / column 0
            const int sl = x == 0 ? lft : dc, st = y == 0 ? top : dc;
            pred = (x == 0 || y == 0) ? (sl + st + 2 * dc + 2) >> 2 : dc;
        }
    }
    return pred;
}

// Fast job (luma 4x4 / 8x8, Cb+Cr 4x4 pair; job word 5 has J5_FAST): the available
// reference samples form one contiguous run [fa, la] of the linear order, so 8.4.4.2.2
// substitution is a clamp.  Lane k gathers reference sample k straight into a register;
// prediction reads its (at most) two per-sample references with ds_bpermute, so the job
// needs one LDS read, one bpermute round trip (two with the 8x8 [1 2 1] filter) and one
// LDS write - no reference array in LDS and no divergent control flow.  r16 = this
// lane's residual sample as loaded (ignored when the TB has none).
template <int LOG2, bool PAIR, typename T = uint8_t>
__device__ __forceinline__ void recon_fast(uint32_t lbase, uint32_t line_top, uint32_t w0, uint32_t w1,
                                           uint32_t w5, int r16, int lane, uint32_t tab, int maxv = 255) {
    constexpr int n = 1 << LOG2;
    constexpr int nn = n * n;
    constexpr uint32_t PB = sizeof(T);
    lbase /= PB; line_top /= PB;                            // byte -> sample addresses
    const int hl = PAIR ? (lane & 31) : lane;
    const int half = PAIR ? (lane >> 5) : 0;
    const int ofs = (int)(w0 & 0x1fffu);
    const int xr = PAIR ? ((ofs - 4096) & 31) : (ofs & 63);
    const int yr = PAIR ? ((ofs - 4096) >> 5) : (ofs >> 6);
    constexpr int ist = PAIR ? 32 : 64;
    const int mode = (int)((w0 >> 17) & 63u);
    // ---- gather: lane k <- reference sample Clip3(fa, la, k) -------------------------------
    // (addresses as 32-bit LDS offsets, selected without branches; NONE: all refs = 128)
    const int k = min(hl, 4 * n);
    const int fa = (int)(w5 & 0xffu), la = (int)((w5 >> 8) & 0xffu);
    const int sref = min(max(k, fa), la);
    const uint32_t orgA = lbase + (PAIR ? kOrgCT<T> : kOrgLT<T>) + (uint32_t)ofs + (uint32_t)half * 1024u;   // TB origin
    const uint32_t lcolA = lbase + (PAIR ? kCLeftT<T> + (uint32_t)half * 32u : kYLeftT<T>) + (uint32_t)yr;
    const uint32_t ltA = line_top + (uint32_t)xr;
    // left refs k < 2n at lb - k * ls, top refs k > 2n at tb + k; the corner k = 2n follows the
    // left formula inside the CTU / left column and the top formula in the line buffer (yr = 0)
    const uint32_t lb = xr == 0 ? lcolA + 2 * n - 1 : orgA - 1 + (2 * n - 1) * ist;
    const int ls = xr == 0 ? 1 : ist;
    const uint32_t tb = (yr == 0 ? ltA : orgA - ist) - 2 * n - 1;
    const int th = 2 * n + (yr > 0 ? 1 : 0);
    const uint32_t sa = tb + sref + (sref < th ? (lb - tb) - (uint32_t)(sref * (ls + 1)) : 0u);
    const int raw = (int)*ldsT<T>(sa);
    // luma: this sample's angular table entry (AngTab4 / AngTab8), read together with the gather
    constexpr bool TAB = !PAIR && (LOG2 == 2 || (LOG2 == 3 && P265R_ANGTAB8));
    uint32_t te = w1;
    if constexpr (TAB) {
        const uint32_t t0 = tab + (LOG2 == 3 ? (uint32_t)kAngTab4Bytes : 0u);
        te = *lds32(t0 + (uint32_t)mode * (uint32_t)(nn * 4) + (uint32_t)((hl & (nn - 1)) * 4));
        asm volatile("" : "+v"(te));
    }
    int v = (w0 & J_NONE) ? (maxv + 1) >> 1 : raw;
    if (!PAIR && LOG2 == 3 && ((w0 >> 24) & 3u)) {           // [1 2 1] (8.4.4.2.3), 8x8: never strong
        // neighbours k -/+ 1 by DPP wave shifts (lane k holds sample k for k <= 4n; no LDS round trip)
        const int vl = wave_from_prev(v), vr = wave_from_next(v);
        const int f = (vl + 2 * v + vr + 2) >> 2;
        v = (k > 0 && k < 4 * n) ? f : v;                       // the two end samples stay unfiltered
    }
    // ---- prediction (8.4.4.2.4-6) fused with reconstruction (8.6.7) ---------------------------
    const int sidx = hl < nn ? hl : 0;
    const int x = sidx & (n - 1), y = sidx >> LOG2;
    const int pred = fast_pred<LOG2, PAIR, TAB>(mode, te, v, x, y, k, hl, half, maxv);
    // every lane stores (no exec-mask juggling): lanes without a sample of this job write a
    // private sample of the (here unused) reference scratch area
    const bool own = hl < nn && (!PAIR || ((w0 >> (15 + half)) & 1u));
    const uint32_t da = own ? orgA + y * ist + x : lbase + kRefT<T> + lane;
    // r16: the loaded sample (an uncoded half reads the zero block, intra_prep.h w3/w4)
    *ldsT<T>(da) = (T)clip_pel(pred + r16, maxv);
    wave_sync();
}

// Fast 16x16 luma job (J5_FAST): as recon_fast, 65 reference samples (lane k holds
// sample k, sample 64 is wave-uniform), 4 predicted samples per lane (a row quarter),
// residual (4 samples) in rw.x / rw.y, one 4-byte LDS store per lane.
template <typename T = uint8_t>
__device__ __forceinline__ void recon_fast16(uint32_t lbase, uint32_t line_top, uint32_t w0, uint32_t w1,
                                             uint32_t w5, uint4 rw, int lane, int maxv = 255) {
    constexpr int n = 16, LOG2 = 4, ist = 64;
    constexpr uint32_t PB = sizeof(T);
    lbase /= PB; line_top /= PB;                            // byte -> sample addresses
    const int ofs = (int)(w0 & 0x1fffu);
    const int xr = ofs & 63, yr = ofs >> 6;
    const int mode = (int)((w0 >> 17) & 63u);
    const int fa = (int)(w5 & 0xffu), la = (int)((w5 >> 8) & 0xffu);
    const uint32_t orgA = lbase + kOrgLT<T> + (uint32_t)ofs;
    const uint32_t lcolA = lbase + kYLeftT<T> + (uint32_t)yr;
    const uint32_t ltA = line_top + (uint32_t)xr;
    const uint32_t lb = xr == 0 ? lcolA + 2 * n - 1 : orgA - 1 + (2 * n - 1) * ist;
    const int ls = xr == 0 ? 1 : ist;
    const uint32_t tb = (yr == 0 ? ltA : orgA - ist) - 2 * n - 1;
    const int th = 2 * n + (yr > 0 ? 1 : 0);
    auto addr = [&](int sref) { return tb + sref + (sref < th ? (lb - tb) - (uint32_t)(sref * (ls + 1)) : 0u); };
    const bool none = (w0 & J_NONE) != 0;
    const int half_v = (maxv + 1) >> 1;
    const int k = lane;
    const int raw = (int)*ldsT<T>(addr(min(max(k, fa), la)));
    const int raw64 = (int)*ldsT<T>(addr(min(max(4 * n, fa), la)));
    int v = none ? half_v : raw;
    const int r64 = none ? half_v : __builtin_amdgcn_readfirstlane(raw64);     // reference sample 64 (end, unfiltered)
    if ((w0 >> 24) & 3u) {                                    // [1 2 1] (8.4.4.2.3)
        const int vl = wave_from_prev(v), vr0 = wave_from_next(v);   // DPP wave shifts
        const int vr = k == 63 ? r64 : vr0;
        const int f = (vl + 2 * v + vr + 2) >> 2;
        v = k > 0 ? f : v;
    }
    auto ref = [&](int i) {                                   // reference i, 0..64
        const int b = __builtin_amdgcn_ds_bpermute(min(i, 63) << 2, v);
        return i >= 64 ? r64 : b;
    };
    auto uref = [&](int i) { return i >= 64 ? r64 : (int)__builtin_amdgcn_readlane(v, i); };
    const int x0 = (lane & 3) << 2, y = lane >> 2;           // samples (x0 .. x0 + 3, y)
    int pred[4];
    if (mode == 0) {
        const int lft = ref(2 * n - 1 - y), trs = uref(3 * n + 1), bls = uref(n - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int x = x0 + i;
            pred[i] = (__mul24(n - 1 - x, lft) + __mul24(x + 1, trs) + __mul24(n - 1 - y, ref(2 * n + 1 + x)) +
                       __mul24(y + 1, bls) + n) >> (LOG2 + 1);
        }
    } else if (mode == 1) {
        const bool in = (k >= n && k < 2 * n) || (k > 2 * n && k <= 3 * n);
        const int dc = (wave_sum<false>(in ? v : 0, 0) + n) >> (LOG2 + 1);
        const int lft = ref(2 * n - 1 - y);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int x = x0 + i;
            const int top = ref(2 * n + 1 + x);
            const int sl = x == 0 ? lft : dc, st = y == 0 ? top : dc;
            pred[i] = (x == 0 || y == 0) ? (sl + st + 2 * dc + 2) >> 2 : dc;
        }
    } else if (P265R_HV_FAST && (w1 & 0xffu) == 0u) {        // modes 10 / 26: copies + boundary smoothing
        if (mode >= 18) {
            const int e = clip_pel(uref(2 * n + 1) + ((ref(2 * n - 1 - y) - uref(2 * n)) >> 1), maxv);
#pragma unroll
            for (int i = 0; i < 4; ++i) pred[i] = ref(2 * n + 1 + x0 + i);
            pred[0] = x0 == 0 ? e : pred[0];
        } else {
            const int l = ref(2 * n - 1 - y), corner = uref(2 * n);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int t = ref(2 * n + 1 + x0 + i);          // every lane: ds_bpermute outside any branch
                pred[i] = y == 0 ? clip_pel(l + ((t - corner) >> 1), maxv) : l;
            }
        }
    } else {
        const int ang = (int)(int8_t)(w1 & 0xffu);
        const int ia = ang_inv(w1);
        auto refk = [&](int r, bool vert) { return ang_ref<2 * n>(-r, ia, vert ? -1 : 1); };
        if (mode >= 18) {                                     // vertical: one projection row per lane
            const int pa = __mul24(y + 1, ang);
            const int idx = pa >> 5, fact = pa & 31;
            int q[5];
#pragma unroll
            for (int m = 0; m < 5; ++m) q[m] = ref(refk(x0 + idx + 1 + m, true));
#pragma unroll
            for (int i = 0; i < 4; ++i) pred[i] = (__mul24(32 - fact, q[i]) + __mul24(fact, q[i + 1]) + 16) >> 5;
            if (!P265R_HV_FAST && mode == 26) {               // x == 0: boundary smoothing (HV_FAST: above)
                const int e = clip_pel(uref(2 * n + 1) + ((ref(2 * n - 1 - y) - uref(2 * n)) >> 1), maxv);
                pred[0] = x0 == 0 ? e : pred[0];
            }
        } else {                                              // horizontal: projection column per sample
            const int corner = uref(2 * n), left0 = uref(2 * n - 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int x = x0 + i;
                const int pa = __mul24(x + 1, ang);
                const int idx = pa >> 5, fact = pa & 31;
                const int r0 = y + idx + 1;
                const int a = ref(refk(r0, false));
                const int k1 = refk(r0 + 1, false);
                const int b = ref((!P265R_HV_FAST && mode == 10) ? 2 * n + 1 + x : k1);
                pred[i] = (__mul24(32 - fact, a) + __mul24(fact, b) + 16) >> 5;
                if (!P265R_HV_FAST && mode == 10) pred[i] = y == 0 ? clip_pel(left0 + ((b - corner) >> 1), maxv) : pred[i];
            }
        }
    }
    uint32_t out[2] = {0u, 0u};                               // (an uncoded TB's residual is the zero block)
    constexpr int SPW = 4 / (int)PB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t wd = i < 2 ? rw.x : rw.y;
        const int res = (int)(int16_t)(wd >> (16 * (i & 1)));
        out[i / SPW] |= (uint32_t)clip_pel(pred[i] + res, maxv) << (8 * (int)PB * (i % SPW));
    }
    if constexpr (PB == 1) *lds32(orgA + y * ist + x0) = out[0];
    else *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(ldsT<T>(orgA + y * ist + x0)) = u32x2_t{out[0], out[1]};
    wave_sync();
}

// Chroma prediction (8.4.4.2.4-6) of sample (x, y) of an nTbS = 2^LOG2 Cb+Cr pair, Cb and Cr
// at once: every value is a packed pair (Cb bits 0..15, Cr bits 16..31).  Packed 8-bit samples
// are < 2^24, so v_mul_u32_u24 weighs both halves with one multiply; every weighted sum stays
// below 2^16 per half (planar / DC 2n x 255 + n, angular 32 x 255 + 16), so the halves never
// carry into each other and one shift + mask divides both.  Lane k of v holds reference k of
// 8.4.4.2.2's linear order.  Chroma (4:2:0) has no DC / horizontal / vertical boundary smoothing.
template <int LOG2, bool TAB = false, typename T = uint8_t>
__device__ __forceinline__ uint32_t cpred(int mode, uint32_t angw, uint32_t v, int x, int y, int k) {
    constexpr int n = 1 << LOG2;
    constexpr uint32_t rnd = (uint32_t)n * 0x00010001u;
    constexpr uint32_t msk = (0xffffu >> (LOG2 + 1)) * 0x00010001u;
    auto ref = [&](int i) { return (uint32_t)__builtin_amdgcn_ds_bpermute(i << 2, (int)v); };
    auto uref = [&](int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, i); };
    if (mode >= 2) {                                           // angular first: the most frequent path
        if (TAB) {                                             // AngTab4 entry (modes 10 / 26 included: fact 0)
            const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(angw & 0xffu), (int)v);
            const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((angw >> 8) & 0xffu), (int)v);
            return pang<T>(angw >> 24, a, (angw >> 16) & 0xffu, b);
        }
        if (P265R_HV_FAST && (angw & 0xffu) == 0u)              // modes 10 / 26: a copy (no chroma smoothing)
            return ref(mode >= 18 ? 2 * n + 1 + x : 2 * n - 1 - y);
        const int ang = (int)(int8_t)(angw & 0xffu);
        const int ia = ang_inv(angw);
        const bool vert = mode >= 18;
        const int ns = vert ? -1 : 1;
        const int along = vert ? y : x, across = vert ? x : y;
        const int pa = __mul24(along + 1, ang);
        const int idx = pa >> 5, fact = pa & 31;
        const int nr0 = -1 - across - idx;
        const uint32_t a = ref(ang_ref<2 * n>(nr0, ia, ns)), b = ref(ang_ref<2 * n>(nr0 - 1, ia, ns));
        return pang<T>(32 - fact, a, fact, b);
    }
    if (mode == 0) {
        const uint32_t lft = ref(2 * n - 1 - y), top = ref(2 * n + 1 + x);
        const uint32_t s = pmul<T>(n - 1 - x, lft) + pmul<T>(x + 1, uref(3 * n + 1)) + pmul<T>(n - 1 - y, top) +
                           pmul<T>(y + 1, uref(n - 1)) + rnd;
        return (s >> (LOG2 + 1)) & msk;
    }
    const bool in = (k >= n && k < 2 * n) || (k > 2 * n && k <= 3 * n);
    const uint32_t s = (uint32_t)wave_sum<false, (LOG2 == 2 ? 1 : (LOG2 == 3 ? 2 : 4))>(in ? (int)v : 0, 0) + rnd;
    return (s >> (LOG2 + 1)) & msk;
}

// Clip1(pred + res) of both halves: pred packed (0..maxv per half), res two int16 residuals
__device__ __forceinline__ uint32_t cquad_recon(uint32_t pred, uint32_t res, int maxv = 255) {
    const int cb = clip_pel((int)(pred & 0xffffu) + (int)(int16_t)(res & 0xffffu), maxv);
    const int cr = clip_pel((int)(pred >> 16) + ((int)res >> 16), maxv);
    return (uint32_t)cb | (uint32_t)cr << 16;
}

// Fast Cb+Cr 8x8 pair (J5_FAST, component mask 3): as recon_fast, with Cb and Cr packed in the
// 16-bit halves of each lane (cpred).  Lane k gathers reference sample Clip3(fa, la, k),
// k = 0..32, of both components (the Cr copy of a neighbour sits 1024 B further in the CTU
// interior, 32 B in the left column, cw B in the line buffer); lane l predicts sample
// (l & 7, l >> 3) of both.  r32 = this lane's residual pair Cb | Cr << 16; line_cb = the row
// above the CTU in the Cb line buffer.
template <typename T = uint8_t>
__device__ __forceinline__ void recon_cfast8(uint32_t lbase, uint32_t line_cb, uint32_t cw, uint32_t w0, uint32_t w1,
                                             uint32_t w5, int r32, int lane, uint32_t tab, int maxv = 255) {
    constexpr int n = 8, ist = 32;
    constexpr uint32_t PB = sizeof(T);
    lbase /= PB; line_cb /= PB;                             // byte -> sample addresses (cw: samples)
    const int ofs = (int)(w0 & 0x1fffu);
    const int xr = (ofs - 4096) & 31, yr = (ofs - 4096) >> 5;
    const int mode = (int)((w0 >> 17) & 63u);
    const int k = min(lane, 4 * n);
    const int fa = (int)(w5 & 0xffu), la = (int)((w5 >> 8) & 0xffu);
    const int sref = min(max(k, fa), la);
    const uint32_t orgA = lbase + kOrgCT<T> + (uint32_t)ofs;                        // Cb TB origin
    const uint32_t lcolA = lbase + kCLeftT<T> + (uint32_t)yr;
    const uint32_t lb = xr == 0 ? lcolA + 2 * n - 1 : orgA - 1 + (2 * n - 1) * ist;
    const int ls = xr == 0 ? 1 : ist;
    const uint32_t tb = (yr == 0 ? line_cb + (uint32_t)xr : orgA - ist) - 2 * n - 1;
    const int th = 2 * n + (yr > 0 ? 1 : 0);
    const bool left = sref < th;
    const uint32_t sa = tb + sref + (left ? (lb - tb) - (uint32_t)(sref * (ls + 1)) : 0u);
    const uint32_t dcr = left ? (xr == 0 ? 32u : 1024u) : (yr == 0 ? cw : 1024u);
    const uint32_t cb = *ldsT<T>(sa), cr = *ldsT<T>(sa + dcr);
    uint32_t te = w1;
    if constexpr (P265R_ANGTAB8) {                            // AngTab8 entry of sample lane
        te = *lds32(tab + (uint32_t)kAngTab4Bytes + (uint32_t)mode * 256u + (uint32_t)lane * 4u);
        asm volatile("" : "+v"(te));
    }
    const uint32_t v = (w0 & J_NONE) ? (uint32_t)((maxv + 1) >> 1) * 0x00010001u : (cb | cr << 16);
    const int x = lane & 7, y = lane >> 3;
    const uint32_t rec = cquad_recon(cpred<3, (bool)P265R_ANGTAB8, T>(mode, te, v, x, y, k), (uint32_t)r32, maxv);
    const uint32_t da = orgA + (uint32_t)(y * ist + x);
    *ldsT<T>(da) = (T)(rec & 0xffffu);
    *ldsT<T>(da + 1024) = (T)(rec >> 16);
    wave_sync();
}

// One stage of a 4x4 quad job (recon_quad): sub-TB Q of the 8x8 region.  Lane k of the
// reference vector holds reference sample Clip3(fa, la, k) (8.4.4.2.2), taken from the
// region's external samples (ext, gathered once per quad) or from the stages already
// reconstructed (rec: lane = region sample y * 8 + x); the source of every reference index is
// a compile-time affine map per stage.  Lanes of sub-TB Q then predict (fast_pred) and
// reconstruct their sample into rec.  CH: chroma quad, every value a packed Cb | Cr << 16 pair.
template <int Q, bool CH, typename T = uint8_t>
__device__ __forceinline__ int quad_stage(int rec, int ext, int lane, int mode, bool none, int fa, int la,
                                          uint32_t te, int r16, int qid, int xs, int ys, int maxv = 255) {
    const int s = min(max(lane, fa), la);                        // substituted reference index
    auto bp = [](int i, int src) { return __builtin_amdgcn_ds_bpermute(i << 2, src); };
    int v;
    if constexpr (Q == 0) {                                      // all external: corner e = 0, left e = 8 - s, top e = s + 4
        v = bp(s <= 8 ? 8 - s : s + 4, ext);
    } else if constexpr (Q == 1) {                               // left: q0's column x = 3; corner / top external
        const int a = bp(59 - 8 * s, rec), b = bp(s + 8, ext);
        v = s < 8 ? a : b;
    } else if constexpr (Q == 2) {                               // left / corner external; top: q0 / q1 row y = 3
        const int a = bp(12 - s, ext), b = bp(s + 15, rec);
        v = s <= 8 ? a : b;
    } else {                                                     // all internal (q2 column, q0 corner, q1 row)
        v = bp(s <= 8 ? 91 - 8 * s : s + 19, rec);
    }
    // only the first stage can find no reference available: stages 1-3 always have the region's earlier
    // sub-blocks (q1: q0's column on the left, q2: q0's row above, q3: both) -- their none bits are 0
    if constexpr (CH) {
        if constexpr (Q == 0) v = none ? (int)((uint32_t)((maxv + 1) >> 1) * 0x00010001u) : v;
        const int rq = (int)cquad_recon(cpred<2, true, T>(mode, te, (uint32_t)v, xs, ys, lane), (uint32_t)r16, maxv);
        return qid == Q ? rq : rec;
    } else {
        if constexpr (Q == 0) v = none ? (maxv + 1) >> 1 : v;
        const int rq = clip_pel(fast_pred<2, false, true>(mode, te, v, xs, ys, lane, lane, 0, maxv) + r16, maxv);
        return qid == Q ? rq : rec;
    }
}

// One quad stage with COMPOSED reference reads (the latency layouts, P265R_QUAD_COMPOSED): every reference
// the stage's prediction reads is taken straight from its source register -- Clip3(fa, la, i) mapped by the
// stage's affine map onto the external samples or the stages already reconstructed -- instead of first
// gathering the stage's reference vector and then reading it: one ds_bpermute round trip per stage instead
// of two, for a few more VALU (the index map per read) and the stage's AngTab4 entry read ahead with the
// external gather.  Luma stages with two sources read one packed register (rec | ext << 16); chroma values
// are Cb | Cr pairs already, so a chroma read takes both candidates and selects.  Same arithmetic as
// quad_stage (fast_pred<2, false, true> / cpred<2, true>), bit for bit.
template <int Q, bool CH, typename T = uint8_t>
__device__ __forceinline__ int quad_stage_c(int rec, int ext, int lane, int mode, bool none, int fa, int la,
                                            uint32_t te, int r16, int qid, int x, int y, int maxv = 255) {
    constexpr int n = 4;
    const int half_v = (maxv + 1) >> 1;
    const uint32_t none_v = CH ? (uint32_t)half_v * 0x00010001u : (uint32_t)half_v;
    // source of substituted reference s: (lane of the source register, from ext?)
    auto src_lane = [](int s) -> int {
        if constexpr (Q == 0) return s <= 8 ? 8 - s : s + 4;
        else if constexpr (Q == 1) return s < 8 ? 59 - 8 * s : s + 8;
        else if constexpr (Q == 2) return s <= 8 ? 12 - s : s + 15;
        else return s <= 8 ? 91 - 8 * s : s + 19;
    };
    auto from_ext = [](int s) -> bool {
        if constexpr (Q == 0) return true;
        else if constexpr (Q == 1) return s >= 8;
        else if constexpr (Q == 2) return s <= 8;
        else return false;
    };
    // luma, two sources: one packed register, the half picked after the read
    const int P = (Q == 1 || Q == 2) && !CH ? (int)(((uint32_t)rec & 0xffffu) | (uint32_t)ext << 16) : (Q == 0 ? ext : rec);
    auto cref = [&](int i) -> uint32_t {                           // per-lane reference index i
        const int s = min(max(i, fa), la);
        const int sl = src_lane(s) << 2;
        uint32_t v;
        if constexpr (Q == 0 || Q == 3) {
            v = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, P);
        } else if constexpr (!CH) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, P);
            v = from_ext(s) ? w >> 16 : w & 0xffffu;
        } else {
            const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, rec), b = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, ext);
            v = from_ext(s) ? b : a;
        }
        if constexpr (Q == 0) v = none ? none_v : v;
        return v;
    };
    auto uref = [&](int i) -> uint32_t {                           // wave-uniform reference index i
        const int s = __builtin_amdgcn_readfirstlane(min(max(i, fa), la));
        const int sl = src_lane(s);
        uint32_t v;
        if constexpr (Q == 0 || Q == 3) {
            v = (uint32_t)__builtin_amdgcn_readlane(P, sl);
        } else if constexpr (!CH) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_readlane(P, sl);
            v = from_ext(s) ? w >> 16 : w & 0xffffu;
        } else {
            v = from_ext(s) ? (uint32_t)__builtin_amdgcn_readlane(ext, sl) : (uint32_t)__builtin_amdgcn_readlane(rec, sl);
        }
        if constexpr (Q == 0) v = none ? none_v : v;
        return v;
    };
    const bool in = (lane >= n && lane < 2 * n) || (lane > 2 * n && lane <= 3 * n);   // DC sum lanes
    if constexpr (CH) {
        constexpr uint32_t rnd = (uint32_t)n * 0x00010001u, msk = (0xffffu >> 3) * 0x00010001u;
        uint32_t pred;
        if (mode >= 2) {                                           // AngTab4 entry (modes 10 / 26 included: fact 0)
            const uint32_t a = cref((int)((te & 0xffu) >> 2)), b = cref((int)(((te >> 8) & 0xffu) >> 2));
            pred = ((pmul<T>(te >> 24, a) + pmul<T>((te >> 16) & 0xffu, b) + 0x00100010u) >> 5) & 0x07ff07ffu;
        } else if (mode == 0) {
            const uint32_t lft = cref(2 * n - 1 - y), top = cref(2 * n + 1 + x);
            const uint32_t sum = pmul<T>(n - 1 - x, lft) + pmul<T>(x + 1, uref(3 * n + 1)) + pmul<T>(n - 1 - y, top) +
                                 pmul<T>(y + 1, uref(n - 1)) + rnd;
            pred = (sum >> 3) & msk;
        } else {
            const uint32_t vk = cref(lane);
            const uint32_t sum = (uint32_t)wave_sum<false, 1>(in ? (int)vk : 0, 0) + rnd;
            pred = (sum >> 3) & msk;
        }
        const int rq = (int)cquad_recon(pred, (uint32_t)r16, maxv);
        return qid == Q ? rq : rec;
    } else {
        int pred;
        if (mode >= 2) {
            if (P265R_HV_FAST && (mode & ~16) == 10) {             // modes 10 / 26: copies + boundary smoothing
                const bool vert = mode >= 18;
                pred = (int)cref(vert ? 2 * n + 1 + x : 2 * n - 1 - y);
                const int b = (int)cref(vert ? 2 * n - 1 - y : 2 * n + 1 + x);
                const int edge = clip_pel((int)uref(vert ? 2 * n + 1 : 2 * n - 1) + ((b - (int)uref(2 * n)) >> 1), maxv);
                pred = (vert ? x : y) == 0 ? edge : pred;
            } else {
                const int a = (int)cref((int)((te & 0xffu) >> 2)), b = (int)cref((int)(((te >> 8) & 0xffu) >> 2));
                pred = (__mul24((int)(te >> 24), a) + __mul24((int)((te >> 16) & 0xffu), b) + 16) >> 5;
            }
        } else if (mode == 0) {
            const int lft = (int)cref(2 * n - 1 - y), top = (int)cref(2 * n + 1 + x);
            pred = (__mul24(n - 1 - x, lft) + __mul24(x + 1, (int)uref(3 * n + 1)) + __mul24(n - 1 - y, top) +
                    __mul24(y + 1, (int)uref(n - 1)) + n) >> 3;
        } else {
            const int vk = (int)cref(lane);
            const int lft = (int)cref(2 * n - 1 - y), top = (int)cref(2 * n + 1 + x);
            const int dc = (wave_sum<false, 1>(in ? vk : 0, 0) + n) >> 3;
            const int sl = x == 0 ? lft : dc, st = y == 0 ? top : dc;
            pred = (x == 0 || y == 0) ? (sl + st + 2 * dc + 2) >> 2 : dc;
        }
        const int rq = clip_pel(pred + r16, maxv);
        return qid == Q ? rq : rec;
    }
}

// 4x4 QUAD job (J5_QUAD, intra_prep.h): the four fast 4x4 TBs of one 8x8 luma region (CH =
// false), or the four Cb+Cr 4x4 pairs of one 8x8 chroma region (CH = true), in one job.  Lane
// l = region sample (l & 7, l >> 3); the 25 external reference samples (column x = -1, rows
// -1..11; row y = -1, columns 0..11) are read from LDS once (chroma: lanes 0-24 read the Cb sample
// and its Cr twin, 1024 B further in the CTU interior, 32 B in the left column, cw B in the line
// buffer, and pack them), the four stages pass their samples to each other through registers
// (ds_bpermute), and the region is written to LDS once.  r16 = this lane's residual sample
// (chroma: the packed Cb | Cr << 16 pair); line_top = the row above the CTU (chroma: the Cb line).
template <bool CH, typename T = uint8_t, bool COMP = false>
__device__ __forceinline__ void recon_quad(uint32_t lbase, uint32_t line_top, uint32_t cw, uint32_t w0, uint32_t w1,
                                           uint32_t w2, uint32_t tab, int r16, int lane, int maxv = 255) {
    constexpr int ist = CH ? 32 : 64, last = ist - 1;           // interior stride, last row / column
    constexpr uint32_t PB = sizeof(T);
    lbase /= PB; line_top /= PB;                                 // byte -> sample addresses (cw: samples)
    const int ofs = (int)(w0 & 0x1fffu);
    const int X = CH ? ((ofs - 4096) & 31) : (ofs & 63), Y = CH ? ((ofs - 4096) >> 5) : (ofs >> 6);
    const uint32_t orgA = lbase + (CH ? kOrgCT<T> : kOrgLT<T>) + (uint32_t)ofs;
    const uint32_t leftA = lbase + (CH ? kCLeftT<T> : kYLeftT<T>);
    // ---- external references: e = 0..12 column x = -1 (row e - 1), e = 13..24 row y = -1 ------
    const int e = min(CH ? (lane & 31) : lane, 24);
    // every candidate computed, then selected: no divergent branch per lane class
    const int r = min(Y - 1 + e, last);                          // rows below the CTU: never available
    const int c = e - 13;
    const uint32_t col = X > 0 ? orgA - 1 + (uint32_t)((r - Y) * ist) : leftA + (uint32_t)r;
    const uint32_t row = Y == 0 ? line_top + (uint32_t)(X + c) : orgA - ist + (uint32_t)min(c, last - X);
    const uint32_t ea = e > 12 ? row : (r < 0 ? line_top + (uint32_t)(X - 1) : col);
    int ext = (int)*ldsT<T>(ea);
    if constexpr (CH) {                                          // Cb | Cr << 16 (same LDS round trip)
        const uint32_t dcr = e > 12 ? (Y == 0 ? cw : 1024u) : (r < 0 ? cw : (X > 0 ? 1024u : 32u));
        ext |= (int)*ldsT<T>(ea + dcr) << 16;
    }
    const int xs = lane & 3, ys = (lane >> 3) & 3;
    const int qid = ((lane >> 4) & 2) | ((lane >> 2) & 1);
    // this lane's AngTab4 entry of mode m (sample (xs, ys) of its sub-TB), read with the stage's gather
    const uint32_t pos4 = (uint32_t)((ys * 4 + xs) * 4);
    // (pinned at the stage start: the read then shares the gather's LDS wait instead of adding one)
    auto ang = [&](uint32_t m) { uint32_t te = *lds32(tab + m * 64u + pos4); asm volatile("" : "+v"(te)); return te; };
    int rec = 0;
    if constexpr (COMP) {
        // composed stages: the four AngTab4 entries read with the external gather (one LDS round trip)
        const uint32_t m0 = (w0 >> 17) & 63u, m1 = (w0 >> 23) & 63u, m2 = w1 & 63u, m3 = (w1 >> 6) & 63u;
        const uint32_t t0 = ang(m0), t1 = ang(m1), t2 = ang(m2), t3 = ang(m3);
        rec = quad_stage_c<0, CH, T>(rec, ext, lane, (int)m0, (w0 >> 29) & 1u, (int)((w1 >> 14) & 31u), (int)((w1 >> 19) & 31u),
                                     t0, r16, qid, xs, ys, maxv);
        rec = quad_stage_c<1, CH, T>(rec, ext, lane, (int)m1, false, (int)((w1 >> 24) & 31u), (int)(w2 & 31u),
                                     t1, r16, qid, xs, ys, maxv);
        rec = quad_stage_c<2, CH, T>(rec, ext, lane, (int)m2, false, (int)((w2 >> 5) & 31u), (int)((w2 >> 10) & 31u),
                                     t2, r16, qid, xs, ys, maxv);
        rec = quad_stage_c<3, CH, T>(rec, ext, lane, (int)m3, false, (int)((w2 >> 15) & 31u), (int)((w2 >> 20) & 31u),
                                     t3, r16, qid, xs, ys, maxv);
    } else {
    P265R_MARK("quad_stage0");
    {
        const uint32_t m = (w0 >> 17) & 63u;
        rec = quad_stage<0, CH, T>(rec, ext, lane, (int)m, (w0 >> 29) & 1u, (int)((w1 >> 14) & 31u), (int)((w1 >> 19) & 31u),
                                   ang(m), r16, qid, xs, ys, maxv);
    }
    P265R_MARK("quad_stage1");
    {
        const uint32_t m = (w0 >> 23) & 63u;
        rec = quad_stage<1, CH, T>(rec, ext, lane, (int)m, (w0 >> 30) & 1u, (int)((w1 >> 24) & 31u), (int)(w2 & 31u),
                                   ang(m), r16, qid, xs, ys, maxv);
    }
    P265R_MARK("quad_stage2");
    {
        const uint32_t m = w1 & 63u;
        rec = quad_stage<2, CH, T>(rec, ext, lane, (int)m, (w1 >> 12) & 1u, (int)((w2 >> 5) & 31u), (int)((w2 >> 10) & 31u),
                                   ang(m), r16, qid, xs, ys, maxv);
    }
    P265R_MARK("quad_stage3");
    {
        const uint32_t m = (w1 >> 6) & 63u;
        rec = quad_stage<3, CH, T>(rec, ext, lane, (int)m, (w1 >> 13) & 1u, (int)((w2 >> 15) & 31u), (int)((w2 >> 20) & 31u),
                                   ang(m), r16, qid, xs, ys, maxv);
    }
    }
    P265R_MARK("quad_store");
    const uint32_t da = lbase + (CH ? kOrgCT<T> : kOrgLT<T>) + (uint32_t)ofs + (uint32_t)((lane >> 3) * ist + (lane & 7));
    *ldsT<T>(da) = (T)((uint32_t)rec & 0xffffu);
    if constexpr (CH) *ldsT<T>(da + 1024) = (T)((uint32_t)rec >> 16);
    wave_sync();
}

// WPE = waves per SIMD the register allocation must allow (1: unconstrained).  W = 10 / 12 need
// 5 / 6 for two workgroups per CU (at most 96 / 80 VGPRs).  W = 8 comes twice: unconstrained
// (≈100 VGPRs) for a batch that runs alone, and register-lean (WPE 6: 80 VGPRs, a few spills)
// for batches overlapping other batches' residual / loop-filter kernels, whose waves then
// fit beside it on every SIMD (p265r.hip launch_rows; measured in DESIGN.md §6).
//
// XG (cross-group chains, the latency regime): every picture's luma chain and chroma chain each run on
// `xg` workgroups of W waves (W = 4: one wave per SIMD, on xg CUs); a wave claims its chain's next row
// from a global ticket (one atomic per row, taken only by a running wave), so a row's predecessor is
// always held by a wave that already runs, whatever part of the chain's workgroups the dispatcher has
// placed (other lanes' or contexts' kernels may hold the rest of the GPU); row progress and the rows'
// bottom lines live in global memory (XgBuf), read and written with agent-scope atomics (coherent across
// the XCDs' L2s), and a CTU's row above is copied from there into the wave's ytop / ctop.  One line per
// CTU row (no parity reuse): a CTU's publish never waits for the row below to have read the line.
struct XgBuf {
    int* prog;                   // [pic][comp][row]: seq << 16 | CTUs done
    uint8_t* lines;              // [pic][comp][row][(wc + 2) * CTB]: the row's bottom samples at + CTB
                                 // (chroma: Cb at + CTB / 2, Cr (wc + 2) * CTB / 2 further)
    int* ticket;                 // [pic][comp]: the chain's next unclaimed row (cleared per run with prog)
    int xg, seq;                 // workgroups per chain; this run's tag
};

template <int W, int WPE, bool XG = false, bool TRCHK = false, typename T = uint8_t>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE)))
void intra_rows_kernel(const DevPic* __restrict__ pics,
                                                           const int16_t* __restrict__ pool,
                                                           const int16_t* __restrict__ resid,
                                                           Geo g, int n_pics, int fs_count, int lead,
                                                           int* __restrict__ err_flag,
                                                           int* __restrict__ dbg, int split, XgBuf xb) {
    // debug trace (P265R_DEBUG_DIAG builds, P265R_DEBUG_SYNC=1): host-mapped words, one per wave
#if defined(P265R_DEBUG_DIAG) && !defined(P265R_DBG_NOTRACE)
#define P265R_TRACE(code) do { if (dbg && lane == 0) __hip_atomic_store(dbg + blockIdx.x * W + wave, (code), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#else
#define P265R_TRACE(code) do { } while (0)
#endif
    static_assert(sizeof(T) == 1 || !XG, "the cross-group layout is 8-bit only");
    constexpr int PB = (int)sizeof(T);                // bytes per sample
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    RowCtrl& ctl = *reinterpret_cast<RowCtrl*>(smem);
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    // row units per picture: (cy, luma), (cy, chroma); split: two workgroups per picture, workgroup
    // parity = the component chain it runs (4:2:0 intra never couples them: no cross-workgroup sync)
    const int units = split ? g.hc : 2 * g.hc;
    // progress words: one per (slot, CTU row, component) in either mode (host: launch_rows_w lds_of)
    const int prog_bytes = (fs_count * 2 * g.hc * 4 + 15) & ~15;
    int* prog = reinterpret_cast<int*>(smem + 256);
    WaveLdsT<T>& L = reinterpret_cast<WaveLdsT<T>*>(smem + 256 + prog_bytes)[wave];
    const int line_bytes = g.w + 2 * g.cw;            // Y | Cb | Cr bottom sample rows (samples)
    T* lines = reinterpret_cast<T*>(smem + 256 + prog_bytes + W * sizeof(WaveLdsT<T>));
    const int maxv = (1 << g.bd[0]) - 1;              // BitDepth: luma = chroma (p265r_create)

    uint32_t* const atab = reinterpret_cast<uint32_t*>(lines + (size_t)fs_count * 2 * line_bytes);   // AngTab4
    if (threadIdx.x == 0) {
        ctl.next_row = 0; ctl.error = 0;
        ctl.cu_slot = -1; ctl.cu_rank = 0;
        if (g.fair) {
            uint32_t xcc, hwid;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
            const int key = (int)((xcc & 7u) * 256u + ((hwid >> 8) & 255u));      // CU_ID, SH_ID, SE_ID (3 bits)
            RowCuSlot* cs = reinterpret_cast<RowCuSlot*>(err_flag + 64) + key;
            ctl.cu_slot = key;
            ctl.cu_rank = __hip_atomic_fetch_add(&cs->count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1;
        }
    }
    if (threadIdx.x < 32) ctl.done[threadIdx.x] = 0;
#ifdef P265R_JOB_STATS
    if (threadIdx.x < 28) ctl.pad[threadIdx.x] = 0;
#endif
    for (int i = threadIdx.x; i < fs_count * 2 * g.hc; i += 64 * W) prog[i] = -1;
    for (int i = threadIdx.x; i < 35 * 16; i += 64 * W) atab[i] = angtab_entry<2>(i >> 4, i & 15);
    if (P265R_ANGTAB8)
        for (int i = threadIdx.x; i < 35 * 64; i += 64 * W) atab[35 * 16 + i] = angtab_entry<3>(i >> 6, i & 63);
    __syncthreads();
#if P265R_PIPE_PRIO > 0
    // A/B: the pipelined build's waves issue ahead of the other lanes' residual / prep / SAO waves
    if (W == 8 && !split) __builtin_amdgcn_s_setprio(P265R_PIPE_PRIO);
#endif

    const int G = split ? (int)(gridDim.x >> 1) : (int)gridDim.x;
    const int b = split ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const int split_comp = (int)(blockIdx.x & 1u);
    const int n_my = b < n_pics ? (n_pics - b + G - 1) / G : 0;
    const int rows_total = XG ? g.hc : n_my * units;
    // XG: this workgroup's chain (picture, component)
    const int xg_chain = XG ? (int)blockIdx.x / xb.xg : 0;
    const size_t xg_row_bytes = (size_t)(g.wc + 2) << g.ctb_log2;
    const int ctb = 1 << g.ctb_log2;
    // bounded spin-wait on an LDS word; false = gave up (error published, caller bails out).
    // Every condition is made wave-uniform (readfirstlane) so the loops are scalar loops.
#ifdef P265R_DEBUG_DIAG
    long long t_wait = 0;
    const long long t_begin = __builtin_amdgcn_s_memtime();
#define P265R_WAIT_T0 const long long t0 = __builtin_amdgcn_s_memtime()
#define P265R_WAIT_ADD t_wait += __builtin_amdgcn_s_memtime() - t0
#else
#define P265R_WAIT_T0 do { } while (0)
#define P265R_WAIT_ADD do { } while (0)
#endif
    auto wait_until = [&](auto ready) -> bool {
        P265R_WAIT_T0;
        for (int spins = 0; spins < (1 << 24); ++spins) {
            if (spins == 0 && __builtin_amdgcn_readfirstlane((int)ready())) return true;
            if (__builtin_amdgcn_readfirstlane((int)ready())) { P265R_WAIT_ADD; return true; }
            if (__builtin_amdgcn_readfirstlane(XG ? __hip_atomic_load(gptr(err_flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : __hip_atomic_load(&ctl.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
                return false;                               // (XG: any chain's failure ends every wait)
            __builtin_amdgcn_s_sleep(XG ? P265R_XG_SLEEP : P265R_SPIN_SLEEP);   // 64 cycles per unit; each poll costs issue slots
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
        int r;
        if constexpr (XG) {
            // the chain's global ticket (the rows of a chain are claimed in order by running waves)
            r = __hip_atomic_fetch_add(gptr_w(xb.ticket) + xg_chain, lane == 0 ? 1 : 0, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            r = __builtin_amdgcn_readlane(r, 0);
        } else {
            r = __hip_atomic_fetch_add(&ctl.next_row, lane == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        r = __builtin_amdgcn_readfirstlane(r);
        if (r >= rows_total || failed) break;
        P265R_TRACE(2 | (r << 8));
        if (!XG && g.fair) {
            // publish the rows this workgroup has dequeued; priority 1 while behind the partner
            const int key = __builtin_amdgcn_readfirstlane(ctl.cu_slot), rank = __builtin_amdgcn_readfirstlane(ctl.cu_rank);
            RowCuSlot* cs = reinterpret_cast<RowCuSlot*>(err_flag + 64) + key;
            if (lane == 0) __hip_atomic_store(&cs->prog[rank], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int other = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&cs->prog[rank ^ 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (r < other) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        const int j = r / units, rem = r - j * units;
        // queue order inside a picture: the luma chain (the longer one) leads by `lead` rows:
        // L0 .. L(d-1), then L(d) C0 L(d+1) C1 ..., then the remaining chroma rows.  Either
        // chain's rows stay in order, so a dequeued row's predecessor is always held by a wave.
        int cy, comp;                                      // comp 0: luma chain, 1: chroma (Cb + Cr)
        if (XG) {
            cy = r; comp = xg_chain & 1;
        } else if (split) {
            cy = rem; comp = split_comp;
        } else {
            const int d = min(lead, g.hc);
            if (rem < d) {
                cy = rem; comp = 0;
            } else {
                const int k = rem - d, pairs = 2 * (g.hc - d);
                if (k < pairs) { cy = (k & 1) ? (k >> 1) : d + (k >> 1); comp = k & 1; }
                else { cy = g.hc - d + (k - pairs); comp = 1; }
            }
        }
        const int slot = j % fs_count, gen = j / fs_count;
        const DevPic* Pp = XG ? pics + (xg_chain >> 1) : pics + b + j * G;
        const p265r_ctu* ctus = uniform(gload(&Pp->ctus));
        const IntraJob* jobs = uniform(gload(&Pp->jobs));
        const uint32_t* jcount = uniform(gload(&Pp->jcount));
        const int zero_res = __builtin_amdgcn_readfirstlane((int)*gptr(&Pp->zero_off));   // the zero block
        // this picture's CTU grid and plane size (a ragged batch: DevPic::wh); the row queue, progress
        // words and line buffers keep the context's layout
        int pwc = g.wc, phc = g.hc, pw = g.w, ph = g.h;
        if (P265R_RAGGED && g.ragged) {
            const Geo pg = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane(*gptr(&Pp->wh)));
            pwc = pg.wc; phc = pg.hc; pw = pg.w; ph = pg.h;
        }
        // picture slot reuse: every row of picture j waits until picture j - fs_count (the
        // slot's previous occupant) has completed all its rows; those rows were dequeued
        // earlier and are held by running waves, so this wait always ends.
        if (!XG && !wait_until([&] {
                return __hip_atomic_load(&ctl.done[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= gen * units;
            })) { failed = true; break; }
        P265R_TRACE(3 | (r << 8));
        if (cy >= phc) {                                   // a row below this (smaller) picture: nothing to do
            __hip_atomic_fetch_add(&ctl.done[slot], lane == 0 ? 1 : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            continue;
        }
        T* line_cur = lines + (size_t)(slot * 2 + (cy & 1)) * line_bytes;
        const T* line_up = lines + (size_t)(slot * 2 + ((cy & 1) ^ 1)) * line_bytes;
        int* my_prog = &prog[(slot * g.hc + cy) * 2 + comp];
        const int* up_prog = &prog[(slot * g.hc + (cy > 0 ? cy - 1 : 0)) * 2 + comp];
        const int tag = ((XG ? xb.seq : j) & 0xffff) << 16;
        // XG: this chain's progress words and lines (global)
        P265R_GLOBAL int* xg_prog = XG ? gptr_w(xb.prog) + (size_t)xg_chain * g.hc : nullptr;
        P265R_GLOBAL uint8_t* xg_line = XG ? gptr_w(xb.lines) + (size_t)xg_chain * g.hc * xg_row_bytes : nullptr;
        if constexpr (XG) {
            if (lane == 0) __hip_atomic_store(xg_prog + cy, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(my_prog, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }

        // CTU header (first TB index | job counts) loaded one CTU ahead, and the next CTU's first
        // 64 job records loaded right after this CTU's last job: a CTU then starts with its
        // records in registers (one dependent round trip, its first residual, instead of three)
        // (jcount: four words per CTU -- the job counts, each list's first job that reads the top-right
        // CTU, one past each list's last job in the bottom-left quadrant, intra_prep.h)
        auto hdr_load = [&](int a) {
            const uint4 jp = gload(reinterpret_cast<const uint4*>(jcount + 4 * a));
            return make_uint4(gload(reinterpret_cast<const uint2*>(ctus + a)).x, jp.x, jp.y, jp.z);
        };
        uint4 hdr_n = hdr_load(cy * pwc);
#ifndef P265R_ROW_PRIO
#define P265R_ROW_PRIO 3
#endif
#if P265R_ROW_PRIO > 0
        // split mode (small batches, one chain per workgroup): the upper rows of a picture issue
        // first -- they lead the wavefront that every lower row trails (C5: one unit's row kernel
        // 2.595 -> 2.567 ms with 8-row priority bands, 2 reps; 4-row bands 2.60)
        if (split) {
            const int pr = __builtin_amdgcn_readfirstlane(cy >> P265R_ROW_PRIO);
            if (pr == 0) __builtin_amdgcn_s_setprio(3);
            else if (pr == 1) __builtin_amdgcn_s_setprio(2);
            else if (pr == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
#endif
        uint4 rec0 = make_uint4(0, 0, 0, 0);
        uint2 rec1 = make_uint2(0, 0);
        bool pre = false;                                  // rec0 / rec1 hold this CTU's first records
        // XG: the next CTU's first job record and residual, fetched after this CTU's publish (its
        // residual load then overlaps the next CTU's dependency poll and row-above copy)
        uint32_t pj0 = 0, pj1 = 0, pj2 = 0, pj3 = 0, pj4 = 0, pj5 = 0;
        u32x2_t rn_pre = {0u, 0u};
        bool pre_issued = false;
        for (int cx = 0; cx < pwc; ++cx) {
            // ---- wait for the row above -------------------------------------------------
            // The CTU above (1-CTU lag) before the CTU starts; the top-right CTU (2-CTU lag) before the
            // first job that reads it (prep: per CTU and chain, `tr`) and, read or not, before this CTU's
            // bottom row goes into the line buffer: that overwrites the row above the CTU for the row
            // below the one above, which reads it up to its CTU cx + 1 (the corner)
            const int x0 = cx << g.ctb_log2, y0 = cy << g.ctb_log2;
            const int addr = cy * pwc + cx;
            // this CTU's job list (intra_prep_kernel): first job = its first TB index; job counts:
            // luma in bits 0..15, chroma (listed first) in bits 16..31 (intra_prep.h)
            const uint32_t tb_begin = (uint32_t)__builtin_amdgcn_readfirstlane(hdr_n.x);
            const uint32_t jc = (uint32_t)__builtin_amdgcn_readfirstlane(hdr_n.y);
            const uint32_t trw = (uint32_t)__builtin_amdgcn_readfirstlane(hdr_n.z);
            const uint32_t brw = XG ? (uint32_t)__builtin_amdgcn_readfirstlane(hdr_n.w) : 0u;
            if (cx + 1 < pwc) hdr_n = hdr_load(addr + 1);    // in flight during this CTU
            const int n_chroma = (int)(jc >> 16);
            const int nt = comp ? n_chroma : (int)(jc & 0xffffu);
            // (deferred only in the latency layouts -- XG and the W = 16 split: the throughput builds keep the
            // 2-CTU-lag start, whose job loop has no per-job test; measured: pipelined step 1.7 % slower with it)
            constexpr bool kDefer = P265R_TR_DEFER && (XG || W == 16);
            const int tr = !kDefer ? 0 : comp ? (int)(trw >> 16) : (int)(trw & 0xffffu);   // first job reading the top-right CTU
            const bool tr_ctu = cy > 0 && cx + 1 < pwc;        // a top-right CTU exists (else nothing to wait for)
            // XG progress counts half CTUs (2 per finished CTU, +1 once the left half of the next one's bottom
            // row is out): at CTB 64 a TB reaches at most half a CTB into the top-right CTU (TBs <= 32 luma,
            // 16 chroma), whose left bottom half is final after its bottom-left quadrant's jobs (prep: `br`)
            const bool halfp = XG && g.ctb_log2 == 6;
            const int u = XG ? 2 : 1;                          // progress units per CTU
            const int need_tr = halfp ? 2 * (cx + 1) + 1 : u * min(cx + 2, pwc);
            const int br = XG ? (comp ? (int)(brw >> 16) : (int)(brw & 0xffffu)) : 0;
            auto up_ready = [&](int need) {
                const int v = XG ? __hip_atomic_load(xg_prog + (cy - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : __hip_atomic_load(up_prog, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                return (v & 0xffff0000) == tag && (v & 0xffff) >= need;
            };
            // XG: the row above's line, x in [x0 + 4 k0 - 4, x0 + 4 k1 - 4) (component units), into ytop /
            // ctop [4 k0, 4 k1): one dword per lane (chroma: lanes 0-31 Cb, 32-63 Cr), agent-scope loads
            // after the progress word that covers them (the writer completed them before storing it)
            const int cts = ctb >> comp;
            auto xg_copy = [&](int k0, int k1) {
                const int h = comp ? lane >> 5 : 0, k = k0 + (comp ? lane & 31 : lane);
                if (k < k1) {
                    const P265R_GLOBAL uint8_t* src = xg_line + (size_t)(cy - 1) * xg_row_bytes +
                                                      (size_t)h * (xg_row_bytes >> 1) + cts + (x0 >> comp) - 4 + 4 * k;
                    const uint32_t v = __hip_atomic_load(reinterpret_cast<const P265R_GLOBAL uint32_t*>(src),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    T* dst = comp ? &L.ctop[h][4 * k] : &L.ytop[4 * k];
                    *reinterpret_cast<uint32_t*>(dst) = v;
                }
                wave_sync();
            };
            auto wait_up = [&](int need) { return wait_until([&] { return up_ready(need); }); };
            // XG: the bottom row's first nd dwords of this chain's plane(s) into line cy, completed, then the
            // progress word 2 cx + half (half = 1: the left half, mid-CTU; the CTU's end writes the whole row)
            auto xg_publish = [&](int nd, int half) {
                const int h = comp ? lane >> 5 : 0, k = comp ? lane & 31 : lane;
                const int hv = min(cts, (comp ? ph >> 1 : ph) - (y0 >> comp));
                if (k < nd) {
                    const T* src = (comp ? L.c[h] : L.y) + (hv - 1) * (comp ? 32 : 64) + 4 * k;
                    P265R_GLOBAL uint8_t* dl = xg_line + (size_t)cy * xg_row_bytes + (size_t)h * (xg_row_bytes >> 1) +
                                               cts + (x0 >> comp) + 4 * k;
                    __hip_atomic_store(reinterpret_cast<P265R_GLOBAL uint32_t*>(dl), *reinterpret_cast<const uint32_t*>(src),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(xg_prog + cy, tag | (2 * cx + half), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
            const bool early = tr_ctu && tr == 0;               // the first job already reads the top-right CTU
            bool tr_done = !tr_ctu || early;                    // waited for the top-right CTU
            if (cy > 0 && !wait_up(early ? need_tr : u * (cx + 1))) { failed = true; break; }
            // (XG) the top-right part of the row above: its left half at CTB 64, all of it otherwise
            const int tr_k1 = (halfp ? cts + cts / 2 : 2 * cts) / 4 + 1;
            if (XG && cy > 0) {
                if (TRCHK && tr_ctu) {
                    // self-check of prep's `tr` (and of the half-CTB reach): the whole top-right part of the copy
                    // holds a position-dependent pattern until its wait (the right half at CTB 64 for good),
                    // so a job that read it early would break parity deterministically rather than by timing
                    const int h = comp ? lane >> 5 : 0, k = cts / 4 + 1 + (comp ? lane & 31 : lane);
                    if (k < 2 * cts / 4 + 1)
                        *reinterpret_cast<uint32_t*>(comp ? &L.ctop[h][4 * k] : &L.ytop[4 * k]) = 0xa55a3cc3u ^ (uint32_t)(k * 0x01030507);
                    wave_sync();
                }
                xg_copy(0, early ? tr_k1 : cts / 4 + 1);
            }
            P265R_TRACE(4 | (cx << 8) | (r << 16));
            const IntraJob* jl = jobs + tb_begin + (comp ? 0 : n_chroma);
            // line buffer row above, per lane component (pair jobs: lanes 32-63 are Cr); XG: the wave's copy
            const T* ltop_l = XG ? &L.ytop[4] : line_up + x0;
            const T* ltop_c = XG ? &L.ctop[lane >> 5][4] : line_up + g.w + (lane >> 5) * g.cw + (x0 >> 1);
            const T* ltop_cb = XG ? &L.ctop[0][4] : line_up + g.w + (x0 >> 1);
            const uint32_t cr_off = XG ? (uint32_t)(sizeof(L.ctop[0]) / PB) : (uint32_t)g.cw;   // Cb -> Cr in the row above (samples)

            // residual of job t: two aligned 16-B loads per lane (fixed shape, pools padded
            // by 64 B), issued while job t-1 is processed.  TB offsets are multiples of 16.
            auto res_addr = [&](uint32_t w0, uint32_t w3, uint32_t w4) {
                const int lg = (int)((w0 >> 13) & 3u) + 2;
                const bool pr = (w0 >> 15) & 3u;
                const int h = pr ? (lane >> 5) : 0;
                const int hl = pr ? (lane & 31) : lane;
                const int ls = 2 * lg - (pr ? 5 : 6);
                const int S = ls > 0 ? (1 << ls) : 1;
                const int sidx = hl * S < (1 << (2 * lg)) ? hl * S : 0;
                return reinterpret_cast<const uint4*>(resid + P265R_RI((int)(h ? w4 : w3)) + (sidx & ~7));
            };
            // fast jobs (J5_FAST): one residual sample per lane (2-B load); w3 / w4 already point
            // at the pool, the residual or the zero block, and lanes past the TB read padding
            auto res_fast = [&](uint32_t w0, uint32_t w3, uint32_t w4) {
                const bool pr = (w0 >> 15) & 3u;
                return resid + P265R_RI((int)(pr && lane >= 32 ? w4 : w3)) + (pr ? (lane & 31) : lane);
            };
            // job records (24 B): 64 at a time into six VGPRs per lane, read per job with v_readlane
            // (scalar loads were measured slower: their lgkmcnt waits serialise with the LDS
            // traffic of the job)
            struct JobS { uint32_t w0, w1, w2, w3, w4, w5; };
            auto refill = [&](int base) {
                if (base + lane < nt) { rec0 = ld16(&jl[base + lane].w[0]); rec1 = ld8(&jl[base + lane].w[4]); }
                else { rec0 = make_uint4(0, 0, 0, 0); rec1 = make_uint2(0, 0); }
            };
            auto sjob = [&](int i) {
                const int l = i & 63;
                auto rl = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane(v, l); };
                return JobS{rl(rec0.x), rl(rec0.y), rl(rec0.z), rl(rec0.w), rl(rec1.x), rl(rec1.y)};
            };
            // prefetched residual of the next job: one sample per lane (fast / quad jobs; chroma: a
            // Cb | Cr << 16 pair) in rn.x, a 16x16 job's four samples in rn.  General jobs
            // (32x32 luma, 16x16 chroma, PCM, non-contiguous availability: ~2 % of the jobs) load their
            // own 32 B per lane when they start: prefetching them too kept eight more VGPRs live
            // across the loop and cost ~10 register copies per job
            u32x2_t rn = {0u, 0u};
            auto issue = [&](const JobS& j, int ji) -> u32x2_t {   // residual loads of job j (index ji)
                if (j.w5 & J5_QUAD) {                       // quads: residual = w3 + 16 * code (15: the zero block)
                    const int q = ((lane >> 4) & 2) | ((lane >> 2) & 1);    // sub-TB of sample (x, y) of the 8x8 region
                    const int i = ((lane >> 1) & 12) + (lane & 3);          // sample index in the 4x4 sub-TB
                    auto at = [&](uint32_t code) { return P265R_RI(code == 15u ? zero_res : (int)j.w3 + (int)(code << 4)) + i; };
                    if ((j.w0 >> 15) & 3u) {                                // chroma: Cb | Cr << 16, codes at 8q + 4h
                        const uint32_t codes = j.w4 >> (8 * q);
                        const uint32_t cb = (uint16_t)*gptr(resid + at(codes & 15u));
                        const uint32_t cr = (uint16_t)*gptr(resid + at((codes >> 4) & 15u));
                        return u32x2_t{cb, cr};     // packed at use: no wait here
                    }
                    return u32x2_t{(uint32_t)(int)*gptr(resid + at((j.w4 >> (4 * q)) & 15u)), 0u};
                } else if ((j.w5 & J5_FAST) && ((j.w0 >> 13) & 15u) == 13u) { // Cb+Cr 8x8: Cb | Cr << 16 of sample lane
                    const uint32_t cb = (uint16_t)*gptr(resid + P265R_RI((int)j.w3) + lane);
                    const uint32_t cr = (uint16_t)*gptr(resid + P265R_RI((int)j.w4) + lane);
                    return u32x2_t{cb, cr};     // packed at use: no wait here
                } else if ((j.w5 & J5_FAST) && ((j.w0 >> 13) & 3u) == 2u) { // 16x16 luma: 4 samples per lane
                    const u32x2_t d = *reinterpret_cast<const P265R_GLOBAL u32x2_t*>(gptr(resid + P265R_RI((int)j.w3) + 4 * lane));
                    return d;
                } else if (j.w5 & J5_FAST) {
                    return u32x2_t{(uint32_t)(int)*gptr(res_fast(j.w0, j.w3, j.w4)), 0u};
                }
                return u32x2_t{0u, 0u};
            };
            JobS cur{0, 0, 0, 0, 0, 0};
            if (nt) {
                if (XG && pre_issued) {
                    cur = JobS{pj0, pj1, pj2, pj3, pj4, pj5};
                    rn = rn_pre;
                } else {
                    if (!pre) refill(0);
                    cur = sjob(0);
                    rn = issue(cur, 0);
                }
            }
            pre = false;
            pre_issued = false;
            // the top-right wait before job tr (the row above the CTU suffices for the jobs before it)
            const int t_trw = tr_done || tr >= nt ? -1 : tr;
            const int t_half = halfp && br < nt ? br : -1;     // XG: publish the bottom row's left half first
            if (TRCHK && t_half >= 0) {
                // self-check of prep's `br`: the bottom row's left half starts poisoned (no job reads it before
                // writing it: unavailable samples) and the CTU's final publish leaves that half of the line to
                // the half-CTU publish alone, so a bottom-left job placed after `br` breaks parity on every run
                const int h = comp ? lane >> 5 : 0, k = comp ? lane & 31 : lane;
                const int hv = min(cts, (comp ? ph >> 1 : ph) - (y0 >> comp));
                if (k < cts / 8)
                    *reinterpret_cast<uint32_t*>((comp ? L.c[h] : L.y) + (hv - 1) * (comp ? 32 : 64) + 4 * k) =
                        0x3cc3a55au ^ (uint32_t)((cx * 64 + k) * 0x01030507);
                wave_sync();
            }
#ifdef P265R_JOB_UNROLL
#pragma unroll P265R_JOB_UNROLL
#endif
            for (int t = 0; t < nt; ++t) {
                P265R_MARK("job_top");
                if (t == t_trw) {                       // (a failed wait runs on; the loop exits after the job)
                    failed = !wait_up(need_tr);
                    if (XG) xg_copy(cts / 4 + 1, tr_k1);
                    tr_done = true;
                }
                if (XG && t == t_half) xg_publish(cts / 8, 1);
#ifdef P265R_JOB_STATS
                const long long tj0 = __builtin_amdgcn_s_memtime();
#endif
                // next job's record and residual are fetched before this job runs; this job
                // works on copies of its own (measured: issuing after the job is slower)
                const uint32_t w0 = cur.w0, w1 = cur.w1, w2 = cur.w2, w3 = cur.w3, w4 = cur.w4, w5 = cur.w5;
                const int c16 = (int)rn.x, c16m = (int)rn.y;
                if (t + 1 < nt) {
                    if (((t + 1) & 63) == 0) refill(t + 1);
#if P265R_LATE_REC
                    // the next record's residual fields only (its whole record is read after this job, into
                    // the registers this one held: no per-job copies of the six record words)
                    const int l = (t + 1) & 63;
                    auto rl = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane(v, l); };
                    rn = issue(JobS{rl(rec0.x), 0u, 0u, rl(rec0.w), rl(rec1.x), rl(rec1.y)}, t + 1);
#else
                    cur = sjob(t + 1);
                    rn = issue(cur, t + 1);
#endif
                }
                const int sel = (int)((w0 >> 13) & 3u) | (((w0 >> 15) & 3u) ? 4 : 0);
                P265R_MARK("job_dispatch");
#ifdef P265R_PAD_SALU
                {   // A/B probe: P265R_PAD_SALU dependent scalar adds per job (issue-bound test)
                    uint32_t z = w0;
#pragma unroll
                    for (int q = 0; q < P265R_PAD_SALU; ++q) asm volatile("s_mov_b32 %0, %0" : "+s"(z));   // (s_mov: leaves SCC alone)
                    asm volatile("" :: "s"(z));
                }
#endif
#ifdef P265R_PAD_VALU
                {   // A/B probe: P265R_PAD_VALU dependent vector adds per job
                    uint32_t z = (uint32_t)lane;
#pragma unroll
                    for (int q = 0; q < P265R_PAD_VALU; ++q) asm volatile("v_add_u32 %0, 1, %0" : "+v"(z));
                    asm volatile("" :: "v"(z));
                }
#endif
                // Opaque copies of the lane id and the LDS bases: keeps the compiler from
                // hoisting every template's lane-derived constants out of the job loop
                // (7 inlined instances would otherwise hold them all live: ~150 VGPRs).
                int ln;
                asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
                uint32_t lbase, tl, tc, tcb, tab;
#if P265R_OPAQUE_S
                asm volatile("s_mov_b32 %0, %1" : "=s"(lbase) : "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&L)));
                asm volatile("s_mov_b32 %0, %1" : "=s"(tab) : "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)atab)));
                asm volatile("s_mov_b32 %0, %1" : "=s"(tcb) : "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ltop_cb)));
#else
                lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&L);
                tab = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)atab);
                tcb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ltop_cb);
#endif
                asm volatile("v_mov_b32 %0, %1" : "=v"(tl) : "v"((uint32_t)(uintptr_t)ltop_l));
                asm volatile("v_mov_b32 %0, %1" : "=v"(tc) : "v"((uint32_t)(uintptr_t)ltop_c));
                WaveLdsT<T>& LL = *reinterpret_cast<WaveLdsT<T>*>(lds_ptr(lbase));
                const T* tlp = reinterpret_cast<const T*>(lds_ptr(tl));
                const T* tcp = reinterpret_cast<const T*>(lds_ptr(tc));
                // (8 bits: the constant 255 folds into every job function, as before the 16-bit path)
                const int mv = PB == 1 ? 255 : maxv;
                if (w5 & J5_QUAD) {
                    // (the latency layout reads the quad stages' references composed: one round trip per stage)
                    constexpr bool kComp = XG && P265R_QUAD_COMPOSED;
                    if ((w0 >> 15) & 3u) recon_quad<true, T, kComp>(lbase, tcb, cr_off, w0, w1, w2, tab, (int)((uint32_t)c16 | (uint32_t)c16m << 16), ln, mv);
                    else recon_quad<false, T, kComp>(lbase, tl, 0u, w0, w1, w2, tab, c16, ln, mv);
                } else if (w5 & J5_FAST) {
                    switch (sel) {
                        case 0: recon_fast<2, false, T>(lbase, tl, w0, w1, w5, c16, ln, tab, mv); break;
                        case 1: recon_fast<3, false, T>(lbase, tl, w0, w1, w5, c16, ln, tab, mv); break;
                        case 2: recon_fast16<T>(lbase, tl, w0, w1, w5, make_uint4((uint32_t)c16, (uint32_t)c16m, 0u, 0u), ln, mv); break;
                        case 5: recon_cfast8<T>(lbase, tcb, cr_off, w0, w1, w5, (int)((uint32_t)c16 | (uint32_t)c16m << 16), ln, tab, mv); break;
                        default: recon_fast<2, true, T>(lbase, tc, w0, w1, w5, c16, ln, tab, mv); break;
                    }
                } else {
                  const uint4* ra_p = res_addr(w0, w3, w4);
                  const uint4 ca = ld16(ra_p), cb = ld16(ra_p + 1);
                  switch (sel) {
                    case 0: recon_job<2, false, T>(LL, tlp, w0, w1, w2, ca, cb, ln, mv); break;
                    case 1: recon_job<3, false, T>(LL, tlp, w0, w1, w2, ca, cb, ln, mv); break;
                    case 2: recon_job<4, false, T>(LL, tlp, w0, w1, w2, ca, cb, ln, mv); break;
                    case 3: recon_job<5, false, T>(LL, tlp, w0, w1, w2, ca, cb, ln, mv); break;
                    case 4: recon_job<2, true, T>(LL, tcp, w0, w1, w2, ca, cb, ln, mv); break;
                    case 5: recon_job<3, true, T>(LL, tcp, w0, w1, w2, ca, cb, ln, mv); break;
                    default: recon_job<4, true, T>(LL, tcp, w0, w1, w2, ca, cb, ln, mv); break;
                  }
                }
                P265R_MARK("job_end");
#ifdef P265R_JOB_STATS
                {   // per job class: cycles (/16) and count, summed in LDS (RowCtrl::pad), P265R_DEBUG_SYNC prints
                    const int jc = (w5 & J5_QUAD) ? (((w0 >> 15) & 3u) ? 1 : 0)
                                 : (w5 & J5_FAST) ? (sel == 5 ? 6 : (sel >= 4 ? 5 : 2 + sel)) : 7 + sel;
                    const int dt = (int)((__builtin_amdgcn_s_memtime() - tj0) >> 4);
                    if (lane == 0) {
                        __hip_atomic_fetch_add(&ctl.pad[2 * jc], dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&ctl.pad[2 * jc + 1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
#endif
#if P265R_LATE_REC
                if (t + 1 < nt) cur = sjob(t + 1);
#endif
            }
            if (failed) break;                             // (wait_until published the error)
            // before this CTU's bottom row goes into the line buffer (whether or not a job read it; XG:
            // one line per row, nothing to overwrite)
            if (!XG && !tr_done && !wait_up(cx + 2)) { failed = true; break; }

            int nt2 = 0;
            if (cx + 1 < pwc) {                            // the next CTU's first 64 job records
                const uint32_t tb2 = (uint32_t)__builtin_amdgcn_readfirstlane(hdr_n.x);
                const uint32_t jc2 = (uint32_t)__builtin_amdgcn_readfirstlane(hdr_n.y);
                const int nc2 = (int)(jc2 >> 16);
                nt2 = comp ? nc2 : (int)(jc2 & 0xffffu);
                const IntraJob* jl2 = jobs + tb2 + (comp ? 0 : nc2);
                if (lane < nt2) { rec0 = ld16(&jl2[lane].w[0]); rec1 = ld8(&jl2[lane].w[4]); }
                else { rec0 = make_uint4(0, 0, 0, 0); rec1 = make_uint2(0, 0); }
                pre = true;
            }
            P265R_TRACE(5 | (cx << 8) | (r << 16));
            // ---- publish the CTU: planes (HBM), bottom line (LDS), right column (LDS) ----------
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                if ((c == 0) != (comp == 0)) continue;          // this chain's planes only (wave-uniform)
                const int sub = c ? 1 : 0;
                const int cs = ctb >> sub;
                const int Wd = c ? pw >> 1 : pw, Ht = c ? ph >> 1 : ph;
                const int xb = x0 >> sub, yb = y0 >> sub;
                const int wv = min(cs, Wd - xb), hv = min(cs, Ht - yb);
                const T* src = c == 0 ? L.y : (c == 1 ? L.c[0] : L.c[1]);
                const int ist = c ? 32 : 64;
                P265R_GLOBAL T* plane = reinterpret_cast<P265R_GLOBAL T*>(gptr_w(uniform(gload(&Pp->rec[c]))));
                const int st = (c ? g.stride[1] : g.stride[0]);      // samples
                constexpr int LC = PB == 1 ? 4 : 3;                    // log2 samples per 16-B chunk
                if (cs * PB >= 16) {
                    // 2^lg 16-B chunks per CTB row (one ds_read_b128 + one 16-B global store per
                    // lane and chunk).  A chunk that straddles the picture's right edge is stored whole:
                    // the plane rows are padded to 64 B (stride >= xb + cs), and nothing reads the
                    // padding (downloads copy the width, SAO / deblocking clamp to it)
                    const int lg = g.ctb_log2 - sub - LC;
                    for (int e = lane; e < (hv << lg); e += 64) {
                        const int yy = e >> lg, xx = (e & ((1 << lg) - 1)) << LC;
                        if (xx < wv)
                            *reinterpret_cast<P265R_GLOBAL u32x4_t*>(plane + (size_t)(yb + yy) * st + xb + xx) =
                                *reinterpret_cast<const u32x4_t*>(src + yy * ist + xx);
                    }
                } else {
                    // 2^lg words (4 bytes) per CTB row, no per-word division; the words past a
                    // picture's right edge idle
                    const int lg = g.ctb_log2 - sub - (LC - 2);
                    for (int e = lane; e < (hv << lg); e += 64) {
                        const int yy = e >> lg, xx = (e & ((1 << lg) - 1)) << (LC - 2);
                        if (xx < wv)
                            *reinterpret_cast<P265R_GLOBAL uint32_t*>(plane + (size_t)(yb + yy) * st + xb + xx) =
                                *reinterpret_cast<const uint32_t*>(src + yy * ist + xx);
                    }
                }
                if constexpr (XG) {                            // bottom row, whole dwords (past the edge: unread)
                    P265R_GLOBAL uint8_t* dl = xg_line + (size_t)cy * xg_row_bytes + (c == 2 ? xg_row_bytes >> 1 : 0) + cs + xb;
                    // (the check instance: the left half stays what the half-CTU publish wrote)
                    if (lane < cs / 4 && !(TRCHK && t_half >= 0 && lane < cs / 8))
                        __hip_atomic_store(reinterpret_cast<P265R_GLOBAL uint32_t*>(dl) + lane,
                                           *reinterpret_cast<const uint32_t*>(src + (hv - 1) * ist + 4 * lane),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    T* lc = line_cur + (c == 0 ? 0 : (c == 1 ? g.w : g.w + g.cw)) + xb;
                    if (lane < wv) lc[lane] = src[(hv - 1) * ist + lane];
                }
                T* lf = c == 0 ? L.yleft : (c == 1 ? L.cleft[0] : L.cleft[1]);
                if (lane < hv) lf[lane] = src[lane * ist + wv - 1];
            }
            if constexpr (XG) {
                // the line's stores complete (at the agent's coherence point) before the progress word
                // that announces them; the plane stores are read only by later kernels
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(xg_prog + cy, tag | (2 * (cx + 1)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (P265R_XG_PRE && pre && nt2 > 0) {     // (the wait above also covered the record loads)
                    const JobS c0 = sjob(0);
                    pj0 = c0.w0; pj1 = c0.w1; pj2 = c0.w2; pj3 = c0.w3; pj4 = c0.w4; pj5 = c0.w5;
                    rn_pre = issue(c0, 0);
                    pre_issued = true;
                }
            } else {
                __hip_atomic_store(my_prog, tag | (cx + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            wave_sync();
        }
        if (failed) break;
        __hip_atomic_fetch_add(&ctl.done[slot], lane == 0 ? 1 : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        P265R_TRACE(6 | (r << 8));
    }
    P265R_TRACE(7);
#ifdef P265R_JOB_STATS
    __syncthreads();
    if (dbg && threadIdx.x < 28)
        atomicAdd(dbg + 3 * gridDim.x * W + 2 * gridDim.x + threadIdx.x, ctl.pad[threadIdx.x]);
#endif
#ifdef P265R_DEBUG_DIAG
    if (dbg) {   // debug statistics: [total cycles, cycles in dependency waits] per wave
        const long long t_all = __builtin_amdgcn_s_memtime() - t_begin;
        const int slotw = gridDim.x * W + 2 * (blockIdx.x * W + wave);
        __hip_atomic_store(dbg + slotw, (int)(t_all >> 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dbg + slotw + 1, (int)(t_wait >> 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (wave == 0) {            // placement of the workgroup: XCC id, HW_ID (CU / SE)
            uint32_t xcc, hwid;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
            const int slotp = 3 * gridDim.x * W + 2 * blockIdx.x;
            __hip_atomic_store(dbg + slotp, (int)xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(dbg + slotp + 1, (int)hwid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
#endif
    (void)dbg;
    // all stores of this wave are issued before it ends (compiler barrier)
    asm volatile("" ::: "memory");
}

}  // namespace p265r
