// Intra job preparation: everything about a transform block that does NOT depend on
// reconstructed sample values, computed for all TBs of the batch in one fully parallel
// pass, so that the serial per-CTU chain of intra_rows_kernel only moves samples.
//
// Per TB (decode order within its CTU) the pass derives
//   * neighbour availability (6.4.1: picture edge, slice / tile of the neighbouring CTU,
//     z-scan order inside the CTB - MinTbAddrZs, pps.py:246-262 / image.py:38-73) for
//     every 4-luma-sample unit of the 4N+1 reference samples, as a bit mask in the
//     linear order of 8.4.4.2.2 (bottom-left .. corner .. top-right);
//   * the filtering decision of 8.4.4.2.3 (intraHorVerDistThres, strong-smoothing
//     candidate), intraPredAngle and invAngle (Table 8-4/8-5);
//   * where its residual lives (coefficient pool for bypass/PCM, residual pool else);
// and pairs every Cb TB with the Cr TB of the same TU (4:2:0: same position, size and
// mode, decoder/tu.py:127-135), so one wave reconstructs both with its two halves.
// Replaces the per-sample tree walks of decoder/cu.py:617-632 and intra.py:82-136.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"
#include "tables.h"

namespace p265r {

// 24-byte job record (words w0..w5; round 5: 32 -> 24 B, the quads' residuals as base + codes).
//  w0: [0,13) LDS offset of the TB origin in WaveLds (luma yr*64+xr, chroma 4096+yr*32+xr)
//      [13,15) log2-2  [15,17) component mask (0 luma, 1 Cb, 2 Cr, 3 Cb+Cr)  [17,23) mode
//      23 PCM  [24,26) filter (0 none, 1 [1 2 1], 2 strong candidate)
//      [26,28) residual in the coefficient pool (bypass/PCM) per half
//      [28,30) coded (residual non-zero) per half   30 all refs available   31 none available
//  w1: [0,8) intraPredAngle (int8)  [8,21) |invAngle| (256 for the modes without one)  21 availability bit 32
//  w2: availability bits 0..31 (unit u: k in [u*us, u*us+us) for u < L, corner u = L,
//      top units u > L; us = 4 luma / 2 chroma samples, L = 2N/us)
//  w3, w4: residual element offset of half 0 (luma / Cb) and half 1 (Cr), int32 relative to
//      the residual pool for every kind of TB: bypass/PCM samples at a negative offset into
//      the coefficient pool (DevPic::pool_rel), uncoded halves at a zero block (zero_off)
//  w5: fast-path job (intra_rows.h recon_fast*): bit 31 set for luma 4x4 .. 16x16 and Cb+Cr
//      4x4 / 8x8 pairs, not PCM, whose available reference samples form ONE contiguous run
//      [fa, la] of the linear order (or none): substitution (8.4.4.2.2) is then
//      s = Clip3(fa, la, k).  fa bits 0..7, la bits 8..15.
// Luma 4x4 QUAD job (w5 has J5_FAST | J5_QUAD): the four fast 4x4 luma TBs of one 8x8
// region (blkIdx 0..3, consecutive in decode order) as ONE job, reconstructed in four
// register-resident stages by intra_rows.h recon_quad:
//  w0: [0,13) LDS offset of the region origin  [13,17) 0  [17,23) mode q0  [23,29) mode q1
//      29 / 30: no reference available for q0 / q1
//  w1: [0,6) mode q2  [6,12) mode q3  12 / 13: none for q2 / q3  [14,19) fa q0  [19,24) la q0
//      [24,29) fa q1
//  w2: [0,5) la q1  [5,10) fa q2  [10,15) la q2  [15,20) fa q3  [20,25) la q3
//  w3: residual base offset; w4: 4-bit code per sub-TB q at bit 4q, residual = w3 + 16 * code, code 15 =
//      the zero block (DevPic::zero_off): coded 4x4 luma TBs of one class sit in decode order in
//      16-sample slots, so the region's coded sub-TBs are consecutive (else no quad)
// Chroma 4x4 QUAD job (w5 has J5_FAST | J5_QUAD, w0 component mask 3): the four fast Cb+Cr
// 4x4 pairs of one 8x8 chroma region (four consecutive TUs in decode order), reconstructed
// by intra_rows.h recon_quad<true> with Cb and Cr packed in the 16-bit halves of one lane.
//  w0: as the luma quad, [15,17) = 3, [0,13) LDS offset of the Cb region origin
//  w1, w2: as the luma quad (modes, none bits, fa / la per sub-TB)
//  w3: residual base offset; w4: 4-bit code per (sub-TB q, component h) at bit 8q + 4h,
//      residual = w3 + 16 * code, code 15 = the zero block (DevPic::zero_off)
// (struct IntraJob: intra.h)

enum : uint32_t {
    J_PCM = 1u << 23,
    J_ALL = 1u << 30,
    J_NONE = 1u << 31,
    J5_FAST = 1u << 31,
    J5_QUAD = 1u << 30,
};

// job words staged in LDS: w1 (intraPredAngle, invAngle, availability bit 32) is rebuilt from the
// mode at emission, bit 32 travels in w5 bit 16 (kJ5Bit32); luma w4 is always the zero block
constexpr uint32_t kJ5Bit32 = 1u << 16;
struct LumaJobLds { uint32_t w0, w2, w3, w5; };

// residual base + 4-bit codes of n offsets (code 15 = the zero block): the coded ones must sit in
// 16-sample slots within 14 slots of their minimum (straight-line, bitwise &)
template <int N>
__device__ __forceinline__ bool quad_codes(const uint32_t* off, uint32_t zero_off, uint32_t& base, uint32_t& codes) {
    int32_t mn = INT32_MAX;
#pragma unroll
    for (int i = 0; i < N; ++i) mn = off[i] != zero_off ? min(mn, (int32_t)off[i]) : mn;
    base = mn == INT32_MAX ? zero_off : (uint32_t)mn;
    codes = 0;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t d = off[i] - (uint32_t)mn;                 // >= 0 for the coded ones: mn is their minimum
        const bool z = off[i] == zero_off;
        ok &= z | (((d & 15u) == 0u) & (d <= 14u * 16u));
        codes |= (z ? 15u : (d >> 4) & 15u) << (4 * i);
    }
    return ok;
}

// the four jobs at slots s..s+3 are the fast 4x4 luma TBs of one 8x8 region, in z-order, and their
// residuals are addressable as base + 16 * code (straight-line: every lane of the prep wave
// evaluates it; bitwise & instead of early returns)
__device__ __forceinline__ bool quad_jobs(const LumaJobLds* j, uint32_t zero_off, uint32_t& base, uint32_t& codes) {
    const uint32_t o = j[0].w0 & 0x1fffu;
    bool ok = ((o & 7u) | ((o >> 6) & 7u)) == 0u;                  // region origin on the 8x8 grid
    uint32_t off[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t w0 = j[i].w0;
        ok &= ((j[i].w5 & J5_FAST) != 0u) & (((w0 >> 13) & 15u) == 0u) &    // fast, 4x4, luma
              ((w0 & 0x1fffu) == o + (uint32_t)((i & 1) * 4 + (i >> 1) * 256));
        off[i] = j[i].w3;
    }
    // (sub-TBs 1-3 always see the earlier sub-TBs of the region: intra_rows.h quad_stage handles "no
    // reference available" for the first stage only)
    ok &= ((j[1].w0 | j[2].w0 | j[3].w0) & J_NONE) == 0u;
    return ok & quad_codes<4>(off, zero_off, base, codes);
}

__device__ __forceinline__ IntraJob make_quad(const LumaJobLds* j, uint32_t base, uint32_t codes) {
    uint32_t mode[4], none[4], fa[4], la[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        mode[i] = (j[i].w0 >> 17) & 63u;
        none[i] = j[i].w0 >> 31;
        fa[i] = j[i].w5 & 31u;
        la[i] = (j[i].w5 >> 8) & 31u;
    }
    IntraJob q;
    q.w[0] = (j[0].w0 & 0x1fffu) | mode[0] << 17 | mode[1] << 23 | none[0] << 29 | none[1] << 30;
    q.w[1] = mode[2] | mode[3] << 6 | none[2] << 12 | none[3] << 13 | fa[0] << 14 | la[0] << 19 | fa[1] << 24;
    q.w[2] = la[1] | fa[2] << 5 | la[2] << 10 | fa[3] << 15 | la[3] << 20;
    q.w[3] = base;
    q.w[4] = codes;
    q.w[5] = J5_FAST | J5_QUAD;
    return q;
}

struct ChromaJobLds { uint32_t w0, w2, w3, w4, w5; };

// the four jobs at slots s..s+3 are fast Cb+Cr 4x4 pairs of one 8x8 chroma region, in z-order,
// and their eight residuals are addressable as base + 16 * code (code <= 14; 15 = zero block):
// coded chroma 4x4 TBs of one class are packed in decode order at upload (p265r.hip), so the
// coded TBs of a region normally sit in consecutive 16-sample slots.  Straight-line, as quad_jobs.
__device__ __forceinline__ bool cquad_jobs(const ChromaJobLds* j, uint32_t zero_off, uint32_t& base, uint32_t& codes) {
    const uint32_t o = j[0].w0 & 0x1fffu;
    bool ok = (o >= 4096u) & ((((o - 4096u) & 7u) | (((o - 4096u) >> 5) & 7u)) == 0u);   // 8x8 chroma grid
    uint32_t off[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t w0 = j[i].w0;
        ok &= ((j[i].w5 & J5_FAST) != 0u) & (((w0 >> 13) & 3u) == 0u) & (((w0 >> 15) & 3u) == 3u) &   // fast 4x4 pair
              ((w0 & 0x1fffu) == o + (uint32_t)((i & 1) * 4 + (i >> 1) * 128));
        off[2 * i] = j[i].w3;
        off[2 * i + 1] = j[i].w4;
    }
    ok &= ((j[1].w0 | j[2].w0 | j[3].w0) & J_NONE) == 0u;        // (as quad_jobs)
    return ok & quad_codes<8>(off, zero_off, base, codes);        // i = 2q + h -> bit 8q + 4h
}

__device__ __forceinline__ IntraJob make_cquad(const ChromaJobLds* j, uint32_t base, uint32_t codes) {
    uint32_t mode[4], none[4], fa[4], la[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        mode[i] = (j[i].w0 >> 17) & 63u;
        none[i] = j[i].w0 >> 31;
        fa[i] = j[i].w5 & 31u;
        la[i] = (j[i].w5 >> 8) & 31u;
    }
    IntraJob q;
    q.w[0] = (j[0].w0 & 0x1fffu) | 3u << 15 | mode[0] << 17 | mode[1] << 23 | none[0] << 29 | none[1] << 30;
    q.w[1] = mode[2] | mode[3] << 6 | none[2] << 12 | none[3] << 13 | fa[0] << 14 | la[0] << 19 | fa[1] << 24;
    q.w[2] = la[1] | fa[2] << 5 | la[2] << 10 | fa[3] << 15 | la[3] << 20;
    q.w[3] = base;
    q.w[4] = codes;
    q.w[5] = J5_FAST | J5_QUAD;
    return q;
}

__device__ __forceinline__ bool tb_same_tu_chroma(const p265r_tb& cb, const p265r_tb& cr) {
    return cb.c_idx == 1 && cr.c_idx == 2 && cb.x == cr.x && cb.y == cr.y && cb.log2_size == cr.log2_size &&
           cb.pred_mode == cr.pred_mode && ((cb.flags ^ cr.flags) & P265R_TB_PCM) == 0;
}

// Global-address-space (not flat) accesses for the prep kernel: a flat load or store also counts
// in lgkmcnt, so every LDS wait of the kernel would wait for the outstanding HBM traffic too.
typedef unsigned int prep_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 prep_ld16(const void* p) {
    const prep_u4 v = *(const __attribute__((address_space(1))) prep_u4*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void prep_st16(void* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    *(__attribute__((address_space(1))) prep_u4*)p = prep_u4{a, b, c, d};
}
typedef unsigned int prep_u2 __attribute__((ext_vector_type(2)));
// one 24-B job record: three 8-B global stores (records are 8-B aligned: a 16-B store would straddle
// a 16-B boundary on every other record)
__device__ __forceinline__ void prep_job_store(IntraJob* dst, const IntraJob& J) {
    typedef __attribute__((address_space(1))) prep_u2 gu2;
    *(gu2*)(&dst->w[0]) = prep_u2{J.w[0], J.w[1]};
    *(gu2*)(&dst->w[2]) = prep_u2{J.w[2], J.w[3]};
    *(gu2*)(&dst->w[4]) = prep_u2{J.w[4], J.w[5]};
}

// grid (CTUs, pictures), 64 threads: one wave per CTU walks its TBs 64 at a time.  A CTU's
// job list is [chroma jobs][luma jobs]; both are staged in LDS (luma words 0, 1, 2, 3, 5, at
// most 256 jobs per CTU; chroma words 0..5, at most 128; p265r.hip validate_picture) so that
// luma and chroma 4x4 quads can be merged before the lists are written, compacted.
constexpr int kMaxCtuLuma = 256;
constexpr int kMaxCtuChroma = 128;
constexpr int kPrepChunks = (kMaxCtuLuma + kMaxCtuChroma + 63) / 64;   // TB records per CTU / 64
__device__ __forceinline__ IntraJob luma_job(const LumaJobLds& l, uint32_t zero_off, uint32_t w1) {
    IntraJob J;
    J.w[0] = l.w0; J.w[1] = w1; J.w[2] = l.w2; J.w[3] = l.w3;
    J.w[4] = zero_off; J.w[5] = l.w5 & ~kJ5Bit32;
    return J;
}
// job word w1 of a staged job: intraPredAngle | |invAngle| << 8 (c_angw), availability bit 32 << 21;
// angv = c_angw[lane] (lanes 0..34), picked per lane with a bpermute instead of a global load
__device__ __forceinline__ uint32_t job_w1(uint32_t w0, uint32_t w5, uint32_t angv) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((w0 >> 17) & 63u) << 2), (int)angv) | ((w5 & kJ5Bit32) ? 1u << 21 : 0u);
}
// grid (wc, hc, pictures), one 64-thread wave per CTU
__global__ __launch_bounds__(64) void intra_prep_kernel(const DevPic* __restrict__ pics, Geo g, BatchView v) {
    __shared__ LumaJobLds sj[kMaxCtuLuma];
    __shared__ ChromaJobLds sc[kMaxCtuChroma];
    P265R_BW_PRIO_SET();
    const DevPic P = pics[blockIdx.z];
    // CTU records from the batch layout (no wait for the DevPic load: both in flight together;
    // slots of the context size, a ragged batch's smaller pictures use the front of theirs)
    const p265r_ctu* ctus = v.ctus0 + (size_t)blockIdx.z * g.wc * g.hc;
    const int cx = blockIdx.x, cy = blockIdx.y;
    if (P265R_RAGGED && g.ragged) {
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)P.wh));
        if (cx >= g.wc || cy >= g.hc) return;
    }
    const int addr = cy * g.wc + cx;
    const int lane = threadIdx.x;
    const uint32_t angv = lane < 35 ? c_angw[lane] : 0u;
    const uint32_t ztv = c_ztab[lane];                            // avail_ztab_word(lane >> 4, lane & 15)
    const int ctb = 1 << g.ctb_log2;
    const int x0 = cx << g.ctb_log2, y0 = cy << g.ctb_log2;
    // this CTU's record and its left / top / top-left / top-right neighbours' first 16 B (slice,
    // tile), all five loads in flight together (clamped addresses, used only where they exist)
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    const u4v* cr = reinterpret_cast<const u4v*>(ctus);
    const u4v me4 = cr[2 * addr];
    const int al = cx > 0 ? addr - 1 : addr, at = cy > 0 ? addr - g.wc : addr;
    const int atl = (cx > 0 && cy > 0) ? addr - g.wc - 1 : addr, atr = (cx + 1 < g.wc && cy > 0) ? addr - g.wc + 1 : addr;
    const u4v nl = cr[2 * al], nt = cr[2 * at], ntl = cr[2 * atl], ntr = cr[2 * atr];
    // dword 1: tb_count | tile_id << 16; dword 2: slice_addr
    auto same = [&](const u4v& o) { return o.z == me4.z && (o.y >> 16) == (me4.y >> 16); };
    unsigned flags = 0;
    if (cx > 0 && same(nl)) flags |= 1u;
    if (cy > 0 && same(nt)) flags |= 2u;
    if (cx > 0 && cy > 0 && same(ntl)) flags |= 4u;
    if (cx + 1 < g.wc && cy > 0 && same(ntr)) flags |= 8u;
    p265r_ctu me;
    __builtin_memcpy(&me, &me4, 16);

    const p265r_tb* tbs = P.tbs + me.tb_begin;
    IntraJob* jobs = P.jobs + me.tb_begin;
    const int cnt = me.tb_count;
    // chroma jobs first (Cb+Cr pairs, unpaired Cb / Cr, decode order), then the luma jobs
    // (decode order): the row kernel runs the two components as independent row chains
    // (4:2:0 intra prediction never reads across components)
    int out_l = 0, out_c = 0;
    auto rank = [&](unsigned long long m) {
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    };
    // every TB record of the CTU is loaded up front, one 16-B load per lane and chunk, all in
    // flight together (tb_count <= 384 at CTB 64, validate_picture); a TB's predecessor and
    // successor come from the neighbouring lanes (DPP wave shifts, chunk edges by v_readlane)
    uint4 rv[kPrepChunks];
    const uint4* tv = reinterpret_cast<const uint4*>(tbs);
#pragma unroll
    for (int i = 0; i < kPrepChunks; ++i) {
        const int t = i * 64 + lane;
        rv[i] = t < cnt ? prep_ld16(tv + t) : make_uint4(0u, 0u, 0u, 0u);
    }
    auto from_prev_lane = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false); };
    auto from_next_lane = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false); };
    auto as_tb = [](uint4 v) { p265r_tb r; __builtin_memcpy(&r, &v, sizeof(r)); return r; };
#pragma unroll
    for (int ci = 0; ci < kPrepChunks; ++ci) {
        const int base = ci * 64;
        if (base >= cnt) break;                                   // wave-uniform
        const int t = base + lane;
        const bool valid = t < cnt;
        const uint4 cv = rv[ci];
        // words 0, 1 (position, size, component, mode, flags) of t - 1; words 0, 1, 3 of t + 1 --
        // neighbouring lanes (DPP), across the chunk edges by v_readlane, selected without branches
        const uint32_t pe_x = ci > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)rv[ci > 0 ? ci - 1 : 0].x, 63) : 0u;
        const uint32_t pe_y = ci > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)rv[ci > 0 ? ci - 1 : 0].y, 63) : 0u;
        const int cn = ci + 1 < kPrepChunks ? ci + 1 : ci;
        const uint32_t ne_x = ci + 1 < kPrepChunks ? (uint32_t)__builtin_amdgcn_readlane((int)rv[cn].x, 0) : 0u;
        const uint32_t ne_y = ci + 1 < kPrepChunks ? (uint32_t)__builtin_amdgcn_readlane((int)rv[cn].y, 0) : 0u;
        const uint32_t ne_w = ci + 1 < kPrepChunks ? (uint32_t)__builtin_amdgcn_readlane((int)rv[cn].w, 0) : 0u;
        const bool has_prev = valid & (t > 0), has_next = valid & (t + 1 < cnt);
        // the DPP moves are pinned here (empty asm): left to the compiler they sink into divergent
        // branches of their selects, each with its own exec-mask save / restore
        uint32_t dp0 = from_prev_lane(cv.x), dp1 = from_prev_lane(cv.y);
        uint32_t dn0 = from_next_lane(cv.x), dn1 = from_next_lane(cv.y), dn3 = from_next_lane(cv.w);
        asm volatile("" : "+v"(dp0), "+v"(dp1), "+v"(dn0), "+v"(dn1), "+v"(dn3));
        const uint32_t p0 = has_prev ? (lane == 0 ? pe_x : dp0) : 0u;
        const uint32_t p1 = has_prev ? (lane == 0 ? pe_y : dp1) : 0u;
        const uint4 nv = make_uint4(lane == 63 ? ne_x : dn0, lane == 63 ? ne_y : dn1, 0u, lane == 63 ? ne_w : dn3);
        p265r_tb rec = as_tb(valid ? cv : make_uint4(0u, 0u, 0u, 0u));
        p265r_tb next = as_tb(has_next ? nv : make_uint4(0u, 0u, 0u, 0u));
        // tb_same_tu_chroma on the raw words: word 0 = x | y << 16, word 1 = log2 | c_idx << 8 |
        // pred_mode << 16 | flags << 24 (Cb then Cr of one TU: same position, size, mode, PCM flag)
        auto same_tu = [](uint32_t cb0, uint32_t cb1, uint32_t cr0, uint32_t cr1) {   // (bitwise: no short circuit)
            return (cb0 == cr0) & ((cb1 & 0xff00u) == 0x0100u) & ((cr1 & 0xff00u) == 0x0200u) &
                   (((cb1 ^ cr1) & (0x00ff00ffu | (uint32_t)P265R_TB_PCM << 24)) == 0u);
        };
        const bool cr_taken = has_prev & same_tu(p0, p1, cv.x, cv.y);
        const bool keep = valid & !cr_taken;
        const bool pair_next = has_next & same_tu(cv.x, cv.y, nv.x, nv.y);
        const bool kl = keep && rec.c_idx == 0;
        const unsigned long long ml = __ballot(kl), mc = __ballot(keep && !kl);
        const int slot = kl ? out_l + rank(ml) : out_c + rank(mc);
        out_l += __popcll(ml);
        out_c += __popcll(mc);
        // every lane computes its job record (straight-line, selects only; lanes without a TB use
        // a 4x4 luma stand-in), only the kept ones store it: no divergent branches in the chunk
        {
            const int lg = max((int)rec.log2_size, 2), n = 1 << lg, c = rec.c_idx;
            const int sub = c ? 1 : 0;
            const bool pair = pair_next;
            const int xr = (int)rec.x - (x0 >> sub), yr = (int)rec.y - (y0 >> sub);
            const uint32_t ofs = c == 0 ? (uint32_t)(yr * 64 + xr) : (uint32_t)(4096 + yr * 32 + xr);
            const uint32_t cm = c == 0 ? 0u : (pair ? 3u : (uint32_t)c);
            const int mode = rec.pred_mode;
            // ---- availability per reference unit, linear order (8.4.4.2.2) -----------------
            const int L = (2 * n) >> (c ? 1 : 2);
            // z-order word of the TB's size and unit row (ztv: lane i holds avail_ztab_word word i)
            const int zs = (31 - __clz(n)) + sub - 2, yu = (yr << sub) >> 2;
            const uint32_t zw = (uint32_t)__builtin_amdgcn_ds_bpermute((zs * 16 + yu) << 2, (int)ztv);
            uint32_t mhi;
            const uint32_t mlo = ref_avail_mask32(c, xr, yr, n, x0, y0, g.w, g.h, ctb, flags, zw, mhi);
            const uint32_t full_lo = L == 16 ? 0xffffffffu : (1u << (2 * L + 1)) - 1u;
            const bool m_full = (mlo == full_lo) & (mhi == (L == 16 ? 1u : 0u)), m_none = (mlo | mhi) == 0u;
            // ---- filtering decision (8.4.4.2.3), luma only in 4:2:0 ---------------------------
            const int dist = min(abs(mode - 26), abs(mode - 10));
            const bool fon = (c == 0) & (n != 4) & (mode != 1) & (dist > (n == 8 ? 7 : (n == 16 ? 1 : 0)));
            const uint32_t filt = fon ? ((n == 32 && g.strong) ? 2u : 1u) : 0u;
            const uint32_t f0 = rec.flags;
            const uint32_t f1 = pair ? next.flags : 0u;
            // half 0 = luma / Cb, half 1 = Cr (an unpaired Cr TB lives in half 1)
            const uint32_t fh0 = cm == 2 ? 0u : f0, fh1 = cm == 2 ? f0 : f1;
            auto raw = [](uint32_t f) { return (f & (P265R_TB_BYPASS | P265R_TB_PCM)) ? 1u : 0u; };
            auto coded = [](uint32_t f) { return (f & (P265R_TB_CBF | P265R_TB_PCM)) ? 1u : 0u; };
            auto roff = [&](uint32_t f, uint32_t off) {
                return !coded(f) ? P.zero_off : (raw(f) ? off + (uint32_t)P.pool_rel : off);
            };
            const uint32_t r0 = roff(f0, rec.coef_off);
            const uint32_t off0 = cm == 2 ? P.zero_off : r0;
            const uint32_t off1 = cm == 2 ? r0 : (pair ? roff(f1, next.coef_off) : P.zero_off);
            const uint32_t w0 = ofs | (uint32_t)(lg - 2) << 13 | cm << 15 | (uint32_t)mode << 17 |
                                ((f0 & P265R_TB_PCM) ? J_PCM : 0u) | filt << 24 | raw(fh0) << 26 | raw(fh1) << 27 |
                                coded(fh0) << 28 | coded(fh1) << 29 | (m_full ? J_ALL : 0u) | (m_none ? J_NONE : 0u);
            const uint32_t w2 = mlo;
            // fast path: one contiguous run of available units [ulo, uhi] -> sample bounds [fa, la]
#ifndef P265R_FAST16
#define P265R_FAST16 1
#endif
            const bool fast_size = ((c == 0) & (n <= (P265R_FAST16 ? 16 : 8))) | ((cm == 3u) & (n <= (g.quad & 4 ? 4 : 8)));
            const int US = c ? 1 : 2;
            const int ulo = mlo ? __ffs((int)mlo) - 1 : 32;
            const int uhi = mhi ? 32 : 31 - __clz((int)(mlo | 1u));
            // the available units form one run [ulo, uhi] (32-bit pieces; mhi = unit 32)
            const uint32_t lo_cut = ulo >= 32 ? 0u : (0xffffffffu << ulo);
            const bool contig = mlo == (mhi ? lo_cut : (lo_cut & (uhi >= 31 ? 0xffffffffu : ((2u << uhi) - 1u))));
            const int fa = ulo < L ? (ulo << US) : (ulo == L ? 2 * n : 2 * n + 1 + ((ulo - L - 1) << US));
            const int la = uhi < L ? ((uhi + 1) << US) - 1 : (uhi == L ? 2 * n : 2 * n + ((uhi - L) << US));
            const bool fast = fast_size & !(f0 & P265R_TB_PCM) & (m_none | contig);
            const uint32_t w5 = !fast ? 0u : (m_none ? J5_FAST : (J5_FAST | (uint32_t)fa | (uint32_t)la << 8));
            const uint32_t w5s = w5 | (mhi ? kJ5Bit32 : 0u);
            if (keep && kl) sj[slot] = LumaJobLds{w0, w2, off0, w5s};
            else if (keep && slot < kMaxCtuChroma) sc[slot] = ChromaJobLds{w0, w2, off0, off1, w5s};
        }
    }
    const int n_luma = out_l, n_chroma = min(out_c, kMaxCtuChroma);
    __syncthreads();
    // ---- 4x4 quads + emission, one pass per 64-slot window: slot s heads a quad when s..s+3 are
    // its four fast TBs / Cb+Cr pairs; a slot is absorbed when one of the three before it heads
    // one (this window's heads from one ballot, the previous window's last three carried).  Every
    // lane reads in-bounds LDS (clamped), only the stores are predicated; no head arrays in LDS
    auto absorbed_mask = [](unsigned long long H, unsigned long long Hp) {
        return (H << 1) | (H << 2) | (H << 3) | (Hp >> 63) | (Hp >> 62) | (Hp >> 61);
    };
    // does a job read the row above the CTU beyond the CTU's own columns (the top-right CTU's bottom row)?
    // Then the row kernel must wait for that CTU before running it; every job before the first such one
    // runs after the CTU above alone (intra_rows.h: the top-right wait moves into the CTU).  A TB at CTB
    // position (xr, 0) reads top samples up to x = xr + 2n - 1; a quad's second sub-block up to X + 11.
    // Only when the top-right CTU is usable (same slice and tile, inside the picture: flags bit 3)
    auto needs_tr = [&](uint32_t w0, bool quad, bool chroma) -> bool {
        const uint32_t o = (w0 & 0x1fffu) - (chroma ? 4096u : 0u);
        const int xr = (int)(o & (chroma ? 31u : 63u)), yr = (int)(o >> (chroma ? 5 : 6));
        const int reach = quad ? xr + 12 : xr + (8 << ((w0 >> 13) & 3u));
        return (yr == 0) & (reach > (chroma ? ctb >> 1 : ctb)) & ((flags & 8u) != 0u);
    };
    // does a job lie in the CTB's bottom-left quadrant?  Once the last such job of the list (either chroma
    // plane: a component-major TB order lists every Cb job before the Cr ones) has run, the left half of the
    // CTB's bottom row is final -- no other job writes it (TBs never straddle a quadrant at CTB 64) -- and the
    // row below may read it as its top-right samples (intra_rows.h, cross-group kernel at CTB 64)
    auto in_bl = [&](uint32_t w0, bool chroma) -> bool {
        const uint32_t o = (w0 & 0x1fffu) - (chroma ? 4096u : 0u);
        const int hq = chroma ? ctb >> 2 : ctb >> 1;
        return ((int)(o & (chroma ? 31u : 63u)) < hq) & ((int)(o >> (chroma ? 5 : 6)) >= hq);
    };
    // self-check of `br` (Geo::tr_check, tests): does a job's EXTENT cover a sample of the bottom row of the
    // CTB's left half?  (Independent of in_bl's origin rule.)  No such job may come at or after `br`.
    auto touches_bl_row = [&](uint32_t w0, bool quad, bool chroma) -> bool {
        const uint32_t o = (w0 & 0x1fffu) - (chroma ? 4096u : 0u);
        const int cts = chroma ? ctb >> 1 : ctb;
        const int xr = (int)(o & (chroma ? 31u : 63u)), yr = (int)(o >> (chroma ? 5 : 6));
        const int ext = quad ? 8 : 4 << ((w0 >> 13) & 3u);
        return (xr < cts / 2) & (yr + ext >= cts);
    };
    auto last_of = [&](unsigned long long m, unsigned long long me, int out) {    // index of m's last job
        return m ? out + (int)__popcll(me & ((2ull << (63 - __clzll((long long)m))) - 1ull)) - 1 : -1;
    };
    auto first_of = [&](unsigned long long m, unsigned long long me, int out) {   // index of m's first job
        return m ? out + (int)__popcll(me & ((1ull << (__ffsll((long long)m) - 1)) - 1ull)) : -1;
    };
    int c_out = 0, tr_c = -1, bl_c = -1, tb_c = -1;
    unsigned long long hp = 0;
    for (int base = 0; base < n_chroma; base += 64) {
        const int s = base + lane;
        const bool valid = s < n_chroma;
        const int s1 = min(s, n_chroma - 1);
        const int sq = min(s, kMaxCtuChroma - 4);                     // (a head: sq = s)
        uint32_t qb = 0, qc = 0;
        const bool hd = ((g.quad & 2) != 0) & (s + 3 < n_chroma) & cquad_jobs(sc + sq, P.zero_off, qb, qc);
        const unsigned long long H = __ballot(hd);
        const bool emit = valid & !((absorbed_mask(H, hp) >> lane) & 1ull);
        hp = H;
        const unsigned long long me_ = __ballot(emit);
        const ChromaJobLds c = sc[s1];
        const uint32_t w1 = job_w1(c.w0, c.w5, angv);
        IntraJob J;
        if (hd) {
            J = make_cquad(sc + sq, qb, qc);
        } else {
            J.w[0] = c.w0; J.w[1] = w1; J.w[2] = c.w2; J.w[3] = c.w3;
            J.w[4] = c.w4; J.w[5] = c.w5 & ~kJ5Bit32;
        }
        if (emit) prep_job_store(jobs + c_out + rank(me_), J);
        if (g.tr_info) {                                        // (uniform)
            if (tr_c < 0) tr_c = first_of(__ballot(emit && needs_tr(J.w[0], hd, true)), me_, c_out);
            bl_c = max(bl_c, last_of(__ballot(emit && in_bl(J.w[0], true)), me_, c_out));
            if (g.tr_check) tb_c = max(tb_c, last_of(__ballot(emit && touches_bl_row(J.w[0], hd, true)), me_, c_out));
        }
        c_out += __popcll(me_);
    }
    int n_out = 0, tr_l = -1, bl_l = -1, tb_l = -1;
    hp = 0;
    for (int base = 0; base < n_luma; base += 64) {
        const int s = base + lane;
        const bool valid = s < n_luma;
        const int s1 = min(s, n_luma - 1), sq = min(s, kMaxCtuLuma - 4);
        uint32_t qb = 0, qc = 0;
        const bool hd = ((g.quad & 1) != 0) & (s + 3 < n_luma) & quad_jobs(sj + sq, P.zero_off, qb, qc);
        const unsigned long long H = __ballot(hd);
        const bool emit = valid & !((absorbed_mask(H, hp) >> lane) & 1ull);
        hp = H;
        const unsigned long long me_ = __ballot(emit);
        const LumaJobLds l = sj[s1];
        const uint32_t w1 = job_w1(l.w0, l.w5, angv);
        const IntraJob J = hd ? make_quad(sj + sq, qb, qc) : luma_job(l, P.zero_off, w1);
        if (emit) prep_job_store(jobs + c_out + n_out + rank(me_), J);
        if (g.tr_info) {
            if (tr_l < 0) tr_l = first_of(__ballot(emit && needs_tr(J.w[0], hd, false)), me_, n_out);
            bl_l = max(bl_l, last_of(__ballot(emit && in_bl(J.w[0], false)), me_, n_out));
            if (g.tr_check) tb_l = max(tb_l, last_of(__ballot(emit && touches_bl_row(J.w[0], hd, false)), me_, n_out));
        }
        n_out += __popcll(me_);
    }
#ifdef P265R_BR_BROKEN      // negative test of the half-CTU publish checks: publish before the last bottom-left job
    const int br_l = bl_l < 0 ? n_out : bl_l, br_c = bl_c < 0 ? c_out : bl_c;
#else
    const int br_l = bl_l < 0 ? n_out : bl_l + 1, br_c = bl_c < 0 ? c_out : bl_c + 1;
#endif
    // a job covering the bottom row's left half at or after `br` would leave the half-CTU publish stale
    // (P265R_BR_BROKEN=2: the broken `br` without this check, so the row kernel's poisoned half line alone
    // must catch it)
#if !(defined(P265R_BR_BROKEN) && P265R_BR_BROKEN == 2)
    if (g.tr_check && lane == 0 && (tb_l >= br_l || tb_c >= br_c)) atomicOr(v.err, 2);
#endif
    // per CTU, luma | chroma << 16 each: job counts; the index of the first job that reads the top-right
    // CTU (= the count when none does); one past the last job in the bottom-left quadrant (= the count when
    // there is none: a CTU row below the picture's last sample row has no reader)
    if (lane == 0) {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        *(__attribute__((address_space(1))) u4*)(P.jcount + 4 * addr) =
            u4{(uint32_t)n_out | (uint32_t)c_out << 16,
#ifdef P265R_TR_BROKEN      // negative test of the row kernel's top-right self-check: no job waits
               (uint32_t)n_out | (uint32_t)c_out << 16,
#else
               (uint32_t)(tr_l < 0 ? n_out : tr_l) | (uint32_t)(tr_c < 0 ? c_out : tr_c) << 16,
#endif
               (uint32_t)br_l | (uint32_t)br_c << 16, 0u};
    }
}

}  // namespace p265r
