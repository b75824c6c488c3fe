// Intra prediction + reconstruction, CU-local wavefront ("row pipeline") schedule.
//
// One workgroup owns whole pictures: its W waves pull CTU ROWS from an LDS row queue
// (pictures of the workgroup in order, rows top to bottom) and walk each row left to
// right.  Row r may start CTU cx once row r-1 has finished CTU min(cx+2, wc) - the
// 2-CTU lag that makes the left, top-left, top and top-right CTUs available.  The
// queue runs across picture boundaries, so waves never idle at a picture's ramp-down.
//
// All neighbour data lives in LDS: the row above comes from a per-picture, per-row-
// parity LINE BUFFER (bottom sample row of every finished CTU), the column on the left
// is the wave's own previous CTU.  Nothing is re-read from HBM and no cross-CU
// hand-off exists, so the only synchronisation is one LDS progress word per row
// (workgroup-scope release/acquire).  Per transform block the wave does three LDS
// round trips (gather, substitute+filter, predict) with wave-local ordering only.
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

struct TbRec {                    // decoded p265r_tb (wave-uniform)
    int x, y, log2, c, mode, flags, off;
};

__device__ __forceinline__ TbRec tb_from_words(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    TbRec t;
    t.x = (int)(w0 & 0xffff); t.y = (int)(w0 >> 16);
    t.log2 = (int)(w1 & 0xff); t.c = (int)((w1 >> 8) & 0xff);
    t.mode = (int)((w1 >> 16) & 0xff); t.flags = (int)(w1 >> 24);
    (void)w2;                      // qp (used by the residual phase) + reserved
    t.off = (int)w3;
    return t;
}

template <int W>
__global__ __launch_bounds__(64 * W) void intra_rows_kernel(const DevPic* __restrict__ pics,
                                                           const int16_t* __restrict__ pool,
                                                           const int16_t* __restrict__ resid,
                                                           Geo g, int n_pics, int fs_count,
                                                           int* __restrict__ err_flag) {
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
    // bounded spin-wait on an LDS word; false = gave up (error published, caller returns)
    auto wait_until = [&](auto ready) -> bool {
        long spins = 0;
        for (;;) {
            if (ready()) return true;
            if (__hip_atomic_load(&ctl.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1l << 24)) {                    // never hang the GPU
                if (lane == 0) { ctl.error = 1; atomicOr(err_flag, 1); }
                return false;
            }
        }
    };

    for (;;) {
        int r = 0;
        if (lane == 0) r = __hip_atomic_fetch_add(&ctl.next_row, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        r = __builtin_amdgcn_readfirstlane(r);
        if (r >= rows_total) break;
        const int j = r / g.hc, cy = r - j * g.hc;
        const int slot = j % fs_count, gen = j / fs_count;
        const DevPic P = pics[b + j * G];
        // picture slot reuse: every row of picture j waits until picture j - fs_count (the
        // slot's previous occupant) has completed all its rows; those rows were dequeued
        // earlier and are held by running waves, so this wait always ends.
        if (!wait_until([&] {
                return __hip_atomic_load(&ctl.done[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= gen * g.hc;
            })) return;
        unsigned char* line_cur = lines + (size_t)(slot * 2 + (cy & 1)) * line_bytes;
        const unsigned char* line_up = lines + (size_t)(slot * 2 + ((cy & 1) ^ 1)) * line_bytes;
        int* my_prog = &prog[slot * g.hc + cy];
        const int* up_prog = &prog[slot * g.hc + (cy > 0 ? cy - 1 : 0)];
        const int tag = (j & 0xffff) << 16;
        if (lane == 0) __hip_atomic_store(my_prog, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);

        for (int cx = 0; cx < g.wc; ++cx) {
            // ---- wait for the row above (2-CTU lag) -------------------------------------
            if (cy > 0) {
                const int need = min(cx + 2, g.wc);
                if (!wait_until([&] {
                        const int v = __hip_atomic_load(up_prog, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        return (v & 0xffff0000) == tag && (v & 0xffff) >= need;
                    })) return;
            }
            const int x0 = cx << g.ctb_log2, y0 = cy << g.ctb_log2;
            const int addr = cy * g.wc + cx;
            const p265r_ctu me = P.ctus[addr];
            unsigned flags = 0;
            if (cx > 0 && ctu_same_region(me, P.ctus[addr - 1])) flags |= 1u;
            if (cy > 0 && ctu_same_region(me, P.ctus[addr - g.wc])) flags |= 2u;
            if (cx > 0 && cy > 0 && ctu_same_region(me, P.ctus[addr - g.wc - 1])) flags |= 4u;
            if (cx + 1 < g.wc && cy > 0 && ctu_same_region(me, P.ctus[addr - g.wc + 1])) flags |= 8u;

            const int nt = me.tb_count;
            const p265r_tb* tbs = P.tbs + me.tb_begin;
            uint4 rec = make_uint4(0, 0, 0, 0);
            if (lane < nt) rec = *reinterpret_cast<const uint4*>(tbs + lane);

            // residual of TB t is loaded while TB t-1 is processed (2 x 16 B per lane, fixed shape)
            auto load_res = [&](const TbRec& t, uint4& a, uint4& b2) {
                const bool coded = t.flags & (P265R_TB_CBF | P265R_TB_PCM);
                const int nn = 1 << (2 * t.log2);
                const int S = nn >= 64 ? (nn >> 6) : 1;
                const int sidx = lane * S < nn ? lane * S : 0;
                const int16_t* base = (t.flags & (P265R_TB_BYPASS | P265R_TB_PCM)) ? pool : resid;
                if (coded) {
                    const int16_t* rp = base + t.off + sidx;
                    if (S == 16) { a = *reinterpret_cast<const uint4*>(rp); b2 = *reinterpret_cast<const uint4*>(rp + 8); }
                    else if (S == 4) { const uint2 v = *reinterpret_cast<const uint2*>(rp); a = make_uint4(v.x, v.y, 0, 0); }
                    else { a = make_uint4((uint32_t)(uint16_t)rp[0], 0, 0, 0); }
                } else {
                    a = make_uint4(0, 0, 0, 0); b2 = a;
                }
            };
            auto rec_of = [&](int t) {
                if ((t & 63) == 0 && t) {          // next chunk of 64 records
                    rec = make_uint4(0, 0, 0, 0);
                    if (t + lane < nt) rec = *reinterpret_cast<const uint4*>(tbs + t + lane);
                }
                const int l = t & 63;
                return tb_from_words(__builtin_amdgcn_readlane(rec.x, l), __builtin_amdgcn_readlane(rec.y, l),
                                     __builtin_amdgcn_readlane(rec.z, l), __builtin_amdgcn_readlane(rec.w, l));
            };

            TbRec cur = nt ? rec_of(0) : TbRec{0, 0, 2, 0, 0, 0, 0};
            uint4 ra = make_uint4(0, 0, 0, 0), rb = ra;
            if (nt) load_res(cur, ra, rb);

            for (int t = 0; t < nt; ++t) {
                const TbRec tb = cur;
                const uint4 ca = ra, cb = rb;
                if (t + 1 < nt) { cur = rec_of(t + 1); load_res(cur, ra, rb); }

                const int c = tb.c;
                const int sub = c ? 1 : 0;
                const int log2 = tb.log2, n = 1 << log2;
                const int xr = tb.x - (x0 >> sub), yr = tb.y - (y0 >> sub);
                const int bd = g.bd[c];
                const int maxv = (1 << bd) - 1;
                uint8_t* interior = c ? L.c[c - 1] : L.y;
                const int ist = c ? 32 : 64;
                const uint8_t* top = line_up + (c == 0 ? 0 : (c == 1 ? g.w : g.w + g.cw)) + (x0 >> sub);
                const uint8_t* left = c ? L.cleft[c - 1] : L.yleft;
                const int nn = n * n;
                const int S = nn >= 64 ? (nn >> 6) : 1;
                const bool own = lane * S < nn;
                const int sidx = lane * S;
                const int sy = sidx >> log2, sx = sidx & (n - 1);

                int pred[16];
                if (tb.flags & P265R_TB_PCM) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) pred[i] = 0;
                } else {
                    // ---- A: gather raw reference samples + availability ------------------
                    const int nref = 4 * n + 1;
                    const int xcl = xr << sub, ycl = yr << sub;
                    unsigned long long m[3] = {0ull, 0ull, 0ull};
#pragma unroll
                    for (int jj = 0; jj < 3; ++jj) {
                        if (jj * 64 < nref) {
                            const int k = lane + 64 * jj;
                            bool av = false;
                            if (k < nref) {
                                const int dx = k <= 2 * n ? -1 : k - 2 * n - 1;
                                const int dy = k < 2 * n ? 2 * n - 1 - k : -1;
                                const int xn = xr + dx, yn = yr + dy;
                                av = nb_available(xn << sub, yn << sub, xcl, ycl, x0, y0, g, ctb, flags);
                                int v = 0;
                                if (av) v = yn < 0 ? top[xn] : (xn < 0 ? left[yn] : interior[yn * ist + xn]);
                                L.ref[0][k] = (uint16_t)v;
                            }
                            m[jj] = __ballot(av);
                        }
                    }
                    wave_sync();
                    const int mode = tb.mode;
                    bool filt = false;
                    if (c == 0 && mode != 1 && n != 4) {
                        const int dist = min(abs(mode - 26), abs(mode - 10));
                        filt = dist > (n == 8 ? 7 : (n == 16 ? 1 : 0));
                    }
                    const bool any = (m[0] | m[1] | m[2]) != 0ull;
                    const int half = 1 << (bd - 1);
                    auto sval = [&](int i) -> int {
                        const int s = subst_src(i, m[0], m[1], m[2]);
                        return s < 0 ? half : (int)L.ref[0][s];
                    };
                    bool strong = false;
                    int corner = 0, bl = 0, tr = 0;
                    if (filt && g.strong && n == 32) {
                        corner = sval(2 * n); bl = sval(0); tr = sval(4 * n);
                        strong = abs(corner + tr - 2 * sval(3 * n)) < (1 << (bd - 5)) &&
                                 abs(corner + bl - 2 * sval(n)) < (1 << (bd - 5));
                    }
                    int dcs = 0;
                    // ---- B: substitution + filtering -> ref[1] ---------------------------
#pragma unroll
                    for (int jj = 0; jj < 3; ++jj) {
                        if (jj * 64 < nref) {
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
                    }
                    wave_sync();
                    const uint16_t* R = L.ref[1];
                    // ---- C: prediction -----------------------------------------------------
                    if (mode == 0) {
                        const int trs = R[3 * n + 1], bls = R[n - 1];
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            if (i < S) {
                                const int x = sx + i, y = sy;
                                pred[i] = ((n - 1 - x) * R[2 * n - 1 - y] + (x + 1) * trs +
                                           (n - 1 - y) * R[2 * n + 1 + x] + (y + 1) * bls + n) >> (log2 + 1);
                            }
                        }
                    } else if (mode == 1) {
                        const int dc = (__ockl_wfred_add_i32(dcs) + n) >> (log2 + 1);
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
                                const int a = vert ? y : x, bb = vert ? x : y;
                                const int idx = ((a + 1) * ang) >> 5, fact = ((a + 1) * ang) & 31;
                                const int r0 = bb + idx + 1;
                                const int k0 = r0 >= 0 ? 2 * n + dir * r0 : 2 * n - dir * ((r0 * inv + 128) >> 8);
                                int v = R[k0];
                                if (fact) {
                                    const int r1 = r0 + 1;
                                    const int k1 = r1 >= 0 ? 2 * n + dir * r1 : 2 * n - dir * ((r1 * inv + 128) >> 8);
                                    v = ((32 - fact) * v + fact * (int)R[k1] + 16) >> 5;
                                }
                                if (c == 0 && n < 32) {
                                    if (mode == 26 && x == 0)
                                        v = min(max((int)R[2 * n + 1] + (((int)R[2 * n - 1 - y] - (int)R[2 * n]) >> 1), 0), maxv);
                                    if (mode == 10 && y == 0)
                                        v = min(max((int)R[2 * n - 1] + (((int)R[2 * n + 1 + x] - (int)R[2 * n]) >> 1), 0), maxv);
                                }
                                pred[i] = v;
                            }
                        }
                    }
                }
                // ---- reconstruction into the wave's CTU image -------------------------------
                if (own) {
                    const uint32_t w8[8] = {ca.x, ca.y, ca.z, ca.w, cb.x, cb.y, cb.z, cb.w};
                    auto resv = [&](int i) { return (int)(int16_t)(w8[i >> 1] >> ((i & 1) * 16)); };
                    uint8_t* dst = interior + (yr + sy) * ist + xr + sx;
                    if (S == 16) {
                        uint32_t w[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            uint32_t v = 0;
#pragma unroll
                            for (int bb = 0; bb < 4; ++bb)
                                v |= (uint32_t)min(max(pred[q * 4 + bb] + resv(q * 4 + bb), 0), maxv) << (8 * bb);
                            w[q] = v;
                        }
                        *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
                    } else if (S == 4) {
                        uint32_t v = 0;
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb) v |= (uint32_t)min(max(pred[bb] + resv(bb), 0), maxv) << (8 * bb);
                        *reinterpret_cast<uint32_t*>(dst) = v;
                    } else {
                        dst[0] = (uint8_t)min(max(pred[0] + resv(0), 0), maxv);
                    }
                }
                wave_sync();
            }

            // ---- publish the CTU: planes (HBM), bottom line (LDS), right column (LDS) ----------
            for (int c = 0; c < 3; ++c) {
                const int sub = c ? 1 : 0;
                const int cs = ctb >> sub;
                const int Wd = c ? g.cw : g.w, Ht = c ? g.ch : g.h;
                const int xb = x0 >> sub, yb = y0 >> sub;
                const int wv = min(cs, Wd - xb), hv = min(cs, Ht - yb);
                const uint8_t* src = c ? L.c[c - 1] : L.y;
                const int ist = c ? 32 : 64;
                uint8_t* plane = P.rec[c];
                const int st = g.stride[c];
                const int gpr = wv >> 2;
                for (int e = lane; e < gpr * hv; e += 64) {
                    const int yy = e / gpr, xx = (e - yy * gpr) << 2;
                    *reinterpret_cast<uint32_t*>(plane + (size_t)(yb + yy) * st + xb + xx) =
                        *reinterpret_cast<const uint32_t*>(src + yy * ist + xx);
                }
                unsigned char* lc = line_cur + (c == 0 ? 0 : (c == 1 ? g.w : g.w + g.cw)) + xb;
                if (lane < wv) lc[lane] = src[(hv - 1) * ist + lane];
                uint8_t* lf = c ? L.cleft[c - 1] : L.yleft;
                if (lane < hv) lf[lane] = src[lane * ist + wv - 1];
            }
            if (lane == 0)
                __hip_atomic_store(my_prog, tag | (cx + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            wave_sync();
        }
        if (lane == 0) __hip_atomic_fetch_add(&ctl.done[slot], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

}  // namespace p265r
