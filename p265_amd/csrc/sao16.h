// SAO only (8.7.3) for 16-bit samples (BitDepth 9..12), batches without deblocking: a
// streaming strip kernel like sao_strip16.h, 8 samples (16 B) per lane.  One wave = one CTB row of one
// component over a strip of 62 x 8 samples (lane l: the 8 samples at x = 496 s + 8 (l - 1); lanes 0 and
// 63 only supply the neighbours of lanes 1 and 62); the wave walks down its CTB row with the rows above,
// at and below the current one in registers, so every sample is read once (+ 2 halo rows per CTB
// height) and written once, each row one coalesced load and store per wave instruction.  A lane's 8
// samples lie in one CTB (8 divides every CTB width down to CTB 16 chroma), so its SaoTypeIdx, class,
// offsets and 8.7.3.2 neighbourhood permissions are per-lane constants; the samples beside the lane's
// column come from lanes l -/+ 1 (DPP wave shifts).  Per sample: band (bandShift = BitDepth - 5) or
// edge class, the SaoOffsetVal lookup by shift, PCM / bypass samples (nofilter) untouched.
//
// The reference only parses the SAO syntax (decoder/sao.py:15-136, SaoOffsetVal sao.py:174-178); the
// filter rests on the spec restatement (oracle/recon_oracle.py sao_picture), as loopfilter16.h does.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"
#include "loopfilter.h"
#include "sao.h"

namespace p265r {

constexpr int kSao16bStrip = 62 * 8;       // output samples per strip

// waves per picture: hc CTB rows x (luma strips + 2 x chroma strips)
__host__ __device__ __forceinline__ int sao16b_units(const Geo& g) {
    return g.hc * ((g.w + kSao16bStrip - 1) / kSao16bStrip + 2 * ((g.cw + kSao16bStrip - 1) / kSao16bStrip));
}

// grid: 4 waves per block, one wave per (picture, CTB row, component, strip), XCD-aware order
__global__ __launch_bounds__(256) void sao16_strip_kernel(const DevPic* __restrict__ pics, Geo g, BatchView v, int n_pics) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) uint16_t gu16;
    P265R_BW_PRIO_SET();
    const int lane = threadIdx.x & 63;
    const int per_pic = sao16b_units(g);
    const int total = per_pic * n_pics;
    const int nblk = (total + 3) >> 2;
    const int bunit = xcd_unit(blockIdx.x, nblk);
    const int unit = __builtin_amdgcn_readfirstlane(bunit * 4 + (int)(threadIdx.x >> 6));
    if (bunit >= nblk || unit >= total) return;                   // whole wave (no barriers below)
    const int pic = unit / per_pic;
    int u = unit - pic * per_pic;
    const int nsl = (g.w + kSao16bStrip - 1) / kSao16bStrip, nsc = (g.cw + kSao16bStrip - 1) / kSao16bStrip;
    // unit order inside a picture: CTB row major, then luma strips, Cb strips, Cr strips
    const int cy = u / (nsl + 2 * nsc);
    u -= cy * (nsl + 2 * nsc);
    int c, sx;
    if (u < nsl) { c = 0; sx = u; }
    else { c = 1 + (u - nsl) / nsc; sx = (u - nsl) % nsc; }
    // CTU records: slots of the context size; a ragged batch's smaller picture uses its own raster
    const uint32_t* crec = reinterpret_cast<const uint32_t*>(v.ctus0 + (size_t)pic * g.wc * g.hc);
    if (P265R_RAGGED && g.ragged) {
        g = pic_geo(g, (uint32_t)__builtin_amdgcn_readfirstlane((int)pics[pic].wh));
        if (cy >= g.hc || sx * kSao16bStrip >= (c ? g.cw : g.w)) return;   // whole wave, outside this picture
    }
    const int sub = c ? 1 : 0;
    const int Ls = g.ctb_log2 - sub, cs = 1 << Ls;
    const int W = c ? g.cw : g.w, H = c ? g.ch : g.h;
    const int st = c ? g.stride[1] : g.stride[0];                 // samples
    const int bd = c ? g.bd[1] : g.bd[0], maxv = (1 << bd) - 1;
    const uint64_t pofs = (uint64_t)pic * v.pic_bytes + v.plane_off[c];
    const gu16* src = (const gu16*)(v.rec0 + pofs);
    gu16* dst = (gu16*)(v.out0 + pofs);
    const int X = sx * kSao16bStrip + 8 * (lane - 1);
    const bool act = lane >= 1 && lane <= 62 && X < W;
    const int Xc = min(max(X, 0), ((W - 1) & ~7));                // every lane reads a valid 16-B column
    const int yb = cy << Ls, ye = min(yb + cs, H);
    const int bx = Xc >> Ls, xb = bx << Ls;
    auto row_ld = [&](int y) {
        return *(const __attribute__((address_space(1))) u4v*)(src + (size_t)min(max(y, 0), H - 1) * st + Xc);
    };
    u4v up = row_ld(yb - 1), cur = row_ld(yb), dn = row_ld(yb + 1);

    // ---- this lane's CTB: SAO parameters, 8.7.3.2 permissions of its 3x3 neighbourhood ----------
    const int rs = cy * g.wc + bx;
    u4v nb[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int nx = min(max(bx + k % 3 - 1, 0), g.wc - 1), ny = min(max(cy + k / 3 - 1, 0), g.hc - 1);
        nb[k] = *(const __attribute__((address_space(1))) u4v*)(crec + (size_t)(ny * g.wc + nx) * 8);
    }
    const u4v mt = *(const __attribute__((address_space(1))) u4v*)(crec + (size_t)rs * 8 + 4);
    const uint8_t* nf = pics[pic].nofilter;
    uint32_t allow = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int dx = k % 3 - 1, dy = k / 3 - 1;
        const int nx = bx + dx, ny = cy + dy;
        bool ok = nx >= 0 && ny >= 0 && nx < g.wc && ny < g.hc;
        const uint32_t ti = nb[4].y >> 16, to = nb[k].y >> 16;
        if (ok && nb[k].z != nb[4].z) {                          // other slice: the later sample's slice flag
            const bool o_first = to < ti || (to == ti && ny * g.wc + nx < rs);
            ok = ((o_first ? nb[4].w : nb[k].w) & P265R_CTU_LF_ACROSS_SLICES) != 0;
        }
        if (!g.lf_tiles && to != ti) ok = false;
        if (ok) allow |= 1u << k;
    }
    auto A = [&](int ay, int ax) { return ((allow >> (ay * 3 + ax)) & 1u) != 0; };
    // record dword 3: flags | SaoTypeIdx[3] << 8; dword 4: class[3] | dbk offsets; 5..7: offsets
    const int typ = (int)((nb[4].w >> (8 * (c + 1))) & 0xffu);
    const int cls = (int)((mt.x >> (8 * c)) & 0xffu);
    const uint32_t o = c == 0 ? mt.y : (c == 1 ? mt.z : mt.w);    // SaoOffsetVal[1..4], signed bytes
    const int ecls = typ == 2 ? (cls & 3) : 0;
    // edge neighbours: a at (dxa, dya), b at (-dxa, -dya) (Table 8-13 hPos / vPos)
    const int dxa = ecls == 1 ? 0 : (ecls == 3 ? 1 : -1);
    const int dya = ecls == 0 ? 0 : -1;

    // ---- which of the lane's 8 samples may change, per row kind (first / inner / last row of the
    // CTB row): a neighbour is usable iff inside the picture and its CTB allowed; only sample 0 / 7 can
    // leave the lane's CTB column, only the CTB row's first / last row its rows; samples at x >= W are
    // stored into the row padding and never read: don't care
    const int n_in = W - Xc;
    const bool ctb_first = Xc == xb, ctb_last = Xc + 8 == xb + cs;
    auto col_bits = [&](int dx, int ay) -> uint32_t {
        if (ay < 0) return 0u;
        if (dx == 0) return A(ay, 1) ? 0xffu : 0u;
        if (dx < 0) return (A(ay, 1) ? 0xfeu : 0u) | ((Xc > 0 && A(ay, ctb_first ? 0 : 1)) ? 1u : 0u);
        const uint32_t inner = n_in >= 8 ? 0x7fu : ((1u << max(n_in - 1, 0)) - 1u);
        return (A(ay, 1) ? inner : 0u) | ((n_in > 8 && A(ay, ctb_last ? 2 : 1)) ? 0x80u : 0u);
    };
    const int ylast = ye - 1;
    auto row_a = [&](int y, int dy) -> int {
        if (dy == 0) return 1;
        if (dy < 0) return y == yb ? 0 : 1;
        return y == ylast ? (y == H - 1 ? -1 : 2) : 1;
    };
    auto mask8 = [&](int y) -> uint32_t {
        if (typ == 0) return 0u;
        if (typ == 1) return 0xffu;
        return col_bits(dxa, row_a(y, dya)) & col_bits(-dxa, row_a(y, -dya));
    };
    const uint32_t m_top = mask8(yb), m_mid = mask8(yb + 1), m_bot = mask8(ylast);

    auto left_of = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x138, 0xf, 0xf, false); };
    auto right_of = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x130, 0xf, 0xf, false); };
    auto smp = [](const u4v& r, int i) -> int {                   // sample i (0..7) of a loaded row
        const uint32_t d = i < 2 ? r.x : (i < 4 ? r.y : (i < 6 ? r.z : r.w));
        return (int)((d >> (16 * (i & 1))) & 0xffffu);
    };
    auto off = [&](int e) { return (int)(int8_t)(o >> (8 * e)); };   // SaoOffsetVal[e + 1]
    const int bsh = bd - 5;

    for (int y = yb; y < ye; ++y) {
        const u4v nxt = row_ld(y + 2);                            // (in flight while this row is filtered)
        // samples beside the lane's column: lane l - 1's sample 7, lane l + 1's sample 0, per row
        const int ul = (int)(left_of(up.w) >> 16), ur = (int)(right_of(up.x) & 0xffffu);
        const int cl = (int)(left_of(cur.w) >> 16), cr = (int)(right_of(cur.x) & 0xffffu);
        const int dl = (int)(left_of(dn.w) >> 16), dr = (int)(right_of(dn.x) & 0xffffu);
        uint32_t nfm = 0;                                         // bit i: sample i untouched (PCM / bypass)
        if (nf) {
            const uint8_t* nr = nf + (size_t)((y << sub) >> 3) * g.nf_w;
            const int b0 = (Xc << sub) >> 3;
            if (nr[b0]) nfm |= sub ? 0x0fu : 0xffu;
            if (sub && b0 + 1 < g.nf_w && nr[b0 + 1]) nfm |= 0xf0u;
        }
        const uint32_t m = (y == yb ? m_top : (y == ylast ? m_bot : m_mid)) & ~nfm;
        uint32_t outw[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int r2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 2 * q + h;
                const int vv = smp(cur, i);
                // a: row dya, column i + dxa; b: row -dya, column i - dxa (every candidate at a
                // compile-time sample index, selected per lane class)
                const int cm = i == 0 ? cl : smp(cur, i > 0 ? i - 1 : 0), cp = i == 7 ? cr : smp(cur, i < 7 ? i + 1 : 7);
                const int um = i == 0 ? ul : smp(up, i > 0 ? i - 1 : 0), up0 = smp(up, i), upp = i == 7 ? ur : smp(up, i < 7 ? i + 1 : 7);
                const int dm = i == 0 ? dl : smp(dn, i > 0 ? i - 1 : 0), dn0 = smp(dn, i), dnp = i == 7 ? dr : smp(dn, i < 7 ? i + 1 : 7);
                const int a = dya == 0 ? (dxa < 0 ? cm : cp) : (dxa < 0 ? um : (dxa == 0 ? up0 : upp));
                const int b = dya == 0 ? (dxa < 0 ? cp : cm) : (dxa < 0 ? dnp : (dxa == 0 ? dn0 : dm));
                int e = 2 + (vv > a) - (vv < a) + (vv > b) - (vv < b);
                e = e == 2 ? 0 : (e < 2 ? e + 1 : e);               // edgeIdx 0..4
                const int k = ((vv >> bsh) - cls) & 31;             // band slot relative to the position
                const int idx = typ == 1 ? (k < 4 ? k + 1 : 0) : e;  // 1..4: SaoOffsetVal[idx]
                const int rv = idx ? min(max(vv + off(idx - 1), 0), maxv) : vv;
                r2[h] = ((m >> i) & 1u) ? rv : vv;
            }
            outw[q] = (uint32_t)r2[0] | (uint32_t)r2[1] << 16;
        }
        if (act)
            *(__attribute__((address_space(1))) u4v*)(dst + (size_t)y * st + Xc) = u4v{outw[0], outw[1], outw[2], outw[3]};
        up = cur;
        cur = dn;
        dn = nxt;
    }
}

}  // namespace p265r
