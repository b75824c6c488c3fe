// SAO only (8.7.3) for 16-bit samples (BitDepth 9..12), batches without deblocking: a
// streaming strip kernel like sao_strip16.h, 8 samples (16 B) per lane.  One wave = one CTB row of one
// component over a strip of 62 x 8 samples (lane l: the 8 samples at x = 496 s + 8 (l - 1); lanes 0 and
// 63 only supply the neighbours of lanes 1 and 62); the wave walks down its CTB row with the rows above,
// at and below the current one in registers, so every sample is read once (+ 2 halo rows per CTB
// height) and written once, each row one coalesced load and store per wave instruction.  A lane's 8
// samples lie in one CTB (8 divides every CTB width down to CTB 16 chroma), so its SaoTypeIdx, class,
// offsets and 8.7.3.2 neighbourhood permissions are per-lane constants; the samples beside the lane's
// column come from lanes l -/+ 1 (DPP wave shifts).  Per sample: band (bandShift = BitDepth - 5) or
// edge class and its SaoOffsetVal, two samples per packed 16-bit instruction; PCM / bypass samples
// (nofilter) untouched.  Main 10, 512 x 1080p: 2.05 ms per-sample form -> 1.44 ms packed (6.4 GB).
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

__device__ __forceinline__ int off_e(uint32_t o, int e) { return (int)(int8_t)(o >> (8 * e)); }   // SaoOffsetVal[e + 1]

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
    // Packed form: two samples per dword and VOP3P instruction.  Every row is kept with its copies shifted by
    // one sample (mi: sample i - 1, pl: sample i + 1; the lane's outer neighbours by DPP), built once when the
    // row is loaded; the lane's edge class picks its neighbour rows a / b once per row.  Per dword: the two
    // signs by clamped packed differences, and one byte-permute lookup of a per-lane table of the offsets
    // biased by 128 (band: slots 0..3, 4 = none; edge: s + 2 = 0..4 -> SaoOffsetVal[1, 2, -, 3, 4]); samples
    // outside the row's mask keep their value.
    typedef short s2v __attribute__((ext_vector_type(2)));
    auto as_s2 = [](uint32_t x) { return __builtin_bit_cast(s2v, x); };
    auto as_u = [](s2v x) { return __builtin_bit_cast(uint32_t, x); };
    auto pmax = [&](uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_max(as_s2(a), as_s2(b))); };
    auto pmin = [&](uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_min(as_s2(a), as_s2(b))); };
    auto psub = [&](uint32_t a, uint32_t b) { return as_u(as_s2(a) - as_s2(b)); };
    auto padd = [&](uint32_t a, uint32_t b) { return as_u(as_s2(a) + as_s2(b)); };
    struct Row { u4v v, mi, pl; };
    auto shifted = [&](const u4v& r) {
        const uint32_t lw = left_of(r.w), rx = right_of(r.x);
        const uint32_t t1 = __builtin_amdgcn_alignbit(r.y, r.x, 16), t2 = __builtin_amdgcn_alignbit(r.z, r.y, 16),
                       t3 = __builtin_amdgcn_alignbit(r.w, r.z, 16);
        return Row{r, u4v{__builtin_amdgcn_alignbit(r.x, lw, 16), t1, t2, t3}, u4v{t1, t2, t3, __builtin_amdgcn_alignbit(rx, r.w, 16)}};
    };
    // the lane's offset table: bytes 0..4 of (thi:tlo), each SaoOffsetVal + 128; byte 5 (= 0) fills the high bytes
    auto ob = [&](int e) { return (uint32_t)(off_e(o, e) + 128) & 0xffu; };
    uint32_t tlo, thi;
    if (typ == 1) { tlo = ob(0) | ob(1) << 8 | ob(2) << 16 | ob(3) << 24; thi = 128u; }
    else { tlo = ob(0) | ob(1) << 8 | 128u << 16 | ob(2) << 24; thi = ob(3); }
    const int bsh = bd - 5;                                       // bandShift
    const uint32_t bshv = (uint32_t)bsh * 0x00010001u, clsv = (uint32_t)cls * 0x00010001u;
    const uint32_t maxvv = (uint32_t)maxv * 0x00010001u;
    Row rup = shifted(up), rcur = shifted(cur), rdn = shifted(dn);
    for (int y = yb; y < ye; ++y) {
        const u4v nxt = row_ld(y + 2);                            // (in flight while this row is filtered)
        uint32_t nfm = 0;                                         // bit i: sample i untouched (PCM / bypass)
        if (nf) {
            const uint8_t* nr = nf + (size_t)((y << sub) >> 3) * g.nf_w;
            const int b0 = (Xc << sub) >> 3;
            if (nr[b0]) nfm |= sub ? 0x0fu : 0xffu;
            if (sub && b0 + 1 < g.nf_w && nr[b0 + 1]) nfm |= 0xf0u;
        }
        const uint32_t m = (y == yb ? m_top : (y == ylast ? m_bot : m_mid)) & ~nfm;
        const u4v av = ecls == 0 ? rcur.mi : (ecls == 1 ? rup.v : (ecls == 2 ? rup.mi : rup.pl));
        const u4v bv = ecls == 0 ? rcur.pl : (ecls == 1 ? rdn.v : (ecls == 2 ? rdn.pl : rdn.mi));
        uint32_t outw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t cv = rcur.v[j];
            uint32_t sel;
            if (typ == 1) {                                       // band slot min(k, 4), k = (v >> bandShift) - position
                const uint32_t k = as_u(as_s2(psub(as_u(__builtin_bit_cast(s2v, cv) >> as_s2(bshv)), clsv))) & 0x001f001fu;
                sel = pmin(k, 0x00040004u);
            } else {                                              // s + 2, s = sign(v - a) + sign(v - b)
                const uint32_t sa = pmax(pmin(psub(cv, av[j]), 0x00010001u), 0xffffffffu);
                const uint32_t sb = pmax(pmin(psub(cv, bv[j]), 0x00010001u), 0xffffffffu);
                sel = padd(padd(sa, sb), 0x00020002u);
            }
            const uint32_t ofs = psub(__builtin_amdgcn_perm(thi, tlo, sel | 0x05000500u), 0x00800080u);
            const uint32_t rv = pmin(pmax(padd(cv, ofs), 0u), maxvv);
            const uint32_t mk = ((m >> (2 * j)) & 1u ? 0x0000ffffu : 0u) | ((m >> (2 * j + 1)) & 1u ? 0xffff0000u : 0u);
            outw[j] = (rv & mk) | (cv & ~mk);
        }
        if (act)
            *(__attribute__((address_space(1))) u4v*)(dst + (size_t)y * st + Xc) = u4v{outw[0], outw[1], outw[2], outw[3]};
        rup = rcur;
        rcur = rdn;
        rdn = shifted(nxt);
    }
}

}  // namespace p265r
