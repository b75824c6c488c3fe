"""CPU oracle: pure-Python/numpy restatement of the HEVC intra reconstruction path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker.  The product
path (p265_amd + libp265r.so) never calls into oracle/.

What it restates (H.265 v1 clause numbers; the reference file:line each function
follows is cited in its docstring):
  * 8.6.3 scaling (dequantisation)          <- decoder/scaling.py:4-47
  * 8.6.4.2 inverse DCT/DST, 8.6.2 residual <- decoder/transform.py:74-109 (reference is
    numerically wrong there; this follows the spec)
  * 8.4.4.2.2 reference sample availability/substitution, 8.4.4.2.3 filtering
                                            <- decoder/intra.py:186-305
  * 8.4.4.2.4-6 planar / DC / angular       <- decoder/intra.py:82-184
  * 8.6.7 picture construction (clip)       <- decoder/reconstruction.py:4-27
  * 6.4.1 z-scan availability               <- decoder/image.py:38-73, pps.py:246-262
  * 8.7.3 SAO (absent in the reference; sao.py:15-136 is syntax only)

Parity status: the front-end records that feed this oracle are pinned by the
reference's 95 golden trace files (tests/golden/gen_sanity_fixture.py).  The
planar, DC, horizontal-family angular, modes 18/26/34, neighbour filtering and
scaling functions are pinned against outputs of the reference's own functions
(tests/golden/gen_component_fixture.py).  The inverse transform, the vertical
angular modes the reference gets wrong, substitution when the bottom-left sample
is present, and SAO filtering have no reference output to pin against: for those
parity is UNPINNED by the reference and rests on spec restatement + known-answer
tests (tests/test_oracle_kat.py).

Sample arrays are raster numpy arrays indexed [y][x] (the reference uses x-major
[x][y] numpy arrays; transpose when comparing).
"""
import numpy as np

# ---------------------------------------------------------------------------
# Tables
# ---------------------------------------------------------------------------

# 64*sqrt(2)*cos(m*pi/64) as the integer values H.265 uses (distinct entries of the
# core transform; index 32 is cos(pi/2) = 0).  The 32x32 matrix follows from cosine
# symmetry; tests/golden/gen_component_fixture.py checks it against transform.py:7-72.
_COS64 = [64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67,
          64, 61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0]


def _cosv(a):
    a %= 128
    if a <= 32:
        return _COS64[a]
    if a < 64:
        return -_COS64[64 - a]
    if a <= 96:
        return -_COS64[a - 64]
    return _COS64[128 - a]


def dct32_matrix():
    """M[k][n]: basis k at spatial position n (transform.py:7-72 layout)."""
    m = np.zeros((32, 32), np.int64)
    for k in range(32):
        for n in range(32):
            m[k, n] = 64 if k == 0 else _cosv(k * (2 * n + 1))
    return m


DCT32 = dct32_matrix()
DST4 = np.array([[29, 55, 74, 84], [74, 74, 0, -74], [84, -29, -74, 55], [55, -84, 74, -29]], np.int64)

# intraPredAngle for modes 2..34 and invAngle for modes 11..25 (intra.py:15-22, spec 8.4.4.2.6)
INTRA_PRED_ANGLE = [32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26,
                    -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32]
INV_ANGLE = [-4096, -1638, -910, -630, -482, -390, -315, -256, -315, -390, -482, -630,
             -910, -1638, -4096]
LEVEL_SCALE = [40, 45, 51, 57, 64, 72]   # scaling.py:28

TB_CBF, TB_TSKIP, TB_BYPASS, TB_PCM = 1, 2, 4, 8
CTU_LF_ACROSS_SLICES = 1


def transform_matrix(log2, tr_type):
    """T[j][i] such that y[i] = sum_j T[j][i] * x[j] (spec 8.6.4.2)."""
    if tr_type == 1:
        return DST4
    step = 1 << (5 - log2)
    return DCT32[::step, : 1 << log2]


# ---------------------------------------------------------------------------
# Residual: scaling (8.6.3), transform (8.6.4.2), residual (8.6.2)
# ---------------------------------------------------------------------------

def dequantize(level, qp, log2, bit_depth):
    """d = Clip3(-32768, 32767, (L*m*levelScale[qP%6] << (qP/6) + (1 << (bdShift-1))) >> bdShift).

    Follows decoder/scaling.py:4-47 (formula at scaling.py:45-46), m = 16 (no scaling lists).
    """
    bd_shift = bit_depth + log2 - 5
    v = (np.asarray(level, np.int64) * 16 * LEVEL_SCALE[qp % 6]) << (qp // 6)
    v = (v + (1 << (bd_shift - 1))) >> bd_shift
    return np.clip(v, -32768, 32767)


def inverse_transform(d, log2, tr_type):
    """Two-stage separable inverse (8.6.4.2) incl. the intermediate clip; transform.py:89-109."""
    t = transform_matrix(log2, tr_type)
    e = t.T @ np.asarray(d, np.int64)              # columns (vertical) first
    g = np.clip((e + 64) >> 7, -32768, 32767)
    return g @ t                                    # then rows


def residual_block(level, log2, c_idx, qp, flags, bit_depth):
    """Residual samples r[y][x] for one TB (8.6.2).  level: N x N TransCoeffLevel [y][x]."""
    level = np.asarray(level, np.int64)
    if flags & (TB_BYPASS | TB_PCM):
        return level.copy()
    d = dequantize(level, qp, log2, bit_depth)
    if flags & TB_TSKIP:
        r = d << (5 + log2)                         # tsShift = 5 + Log2(nTbS) (= 7 for 4x4)
    else:
        tr_type = 1 if (log2 == 2 and c_idx == 0) else 0   # DST for intra luma 4x4
        r = inverse_transform(d, log2, tr_type)
    bd_shift = 20 - bit_depth
    return (r + (1 << (bd_shift - 1))) >> bd_shift


# ---------------------------------------------------------------------------
# Intra reference samples.  Linear order L[k] (k = 0..4N):
#   k = 0 .. 2N-1 : p[-1][2N-1-k]   (bottom-left upwards, left column)
#   k = 2N        : p[-1][-1]       (corner)
#   k = 2N+1+x    : p[x][-1]        (top row, x = 0..2N-1)
# This is exactly the scan order of the substitution process (intra.py:191-203).
# ---------------------------------------------------------------------------

def ref_positions(n):
    """(dx, dy) offsets from the TB's top-left sample for each linear index."""
    k = np.arange(4 * n + 1)
    dx = np.where(k < 2 * n, -1, np.where(k == 2 * n, -1, k - 2 * n - 1))
    dy = np.where(k < 2 * n, 2 * n - 1 - k, -1)
    return dx, dy


def substitute(vals, avail, bit_depth):
    """8.4.4.2.2 substitution over the linear order (intra.py:230-255, spec-correct form)."""
    vals = np.asarray(vals, np.int64).copy()
    avail = np.asarray(avail, bool)
    if not avail.any():
        return np.full(vals.shape, 1 << (bit_depth - 1), np.int64)
    if not avail[0]:
        vals[0] = vals[np.argmax(avail)]
    for k in range(1, len(vals)):
        if not avail[k]:
            vals[k] = vals[k - 1]
    return vals


def filter_flag(mode, n, c_idx):
    """8.4.4.2.3 filterFlag (intra.py:259-276); luma only in 4:2:0."""
    if c_idx != 0 or mode == 1 or n == 4:
        return False
    min_dist = min(abs(mode - 26), abs(mode - 10))
    thres = {8: 7, 16: 1, 32: 0}[n]
    return min_dist > thres


def filter_refs(p, n, mode, c_idx, strong_enabled, bit_depth):
    """8.4.4.2.3 [1 2 1] / strong bilinear filtering (intra.py:277-303)."""
    p = np.asarray(p, np.int64)
    if not filter_flag(mode, n, c_idx):
        return p.copy()
    corner, bl, tr = p[2 * n], p[0], p[4 * n]
    left_mid, top_mid = p[n], p[3 * n]     # p[-1][N-1], p[N-1][-1]
    if (strong_enabled and n == 32 and abs(corner + tr - 2 * top_mid) < (1 << (bit_depth - 5))
            and abs(corner + bl - 2 * left_mid) < (1 << (bit_depth - 5))):
        out = np.empty_like(p)
        out[2 * n] = corner
        y = np.arange(63)                          # pF[-1][y] = ((63-y)*c + (y+1)*p[-1][63] + 32) >> 6
        out[2 * n - 1 - y] = ((63 - y) * corner + (y + 1) * bl + 32) >> 6
        out[0] = bl
        x = np.arange(63)
        out[2 * n + 1 + x] = ((63 - x) * corner + (x + 1) * tr + 32) >> 6
        out[4 * n] = tr
        return out
    out = p.copy()
    out[1:-1] = (p[:-2] + 2 * p[1:-1] + p[2:] + 2) >> 2
    return out


def predict(p, n, mode, c_idx, bit_depth):
    """Intra prediction samples pred[y][x] from the (filtered) linear reference array.

    planar 8.4.4.2.5 (intra.py:82-94), DC 8.4.4.2.5 (intra.py:96-122), angular
    8.4.4.2.6 (intra.py:124-184, with the Appendix-A defects fixed).
    """
    p = np.asarray(p, np.int64)
    log2 = n.bit_length() - 1
    left = lambda y: p[2 * n - 1 - y]          # p[-1][y], y = -1 .. 2N-1
    top = lambda x: p[2 * n + 1 + x]           # p[x][-1], x = -1 .. 2N-1
    ys, xs = np.mgrid[0:n, 0:n]
    maxv = (1 << bit_depth) - 1
    if mode == 0:
        return ((n - 1 - xs) * left(ys) + (xs + 1) * top(n) + (n - 1 - ys) * top(xs)
                + (ys + 1) * left(n) + n) >> (log2 + 1)
    if mode == 1:
        dc = (int(sum(top(x) for x in range(n))) + int(sum(left(y) for y in range(n))) + n) >> (log2 + 1)
        pred = np.full((n, n), dc, np.int64)
        if c_idx == 0 and n < 32:
            pred[0, 0] = (left(0) + 2 * dc + top(0) + 2) >> 2
            pred[0, 1:] = (top(np.arange(1, n)) + 3 * dc + 2) >> 2
            pred[1:, 0] = (left(np.arange(1, n)) + 3 * dc + 2) >> 2
        return pred
    angle = INTRA_PRED_ANGLE[mode - 2]
    vertical = mode >= 18
    main = top if vertical else left           # ref[x] = p[-1+x][-1] (vertical) / p[-1][-1+x]
    side = left if vertical else top
    ref = {x: main(x - 1) for x in range(0, 2 * n + 1)}
    if angle < 0 and (n * angle) >> 5 < -1:
        inv = INV_ANGLE[mode - 11]
        for x in range((n * angle) >> 5, 0):
            ref[x] = side(-1 + ((x * inv + 128) >> 8))
    pred = np.empty((n, n), np.int64)
    for a in range(n):          # a: position along the prediction direction (y for vertical)
        idx = ((a + 1) * angle) >> 5
        fact = ((a + 1) * angle) & 31
        for b in range(n):      # b: position along the main reference
            if fact:
                v = ((32 - fact) * ref[b + idx + 1] + fact * ref[b + idx + 2] + 16) >> 5
            else:
                v = ref[b + idx + 1]
            if vertical:
                pred[a, b] = v
            else:
                pred[b, a] = v
    if c_idx == 0 and n < 32:
        if mode == 26:
            pred[:, 0] = np.clip(top(0) + ((left(np.arange(n)) - left(-1)) >> 1), 0, maxv)
        elif mode == 10:
            pred[0, :] = np.clip(left(0) + ((top(np.arange(n)) - top(-1)) >> 1), 0, maxv)
    return pred


# ---------------------------------------------------------------------------
# Picture-level geometry: CtbAddrRsToTs, MinTbAddrZs (6.5.1/6.5.2; pps.py:152-262)
# ---------------------------------------------------------------------------

class Geometry:
    def __init__(self, params, ctus):
        self.w, self.h = int(params["pic_width"]), int(params["pic_height"])
        self.ctb_log2 = int(params["ctb_log2_size"])
        self.min_tb_log2 = int(params["min_tb_log2_size"])
        self.ctb = 1 << self.ctb_log2
        self.wc = (self.w + self.ctb - 1) >> self.ctb_log2
        self.hc = (self.h + self.ctb - 1) >> self.ctb_log2
        tile = np.asarray(ctus["tile_id"], np.int64)
        order = np.lexsort((np.arange(len(tile)), tile))          # TS order = (tile, raster)
        self.rs2ts = np.empty(len(tile), np.int64)
        self.rs2ts[order] = np.arange(len(tile))
        self.ts_order = order
        self.tile = tile
        self.slice_addr = np.asarray(ctus["slice_addr"], np.int64)
        shift = self.ctb_log2 - self.min_tb_log2
        n_min = 1 << shift
        mort = np.zeros((n_min, n_min), np.int64)                # [y][x] within a CTB
        for y in range(n_min):
            for x in range(n_min):
                v = 0
                for i in range(shift):
                    m = 1 << i
                    v += (m * m if (x & m) else 0) + (2 * m * m if (y & m) else 0)
                mort[y, x] = v
        self.morton = mort
        self.shift = shift

    def ctb_of(self, x, y):
        return (y >> self.ctb_log2) * self.wc + (x >> self.ctb_log2)

    def min_tb_addr_zs(self, x, y):
        c = self.ctb_of(x, y)
        m = (1 << self.ctb_log2) - 1
        return (int(self.rs2ts[c]) << (2 * self.shift)) + int(
            self.morton[(y & m) >> self.min_tb_log2, (x & m) >> self.min_tb_log2])

    def available(self, xc, yc, xn, yn):
        """6.4.1 z-scan availability (image.py:38-73)."""
        if xn < 0 or yn < 0 or xn >= self.w or yn >= self.h:
            return False
        if self.min_tb_addr_zs(xn, yn) > self.min_tb_addr_zs(xc, yc):
            return False
        a, b = self.ctb_of(xc, yc), self.ctb_of(xn, yn)
        if a != b and (self.slice_addr[a] != self.slice_addr[b] or self.tile[a] != self.tile[b]):
            return False
        return True


def _plane_shapes(params):
    w, h = int(params["pic_width"]), int(params["pic_height"])
    return [(h, w), (h // 2, w // 2), (h // 2, w // 2)]


def reconstruct_picture(params, pic):
    """Pre-SAO reconstruction of one picture from records (see p265_amd/records.py).

    pic: dict with 'ctus' (structured, raster order), 'tbs' (structured) and 'coef' (int16).
    Returns [Y, Cb, Cr] as int64 arrays [y][x].  CTUs are visited in tile-scan order and
    TBs in their record (decode) order, as Cu.decode_leaf would (cu.py:483-494, 595-615).
    """
    geo = Geometry(params, pic["ctus"])
    planes = [np.zeros(s, np.int64) for s in _plane_shapes(params)]
    bd = [int(params["bit_depth_luma"]), int(params["bit_depth_chroma"]), int(params["bit_depth_chroma"])]
    strong = bool(params["strong_intra_smoothing"])
    ctus, tbs, coef = pic["ctus"], pic["tbs"], pic["coef"]
    for rs in geo.ts_order:
        c = ctus[rs]
        for t in tbs[int(c["tb_begin"]): int(c["tb_begin"]) + int(c["tb_count"])]:
            _recon_tb(geo, planes, t, coef, bd, strong)
    return planes


def _recon_tb(geo, planes, t, coef, bd, strong):
    c_idx, log2 = int(t["c_idx"]), int(t["log2_size"])
    n = 1 << log2
    x0, y0 = int(t["x"]), int(t["y"])
    flags, mode = int(t["flags"]), int(t["pred_mode"])
    plane = planes[c_idx]
    sub = 0 if c_idx == 0 else 1
    if flags & (TB_CBF | TB_PCM):
        off = int(t["coef_off"])
        level = np.asarray(coef[off: off + n * n], np.int64).reshape(n, n)
        res = residual_block(level, log2, c_idx, int(t["qp"]), flags, bd[c_idx])
    else:
        res = np.zeros((n, n), np.int64)
    if flags & TB_PCM:
        pred = np.zeros((n, n), np.int64)
    else:
        dx, dy = ref_positions(n)
        xc, yc = x0 << sub, y0 << sub
        avail = np.array([geo.available(xc, yc, (x0 + a) << sub, (y0 + b) << sub) for a, b in zip(dx, dy)])
        vals = np.zeros(4 * n + 1, np.int64)
        for k in np.nonzero(avail)[0]:
            vals[k] = plane[y0 + dy[k], x0 + dx[k]]
        p = substitute(vals, avail, bd[c_idx])
        p = filter_refs(p, n, mode, c_idx, strong, bd[c_idx])
        pred = predict(p, n, mode, c_idx, bd[c_idx])
    h, w = plane.shape
    rec = np.clip(pred + res, 0, (1 << bd[c_idx]) - 1)     # reconstruction.py:23-25
    plane[y0:min(y0 + n, h), x0:min(x0 + n, w)] = rec[: h - y0, : w - x0]


# ---------------------------------------------------------------------------
# SAO 8.7.3 (CTB granularity; pre-deblocking input)
# ---------------------------------------------------------------------------

_EO_POS = [((-1, 0), (1, 0)), ((0, -1), (0, 1)), ((-1, -1), (1, 1)), ((1, -1), (-1, 1))]  # (dx, dy)


def sao_picture(params, pic, recon):
    """Apply SAO to pre-SAO planes ``recon`` -> new planes (8.7.3.1-8.7.3.2)."""
    geo = Geometry(params, pic["ctus"])
    out = [r.copy() for r in recon]
    if not int(params["sample_adaptive_offset"]):
        return out
    ctus = pic["ctus"]
    nofilter = pic.get("nofilter")
    lf_tiles = bool(params["loop_filter_across_tiles"])
    for rs in range(len(ctus)):
        rx, ry = rs % geo.wc, rs // geo.wc
        c = ctus[rs]
        for c_idx in range(3):
            typ = int(c["sao_type"][c_idx])
            if typ == 0:
                continue
            sub = 0 if c_idx == 0 else 1
            bd = int(params["bit_depth_luma"] if c_idx == 0 else params["bit_depth_chroma"])
            rec = recon[c_idx]
            H, W = rec.shape
            cs = geo.ctb >> sub
            x0, y0 = rx * cs, ry * cs
            x1, y1 = min(x0 + cs, W), min(y0 + cs, H)
            blk = rec[y0:y1, x0:x1]
            offs = [0] + [int(v) for v in c["sao_offset"][c_idx]]
            if typ == 1:
                shift = bd - 5
                table = np.zeros(32, np.int64)
                band = int(c["sao_class"][c_idx])
                for k in range(4):
                    table[(k + band) & 31] = k + 1
                idx = table[blk >> shift]
                new = np.clip(blk + np.asarray(offs)[idx], 0, (1 << bd) - 1)
            else:
                (ax, ay), (bx, by) = _EO_POS[int(c["sao_class"][c_idx])]
                yy, xx = np.mgrid[y0:y1, x0:x1]
                ok = np.ones(blk.shape, bool)
                nb = []
                for dx, dy in ((ax, ay), (bx, by)):
                    xn, yn = xx + dx, yy + dy
                    inside = (xn >= 0) & (yn >= 0) & (xn < W) & (yn < H)
                    ok &= inside
                    xn_c, yn_c = np.clip(xn, 0, W - 1), np.clip(yn, 0, H - 1)
                    nb.append(rec[yn_c, xn_c])
                    # neighbour CTB checks (slices / tiles), evaluated per neighbouring CTB
                    nrs = ((yn_c << sub) >> geo.ctb_log2) * geo.wc + ((xn_c << sub) >> geo.ctb_log2)
                    for other in np.unique(nrs[inside]):
                        if other == rs:
                            continue
                        bad = False
                        if geo.slice_addr[other] != geo.slice_addr[rs]:
                            if geo.rs2ts[other] < geo.rs2ts[rs]:
                                bad = not (int(ctus[rs]["flags"]) & CTU_LF_ACROSS_SLICES)
                            else:
                                bad = not (int(ctus[other]["flags"]) & CTU_LF_ACROSS_SLICES)
                        if not lf_tiles and geo.tile[other] != geo.tile[rs]:
                            bad = True
                        if bad:
                            ok &= ~((nrs == other) & inside)
                edge = 2 + np.sign(blk - nb[0]) + np.sign(blk - nb[1])
                edge = np.where(edge == 2, 0, np.where(edge < 2, edge + 1, edge))
                new = np.where(ok, np.clip(blk + np.asarray(offs)[edge], 0, (1 << bd) - 1), blk)
            if nofilter is not None:
                yy, xx = np.mgrid[y0:y1, x0:x1]
                nfw = (geo.w + 7) >> 3
                skip = np.asarray(nofilter)[((yy << sub) >> 3) * nfw + ((xx << sub) >> 3)] != 0
                new = np.where(skip, blk, new)
            out[c_idx][y0:y1, x0:x1] = new
    return out


def decode_picture(params, pic):
    """Pre-SAO recon followed by SAO. Returns (recon, out), each [Y, Cb, Cr]."""
    rec = reconstruct_picture(params, pic)
    return rec, sao_picture(params, pic, rec)
