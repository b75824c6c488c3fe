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
  * 8.7.2 deblocking (absent in the reference: pps.py:122-131 / slice.py:170-179 parse
    its controls, no filter exists)
  * 8.7.3 SAO (absent in the reference; sao.py:15-136 is syntax only)

Parity status: the front-end records that feed this oracle are pinned by the
reference's 95 golden trace files (tests/golden/gen_sanity_fixture.py).  The
planar, DC, horizontal-family angular, modes 18/26/34, neighbour filtering and
scaling functions are pinned against outputs of the reference's own functions
(tests/golden/gen_component_fixture.py).  The inverse transform, the vertical
angular modes the reference gets wrong, substitution when the bottom-left sample
is present, deblocking and SAO filtering have no reference output to pin against: for those
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

# ---------------------------------------------------------------------------
# Scaling lists (7.3.4 syntax, 7.4.5 semantics / ScalingFactor derivation) -- the ScalingFactor
# branch of decoder/scaling.py:32-44 (m[x][y] = sps.scaling_factor[size_id][matrix_id][x][y]).
# The reference's list derivation (sld.py) is broken, its default tables are data:
# Table 7-6 below equals sld.py:13-33 (tests/test_scaling_lists.py).
# ---------------------------------------------------------------------------
SL_DEFAULT_8X8_INTRA = [16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18, 17, 18, 18, 17, 18, 21, 19,
                        20, 21, 20, 19, 21, 24, 22, 22, 24, 24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29, 31, 35,
                        35, 31, 29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115]
SL_DEFAULT_8X8_INTER = [16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18, 18, 18, 18, 18, 18, 20, 20,
                        20, 20, 20, 20, 20, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28, 28, 28,
                        28, 28, 28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91]
# ABI layout of the intra ScalingFactor arrays (include/p265r.h p265r_set_scaling_factors): m[y][x] per
# (sizeId, matrixId): 4x4 Y/Cb/Cr, 8x8 Y/Cb/Cr, 16x16 Y/Cb/Cr, 32x32 Y; 2032 bytes
SF_OFFSETS = {(0, 0): 0, (0, 1): 16, (0, 2): 32, (1, 0): 48, (1, 1): 112, (1, 2): 176,
              (2, 0): 240, (2, 1): 496, (2, 2): 752, (3, 0): 1008}
SF_BYTES = 2032


def diag_scan(blk):
    """6.5.3 up-right diagonal scan of a blk x blk block: [(x, y)] in scan order."""
    out, x, y = [], 0, 0
    while len(out) < blk * blk:
        while y >= 0:
            if x < blk and y < blk:
                out.append((x, y))
            y -= 1
            x += 1
        y, x = x, 0
    return out


def default_scaling_list(size_id, matrix_id):
    """Table 7-5 (4x4: flat 16) / Table 7-6 (8x8 and larger: intra for matrixId 0..2, inter 3..5)."""
    if size_id == 0:
        return [16] * 16
    return list(SL_DEFAULT_8X8_INTRA if matrix_id < 3 else SL_DEFAULT_8X8_INTER)


def scaling_lists_from_syntax(sld):
    """scaling_list_data() syntax values -> (ScalingList[sizeId][matrixId], dc[sizeId][matrixId]) (7.4.5).

    ``sld``: {(size_id, matrix_id): ("pred", delta) | ("coded", dc_coef_minus8 or None, [delta_coef, ...])} for
    sizeId 0..3, matrixId 0..5 (sizeId 3: 0 and 3, the numbering of the 2016+ editions; v1's 0 / 1 code the
    same two lists).  Predicted lists copy refMatrixId = matrixId - delta * (sizeId == 3 ? 3 : 1), or the
    default list (Table 7-5/7-6) and DC 16 when delta is 0."""
    lists, dcs = {}, {}
    for size_id in range(4):
        for matrix_id in range(0, 6, 3 if size_id == 3 else 1):
            kind = sld[(size_id, matrix_id)]
            if kind[0] == "pred":
                delta = kind[1]
                if delta == 0:
                    lists[(size_id, matrix_id)] = default_scaling_list(size_id, matrix_id)
                    dcs[(size_id, matrix_id)] = 16
                else:
                    ref = matrix_id - delta * (3 if size_id == 3 else 1)
                    lists[(size_id, matrix_id)] = list(lists[(size_id, ref)])
                    dcs[(size_id, matrix_id)] = dcs.get((size_id, ref), 16)
            else:
                _, dc_minus8, deltas = kind
                nxt = 8
                if size_id > 1:
                    nxt = dc_minus8 + 8
                    dcs[(size_id, matrix_id)] = nxt
                vals = []
                for dlt in deltas:
                    nxt = (nxt + dlt + 256) % 256
                    vals.append(nxt)
                lists[(size_id, matrix_id)] = vals
    return lists, dcs


def scaling_factors(lists, dcs):
    """ScalingFactor (7.4.5) of the intra matrices used by 4:2:0 (sizeId 0..2: Y, Cb, Cr; sizeId 3: Y) as
    {(size_id, matrix_id): m[y][x]} (int64 arrays; the spec's ScalingFactor[..][x][y] transposed)."""
    out = {}
    for (size_id, matrix_id) in SF_OFFSETS:
        n = 4 << size_id
        lst = lists[(size_id, matrix_id)]
        blk = 4 if size_id == 0 else 8
        rep = n // blk
        m = np.zeros((n, n), np.int64)
        for i, (x, y) in enumerate(diag_scan(blk)):
            m[y * rep:(y + 1) * rep, x * rep:(x + 1) * rep] = lst[i]
        if size_id > 1:
            m[0, 0] = dcs[(size_id, matrix_id)]
        out[(size_id, matrix_id)] = m
    return out


def scaling_factor_bytes(factors):
    """{(size_id, matrix_id): m[y][x]} -> the 2032-byte ABI array (p265r_set_scaling_factors)."""
    b = np.zeros(SF_BYTES, np.uint8)
    for k, off in SF_OFFSETS.items():
        m = np.asarray(factors[k])
        b[off:off + m.size] = m.reshape(-1)
    return b


def factor_of(sf_bytes, log2, c_idx):
    """m[y][x] of a TB (log2 size, component) from the 2032-byte ABI array (intra: matrixId = c_idx)."""
    off = SF_OFFSETS[(log2 - 2, c_idx)]
    n = 1 << log2
    return np.asarray(sf_bytes[off:off + n * n], np.int64).reshape(n, n)


CTU_LF_ACROSS_SLICES, CTU_DEBLOCK = 1, 2

# Table 8-12: beta' (Q = 0..51) and tC' (Q = 0..53)
BETA_TABLE = [0] * 16 + list(range(6, 19)) + list(range(20, 65, 2))
TC_TABLE = ([0] * 18 + [1] * 9 + [2] * 4 + [3] * 4 + [4] * 3 + [5] * 2 + [6] * 2
            + [7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24])
assert len(BETA_TABLE) == 52 and len(TC_TABLE) == 54


def qpc_from_qpi(qpi):
    """Table 8-10 (ChromaArrayType == 1); the reference's copy is cu.py:575-591."""
    if qpi < 30:
        return qpi
    if qpi >= 43:
        return qpi - 6
    return [29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37][qpi - 30]


def transform_matrix(log2, tr_type):
    """T[j][i] such that y[i] = sum_j T[j][i] * x[j] (spec 8.6.4.2)."""
    if tr_type == 1:
        return DST4
    step = 1 << (5 - log2)
    return DCT32[::step, : 1 << log2]


# ---------------------------------------------------------------------------
# Residual: scaling (8.6.3), transform (8.6.4.2), residual (8.6.2)
# ---------------------------------------------------------------------------

def dequantize(level, qp, log2, bit_depth, m=None):
    """d = Clip3(-32768, 32767, (L*m*levelScale[qP%6] << (qP/6) + (1 << (bdShift-1))) >> bdShift).

    Follows decoder/scaling.py:4-47 (formula at scaling.py:45-46): m = 16 without scaling lists, else the
    TB's ScalingFactor m[y][x] (scaling.py:32-44; applied to 4x4 transform-skip blocks too, 8.6.4.2).
    """
    bd_shift = bit_depth + log2 - 5
    mm = 16 if m is None else np.asarray(m, np.int64)
    v = (np.asarray(level, np.int64) * mm * LEVEL_SCALE[qp % 6]) << (qp // 6)
    v = (v + (1 << (bd_shift - 1))) >> bd_shift
    return np.clip(v, -32768, 32767)


def inverse_transform(d, log2, tr_type):
    """Two-stage separable inverse (8.6.4.2) incl. the intermediate clip; transform.py:89-109."""
    t = transform_matrix(log2, tr_type)
    e = t.T @ np.asarray(d, np.int64)              # columns (vertical) first
    g = np.clip((e + 64) >> 7, -32768, 32767)
    return g @ t                                    # then rows


def residual_block(level, log2, c_idx, qp, flags, bit_depth, m=None):
    """Residual samples r[y][x] for one TB (8.6.2).  level: N x N TransCoeffLevel [y][x]; m: its
    ScalingFactor [y][x] (None: flat 16)."""
    level = np.asarray(level, np.int64)
    if flags & (TB_BYPASS | TB_PCM):
        return level.copy()
    d = dequantize(level, qp, log2, bit_depth, m)
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
    sf = params.get("scaling_factors") if int(params.get("scaling_list_enabled", 0)) else None
    if int(params.get("scaling_list_enabled", 0)) and sf is None:
        raise ValueError("scaling_list_enabled needs params['scaling_factors'] (scaling_factor_bytes)")
    ctus, tbs, coef = pic["ctus"], pic["tbs"], pic["coef"]
    for rs in geo.ts_order:
        c = ctus[rs]
        for t in tbs[int(c["tb_begin"]): int(c["tb_begin"]) + int(c["tb_count"])]:
            _recon_tb(geo, planes, t, coef, bd, strong, sf)
    return planes


def _recon_tb(geo, planes, t, coef, bd, strong, sf=None):
    c_idx, log2 = int(t["c_idx"]), int(t["log2_size"])
    n = 1 << log2
    x0, y0 = int(t["x"]), int(t["y"])
    flags, mode = int(t["flags"]), int(t["pred_mode"])
    plane = planes[c_idx]
    sub = 0 if c_idx == 0 else 1
    if flags & (TB_CBF | TB_PCM):
        off = int(t["coef_off"])
        level = np.asarray(coef[off: off + n * n], np.int64).reshape(n, n)
        m = None if sf is None else factor_of(sf, log2, c_idx)
        res = residual_block(level, log2, c_idx, int(t["qp"]), flags, bd[c_idx], m)
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
# SAO 8.7.3 (CTB granularity; input = the deblocked picture)
# ---------------------------------------------------------------------------

_EO_POS = [((-1, 0), (1, 0)), ((0, -1), (0, 1)), ((-1, -1), (1, 1)), ((1, -1), (-1, 1))]  # (dx, dy)


def sao_picture(params, pic, recon):
    """Apply SAO to the deblocked planes ``recon`` -> new planes (8.7.3.1-8.7.3.2)."""
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


# ---------------------------------------------------------------------------
# Deblocking 8.7.2 (all-intra: bS = 2 on every transform-block edge of the 8x8 grid)
# ---------------------------------------------------------------------------

def _clip3(lo, hi, v):
    return lo if v < lo else (hi if v > hi else v)


def deblock_luma_segment(p, q, qp_p, qp_q, beta_offset_div2, tc_offset_div2, no_p, no_q, bit_depth=8, bs=2):
    """One 4-line luma edge segment: decisions 8.7.2.5.3 / 8.7.2.5.6, filtering 8.7.2.5.7.

    p[i][k], q[i][k]: sample i away from the edge (i = 0..3) on line k (k = 0..3).
    Returns new (p, q) as lists of lists (only p0..p2 / q0..q2 can change).
    """
    p = [list(map(int, r)) for r in p]
    q = [list(map(int, r)) for r in q]
    qpl = (qp_q + qp_p + 1) >> 1
    beta = BETA_TABLE[_clip3(0, 51, qpl + (beta_offset_div2 << 1))] * (1 << (bit_depth - 8))
    tc = TC_TABLE[_clip3(0, 53, qpl + 2 * (bs - 1) + (tc_offset_div2 << 1))] * (1 << (bit_depth - 8))
    dp0 = abs(p[2][0] - 2 * p[1][0] + p[0][0])
    dp3 = abs(p[2][3] - 2 * p[1][3] + p[0][3])
    dq0 = abs(q[2][0] - 2 * q[1][0] + q[0][0])
    dq3 = abs(q[2][3] - 2 * q[1][3] + q[0][3])
    dpq0, dpq3 = dp0 + dq0, dp3 + dq3
    dp, dq = dp0 + dp3, dq0 + dq3
    d = dpq0 + dpq3
    if d >= beta:
        return p, q

    def dsam(k, dpq):
        return (dpq < (beta >> 2) and abs(p[3][k] - p[0][k]) + abs(q[0][k] - q[3][k]) < (beta >> 3)
                and abs(p[0][k] - q[0][k]) < ((5 * tc + 1) >> 1))

    strong = dsam(0, 2 * dpq0) and dsam(3, 2 * dpq3)
    dep = dp < ((beta + (beta >> 1)) >> 3)
    deq = dq < ((beta + (beta >> 1)) >> 3)
    maxv = (1 << bit_depth) - 1
    for k in range(4):
        p0, p1, p2, p3 = p[0][k], p[1][k], p[2][k], p[3][k]
        q0, q1, q2, q3 = q[0][k], q[1][k], q[2][k], q[3][k]
        if strong:
            np_ = [_clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3),
                   _clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2),
                   _clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3)]
            nq = [_clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3),
                  _clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2),
                  _clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3)]
            ndp = ndq = 3
        else:
            delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4
            if abs(delta) >= tc * 10:
                continue
            delta = _clip3(-tc, tc, delta)
            np_ = [_clip3(0, maxv, p0 + delta), p1, p2]
            nq = [_clip3(0, maxv, q0 - delta), q1, q2]
            if dep:
                np_[1] = _clip3(0, maxv, p1 + _clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1))
            if deq:
                nq[1] = _clip3(0, maxv, q1 + _clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1))
            ndp, ndq = (2 if dep else 1), (2 if deq else 1)
        if no_p:
            ndp = 0
        if no_q:
            ndq = 0
        for i in range(ndp):
            p[i][k] = np_[i]
        for i in range(ndq):
            q[i][k] = nq[i]
    return p, q


def deblock_chroma_line(p0, p1, q0, q1, tc, no_p, no_q, bit_depth=8):
    """8.7.2.5.5 filtering of one chroma line across an edge (bS = 2)."""
    maxv = (1 << bit_depth) - 1
    delta = _clip3(-tc, tc, ((((q0 - p0) << 2) + p1 - q1 + 4) >> 3))
    return (p0 if no_p else _clip3(0, maxv, p0 + delta)), (q0 if no_q else _clip3(0, maxv, q0 - delta))


def chroma_tc(qp_p, qp_q, c_qp_pic_offset, tc_offset_div2, bit_depth=8):
    """tC of a chroma edge (8.7.2.5.5): QpC from Table 8-10 on ((QpQ + QpP + 1) >> 1) + cQpPicOffset."""
    qpc = qpc_from_qpi(((qp_q + qp_p + 1) >> 1) + c_qp_pic_offset)
    return TC_TABLE[_clip3(0, 53, qpc + 2 + (tc_offset_div2 << 1))] * (1 << (bit_depth - 8))


def _unpack_offsets(v):
    b, t = int(v) & 15, (int(v) >> 4) & 15
    return (b - 16 if b >= 8 else b), (t - 16 if t >= 8 else t)


def deblock_picture(params, pic, recon):
    """8.7.2 deblocking of the reconstructed planes -> new planes [Y, Cb, Cr].

    Edges: luma transform-block boundaries (the spec's transform and, for intra NxN,
    prediction edges; the latter sit at 4-sample offsets and never reach the 8x8 grid)
    on the 8x8 luma grid, found here from a per-4x4 map of TB indices.  bS = 2 for every
    edge (all-intra).  All vertical edges of the picture are filtered first (input: the
    reconstruction), then all horizontal edges (input: the vertically filtered picture).
    filterEdgeFlag (8.7.2.3): no edge on the picture boundary; at a tile boundary only
    with loop_filter_across_tiles; at a slice boundary only with the flag of the slice
    containing q0; no edge owned by a CTU whose slice has deblocking disabled.  The
    slice's offsets are those of the CTU containing q0.
    """
    ctus = pic["ctus"]
    out = [np.array(r, np.int64, copy=True) for r in recon]
    if not (np.asarray(ctus["flags"]) & CTU_DEBLOCK).any():
        return out
    geo = Geometry(params, ctus)
    w, h = geo.w, geo.h
    bd = [int(params["bit_depth_luma"]), int(params["bit_depth_chroma"]), int(params["bit_depth_chroma"])]
    lf_tiles = bool(params["loop_filter_across_tiles"])
    cqp = [0, int(params.get("pps_cb_qp_offset", 0)), int(params.get("pps_cr_qp_offset", 0))]
    tbid = np.full((h >> 2, w >> 2), -1, np.int64)
    qp4 = np.zeros((h >> 2, w >> 2), np.int64)
    for i, t in enumerate(pic["tbs"]):
        if int(t["c_idx"]) != 0:
            continue
        x4, y4, n4 = int(t["x"]) >> 2, int(t["y"]) >> 2, 1 << (int(t["log2_size"]) - 2)
        tbid[y4:y4 + n4, x4:x4 + n4] = i
        qp4[y4:y4 + n4, x4:x4 + n4] = int(t["qp"]) - 6 * (bd[0] - 8)     # QpY = Qp'Y - QpBdOffsetY
    nofilter = pic.get("nofilter")
    nfw = (w + 7) >> 3

    def nf(x, y):
        return nofilter is not None and bool(nofilter[(y >> 3) * nfw + (x >> 3)])

    def edge_ok(xp, yp, xq, yq):
        """bS = 2 and filterEdgeFlag for the luma positions of p0 and q0."""
        if tbid[yp >> 2, xp >> 2] == tbid[yq >> 2, xq >> 2]:
            return False
        a, b = geo.ctb_of(xq, yq), geo.ctb_of(xp, yp)
        cq = ctus[a]
        if not (int(cq["flags"]) & CTU_DEBLOCK):
            return False
        if a != b:
            if not lf_tiles and geo.tile[a] != geo.tile[b]:
                return False
            if geo.slice_addr[a] != geo.slice_addr[b] and not (int(cq["flags"]) & CTU_LF_ACROSS_SLICES):
                return False
        return True

    for vertical in (True, False):
        # ---- luma: edges every 8 samples, 4-line segments ----------------------------
        Y = out[0]
        e_max, s_max = (w, h) if vertical else (h, w)
        for e in range(8, e_max, 8):
            for s0 in range(0, s_max, 4):
                xq, yq = (e, s0) if vertical else (s0, e)
                xp, yp = (e - 1, s0) if vertical else (s0, e - 1)
                if not edge_ok(xp, yp, xq, yq):
                    continue
                beta_off, tc_off = _unpack_offsets(ctus[geo.ctb_of(xq, yq)]["deblock_offsets"])
                if vertical:
                    P = [[Y[s0 + k, e - 1 - i] for k in range(4)] for i in range(4)]
                    Q = [[Y[s0 + k, e + i] for k in range(4)] for i in range(4)]
                else:
                    P = [[Y[e - 1 - i, s0 + k] for k in range(4)] for i in range(4)]
                    Q = [[Y[e + i, s0 + k] for k in range(4)] for i in range(4)]
                P, Q = deblock_luma_segment(P, Q, qp4[yp >> 2, xp >> 2], qp4[yq >> 2, xq >> 2], beta_off, tc_off,
                                            nf(xp, yp), nf(xq, yq), bd[0])
                for i in range(3):
                    for k in range(4):
                        if vertical:
                            Y[s0 + k, e - 1 - i], Y[s0 + k, e + i] = P[i][k], Q[i][k]
                        else:
                            Y[e - 1 - i, s0 + k], Y[e + i, s0 + k] = P[i][k], Q[i][k]
        # ---- chroma (4:2:0): edges every 8 chroma samples, bS of the luma edge at 2x --------
        for c in (1, 2):
            C = out[c]
            ch, cw = C.shape
            e_max, s_max = (cw, ch) if vertical else (ch, cw)
            for e in range(8, e_max, 8):
                for s0 in range(0, s_max, 4):
                    xq, yq = ((e, s0) if vertical else (s0, e))
                    xp, yp = ((e - 1, s0) if vertical else (s0, e - 1))
                    lq = (xq << 1, yq << 1)
                    lp = ((xq << 1) - 1, yq << 1) if vertical else (xq << 1, (yq << 1) - 1)
                    if not edge_ok(lp[0], lp[1], lq[0], lq[1]):
                        continue
                    _, tc_off = _unpack_offsets(ctus[geo.ctb_of(*lq)]["deblock_offsets"])
                    tc = chroma_tc(qp4[lp[1] >> 2, lp[0] >> 2], qp4[lq[1] >> 2, lq[0] >> 2], cqp[c], tc_off, bd[c])
                    no_p, no_q = nf(*lp), nf(*lq)
                    for k in range(4):
                        if vertical:
                            r = s0 + k
                            C[r, e - 1], C[r, e] = deblock_chroma_line(C[r, e - 1], C[r, e - 2], C[r, e], C[r, e + 1],
                                                                       tc, no_p, no_q, bd[c])
                        else:
                            x = s0 + k
                            C[e - 1, x], C[e, x] = deblock_chroma_line(C[e - 1, x], C[e - 2, x], C[e, x], C[e + 1, x],
                                                                       tc, no_p, no_q, bd[c])
    return out


def decode_picture(params, pic):
    """Reconstruction, then the in-loop filters (deblocking, SAO).  Returns (recon, out),
    each [Y, Cb, Cr]: recon is the deblocking input, out the decoded picture."""
    rec = reconstruct_picture(params, pic)
    return rec, sao_picture(params, pic, deblock_picture(params, pic, rec))
