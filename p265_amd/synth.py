"""Seeded synthetic all-intra pictures (records) for parity tests and the benchmark.

Shapes follow SURVEY.md §8(d) (statistics measured on sanity.bin, Appendix B):
  * CU quadtree probabilities hit the luma area mix 26.2 % 4x4 / 30.7 % 8x8 /
    26.3 % 16x16 / 16.8 % 32x32 TBs, with ~41 % of 8x8 CUs NxN;
  * cbf_luma ~73/82/95/100 % for 4/8/16/32, chroma cbf ~13 %;
  * non-zero density per coded luma TB ~22/13/16/20 %, low-frequency biased,
    geometric magnitudes (p ~ 0.6), uniform signs;
  * transform_skip on ~0.8 % of coded luma 4x4; SAO per CTU ~2 % off / 16 % BO / 82 % EO.
Deblocking is considered disabled (the SAO input is the reconstruction).

``perf=True`` uses the mode histogram of sanity.bin and QP 32; ``perf=False`` (parity)
uses uniform modes 0..34, QP 22..37, random strong-smoothing-prone flat areas and
optional multiple slices / tiles.

Above 8 bits (params bit_depth_luma / _chroma, Main 10) the records carry qP' = QpY + QpBdOffset
(parity pictures draw QpY from -QpBdOffsetY.. as well), SAO offsets use the whole
sao_offset_abs range (cMax = (1 << (Min(BitDepth, 10) - 5)) - 1) and PCM samples the whole
sample range; at 8 bits every random draw is the one it always was.
"""
import numpy as np

from . import frontend
from . import records as R

# luma intra mode histogram of sanity.bin (Appendix B), rest spread uniformly
_MODE_W = np.full(35, 40.0)
for _m, _c in {0: 1091, 1: 811, 10: 689, 26: 723, 9: 409, 25: 428}.items():
    _MODE_W[_m] = _c
_MODE_P = _MODE_W / _MODE_W.sum()
_DENS = {2: 0.22, 3: 0.13, 4: 0.16, 5: 0.20}
_CBF_L = {2: 0.73, 3: 0.82, 4: 0.95, 5: 1.0}


def _coef_block(rng, log2, density):
    n = 1 << log2
    ys, xs = np.mgrid[0:n, 0:n]
    w = np.exp(-(xs + ys) / max(1.0, n / 3.0))
    p = np.minimum(1.0, w * density * n * n / w.sum())
    mask = rng.random((n, n)) < p
    mask[0, 0] |= not mask.any()
    mag = rng.geometric(0.6, (n, n))
    big = rng.random((n, n)) < 0.02
    mag = np.where(big, rng.integers(1, 2000, (n, n)), mag)
    sgn = rng.choice(np.array([-1, 1]), (n, n))
    return np.where(mask, mag * sgn, 0).astype(np.int16)


def uniform_tiles(wc, hc, cols, rows):
    """TileId per CTU (raster) for a uniform cols x rows tiling (6.5.1 uniform_spacing)."""
    cb = [(i * wc) // cols for i in range(cols + 1)]
    rb = [(j * hc) // rows for j in range(rows + 1)]
    tid = np.zeros(wc * hc, np.int64)
    for y in range(hc):
        for x in range(wc):
            tx = max(i for i in range(cols) if cb[i] <= x)
            ty = max(j for j in range(rows) if rb[j] <= y)
            tid[y * wc + x] = ty * cols + tx
    return tid


def make_picture(params, seed, perf=True, tiles=(1, 1), n_slices=1, sao=True, tskip_rate=0.008,
                 bypass_rate=0.0, lf_across_slices=True, deblocking=False, pcm_rate=0.0):
    """One synthetic picture (records.Picture) for ``params``.

    ``deblocking``: False (SURVEY §8(d) perf config), True (on, zero offsets) or "random"
    (per slice: on with probability 0.8, slice_beta/tc_offset_div2 uniform in -6..6).
    ``pcm_rate``: fraction of 8x8..32x32 CUs coded as PCM with pcm_loop_filter_disabled.
    """
    rng = np.random.default_rng(seed)
    p = params
    w, h = int(p["pic_width"]), int(p["pic_height"])
    ctb_log2 = int(p["ctb_log2_size"])
    wc, hc = R.ctb_grid(p)
    b = frontend.PictureBuilder(p, pcm_loop_filter_disabled=pcm_rate > 0)
    tile = uniform_tiles(wc, hc, *tiles)
    order = np.lexsort((np.arange(wc * hc), tile))          # tile-scan order
    # slices: contiguous runs in tile-scan order
    cuts = sorted(rng.choice(np.arange(1, wc * hc), n_slices - 1, replace=False)) if n_slices > 1 else []
    slice_of_ts = np.zeros(wc * hc, np.int64)
    for cpos in cuts:
        slice_of_ts[cpos:] += 1
    slice_addr_ts = np.zeros(wc * hc, np.int64)
    first = {}
    for ts, rs in enumerate(order):
        s = slice_of_ts[ts]
        first.setdefault(s, rs)
        slice_addr_ts[ts] = first[s]
    slice_lf = {s: (lf_across_slices if isinstance(lf_across_slices, bool) else bool(rng.integers(0, 2)))
                for s in first}
    if deblocking == "random":
        slice_dbk = {s: (bool(rng.random() < 0.8), int(rng.integers(-6, 7)), int(rng.integers(-6, 7))) for s in first}
    else:
        slice_dbk = {s: (bool(deblocking), 0, 0) for s in first}
    max_tb = int(p["max_tb_log2_size"])
    flat_bias = 0.0 if perf else 0.3
    bdy, bdc = int(p["bit_depth_luma"]), int(p["bit_depth_chroma"])
    offy, offc = R.qp_bd_offset(p, 0), R.qp_bd_offset(p, 1)

    def qps():
        # QpY, then qP' of each component (+ QpBdOffset): what the TB records carry
        # (above 10 bits up to QpY 51: Qp'Y then passes 63, the deblocking map's 8-bit limit)
        qy = 32 if perf else int(rng.integers(22 - offy, 52 if bdy > 10 else 38))
        qcb, qcr = frontend.chroma_qp(qy, 0, 0, offc)
        return qy + offy, qcb + offc, qcr + offc

    def mode():
        return int(rng.choice(35, p=_MODE_P)) if perf else int(rng.integers(0, 35))

    def chroma_mode(luma):
        icm = int(rng.integers(0, 5))
        if icm == 4:
            return luma
        cand = [0, 26, 10, 1][icm]
        return 34 if cand == luma else cand

    def tu_leaf(x, y, log2, blk, sub_split_ok):
        cbf_l = int(rng.random() < _CBF_L[log2])
        cbf_c = [int(rng.random() < 0.13), int(rng.random() < 0.13)]
        coef = [None, None, None]
        ts = [0, 0, 0]
        if cbf_l:
            dens = _DENS[log2] * (0.2 if rng.random() < flat_bias else 1.0)
            coef[0] = _coef_block(rng, log2, dens)
            if log2 == 2 and rng.random() < tskip_rate:
                ts[0] = 1
        clog2 = log2 - 1 if log2 > 2 else 2
        for c in (1, 2):
            if cbf_c[c - 1] and (log2 > 2 or blk == 3):
                coef[c] = _coef_block(rng, clog2, 0.15)
                if clog2 == 2 and rng.random() < tskip_rate:
                    ts[c] = 1
        return dict(x=x, y=y, log2=log2, blk=blk, cbf=[cbf_l] + cbf_c, tskip=ts, coef=coef)

    def tu_tree(x, y, log2, depth, max_depth, blk, out, forced=False):
        split = forced or log2 > max_tb
        if not split and log2 > 2 and depth < max_depth:
            split = rng.random() < {5: 0.225, 4: 0.23, 3: 0.20}.get(log2, 0.0)
        if split:
            hlf = 1 << (log2 - 1)
            for i in range(4):
                tu_tree(x + hlf * (i % 2), y + hlf * (i // 2), log2 - 1, depth + 1, max_depth, i, out)
        else:
            out.append(tu_leaf(x, y, log2, blk, False))

    def cu_tree(x, y, log2):
        if x >= w or y >= h:
            return
        n = 1 << log2
        inside = x + n <= w and y + n <= h
        if log2 > 3 and (not inside or rng.random() < {6: 0.973, 5: 0.813, 4: 0.627}[log2]):
            hlf = n >> 1
            for i in range(4):
                cu_tree(x + hlf * (i % 2), y + hlf * (i // 2), log2 - 1)
            return
        qy, qcb, qcr = qps()
        if pcm_rate > 0 and log2 <= 5 and rng.random() < pcm_rate:
            n = 1 << log2
            smp = [rng.integers(0, 1 << (bdy if c == 0 else bdc), (n >> (c > 0), n >> (c > 0))).astype(np.int16)
                   for c in range(3)]
            b.add_cu(x, y, log2, 0, [0] * 4, 0, qy, qcb, qcr, [], pcm=True, pcm_samples=smp)
            return
        nxn = log2 == 3 and rng.random() < 0.41
        modes = [mode() for _ in range(4 if nxn else 1)] + [0] * (0 if nxn else 3)
        mc = chroma_mode(modes[0])
        tus = []
        if nxn:
            tu_tree(x, y, log2, 0, 3, 0, tus, forced=True)
        else:
            tu_tree(x, y, log2, 0, 2, 0, tus)
        byp = bypass_rate > 0 and rng.random() < bypass_rate
        b.add_cu(x, y, log2, 1 if nxn else 0, modes, mc, qy, qcb, qcr, tus, bypass=byp)

    for ts, rs in enumerate(order):
        cx, cy = rs % wc, rs // wc
        cu_tree(cx << ctb_log2, cy << ctb_log2, ctb_log2)
        if sao:
            typ = [0, 0, 0]
            r = rng.random()
            typ[0] = 0 if r < 0.02 else (1 if r < 0.18 else 2)
            r = rng.random()
            typ[1] = typ[2] = 0 if r < 0.3 else (1 if r < 0.5 else 2)
            ab = rng.integers(0, 1 << (min(max(bdy, bdc), 10) - 5), (3, 4))     # 0..cMax
            sg = rng.integers(0, 2, (3, 4))
            band = rng.integers(0, 32, 3)
            eo = rng.integers(0, 4, 3)
            eo[2] = eo[1]
        else:
            typ, ab, sg, band, eo = [0, 0, 0], None, None, (0, 0, 0), (0, 0, 0)
        s = int(slice_of_ts[ts])
        on, bo, to = slice_dbk[s]
        b.add_ctu(int(rs), slice_addr=int(slice_addr_ts[ts]), tile_id=int(tile[rs]), lf_across_slices=slice_lf[s],
                  sao_type=typ, sao_abs=ab, sao_sign=sg, sao_band=band, sao_eo=eo,
                  deblocking=on, beta_offset_div2=bo, tc_offset_div2=to)
    return b.finish(meta={"seed": seed, "perf": perf, "tiles": tiles, "slices": n_slices, "deblocking": deblocking})


def c2_picture(seed=267):
    """Config 2: a single 64x64 CTB holding one 32x32 intra CU (DC), one 32x32 TU with a
    fixed + random coefficient pattern, picture 32x32 (one CTB, CtbSizeY 32)."""
    params = R.make_params(pic_width=32, pic_height=32, ctb_log2_size=5, sample_adaptive_offset=0)
    rng = np.random.default_rng(seed)
    co = np.zeros((32, 32), np.int16)
    co[0, 0] = 64
    co[0, 1], co[1, 0], co[2, 3] = -12, 9, 3
    co[:8, :8] += _coef_block(rng, 3, 0.3)
    tu = dict(x=0, y=0, log2=5, blk=0, cbf=[1, 0, 0], tskip=[0, 0, 0], coef=[co, None, None])
    b = frontend.PictureBuilder(params)
    b.add_cu(0, 0, 5, 0, [1, 0, 0, 0], 1, 32, 31, 31, [tu])
    b.add_ctu(0)
    return params, b.finish(meta={"config": 2})
