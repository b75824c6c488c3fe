"""Tile-sharded decoding with in-loop filters across tile edges (config C5).

With tiles, intra prediction never crosses a tile edge (6.4.1; decoder/image.py:65-71),
so every tile reconstructs on its own (``p265_amd/tiles.py``).  When
loop_filter_across_tiles_enabled_flag is 1, deblocking (8.7.2) and SAO (8.7.3) DO cross
the edge: the filter of a tile's border CTBs needs, from each neighbouring tile,

  * the reconstructed samples within 4 samples of the edge (luma and chroma: the loop
    filter window of loopfilter.h reaches exactly 4 samples past its CTB),
  * the CTU records of the CTBs along the edge (slice / tile ids, loop-filter flags,
    deblocking offsets) and their luma TB records (transform edges and QpY for the
    deblocking map),
  * the PCM / bypass "no filter" bytes of those CTBs' 8x8 blocks.

That is the halo.  Each tile's owner then runs the in-loop filters alone on an
*extended tile*: the tile plus a ring of one CTB (clipped to the picture), whose ring
holds only the halo (the rest of the ring is never read by the tile's own windows), as
a picture with ``recon_input`` (P265R_PIC_RECON_INPUT: the library skips residual and
intra and runs deblocking + SAO), and keeps the tile's part of the output.

The exchange is a real point-to-point step: ``exchange`` sends each neighbour its
halo with ncclSend / ncclRecv (RCCL over xGMI, p265_amd/rccl.py; over the socket control
plane of p265_amd/comm.py in CPU-only runs).  Everything here is host-side plumbing; the filtering runs in libp265r.so.
"""
import io

import numpy as np

from . import records as R

HALO = 4          # samples of a neighbouring tile the loop filter reads (luma and chroma)


class TileGrid:
    """Tile columns / rows in CTBs (6.5.1), for one picture size."""

    def __init__(self, params, cols, rows):
        self.params = params
        self.ctb_log2 = int(params["ctb_log2_size"])
        self.ctb = 1 << self.ctb_log2
        self.w, self.h = int(params["pic_width"]), int(params["pic_height"])
        self.wc, self.hc = R.ctb_grid(params)
        self.cols, self.rows = list(cols), list(rows)
        assert self.cols[0] == 0 and self.cols[-1] == self.wc and self.rows[0] == 0 and self.rows[-1] == self.hc

    @classmethod
    def from_picture(cls, params, pic):
        from .tiles import tile_grid
        cols, rows = tile_grid(params, pic)
        return cls(params, cols, rows)

    @property
    def n_tiles(self):
        return (len(self.cols) - 1) * (len(self.rows) - 1)

    def rect(self, t):
        """CTB rect [c0, c1) x [r0, r1) of tile t (tile-scan = raster order of tiles)."""
        nx = len(self.cols) - 1
        tx, ty = t % nx, t // nx
        return self.cols[tx], self.cols[tx + 1], self.rows[ty], self.rows[ty + 1]

    def ext_rect(self, t):
        c0, c1, r0, r1 = self.rect(t)
        return max(c0 - 1, 0), min(c1 + 1, self.wc), max(r0 - 1, 0), min(r1 + 1, self.hc)

    def luma_rect(self, rect):
        c0, c1, r0, r1 = rect
        return c0 * self.ctb, min(c1 * self.ctb, self.w), r0 * self.ctb, min(r1 * self.ctb, self.h)

    def neighbours(self, t):
        """Tiles whose CTBs lie in t's extended rect (edge and corner neighbours)."""
        e = self.ext_rect(t)
        out = []
        for n in range(self.n_tiles):
            if n == t:
                continue
            c0, c1, r0, r1 = self.rect(n)
            if c0 < e[1] and e[0] < c1 and r0 < e[3] and e[2] < r1:
                out.append(n)
        return out


def _isect(a, b):
    return max(a[0], b[0]), min(a[1], b[1]), max(a[2], b[2]), min(a[3], b[3])


class TileData:
    """What the owner of tile t has: the records of its own CTBs (full-picture coordinates,
    as its front-end parsed them) and, after reconstruction, its reconstructed samples."""

    def __init__(self, grid, pic, t):
        self.grid, self.t = grid, t
        c0, c1, r0, r1 = grid.rect(t)
        self.ctus = {}
        self.tbs = {}
        for y in range(r0, r1):
            for x in range(c0, c1):
                rs = y * grid.wc + x
                c = pic.ctus[rs]
                self.ctus[rs] = c.copy()
                b, n = int(c["tb_begin"]), int(c["tb_count"])
                self.tbs[rs] = pic.tbs[b:b + n].copy()
        self.nofilter = pic.nofilter
        self.recon = None          # [Y, Cb, Cr] of the tile rect, set after reconstruction

    def halo_for(self, t_dst):
        """Payload this tile sends to tile t_dst (bytes; numpy .npz, no pickles)."""
        g = self.grid
        ring = _isect(g.ext_rect(t_dst), g.rect(self.t))
        rs_list = [y * g.wc + x for y in range(ring[2], ring[3]) for x in range(ring[0], ring[1])]
        ctus = np.array([self.ctus[rs] for rs in rs_list], R.CTU_DTYPE)
        luma = [self.tbs[rs][self.tbs[rs]["c_idx"] == 0] for rs in rs_list]
        counts = np.array([len(t) for t in luma], np.int64)
        tbs = np.concatenate(luma) if luma else np.zeros(0, R.TB_DTYPE)
        # samples: the part of this tile within HALO samples of t_dst's rect
        lx0, lx1, ly0, ly1 = g.luma_rect(g.rect(t_dst))
        mx0, mx1, my0, my1 = g.luma_rect(g.rect(self.t))
        arrays = {"rs": np.array(rs_list, np.int64), "ctus": ctus, "tbs": tbs, "counts": counts}
        for c in range(3):
            s = 0 if c == 0 else 1
            bx0, bx1 = max((lx0 >> s) - HALO, mx0 >> s), min((lx1 >> s) + HALO, mx1 >> s)
            by0, by1 = max((ly0 >> s) - HALO, my0 >> s), min((ly1 >> s) + HALO, my1 >> s)
            box = np.array([bx0, bx1, by0, by1], np.int64)
            arrays["box%d" % c] = box
            if bx1 > bx0 and by1 > by0:
                arrays["smp%d" % c] = self.recon[c][by0 - (my0 >> s):by1 - (my0 >> s), bx0 - (mx0 >> s):bx1 - (mx0 >> s)]
            else:
                arrays["smp%d" % c] = np.zeros((0, 0), np.uint8)
        if self.nofilter is not None:
            nfw = (g.w + 7) // 8
            blocks = []
            for rs in rs_list:
                cx, cy = (rs % g.wc) * g.ctb, (rs // g.wc) * g.ctb
                for by in range(cy // 8, min(cy + g.ctb, g.h) // 8):
                    for bx in range(cx // 8, min(cx + g.ctb, g.w) // 8):
                        blocks.append((by * nfw + bx, self.nofilter[by * nfw + bx]))
            arrays["nf"] = np.array(blocks, np.int64).reshape(-1, 2)
        buf = io.BytesIO()
        np.savez(buf, **arrays)
        return buf.getvalue()


def ext_picture(params, grid, own, halos):
    """(ext_params, ext Picture with recon_input, (x0, y0) luma origin, inner luma rect) for
    tile own.t from its own TileData and the halo payloads received from its neighbours."""
    g = grid
    e = g.ext_rect(own.t)
    ex0, ex1, ey0, ey1 = g.luma_rect(e)
    ew, eh = ex1 - ex0, ey1 - ey0
    kw = dict(R.params_dict(params))
    kw.update(pic_width=ew, pic_height=eh)
    ep = R.make_params(**kw)
    ewc, ehc = e[1] - e[0], e[3] - e[2]
    ctus = np.zeros(ewc * ehc, R.CTU_DTYPE)
    tbs_of = {}
    planes = [np.zeros((eh, ew), np.uint8), np.zeros((eh // 2, ew // 2), np.uint8), np.zeros((eh // 2, ew // 2), np.uint8)]
    nfw_full = (g.w + 7) // 8
    nfw, nfh = (ew + 7) // 8, (eh + 7) // 8
    nf = np.zeros(nfw * nfh, np.uint8)
    any_nf = own.nofilter is not None

    def put_ctu(rs, rec, tb):
        x, y = rs % g.wc - e[0], rs // g.wc - e[2]
        ctus[y * ewc + x] = rec
        t = tb.copy()
        sub = (t["c_idx"] > 0).astype(np.int64)
        t["x"] = t["x"].astype(np.int64) - (ex0 >> sub)
        t["y"] = t["y"].astype(np.int64) - (ey0 >> sub)
        t["flags"] = 0                              # no coefficients: the map needs position, size, QpY
        t["coef_off"] = 0
        tbs_of[y * ewc + x] = t[t["c_idx"] == 0]

    def put_nf(idx_val):
        for idx, v in idx_val:
            by, bx = int(idx) // nfw_full, int(idx) % nfw_full
            nf[(by - ey0 // 8) * nfw + (bx - ex0 // 8)] = v

    for rs, rec in own.ctus.items():
        put_ctu(rs, rec, own.tbs[rs])
    mx0, mx1, my0, my1 = g.luma_rect(g.rect(own.t))
    for c in range(3):
        s = 0 if c == 0 else 1
        planes[c][(my0 - ey0) >> s:(my1 - ey0) >> s, (mx0 - ex0) >> s:(mx1 - ex0) >> s] = own.recon[c]
    if any_nf:
        for rs in own.ctus:
            cx, cy = (rs % g.wc) * g.ctb, (rs // g.wc) * g.ctb
            for by in range(cy // 8, min(cy + g.ctb, g.h) // 8):
                for bx in range(cx // 8, min(cx + g.ctb, g.w) // 8):
                    nf[(by - ey0 // 8) * nfw + (bx - ex0 // 8)] = own.nofilter[by * nfw_full + bx]
    for payload in halos:
        z = np.load(io.BytesIO(payload), allow_pickle=False)
        tbs = z["tbs"]
        off = 0
        for rs, rec, n in zip(z["rs"], z["ctus"], z["counts"]):
            put_ctu(int(rs), rec, tbs[off:off + int(n)])
            off += int(n)
        for c in range(3):
            s = 0 if c == 0 else 1
            bx0, bx1, by0, by1 = (int(v) for v in z["box%d" % c])
            if bx1 > bx0 and by1 > by0:
                planes[c][by0 - (ey0 >> s):by1 - (ey0 >> s), bx0 - (ex0 >> s):bx1 - (ex0 >> s)] = z["smp%d" % c]
        if "nf" in z.files:
            any_nf = True
            put_nf(z["nf"])
    # records in raster order of the extended picture
    begin = 0
    parts = []
    for i in range(ewc * ehc):
        t = tbs_of.get(i, np.zeros(0, R.TB_DTYPE))
        ctus[i]["tb_begin"] = begin
        ctus[i]["tb_count"] = len(t)
        begin += len(t)
        parts.append(t)
    tb_all = np.concatenate(parts) if parts else np.zeros(0, R.TB_DTYPE)
    pic = R.Picture(ctus=ctus, tbs=tb_all, coef=np.zeros(0, np.int16), nofilter=nf if any_nf else None,
                    meta={"tile": own.t, "ext_origin": (ex0, ey0)}, recon_input=planes)
    R.validate(ep, pic)
    return ep, pic, (ex0, ey0), (mx0, mx1, my0, my1)


def crop_inner(out_planes, origin, inner):
    """The tile's own part of the extended picture's output planes."""
    ex0, ey0 = origin
    mx0, mx1, my0, my1 = inner
    res = []
    for c in range(3):
        s = 0 if c == 0 else 1
        res.append(np.ascontiguousarray(out_planes[c][(my0 - ey0) >> s:(my1 - ey0) >> s,
                                                      (mx0 - ex0) >> s:(mx1 - ex0) >> s]))
    return res


def recon_only(params, pic):
    """Records for reconstruction only (no in-loop filter flags): the tile's first pass."""
    ctus = pic.ctus.copy()
    ctus["flags"] &= np.uint8(0xff & ~R.CTU_DEBLOCK)
    ctus["sao_type"] = 0
    kw = dict(R.params_dict(params))
    kw.update(sample_adaptive_offset=0)
    return R.make_params(**kw), R.Picture(ctus=ctus, tbs=pic.tbs, coef=pic.coef, nofilter=pic.nofilter,
                                          meta=dict(pic.meta))


# ---------------------------------------------------------------------------------------
# point-to-point exchange (RCCL send / recv, p265_amd/dist.py)
# ---------------------------------------------------------------------------------------

def exchange(sends, recvs):
    """sends: [(dst_rank, tag, bytes)], recvs: [(src_rank, tag)] -> {tag: bytes}, over the
    process group of p265_amd.dist (ncclSend / ncclRecv on the GPU box; the socket control
    plane on CPU).  Every rank calls it, also with nothing to send."""
    from . import dist
    return dist.exchange(sends, recvs)
