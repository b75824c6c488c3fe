"""Tile sub-pictures for tile-sharded decoding (config C5).

With tiles, intra prediction never crosses a tile edge (6.4.1: a neighbour in another
tile is unavailable; decoder/image.py:65-71), and when
loop_filter_across_tiles_enabled_flag is 0 neither does SAO (8.7.3.2).  A tile is then
exactly a picture of its own size: ``split`` re-bases a picture's records onto one
tile, ``stitch`` puts decoded tiles back.  With the flag at 1, deblocking and SAO of a
tile's border need the neighbour tiles' samples: ``split(recon_only=True)`` gives the
reconstruction pass and p265_amd/halo.py the halo exchange + filtering pass.
"""
import numpy as np

from . import records as R


def tile_grid(params, pic):
    """Column/row boundaries (in CTBs) of the tiles, recovered from the CTU tile ids."""
    wc, hc = R.ctb_grid(params)
    tid = pic.ctus["tile_id"].astype(np.int64).reshape(hc, wc)
    cols = [0] + [x for x in range(1, wc) if tid[0, x] != tid[0, x - 1]] + [wc]
    rows = [0] + [y for y in range(1, hc) if tid[y, 0] != tid[y - 1, 0]] + [hc]
    return cols, rows


def split(params, pic, recon_only=False):
    """[(tile_params, tile_picture, (x0, y0) luma origin)] for every tile, in tile-scan order.

    With loop_filter_across_tiles_enabled_flag = 1 a tile's in-loop filters need its
    neighbours' samples: split then only serves the reconstruction pass (``recon_only``:
    in-loop filter flags cleared) and p265_amd/halo.py does the filtering."""
    if int(params["loop_filter_across_tiles"]) and not recon_only:
        raise NotImplementedError("loop_filter_across_tiles_enabled_flag=1: split(recon_only=True) + halo.py")
    if recon_only:
        from .halo import recon_only as _ro
        params, pic = _ro(params, pic)
    ctb_log2 = int(params["ctb_log2_size"])
    ctb = 1 << ctb_log2
    w, h = int(params["pic_width"]), int(params["pic_height"])
    wc, _ = R.ctb_grid(params)
    cols, rows = tile_grid(params, pic)
    out = []
    for ty in range(len(rows) - 1):
        for tx in range(len(cols) - 1):
            c0, c1, r0, r1 = cols[tx], cols[tx + 1], rows[ty], rows[ty + 1]
            x0, y0 = c0 * ctb, r0 * ctb
            tw, th = min(c1 * ctb, w) - x0, min(r1 * ctb, h) - y0
            kw = dict(R.params_dict(params))
            kw.update(pic_width=tw, pic_height=th)
            tp = R.make_params(**kw)
            ctus = np.zeros((r1 - r0) * (c1 - c0), R.CTU_DTYPE)
            tbs_parts, coef_parts, ncoef, ntb = [], [], 0, 0
            for yy in range(r0, r1):
                for xx in range(c0, c1):
                    src = pic.ctus[yy * wc + xx]
                    dst_i = (yy - r0) * (c1 - c0) + (xx - c0)
                    ctus[dst_i] = src
                    b, n = int(src["tb_begin"]), int(src["tb_count"])
                    t = pic.tbs[b:b + n].copy()
                    sub = (t["c_idx"] > 0).astype(np.int64)
                    t["x"] = t["x"].astype(np.int64) - (x0 >> sub)
                    t["y"] = t["y"].astype(np.int64) - (y0 >> sub)
                    coded = (t["flags"] & (R.TB_CBF | R.TB_PCM)) != 0
                    for i in np.nonzero(coded)[0]:
                        nn = 1 << (2 * int(t["log2_size"][i]))
                        o = int(t["coef_off"][i])
                        coef_parts.append(pic.coef[o:o + nn])
                        t["coef_off"][i] = ncoef
                        ncoef += nn
                    ctus["tb_begin"][dst_i] = ntb
                    ntb += n
                    tbs_parts.append(t)
            # slice addresses are only compared for equality: keep them as they are
            nf = None
            if pic.nofilter is not None:
                full = pic.nofilter.reshape((h + 7) // 8, (w + 7) // 8)
                nf = np.ascontiguousarray(full[y0 // 8:(y0 + th + 7) // 8, x0 // 8:(x0 + tw + 7) // 8]).reshape(-1)
            tpic = R.Picture(ctus=ctus, tbs=np.concatenate(tbs_parts) if tbs_parts else np.zeros(0, R.TB_DTYPE),
                             coef=np.concatenate(coef_parts).astype(np.int16) if coef_parts else np.zeros(0, np.int16),
                             nofilter=nf, meta={"tile": (tx, ty), "origin": (x0, y0)}, size=(tw, th))
            R.validate(tp, tpic)
            out.append((tp, tpic, (x0, y0)))
    return out


def ragged_params(parts):
    """One context for all tile units of ``split`` (uneven tiles included): the parameter set of
    the largest tile; every tile picture carries its own size (Picture.size), so the units run
    as ONE ragged batch -- one launch per phase (p265r_picture.pic_width / pic_height)."""
    tp0 = parts[0][0]
    kw = dict(R.params_dict(tp0))
    kw.update(pic_width=max(int(tp["pic_width"]) for tp, _, _ in parts),
              pic_height=max(int(tp["pic_height"]) for tp, _, _ in parts))
    return R.make_params(**kw)


def stitch(params, tiles, planes_per_tile):
    """Assemble decoded tile planes ([Y, Cb, Cr] per tile) into full-picture planes."""
    w, h = int(params["pic_width"]), int(params["pic_height"])
    out = [np.zeros((h, w), np.uint8), np.zeros((h // 2, w // 2), np.uint8), np.zeros((h // 2, w // 2), np.uint8)]
    for (tp, _, (x0, y0)), planes in zip(tiles, planes_per_tile):
        for c in range(3):
            s = 0 if c == 0 else 1
            ph, pw = planes[c].shape
            out[c][(y0 >> s):(y0 >> s) + ph, (x0 >> s):(x0 >> s) + pw] = planes[c]
    return out
