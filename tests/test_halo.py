"""Tile halo exchange (C5 with loop_filter_across_tiles_enabled_flag = 1), CPU side.

Each tile is reconstructed alone, receives from its neighbours the samples within 4 of
its edges plus the edge CTUs' records (p265_amd/halo.py), and runs the in-loop filters
on its extended tile; the stitched result must equal whole-picture decoding.  Here the
filters are the oracle's (the GPU path is tests/test_gpu_parity.py::test_tile_halo_*),
and the exchange runs between two rank processes (p265_amd.dist.exchange over the socket
control plane; RCCL send / recv on the GPU box).
"""
import os

import numpy as np
import pytest

from oracle import recon_oracle as O
from p265_amd import halo, synth, tiles
from p265_amd import records as R


def _case(seed=31, tiles_xy=(2, 2), w=264, h=200, ctb_log2=5, deblocking="random"):
    params = R.make_params(pic_width=w, pic_height=h, ctb_log2_size=ctb_log2, loop_filter_across_tiles=1,
                           pps_cb_qp_offset=2, pps_cr_qp_offset=-1)
    pic = synth.make_picture(params, seed, perf=False, tiles=tiles_xy, n_slices=3, lf_across_slices=None,
                             deblocking=deblocking, bypass_rate=0.04, pcm_rate=0.02)
    return params, pic


def _tile_recons(params, pic):
    out = []
    for tp, tpic, _ in tiles.split(params, pic, recon_only=True):
        out.append([p.astype(np.uint8) for p in O.reconstruct_picture(R.params_dict(tp), tpic.as_oracle_dict())])
    return out


def _filter_ext(ep, epic):
    pd = R.params_dict(ep)
    d = epic.as_oracle_dict()
    rec = [np.asarray(p, np.int64) for p in epic.recon_input]
    return O.sao_picture(pd, d, O.deblock_picture(pd, d, rec))


def _check_tiles(params, pic, outs_per_tile, grid):
    _, ref = O.decode_picture(R.params_dict(params), pic.as_oracle_dict())
    for t, planes in outs_per_tile.items():
        x0, x1, y0, y1 = grid.luma_rect(grid.rect(t))
        for c in range(3):
            s = 0 if c == 0 else 1
            np.testing.assert_array_equal(planes[c], ref[c][y0 >> s:y1 >> s, x0 >> s:x1 >> s],
                                          err_msg="tile %d c%d" % (t, c))


@pytest.mark.parametrize("tiles_xy,ctb_log2,w,h", [((2, 2), 5, 264, 200), ((3, 2), 4, 200, 136), ((2, 1), 6, 264, 136)])
def test_halo_filtering_equals_whole_picture(tiles_xy, ctb_log2, w, h):
    params, pic = _case(tiles_xy=tiles_xy, ctb_log2=ctb_log2, w=w, h=h)
    grid = halo.TileGrid.from_picture(params, pic)
    recons = _tile_recons(params, pic)
    datas = []
    for t in range(grid.n_tiles):
        d = halo.TileData(grid, pic, t)
        d.recon = recons[t]
        datas.append(d)
    outs = {}
    for t in range(grid.n_tiles):
        payloads = [datas[n].halo_for(t) for n in grid.neighbours(t)]
        ep, epic, origin, inner = halo.ext_picture(params, grid, datas[t], payloads)
        outs[t] = halo.crop_inner(_filter_ext(ep, epic), origin, inner)
    _check_tiles(params, pic, outs, grid)


def test_without_halo_the_tile_border_differs():
    """Control: filtering a tile without its neighbours' samples gives a different border."""
    params, pic = _case(deblocking=True)
    grid = halo.TileGrid.from_picture(params, pic)
    recons = _tile_recons(params, pic)
    d = halo.TileData(grid, pic, 0)
    d.recon = recons[0]
    ep, epic, origin, inner = halo.ext_picture(params, grid, d, [])
    got = halo.crop_inner(_filter_ext(ep, epic), origin, inner)
    _, ref = O.decode_picture(R.params_dict(params), pic.as_oracle_dict())
    x0, x1, y0, y1 = grid.luma_rect(grid.rect(0))
    assert (got[0] != ref[0][y0:y1, x0:x1]).any()


def _rank_main(rank, world):
    params, pic = _case(seed=77)
    grid = halo.TileGrid.from_picture(params, pic)
    owner = {t: t % world for t in range(grid.n_tiles)}
    recons = _tile_recons(params, pic)            # (every rank could; each keeps only its own)
    mine = {}
    for t in range(grid.n_tiles):
        if owner[t] == rank:
            mine[t] = halo.TileData(grid, pic, t)
            mine[t].recon = recons[t]
    sends, recvs = [], []
    for t, d in mine.items():
        for n in grid.neighbours(t):
            if owner[n] != rank:
                recvs.append((owner[n], (n, t)))
        for dst_t in range(grid.n_tiles):
            if t in grid.neighbours(dst_t) and owner[dst_t] != rank:
                sends.append((owner[dst_t], (t, dst_t), d.halo_for(dst_t)))
    tag_key = lambda k: k[0] * 100 + k[1]
    got = halo.exchange([(d, tag_key(k), b) for d, k, b in sends], [(s, tag_key(k)) for s, k in recvs])
    outs = {}
    for t, d in mine.items():
        payloads = []
        for n in grid.neighbours(t):
            payloads.append(mine[n].halo_for(t) if owner[n] == rank else got[tag_key((n, t))])
        ep, epic, origin, inner = halo.ext_picture(params, grid, d, payloads)
        outs[t] = halo.crop_inner(_filter_ext(ep, epic), origin, inner)
    _check_tiles(params, pic, outs, grid)
    return "ok"


def test_halo_exchange_two_ranks():
    from ranks import run_ranks
    assert run_ranks(_rank_main, 2) == {0: "ok", 1: "ok"}
