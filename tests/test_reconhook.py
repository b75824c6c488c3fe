"""The reference-side drop-in adapter (p265_amd.frontend.ReconHook) on duck-typed stand-ins of
the reference's Cu / Tu / Ctu / slice-header objects (CPU only).

tests/golden/gen_sanity_fixture.py drives the same hook with the LIVE reference objects on
sanity.bin and asserts the records equal the committed capture ("reconhook_identical" in
sanity_frontend.json).  Here the cases sanity.bin lacks: NxN CUs with per-PB modes, the chroma
4x4 pair a luma 4x4 quad keeps on its blkIdx-3 leaf (tu.py:127-135), transquant bypass, PCM
(samples under their syntax names, PcmBitDepth < BitDepth, pcm_loop_filter_disabled) and the
read-back surface get_reconstructed_sample (cu.py:617-632, luma coordinates for every
component).
"""
import dataclasses
import json
import os
from types import SimpleNamespace as NS

import numpy as np

from oracle import c_oracle
from p265_amd import frontend, recon
from p265_amd import records as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _md(entries):
    """x-major md_dict {x: {y: mode}} as cu.py:184-263 keeps IntraPredModeY."""
    d = {}
    for (x, y), m in entries.items():
        d.setdefault(x, {})[y] = m
    return d


class _Tree:
    def __init__(self, leaves):
        self._leaves = leaves

    def get_leaves(self):
        return self._leaves


def _leaf(x, y, log2, idx, cbf, coef_yx, tskip=None):
    """A reference TU leaf: trans_coeff_level x-major (tu.py:87-90); transform_skip_flag only
    exists when some cbf is set (tu.py:104)."""
    leaf = NS(x=x, y=y, log2size=log2, idx=idx, cbf_luma=cbf[0], cbf_cb=cbf[1], cbf_cr=cbf[2],
              trans_coeff_level=[np.asarray(c).T if c is not None else np.zeros((4, 4), int) for c in coef_yx])
    if any(cbf):
        leaf.transform_skip_flag = np.array(tskip or [0, 0, 0], bool)
    return leaf


def _cu(x, y, log2, part_mode, modes_xy, mode_c, leaves, qp=30, bypass=0):
    return NS(x=x, y=y, size=1 << log2, log2size=log2, part_mode=part_mode, intra_pred_mode_y=_md(modes_xy),
              intra_pred_mode_c=mode_c, qp_y=qp, qp_cb=qp - 1, qp_cr=qp - 2, cu_transquant_bypass_flag=bypass,
              pcm_flag=0, tu=_Tree(leaves))


def _blk(rng, n):
    b = np.zeros((n, n), np.int16)
    b[0, 0] = rng.integers(-40, 40)
    b[rng.integers(0, n), rng.integers(0, n)] = rng.integers(-9, 9)
    return b


def _build(rng, hook_side):
    """The same 64x64 picture built through ReconHook (hook_side) or PictureBuilder.add_cu."""
    params = R.make_params(pic_width=64, pic_height=64, ctb_log2_size=6)
    hook = frontend.ReconHook(params, pcm_bit_depth_luma=6, pcm_bit_depth_chroma=5, pcm_loop_filter_disabled=True)
    b = frontend.PictureBuilder(params, pcm_loop_filter_disabled=True)
    # CU 0: 8x8 NxN at (0, 0), four 4x4 luma TBs with their own modes; chroma pair on blkIdx 3
    ys = [_blk(rng, 4) for _ in range(4)]
    cb, cr = _blk(rng, 4), _blk(rng, 4)
    modes = {(0, 0): 2, (4, 0): 18, (0, 4): 26, (4, 4): 34}
    leaves, tus = [], []
    for i, (lx, ly) in enumerate([(0, 0), (4, 0), (0, 4), (4, 4)]):
        cbf = [1, 1, 1] if i == 3 else [1, 1, 1]
        co = [ys[i], cb if i == 3 else None, cr if i == 3 else None]
        leaves.append(_leaf(lx, ly, 2, i, cbf, co, tskip=[1 if i == 1 else 0, 0, 0]))
        tus.append(dict(x=lx, y=ly, log2=2, blk=i, cbf=cbf, tskip=[1 if i == 1 else 0, 0, 0], coef=co))
    cu0 = _cu(0, 0, 3, 1, modes, 4, leaves)
    # CU 1: 8x8 2Nx2N at (8, 0), cu_transquant_bypass, one 8x8 TU with Cb only
    y8, cb4 = _blk(rng, 8), _blk(rng, 4)
    cu1 = _cu(8, 0, 3, 0, {(8, 0): 10}, 0, [_leaf(8, 0, 3, 0, [1, 1, 0], [y8, cb4, None])], bypass=1)
    # CU 2: 16x16 PCM at (16, 0): 6-bit luma / 5-bit chroma samples, raster (7.3.8.7)
    pl = rng.integers(0, 64, 256)
    pc = rng.integers(0, 32, 128)
    cu2 = NS(x=16, y=0, size=16, log2size=4, part_mode=0, pcm_flag=1, pcm_sample_luma=pl.tolist(),
             pcm_sample_chroma=pc.tolist(), qp_y=30, qp_cb=29, qp_cr=28, cu_transquant_bypass_flag=0, tu=None)
    # the rest of the CTB: 16x16 / 32x32 CUs with one TU each
    rest = [(32, 0, 5), (0, 32, 5), (32, 32, 5), (0, 16, 4), (16, 16, 4), (0, 8, 3), (8, 8, 3)]
    cus = [cu0, cu1, cu2]
    for k, (x, y, lg) in enumerate(rest):
        yb, cbb = _blk(rng, 1 << lg), _blk(rng, 1 << (lg - 1))
        cus.append(_cu(x, y, lg, 0, {(x, y): (7 * k + 1) % 35}, 4, [_leaf(x, y, lg, 0, [1, k % 2, 0], [yb, cbb, None])]))
    # Cr shares Cb's SaoTypeIdx (7.4.9.3.2), with its own band position
    sao = NS(sao_type_idx=[2, 1, 1], sao_offset_abs=[[1, 2, 3, 4]] * 3, sao_offset_sign=[[1, 0, 1, 0]] * 3,
             sao_band_position=[0, 7, 3], sao_eo_class=[1, 0, 0])
    ctu = NS(addr_rs=0, slice_addr=0, sao=sao)
    sh = NS(slice_sao_luma_flag=1, slice_sao_chroma_flag=1)
    pps = NS(pps_deblocking_filter_disabled_flag=0, pps_loop_filter_across_slices_enabled_flag=1,
             pps_beta_offset_div2=2, pps_tc_offset_div2=-1)
    if hook_side:
        for c in cus:
            hook.on_decode_leaf(c)
        hook.on_ctu_parsed(ctu, sh, pps)
        return params, hook.on_end_of_picture()
    b.add_cu(0, 0, 3, 1, [2, 18, 26, 34], 4, 30, 29, 28, tus)
    b.add_cu(8, 0, 3, 0, [10, 0, 0, 0], 0, 30, 29, 28,
             [dict(x=8, y=0, log2=3, blk=0, cbf=[1, 1, 0], tskip=[0, 0, 0], coef=[y8, cb4, None])], bypass=True)
    b.add_cu(16, 0, 4, 0, [0] * 4, 0, 30, 29, 28, [], pcm=True,
             pcm_samples=[(pl.reshape(16, 16) << 2).astype(np.int16), (pc[:64].reshape(8, 8) << 3).astype(np.int16),
                          (pc[64:].reshape(8, 8) << 3).astype(np.int16)])
    for k, (x, y, lg) in enumerate(rest):
        c = cus[3 + k]
        leaf = c.tu.get_leaves()[0]
        b.add_cu(x, y, lg, 0, [(7 * k + 1) % 35, 0, 0, 0], 4, 30, 29, 28,
                 [dict(x=x, y=y, log2=lg, blk=0, cbf=[1, k % 2, 0], tskip=[0, 0, 0],
                       coef=[leaf.trans_coeff_level[0].T, leaf.trans_coeff_level[1].T, None])])
    b.add_ctu(0, sao_type=(2, 1, 1), sao_abs=[[1, 2, 3, 4]] * 3, sao_sign=[[1, 0, 1, 0]] * 3, sao_band=(0, 7, 3),
              sao_eo=(1, 0, 0), deblocking=True, beta_offset_div2=2, tc_offset_div2=-1)
    return params, b.finish()


def test_hook_records_equal_the_builder():
    params, hooked = _build(np.random.default_rng(5), True)
    _, built = _build(np.random.default_rng(5), False)
    for name in ("ctus", "tbs", "coef", "nofilter"):
        np.testing.assert_array_equal(getattr(hooked, name), getattr(built, name), err_msg=name)
    tb = hooked.tbs
    # NxN: four luma 4x4 TBs with the per-PB modes, then ONE Cb + Cr 4x4 pair at chroma (0, 0)
    assert list(tb["pred_mode"][:4]) == [2, 18, 26, 34] and list(tb["c_idx"][:6]) == [0, 0, 0, 0, 1, 2]
    assert (tb["x"][4], tb["y"][4], tb["log2_size"][4]) == (0, 0, 2)
    assert tb["flags"][1] & R.TB_TSKIP
    # bypass CU: TB flags + no-filter map; PCM CU: samples shifted to BitDepth, no-filter map
    assert all(tb["flags"][6:8] & R.TB_BYPASS)
    pcm = tb[(tb["flags"] & R.TB_PCM) != 0]
    assert len(pcm) == 3 and list(pcm["c_idx"]) == [0, 1, 2]
    assert int(hooked.coef[int(pcm["coef_off"][0])]) % 4 == 0
    nf = hooked.nofilter.reshape(8, 8)
    assert nf[0, 1] == 1 and nf[0, 2] == nf[1, 3] == 1 and nf[0, 0] == 0
    R.validate(params, hooked)


def test_decoded_picture_read_back_uses_luma_coordinates():
    params, pic = _build(np.random.default_rng(6), True)
    (rec, out), = c_oracle.decode(params, [pic])
    dp = recon.DecodedPicture([np.asarray(p, np.uint8) for p in out], [np.asarray(p, np.uint8) for p in rec])
    for (x, y) in [(0, 0), (5, 3), (17, 9), (63, 63), (40, 22)]:
        assert dp.get_reconstructed_sample(x, y, 0) == rec[0][y, x]
        assert dp.get_reconstructed_sample(x, y, 1) == rec[1][y >> 1, x >> 1]
        assert dp.get_reconstructed_sample(x, y, 2) == rec[2][y >> 1, x >> 1]
        assert dp.get_output_sample(x, y, 2) == out[2][y >> 1, x >> 1]
    # a PCM CU reconstructs to its samples << (BitDepth - PcmBitDepth) (8.4.4.1)
    assert dp.get_reconstructed_sample(16, 0, 0) % 4 == 0 and dp.get_reconstructed_sample(16, 0, 1) % 8 == 0


def test_live_reference_hook_was_verified():
    """gen_sanity_fixture.py ran the hook on the live reference objects: identical records."""
    meta = json.load(open(os.path.join(GOLDEN, "sanity_frontend.json")))
    assert meta["reconhook_identical"] is True
    _, pics = frontend.pictures_from_frontend_npz(os.path.join(GOLDEN, "sanity_frontend.npz"))
    assert meta["reconhook_tb_records"] == sum(len(p.tbs) for p in pics)


def test_hook_takes_tile_ids_from_the_pps():
    """The reference's Ctu has no tile id (ctu.py sets addr_rs / addr_ts / slice_addr only): TileId
    is pps.tile_id_rs (pps.py:215-227, read by image.py:65).  A 2x2-tiled picture through the hook
    must carry those ids, or availability and the loop filters would cross the tile edges."""
    params = R.make_params(pic_width=128, pic_height=128, ctb_log2_size=6, loop_filter_across_tiles=0)
    hook = frontend.ReconHook(params)
    sao = NS(sao_type_idx=[0, 0, 0], sao_offset_abs=[[0] * 4] * 3, sao_offset_sign=[[0] * 4] * 3,
             sao_band_position=[0, 0, 0], sao_eo_class=[0, 0, 0])
    sh = NS(slice_sao_luma_flag=0, slice_sao_chroma_flag=0)
    pps = NS(pps_deblocking_filter_disabled_flag=0, pps_loop_filter_across_slices_enabled_flag=1,
             pps_beta_offset_div2=0, pps_tc_offset_div2=0, tile_id_rs=[0, 1, 2, 3])
    rng = np.random.default_rng(11)
    for rs in range(4):
        cx, cy = (rs % 2) * 64, (rs // 2) * 64
        for k in range(4):
            x, y = cx + (k % 2) * 32, cy + (k // 2) * 32
            hook.on_decode_leaf(_cu(x, y, 5, 0, {(x, y): int(rng.integers(0, 35))}, 4,
                                    [_leaf(x, y, 5, 0, [1, 0, 0], [_blk(rng, 32), None, None])]))
        hook.on_ctu_parsed(NS(addr_rs=rs, slice_addr=0, sao=sao), sh, pps)
    pic = hook.on_end_of_picture()
    assert list(pic.ctus["tile_id"]) == [0, 1, 2, 3]
    R.validate(params, pic)
    # the ids matter: tiles are independent, so the tiled decode differs from the untiled one
    untiled = pic.ctus.copy()
    untiled["tile_id"] = 0
    (rec_t, _), = c_oracle.decode(params, [pic])
    (rec_f, _), = c_oracle.decode(params, [dataclasses.replace(pic, ctus=untiled)])
    assert any((rec_t[c] != rec_f[c]).any() for c in range(3))
