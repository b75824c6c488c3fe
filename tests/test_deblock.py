"""Deblocking (H.265 8.7.2) in the CPU oracle: known-answer tests and C/Python agreement.

The reference parses the deblocking controls (decoder/pps.py:122-131, slice.py:170-179)
but has no deblocking filter, so there is nothing of the reference's to pin against:
parity is UNPINNED by the reference and rests on the spec restatement, the hand-worked
cases below and the agreement of the two independent oracle restatements.
"""
import numpy as np
import pytest

from oracle import c_oracle
from oracle import recon_oracle as O
from p265_amd import frontend, synth
from p265_amd import records as R


def _seg(pv, qv):
    """4-line segment with constant rows: p[i][k] = pv[i], q[i][k] = qv[i]."""
    return [[pv[i]] * 4 for i in range(4)], [[qv[i]] * 4 for i in range(4)]


def test_tables():
    assert O.BETA_TABLE[15] == 0 and O.BETA_TABLE[16] == 6 and O.BETA_TABLE[28] == 18
    assert O.BETA_TABLE[29] == 20 and O.BETA_TABLE[51] == 64
    assert O.TC_TABLE[17] == 0 and O.TC_TABLE[18] == 1 and O.TC_TABLE[27] == 2 and O.TC_TABLE[53] == 24
    assert [O.qpc_from_qpi(q) for q in (29, 30, 34, 35, 42, 43, 51)] == [29, 29, 33, 33, 37, 37, 45]


def test_weak_filter_step_edge():
    # QP 32: beta = 26, tc = tC'(34) = 3.  |p0 - q0| = 10 >= (5 tc + 1) >> 1 = 8 -> normal filter;
    # dp = dq = 0 < (26 + 13) >> 3 -> p1 / q1 also filtered.
    # delta = (9*10 - 3*10 + 8) >> 4 = 4 -> clipped to tc = 3
    # dp1 = Clip3(-1, 1, (100 - 100 + 3) >> 1) = 1 ; dq1 = Clip3(-1, 1, (110 - 110 - 3) >> 1) = -1
    p, q = _seg([100] * 4, [110] * 4)
    p, q = O.deblock_luma_segment(p, q, 32, 32, 0, 0, False, False)
    assert [r[0] for r in p] == [103, 101, 100, 100]
    assert [r[0] for r in q] == [107, 109, 110, 110]
    assert all(len(set(r)) == 1 for r in p + q)               # every line filtered the same


def test_strong_filter_small_step():
    # |p0 - q0| = 4 < 8, flat sides -> strong filter (8.7.2.5.7), clipped to +-2 tc = 6
    p, q = _seg([100] * 4, [104] * 4)
    p, q = O.deblock_luma_segment(p, q, 32, 32, 0, 0, False, False)
    assert [r[0] for r in p] == [102, 101, 101, 100]
    assert [r[0] for r in q] == [103, 103, 104, 104]


def test_no_filter_on_texture_and_low_qp():
    p, q = _seg([100, 130, 100, 130], [110, 80, 110, 80])    # d = 120 >= beta
    p2, q2 = O.deblock_luma_segment(p, q, 32, 32, 0, 0, False, False)
    assert p2 == p and q2 == q
    p, q = _seg([100] * 4, [110] * 4)                          # QP 15: beta' = 0
    p2, q2 = O.deblock_luma_segment(p, q, 15, 15, 0, 0, False, False)
    assert p2 == p and q2 == q
    # a big step (|delta| >= 10 tc) is a real edge: untouched
    # delta = (9*100 - 3*100 + 8) >> 4 = 38
    p, q = _seg([100] * 4, [200] * 4)
    p2, q2 = O.deblock_luma_segment(p, q, 51, 51, 0, 0, False, False)
    assert p2[0][0] == 124                                     # QP 51: tc = tC'(53) = 24, 38 < 240 -> clipped to tc
    p2, q2 = O.deblock_luma_segment(p, q, 32, 32, 0, 0, False, False)
    assert p2 == p and q2 == q                                 # tc = 3: |delta| = 38 >= 30


def test_offsets_and_nofilter_side():
    p, q = _seg([100] * 4, [110] * 4)
    # tc_offset_div2 = +6 -> Q = 34 + 12 = 46 -> tc' = 11; |p0 - q0| = 10 < 28 -> strong
    p2, q2 = O.deblock_luma_segment(p, q, 32, 32, 0, 6, False, False)
    assert p2[0][0] == (100 + 200 + 200 + 220 + 110 + 4) >> 3
    # PCM / bypass on the P side (nDp = 0): only Q changes
    p3, q3 = O.deblock_luma_segment(p, q, 32, 32, 0, 6, True, False)
    assert p3 == p and q3 == q2


def test_chroma_line():
    # qPi = 32 -> QpC = 31 -> tc = tC'(33) = 3 ; delta = Clip3(-3, 3, (40 + 100 - 110 + 4) >> 3 = 4) = 3
    tc = O.chroma_tc(32, 32, 0, 0)
    assert tc == 3
    assert O.deblock_chroma_line(100, 100, 110, 110, tc, False, False) == (103, 107)
    assert O.deblock_chroma_line(100, 100, 110, 110, tc, False, True) == (103, 110)
    assert O.chroma_tc(32, 32, 12, 0) == O.TC_TABLE[O.qpc_from_qpi(44) + 2]


def _two_tb_picture(deblocking=True, lf_across_slices=True, two_slices=False, two_tiles=False, lf_tiles=1):
    """32x16 picture, CTB 16: two CTUs, each one 16x16 luma TB (DC) + 8x8 chroma TBs."""
    params = R.make_params(pic_width=32, pic_height=16, ctb_log2_size=4, sample_adaptive_offset=0,
                           loop_filter_across_tiles=lf_tiles)
    b = frontend.PictureBuilder(params)
    for i in range(2):
        tu = dict(x=16 * i, y=0, log2=4, blk=0, cbf=[1, 0, 0], tskip=[0, 0, 0],
                  coef=[np.pad(np.array([[2 * (1 - 2 * i)]], np.int16), ((0, 15), (0, 15))), None, None])
        b.add_cu(16 * i, 0, 4, 0, [1, 0, 0, 0], 1, 37, 34, 34, [tu])
        b.add_ctu(i, slice_addr=i if two_slices else 0, tile_id=i if two_tiles else 0,
                  lf_across_slices=lf_across_slices, deblocking=deblocking)
    return params, b.finish()


def test_picture_edge_rules():
    params, pic = _two_tb_picture()
    pd = R.params_dict(params)
    rec, out = O.decode_picture(pd, pic.as_oracle_dict())
    d = out[0] - rec[0]
    assert d[:, 13:19].any() and not d[:, :13].any() and not d[:, 19:].any()   # only around x = 16
    # off in the Q-side slice, or across a slice / tile boundary without permission: untouched
    for kw in (dict(deblocking=False), dict(two_slices=True, lf_across_slices=False),
               dict(two_tiles=True, lf_tiles=0)):
        params, pic = _two_tb_picture(**kw)
        rec, out = O.decode_picture(R.params_dict(params), pic.as_oracle_dict())
        for c in range(3):
            np.testing.assert_array_equal(out[c], rec[c])
    params, pic = _two_tb_picture(two_slices=True, lf_across_slices=True)
    rec, out = O.decode_picture(R.params_dict(params), pic.as_oracle_dict())
    assert (out[0] != rec[0]).any()


def _c_vs_py(params, pics):
    got = c_oracle.decode(params, pics, threads=4)
    pd = R.params_dict(params)
    for i, p in enumerate(pics):
        rec, out = O.decode_picture(pd, p.as_oracle_dict())
        for c in range(3):
            np.testing.assert_array_equal(got[i][0][c], rec[c])
            np.testing.assert_array_equal(got[i][1][c], out[c], err_msg="pic %d c%d" % (i, c))


@pytest.mark.parametrize("ctb_log2,w,h,tiles,slices,sao", [(6, 200, 136, (1, 1), 1, True), (5, 264, 200, (3, 2), 4, True),
                                                          (4, 72, 40, (1, 1), 3, False), (6, 136, 72, (2, 1), 2, True)])
def test_c_oracle_equals_python_with_deblocking(ctb_log2, w, h, tiles, slices, sao):
    params = R.make_params(pic_width=w, pic_height=h, ctb_log2_size=ctb_log2, sample_adaptive_offset=int(sao),
                           loop_filter_across_tiles=int(w % 3 == 0), pps_cb_qp_offset=(w % 7) - 3,
                           pps_cr_qp_offset=3 - (h % 7))
    pics = [synth.make_picture(params, 900 + s, perf=False, tiles=tiles, n_slices=slices, lf_across_slices=None,
                               deblocking="random", bypass_rate=0.04, pcm_rate=0.03, sao=sao) for s in range(2)]
    _c_vs_py(params, pics)


def test_deblocking_changes_sanity_output():
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "sanity_frontend.npz")
    params, on = frontend.pictures_from_frontend_npz(path)
    _, off = frontend.pictures_from_frontend_npz(path, deblocking=False)
    assert (on[0].ctus["flags"] & R.CTU_DEBLOCK).all() and not (off[0].ctus["flags"] & R.CTU_DEBLOCK).any()
    pd = R.params_dict(params)
    rec_on, out_on = O.decode_picture(pd, on[0].as_oracle_dict())
    rec_off, out_off = O.decode_picture(pd, off[0].as_oracle_dict())
    np.testing.assert_array_equal(rec_on[0], rec_off[0])        # deblocking is after reconstruction
    assert (out_on[0] != out_off[0]).mean() > 0.05
