"""The C restatement of the oracle equals the Python one (CPU only).

The C oracle is what the GPU parity tests use at full 1080p/4K sizes and what bench.py
times as the CPU baseline, so it must agree bit for bit with oracle/recon_oracle.py
(which is itself pinned against the reference, tests/test_oracle_vs_reference.py).
"""
import os

import numpy as np
import pytest

from oracle import c_oracle
from oracle import recon_oracle as O
from p265_amd import frontend, synth
from p265_amd import records as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _same(params, pics):
    got = c_oracle.decode(params, pics, threads=4)
    pd = R.params_dict(params)
    for i, p in enumerate(pics):
        rec, out = O.decode_picture(pd, p.as_oracle_dict())
        for c in range(3):
            np.testing.assert_array_equal(got[i][0][c], rec[c], err_msg="pic %d recon c%d" % (i, c))
            np.testing.assert_array_equal(got[i][1][c], out[c], err_msg="pic %d out c%d" % (i, c))


def test_sanity_frames():
    params, pics = frontend.pictures_from_frontend_npz(os.path.join(GOLDEN, "sanity_frontend.npz"))
    _same(params, pics)


@pytest.mark.parametrize("ctb_log2,w,h,tiles,slices", [(6, 200, 136, (1, 1), 1), (5, 264, 200, (3, 2), 4),
                                                      (4, 72, 40, (1, 1), 2), (6, 136, 72, (2, 1), 1)])
def test_synthetic(ctb_log2, w, h, tiles, slices):
    params = R.make_params(pic_width=w, pic_height=h, ctb_log2_size=ctb_log2, loop_filter_across_tiles=int(w % 3 == 0))
    pics = [synth.make_picture(params, 700 + s, perf=False, tiles=tiles, n_slices=slices, lf_across_slices=None,
                               tskip_rate=0.3, bypass_rate=0.05) for s in range(2)]
    _same(params, pics)


def test_no_sao():
    params = R.make_params(pic_width=128, pic_height=64, sample_adaptive_offset=0, strong_intra_smoothing=0)
    _same(params, [synth.make_picture(params, 9, perf=False)])


@pytest.mark.parametrize("ctb_log2,w,h,tiles,slices", [(6, 200, 136, (1, 1), 1), (5, 264, 200, (3, 2), 4), (4, 72, 40, (1, 1), 2)])
def test_synthetic_main10(ctb_log2, w, h, tiles, slices):
    """BitDepth 10 (Main 10; uint16 planes): scaling / clip / substitution / SAO band shift / deblocking
    thresholds and QpY = qP' - 12, with deblocking on random slices, PCM, bypass, transform skip."""
    params = R.make_params(pic_width=w, pic_height=h, ctb_log2_size=ctb_log2, loop_filter_across_tiles=int(w % 3 == 0),
                           bit_depth_luma=10, bit_depth_chroma=10, pps_cb_qp_offset=-2, pps_cr_qp_offset=3)
    pics = [synth.make_picture(params, 1700 + s, perf=bool(s), tiles=tiles, n_slices=slices, lf_across_slices=None,
                               tskip_rate=0.3, bypass_rate=0.05, pcm_rate=0.03, deblocking="random") for s in range(2)]
    assert max(int(pics[0].tbs["qp"].max()), int(pics[1].tbs["qp"].max())) > 37     # qP' = QpY + 12 (QpY <= 37)
    _same(params, pics)
    got = c_oracle.decode(params, pics[:1])[0][1]
    assert got[0].dtype == np.uint16 and got[0].max() > 255


@pytest.mark.parametrize("bd", [11, 12])
def test_synthetic_high_bit_depth(bd):
    """BitDepth 11 / 12 (uint16 planes; QpBdOffset 18 / 24, SAO offsets << (BitDepth - 10)): the C twin equals
    the Python oracle with deblocking, PCM, bypass, transform skip, tiles and slices."""
    params = R.make_params(pic_width=200, pic_height=136, ctb_log2_size=5, bit_depth_luma=bd, bit_depth_chroma=bd,
                           pps_cb_qp_offset=1, pps_cr_qp_offset=-2)
    pics = [synth.make_picture(params, 1900 + bd + s, perf=bool(s), tiles=(2, 2), n_slices=2, lf_across_slices=None,
                               tskip_rate=0.3, bypass_rate=0.05, pcm_rate=0.03, deblocking="random") for s in range(2)]
    _same(params, pics)
    got = c_oracle.decode(params, pics[:1])[0][1]
    assert got[0].dtype == np.uint16 and got[0].max() > (1 << (bd - 1))
