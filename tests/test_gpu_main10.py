"""Main 10 (BitDepth 10) on the GPU through the C ABI vs the oracles, bit-exact.

The 16-bit sample path (uint16_t planes; the row pipeline on 16-bit LDS tiles, intra_rows_kernel<..., uint16_t>
(int16_t at BitDepth 11-12),
and the per-diagonal kernel intra_step_kernel<uint16_t> (P265R_SCHEDULE=steps); sao16.h for SAO-only batches,
loopfilter16.h; the residual kernels with bdShift = BitDepth + log2 - 5 and 20 - BitDepth) against
oracle/recon_oracle.py (pinned at 10 bits by tests/golden/ref_components_bd10.npz from the reference's
own scaling / prediction / reconstruction, tests/test_oracle_vs_reference.py) and its C twin.
"""
import numpy as np
import pytest

from oracle import c_oracle
from oracle import recon_oracle as O
from p265_amd import digest, synth
from p265_amd import records as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def recon_mod():
    from p265_amd import recon
    if recon.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return recon


def _check(recon_mod, params, pics, label, c_ref=False):
    with recon_mod.ReconContext(params) as ctx:
        assert ctx.describe()["bit_depth"] == int(params["bit_depth_luma"])
        outs, recs = ctx.decode(pics, with_recon=True)
    if c_ref:
        refs = c_oracle.decode(params, pics, threads=8)
    else:
        pd = R.params_dict(params)
        refs = [O.decode_picture(R.params_dict(R.pic_params(params, p)), p.as_oracle_dict()) for p in pics]
    for i in range(len(pics)):
        for c in range(3):
            assert outs[i][c].dtype == np.uint16
            np.testing.assert_array_equal(recs[i][c], refs[i][0][c], err_msg="%s pic %d recon c%d" % (label, i, c))
            np.testing.assert_array_equal(outs[i][c], refs[i][1][c], err_msg="%s pic %d out c%d" % (label, i, c))
    return outs


@pytest.mark.parametrize("ctb_log2,w,h,deblocking", [(6, 352, 288, False), (5, 200, 136, "random"), (4, 72, 40, True),
                                                     (6, 136, 72, "random")])
def test_main10_uniform_modes(recon_mod, ctb_log2, w, h, deblocking):
    params = R.make_params(pic_width=w, pic_height=h, ctb_log2_size=ctb_log2, bit_depth_luma=10, bit_depth_chroma=10,
                           pps_cb_qp_offset=(w % 5) - 2, pps_cr_qp_offset=2 - (h % 5))
    pics = [synth.make_picture(params, 5100 + 10 * ctb_log2 + s, perf=False, deblocking=deblocking) for s in range(3)]
    _check(recon_mod, params, pics, "main10 uniform")


@pytest.mark.parametrize("deblocking", ["random", False])
@pytest.mark.parametrize("ctb_log2,lf_tiles", [(5, 0), (4, 1), (6, 0)])
def test_main10_slices_tiles_pcm_bypass_tskip(recon_mod, deblocking, ctb_log2, lf_tiles):
    """Slices (with and without loop filtering across them), tiles, PCM, bypass, transform skip; without
    deblocking the batch takes the streaming SAO kernel (sao16.h), with it loopfilter16.h."""
    params = R.make_params(pic_width=264, pic_height=200, ctb_log2_size=ctb_log2, loop_filter_across_tiles=lf_tiles,
                           bit_depth_luma=10, bit_depth_chroma=10)
    pics = [synth.make_picture(params, 5200 + s + 10 * ctb_log2, perf=False, tiles=(3, 2), n_slices=4,
                               lf_across_slices=None, deblocking=deblocking, bypass_rate=0.05, pcm_rate=0.03,
                               tskip_rate=0.3) for s in range(2)]
    _check(recon_mod, params, pics, "main10 tiles")


def test_main10_no_sao(recon_mod):
    params = R.make_params(pic_width=128, pic_height=64, sample_adaptive_offset=0, bit_depth_luma=10, bit_depth_chroma=10)
    _check(recon_mod, params, [synth.make_picture(params, 5300 + s, perf=False) for s in range(2)], "main10 nosao")
    params = R.make_params(pic_width=128, pic_height=64, sample_adaptive_offset=0, bit_depth_luma=10, bit_depth_chroma=10)
    _check(recon_mod, params, [synth.make_picture(params, 5310, perf=False, deblocking=True)], "main10 dbk only")


def test_main10_1080p_with_deblocking(recon_mod):
    params = R.make_params(pic_width=1920, pic_height=1080, bit_depth_luma=10, bit_depth_chroma=10)
    pics = [synth.make_picture(params, 5400 + s, perf=True, deblocking=bool(s)) for s in range(2)]
    _check(recon_mod, params, pics, "main10 1080p", c_ref=True)


def test_main10_9bit(recon_mod):
    params = R.make_params(pic_width=200, pic_height=136, ctb_log2_size=5, bit_depth_luma=9, bit_depth_chroma=9)
    pics = [synth.make_picture(params, 5500 + s, perf=False, deblocking="random", pcm_rate=0.02) for s in range(2)]
    _check(recon_mod, params, pics, "9-bit")


@pytest.mark.parametrize("deblocking", [True, False])
def test_main10_ragged_batch_and_digest(recon_mod, deblocking):
    """A ragged 10-bit batch (four picture sizes) and the device digest of uint16 planes (32-bit words of two
    samples) equal the host digest of the oracle's planes."""
    big = R.make_params(pic_width=264, pic_height=200, ctb_log2_size=5, bit_depth_luma=10, bit_depth_chroma=10)
    sizes = [(264, 200), (128, 72), (40, 200), (264, 8)]
    pics = []
    for k, (w, h) in enumerate(sizes):
        pp = R.pic_params(big, R.Picture(ctus=None, tbs=None, coef=None, size=(w, h)))
        pic = synth.make_picture(pp, 5600 + k, perf=bool(k % 2), deblocking=deblocking)
        pic.size = (w, h)
        pics.append(pic)
    _check(recon_mod, big, pics, "main10 ragged")
    with recon_mod.ReconContext(big) as ctx:
        b = ctx.upload(pics)
        ctx.run(b)
        got, got_rec = ctx.digest(b), ctx.digest(b, recon=True)
        b.free()
    for i, pic in enumerate(pics):
        rec_ref, out_ref = O.decode_picture(R.params_dict(R.pic_params(big, pic)), pic.as_oracle_dict())
        assert np.array_equal(got[i], digest.picture_digest([np.asarray(p, np.uint16) for p in out_ref])), "out %d" % i
        assert np.array_equal(got_rec[i], digest.picture_digest([np.asarray(p, np.uint16) for p in rec_ref])), "rec %d" % i


def test_main10_row_pipeline_and_schedules(recon_mod, monkeypatch):
    """The 16-bit row pipeline (W = 12 alone, W = 8 while another lane runs, the component split of a small
    batch) and the per-diagonal schedule (P265R_SCHEDULE=steps) give the same planes."""
    params = R.make_params(pic_width=352, pic_height=288, bit_depth_luma=10, bit_depth_chroma=10)
    pics = [synth.make_picture(params, 5700 + s, perf=bool(s % 2), deblocking=bool(s % 3 == 0), tskip_rate=0.2)
            for s in range(6)]
    ref = _check(recon_mod, params, pics, "main10 rows")
    with recon_mod.ReconContext(params) as ctx:
        ctx.set_pipeline(2)
        ba, bb = ctx.upload(pics[:3]), ctx.upload(pics[3:])
        for _ in range(2):
            ctx.run(ba)
            ctx.run(bb)
        ctx.sync()
        outs = ctx.download(ba) + ctx.download(bb)
        d = ctx.describe()
        ba.free(); bb.free()
    assert d["schedule"] == "rows"
    for i in range(6):
        for c in range(3):
            np.testing.assert_array_equal(outs[i][c], ref[i][c], err_msg="pipelined pic %d c%d" % (i, c))
    monkeypatch.setenv("P265R_SCHEDULE", "steps")
    with recon_mod.ReconContext(params) as ctx:
        assert ctx.describe()["schedule"] == "steps"
        outs = ctx.decode(pics)
    for i in range(6):
        for c in range(3):
            np.testing.assert_array_equal(outs[i][c], ref[i][c], err_msg="steps pic %d c%d" % (i, c))


@pytest.mark.parametrize("schedule", ["rows", "steps"])
@pytest.mark.parametrize("bd", [11, 12])
@pytest.mark.parametrize("case", ["uniform", "tiles", "sao_only", "ragged"])
def test_high_bit_depth(recon_mod, monkeypatch, schedule, bd, case):
    """BitDepth 11 / 12 against the oracles: the row pipeline (intra_rows_kernel<..., int16_t>: the packed
    Cb | Cr angular sums split into 6-bit halves, pang) and the per-diagonal kernel intra_step_kernel<uint16_t>
    (P265R_SCHEDULE=steps); loopfilter16.h / sao16.h; the residual kernels at bdShift BitDepth + log2 - 5 /
    20 - BitDepth.  The synthetic pictures reach QpY 51 above 10 bits (Qp'Y up to 75: the uint16 deblocking map)."""
    if schedule == "steps":
        monkeypatch.setenv("P265R_SCHEDULE", "steps")
    if case == "ragged":
        big = R.make_params(pic_width=264, pic_height=200, ctb_log2_size=5, bit_depth_luma=bd, bit_depth_chroma=bd)
        pics = []
        for k, (w, h) in enumerate([(264, 200), (128, 72), (40, 200)]):
            pp = R.pic_params(big, R.Picture(ctus=None, tbs=None, coef=None, size=(w, h)))
            pic = synth.make_picture(pp, 5800 + bd + k, perf=bool(k % 2), deblocking=bool(k % 2))
            pic.size = (w, h)
            pics.append(pic)
        with recon_mod.ReconContext(big) as ctx:
            assert ctx.describe()["schedule"] == schedule
        _check(recon_mod, big, pics, "bd%d ragged %s" % (bd, schedule))
        return
    params = R.make_params(pic_width=200, pic_height=136, ctb_log2_size=5 if case != "uniform" else 6,
                           bit_depth_luma=bd, bit_depth_chroma=bd, loop_filter_across_tiles=0,
                           pps_cb_qp_offset=-1, pps_cr_qp_offset=2)
    kw = dict(uniform=dict(perf=False, deblocking=True),
              tiles=dict(perf=False, tiles=(2, 2), n_slices=3, lf_across_slices=None, deblocking="random",
                         bypass_rate=0.05, pcm_rate=0.03, tskip_rate=0.3),
              sao_only=dict(perf=True, deblocking=False, tskip_rate=0.2, pcm_rate=0.02))[case]
    pics = [synth.make_picture(params, 5900 + bd + s, **kw) for s in range(2)]
    with recon_mod.ReconContext(params) as ctx:
        assert ctx.describe()["schedule"] == schedule
    _check(recon_mod, params, pics, "bd%d %s %s" % (bd, case, schedule))


def test_unsupported_bit_depths_rejected(recon_mod):
    from p265_amd import _lib
    for bl, bc in ((13, 13), (14, 14), (12, 10), (10, 8), (8, 10)):
        params = R.make_params(pic_width=64, pic_height=64, bit_depth_luma=bl, bit_depth_chroma=bc)
        with pytest.raises(_lib.P265RError) as ei:
            recon_mod.ReconContext(params)
        assert ei.value.code == _lib.EUNSUPPORTED
