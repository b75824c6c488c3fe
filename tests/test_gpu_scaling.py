"""Scaling lists on the GPU (scaling_list_enabled; the ScalingFactor branch of decoder/scaling.py:32-44)
through the C ABI (p265r_set_scaling_factors) vs the oracles, bit-exact: random factors (1..255) and the
default lists (Table 7-5 / 7-6), 8 and 10 bits, every TB size, transform skip, deblocking."""
import numpy as np
import pytest

from oracle import c_oracle
from oracle import recon_oracle as O
from p265_amd import synth
from p265_amd import records as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def recon_mod():
    from p265_amd import recon
    if recon.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return recon


def _factors(kind, seed=0):
    if kind == "default":
        lists, dcs = O.scaling_lists_from_syntax({(s, m): ("pred", 0) for s in range(4) for m in range(0, 6, 3 if s == 3 else 1)})
        return O.scaling_factor_bytes(O.scaling_factors(lists, dcs))
    rng = np.random.default_rng(seed)
    return O.scaling_factor_bytes({k: rng.integers(1, 256, (4 << k[0], 4 << k[0])) for k in O.SF_OFFSETS})


@pytest.mark.parametrize("kind", ["random", "default"])
@pytest.mark.parametrize("bd,ctb_log2,w,h,deblocking", [(8, 6, 200, 136, False), (8, 5, 264, 200, "random"),
                                                        (10, 6, 136, 72, True), (8, 4, 72, 40, False)])
def test_scaling_lists_parity(recon_mod, kind, bd, ctb_log2, w, h, deblocking):
    params = R.make_params(pic_width=w, pic_height=h, ctb_log2_size=ctb_log2, scaling_list_enabled=1,
                           bit_depth_luma=bd, bit_depth_chroma=bd)
    sf = _factors(kind, seed=w + bd)
    pics = [synth.make_picture(params, 6300 + s, perf=bool(s), tskip_rate=0.3, deblocking=deblocking, bypass_rate=0.02)
            for s in range(3)]
    with recon_mod.ReconContext(params, scaling=sf) as ctx:
        outs, recs = ctx.decode(pics, with_recon=True)
    pd = R.params_dict(params)
    pd["scaling_factors"] = sf
    for i, p in enumerate(pics):
        rec_ref, out_ref = O.decode_picture(pd, p.as_oracle_dict())
        for c in range(3):
            np.testing.assert_array_equal(recs[i][c], rec_ref[c], err_msg="pic %d recon c%d" % (i, c))
            np.testing.assert_array_equal(outs[i][c], out_ref[c], err_msg="pic %d out c%d" % (i, c))


def test_scaling_lists_1080p(recon_mod):
    params = R.make_params(pic_width=1920, pic_height=1080, scaling_list_enabled=1)
    sf = _factors("random", 7)
    pics = [synth.make_picture(params, 6400, perf=True)]
    with recon_mod.ReconContext(params, scaling=sf) as ctx:
        outs = ctx.decode(pics)
    ref = c_oracle.decode(params, pics, threads=8, scaling=sf)
    for c in range(3):
        np.testing.assert_array_equal(outs[0][c], ref[0][1][c])


def test_scaling_factor_contract(recon_mod):
    from p265_amd import _lib
    params = R.make_params(pic_width=64, pic_height=64, scaling_list_enabled=1)
    pic = synth.make_picture(params, 3)
    with recon_mod.ReconContext(params) as ctx:
        with pytest.raises(_lib.P265RError) as ei:          # enabled, but no table given
            ctx.decode([pic])
        assert ei.value.code == _lib.ESTATE
        bad = _factors("default")
        bad[100] = 0
        with pytest.raises(_lib.P265RError) as ei:
            ctx.set_scaling_factors(bad)
        assert ei.value.code == _lib.EINVAL
        with pytest.raises(_lib.P265RError) as ei:
            ctx.set_scaling_factors(bad[:100])
        assert ei.value.code == _lib.EINVAL
    with recon_mod.ReconContext(R.make_params(pic_width=64, pic_height=64)) as ctx:
        with pytest.raises(_lib.P265RError) as ei:           # scaling lists off: no table to set
            ctx.set_scaling_factors(_factors("default"))
        assert ei.value.code == _lib.ESTATE
