"""Encode -> parse round trips for the syntax sanity.bin does not exercise (CPU only).

tests/streamgen.py writes streams from random syntax decisions and builds the records
the reference's decode_leaf hook would produce for them (frontend.PictureBuilder).
The native front-end (libp265fe.so) must parse each stream back into exactly those
records.  The reference cannot parse any of these features (pps.py:61-93 tiles,
slice.py:177 deblocking override, slice.py:181-189 entry points, slice.py:295
end_of_subset_one_bit, nalu.py:130 SEI), so parity there rests on this round trip
plus the spec restatement; the shared syntax is pinned by sanity.bin (test_bitstream.py).
"""
import numpy as np
import pytest

import streamgen
from p265_amd import bitstream

CASES = {
    "defaults": dict(),
    "plain": dict(sign_hiding=False, tskip=False, sao=False, strong=False),
    "tiles_uniform": dict(tiles=(2, 2)),
    "tiles_explicit": dict(tiles=([3, 5], [2, 4])),
    "wpp": dict(wpp=True),
    "tiles_wpp": dict(tiles=(2, 2), wpp=True),
    "slices": dict(slices=[(0, False), (13, False), (30, True)]),
    "dependent_slices_wpp": dict(slices=[(0, False), (5, True), (17, True), (40, False)], wpp=True),
    "tiles_slices": dict(tiles=(3, 2), slices=[(0, False), (16, False), (20, True)]),
    "qp_delta_ctb": dict(qp_delta_depth=0),
    "qp_delta_d1": dict(qp_delta_depth=1),
    "qp_delta_d2_ctb32": dict(qp_delta_depth=2, ctb_log2=5, width=192, height=128),
    "pcm_lf_off": dict(pcm=(3, 4, True)),
    "pcm_bypass": dict(pcm=(3, 3, False), bypass=True),
    "bypass": dict(bypass=True),
    "deblocking_override": dict(deblocking="override", slices=[(0, False), (20, False), (33, False)]),
    "deblocking_off": dict(deblocking="off"),
    "chroma_qp_offsets": dict(slice_chroma_offsets=(3, -5), cb_qp_offset=-4, cr_qp_offset=6, qp_delta_depth=1),
    "conformance_window": dict(conf_window=(1, 3, 2, 5), width=136, height=104),
    "ctb64_ragged": dict(width=200, height=72, ctb_log2=6, max_tb_log2=5, max_th_depth=2),
    "ctb32_mincb16": dict(ctb_log2=5, min_cb_log2=4, max_tb_log2=5, max_th_depth=3),
    "poc_idr_period": dict(frames=4, idr_period=3, log2_max_poc_lsb=4),
    "lf_flags_off": dict(lf_across_tiles=0, tiles=(2, 1), lf_across_slices=0),
    # Main 10: bit_depth_*_minus8 = 2, QpBdOffset 12 (cu_qp_delta range, QpY wrap, negative QpY), sao_offset_abs
    # cMax 31, PCM at 9 / 8 bits shifted to 10
    "main10": dict(bit_depth=10, qp_delta_depth=1, init_qp=14, slice_qp_delta=-20, pcm=(3, 4, True)),
    "main10_tiles_wpp_bypass": dict(bit_depth=10, tiles=(2, 2), wpp=True, bypass=True, qp_delta_depth=0),
    "main9_chroma_offsets": dict(bit_depth=9, slice_chroma_offsets=(3, -5), cb_qp_offset=-4, cr_qp_offset=6,
                                 qp_delta_depth=1, deblocking="override", slices=[(0, False), (20, False)]),
    # BitDepth 12 (QpBdOffset 24, SaoOffsetVal << 2, PCM at 11 / 10 bits)
    "main12_tiles": dict(bit_depth=12, tiles=(2, 2), qp_delta_depth=1, init_qp=4, slice_qp_delta=-25, pcm=(3, 4, True)),
    # scaling lists (7.3.4): enabled with the default lists, random lists in the SPS, SPS lists overridden by the PPS
    "scaling_default": dict(scaling_lists="default"),
    "scaling_sps": dict(scaling_lists="sps", tskip=True),
    "scaling_pps_main10": dict(scaling_lists="pps", bit_depth=10, ctb_log2=5, width=160, height=96),
}


def roundtrip(seed, threads=2, **cfg):
    g = streamgen.StreamGen(seed, **cfg)
    data, pics = g.stream()
    dec = bitstream.decode_stream(data, threads=threads)
    assert len(dec) == len(pics)
    for d, (prm, p, poc) in zip(dec, pics):
        assert d.params.tobytes() == prm.tobytes()
        assert d.poc == poc
        assert np.array_equal(d.picture.ctus, p.ctus)
        assert np.array_equal(d.picture.tbs, p.tbs)
        assert np.array_equal(d.picture.coef, p.coef)
        if g.scaling_factors is None:
            assert d.scaling is None
        else:
            assert np.array_equal(d.scaling, g.scaling_factors)
        if p.nofilter is None:
            assert d.picture.nofilter is None
        else:
            assert np.array_equal(d.picture.nofilter, p.nofilter)
    return g, dec


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("seed", [0, 1])
def test_roundtrip(name, seed):
    roundtrip(1000 + 17 * seed + len(name), **CASES[name])


def test_tile_and_slice_records():
    g, dec = roundtrip(7, tiles=(2, 2), slices=[(0, False), (24, False), (30, True)])
    ctus = dec[0].picture.ctus
    assert sorted(set(int(t) for t in ctus["tile_id"])) == [0, 1, 2, 3]
    # slice 2 starts at tile-scan address 24 -> SliceAddrRs of its CTBs; the dependent segment keeps it
    addrs = sorted(set(int(a) for a in ctus["slice_addr"]))
    assert addrs == [0, g.ts_to_rs[24]]


def test_conformance_window_and_counts():
    g, dec = roundtrip(9, conf_window=(1, 3, 2, 5), width=136, height=104)
    assert dec[0].crop == (2, 6, 4, 10)          # SubWidthC / SubHeightC = 2 for 4:2:0
    assert dec[0].n_slices == 1 and dec[0].n_cus > 0


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind", ["md5", "crc", "checksum"])
def test_decoded_picture_hash_sei_is_reported(kind, bd):
    g = streamgen.StreamGen(11, hash_sei=kind, bit_depth=bd)
    data, pics = g.stream()
    dec = bitstream.decode_stream(data)
    want_type, want = g.last_hash
    assert dec[0].hash_type == want_type
    assert dec[0].hash == want


def test_output_order_follows_poc_within_each_sequence():
    g, dec = roundtrip(5, frames=5, idr_period=2)
    assert [d.poc for d in dec] == [0, 1, 0, 1, 0]
    assert [d.output_rank for d in dec] == [0, 1, 2, 3, 4]
    assert [d.nal_unit_type for d in dec] == [19, 1, 19, 1, 19]


def test_unsupported_and_missing_parameter_sets():
    g = streamgen.StreamGen(3)
    data, _ = g.stream()
    # drop the SPS: the PPS/slices refer to a missing SPS
    nals = data.split(b"\x00\x00\x00\x01")[1:]
    no_sps = b"".join(b"\x00\x00\x00\x01" + n for n in nals if (n[0] >> 1) & 63 != 33)
    with pytest.raises(bitstream.BitstreamError):
        bitstream.decode_stream(no_sps)
    # truncated slice data
    with pytest.raises(bitstream.BitstreamError):
        bitstream.decode_stream(data[:len(data) - 40])


@pytest.mark.parametrize("kind", ["md5", "crc", "checksum"])
def test_hash_of_16bit_planes_matches_the_encoder(kind):
    """bitstream.plane_hash (the decoder's D.3.19 check) of uint16 planes equals the test encoder's
    independent restatement (streamgen.picture_hash): two bytes per sample, the checksum's high byte."""
    from p265_amd import bitstream as B
    rng = np.random.default_rng(4)
    planes = [rng.integers(0, 1024, (40, 24)).astype(np.uint16), rng.integers(0, 1024, (20, 12)).astype(np.uint16),
              rng.integers(0, 1024, (20, 12)).astype(np.uint16)]
    want = streamgen.picture_hash(planes, kind)
    code = {"md5": B.HASH_MD5, "crc": B.HASH_CRC, "checksum": B.HASH_CHECKSUM}[kind]
    assert [B.plane_hash(p, code) for p in planes] == want


@pytest.mark.parametrize("kind", ["default", "sps", "pps"])
def test_scaling_factors_from_the_front_end(kind):
    """The front-end's ScalingFactor table (fe_ps.cpp, 7.4.5) equals the oracle's derivation from the
    same scaling_list_data syntax (oracle/recon_oracle.py scaling_lists_from_syntax / scaling_factors)."""
    from oracle import recon_oracle as O
    g, dec = roundtrip(31 + len(kind), scaling_lists=kind)
    sf = dec[0].scaling
    assert sf.dtype == np.uint8 and sf.size == O.SF_BYTES and sf.min() >= 1
    if kind == "default":
        assert (O.factor_of(sf, 2, 0) == 16).all() and O.factor_of(sf, 3, 0)[7, 7] == 115
    else:
        sld = g.pps_sld if kind == "pps" else g.sps_sld
        lists, dcs = O.scaling_lists_from_syntax(sld)
        for (size_id, m), dc in dcs.items():
            if size_id >= 2 and (size_id, m) in O.SF_OFFSETS:   # DC: 16x16 / 32x32 intra matrices
                assert O.factor_of(sf, size_id + 2, m)[0, 0] == dc
        want = O.scaling_factor_bytes(O.scaling_factors(lists, dcs))
        assert np.array_equal(sf, want)


def test_scaling_list_syntax_errors_are_rejected():
    """A coded list value of 0 (7.4.5: nextCoef > 0) and a refMatrixId below 0 are stream errors."""
    g = streamgen.StreamGen(5, scaling_lists="sps")
    g.sps_sld[(0, 0)] = ("coded", None, [-8] + [0] * 15)
    with pytest.raises(bitstream.BitstreamError):
        bitstream.decode_stream(g.stream()[0])
    g = streamgen.StreamGen(5, scaling_lists="sps")
    g.sps_sld[(1, 1)] = ("pred", 2)
    with pytest.raises(bitstream.BitstreamError):
        bitstream.decode_stream(g.stream()[0])
