"""End to end on the MI355X: bitstream -> native front-end -> HIP back-end -> planes.

Each generated stream carries a decoded-picture-hash SEI (D.3.19) computed from the
C oracle's decode of the generator's own records, so the decoder's built-in hash check
is the parity check (and the planes are compared with the oracle directly as well).
sanity.bin (the reference's stream) is decoded from its bytes and compared with the
oracle on the reference-captured records.
"""
import os

import numpy as np
import pytest

import streamgen
from oracle import c_oracle
from p265_amd import frontend

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dec_mod():
    from p265_amd import decoder, recon
    if recon.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return decoder


def oracle_planes(params, pic, scaling=None):
    return c_oracle.decode(params, [pic], with_recon=False, scaling=scaling)[0][1]


def test_sanity_bin_end_to_end(dec_mod):
    data = open(os.path.join(GOLDEN, "sanity.bin"), "rb").read()
    frames = dec_mod.decode_bytes(data)
    params, pics = frontend.pictures_from_frontend_npz(os.path.join(GOLDEN, "sanity_frontend.npz"))
    assert [f.poc for f in frames] == [0, 1, 2]
    for f, p in zip(frames, pics):
        want = oracle_planes(params, p)
        for c in range(3):
            np.testing.assert_array_equal(f.planes[c], want[c])


CASES = {
    "tiles_wpp": dict(tiles=(2, 2), wpp=True, width=192, height=128),
    "slices_dependent": dict(slices=[(0, False), (9, True), (20, False), (31, True)], deblocking="override"),
    "pcm_bypass_qp": dict(pcm=(3, 4, True), bypass=True, qp_delta_depth=1),
    "chroma_offsets": dict(slice_chroma_offsets=(2, -3), cb_qp_offset=3, cr_qp_offset=-2, qp_delta_depth=2,
                           ctb_log2=5, width=160, height=96),
    "ctb64_ragged_crop": dict(width=200, height=136, ctb_log2=6, max_tb_log2=5, max_th_depth=2,
                              conf_window=(2, 3, 1, 4)),
    "lf_off_tiles": dict(tiles=([2, 6], [3, 3]), lf_across_tiles=0, lf_across_slices=0,
                         slices=[(0, False), (30, False)]),
    "multi_frame": dict(frames=3, idr_period=2),
    "main10": dict(bit_depth=10, pcm=(3, 4, True), bypass=True, qp_delta_depth=1, init_qp=14, slice_qp_delta=-18,
                   deblocking="override", slices=[(0, False), (20, False)]),
    "main10_tiles_wpp_ctb32": dict(bit_depth=10, tiles=(2, 2), wpp=True, ctb_log2=5, width=192, height=128),
    "bd12_slices_pcm": dict(bit_depth=12, pcm=(3, 4, True), bypass=True, qp_delta_depth=1, init_qp=4,
                            slice_qp_delta=-20, deblocking="override", slices=[(0, False), (20, False)]),
    # scaling lists: the front-end's ScalingFactor table (SPS lists, PPS override, defaults) into the residual kernels
    "scaling_sps_tskip": dict(scaling_lists="sps", tskip=True, qp_delta_depth=1),
    "scaling_pps_main10": dict(scaling_lists="pps", bit_depth=10, ctb_log2=5, width=160, height=96, frames=2),
    "scaling_default_tiles": dict(scaling_lists="default", tiles=(2, 2), deblocking="override",
                                  slices=[(0, False), (20, False)]),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("kind", ["md5", "crc"])
def test_generated_streams_match_their_picture_hash(dec_mod, name, kind):
    g = streamgen.StreamGen(4000 + len(name), hash_sei=kind, **CASES[name])
    data, pics = g.stream(planes_fn=oracle_planes)
    frames = dec_mod.decode_bytes(data, batch=2)           # raises HashMismatch on any difference
    assert len(frames) == len(pics)
    assert all(f.hash_ok for f in frames)
    for f in frames:
        prm, pic, poc = pics[f.decode_index]
        assert f.poc == poc
        want = oracle_planes(prm, pic, scaling=g.scaling_factors)
        for c in range(3):
            np.testing.assert_array_equal(f.planes[c], want[c])


def test_hash_mismatch_is_reported(dec_mod):
    g = streamgen.StreamGen(77, hash_sei="md5")
    data, pics = g.stream()                                # random (wrong) hash values
    with pytest.raises(dec_mod.HashMismatch):
        dec_mod.decode_bytes(data)
    frames = dec_mod.decode_bytes(data, verify_hash=False)
    assert frames[0].hash_ok is False


def test_cli_writes_cropped_yuv(dec_mod, tmp_path):
    from p265_amd import dec
    g = streamgen.StreamGen(78, hash_sei="md5", conf_window=(1, 2, 3, 1), width=136, height=104, frames=2)
    data, pics = g.stream(planes_fn=oracle_planes)
    src = tmp_path / "s.bin"
    src.write_bytes(data)
    out = tmp_path / "o.yuv"
    assert dec.main(["-b", str(src), "-o", str(out)]) == 0
    w, h = 136 - 2 * (1 + 2), 104 - 2 * (3 + 1)
    assert out.stat().st_size == 2 * (w * h + 2 * (w // 2) * (h // 2))
    raw = np.frombuffer(out.read_bytes(), np.uint8)
    want = oracle_planes(*pics[0][:2])[0][6:6 + h, 2:2 + w]
    np.testing.assert_array_equal(raw[:w * h].reshape(h, w), want)
    # Main 10: 16-bit little-endian samples (yuv420p10le)
    g = streamgen.StreamGen(79, hash_sei="md5", bit_depth=10, width=136, height=104, frames=1)
    data, pics = g.stream(planes_fn=oracle_planes)
    src.write_bytes(data)
    assert dec.main(["-b", str(src), "-o", str(out)]) == 0
    assert out.stat().st_size == 2 * (136 * 104 * 3 // 2)
    raw = np.frombuffer(out.read_bytes(), "<u2")
    np.testing.assert_array_equal(raw[:136 * 104].reshape(104, 136), oracle_planes(*pics[0][:2])[0])


@pytest.mark.parametrize("name", ["synth_1080p_4pic.bin", "synth_4k_tiles.bin", "synth_main10.bin"])
def test_committed_streams_match_their_md5(dec_mod, name):
    data = open(os.path.join(GOLDEN, name), "rb").read()
    frames = dec_mod.decode_bytes(data)                     # raises HashMismatch on any difference
    assert frames and all(f.hash_ok for f in frames)


def test_c5_tile_units_on_the_gpu(dec_mod):
    """C5 from real bytes: each (picture, tile) unit decoded as its own sub-picture through
    libp265r.so, stitched, equal to the stream's MD5 (what each of the 8 ranks does)."""
    import hashlib
    from p265_amd import bitstream, recon, tiles
    pics = bitstream.decode_stream(open(os.path.join(GOLDEN, "synth_4k_tiles.bin"), "rb").read())
    for p in pics:
        parts = tiles.split(p.params, p.picture)
        planes = []
        for tp, tpic, _ in parts:
            with recon.ReconContext(tp) as ctx:
                planes.append(ctx.decode([tpic])[0])
        full = tiles.stitch(p.params, parts, planes)
        assert [hashlib.md5(full[c].tobytes()).digest() for c in range(3)] == p.hash


def test_decoder_abandoned_midway_ends_its_threads(dec_mod):
    """Leaving the decode_chunks generator after one frame (or on an exception) stops the parse
    and submit threads and frees the batches in flight: no hang, and the next decode works."""
    import threading
    data = open(os.path.join(GOLDEN, "synth_1080p_4pic.bin"), "rb").read() * 4
    before = threading.active_count()
    gen = dec_mod.decode_chunks([data[i:i + 100000] for i in range(0, len(data), 100000)], batch=2, depth=2)
    first = next(gen)
    assert first.hash_ok
    gen.close()
    assert threading.active_count() <= before + 1            # (the hash pool's threads are gone too)
    frames = dec_mod.decode_bytes(data[:len(data) // 4])
    assert len(frames) == 4 and all(f.hash_ok for f in frames)
