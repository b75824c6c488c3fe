"""Native syntax front-end (libp265fe.so) against the reference's own parse of sanity.bin.

`tests/golden/sanity.bin` is the reference's test bitstream (a data file of its `make
check`, /root/reference/sanity.bin).  `tests/golden/sanity_frontend.npz` holds what the
reference's Python front-end hands to `Cu.decode_leaf` / `Sao.parse` for that stream,
captured by gen_sanity_fixture.py after checking all 95 files of the reference's
test/golden/ byte for byte.  The native front-end must reproduce those records exactly.
"""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from p265_amd import bitstream, frontend
from p265_amd import records as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def sanity_bytes():
    with open(os.path.join(GOLDEN, "sanity.bin"), "rb") as f:
        return f.read()


@pytest.fixture(scope="module")
def reference_records():
    return frontend.pictures_from_frontend_npz(os.path.join(GOLDEN, "sanity_frontend.npz"))


def test_sanity_bin_is_the_reference_stream(sanity_bytes):
    meta = json.load(open(os.path.join(GOLDEN, "sanity_frontend.json")))
    assert hashlib.sha256(sanity_bytes).hexdigest() == meta["bitstream_sha256"]


@pytest.mark.parametrize("threads", [1, 3])
def test_native_front_end_reproduces_reference_records(sanity_bytes, reference_records, threads):
    params, ref = reference_records
    pics = bitstream.decode_stream(sanity_bytes, threads=threads)
    assert len(pics) == len(ref) == 3
    for d, r in zip(pics, ref):
        assert d.params.tobytes() == params.tobytes()
        assert np.array_equal(d.picture.ctus, r.ctus)
        assert np.array_equal(d.picture.tbs, r.tbs)
        assert np.array_equal(d.picture.coef, r.coef)
        assert d.picture.nofilter is None and r.nofilter is None


def test_sanity_stream_metadata(sanity_bytes):
    meta = json.load(open(os.path.join(GOLDEN, "sanity_frontend.json")))
    pics = bitstream.decode_stream(sanity_bytes)
    assert [p.poc for p in pics] == [0, 1, 2]
    assert [p.output_rank for p in pics] == [0, 1, 2]
    # IDR_W_RADL then two TRAIL_R, one slice each, no SEI
    assert [p.nal_unit_type for p in pics] == [19, 1, 1]
    assert [p.n_slices for p in pics] == [1, 1, 1]
    assert sum(p.n_cus for p in pics) == meta["n_cus"] == 2763
    assert all(p.hash_type == bitstream.HASH_NONE for p in pics)
    assert all(p.crop == (0, 0, 0, 0) for p in pics)


def test_truncated_and_corrupted_streams_fail_cleanly(sanity_bytes):
    """Malformed input raises BitstreamError (never crashes the process)."""
    with pytest.raises(bitstream.BitstreamError):
        bitstream.decode_stream(sanity_bytes[:9000])
    rng = random.Random(265)
    outcomes = {"ok": 0, "error": 0}
    for _ in range(150):
        b = bytearray(sanity_bytes)
        for _ in range(rng.randint(1, 6)):
            pos = rng.randrange(80, len(b))
            b[pos] ^= 1 << rng.randrange(8)
        try:
            bitstream.decode_stream(bytes(b), threads=2)
            outcomes["ok"] += 1
        except bitstream.BitstreamError:
            outcomes["error"] += 1
    assert outcomes["error"] > 0


def test_empty_stream_has_no_pictures():
    assert bitstream.decode_stream(b"") == []
    assert bitstream.decode_stream(b"\x00\x00\x00\x01") == []


def test_md5_plane_hash_paths_agree():
    """plane_hash's MD5 (hashlib over the raster bytes) equals the library's D.3.19 MD5, for
    contiguous planes, strided views and odd sizes."""
    import numpy as np
    from p265_amd import bitstream as B
    rng = np.random.default_rng(3)
    for shp in [(1080, 1920), (540, 960), (7, 13), (1, 1)]:
        p = rng.integers(0, 256, shp, dtype=np.uint8)
        assert B.plane_hash(p, B.HASH_MD5) == B.plane_hash_native(p, B.HASH_MD5)
        v = p[:, ::-1] if shp[1] > 1 else p
        assert B.plane_hash(v, B.HASH_MD5) == B.plane_hash_native(v, B.HASH_MD5)
