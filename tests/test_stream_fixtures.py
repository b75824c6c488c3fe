"""The committed synthetic bitstreams (tests/golden/gen_streams.py), CPU only.

Each picture of these streams carries an MD5 decoded-picture-hash SEI.  Parsing the bytes
with the native front-end and reconstructing with the C oracle must reproduce every hash;
config C5 (4K, 2x2 tiles, 2 pictures) is also decoded tile by tile as independent
sub-pictures, sharded over two rank processes (socket control plane) as the 8-GPU run shards it, and
stitched back.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import c_oracle
from p265_amd import bitstream, dist, tiles

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(GOLDEN, "synth_streams.json")))


def _load(name):
    return open(os.path.join(GOLDEN, name), "rb").read()


@pytest.mark.parametrize("name", sorted(META))
def test_fixture_parses_and_matches_its_md5(name):
    data = _load(name)
    assert len(data) == META[name]["bytes"]
    pics = bitstream.decode_stream(data)
    assert len(pics) == META[name]["pictures"]
    assert sum(len(p.picture.ctus) for p in pics) == META[name]["ctus"]
    for p in pics:
        assert p.hash_type == bitstream.HASH_MD5
        planes = c_oracle.decode(p.params, [p.picture], with_recon=False)[0][1]
        assert [hashlib.md5(np.ascontiguousarray(planes[c]).tobytes()).digest() for c in range(3)] == p.hash


def test_1080p_fixture_has_the_surveyed_statistics():
    pics = bitstream.decode_stream(_load("synth_1080p_4pic.bin"))
    tbs = np.concatenate([p.picture.tbs for p in pics])
    luma = tbs[tbs["c_idx"] == 0]
    area = np.array([np.sum((luma["log2_size"] == k) * (1 << (2 * k))) for k in (2, 3, 4, 5)], float)
    area /= area.sum()
    # 26.2 / 30.7 / 26.3 / 16.8 % of luma area in 4/8/16/32 TBs
    assert np.all(np.abs(area - np.array([0.262, 0.307, 0.263, 0.168])) < 0.06)
    assert 250 < META["synth_1080p_4pic.bin"]["bytes_per_ctu"] < 380          # sanity.bin: 316 B/CTU
    assert all(int(p.params["pic_width"]) == 1920 and int(p.params["pic_height"]) == 1080 for p in pics)


def _c5_worker(rank, world):
    pics = bitstream.decode_stream(_load("synth_4k_tiles.bin"))          # every rank parses the stream
    params = dist.broadcast_params(pics[0].params)
    digests = []
    for f, t in dist.unit_shard(len(pics), 4, rank, world):
        tp, tpic, origin = tiles.split(params, pics[f].picture)[t]
        planes = c_oracle.decode(tp, [tpic], with_recon=False)[0][1]
        digests.append(("%d/%d" % (f, t), [np.ascontiguousarray(planes[c]).tobytes().hex() for c in range(3)]))
    return dist.gather_digests(digests)


def test_c5_tile_units_sharded_over_two_ranks_reproduce_the_md5():
    from ranks import run_ranks
    merged = run_ranks(_c5_worker, 2)[0]
    pics = bitstream.decode_stream(_load("synth_4k_tiles.bin"))
    assert len(merged) == 8                                               # 2 pictures x 4 tiles
    for f, p in enumerate(pics):
        parts = tiles.split(p.params, p.picture)
        planes_per_tile = []
        for t, (tp, _, _) in enumerate(parts):
            hexes = merged["%d/%d" % (f, t)]
            w, h = int(tp["pic_width"]), int(tp["pic_height"])
            shapes = [(h, w), (h // 2, w // 2), (h // 2, w // 2)]
            planes_per_tile.append([np.frombuffer(bytes.fromhex(hx), np.uint8).reshape(s)
                                    for hx, s in zip(hexes, shapes)])
        full = tiles.stitch(p.params, parts, planes_per_tile)
        assert [hashlib.md5(full[c].tobytes()).digest() for c in range(3)] == p.hash
