"""Sharding logic of the multi-GPU path, on CPU: tile sub-pictures (C5), a world_size-2
run of frame sharding (C4) with the params broadcast over the socket control plane
(p265_amd/comm.py), and the control-plane collectives with three ranks.  The decode inside
the ranks uses the C oracle (no GPU here); tests/test_a_multirank.py runs the same shard
plans through libp265r.so on the GPU box, and bench.py broadcasts the params with RCCL."""
import os

import numpy as np
import pytest

from oracle import c_oracle
from p265_amd import dist, synth, tiles
from p265_amd import records as R


def test_shard_plans_cover_everything_once():
    for world in (1, 2, 3, 8):
        got = sorted(f for r in range(world) for f in dist.frame_shard(13, r, world))
        assert got == list(range(13))
        units = sorted(u for r in range(world) for u in dist.unit_shard(2, 4, r, world))
        assert units == [(f, t) for f in range(2) for t in range(4)]
    assert [len(dist.unit_shard(2, 4, r, 8)) for r in range(8)] == [1] * 8      # C5: 8 units on 8 GPUs


@pytest.mark.parametrize("w,h,grid", [(320, 192, (2, 2)), (264, 200, (3, 2)), (512, 288, (2, 1))])
def test_tiles_decode_like_the_whole_picture(w, h, grid):
    params = R.make_params(pic_width=w, pic_height=h, ctb_log2_size=5, loop_filter_across_tiles=0)
    pic = synth.make_picture(params, 31, perf=False, tiles=grid, n_slices=2, lf_across_slices=None)
    whole = c_oracle.decode(params, [pic])[0][1]
    parts = tiles.split(params, pic)
    assert len(parts) == grid[0] * grid[1]
    decoded = [c_oracle.decode(tp, [tpic])[0][1] for tp, tpic, _ in parts]
    stitched = tiles.stitch(params, parts, decoded)
    for c in range(3):
        np.testing.assert_array_equal(stitched[c], whole[c])


def test_tile_split_refuses_cross_tile_loop_filter():
    params = R.make_params(pic_width=128, pic_height=64, loop_filter_across_tiles=1)
    pic = synth.make_picture(params, 2, tiles=(2, 1))
    with pytest.raises(NotImplementedError):
        tiles.split(params, pic)


def _worker(rank, world):
    import hashlib
    params = R.make_params(pic_width=192, pic_height=128) if rank == 0 else R.make_params()   # ranks disagree...
    params = dist.broadcast_params(params)                                                      # ...until broadcast
    mine = dist.frame_shard(6, rank, world)
    pics = [synth.make_picture(params, 900 + f) for f in mine]
    outs = c_oracle.decode(params, pics)
    dig = [(f, hashlib.sha256(b"".join(o[1][c].tobytes() for c in range(3))).hexdigest()) for f, o in zip(mine, outs)]
    merged = dist.gather_digests(dig)
    t = dist.max_over_ranks(float(rank + 1))
    return len(merged), t, int(params["pic_width"]), merged


def test_world2_frame_sharding_over_the_control_plane():
    import hashlib
    from ranks import run_ranks
    res = run_ranks(_worker, 2)
    for rank in (0, 1):
        n, t, width, merged = res[rank]
        assert (n, t, width) == (6, 2.0, 192)
    params = R.make_params(pic_width=192, pic_height=128)
    ref = c_oracle.decode(params, [synth.make_picture(params, 900 + f) for f in range(6)])
    for f in range(6):
        assert res[0][3][f] == hashlib.sha256(b"".join(ref[f][1][c].tobytes() for c in range(3))).hexdigest()


def _comm_worker(rank, world):
    from p265_amd import dist as D
    from p265_amd.comm import pack_map, unpack_map
    c = D.group().ctrl
    got = {}
    got["bcast"] = c.bcast(b"hello" if rank == 2 else b"", src=2)
    got["allgather"] = c.allgather(bytes([rank]) * (rank + 1))
    got["max"] = c.max(float(10 - rank))
    c.barrier()
    got["a2a"] = c.alltoall({d: b"%d->%d" % (rank, d) for d in range(world) if d != rank})
    got["map"] = unpack_map(pack_map({3: b"x", -1: b""}))
    sends = [((rank + 1) % world, 100 * rank + 1, b"a" * (rank + 1)), ((rank + 2) % world, 100 * rank + 2, b"")]
    recvs = [((rank - 1) % world, 100 * ((rank - 1) % world) + 1), ((rank - 2) % world, 100 * ((rank - 2) % world) + 2)]
    got["exchange"] = D.exchange(sends, recvs)
    return got


def test_control_plane_collectives_three_ranks():
    from ranks import run_ranks
    res = run_ranks(_comm_worker, 3)
    for r in range(3):
        g = res[r]
        assert g["bcast"] == b"hello"
        assert g["allgather"] == [b"\x00", b"\x01\x01", b"\x02\x02\x02"]
        assert g["max"] == 10.0
        assert g["a2a"] == {s: b"%d->%d" % (s, r) for s in range(3) if s != r}
        assert g["map"] == {3: b"x", -1: b""}
        p1, p2 = (r - 1) % 3, (r - 2) % 3
        assert g["exchange"] == {100 * p1 + 1: b"a" * (p1 + 1), 100 * p2 + 2: b""}


def test_product_package_has_no_torch():
    """north_star: the host side calls the HIP kernels through ctypes, no PyTorch."""
    import glob
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "p265_amd")
    for f in glob.glob(os.path.join(root, "*.py")):
        src = open(f).read()
        assert "import torch" not in src and "from torch" not in src, f


def test_rccl_binding_loads():
    """librccl.so.1 and the HIP runtime bind through ctypes (no device needed for the symbols)."""
    from p265_amd import rccl
    h = rccl.lib()
    for name in ("ncclGetUniqueId", "ncclCommInitRank", "ncclBroadcast", "ncclSend", "ncclRecv", "ncclGroupStart"):
        assert hasattr(h, name)
    assert rccl.version() >= 20000
