"""Sharding logic of the multi-GPU path, on CPU: tile sub-pictures (C5) and a
world_size-2 gloo run of frame sharding (C4) with the params broadcast.  The decode
inside the ranks uses the C oracle (no GPU here); on the MI355X box bench.py runs the
same shard plan through libp265r.so with the nccl (RCCL) backend."""
import os
import socket

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


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import hashlib
    import torch.distributed as tdist
    tdist.init_process_group("gloo")
    params = R.make_params(pic_width=192, pic_height=128) if rank == 0 else R.make_params()   # ranks disagree...
    params = dist.broadcast_params(params)                                                      # ...until broadcast
    mine = dist.frame_shard(6, rank, world)
    pics = [synth.make_picture(params, 900 + f) for f in mine]
    outs = c_oracle.decode(params, pics)
    dig = [(f, hashlib.sha256(b"".join(o[1][c].tobytes() for c in range(3))).hexdigest()) for f, o in zip(mine, outs)]
    merged = dist.gather_digests(dig)
    t = dist.max_over_ranks(float(rank + 1))
    if rank == 0:
        np.save(os.path.join(out_dir, "result.npy"), np.array([len(merged), t, int(params["pic_width"])]))
        import json
        json.dump(merged, open(os.path.join(out_dir, "digests.json"), "w"))
    tdist.destroy_process_group()


def test_gloo_world2_frame_sharding(tmp_path):
    import json
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    n, t, width = np.load(tmp_path / "result.npy")
    assert (n, t, width) == (6, 2.0, 192)
    merged = json.load(open(tmp_path / "digests.json"))
    import hashlib
    params = R.make_params(pic_width=192, pic_height=128)
    ref = c_oracle.decode(params, [synth.make_picture(params, 900 + f) for f in range(6)])
    for f in range(6):
        assert merged[str(f)] == hashlib.sha256(b"".join(ref[f][1][c].tobytes() for c in range(3))).hexdigest()
