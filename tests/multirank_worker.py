#!/usr/bin/env python3
"""One rank of the multi-process product-path test (tests/test_a_multirank.py, GPU box).

Started as a child process per rank by the test (never exec'd from a process that touched
the GPU), with the launcher environment torch.distributed.run would set (RANK, WORLD_SIZE,
MASTER_ADDR; P265_CTRL_PORT for the socket control plane).  Every rank decodes through
libp265r.so on HIP device ``--device`` (both ranks share device 0 on a one-GPU box, so the
group has no RCCL communicator: two RCCL ranks cannot share a device; the params and
halos then travel over the control plane, the same bytes ncclBroadcast / ncclSend carry on
an 8-GPU node):

* C4: picture f -> rank f mod N (dist.frame_shard), params broadcast from rank 0, SHA-256
  digests of the decoded planes gathered on every rank;
* C5: (picture, tile) units of tests/golden/synth_4k_tiles.bin (parsed by the native
  front-end on every rank) -> ranks (dist.unit_shard), each tile decoded as its own
  sub-picture; planes written to OUT/c5_<f>_<t>.npy for the parent to stitch and check
  against the stream's MD5 SEI;
* C5 with loop_filter_across_tiles_enabled_flag = 1: every rank reconstructs its tiles,
  the halos go point to point (dist.exchange), every rank filters its extended tiles;
  outputs to OUT/halo_<t>.npy.

Rank 0 writes OUT/result.json.
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from p265_amd import bitstream, dist, halo, recon, synth, tiles  # noqa: E402
from p265_amd import records as R  # noqa: E402


def c4(device, rank, world):
    params = R.make_params(pic_width=320, pic_height=192) if rank == 0 else R.make_params()
    params = dist.broadcast_params(params)
    mine = dist.frame_shard(6, rank, world)
    pics = [synth.make_picture(params, 900 + f) for f in mine]
    with recon.ReconContext(params, device=device) as ctx:
        outs = ctx.decode(pics)
    dig = [(f, hashlib.sha256(b"".join(np.ascontiguousarray(o[c]).tobytes() for c in range(3))).hexdigest())
           for f, o in zip(mine, outs)]
    return dist.gather_digests(dig), int(params["pic_width"])


def c5(device, rank, world, out):
    pics = bitstream.decode_stream(open(os.path.join(ROOT, "tests", "golden", "synth_4k_tiles.bin"), "rb").read())
    params = dist.broadcast_params(pics[0].params)
    done = []
    units = dist.unit_shard(len(pics), 4, rank, world)
    by_params = {}
    for f, t in units:
        tp, tpic, _ = tiles.split(params, pics[f].picture)[t]
        by_params.setdefault(tp.tobytes(), (tp, []))[1].append(((f, t), tpic))
    for tp, items in by_params.values():
        with recon.ReconContext(tp, device=device) as ctx:
            outs = ctx.decode([p for _, p in items])
        for ((f, t), _), planes in zip(items, outs):
            np.savez(os.path.join(out, "c5_%d_%d.npz" % (f, t)), *planes)
            done.append(("%d/%d" % (f, t), rank))
    return dist.gather_digests(done)


def c5_halo(device, rank, world, out):
    params = R.make_params(pic_width=264, pic_height=200, ctb_log2_size=5, loop_filter_across_tiles=1,
                           pps_cb_qp_offset=2, pps_cr_qp_offset=-1)
    pic = synth.make_picture(params, 77, perf=False, tiles=(2, 2), n_slices=3, lf_across_slices=None,
                             deblocking="random", bypass_rate=0.04, pcm_rate=0.02)
    grid = halo.TileGrid.from_picture(params, pic)
    owner = {t: t % world for t in range(grid.n_tiles)}
    parts = tiles.split(params, pic, recon_only=True)
    mine = {}
    for t, (tp, tpic, _) in enumerate(parts):
        if owner[t] != rank:
            continue
        with recon.ReconContext(tp, device=device) as ctx:
            d = halo.TileData(grid, pic, t)
            d.recon = ctx.decode([tpic])[0]                # recon-only pass: out = reconstruction
        mine[t] = d
    sends, recvs = [], []
    for t, d in mine.items():
        for n in grid.neighbours(t):
            if owner[n] != rank:
                recvs.append((owner[n], n * 100 + t))
        for dst in range(grid.n_tiles):
            if t in grid.neighbours(dst) and owner[dst] != rank:
                sends.append((owner[dst], t * 100 + dst, d.halo_for(dst)))
    got = halo.exchange(sends, recvs)
    for t, d in mine.items():
        payloads = [mine[n].halo_for(t) if owner[n] == rank else got[n * 100 + t] for n in grid.neighbours(t)]
        ep, epic, origin, inner = halo.ext_picture(params, grid, d, payloads)
        with recon.ReconContext(ep, device=device) as ctx:
            planes = halo.crop_inner(ctx.decode([epic])[0], origin, inner)
        np.savez(os.path.join(out, "halo_%d.npz" % t), *planes)
    return dist.gather_digests([(str(t), rank) for t in mine])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    rank, world, _ = dist.init(rccl=False)
    try:
        c4_digests, width = c4(a.device, rank, world)
        c5_units = c5(a.device, rank, world, a.out)
        halo_units = c5_halo(a.device, rank, world, a.out)
        dist.barrier()
        if rank == 0:
            json.dump({"world": world, "width": width, "c4": {str(k): v for k, v in c4_digests.items()},
                       "c5": c5_units, "halo": halo_units}, open(os.path.join(a.out, "result.json"), "w"))
    finally:
        dist.finalize()


if __name__ == "__main__":
    main()
