"""Multi-GPU sharding: one process per GPU, RCCL over xGMI through ctypes (no PyTorch).

The path shards naturally: all-intra pictures are independent
(each slice re-initialises CABAC, decoder/slice.py:244-245) and tiles are independent
for prediction (availability stops at tile edges, decoder/image.py:65-71).  So:

* C4: picture f -> rank f mod world (``frame_shard``), no data-path collective;
* C5: (picture, tile) units -> ranks (``unit_shard``), each tile decoded as its own
  sub-picture (p265_amd/tiles.py) when loop_filter_across_tiles_enabled_flag == 0;
  with the flag at 1, tile halos go point to point (``exchange``: ncclSend / ncclRecv);
* the only collective is ``broadcast_params``: the 32-byte SPS/PPS POD from rank 0,
  once per stream (ncclBroadcast over xGMI when the group has an RCCL communicator).

Ranks meet over the socket control plane of p265_amd/comm.py (RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR / MASTER_PORT as torch.distributed.run sets them), which also
carries the RCCL unique id, the barriers and the MAX over ranks of the bench timing.
Without a GPU (CPU tests) the group has no RCCL communicator and the bytes of the params
and halos travel over the control plane instead.
"""
import os
import struct

import numpy as np

from . import records as R
from .comm import SocketComm


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


class Group:
    def __init__(self, rank, world, local, ctrl, nccl=None):
        self.rank, self.world, self.local = rank, world, local
        self.ctrl, self.nccl = ctrl, nccl

    def close(self):
        if self.nccl is not None:
            self.nccl.close()
            self.nccl = None
        self.ctrl.close()


_group = None


def init(device=None, rccl=None):
    """Join the process group from the launcher's environment; returns (rank, world, local).

    ``device``: HIP device of this rank for the RCCL communicator (default LOCAL_RANK when
    ``rccl``).  ``rccl``: None = only when world > 1; True = always (also world 1: a
    one-rank communicator); False = control plane only (CPU)."""
    global _group
    rank, world, local = env_ranks()
    if _group is not None:
        return _group.rank, _group.world, _group.local
    ctrl = SocketComm.from_env()
    nccl = None
    if rccl is None:
        rccl = world > 1
    if rccl:
        from .rccl import Rccl
        nccl = Rccl(rank, world, local if device is None else device, ctrl)
    _group = Group(rank, world, local, ctrl, nccl)
    return rank, world, local


def group():
    return _group


def finalize():
    global _group
    if _group is not None:
        _group.close()
        _group = None


def allgather_json(obj):
    """Every rank's JSON-able ``obj`` -> the list over ranks (control plane), on every rank."""
    import json
    g = _group
    if g is None or g.world == 1:
        return [obj]
    return [json.loads(p.decode()) for p in g.ctrl.allgather(json.dumps(obj).encode())]


def rccl_ranks():
    """ncclCommCount of every rank's communicator (the ranks RCCL itself sees), gathered over the control
    plane; None when the group has no RCCL communicator (CPU, --no-rccl)."""
    g = _group
    if g is None:
        return None
    mine = g.nccl.count() if g.nccl is not None else None
    got = allgather_json(mine)
    return None if all(c is None for c in got) else got


def broadcast_params(params, src=0):
    """Broadcast the params POD (records.PARAMS_DTYPE) from ``src`` to every rank:
    ncclBroadcast of its 32 bytes on a hipMalloc'd buffer, or over the control plane."""
    g = _group
    if g is None or (g.world == 1 and g.nccl is None):
        return params
    raw = np.asarray(params, R.PARAMS_DTYPE).tobytes() if g.rank == src else b""
    if g.nccl is not None:
        out = g.nccl.broadcast(raw, root=src, nbytes=R.PARAMS_DTYPE.itemsize)
    else:
        out = g.ctrl.bcast(raw, src=src)
    p = np.frombuffer(out, R.PARAMS_DTYPE)[0]
    if int(p["version"]) != R.ABI_VERSION:
        raise RuntimeError("broadcast params: ABI version mismatch")
    return p


def frame_shard(n_frames, rank, world):
    """C4: picture f is decoded by rank f mod world."""
    return list(range(rank, n_frames, world))


def unit_shard(n_frames, n_tiles, rank, world):
    """C5: (picture, tile) units in picture-major order, dealt round-robin to ranks."""
    units = [(f, t) for f in range(n_frames) for t in range(n_tiles)]
    return units[rank::world]


def max_over_ranks(value):
    """MAX of a float over ranks (the bench's job time)."""
    g = _group
    if g is None or g.world == 1:
        return value
    return g.ctrl.max(value)


def barrier():
    g = _group
    if g is not None and g.world > 1:
        g.ctrl.barrier()


def gather_digests(digests):
    """Every rank's list of (unit id, digest) -> one dict on every rank (control plane).

    Contract: unit ids are str or int, digests str (hex), int or a list of str -- the list
    travels as JSON, so anything else (bytes, tuples) is rejected here rather than silently
    changed."""
    import json
    for k, v in digests:
        ok_v = isinstance(v, (str, int)) or (isinstance(v, list) and all(isinstance(x, str) for x in v))
        if not isinstance(k, (str, int)) or not ok_v:
            raise TypeError("gather_digests: unit ids and digests must be str or int, got %r: %r" % (k, v))
    g = _group
    if g is None or g.world == 1:
        return dict(digests)
    merged = {}
    for part in g.ctrl.allgather(json.dumps([[k, v] for k, v in digests]).encode()):
        merged.update({k: v for k, v in json.loads(part.decode())})
    return merged


def exchange(sends, recvs):
    """sends: [(dst_rank, tag, bytes)], recvs: [(src_rank, tag)] -> {tag: bytes}.

    The payload sizes go over the control plane, the payloads point to point with RCCL
    (ncclSend / ncclRecv, one group) when the group has a communicator, else over the
    control plane too.  Several messages between one pair of ranks are concatenated in tag
    order."""
    g = _group
    by_dst = {}
    for dst, tag, data in sorted(sends, key=lambda s: (s[0], s[1])):
        by_dst.setdefault(int(dst), []).append((int(tag), bytes(data)))
    heads = {d: struct.pack("<I", len(m)) + b"".join(struct.pack("<qQ", t, len(b)) for t, b in m)
             for d, m in by_dst.items()}
    if g.nccl is not None:
        got_heads = g.ctrl.alltoall(heads)
        sizes = {}
        for src, h in got_heads.items():
            (n,) = struct.unpack_from("<I", h, 0)
            sizes[src] = sum(struct.unpack_from("<qQ", h, 4 + 16 * i)[1] for i in range(n))
        # zero-byte payloads are skipped on both sides (Rccl.exchange filters them too)
        payloads = g.nccl.exchange({d: p for d, p in ((d, b"".join(b for _, b in m)) for d, m in by_dst.items()) if p},
                                   {s: n for s, n in sizes.items() if n})
    else:
        got = g.ctrl.alltoall({d: heads[d] + b"".join(b for _, b in m) for d, m in by_dst.items()})
        got_heads, payloads = {}, {}
        for src, blob in got.items():
            (n,) = struct.unpack_from("<I", blob, 0)
            hl = 4 + 16 * n
            got_heads[src], payloads[src] = blob[:hl], blob[hl:]
    out = {}
    for src, h in got_heads.items():
        (n,) = struct.unpack_from("<I", h, 0)
        off = 0
        for i in range(n):
            tag, ln = struct.unpack_from("<qQ", h, 4 + 16 * i)
            out[tag] = payloads.get(src, b"")[off:off + ln]
            off += ln
    want = {int(t) for _, t in recvs}
    missing = want - set(out)
    if missing:
        raise RuntimeError("exchange: no message for tags %s" % sorted(missing))
    return {t: out[t] for t in want}
