"""Multi-GPU sharding (one process per GPU, torch.distributed over RCCL/xGMI).

The path shards naturally: all-intra pictures are independent
(each slice re-initialises CABAC, decoder/slice.py:244-245) and tiles are independent
for prediction (availability stops at tile edges, decoder/image.py:65-71).  So:

* C4: picture f -> rank f mod world (``frame_shard``), no data-path collective;
* C5: (picture, tile) units -> ranks (``unit_shard``), each tile decoded as its own
  sub-picture (p265_amd/tiles.py) when loop_filter_across_tiles_enabled_flag == 0;
* the only collective is ``broadcast_params``: the 32-byte SPS/PPS POD from rank 0,
  once per stream (RCCL broadcast over xGMI when the backend is "nccl").

Timing helpers follow the bench contract: barrier, then MAX of elapsed over ranks.
"""
import os

import numpy as np

from . import records as R


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend="nccl"):
    """Initialise torch.distributed from the torchrun environment; returns (rank, world, local)."""
    import torch
    import torch.distributed as dist
    rank, world, local = env_ranks()
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend)
    return rank, world, local


def _device(backend):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def broadcast_params(params, src=0):
    """Broadcast the params POD (records.PARAMS_DTYPE) from ``src`` to every rank."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return params
    backend = dist.get_backend()
    buf = np.zeros(R.PARAMS_DTYPE.itemsize, np.uint8)
    if dist.get_rank() == src:
        buf[:] = np.frombuffer(np.asarray(params, R.PARAMS_DTYPE).tobytes(), np.uint8)
    t = torch.from_numpy(buf).to(_device(backend))
    dist.broadcast(t, src=src)
    out = np.frombuffer(t.cpu().numpy().tobytes(), R.PARAMS_DTYPE)[0]
    if int(out["version"]) != R.ABI_VERSION:
        raise RuntimeError("broadcast params: ABI version mismatch")
    return out


def frame_shard(n_frames, rank, world):
    """C4: picture f is decoded by rank f mod world."""
    return list(range(rank, n_frames, world))


def unit_shard(n_frames, n_tiles, rank, world):
    """C5: (picture, tile) units in picture-major order, dealt round-robin to ranks."""
    units = [(f, t) for f in range(n_frames) for t in range(n_tiles)]
    return units[rank::world]


def max_over_ranks(value):
    """MAX of a float over ranks (the bench's job time)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([float(value)], dtype=torch.float64, device=_device(dist.get_backend()))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def gather_digests(digests):
    """all_gather of per-rank lists of (unit id, 32-byte digest) -> dict on every rank."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(digests)
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, list(digests))
    merged = {}
    for part in out:
        merged.update(dict(part))
    return merged
