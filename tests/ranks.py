"""Multi-process helpers for the N>1 tests: spawn `world` rank processes that join the
socket control plane of p265_amd.comm (the launcher environment torch.distributed.run
would set: RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR, plus P265_CTRL_PORT) and collect
one picklable result per rank."""
import multiprocessing as mp
import os
import socket
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(fn, rank, world, port, args, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      P265_CTRL_PORT=str(port))
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from p265_amd import dist
    try:
        dist.init(rccl=False)
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
    except BaseException:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "error", traceback.format_exc()))
    finally:
        dist.finalize()


def run_ranks(fn, world, *args, timeout=240):
    """fn(rank, world, *args) in `world` spawned processes -> {rank: result}; raises on any error."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out, errors = {}, []
    try:
        for _ in procs:
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                errors.append("rank %d:\n%s" % (rank, res))
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errors:
        raise AssertionError("\n".join(errors))
    return out
