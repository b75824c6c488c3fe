"""ctypes binding of RCCL (librccl.so.1 of /opt/rocm): the xGMI collectives of the
multi-GPU path, without PyTorch.

SURVEY §8(e): the path shards with no data-path collective; the one collective is the
broadcast of the 32-byte SPS/PPS POD (p265r_params) from rank 0 at stream start, and, for
C5 with loop_filter_across_tiles_enabled_flag = 1, a point-to-point exchange of tile
halos (ncclSend / ncclRecv inside one group).  The RCCL unique id travels over the
socket control plane (p265_amd/comm.py): ncclGetUniqueId on rank 0 -> broadcast of the
128 bytes -> ncclCommInitRank on every rank.
"""
import ctypes
import os

from . import hip

ncclUint8, ncclInt64, ncclFloat64 = 1, 4, 8
ncclSum, ncclMax = 0, 2


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


class RcclError(RuntimeError):
    pass


_nccl = None


def lib():
    global _nccl
    if _nccl is None:
        hip.lib()                                   # the same HIP runtime first
        path = os.path.join(hip.ROCM, "lib", "librccl.so.1")
        try:
            h = ctypes.CDLL(path if os.path.exists(path) else "librccl.so.1")
        except OSError as e:
            raise RcclError("cannot load librccl.so.1: %s" % e)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        sig = {
            "ncclGetUniqueId": [ctypes.POINTER(UniqueId)],
            "ncclCommInitRank": [ctypes.POINTER(vp), i, UniqueId, i],
            "ncclCommDestroy": [vp],
            "ncclCommCount": [vp, ctypes.POINTER(i)],
            "ncclBroadcast": [vp, vp, sz, i, i, vp, vp],
            "ncclAllReduce": [vp, vp, sz, i, i, vp, vp],
            "ncclSend": [vp, sz, i, i, vp, vp],
            "ncclRecv": [vp, sz, i, i, vp, vp],
            "ncclGroupStart": [],
            "ncclGroupEnd": [],
            "ncclGetVersion": [ctypes.POINTER(i)],
        }
        for name, args in sig.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        h.ncclGetErrorString.argtypes = [ctypes.c_int]
        h.ncclGetErrorString.restype = ctypes.c_char_p
        _nccl = h
    return _nccl


def check(rc, what):
    if rc != 0:
        raise RcclError("%s failed: %s (%d)" % (what, lib().ncclGetErrorString(rc).decode(), rc))


def version():
    v = ctypes.c_int(0)
    check(lib().ncclGetVersion(ctypes.byref(v)), "ncclGetVersion")
    return v.value


class Rccl:
    """One RCCL communicator per process (rank) on HIP device ``device``."""

    def __init__(self, rank, world, device, ctrl=None):
        self.rank, self.world, self.device = int(rank), int(world), int(device)
        h = lib()
        hip.set_device(self.device)
        uid = UniqueId()
        if self.rank == 0:
            check(h.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        if self.world > 1:
            if ctrl is None:
                raise RcclError("world > 1 needs a control plane for the unique id")
            raw = ctrl.bcast(bytes(uid.internal) if self.rank == 0 else b"")
            ctypes.memmove(ctypes.addressof(uid), raw, 128)
        self.comm = ctypes.c_void_p()
        check(h.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank), "ncclCommInitRank")
        self.stream = hip.Stream()

    def count(self):
        """ncclCommCount: the number of ranks in this communicator, as RCCL reports it."""
        n = ctypes.c_int(0)
        check(lib().ncclCommCount(self.comm, ctypes.byref(n)), "ncclCommCount")
        return n.value

    def broadcast(self, data: bytes, root=0, nbytes=None) -> bytes:
        """ncclBroadcast of a byte string from ``root`` (others pass b"" and ``nbytes``)."""
        n = len(data) if self.rank == root else int(nbytes)
        buf = hip.DeviceBuffer(n)
        try:
            if self.rank == root:
                buf.upload(data)
            check(lib().ncclBroadcast(buf.ptr, buf.ptr, n, ncclUint8, root, self.comm, self.stream.handle),
                  "ncclBroadcast")
            self.stream.synchronize()
            return buf.download(n)
        finally:
            buf.free()

    def exchange(self, sends, recv_sizes):
        """Point-to-point: sends {dst: bytes}, recv_sizes {src: nbytes} -> {src: bytes}; one
        ncclGroupStart/End around every ncclSend / ncclRecv (no ordering deadlock).

        Zero-byte messages are dropped on BOTH sides (an empty payload is neither sent nor
        received; its source maps to b""): RCCL matches a zero-byte ncclSend like any other, so
        posting it on one side only would pair it with a later exchange's receive."""
        h = lib()
        sends = {d: b for d, b in sends.items() if len(b)}
        empty = {s for s, n in recv_sizes.items() if not n}
        recv_sizes = {s: n for s, n in recv_sizes.items() if n}
        out_bufs, in_bufs = {}, {}
        try:
            for dst, data in sends.items():
                b = out_bufs[dst] = hip.DeviceBuffer(len(data))
                b.upload(data)
            for src, n in recv_sizes.items():
                in_bufs[src] = hip.DeviceBuffer(n)
            check(h.ncclGroupStart(), "ncclGroupStart")
            for dst, data in sorted(sends.items()):
                check(h.ncclSend(out_bufs[dst].ptr, len(data), ncclUint8, int(dst), self.comm, self.stream.handle),
                      "ncclSend")
            for src, n in sorted(recv_sizes.items()):
                check(h.ncclRecv(in_bufs[src].ptr, int(n), ncclUint8, int(src), self.comm, self.stream.handle),
                      "ncclRecv")
            check(h.ncclGroupEnd(), "ncclGroupEnd")
            self.stream.synchronize()
            out = {src: in_bufs[src].download(n) for src, n in recv_sizes.items()}
            out.update({src: b"" for src in empty})
            return out
        finally:
            for b in list(out_bufs.values()) + list(in_bufs.values()):
                b.free()

    def close(self):
        if self.comm:
            lib().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
        self.stream.destroy()
