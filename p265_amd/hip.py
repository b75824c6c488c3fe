"""Minimal ctypes binding of the HIP runtime (libamdhip64.so.7 of /opt/rocm).

The product path is PyTorch-free (BASELINE north_star: "no PyTorch"): libp265r.so links
the system HIP runtime by RUNPATH (/opt/rocm-7.2.0/lib), and this module binds the SAME
shared object, so one process holds one HIP runtime.  Used for the device buffers of the
RCCL communicator (p265_amd/rccl.py) and for bench.py's device-copy bandwidth probe.
(Keep PyTorch out of a process that uses this: the torch wheel bundles its own
libamdhip64 under another file name, which would load a second runtime.)
"""
import ctypes
import os

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

H2D, D2H, D2D = 1, 2, 3          # hipMemcpyKind


class HipError(RuntimeError):
    pass


_hip = None


def lib():
    """Load libamdhip64.so.7 once (the file libp265r.so's RUNPATH resolves)."""
    global _hip
    if _hip is None:
        cands = [os.path.join(ROCM, "lib", "libamdhip64.so.7"), "libamdhip64.so.7"]
        err = None
        for c in cands:
            try:
                h = ctypes.CDLL(c, mode=ctypes.RTLD_GLOBAL)
                break
            except OSError as e:
                err = e
        else:
            raise HipError("cannot load libamdhip64.so.7: %s" % err)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        sig = {
            "hipGetDeviceCount": [ctypes.POINTER(ctypes.c_int)],
            "hipSetDevice": [ctypes.c_int],
            "hipMalloc": [ctypes.POINTER(vp), sz],
            "hipFree": [vp],
            "hipMemcpy": [vp, vp, sz, ctypes.c_int],
            "hipMemcpyAsync": [vp, vp, sz, ctypes.c_int, vp],
            "hipMemset": [vp, ctypes.c_int, sz],
            "hipStreamCreate": [ctypes.POINTER(vp)],
            "hipStreamDestroy": [vp],
            "hipStreamSynchronize": [vp],
            "hipDeviceSynchronize": [],
            "hipEventCreate": [ctypes.POINTER(vp)],
            "hipEventDestroy": [vp],
            "hipEventRecord": [vp, vp],
            "hipEventSynchronize": [vp],
            "hipEventElapsedTime": [ctypes.POINTER(ctypes.c_float), vp, vp],
            "hipHostMalloc": [ctypes.POINTER(vp), sz, ctypes.c_uint],
            "hipHostFree": [vp],
        }
        for name, args in sig.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        h.hipGetErrorString.argtypes = [ctypes.c_int]
        h.hipGetErrorString.restype = ctypes.c_char_p
        _hip = h
    return _hip


def check(rc, what):
    if rc != 0:
        raise HipError("%s failed: %s (%d)" % (what, lib().hipGetErrorString(rc).decode(), rc))


def device_count():
    n = ctypes.c_int(0)
    rc = lib().hipGetDeviceCount(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_device(d):
    check(lib().hipSetDevice(int(d)), "hipSetDevice")


def synchronize():
    check(lib().hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceBuffer:
    """hipMalloc'd bytes on the current device."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = ctypes.c_void_p()
        check(lib().hipMalloc(ctypes.byref(self.ptr), max(1, self.nbytes)), "hipMalloc(%d)" % self.nbytes)

    def upload(self, data: bytes):
        assert len(data) <= self.nbytes
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        check(lib().hipMemcpy(self.ptr, buf, len(data), H2D), "hipMemcpy H2D")

    def download(self, n=None) -> bytes:
        n = self.nbytes if n is None else int(n)
        buf = ctypes.create_string_buffer(max(1, n))
        check(lib().hipMemcpy(buf, self.ptr, n, D2H), "hipMemcpy D2H")
        return buf.raw[:n]

    def free(self):
        if self.ptr:
            lib().hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self):
        self.handle = ctypes.c_void_p()
        check(lib().hipStreamCreate(ctypes.byref(self.handle)), "hipStreamCreate")

    def synchronize(self):
        check(lib().hipStreamSynchronize(self.handle), "hipStreamSynchronize")

    def destroy(self):
        if self.handle:
            lib().hipStreamDestroy(self.handle)
            self.handle = ctypes.c_void_p()


def copy_bandwidth_gbs(device, nbytes=4 << 30, reps=10):
    """Achievable HBM bandwidth: device-to-device hipMemcpyAsync (read + write bytes / time),
    timed with HIP events on one stream."""
    h = lib()
    set_device(device)
    a, b = DeviceBuffer(nbytes), DeviceBuffer(nbytes)
    st = Stream()
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    check(h.hipEventCreate(ctypes.byref(e0)), "hipEventCreate")
    check(h.hipEventCreate(ctypes.byref(e1)), "hipEventCreate")
    try:
        check(h.hipMemset(a.ptr, 1, nbytes), "hipMemset")
        check(h.hipMemcpyAsync(b.ptr, a.ptr, nbytes, D2D, st.handle), "hipMemcpyAsync")
        st.synchronize()
        check(h.hipEventRecord(e0, st.handle), "hipEventRecord")
        for _ in range(reps):
            check(h.hipMemcpyAsync(b.ptr, a.ptr, nbytes, D2D, st.handle), "hipMemcpyAsync")
        check(h.hipEventRecord(e1, st.handle), "hipEventRecord")
        check(h.hipEventSynchronize(e1), "hipEventSynchronize")
        ms = ctypes.c_float()
        check(h.hipEventElapsedTime(ctypes.byref(ms), e0, e1), "hipEventElapsedTime")
        return round(2 * nbytes * reps / (ms.value * 1e-3) / 1e9, 1)
    finally:
        h.hipEventDestroy(e0)
        h.hipEventDestroy(e1)
        st.destroy()
        a.free()
        b.free()


def pinned_copy_gbs(device, nbytes=1 << 30, reps=5):
    """Host <-> device copy rates from pinned host memory (hipHostMalloc + hipMemcpyAsync, HIP events):
    the PCIe ceiling of the back-end's uploads and downloads.  GB/s per direction."""
    h = lib()
    set_device(device)
    host = ctypes.c_void_p()
    check(h.hipHostMalloc(ctypes.byref(host), nbytes, 0), "hipHostMalloc")
    dev = DeviceBuffer(nbytes)
    st = Stream()
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    check(h.hipEventCreate(ctypes.byref(e0)), "hipEventCreate")
    check(h.hipEventCreate(ctypes.byref(e1)), "hipEventCreate")
    out = {}
    try:
        ctypes.memset(host, 1, nbytes)
        for name, dst, src, kind in (("h2d_gbs", dev.ptr, host, H2D), ("d2h_gbs", host, dev.ptr, D2H)):
            check(h.hipMemcpyAsync(dst, src, nbytes, kind, st.handle), "hipMemcpyAsync")
            st.synchronize()
            check(h.hipEventRecord(e0, st.handle), "hipEventRecord")
            for _ in range(reps):
                check(h.hipMemcpyAsync(dst, src, nbytes, kind, st.handle), "hipMemcpyAsync")
            check(h.hipEventRecord(e1, st.handle), "hipEventRecord")
            check(h.hipEventSynchronize(e1), "hipEventSynchronize")
            ms = ctypes.c_float()
            check(h.hipEventElapsedTime(ctypes.byref(ms), e0, e1), "hipEventElapsedTime")
            out[name] = round(nbytes * reps / (ms.value * 1e-3) / 1e9, 2)
        return out
    finally:
        h.hipEventDestroy(e0)
        h.hipEventDestroy(e1)
        st.destroy()
        dev.free()
        h.hipHostFree(host)
