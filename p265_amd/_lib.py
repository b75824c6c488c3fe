"""ctypes binding of libp265r.so (the C ABI in include/p265r.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) and loaded from
``p265_amd/libp265r.so``.  There is no fallback: if the library is missing or fails to
load, every entry point raises ``LibraryNotFound`` -- the product path never silently
degrades to a CPU implementation.

The product path does not use PyTorch: libp265r.so binds the system HIP runtime
(RUNPATH /opt/rocm-7.2.0/lib), the same file p265_amd/hip.py and p265_amd/rccl.py load.
A host that also uses PyTorch must load torch BEFORE this library (the torch wheel
bundles its own libamdhip64 under another file name; imported first, the dynamic linker
binds libp265r.so to that one runtime instead of loading a second).
"""
import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("P265R_LIB", os.path.join(HERE, "libp265r.so"))

DIGEST_SLOTS = 64                # P265R_DIGEST_SLOTS
SCALING_FACTOR_BYTES = 2032      # P265R_SCALING_FACTOR_BYTES

# error codes (include/p265r.h)
OK, EINVAL, ENOMEM, EHIP, EUNSUPPORTED, ERANGE, ESTATE, ENODEV = 0, -1, -2, -3, -4, -5, -6, -7


class LibraryNotFound(RuntimeError):
    pass


class P265RError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = "%s failed: %s (%d)" % (what, strerror(code), code)
        hip = last_hip_error()
        if hip:
            msg += " [%s]" % hip
        super().__init__(msg)


class Params(ctypes.Structure):
    _fields_ = [("version", ctypes.c_uint32), ("pic_width", ctypes.c_uint16), ("pic_height", ctypes.c_uint16),
                ("chroma_format_idc", ctypes.c_uint8), ("bit_depth_luma", ctypes.c_uint8),
                ("bit_depth_chroma", ctypes.c_uint8), ("ctb_log2_size", ctypes.c_uint8),
                ("min_tb_log2_size", ctypes.c_uint8), ("max_tb_log2_size", ctypes.c_uint8),
                ("strong_intra_smoothing", ctypes.c_uint8), ("constrained_intra_pred", ctypes.c_uint8),
                ("sample_adaptive_offset", ctypes.c_uint8), ("loop_filter_across_tiles", ctypes.c_uint8),
                ("scaling_list_enabled", ctypes.c_uint8), ("pps_cb_qp_offset", ctypes.c_int8),
                ("pps_cr_qp_offset", ctypes.c_int8), ("reserved", ctypes.c_uint8 * 11)]


class PictureC(ctypes.Structure):
    _fields_ = [("ctus", ctypes.c_void_p), ("tbs", ctypes.c_void_p), ("n_tbs", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("coef", ctypes.c_void_p), ("n_coef", ctypes.c_uint64),
                ("nofilter", ctypes.c_void_p), ("out", ctypes.c_void_p * 3), ("recon", ctypes.c_void_p * 3),
                ("pic_width", ctypes.c_uint16), ("pic_height", ctypes.c_uint16), ("reserved", ctypes.c_uint32)]


class Timings(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("residual_ms", ctypes.c_double), ("intra_ms", ctypes.c_double),
                ("sao_ms", ctypes.c_double), ("intra_launches", ctypes.c_int32),
                ("residual_launches", ctypes.c_int32), ("sao_launches", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


assert ctypes.sizeof(Params) == 32 and ctypes.sizeof(PictureC) == 104

# every symbol include/p265r.h declares, with (restype, argtypes)
_vp = ctypes.c_void_p
SIGNATURES = {
    "p265r_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(Params), ctypes.POINTER(_vp)]),
    "p265r_destroy": (None, [_vp]),
    "p265r_batch_upload": (ctypes.c_int, [_vp, ctypes.POINTER(PictureC), ctypes.c_int, ctypes.POINTER(_vp)]),
    "p265r_batch_run": (ctypes.c_int, [_vp, _vp]),
    "p265r_batch_download": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(PictureC), ctypes.c_int]),
    "p265r_batch_status": (ctypes.c_int, [_vp, _vp]),
    "p265r_batch_digest": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "p265r_batch_digest_async": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int]),
    "p265r_batch_digest_slots": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "p265r_batch_job_count": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "p265r_batch_free": (ctypes.c_int, [_vp, _vp]),
    "p265r_submit": (ctypes.c_int, [_vp, ctypes.POINTER(PictureC), ctypes.c_int]),
    "p265r_wait": (ctypes.c_int, [_vp]),
    "p265r_sync": (ctypes.c_int, [_vp]),
    "p265r_set_pipeline": (ctypes.c_int, [_vp, ctypes.c_int]),
    "p265r_set_row_waves": (ctypes.c_int, [_vp, ctypes.c_int]),
    "p265r_set_scaling_factors": (ctypes.c_int, [_vp, ctypes.c_void_p, ctypes.c_int]),
    "p265r_set_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "p265r_last_timings": (ctypes.c_int, [_vp, ctypes.POINTER(Timings)]),
    "p265r_timings_total": (ctypes.c_int, [_vp, ctypes.POINTER(Timings), ctypes.POINTER(ctypes.c_int)]),
    "p265r_device_count": (ctypes.c_int, []),
    "p265r_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "p265r_last_hip_error": (ctypes.c_char_p, []),
    "p265r_abi_version": (ctypes.c_uint32, []),
    "p265r_describe": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load libp265r.so once; raise LibraryNotFound (never fall back)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise LibraryNotFound("%s not built: run `make` or __graft_entry__.build()" % LIB_PATH)
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise LibraryNotFound("cannot load %s: %s" % (LIB_PATH, e))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.p265r_abi_version() != 2:
            raise LibraryNotFound("ABI version mismatch")
        _lib = lib
        return lib


def strerror(code):
    try:
        return load().p265r_strerror(code).decode()
    except LibraryNotFound:
        return "error %d" % code


def last_hip_error():
    try:
        return load().p265r_last_hip_error().decode()
    except LibraryNotFound:
        return ""


def check(code, what):
    if code < 0:
        raise P265RError(code, what)
    return code
