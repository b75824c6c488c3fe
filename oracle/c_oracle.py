"""ctypes wrapper of oracle/build/liboracle_p265.so (C restatement of the oracle).

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg.
"""
import ctypes
import os

import numpy as np

from p265_amd import records as R
from p265_amd._lib import Params, PictureC  # struct layouts only (libp265r is not loaded)

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "liboracle_p265.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise FileNotFoundError("%s not built: run `make -C oracle`" % LIB)
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_decode.restype = ctypes.c_int
        _lib.oracle_decode.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(PictureC), ctypes.c_int, ctypes.c_int]
        _lib.oracle_decode_sl.restype = ctypes.c_int
        _lib.oracle_decode_sl.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.POINTER(PictureC), ctypes.c_int,
                                          ctypes.c_int]
    return _lib


def decode(params, pics, threads=0, with_recon=True, scaling=None):
    """[(recon planes, out planes)] for each picture, computed by the C oracle.  Pictures with a
    size of their own (Picture.size, a ragged batch) are decoded with their own parameter set.
    ``scaling``: the 2032-byte intra ScalingFactor array when params.scaling_list_enabled."""
    groups = {}
    for i, p in enumerate(pics):
        pp = R.pic_params(params, p)
        groups.setdefault(pp.tobytes(), (pp, []))[1].append(i)
    if len(groups) > 1 or (groups and next(iter(groups.values()))[0] is not params):
        res = [None] * len(pics)
        for pp, idx in groups.values():
            for i, r in zip(idx, _decode(pp, [pics[i] for i in idx], threads, with_recon, scaling)):
                res[i] = r
        return res
    return _decode(params, pics, threads, with_recon, scaling)


def _decode(params, pics, threads, with_recon, scaling=None):
    lib = load()
    pc = Params()
    for name, _ in Params._fields_:
        if name != "reserved":
            setattr(pc, name, int(params[name]))
    w, h = int(params["pic_width"]), int(params["pic_height"])
    shapes = [(h, w), (h // 2, w // 2), (h // 2, w // 2)]
    arr = (PictureC * len(pics))()
    keep, res = [], []
    for i, p in enumerate(pics):
        ctus = np.ascontiguousarray(p.ctus, R.CTU_DTYPE)
        tbs = np.ascontiguousarray(p.tbs, R.TB_DTYPE)
        coef = np.ascontiguousarray(p.coef, np.int16)
        keep += [ctus, tbs, coef]
        a = arr[i]
        a.ctus, a.tbs, a.n_tbs = ctus.ctypes.data, tbs.ctypes.data, len(tbs)
        a.coef, a.n_coef = (coef.ctypes.data if len(coef) else None), len(coef)
        if p.nofilter is not None:
            nf = np.ascontiguousarray(p.nofilter, np.uint8)
            keep.append(nf)
            a.nofilter = nf.ctypes.data
        dts = R.plane_dtypes(params)
        rec = [np.zeros(s, dt) for s, dt in zip(shapes, dts)]
        out = [np.zeros(s, dt) for s, dt in zip(shapes, dts)]
        for k in range(3):
            a.out[k] = out[k].ctypes.data
            if with_recon:
                a.recon[k] = rec[k].ctypes.data
        res.append((rec, out))
    sf = None if scaling is None else np.ascontiguousarray(scaling, np.uint8)
    if sf is not None and sf.size != 2032:
        raise ValueError("scaling factors: 2032 bytes expected, got %d" % sf.size)
    rc = lib.oracle_decode_sl(ctypes.byref(pc), None if sf is None else sf.ctypes.data, arr, len(pics), int(threads))
    if rc:
        raise RuntimeError("oracle_decode failed: %d" % rc)
    return res
