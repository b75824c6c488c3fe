"""ctypes binding of libp265fe.so: the native HEVC syntax front-end (include/p265fe.h).

Replaces the reference's Python parse loop (dec.py:18-64 -> nalu.py -> slice.py ->
ctu.py / cu.py / tu.py / sao.py with the CABAC engine of cabac.py) for all-intra
streams.  ``decode_stream(data)`` parses a whole Annex-B byte stream on host threads
and returns, per picture in decode order, the back-end records that the reference's
per-CU hook would have produced (``records.Picture``) plus the picture's params,
POC, output rank, conformance window and decoded-picture hash.  ``StreamParser``
does the same incrementally: ``feed()`` arbitrary chunks, get the pictures completed
so far (bounded memory for arbitrarily long streams).

The record arrays are read-only zero-copy views of buffers the library owns; they
keep those buffers alive.  There is no fallback: a missing library raises
``LibraryNotFound``; a malformed or unsupported stream raises ``BitstreamError`` /
``UnsupportedStream``.
"""
import ctypes
import hashlib
import os
import threading
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from . import records as R

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("P265FE_LIB", os.path.join(HERE, "libp265fe.so"))

ABI_VERSION = 4
OK, EINVAL, ENOMEM, EUNSUPPORTED, EBITSTREAM = 0, -1, -2, -4, -8
HASH_NONE, HASH_MD5, HASH_CRC, HASH_CHECKSUM = -1, 0, 1, 2
FLUSH = 1
ASYNC = 2                       # p265fe_feed: P265FE_ASYNC


class BitstreamError(ValueError):
    pass


class UnsupportedStream(BitstreamError):
    pass


class PictureInfoC(ctypes.Structure):
    _fields_ = [("params", _lib.Params), ("ctus", ctypes.c_void_p), ("tbs", ctypes.c_void_p),
                ("n_tbs", ctypes.c_uint32), ("n_ctus", ctypes.c_uint32), ("coef", ctypes.c_void_p),
                ("n_coef", ctypes.c_uint64), ("nofilter", ctypes.c_void_p), ("poc", ctypes.c_int32),
                ("output_rank", ctypes.c_int32), ("crop_left", ctypes.c_uint16), ("crop_right", ctypes.c_uint16),
                ("crop_top", ctypes.c_uint16), ("crop_bottom", ctypes.c_uint16), ("nal_unit_type", ctypes.c_uint8),
                ("hash_type", ctypes.c_int8), ("n_slices", ctypes.c_uint16), ("n_cus", ctypes.c_uint32),
                ("hash", (ctypes.c_uint8 * 16) * 3), ("cvs_id", ctypes.c_int32),
                ("max_num_reorder", ctypes.c_uint8), ("output_flag", ctypes.c_uint8), ("reserved", ctypes.c_uint16),
                ("scaling_factors", ctypes.c_void_p)]


_vp = ctypes.c_void_p
SIGNATURES = {
    "p265fe_create": (ctypes.c_int, [ctypes.POINTER(_vp)]),
    "p265fe_destroy": (None, [_vp]),
    "p265fe_decode": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]),
    "p265fe_picture": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(PictureInfoC)]),
    "p265fe_feed": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]),
    "p265fe_take": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "p265fe_wait": (ctypes.c_int, [_vp, ctypes.c_int]),
    "p265fe_pictures_get": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(PictureInfoC)]),
    "p265fe_pictures_free": (None, [_vp]),
    "p265fe_last_error": (ctypes.c_char_p, [_vp]),
    "p265fe_abi_version": (ctypes.c_uint32, []),
    "p265fe_plane_hash": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_char_p]),
}

_lock = threading.Lock()
_handle = None


def load():
    global _handle
    with _lock:
        if _handle is None:
            if not os.path.exists(LIB_PATH):
                raise _lib.LibraryNotFound("%s not built (run `make` or __graft_entry__.build())" % LIB_PATH)
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            if lib.p265fe_abi_version() != ABI_VERSION:
                raise _lib.LibraryNotFound("libp265fe.so ABI version mismatch (rebuild)")
            _handle = lib
        return _handle


@dataclass
class DecodedPicture:
    """One picture of the stream: back-end records + stream-level metadata."""
    params: np.ndarray
    picture: R.Picture
    poc: int
    output_rank: int            # decode_stream: rank in output order (-1: not output); StreamParser: -1
    crop: tuple                 # conformance window (left, right, top, bottom) in luma samples
    nal_unit_type: int
    n_slices: int
    n_cus: int
    hash_type: int
    hash: Optional[list]        # per component bytes of the decoded picture hash SEI
    cvs_id: int = 0             # coded video sequence (IRAP with NoRaslOutputFlag) counter
    max_num_reorder: int = 0    # sps_max_num_reorder_pics of its SPS (output bumping, C.5.2.2)
    output_flag: bool = True    # PicOutputFlag
    scaling: Optional[np.ndarray] = None   # the 2032-byte intra ScalingFactor table (scaling_list_enabled)


class _Owner:
    """Destroys one p265fe_decoder when the last object referring to it goes away."""

    def __init__(self, lib, handle):
        self.lib, self.handle = lib, handle

    def __del__(self):
        if self.handle:
            self.lib.p265fe_destroy(self.handle)
            self.handle = None


class _SetOwner:
    """Frees one p265fe_pictures set when the last record array viewing it goes away."""

    def __init__(self, lib, handle):
        self.lib, self.handle = lib, handle

    def __del__(self):
        if self.handle:
            self.lib.p265fe_pictures_free(self.handle)
            self.handle = None


def _params_np(pc):
    kw = {name: getattr(pc, name) for name, _ in _lib.Params._fields_ if name not in ("version", "reserved")}
    return R.make_params(**kw)


def _view(ptr, n, dtype, owner):
    """Zero-copy numpy view of a library-owned buffer (no first-touch copy of the records)."""
    if n == 0:
        return np.zeros(0, dtype)
    buf = (ctypes.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    buf._p265fe_owner = owner
    return np.frombuffer(buf, dtype=dtype, count=n)


def plane_hash(plane, hash_type):
    """decoded_picture_hash value (D.3.19) of one uint8 or uint16 plane, as the SEI carries it.

    MD5 and CRC run over pictureData: the samples in raster order, one byte each at BitDepth 8 and
    two (little-endian) above (D.3.19), so a uint16 plane is hashed as its bytes (the CRC through
    p265fe_plane_hash on a row of 2W bytes).  MD5 comes from hashlib (no GIL, faster than the
    library's portable MD5).  The checksum sums per SAMPLE ((sample & 0xFF) ^ xorMask, plus
    (sample >> 8) ^ xorMask above 8 bits, D-23): p265fe_plane_hash at 8 bits, numpy above."""
    p = np.ascontiguousarray(plane)
    if p.dtype == np.uint16:
        p = p.astype("<u2", copy=False)
        if int(hash_type) == HASH_MD5:
            return hashlib.md5(memoryview(p).cast("B")).digest()
        if int(hash_type) == HASH_CRC:
            return plane_hash_native(p.view(np.uint8), hash_type)
        if int(hash_type) == HASH_CHECKSUM:
            h, w = p.shape
            x, y = np.arange(w, dtype=np.uint64), np.arange(h, dtype=np.uint64)[:, None]
            mask = (x & np.uint64(0xFF)) ^ (y & np.uint64(0xFF)) ^ (x >> np.uint64(8)) ^ (y >> np.uint64(8))
            v = p.astype(np.uint64)
            s = int((((v & np.uint64(0xFF)) ^ mask).sum() + ((v >> np.uint64(8)) ^ mask).sum())) & 0xFFFFFFFF
            return s.to_bytes(4, "big")
        raise ValueError("unknown hash type %r" % hash_type)
    p = np.ascontiguousarray(plane, np.uint8)
    if int(hash_type) == HASH_MD5:
        return hashlib.md5(memoryview(p).cast("B")).digest()
    return plane_hash_native(p, hash_type)


def plane_hash_native(plane, hash_type):
    """p265fe_plane_hash (the library's D.3.19 implementation for MD5, CRC and checksum)."""
    lib = load()
    p = np.ascontiguousarray(plane, np.uint8)
    out = ctypes.create_string_buffer(16)
    rc = lib.p265fe_plane_hash(p.ctypes.data, p.shape[1], p.shape[0], p.strides[0], int(hash_type), out)
    if rc != OK:
        raise ValueError("p265fe_plane_hash failed (%d)" % rc)
    return out.raw[:{HASH_MD5: 16, HASH_CRC: 2, HASH_CHECKSUM: 4}[int(hash_type)]]


def _fail(lib, h, n, what):
    msg = lib.p265fe_last_error(h).decode(errors="replace")
    cls = UnsupportedStream if n == EUNSUPPORTED else BitstreamError
    raise cls("%s: %s (%d)" % (what, msg, n))


def _collect(get, n, owner, validate, base=0):
    out = []
    info = PictureInfoC()
    for i in range(n):
        rc = get(i, ctypes.byref(info))
        if rc != OK:
            raise BitstreamError("picture %d: info failed (%d)" % (base + i, rc))
        params = _params_np(info.params)
        ctus = _view(info.ctus, info.n_ctus, R.CTU_DTYPE, owner)
        tbs = _view(info.tbs, info.n_tbs, R.TB_DTYPE, owner)
        coef = _view(info.coef, int(info.n_coef), np.int16, owner)
        nof = None
        if info.nofilter:
            w, hh = int(params["pic_width"]), int(params["pic_height"])
            nof = _view(info.nofilter, ((w + 7) // 8) * ((hh + 7) // 8), np.uint8, owner)
        for arr in (ctus, tbs, coef, nof):
            if arr is not None:
                arr.flags.writeable = False
        pic = R.Picture(ctus=ctus, tbs=tbs, coef=coef, nofilter=nof,
                        meta={"poc": int(info.poc), "decode_index": base + i})
        if validate:
            R.validate(params, pic)
        hl = {HASH_MD5: 16, HASH_CRC: 2, HASH_CHECKSUM: 4}.get(int(info.hash_type))
        hv = [bytes(info.hash[c][:hl]) for c in range(3)] if hl else None
        out.append(DecodedPicture(params=params, picture=pic, poc=int(info.poc),
                                  output_rank=int(info.output_rank),
                                  crop=(info.crop_left, info.crop_right, info.crop_top, info.crop_bottom),
                                  nal_unit_type=int(info.nal_unit_type), n_slices=int(info.n_slices),
                                  n_cus=int(info.n_cus), hash_type=int(info.hash_type), hash=hv,
                                  cvs_id=int(info.cvs_id), max_num_reorder=int(info.max_num_reorder),
                                  output_flag=bool(info.output_flag),
                                  scaling=(np.ctypeslib.as_array(ctypes.cast(info.scaling_factors, ctypes.POINTER(ctypes.c_uint8)),
                                                                 (2032,)).copy() if info.scaling_factors else None)))
    return out


def decode_stream(data: bytes, threads: int = 0, validate: bool = False):
    """Parse a whole Annex-B HEVC byte stream; returns [DecodedPicture] in decode order.

    ``validate`` re-runs the host-side record checks (the back-end's upload validates
    every record again in C++ before any kernel sees it)."""
    lib = load()
    h = ctypes.c_void_p()
    if lib.p265fe_create(ctypes.byref(h)) != OK:
        raise MemoryError("p265fe_create failed")
    owner = _Owner(lib, h)
    n = lib.p265fe_decode(h, bytes(data), len(data), int(threads))
    if n < 0:
        _fail(lib, h, n, "p265fe_decode")
    return _collect(lambda i, ref: lib.p265fe_picture(h, i, ref), n, owner, validate)


class StreamParser:
    """Incremental parsing of an Annex-B stream fed in arbitrary chunks.

    ``feed(chunk)`` returns the pictures completed so far, in decode order; stream state
    (parameter sets, POC, a partial access unit or NAL unit) carries over between calls;
    ``feed(b"", flush=True)`` ends the stream.  Output order is the caller's (see
    decoder.OutputQueue): ``output_rank`` stays -1 here.

    ``asynchronous=True`` (P265FE_ASYNC): ``feed`` only submits the complete access units to the
    decoder's persistent parse workers and returns the pictures parsed so far (a decode-order
    prefix, possibly empty); ``wait(all)`` blocks for the next one (or all) and returns them, so
    the parsing of one chunk overlaps the slowest pictures of the previous one."""

    def __init__(self, threads: int = 0, validate: bool = False, asynchronous: bool = False):
        self.lib = load()
        h = ctypes.c_void_p()
        if self.lib.p265fe_create(ctypes.byref(h)) != OK:
            raise MemoryError("p265fe_create failed")
        self._owner = _Owner(self.lib, h)
        self.h = h
        self.threads = int(threads)
        self.validate = validate
        self.asynchronous = bool(asynchronous)
        self.n_pictures = 0
        self.pending = 0            # async: submitted and not yet taken

    def feed(self, data: bytes, flush: bool = False):
        lib = self.lib
        data = bytes(data)
        flags = (FLUSH if flush else 0) | (ASYNC if self.asynchronous else 0)
        n = lib.p265fe_feed(self.h, data, len(data), self.threads, flags)
        if n < 0:
            _fail(lib, self.h, n, "p265fe_feed")
        if self.asynchronous:
            self.pending = n
        return self._take()

    def wait(self, all: bool = False):
        """Async: block until the next picture in decode order is parsed (or every submitted one,
        ``all``), then take the parsed prefix ([] when nothing is pending)."""
        if not self.pending:
            return []
        n = self.lib.p265fe_wait(self.h, 1 if all else 0)
        if n < 0:
            _fail(self.lib, self.h, n, "p265fe_wait")
        return self._take()

    def _take(self):
        lib = self.lib
        sp = ctypes.c_void_p()
        cnt = lib.p265fe_take(self.h, ctypes.byref(sp))
        if cnt < 0:
            if cnt in (EBITSTREAM, EUNSUPPORTED):
                if self.asynchronous:       # the failed picture is reported once and dropped (p265fe.h)
                    self.pending = max(0, self.pending - 1)
                    self.n_pictures += 1
                _fail(lib, self.h, cnt, "p265fe_take")
            raise MemoryError("p265fe_take failed (%d)" % cnt)
        owner = _SetOwner(lib, sp)
        pics = _collect(lambda i, ref: lib.p265fe_pictures_get(sp, i, ref), cnt, owner, self.validate,
                        base=self.n_pictures)
        self.n_pictures += cnt
        if self.asynchronous:
            self.pending -= cnt
        return pics
