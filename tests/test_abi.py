"""C ABI checks that need no GPU: the library loads, exports every function the
header declares, and its structs match the numpy record layout."""
import ctypes
import os
import re

import numpy as np

from p265_amd import _lib
from p265_amd import records as R

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "p265r.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(p265r_[a-z_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported_and_bound():
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, n


def test_struct_layouts_match_records():
    assert ctypes.sizeof(_lib.Params) == R.PARAMS_DTYPE.itemsize == 32
    assert R.CTU_DTYPE.itemsize == 32 and R.TB_DTYPE.itemsize == 16
    assert ctypes.sizeof(_lib.PictureC) == 104
    assert ctypes.sizeof(_lib.Timings) == 48
    # offsets the kernels read (intra_rows.h: tb_from_words / res_addr)
    assert R.TB_DTYPE.fields["coef_off"][1] == 12 and R.TB_DTYPE.fields["flags"][1] == 7
    assert R.CTU_DTYPE.fields["sao_offset"][1] == 20


def test_version_errors_and_no_device_path():
    lib = _lib.load()
    assert lib.p265r_abi_version() == 2
    for code in (0, -1, -2, -3, -4, -5, -6, -7):
        assert lib.p265r_strerror(code)
    n = lib.p265r_device_count()
    assert n >= 0
    if n == 0:                                   # CPU container: create must fail cleanly, not crash
        p = _lib.Params()
        p.version, p.pic_width, p.pic_height, p.chroma_format_idc = 2, 64, 64, 1
        p.bit_depth_luma = p.bit_depth_chroma = 8
        p.ctb_log2_size, p.min_tb_log2_size, p.max_tb_log2_size = 6, 2, 5
        h = ctypes.c_void_p()
        assert lib.p265r_create(0, ctypes.byref(p), ctypes.byref(h)) == _lib.ENODEV
        assert not h.value


def test_invalid_params_rejected_before_device():
    lib = _lib.load()
    p = _lib.Params()
    h = ctypes.c_void_p()
    assert lib.p265r_create(0, ctypes.byref(p), ctypes.byref(h)) == _lib.EINVAL      # version 0
    p.version, p.pic_width, p.pic_height, p.chroma_format_idc = 2, 64, 64, 1
    p.ctb_log2_size, p.min_tb_log2_size, p.max_tb_log2_size = 6, 2, 5
    for bl, bc in ((13, 13), (10, 8), (8, 9), (7, 7)):        # one depth of 8..12 for luma and chroma
        p.bit_depth_luma, p.bit_depth_chroma = bl, bc
        assert lib.p265r_create(0, ctypes.byref(p), ctypes.byref(h)) == _lib.EUNSUPPORTED
    assert lib.p265r_wait(None) == _lib.EINVAL


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    try:
        _lib.load()
    except _lib.LibraryNotFound:
        return
    raise AssertionError("load() must raise when the library is missing (no CPU fallback)")


FE_HEADER = os.path.join(os.path.dirname(HEADER), "p265fe.h")


def test_front_end_exports_every_declared_symbol():
    from p265_amd import bitstream
    lib = bitstream.load()
    names = sorted(set(re.findall(r"\b(p265fe_[a-z_]+)\s*\(", open(FE_HEADER).read())))
    assert len(names) >= 11
    for n in names:
        assert hasattr(lib, n), n
        assert n in bitstream.SIGNATURES, n
    assert lib.p265fe_abi_version() == 4
    # p265fe_picture_info layout: 32 B params + pointers/counters + 48 B hash + the scaling factor pointer
    assert ctypes.sizeof(bitstream.PictureInfoC) == 168
    h = ctypes.c_void_p()
    assert lib.p265fe_create(ctypes.byref(h)) == 0
    assert lib.p265fe_picture(h, 0, None) == bitstream.EINVAL
    lib.p265fe_destroy(h)


def test_probe_library_exports_its_measurement_entry_points():
    """libp265probe.so (bench.py's measurement helper, not the product path): the issue-ceiling and the
    HBM stream-rate probes."""
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(HEADER)), "p265_amd", "libp265probe.so"))
    for name in ("p265probe_issue", "p265probe_stream"):
        assert hasattr(lib, name), name
