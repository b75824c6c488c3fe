"""Record format of the reconstruction batch (numpy mirror of include/p265r.h).

The reference decoder keeps everything the hot path needs inside its syntax-tree
objects (decoder/cu.py, decoder/tu.py, decoder/sao.py) and reads it back per sample
through tree walks (tu.py:667-701, ctu.py:33-71).  The MI355X back-end instead
receives flat, fixed-size records per picture:

  CTU_DTYPE  one per CTU (raster order): TB range, slice/tile ids, SAO parameters
  TB_DTYPE   one per transform block in decode order: position, size, component,
             intra mode, flags, qP, offset of its dense int16 coefficients
  coef       int16 TransCoeffLevel, N*N raster [y][x] per coded TB

``Picture`` bundles them; ``Params`` is the 32-byte sequence-parameter POD.
"""
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

ABI_VERSION = 2                 # include/p265r.h P265R_ABI_VERSION (2: per-picture size)

TB_CBF, TB_TSKIP, TB_BYPASS, TB_PCM = 0x01, 0x02, 0x04, 0x08
PIC_RECON_INPUT = 0x01
CTU_LF_ACROSS_SLICES, CTU_DEBLOCK = 0x01, 0x02

PARAMS_DTYPE = np.dtype([
    ("version", "<u4"), ("pic_width", "<u2"), ("pic_height", "<u2"),
    ("chroma_format_idc", "u1"), ("bit_depth_luma", "u1"), ("bit_depth_chroma", "u1"),
    ("ctb_log2_size", "u1"), ("min_tb_log2_size", "u1"), ("max_tb_log2_size", "u1"),
    ("strong_intra_smoothing", "u1"), ("constrained_intra_pred", "u1"),
    ("sample_adaptive_offset", "u1"), ("loop_filter_across_tiles", "u1"),
    ("scaling_list_enabled", "u1"), ("pps_cb_qp_offset", "i1"), ("pps_cr_qp_offset", "i1"),
    ("reserved", "u1", 11)])
assert PARAMS_DTYPE.itemsize == 32

CTU_DTYPE = np.dtype([
    ("tb_begin", "<u4"), ("tb_count", "<u2"), ("tile_id", "<u2"), ("slice_addr", "<u4"),
    ("flags", "u1"), ("sao_type", "u1", 3), ("sao_class", "u1", 3), ("deblock_offsets", "u1"),
    ("sao_offset", "i1", (3, 4))])
assert CTU_DTYPE.itemsize == 32

TB_DTYPE = np.dtype([
    ("x", "<u2"), ("y", "<u2"), ("log2_size", "u1"), ("c_idx", "u1"), ("pred_mode", "u1"),
    ("flags", "u1"), ("qp", "u1"), ("reserved", "u1", 3), ("coef_off", "<u4")])
assert TB_DTYPE.itemsize == 16

PARAM_KEYS = [n for n in PARAMS_DTYPE.names if n not in ("version", "reserved")]


def make_params(**kw) -> np.ndarray:
    """Build a params record; unspecified fields default to the sanity.bin-like SPS/PPS."""
    d = dict(pic_width=352, pic_height=288, chroma_format_idc=1, bit_depth_luma=8,
             bit_depth_chroma=8, ctb_log2_size=6, min_tb_log2_size=2, max_tb_log2_size=5,
             strong_intra_smoothing=1, constrained_intra_pred=0, sample_adaptive_offset=1,
             loop_filter_across_tiles=1, scaling_list_enabled=0, pps_cb_qp_offset=0, pps_cr_qp_offset=0)
    for k, v in kw.items():
        if k not in d:
            raise KeyError("unknown params field %r" % k)
        d[k] = v
    p = np.zeros((), PARAMS_DTYPE)
    p["version"] = ABI_VERSION
    for k, v in d.items():
        p[k] = v
    return p


def plane_dtypes(params):
    """numpy sample type of the Y, Cb, Cr planes: uint8 at BitDepth 8, uint16 (little-endian) above
    (include/p265r.h p265r_picture.out / recon)."""
    dy = np.uint8 if int(params["bit_depth_luma"]) <= 8 else np.uint16
    dc = np.uint8 if int(params["bit_depth_chroma"]) <= 8 else np.uint16
    return [dy, dc, dc]


def qp_bd_offset(params, c_idx=0) -> int:
    """QpBdOffsetY / QpBdOffsetC = 6 * (BitDepth - 8) (7.4.3.2.1)."""
    return 6 * (int(params["bit_depth_luma" if c_idx == 0 else "bit_depth_chroma"]) - 8)


def deblock_offsets(beta_offset_div2, tc_offset_div2) -> int:
    """P265R_DEBLOCK_OFFSETS: two 4-bit two's-complement fields (each -6..6)."""
    for v in (beta_offset_div2, tc_offset_div2):
        if not -6 <= v <= 6:
            raise ValueError("deblocking offset_div2 out of range: %d" % v)
    return (beta_offset_div2 & 15) | ((tc_offset_div2 & 15) << 4)


def unpack_deblock_offsets(v):
    """(slice_beta_offset_div2, slice_tc_offset_div2) of a CTU record's deblock_offsets byte."""
    b, t = int(v) & 15, (int(v) >> 4) & 15
    return (b - 16 if b >= 8 else b), (t - 16 if t >= 8 else t)


def params_dict(p) -> dict:
    return {k: int(p[k]) for k in PARAM_KEYS}


def pic_params(params, pic):
    """The parameter set one picture of a batch decodes with: the context's ``params``, with the
    picture's own size when it has one (Picture.size, a ragged batch)."""
    if pic is None or pic.size is None:
        return params
    w, h = (int(v) for v in pic.size)
    if w == int(params["pic_width"]) and h == int(params["pic_height"]):
        return params
    if w > int(params["pic_width"]) or h > int(params["pic_height"]) or w <= 0 or h <= 0 or w % 8 or h % 8:
        raise RecordError("picture size %dx%d does not fit the context's %dx%d (multiples of 8)"
                          % (w, h, int(params["pic_width"]), int(params["pic_height"])))
    kw = params_dict(params)
    kw.update(pic_width=w, pic_height=h)
    return make_params(**kw)


def ctb_grid(p):
    ctb = 1 << int(p["ctb_log2_size"])
    w, h = int(p["pic_width"]), int(p["pic_height"])
    return (w + ctb - 1) // ctb, (h + ctb - 1) // ctb


@dataclass
class Picture:
    """Records of one picture (the C struct p265r_picture without the output planes)."""
    ctus: np.ndarray                      # CTU_DTYPE, raster order
    tbs: np.ndarray                       # TB_DTYPE
    coef: np.ndarray                      # int16
    nofilter: Optional[np.ndarray] = None  # uint8 per 8x8 luma block or None
    meta: dict = field(default_factory=dict)
    # P265R_PIC_RECON_INPUT: the reconstruction [Y, Cb, Cr] (uint8) is given; only the
    # in-loop filters run on it (TB records then serve the deblocking map only)
    recon_input: Optional[list] = None
    # this picture's luma (width, height) when it is smaller than the batch context's params
    # (p265r_picture.pic_width / pic_height): the uneven tiles of one picture in one batch
    size: Optional[tuple] = None

    def as_oracle_dict(self):
        return {"ctus": self.ctus, "tbs": self.tbs, "coef": self.coef, "nofilter": self.nofilter}

    @property
    def n_coded_coef(self):
        m = (self.tbs["flags"] & (TB_CBF | TB_PCM)) != 0
        return int(np.sum(1 << (2 * self.tbs["log2_size"][m].astype(np.int64))))


class RecordError(ValueError):
    pass


def check_shapes(params, pic: Picture):
    """The checks the C ABI cannot do itself (array dtypes and lengths behind the raw
    pointers); everything inside the records is validated again by p265r_batch_upload."""
    params = pic_params(params, pic)
    wc, hc = ctb_grid(params)
    if pic.ctus.dtype != CTU_DTYPE or pic.tbs.dtype != TB_DTYPE or pic.coef.dtype != np.int16:
        raise RecordError("record dtypes do not match the ABI")
    if len(pic.ctus) != wc * hc:
        raise RecordError("expected %d CTUs, got %d" % (wc * hc, len(pic.ctus)))
    w, h = int(params["pic_width"]), int(params["pic_height"])
    if pic.nofilter is not None and len(pic.nofilter) != ((w + 7) // 8) * ((h + 7) // 8):
        raise RecordError("nofilter map has the wrong size")


def validate(params, pic: Picture):
    """Host-side checks mirroring the C++ ones (p265_amd/csrc/p265r.hip: validate_picture).

    The kernels assume every record lies inside its CTU and picture; these checks are
    what keeps a malformed record from faulting the GPU.
    """
    params = pic_params(params, pic)
    wc, hc = ctb_grid(params)
    if pic.ctus.dtype != CTU_DTYPE or pic.tbs.dtype != TB_DTYPE or pic.coef.dtype != np.int16:
        raise RecordError("record dtypes do not match the ABI")
    if len(pic.ctus) != wc * hc:
        raise RecordError("expected %d CTUs, got %d" % (wc * hc, len(pic.ctus)))
    ctb_log2 = int(params["ctb_log2_size"])
    w, h = int(params["pic_width"]), int(params["pic_height"])
    tbs = pic.tbs
    begin = pic.ctus["tb_begin"].astype(np.int64)
    end = begin + pic.ctus["tb_count"]
    if (end > len(tbs)).any():
        raise RecordError("CTU TB range outside the TB array")
    lg = tbs["log2_size"].astype(np.int64)
    c = tbs["c_idx"].astype(np.int64)
    if ((lg < 2) | (lg > 5)).any() or (c > 2).any() or (tbs["pred_mode"] > 34).any():
        raise RecordError("TB size / component / mode out of range")
    if ((c > 0) & (lg > 4)).any():
        raise RecordError("4:2:0 chroma TB larger than 16x16")
    if (pic.ctus["tb_count"].astype(np.int64) > 3 * (1 << (2 * (ctb_log2 - 2))) // 2).any():
        raise RecordError("CTU lists more TBs than it has 4x4 units")
    cs = np.concatenate([[0], np.cumsum(tbs["c_idx"] == 0)])
    if ((cs[end] - cs[begin]) > (1 << (2 * (ctb_log2 - 2)))).any():
        raise RecordError("CTU lists more luma TBs than it has 4x4 units")
    cc = np.concatenate([[0], np.cumsum(tbs["c_idx"] != 0)])
    if ((cc[end] - cc[begin]) > 2 * (1 << (2 * (ctb_log2 - 3)))).any():
        raise RecordError("CTU lists more chroma TBs than it has 4x4 chroma units")
    sub = (c > 0).astype(np.int64)
    xl, yl = tbs["x"].astype(np.int64) << sub, tbs["y"].astype(np.int64) << sub
    nl = (1 << lg) << sub
    if ((xl >= w) | (yl >= h)).any():
        raise RecordError("TB outside picture")
    counts = pic.ctus["tb_count"].astype(np.int64)
    owner = np.repeat(np.arange(len(pic.ctus)), counts)
    # idx[k] = TB index of the k-th (CTU, TB) pair: tb_begin of its CTU + rank inside the CTU
    first = np.cumsum(counts) - counts
    idx = np.repeat(begin, counts) + (np.arange(int(counts.sum())) - np.repeat(first, counts))
    if len(idx):
        cx, cy = (owner % wc) << ctb_log2, (owner // wc) << ctb_log2
        ctb = 1 << ctb_log2
        bad = ((xl[idx] < cx) | (yl[idx] < cy) | (xl[idx] + nl[idx] > cx + ctb) | (yl[idx] + nl[idx] > cy + ctb))
        if bad.any():
            raise RecordError("TB not inside its CTU")
    coded = (tbs["flags"] & (TB_CBF | TB_PCM)) != 0
    if (tbs["coef_off"][coded].astype(np.int64) + (1 << (2 * lg[coded])) > len(pic.coef)).any():
        raise RecordError("coefficient range outside coef array")
    if (pic.ctus["sao_type"] > 2).any():
        raise RecordError("bad SaoTypeIdx")
    st, sc = pic.ctus["sao_type"], pic.ctus["sao_class"]
    if ((st[:, 1] != st[:, 2]) | ((st[:, 1] == 2) & (sc[:, 1] != sc[:, 2]))).any():
        raise RecordError("Cb and Cr must share SaoTypeIdx and SaoEoClass (7.4.9.3.2)")
    nib = np.stack([pic.ctus["deblock_offsets"] & 15, pic.ctus["deblock_offsets"] >> 4])
    if ((nib == 7) | (nib == 8) | (nib == 9)).any():
        raise RecordError("deblocking offset_div2 outside -6..6")
    if pic.nofilter is not None and len(pic.nofilter) != ((w + 7) // 8) * ((h + 7) // 8):
        raise RecordError("nofilter map has the wrong size")
