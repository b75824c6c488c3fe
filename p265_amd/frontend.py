"""Drop-in surface for the p265 Python front-end (decoder.ctu / decoder.cu call shape).

The reference front-end parses a CTU (decoder/ctu.py:24-30: Sao.parse, then the CU
quadtree), and for every leaf CU calls ``Cu.decode_leaf()`` (decoder/cu.py:483-494),
which would run the per-CU reconstruction if it were not dead code.  This module
keeps that call surface but turns it into record building:

* ``PictureBuilder.add_cu`` is what ``Cu.decode_leaf`` calls per leaf CU: it walks
  the CU's TU leaves in decode (z-)order exactly like ``Cu.decode_intra`` /
  ``IntraPu.decode`` would (cu.py:595-615, intra.py:39-56, with the chroma 4x4
  rule of tu.py:127-135) and appends one TB record per transform block.
* ``PictureBuilder.add_ctu`` is what ``Ctu.parse`` calls after ``Sao.parse``
  (ctu.py:27-28): it converts the SAO syntax (sao.py:122-215) into SaoOffsetVal.
* ``finish()`` is the end-of-picture hook (slice.py:284-286): it returns the
  ``records.Picture`` that ``recon.ReconContext.submit`` takes.

``ReconHook`` adapts live reference objects (duck-typed attribute access, no import
of the reference) onto a builder; ``pictures_from_frontend_npz`` rebuilds pictures
from the committed front-end capture of sanity.bin.
"""
import json

import numpy as np

from . import records as R

# Chroma QP mapping for ChromaArrayType == 1 (cu.py:575-591, spec Table 8-10).
def qpc_from_qpi(qpi):
    if qpi < 30:
        return qpi
    if qpi >= 43:
        return qpi - 6
    return [29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37][qpi - 30]


def chroma_qp(qp_y, cb_qp_offset, cr_qp_offset, qp_bd_offset_c=0):
    """QpCb/QpCr from QpY and the pps+slice offsets (cu.py:573-591)."""
    def one(off):
        qpi = min(max(qp_y + off, -qp_bd_offset_c), 57)
        return qpc_from_qpi(qpi)
    return one(cb_qp_offset), one(cr_qp_offset)


def sao_offset_val(sao_type, offset_abs, offset_sign, bit_depth):
    """SaoOffsetVal[1..4] (7.4.9.3.2): EO signs are inferred (+,+,-,-), BO signs are coded.

    The reference never infers the EO signs on the non-merge path (sao.py:50-77,
    111-116), so coded signs are ignored for EO here.
    """
    shift = bit_depth - min(bit_depth, 10)
    out = []
    for i in range(4):
        a = int(offset_abs[i])
        if sao_type == 2:
            s = -1 if i >= 2 else 1
        else:
            s = -1 if int(offset_sign[i]) else 1
        out.append(s * (a << shift))
    return out


class PictureBuilder:
    """Accumulates the TB/CTU records of one picture in decode order."""

    def __init__(self, params, pcm_loop_filter_disabled=False):
        self.params = params
        self.wc, self.hc = R.ctb_grid(params)
        self.ctb_log2 = int(params["ctb_log2_size"])
        self.ctus = np.zeros(self.wc * self.hc, R.CTU_DTYPE)
        self.ctus["flags"] = R.CTU_LF_ACROSS_SLICES
        self._tb_rows = {}           # ctu addr -> list of TB tuples
        self._coef = []
        self._ncoef = 0
        self._nofilter = None
        self.pcm_lf_disabled = bool(pcm_loop_filter_disabled)

    # -- coefficient storage -------------------------------------------------
    def _store(self, block):
        block = np.ascontiguousarray(block, np.int16).reshape(-1)
        off = self._ncoef
        self._coef.append(block)
        self._ncoef += block.size
        return off

    def _tb(self, addr, x, y, log2, c_idx, mode, flags, qp, coef_off):
        self._tb_rows.setdefault(addr, []).append((x, y, log2, c_idx, mode, flags, qp, coef_off))

    def _mark_nofilter(self, x, y, log2):
        w, h = int(self.params["pic_width"]), int(self.params["pic_height"])
        nw, nh = (w + 7) // 8, (h + 7) // 8
        if self._nofilter is None:
            self._nofilter = np.zeros(nw * nh, np.uint8)
        n8 = max(1, (1 << log2) >> 3)
        for j in range(n8):
            for i in range(n8):
                bx, by = (x >> 3) + i, (y >> 3) + j
                if bx < nw and by < nh:
                    self._nofilter[by * nw + bx] = 1

    # -- the per-leaf-CU hook (Cu.decode_leaf) --------------------------------
    def add_cu(self, x, y, log2, part_mode, modes_y, mode_c, qp_y, qp_cb, qp_cr, tus,
               bypass=False, pcm=False, pcm_samples=None):
        """Append the TBs of one leaf intra CU.

        qp_* are qP values incl. QpBdOffset.  ``tus``: TU leaves in z-order, each a dict
        with x, y, log2, blk (blkIdx), cbf (3), tskip (3) and coef (3 arrays [y][x] or None).
        ``pcm_samples``: for a PCM CU, three arrays [y][x] already at BitDepth.
        """
        addr = (y >> self.ctb_log2) * self.wc + (x >> self.ctb_log2)
        byp = R.TB_BYPASS if bypass else 0
        if bypass or (pcm and self.pcm_lf_disabled):
            self._mark_nofilter(x, y, log2)
        if pcm:
            for c in range(3):
                lg = log2 if c == 0 else log2 - 1
                sub = 0 if c == 0 else 1
                off = self._store(pcm_samples[c])
                # qp of a PCM TB is not used for scaling; the luma one carries QpY for deblocking
                self._tb(addr, x >> sub, y >> sub, lg, c, 0, R.TB_PCM, (qp_y, qp_cb, qp_cr)[c], off)
            return
        half = (1 << log2) >> 1
        for t in tus:
            tx, ty, tl = int(t["x"]), int(t["y"]), int(t["log2"])
            pu = (((ty - y) >= half) * 2 + ((tx - x) >= half)) if part_mode == 1 else 0
            self._emit(addr, tx, ty, tl, 0, int(modes_y[pu]), t, 0, qp_y, byp)
            if tl > 2:
                for c, qp in ((1, qp_cb), (2, qp_cr)):
                    self._emit(addr, tx >> 1, ty >> 1, tl - 1, c, mode_c, t, c, qp, byp)
            elif int(t["blk"]) == 3:             # luma 4x4 quad: chroma 4x4 after blkIdx 3
                for c, qp in ((1, qp_cb), (2, qp_cr)):
                    self._emit(addr, (tx - 4) >> 1, (ty - 4) >> 1, 2, c, mode_c, t, c, qp, byp)

    def _emit(self, addr, x, y, log2, c_idx, mode, t, c, qp, byp):
        flags = byp
        off = 0
        if int(t["cbf"][c]):
            flags |= R.TB_CBF
            co = t["coef"][c]
            n = 1 << log2
            if co is None:
                co = np.zeros((n, n), np.int16)
            off = self._store(co)
        if int(t["tskip"][c]):
            flags |= R.TB_TSKIP
        self._tb(addr, x, y, log2, c_idx, mode, flags, qp, off)

    # -- the per-CTU hook (Ctu.parse after Sao.parse) -------------------------
    def add_ctu(self, addr, slice_addr=0, tile_id=0, lf_across_slices=True,
                sao_type=(0, 0, 0), sao_abs=None, sao_sign=None, sao_band=(0, 0, 0), sao_eo=(0, 0, 0),
                deblocking=False, beta_offset_div2=0, tc_offset_div2=0):
        """``deblocking``: !slice_deblocking_filter_disabled_flag of the CTU's slice, with its
        slice_beta_offset_div2 / slice_tc_offset_div2 (slice.py:170-175, pps.py:122-131)."""
        c = self.ctus[addr]
        c["slice_addr"] = slice_addr
        c["tile_id"] = tile_id
        c["flags"] = (R.CTU_LF_ACROSS_SLICES if lf_across_slices else 0) | (R.CTU_DEBLOCK if deblocking else 0)
        c["deblock_offsets"] = R.deblock_offsets(int(beta_offset_div2), int(tc_offset_div2)) if deblocking else 0
        for ci in range(3):
            t = int(sao_type[ci])
            c["sao_type"][ci] = t
            if t == 0:
                continue
            bd = int(self.params["bit_depth_luma" if ci == 0 else "bit_depth_chroma"])
            c["sao_class"][ci] = int(sao_band[ci]) if t == 1 else int(sao_eo[ci])
            c["sao_offset"][ci] = sao_offset_val(t, sao_abs[ci], sao_sign[ci] if sao_sign is not None
                                                 else (0, 0, 0, 0), bd)
        self.ctus[addr] = c

    # -- end of picture ---------------------------------------------------------
    def finish(self, meta=None) -> R.Picture:
        rows, begin = [], 0
        order = sorted(self._tb_rows)             # any order works; raster keeps it simple
        for addr in order:
            lst = self._tb_rows[addr]
            self.ctus["tb_begin"][addr] = begin
            self.ctus["tb_count"][addr] = len(lst)
            rows.extend(lst)
            begin += len(lst)
        tbs = np.zeros(len(rows), R.TB_DTYPE)
        if rows:
            a = np.array(rows, np.int64)
            for i, name in enumerate(("x", "y", "log2_size", "c_idx", "pred_mode", "flags", "qp", "coef_off")):
                tbs[name] = a[:, i]
        coef = np.concatenate(self._coef) if self._coef else np.zeros(0, np.int16)
        pic = R.Picture(ctus=self.ctus, tbs=tbs, coef=coef, nofilter=self._nofilter, meta=meta or {})
        R.validate(self.params, pic)
        return pic


class ReconHook:
    """Adapter for live reference objects (duck-typed), i.e. the lines a maintainer adds
    to decoder/cu.py:487 (``self.ctx.recon.on_decode_leaf(self)``), ctu.py:28
    (``self.ctx.recon.on_ctu_parsed(self, self.ctx.img.slice_hdr, self.ctx.pps)``) and
    slice.py:284-286 (``pic = self.ctx.recon.on_end_of_picture()``).

    Reads exactly the attributes Cu.decode_intra / IntraPu / scaling would have read:
    cu.x/y/size/log2size/part_mode/intra_pred_mode_y (x-major md_dict)/intra_pred_mode_c/
    qp_y/qp_cb/qp_cr, cu.cu_transquant_bypass_flag/pcm_flag, and the TU leaves' x/y/log2size/
    idx, cbf_luma/cbf_cb/cbf_cr, transform_skip_flag and trans_coeff_level (x-major,
    tu.py:87-90; a luma 4x4 quad's shared chroma pair lives on its blkIdx-3 leaf,
    tu.py:127-135).  PCM CUs: the reference calls an undefined decode_pcm (cu.py:484-485) and
    never stores the samples, so the hook reads them under their syntax names (7.3.8.7):
    ``cu.pcm_sample_luma`` (nCbS^2 values, raster) and ``cu.pcm_sample_chroma`` (Cb then Cr,
    (nCbS/2)^2 each), at PcmBitDepth, shifted to BitDepth as 8.4.4.1 (pcm_bit_depth_*).
    ``pcm_loop_filter_disabled``: pcm_loop_filter_disabled_flag of the SPS.
    """

    def __init__(self, params, qp_bd_offset_y=0, qp_bd_offset_c=0, pcm_bit_depth_luma=8, pcm_bit_depth_chroma=8,
                 pcm_loop_filter_disabled=False):
        self.params = params
        self.off_y, self.off_c = qp_bd_offset_y, qp_bd_offset_c
        self.pcm_shift = (int(params["bit_depth_luma"]) - int(pcm_bit_depth_luma),
                          int(params["bit_depth_chroma"]) - int(pcm_bit_depth_chroma))
        self.pcm_lf_disabled = bool(pcm_loop_filter_disabled)
        self.builder = PictureBuilder(params, pcm_loop_filter_disabled=self.pcm_lf_disabled)
        self.pictures = []

    def _pcm_samples(self, cu):
        n = int(cu.size)
        h = n >> 1
        luma = np.asarray(cu.pcm_sample_luma, np.int64).reshape(n, n) << self.pcm_shift[0]
        ch = np.asarray(cu.pcm_sample_chroma, np.int64).reshape(2, h, h) << self.pcm_shift[1]
        return [luma.astype(np.int16), ch[0].astype(np.int16), ch[1].astype(np.int16)]

    def on_decode_leaf(self, cu):
        modes = [0, 0, 0, 0]
        pm = int(getattr(cu, "part_mode", 0))
        qps = (cu.qp_y + self.off_y, cu.qp_cb + self.off_c, cu.qp_cr + self.off_c)
        bypass = bool(getattr(cu, "cu_transquant_bypass_flag", 0))
        if getattr(cu, "pcm_flag", 0):
            self.builder.add_cu(cu.x, cu.y, cu.log2size, pm, modes, 0, *qps, [], bypass=bypass, pcm=True,
                                pcm_samples=self._pcm_samples(cu))
            return
        h = cu.size >> 1
        for i in range(4 if pm == 1 else 1):
            modes[i] = int(cu.intra_pred_mode_y[cu.x + h * (i % 2)][cu.y + h * (i // 2)])
        tus = []
        if getattr(cu, "tu", None) is not None:
            for leaf in cu.tu.get_leaves():
                tsf = getattr(leaf, "transform_skip_flag", None)
                cbf = [int(getattr(leaf, "cbf_luma", 0)), int(leaf.cbf_cb), int(leaf.cbf_cr)]
                tus.append(dict(x=leaf.x, y=leaf.y, log2=leaf.log2size, blk=getattr(leaf, "idx", 0), cbf=cbf,
                                tskip=[int(tsf[c]) if tsf is not None else 0 for c in range(3)],
                                coef=[np.asarray(leaf.trans_coeff_level[c]).T for c in range(3)]))
        self.builder.add_cu(cu.x, cu.y, cu.log2size, pm, modes, int(getattr(cu, "intra_pred_mode_c", 0)),
                            *qps, tus, bypass=bypass)

    def on_ctu_parsed(self, ctu, slice_hdr, pps=None):
        s = ctu.sao
        on = bool(slice_hdr.slice_sao_luma_flag or slice_hdr.slice_sao_chroma_flag)
        pps = pps if pps is not None else getattr(slice_hdr, "pps", None)
        # slice_deblocking_filter_disabled_flag is never assigned by the reference (slice.py:170-178
        # reads it); absent an override it is inferred from the PPS (pps.py:122-131)
        dbk_off = bool(getattr(slice_hdr, "slice_deblocking_filter_disabled_flag",
                               getattr(pps, "pps_deblocking_filter_disabled_flag", 0)))
        lf_across = getattr(slice_hdr, "slice_loop_filter_across_slices_enabled_flag",
                            getattr(pps, "pps_loop_filter_across_slices_enabled_flag", 1))
        # the reference's Ctu carries no tile id: TileId lives in pps.tile_id_rs (pps.py:215-227,
        # read by image.py:65 for availability); a duck-typed ctu.tile_id is the fallback
        tids = getattr(pps, "tile_id_rs", None)
        tile_id = int(tids[ctu.addr_rs]) if tids is not None else int(getattr(ctu, "tile_id", 0))
        self.builder.add_ctu(ctu.addr_rs, slice_addr=getattr(ctu, "slice_addr", 0),
                             tile_id=tile_id,
                             lf_across_slices=bool(lf_across),
                             deblocking=not dbk_off,
                             beta_offset_div2=int(getattr(slice_hdr, "slice_beta_offset_div2",
                                                          getattr(pps, "pps_beta_offset_div2", 0))),
                             tc_offset_div2=int(getattr(slice_hdr, "slice_tc_offset_div2",
                                                        getattr(pps, "pps_tc_offset_div2", 0))),
                             sao_type=s.sao_type_idx if on else (0, 0, 0),
                             sao_abs=s.sao_offset_abs if on else None,
                             sao_sign=s.sao_offset_sign if on else None,
                             sao_band=s.sao_band_position if on else (0, 0, 0),
                             sao_eo=s.sao_eo_class if on else (0, 0, 0))

    def on_end_of_picture(self, meta=None):
        pic = self.builder.finish(meta)
        self.pictures.append(pic)
        self.builder = PictureBuilder(self.params, pcm_loop_filter_disabled=self.pcm_lf_disabled)
        return pic


def params_from_frontend(d):
    return R.make_params(
        pic_width=d["pic_width"], pic_height=d["pic_height"], chroma_format_idc=d["chroma_format_idc"],
        bit_depth_luma=d["bit_depth_luma"], bit_depth_chroma=d["bit_depth_chroma"],
        ctb_log2_size=d["ctb_log2_size"], min_tb_log2_size=d["min_tb_log2_size"],
        max_tb_log2_size=d["max_tb_log2_size"], strong_intra_smoothing=d["strong_intra_smoothing"],
        constrained_intra_pred=d["constrained_intra_pred"], sample_adaptive_offset=d["sample_adaptive_offset"],
        loop_filter_across_tiles=d["loop_filter_across_tiles"], scaling_list_enabled=d["scaling_list_enabled"],
        pps_cb_qp_offset=d.get("pps_cb_qp_offset", 0), pps_cr_qp_offset=d.get("pps_cr_qp_offset", 0))


def pictures_from_frontend_npz(path, deblocking=None):
    """Rebuild (params, [Picture]) from tests/golden/sanity_frontend.npz.

    ``deblocking`` None follows the stream: sanity.bin has deblocking_filter_control_present_flag
    = 0 (test/golden/pps.log:23), i.e. deblocking on with zero offsets in every slice.
    """
    z = np.load(path, allow_pickle=False)
    pd = json.loads(bytes(z["params"]).decode())
    params = params_from_frontend(pd)
    if deblocking is None:
        deblocking = not pd.get("deblocking_filter_control_present", 0)
    cus, tus, coefs, ctus = z["cus"], z["tus"], z["coefs"], z["ctus"]
    # dense coefficient blocks per (tu, c): [y][x]
    blocks = {}
    for r in coefs:
        key = (int(r["tu"]), int(r["c"]))
        tl = int(tus[key[0]]["log2"])
        n = 1 << (tl if (key[1] == 0 or tl == 2) else tl - 1)
        b = blocks.get(key)
        if b is None:
            b = blocks[key] = np.zeros((n, n), np.int16)
        b[int(r["y"]), int(r["x"])] = int(r["v"])
    tus_by_cu = {}
    for i, t in enumerate(tus):
        tus_by_cu.setdefault(int(t["cu"]), []).append(i)
    pics = []
    for f in range(pd["n_frames"]):
        b = PictureBuilder(params)
        for ci in np.nonzero(cus["frame"] == f)[0]:
            cu = cus[ci]
            tl = []
            for ti in tus_by_cu.get(int(ci), []):
                t = tus[ti]
                tl.append(dict(x=int(t["x"]), y=int(t["y"]), log2=int(t["log2"]), blk=int(t["blk"]),
                               cbf=[int(v) for v in t["cbf"]], tskip=[int(v) for v in t["tskip"]],
                               coef=[blocks.get((ti, c)) for c in range(3)]))
            b.add_cu(int(cu["x"]), int(cu["y"]), int(cu["log2"]), int(cu["part_mode"]),
                     [int(v) for v in cu["mode_y"]], int(cu["mode_c"]), int(cu["qp_y"]),
                     int(cu["qp_cb"]), int(cu["qp_cr"]), tl, bypass=bool(cu["bypass"]), pcm=bool(cu["pcm"]))
        for r in ctus[ctus["frame"] == f]:
            b.add_ctu(int(r["ctu"]), slice_addr=int(r["slice_addr"]), lf_across_slices=bool(r["lf_across_slices"]),
                      sao_type=r["sao_type"], sao_abs=r["sao_abs"], sao_sign=r["sao_sign"],
                      sao_band=r["sao_band"], sao_eo=r["sao_eo"], deblocking=deblocking)
        pics.append(b.finish(meta={"source": "sanity.bin", "frame": f}))
    return params, pics
