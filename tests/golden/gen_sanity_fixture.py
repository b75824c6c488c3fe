#!/usr/bin/env python3
"""Capture the front-end records of /root/reference/sanity.bin (THIS CONTAINER ONLY).

Runs the reference's own CABAC/syntax front-end (py2 source through the in-memory
shim in _refshim.py), first re-checks that its trace reproduces every file under
/root/reference/test/golden byte for byte (the reference's `make check`, extended
to all 95 files), then records exactly what the reference hands to the (dead)
reconstruction hook `Cu.decode_leaf` (decoder/cu.py:483-488) and what
`Ctu.parse` -> `Sao.parse` (decoder/ctu.py:27-28, decoder/sao.py:15-136) leaves
on each CTU:

* per leaf CU (in decode order): position, size, part_mode, luma intra modes
  (decoder/cu.py:175-265), chroma mode (cu.py:267-279), QpY/QpCb/QpCr
  (cu.py:496-593), cu_transquant_bypass_flag, pcm_flag;
* per TU leaf (decoder/tu.py:84-135): position, size, depth, blkIdx, cbf_luma /
  cbf_cb / cbf_cr, transform_skip_flag[3] and the non-zero TransCoeffLevel
  values after sign-data hiding (tu.py:320-340), kept sparse;
* per CTU: the SAO syntax (sao.py:122-215) and the slice-level flags.

Output: tests/golden/sanity_frontend.npz (data only: inputs of the hot path)
plus tests/golden/sanity_frontend.json (provenance + golden-match summary).

The same decode also drives the drop-in adapter p265_amd.frontend.ReconHook with the LIVE
reference objects -- exactly the calls INTEGRATION.md tells a maintainer to add at
cu.py:487 (on_decode_leaf), ctu.py:28 (on_ctu_parsed) and slice.py:284-286
(on_end_of_picture) -- and asserts that the records it builds equal, bit for bit, the
records rebuilt from the committed capture (frontend.pictures_from_frontend_npz).  The npz
is rewritten only if its arrays changed (zip timestamps would change its hash).

Usage:  PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/gen_sanity_fixture.py
"""
import filecmp
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refshim  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from p265_amd import frontend  # noqa: E402
from p265_amd import records as R  # noqa: E402

WORK = "/tmp/p265_sanity_fixture"
BITSTREAM = os.path.join(_refshim.REF_ROOT, "sanity.bin")
GOLDEN_DIR = os.path.join(_refshim.REF_ROOT, "test", "golden")


class _Args:
    bitstream = BITSTREAM
    skip_syntax_dump = 0
    output = None
    plot = None


def main():
    t0 = time.time()
    mods = _refshim.install(WORK)
    cu_mod, ctu_mod, slice_mod = mods["cu"], mods["ctu"], mods["slice"]

    state = {"frame": 0, "hook": None}
    cus, tus, coefs, ctus = [], [], [], []

    orig_decode_leaf = cu_mod.Cu.decode_leaf
    orig_ctu_parse = ctu_mod.Ctu.parse
    orig_sd_parse = slice_mod.SliceSegmentData.parse

    def hook(ctx):
        if state["hook"] is None:                   # created once the SPS / PPS are active
            sps = ctx.sps
            prm = R.make_params(pic_width=sps.pic_width_in_luma_samples, pic_height=sps.pic_height_in_luma_samples,
                                chroma_format_idc=sps.chroma_format_idc, bit_depth_luma=sps.bit_depth_y,
                                bit_depth_chroma=sps.bit_depth_c, ctb_log2_size=sps.ctb_log2_size_y,
                                min_tb_log2_size=sps.log2_min_transform_block_size,
                                max_tb_log2_size=sps.log2_max_transform_block_size,
                                strong_intra_smoothing=int(sps.strong_intra_smoothing_enabled_flag),
                                sample_adaptive_offset=int(sps.sample_adaptive_offset_enabled_flag))
            state["hook"] = frontend.ReconHook(prm, sps.qp_bd_offset_y, sps.qp_bd_offset_c)
        return state["hook"]

    def decode_leaf(self):
        orig_decode_leaf(self)                      # runs decode_qp (cu.py:487)
        hook(self.ctx).on_decode_leaf(self)         # the maintainer's line at cu.py:487
        root = self.get_root()
        sps = self.ctx.sps
        if self.pred_mode != self.MODE_INTRA:
            raise RuntimeError("sanity.bin is all-intra")
        modes = [255, 255, 255, 255]
        if self.pcm_flag == 0:
            if self.part_mode == 1:                 # PART_NxN: 4 luma PBs
                h = self.size >> 1
                for i in range(4):
                    modes[i] = int(self.intra_pred_mode_y[self.x + h * (i % 2)][self.y + h * (i // 2)])
            else:
                modes[0] = int(self.intra_pred_mode_y[self.x][self.y])
            mode_c = int(self.intra_pred_mode_c)
        else:
            mode_c = 255
        cu_idx = len(cus)
        cus.append((state["frame"], root.addr_rs, self.x, self.y, self.log2size, self.part_mode,
                    *modes, mode_c, self.qp_y + sps.qp_bd_offset_y, self.qp_cb + sps.qp_bd_offset_c,
                    self.qp_cr + sps.qp_bd_offset_c, int(self.cu_transquant_bypass_flag), int(self.pcm_flag)))
        if self.pcm_flag or not getattr(self, "rqt_root_cbf", 0):
            return
        for leaf in self.tu.get_leaves():           # depth-first = z-order (tree.py:48-54)
            tsf = getattr(leaf, "transform_skip_flag", None)
            ts = [int(tsf[c]) if tsf is not None else 0 for c in range(3)]
            tu_idx = len(tus)
            tus.append((cu_idx, leaf.x, leaf.y, leaf.log2size, leaf.depth, getattr(leaf, "idx", 0),
                        int(getattr(leaf, "cbf_luma", 0)), int(leaf.cbf_cb), int(leaf.cbf_cr), *ts))
            for c in range(3):
                arr = np.asarray(leaf.trans_coeff_level[c])       # [x][y] (x-major)
                xs, ys = np.nonzero(arr)
                for x, y in zip(xs, ys):
                    coefs.append((tu_idx, c, int(x), int(y), int(arr[x, y])))

    def ctu_parse(self):
        orig_ctu_parse(self)
        sh = self.ctx.img.slice_hdr
        hook(self.ctx).on_ctu_parsed(self, sh, self.ctx.pps)      # the maintainer's line at ctu.py:28
        s = self.sao
        sao_on = bool(sh.slice_sao_luma_flag or sh.slice_sao_chroma_flag)
        typ = [int(v) for v in s.sao_type_idx] if sao_on else [0, 0, 0]
        ab = [[int(v) for v in row] for row in s.sao_offset_abs] if sao_on else [[0] * 4] * 3
        sg = [[int(v) for v in row] for row in s.sao_offset_sign] if sao_on else [[0] * 4] * 3
        band = [int(v) for v in s.sao_band_position] if sao_on else [0, 0, 0]
        eo = [int(v) for v in s.sao_eo_class] if sao_on else [0, 0, 0]
        lf_across = getattr(sh, "slice_loop_filter_across_slices_enabled_flag",
                            self.ctx.pps.pps_loop_filter_across_slices_enabled_flag)
        ctus.append((state["frame"], self.addr_rs, self.slice_addr, int(sh.slice_sao_luma_flag),
                     int(sh.slice_sao_chroma_flag), int(lf_across),
                     int(getattr(sh, "slice_deblocking_filter_disabled_flag", 0)), sh.slice_qp_y,
                     *typ, *sum(ab, []), *sum(sg, []), *band, *eo))

    def sd_parse(self):
        eop = orig_sd_parse(self)
        if eop:
            hook(self.ctx).on_end_of_picture({"source": "sanity.bin", "frame": state["frame"]})   # slice.py:284-286
            state["frame"] += 1
        return eop

    cu_mod.Cu.decode_leaf = decode_leaf
    ctu_mod.Ctu.parse = ctu_parse
    slice_mod.SliceSegmentData.parse = sd_parse

    d = mods["dec"].Decoder(_Args())
    try:
        d.decode()
    except SystemExit:
        pass
    for h in list(mods["log"].main.handlers):
        h.flush()
    ctx = d.ctx
    t_dec = time.time() - t0

    # The reference's own regression check (Makefile:13-20), over all golden files.
    subprocess.run([sys.executable, "-B", os.path.join(_refshim.REF_ROOT, "tools", "gen_logs.py")],
                   cwd=os.path.join(WORK, "logs"), check=True,
                   env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    golden = sorted(os.listdir(GOLDEN_DIR))
    mismatch = [g for g in golden
                if not os.path.exists(os.path.join(WORK, "logs", g))
                or not filecmp.cmp(os.path.join(WORK, "logs", g), os.path.join(GOLDEN_DIR, g), shallow=False)]
    if mismatch:
        raise SystemExit("front-end trace differs from reference goldens: %s" % mismatch[:10])

    sps, pps = ctx.sps, ctx.pps
    params = dict(
        pic_width=sps.pic_width_in_luma_samples, pic_height=sps.pic_height_in_luma_samples,
        chroma_format_idc=sps.chroma_format_idc, bit_depth_luma=sps.bit_depth_y,
        bit_depth_chroma=sps.bit_depth_c, ctb_log2_size=sps.ctb_log2_size_y,
        min_cb_log2_size=sps.min_cb_log2_size_y,
        min_tb_log2_size=sps.log2_min_transform_block_size,
        max_tb_log2_size=sps.log2_max_transform_block_size,
        strong_intra_smoothing=int(sps.strong_intra_smoothing_enabled_flag),
        constrained_intra_pred=int(pps.constrained_intra_pred_flag),
        sample_adaptive_offset=int(sps.sample_adaptive_offset_enabled_flag),
        pcm_enabled=int(sps.pcm_enabled_flag), scaling_list_enabled=int(sps.scaling_list_enabled_flag),
        transform_skip_enabled=int(pps.transform_skip_enabled_flag),
        sign_data_hiding=int(pps.sign_data_hiding_enabled_flag),
        tiles_enabled=int(pps.tiles_enabled_flag),
        loop_filter_across_tiles=int(getattr(pps, "loop_filter_across_tiles_enabled_flag", 1)),
        pps_loop_filter_across_slices=int(pps.pps_loop_filter_across_slices_enabled_flag),
        deblocking_filter_control_present=int(pps.deblocking_filter_control_present_flag),
        n_frames=state["frame"])

    cu_dt = np.dtype([("frame", "u1"), ("ctu", "u2"), ("x", "u2"), ("y", "u2"), ("log2", "u1"),
                      ("part_mode", "u1"), ("mode_y", "u1", 4), ("mode_c", "u1"), ("qp_y", "u1"),
                      ("qp_cb", "u1"), ("qp_cr", "u1"), ("bypass", "u1"), ("pcm", "u1")])
    tu_dt = np.dtype([("cu", "u4"), ("x", "u2"), ("y", "u2"), ("log2", "u1"), ("depth", "u1"),
                      ("blk", "u1"), ("cbf", "u1", 3), ("tskip", "u1", 3)])
    coef_dt = np.dtype([("tu", "u4"), ("c", "u1"), ("x", "u1"), ("y", "u1"), ("v", "i2")])
    ctu_dt = np.dtype([("frame", "u1"), ("ctu", "u2"), ("slice_addr", "u2"), ("sao_luma", "u1"),
                       ("sao_chroma", "u1"), ("lf_across_slices", "u1"), ("deblock_disabled", "u1"),
                       ("slice_qp", "i1"), ("sao_type", "u1", 3), ("sao_abs", "u1", (3, 4)),
                       ("sao_sign", "u1", (3, 4)), ("sao_band", "u1", 3), ("sao_eo", "u1", 3)])

    def pack(rows, dt):
        out = np.zeros(len(rows), dt)
        for i, r in enumerate(rows):
            flat, k = list(r), 0
            rec = []
            for name in dt.names:
                shp = dt[name].shape
                n = int(np.prod(shp)) if shp else 1
                v = flat[k:k + n]
                k += n
                rec.append(np.array(v).reshape(shp) if shp else v[0])
            out[i] = tuple(rec)
        return out

    cu_a, tu_a, coef_a, ctu_a = pack(cus, cu_dt), pack(tus, tu_dt), pack(coefs, coef_dt), pack(ctus, ctu_dt)
    out = os.path.join(HERE, "sanity_frontend.npz")
    arrays = dict(cus=cu_a, tus=tu_a, coefs=coef_a, ctus=ctu_a, params=np.frombuffer(json.dumps(params).encode(), np.uint8))
    same = False
    if os.path.exists(out):
        old = np.load(out, allow_pickle=False)
        same = set(old.files) == set(arrays) and all(np.array_equal(old[k], v) and old[k].dtype == v.dtype
                                                     for k, v in arrays.items())
    if not same:
        np.savez_compressed(out, **arrays)
    print("capture %s the committed npz" % ("equals" if same else "REWROTE"))

    # the drop-in adapter, driven by the live reference objects, builds the same records
    _, rebuilt = frontend.pictures_from_frontend_npz(out)
    hooked = state["hook"].pictures
    if len(hooked) != len(rebuilt):
        raise SystemExit("ReconHook built %d pictures, capture %d" % (len(hooked), len(rebuilt)))
    for i, (a, b) in enumerate(zip(hooked, rebuilt)):
        for name in ("ctus", "tbs", "coef"):
            if not np.array_equal(getattr(a, name), getattr(b, name)):
                raise SystemExit("ReconHook records differ from the capture: picture %d %s" % (i, name))
        if (a.nofilter is None) != (b.nofilter is None) or (a.nofilter is not None and not np.array_equal(a.nofilter, b.nofilter)):
            raise SystemExit("ReconHook no-filter map differs: picture %d" % i)
    print("ReconHook records identical (%d pictures, %d TB records)" % (len(hooked), sum(len(p.tbs) for p in hooked)))
    with open(BITSTREAM, "rb") as f:
        bs_sha = hashlib.sha256(f.read()).hexdigest()
    old_meta = {}
    if os.path.exists(os.path.join(HERE, "sanity_frontend.json")):
        old_meta = json.load(open(os.path.join(HERE, "sanity_frontend.json")))
    meta = dict(old_meta)       # keeps fields other scripts add (pin_sanity_yuv.py: decoded-YUV hashes)
    meta.update(generator="tests/golden/gen_sanity_fixture.py", bitstream="reference:sanity.bin",
                bitstream_sha256=bs_sha, golden_files_checked=len(golden), golden_files_matching=len(golden),
                n_frames=state["frame"], n_cus=len(cus), n_tus=len(tus), n_nonzero_coefs=len(coefs),
                n_ctus=len(ctus), decode_seconds=round(t_dec, 1), params=params,
                npz_sha256=hashlib.sha256(open(out, "rb").read()).hexdigest(),
                reconhook_identical=True,
                reconhook_tb_records=int(sum(len(p.tbs) for p in hooked)))
    with open(os.path.join(HERE, "sanity_frontend.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
