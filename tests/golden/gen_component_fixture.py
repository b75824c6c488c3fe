#!/usr/bin/env python3
"""Golden vectors from the reference's own hot-path functions (THIS CONTAINER ONLY).

The reference's reconstruction never runs end to end (decoder/cu.py:487-488) and is
wrong in places, but several of its functions are correct
restatements of H.265 and can be called in isolation with stand-in PU objects:

  * IntraPu.decode_intra_planar            decoder/intra.py:82-94
  * IntraPu.decode_intra_dc                decoder/intra.py:96-122
  * IntraPu.decode_intra_angular           decoder/intra.py:124-184, for the modes it gets
    right: 2..17 (mode 10 only for chroma or nTbS 32, intra.py:184 calls an undefined
    clip), 18 and 26 (the vertical family with iFact != 0 is wrong, intra.py:155-158;
    mode 34 reads past its ref dict)
  * IntraPu.decode_neighbor                decoder/intra.py:186-305, luma, for availability
    patterns where p[-1][2N-1] is unavailable or nothing is missing (the substitution
    indentation defect, intra.py:243-255, only shows otherwise)
  * scaling.inverse_scaling                decoder/scaling.py:4-47
  * reconstruction.reconstruction          decoder/reconstruction.py:4-27

This script feeds them seeded random inputs, stores inputs + the reference's outputs
in tests/golden/ref_components.npz, and asserts at generation time that the tables of
oracle/recon_oracle.py equal the reference's (transform.py:5-72, intra.py:15-22).

Usage:  PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/gen_component_fixture.py [--bit-depth 10]

--bit-depth 10 (Main 10) and 12 write ref_components_bd10.npz / bd12.npz (+ .json): the same functions with the SPS's
BitDepthY = BitDepthC = 10 and QpBdOffset = 12 (scaling.py:14-26 bdShift and qP, reconstruction.py:25
and utils.py:11-15 clip, intra.py:241 substitution default, intra.py:280-281 strong-filter threshold,
intra.py:160 edge-filter clip), samples 0..1023 and QpY -12..51.  The 8-bit run is unchanged.
"""
import contextlib
import hashlib
import importlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import _refshim  # noqa: E402
from oracle import recon_oracle as O  # noqa: E402

SEED = 265


class _NS:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _md(neigh):
    """reference-style x-major neighbour dict from linear L."""
    n = (len(neigh) - 1) // 4
    d = {}
    dx, dy = O.ref_positions(n)
    for k in range(len(neigh)):
        d.setdefault(int(dx[k]), {})[int(dy[k])] = int(neigh[k])
    return d


def main(bd=8):
    mods = _refshim.install("/tmp/p265_component_fixture")
    _refshim.silence(mods)
    intra, scaling, transform, recon = mods["intra"], mods["scaling"], mods["transform"], mods["reconstruction"]

    # ---- tables --------------------------------------------------------------------
    assert np.array_equal(np.array(transform.trans_matrix_type0), O.DCT32), "DCT32 differs"
    assert np.array_equal(np.array(transform.trans_matrix_type1), O.DST4), "DST4 differs"
    assert list(intra.IntraPu.pred_angle_table) == O.INTRA_PRED_ANGLE
    assert list(intra.IntraPu.inv_angle_table) == O.INV_ANGLE

    rng = np.random.default_rng(SEED)
    sh = bd - 8                                        # sample ranges scale with the bit depth (0 at 8 bits)
    off = 6 * sh                                       # QpBdOffsetY / QpBdOffsetC
    mx = (1 << bd) - 1
    dt = np.uint8 if bd == 8 else np.uint16
    sps = _NS(bit_depth_y=bd, bit_depth_c=bd, strong_intra_smoothing_enabled_flag=1, qp_bd_offset_y=off,
              qp_bd_offset_c=off, scaling_list_enabled_flag=0)

    # ---- prediction ----------------------------------------------------------------
    modes_ok = [0, 1] + list(range(2, 18)) + [18, 26]
    P_n, P_mode, P_c, P_L, P_out = [], [], [], [], []
    for case in range(480):
        n = [4, 8, 16, 32][case % 4]
        mode = modes_ok[(case // 4) % len(modes_ok)]
        c_idx = int(rng.integers(0, 2))
        if mode == 10 and c_idx == 0 and n < 32:
            c_idx = 1
        style = case % 3                    # smooth ramps / random / near-flat
        if style == 0:
            base = rng.integers(0, 200 << sh)
            L = np.clip(base + np.cumsum(rng.integers(-3, 4, 4 * n + 1)), 0, mx)
        elif style == 1:
            L = rng.integers(0, mx + 1, 4 * n + 1)
        else:
            L = np.clip((128 << sh) + rng.integers(-2, 3, 4 * n + 1), 0, mx)
        cu = _NS(ctx=_NS(sps=sps))
        pu = intra.IntraPu(cu, c_idx, mode, int(np.log2(n)), 0, 0)
        nb = _md(L)
        if mode == 0:
            pu.decode_intra_planar(nb, 0, 0, int(np.log2(n)))
        elif mode == 1:
            pu.decode_intra_dc(nb, 0, 0, int(np.log2(n)))
        else:
            pu.decode_intra_angular(nb, 0, 0, int(np.log2(n)))
        out = np.zeros((32, 32), dt)
        out[:n, :n] = np.asarray(pu.predicted_samples).T        # -> [y][x]
        Lp = np.zeros(129, dt)
        Lp[: 4 * n + 1] = L
        P_n.append(n); P_mode.append(mode); P_c.append(c_idx); P_L.append(Lp); P_out.append(out)

    # ---- neighbour substitution + filtering (luma) -----------------------------------
    F_n, F_mode, F_avail, F_vals, F_out = [], [], [], [], []
    for case in range(360):
        n = [4, 8, 16, 32][case % 4]
        mode = int(rng.integers(0, 35))
        kind = (case // 4) % 4
        m = 4 * n + 1
        if kind == 0:
            avail = np.ones(m, bool)
        elif kind == 1:
            avail = np.zeros(m, bool)
        elif kind == 2:                     # typical: bottom-left run missing
            avail = np.ones(m, bool)
            avail[: int(rng.integers(1, 2 * n + 1))] = False
        else:                               # random, first entry missing
            avail = rng.random(m) < 0.6
            avail[0] = False
        style = case % 2
        if style == 0:
            vals = np.clip(rng.integers(20 << sh, 230 << sh) + np.cumsum(rng.integers(-1, 2, m)), 0, mx)
        else:
            vals = rng.integers(0, mx + 1, m)
        dx, dy = O.ref_positions(n)
        x0 = y0 = 64
        lut = {(x0 + int(a), y0 + int(b)): (bool(av), int(v)) for a, b, av, v in zip(dx, dy, avail, vals)}
        img = _NS(check_availability=lambda xc, yc, xn, yn: lut[(xn, yn)][0],
                  get_ctu=lambda xn, yn: _NS(
                      get_pred_mode=lambda x, y: 1,
                      get_leaf_cu=lambda x, y: _NS(get_reconstructed_sample=lambda xx, yy, c: lut[(xx, yy)][1])))
        cu = _NS(ctx=_NS(sps=sps, img=img, pps=_NS(constrained_intra_pred_flag=0)), MODE_INTRA=1)
        pu = intra.IntraPu(cu, 0, mode, int(np.log2(n)), x0, y0)
        with contextlib.redirect_stdout(io.StringIO()):
            nb = pu.decode_neighbor(x0, y0, int(np.log2(n)), 0)
        got = np.array([nb[int(a)][int(b)] for a, b in zip(dx, dy)], np.int64)
        pad = lambda a, dt: np.pad(np.asarray(a, dt), (0, 129 - m))
        F_n.append(n); F_mode.append(mode); F_avail.append(pad(avail, np.uint8)); F_vals.append(pad(vals, dt))
        F_out.append(pad(got, dt))

    # ---- scaling ---------------------------------------------------------------------
    S_n, S_qp, S_c, S_lvl, S_out = [], [], [], [], []
    for case in range(240):
        n = [4, 8, 16, 32][case % 4]
        qp = int(rng.integers(-off, 52))                  # QpY; the reference adds QpBdOffset (scaling.py:14-18)
        c_idx = int(rng.integers(0, 3))
        lvl = np.zeros((n, n), np.int64)
        mask = rng.random((n, n)) < 0.3
        mag = rng.geometric(0.3, (n, n))
        if case % 5 == 0:
            mag = rng.integers(1, 32768, (n, n))          # large levels: exercise the clip
        lvl[mask] = (mag * rng.choice([-1, 1], (n, n)))[mask]
        lvl = np.clip(lvl, -32768, 32767)
        tu = _NS(get_trans_coeff_level=lambda x, y, c: int(lvl[y, x]))    # [y][x] here, (x,y) there
        cu = _NS(ctx=_NS(sps=sps), tu=tu, qp_y=qp, qp_cb=qp, qp_cr=qp, cu_transquant_bypass_flag=0)
        pu = intra.IntraPu(cu, c_idx, 0, int(np.log2(n)), 0, 0)
        scaling.inverse_scaling(pu=pu, x0=0, y0=0, log2size=int(np.log2(n)))
        out = np.zeros((32, 32), np.int16)
        out[:n, :n] = np.asarray(pu.scaled_samples).T
        lp = np.zeros((32, 32), np.int16)
        lp[:n, :n] = lvl
        S_n.append(n); S_qp.append(qp + off); S_c.append(c_idx); S_lvl.append(lp); S_out.append(out)   # qP

    # ---- reconstruction clip -----------------------------------------------------------
    R_pred = rng.integers(0, mx + 1, (64, 8, 8))
    R_res = rng.integers(-300 << sh, 300 << sh, (64, 8, 8))
    R_out = []
    for i in range(64):
        cu = _NS(ctx=_NS(sps=sps))
        pu = intra.IntraPu(cu, i % 3, 0, 3, 0, 0)
        pu.predicted_samples[:] = R_pred[i].T
        pu.transformed_samples[:] = R_res[i].T
        recon.reconstruction(pu, 0, 0, 3)
        R_out.append(np.asarray(pu.reconstructed_samples).T.astype(dt))

    tag = "" if bd == 8 else "_bd%d" % bd
    out = os.path.join(HERE, "ref_components%s.npz" % tag)
    np.savez_compressed(
        out,
        pred_n=np.array(P_n, np.uint8), pred_mode=np.array(P_mode, np.uint8), pred_c=np.array(P_c, np.uint8),
        pred_L=np.array(P_L), pred_out=np.array(P_out),
        filt_n=np.array(F_n, np.uint8), filt_mode=np.array(F_mode, np.uint8), filt_avail=np.array(F_avail),
        filt_vals=np.array(F_vals), filt_out=np.array(F_out),
        scal_n=np.array(S_n, np.uint8), scal_qp=np.array(S_qp, np.uint8), scal_c=np.array(S_c, np.uint8),
        scal_level=np.array(S_lvl), scal_out=np.array(S_out),
        rec_pred=R_pred.astype(dt), rec_res=R_res.astype(np.int16), rec_out=np.array(R_out))
    meta = dict(generator="tests/golden/gen_component_fixture.py", seed=SEED,
                tables_match_reference=["transform.py:5 DST4", "transform.py:7-72 DCT32",
                                        "intra.py:15-18 intraPredAngle", "intra.py:19-22 invAngle"],
                cases=dict(pred=len(P_n), filter=len(F_n), scaling=len(S_n), reconstruction=64),
                bit_depth=bd, strong_intra_smoothing=1,
                npz_sha256=hashlib.sha256(open(out, "rb").read()).hexdigest())
    with open(os.path.join(HERE, "ref_components%s.json" % tag), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1))


def main_scaling():
    """--scaling: the ScalingFactor branch of scaling.inverse_scaling (scaling.py:32-44, m[x][y] =
    sps.scaling_factor[size_id][matrix_id][x][y]) on seeded random factors (1..255) and levels, 8 and 10
    bits, every size and intra component; and the default scaling lists of sld.py (Table 7-5 / 7-6, data).
    Writes ref_scaling.npz / .json."""
    mods = _refshim.install("/tmp/p265_component_fixture")
    _refshim.silence(mods)
    intra, scaling, sld = mods["intra"], mods["scaling"], importlib.import_module("sld")
    rng = np.random.default_rng(SEED + 1)
    cases = dict(n=[], qp=[], c=[], bd=[], level=[], m=[], out=[])
    for case in range(200):
        n = [4, 8, 16, 32][case % 4]
        log2 = int(np.log2(n))
        c_idx = 0 if n == 32 else int(rng.integers(0, 3))
        bd = 8 if case % 2 == 0 else 10
        off = 6 * (bd - 8)
        qp = int(rng.integers(-off, 52))
        sf = np.zeros((4, 6, 32, 32), np.int64)
        mx = rng.integers(1, 256, (n, n))                 # [x][y] as the reference indexes it
        sf[log2 - 2][c_idx][:n, :n] = mx
        sps = _NS(bit_depth_y=bd, bit_depth_c=bd, qp_bd_offset_y=off, qp_bd_offset_c=off,
                  scaling_list_enabled_flag=1, scaling_factor=sf)
        lvl = np.zeros((n, n), np.int64)
        mask = rng.random((n, n)) < 0.4
        mag = rng.geometric(0.2, (n, n)) if case % 5 else rng.integers(1, 32768, (n, n))
        lvl[mask] = (mag * rng.choice([-1, 1], (n, n)))[mask]
        lvl = np.clip(lvl, -32768, 32767)
        tu = _NS(get_trans_coeff_level=lambda x, y, c: int(lvl[y, x]))
        cu = _NS(ctx=_NS(sps=sps), tu=tu, qp_y=qp, qp_cb=qp, qp_cr=qp, cu_transquant_bypass_flag=0,
                 is_intra_mode=lambda: True)
        pu = intra.IntraPu(cu, c_idx, 0, log2, 0, 0)
        scaling.inverse_scaling(pu=pu, x0=0, y0=0, log2size=log2)
        out = np.zeros((32, 32), np.int16)
        out[:n, :n] = np.asarray(pu.scaled_samples).T
        pad = np.zeros((32, 32), np.int64)
        pad[:n, :n] = lvl
        mpad = np.zeros((32, 32), np.uint8)
        mpad[:n, :n] = mx.T                               # stored [y][x]
        for k, v in (("n", n), ("qp", qp + off), ("c", c_idx), ("bd", bd), ("level", pad.astype(np.int16)),
                     ("m", mpad), ("out", out)):
            cases[k].append(v)
    d = sld.ScalingListData
    out = os.path.join(HERE, "ref_scaling.npz")
    np.savez_compressed(out, n=np.array(cases["n"], np.uint8), qp=np.array(cases["qp"], np.uint8),
                        c=np.array(cases["c"], np.uint8), bd=np.array(cases["bd"], np.uint8),
                        level=np.array(cases["level"]), m=np.array(cases["m"]), out=np.array(cases["out"]),
                        default_4x4=np.array(d.default_scaling_list_4x4, np.uint8),
                        default_8x8_intra=np.array(d.default_scaling_list_8x8_intra, np.uint8),
                        default_8x8_inter=np.array(d.default_scaling_list_8x8_inter, np.uint8))
    meta = dict(generator="tests/golden/gen_component_fixture.py --scaling", seed=SEED + 1, cases=len(cases["n"]),
                functions=["scaling.py:4-47 (ScalingFactor branch, scaling.py:32-44)",
                           "sld.py:4-33 default_scaling_list_* (Table 7-5 / 7-6)"],
                npz_sha256=hashlib.sha256(open(out, "rb").read()).hexdigest())
    with open(os.path.join(HERE, "ref_scaling.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--bit-depth", type=int, default=8, choices=(8, 10, 12))
    ap.add_argument("--scaling", action="store_true", help="the ScalingFactor vectors (ref_scaling.npz) instead")
    args = ap.parse_args()
    if args.scaling:
        main_scaling()
    else:
        main(args.bit_depth)
