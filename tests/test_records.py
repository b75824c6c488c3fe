"""Host-side record building (the decode_leaf hook) and validation, CPU only."""
import os

import numpy as np
import pytest

from p265_amd import frontend, synth
from p265_amd import records as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def sanity():
    return frontend.pictures_from_frontend_npz(os.path.join(GOLDEN, "sanity_frontend.npz"))


def test_sanity_front_end_statistics_match_the_reference_stream(sanity):
    """Counts from SURVEY.md Appendix B (measured on the reference's own parse)."""
    params, pics = sanity
    assert (int(params["pic_width"]), int(params["pic_height"]), int(params["ctb_log2_size"])) == (352, 288, 6)
    tbs = np.concatenate([p.tbs for p in pics])
    luma = tbs[tbs["c_idx"] == 0]
    cnt = {(lg, cb): int(((luma["log2_size"] == lg) & ((luma["flags"] & 1) == cb)).sum())
           for lg in (2, 3, 4, 5) for cb in (0, 1)}
    assert cnt == {(2, 1): 3616, (2, 0): 1364, (3, 1): 1190, (3, 0): 269, (4, 1): 297, (4, 0): 15,
                   (5, 1): 50, (5, 0): 0}
    assert int(((luma["flags"] & R.TB_TSKIP) != 0).sum()) == 41
    nz = {c: int(sum(np.count_nonzero(p.coef[int(t["coef_off"]): int(t["coef_off"]) + (1 << 2 * int(t["log2_size"]))])
                     for p in pics for t in p.tbs[(p.tbs["c_idx"] == c) & ((p.tbs["flags"] & 1) != 0)]))
          for c in range(3)}
    assert nz == {0: 13021 + 9822 + 12269 + 10250, 1: 432 + 151 + 105, 2: 480 + 281 + 344}
    # luma area covers the 3 pictures exactly
    assert int(np.sum(1 << (2 * luma["log2_size"].astype(np.int64)))) == 3 * 352 * 288
    sao = np.concatenate([p.ctus["sao_type"] for p in pics])
    combos = {}
    for row in sao:
        combos[tuple(int(v) for v in row)] = combos.get(tuple(int(v) for v in row), 0) + 1
    assert combos == {(0, 0, 0): 2, (1, 0, 0): 14, (2, 0, 0): 57, (2, 1, 1): 10, (2, 2, 2): 7}


def test_chroma_area_and_decode_order(sanity):
    params, pics = sanity
    for p in pics:
        for c in (1, 2):
            t = p.tbs[p.tbs["c_idx"] == c]
            assert int(np.sum(1 << (2 * t["log2_size"].astype(np.int64)))) == 176 * 144
        # within each CTU: Cb and Cr TBs come in adjacent pairs with identical geometry
        for ctu in p.ctus:
            tb = p.tbs[int(ctu["tb_begin"]): int(ctu["tb_begin"]) + int(ctu["tb_count"])]
            idx = np.nonzero(tb["c_idx"] == 1)[0]
            assert np.all(tb["c_idx"][idx + 1] == 2)
            for f in ("x", "y", "log2_size", "pred_mode"):
                assert np.all(tb[f][idx] == tb[f][idx + 1])


def test_eo_signs_inferred_and_bo_signs_kept():
    assert frontend.sao_offset_val(2, [1, 2, 3, 4], [1, 1, 0, 0], 8) == [1, 2, -3, -4]
    assert frontend.sao_offset_val(1, [1, 2, 3, 4], [1, 0, 1, 0], 8) == [-1, 2, -3, 4]
    assert frontend.sao_offset_val(1, [31, 0, 0, 0], [0, 0, 0, 0], 12) == [124, 0, 0, 0]


def test_chroma_qp_table():
    assert [frontend.qpc_from_qpi(q) for q in range(28, 46)] == [28, 29, 29, 30, 31, 32, 33, 33, 34, 34, 35, 35,
                                                                  36, 36, 37, 37, 38, 39]


def test_validation_rejects_bad_records():
    params = R.make_params(pic_width=64, pic_height=64)
    pic = synth.make_picture(params, 1)
    R.validate(params, pic)
    for field, val in (("x", 70), ("log2_size", 6), ("c_idx", 3), ("pred_mode", 35)):
        bad = R.Picture(pic.ctus.copy(), pic.tbs.copy(), pic.coef)
        bad.tbs[field][0] = val
        with pytest.raises(R.RecordError):
            R.validate(params, bad)
    bad = R.Picture(pic.ctus.copy(), pic.tbs.copy(), pic.coef)
    coded = np.nonzero(bad.tbs["flags"] & 1)[0][0]
    bad.tbs["coef_off"][coded] = len(pic.coef)
    with pytest.raises(R.RecordError):
        R.validate(params, bad)
    with pytest.raises(R.RecordError):
        R.validate(params, R.Picture(pic.ctus[:0], pic.tbs, pic.coef))
    # 4:2:0 chroma TBs stop at 16x16; a CTU cannot list more TBs than 1.5 per 4x4 luma unit
    bad = R.Picture(pic.ctus.copy(), pic.tbs.copy(), pic.coef)
    k = int(np.nonzero(bad.tbs["c_idx"] > 0)[0][0])
    bad.tbs["log2_size"][k], bad.tbs["x"][k], bad.tbs["y"][k] = 5, 0, 0
    with pytest.raises(R.RecordError):
        R.validate(params, bad)
    reps = 385 // len(pic.tbs) + 1
    bad = R.Picture(pic.ctus.copy(), np.concatenate([pic.tbs] * reps), pic.coef)
    bad.ctus["tb_count"][0] = 385
    with pytest.raises(R.RecordError):
        R.validate(params, bad)
    # ... nor more chroma TBs than 4x4 chroma units (128 at CTB 64: intra_prep.h kMaxCtuChroma)
    with pytest.raises(R.RecordError):
        R.validate(params, chroma_overfull(pic))


def chroma_overfull(pic):
    """CTU 0 lists 129 chroma 4x4 TBs (all at its origin) and nothing else."""
    k = int(np.nonzero((pic.tbs["c_idx"] == 1) & (pic.ctus["tb_begin"][0] <= np.arange(len(pic.tbs))))[0][0])
    one = pic.tbs[k:k + 1].copy()
    one["log2_size"], one["x"], one["y"], one["flags"] = 2, 0, 0, 0
    tbs = np.concatenate([np.repeat(one, 129), pic.tbs])
    ctus = pic.ctus.copy()
    ctus["tb_begin"] += 129
    ctus["tb_begin"][0], ctus["tb_count"][0] = 0, 129
    return R.Picture(ctus, tbs, pic.coef)


def test_synthetic_mix_follows_the_sanity_statistics():
    params = R.make_params(pic_width=640, pic_height=384)
    pic = synth.make_picture(params, 5, perf=True)
    luma = pic.tbs[pic.tbs["c_idx"] == 0]
    area = {lg: float(np.sum(luma["log2_size"] == lg) * 4 ** lg / (640 * 384)) for lg in (2, 3, 4, 5)}
    for lg, target in {2: 0.262, 3: 0.307, 4: 0.263, 5: 0.168}.items():
        assert abs(area[lg] - target) < 0.07, (lg, area)


def test_chroma_sao_must_share_type_and_class():
    params = R.make_params(pic_width=64, pic_height=64)
    pic = synth.make_picture(params, 3)
    R.validate(params, pic)
    for typ, cls in (((0, 2, 1), (0, 0, 0)), ((0, 2, 2), (0, 1, 3))):
        bad = R.Picture(ctus=pic.ctus.copy(), tbs=pic.tbs, coef=pic.coef)
        bad.ctus["sao_type"][0] = typ
        bad.ctus["sao_class"][0] = cls
        with pytest.raises(R.RecordError):
            R.validate(params, bad)
