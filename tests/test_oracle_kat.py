"""Known-answer tests of the CPU oracle for the parts the reference cannot pin.

The reference's inverse transform is numerically wrong (decoder/transform.py:81-109,
SURVEY.md Appendix A) and it has no SAO filter (decoder/sao.py is syntax only), so
these parts of oracle/recon_oracle.py are checked here against properties of the
H.265 transform and hand-worked cases instead (parity with the reference: unpinned).
"""
import numpy as np
import pytest

from oracle import recon_oracle as O


# ---------------------------------------------------------------------------------
# transform
# ---------------------------------------------------------------------------------

def test_dct_rows_nearly_orthogonal():
    m = O.DCT32
    g = m @ m.T
    off = g - np.diag(np.diag(g))
    assert np.all(np.diag(g) >= 130960) and np.all(np.diag(g) <= 131244)   # SURVEY §8(c) KAT
    assert np.abs(off).max() <= 400                                         # < 0.31 % of the diagonal


def test_sub_matrices_are_the_smaller_dcts():
    m = O.DCT32
    np.testing.assert_array_equal(m[[0, 8, 16, 24], :4], [[64] * 4, [83, 36, -36, -83], [64, -64, -64, 64],
                                                            [36, -83, 83, -36]])
    for log2 in (2, 3, 4):
        t = O.transform_matrix(log2, 0)
        n = 1 << log2
        # every row of the N-point matrix is symmetric (even k) or antisymmetric (odd k)
        for k in range(n):
            np.testing.assert_array_equal(t[k], (-1) ** k * t[k][::-1])


def _butterfly_inverse(x, log2):
    """Even/odd (partial butterfly) inverse DCT, written independently of the matrix form."""
    n = 1 << log2
    if n == 4:
        e0 = 64 * x[0] + 64 * x[2]
        e1 = 64 * x[0] - 64 * x[2]
        o0 = 83 * x[1] + 36 * x[3]
        o1 = 36 * x[1] - 83 * x[3]
        return np.array([e0 + o0, e1 + o1, e1 - o1, e0 - o0])
    even = _butterfly_inverse(x[0::2], log2 - 1)
    t = O.transform_matrix(log2, 0)
    odd = np.array([sum(t[2 * j + 1][k] * x[2 * j + 1] for j in range(n // 2)) for k in range(n // 2)])
    return np.concatenate([even + odd, (even - odd)[::-1]])


@pytest.mark.parametrize("log2", [2, 3, 4, 5])
def test_matrix_inverse_equals_butterfly(log2):
    rng = np.random.default_rng(log2)
    n = 1 << log2
    t = O.transform_matrix(log2, 0)
    for _ in range(20):
        x = rng.integers(-32768, 32768, n)
        np.testing.assert_array_equal(x @ t, _butterfly_inverse(x, log2))


def test_dst_formula_matches_hm_style_inverse():
    rng = np.random.default_rng(4)
    for _ in range(50):
        c = rng.integers(-2000, 2000, 4)
        c0, c1, c2, c3 = (int(v) for v in c)
        # HM-style fast inverse DST, written out
        k0, k1, k2, k3 = c0 + c2, c2 + c3, c0 - c3, 74 * c1
        exp = [29 * k0 + 55 * k1 + k3, 55 * k2 - 29 * k1 + k3, 74 * (c0 - c2 + c3), 55 * k0 + 29 * k2 - k3]
        np.testing.assert_array_equal(c @ O.DST4, exp)


@pytest.mark.parametrize("log2", [2, 3, 4, 5])
@pytest.mark.parametrize("c_idx", [0, 1])
def test_dc_only_gives_flat_residual(log2, c_idx):
    n = 1 << log2
    for dcv in (-500, -37, 1, 12, 300):
        lvl = np.zeros((n, n), np.int64)
        lvl[0, 0] = dcv
        r = O.residual_block(lvl, log2, c_idx, 30, O.TB_CBF, 8)
        if log2 == 2 and c_idx == 0:
            continue                              # luma 4x4 uses the DST: not flat
        assert np.all(r == r[0, 0]), (log2, c_idx, dcv)


def test_dc_value_known_answer():
    # 8x8, qP 30 (levelScale 40, shift 5): d = (64*16*40 << 5 + 2^5) >> 6 = 20480
    lvl = np.zeros((8, 8), np.int64)
    lvl[0, 0] = 64
    d = O.dequantize(lvl, 30, 3, 8)
    assert d[0, 0] == (64 * 16 * 40 * 32 + 32) >> 6
    r = O.residual_block(lvl, 3, 0, 30, O.TB_CBF, 8)
    e = (64 * int(d[0, 0]) + 64) >> 7
    assert np.all(r == (64 * e + 2048) >> 12)


def test_transform_skip_and_bypass():
    lvl = np.arange(16).reshape(4, 4) - 8
    r = O.residual_block(lvl, 2, 0, 4, O.TB_CBF | O.TB_TSKIP, 8)
    d = O.dequantize(lvl, 4, 2, 8)
    np.testing.assert_array_equal(r, ((d << 7) + 2048) >> 12)
    np.testing.assert_array_equal(O.residual_block(lvl, 2, 0, 4, O.TB_CBF | O.TB_BYPASS, 8), lvl)


def test_dequant_clips_to_int16():
    lvl = np.full((4, 4), 32767)
    assert O.dequantize(lvl, 51, 2, 8).max() == 32767
    assert O.dequantize(-lvl, 51, 2, 8).min() == -32768


# ---------------------------------------------------------------------------------
# intra prediction (hand-worked cases for modes the reference gets wrong)
# ---------------------------------------------------------------------------------

def _L(n, left, top, corner):
    """linear array from p[-1][0..2n-1] (left), p[0..2n-1][-1] (top), p[-1][-1]."""
    return np.array(list(left[::-1]) + [corner] + list(top), np.int64)


def test_vertical_mode_26_is_copy_with_edge_filter():
    n = 4
    top = [10, 20, 30, 40, 50, 60, 70, 80]
    left = [12, 14, 16, 18, 0, 0, 0, 0]
    p = _L(n, left, top, 8)
    pred = O.predict(p, n, 26, 0, 8)
    np.testing.assert_array_equal(pred[:, 1:], np.tile(top[1:4], (4, 1)))
    np.testing.assert_array_equal(pred[:, 0], [10 + ((v - 8) >> 1) for v in left[:4]])
    np.testing.assert_array_equal(O.predict(p, n, 26, 1, 8), np.tile(top[:4], (4, 1)))  # chroma: no edge filter


def test_diagonal_mode_34_and_2():
    n = 4
    top = list(range(100, 108))
    left = list(range(200, 208))
    p = _L(n, left, top, 50)
    pred34 = O.predict(p, n, 34, 1, 8)             # down-left from the top row: pred[y][x] = top[x + y + 1]
    for y in range(4):
        for x in range(4):
            assert pred34[y, x] == top[x + y + 1]
    pred2 = O.predict(p, n, 2, 1, 8)               # up-right from the left column: pred[y][x] = left[x + y + 1]
    for y in range(4):
        for x in range(4):
            assert pred2[y, x] == left[x + y + 1]


def test_mode_18_diagonal_down_right():
    n = 4
    top = list(range(100, 108))
    left = list(range(200, 208))
    p = _L(n, left, top, 50)
    pred = O.predict(p, n, 18, 1, 8)
    for y in range(4):
        for x in range(4):
            d = x - y
            exp = top[d - 1] if d > 0 else (50 if d == 0 else left[-d - 1])
            assert pred[y, x] == exp, (x, y)


def test_fractional_vertical_mode_with_negative_angle():
    # mode 23 (angle -9, invAngle -910) on nTbS 8: extension uses (x*invAngle+128)>>8
    n = 8
    rng = np.random.default_rng(1)
    p = rng.integers(0, 256, 4 * n + 1)
    pred = O.predict(p, n, 23, 1, 8)
    top = lambda x: int(p[2 * n + 1 + x])
    left = lambda y: int(p[2 * n - 1 - y])
    ref = {x: top(x - 1) for x in range(0, 2 * n + 1)}
    for x in range((n * -9) >> 5, 0):
        ref[x] = left(-1 + ((x * -910 + 128) >> 8))
    for y in range(n):
        idx, f = ((y + 1) * -9) >> 5, ((y + 1) * -9) & 31
        for x in range(n):
            exp = ((32 - f) * ref[x + idx + 1] + f * ref[x + idx + 2] + 16) >> 5 if f else ref[x + idx + 1]
            assert pred[y, x] == exp


def test_substitution_rules():
    av = np.array([0, 0, 1, 0, 1, 0, 0, 1, 0], bool)
    v = np.array([9, 9, 5, 9, 7, 9, 9, 3, 9])
    np.testing.assert_array_equal(O.substitute(v, av, 8), [5, 5, 5, 5, 7, 7, 7, 3, 3])
    np.testing.assert_array_equal(O.substitute(v, np.zeros(9, bool), 8), [128] * 9)


def test_strong_smoothing_bilinear():
    n = 32
    p = np.full(4 * n + 1, 100, np.int64)
    p[0] = 104           # p[-1][63]
    p[4 * n] = 96        # p[63][-1]
    f = O.filter_refs(p, n, 0, 0, True, 8)
    assert f[2 * n] == 100 and f[0] == 104 and f[4 * n] == 96
    for y in range(63):
        assert f[2 * n - 1 - y] == ((63 - y) * 100 + (y + 1) * 104 + 32) >> 6


# ---------------------------------------------------------------------------------
# SAO (8.7.3)
# ---------------------------------------------------------------------------------

def _one_ctb_pic(typ, cls, offs, ctb_log2=4):
    from p265_amd import records as R
    ctus = np.zeros(1, R.CTU_DTYPE)
    ctus["flags"] = 1
    ctus["sao_type"][0] = [typ, 0, 0]
    ctus["sao_class"][0] = [cls, 0, 0]
    ctus["sao_offset"][0][0] = offs
    params = dict(pic_width=16, pic_height=16, ctb_log2_size=ctb_log2, min_tb_log2_size=2,
                  sample_adaptive_offset=1, loop_filter_across_tiles=1, bit_depth_luma=8, bit_depth_chroma=8)
    return params, {"ctus": ctus, "tbs": np.zeros(0, R.TB_DTYPE), "coef": np.zeros(0, np.int16)}


def test_sao_band_offset():
    params, pic = _one_ctb_pic(1, 4, [1, 2, 3, 4])          # bands 4..7 = sample values 32..63
    rec = [np.arange(256).reshape(16, 16).astype(np.int64), np.zeros((8, 8), np.int64), np.zeros((8, 8), np.int64)]
    out = O.sao_picture(params, pic, rec)[0]
    v = rec[0]
    exp = v + np.where((v >> 3) == 4, 1, 0) + np.where((v >> 3) == 5, 2, 0) + np.where((v >> 3) == 6, 3, 0) \
        + np.where((v >> 3) == 7, 4, 0)
    np.testing.assert_array_equal(out, exp)


def test_sao_edge_offset_local_min_max_and_picture_edge():
    params, pic = _one_ctb_pic(2, 0, [3, 1, -1, -3])         # horizontal EO
    y = np.full((16, 16), 50, np.int64)
    y[5, 5] = 40        # local minimum -> edgeIdx 1 -> +3
    y[7, 7] = 60        # local maximum -> edgeIdx 4 -> -3
    y[9, 0] = 10        # on the picture edge (left neighbour outside): untouched
    rec = [y, np.zeros((8, 8), np.int64), np.zeros((8, 8), np.int64)]
    out = O.sao_picture(params, pic, rec)[0]
    assert out[5, 5] == 43 and out[7, 7] == 57 and out[9, 0] == 10
    assert out[5, 4] == 50 - 1 and out[5, 6] == 50 - 1        # edgeIdx 3 (greater than one neighbour) -> -1
    assert out[2, 2] == 50                                    # flat -> edgeIdx 0


# ---------------------------------------------------------------------------------
# Main 10 (BitDepth 10): hand-worked cases of the bit-depth-dependent steps
# ---------------------------------------------------------------------------------

def test_dequant_10bit_equals_8bit_at_qp_plus_qpbdoffset():
    # 8.6.3: d = (L * 16 * levelScale[qP % 6] << (qP / 6) + (1 << (bdShift - 1))) >> bdShift with
    # bdShift = BitDepth + log2 - 5: at BitDepth 10 and qP' = qP + 12 both shifts grow by 2 -- same d
    rng = np.random.default_rng(10)
    for log2 in (2, 3, 4, 5):
        lvl = rng.integers(-3000, 3000, (1 << log2, 1 << log2))
        for qp in range(0, 52, 3):
            np.testing.assert_array_equal(O.dequantize(lvl, qp + 12, log2, 10), O.dequantize(lvl, qp, log2, 8))


def test_dc_only_residual_10bit():
    # L = 1 at (0, 0), qP' 16, 4x4 DCT (chroma): d = (16 * 64 << 2 + 64) >> 7 = 32; stage 1: (64 * 32 + 64) >> 7
    # = 16; stage 2 (bdShift 20 - 10 = 10): (64 * 16 + 512) >> 10 = 1 in every sample (at 8 bits: 0)
    lvl = np.zeros((4, 4), np.int64)
    lvl[0, 0] = 1
    np.testing.assert_array_equal(O.residual_block(lvl, 2, 1, 16, 0x01, 10), np.ones((4, 4)))
    np.testing.assert_array_equal(O.residual_block(lvl, 2, 1, 4, 0x01, 8), np.zeros((4, 4)))


def test_sao_band_offset_10bit():
    # bandShift = BitDepth - 5 = 5: bands of 32 sample values; SaoOffsetVal as coded (shift 10 - Min(10, 10) = 0)
    params, pic = _one_ctb_pic(1, 4, [1, 2, 3, 31])
    params.update(bit_depth_luma=10, bit_depth_chroma=10)
    v = (np.arange(256).reshape(16, 16) * 4).astype(np.int64)          # 0 .. 1020
    rec = [v, np.zeros((8, 8), np.int64), np.zeros((8, 8), np.int64)]
    out = O.sao_picture(params, pic, rec)[0]
    exp = v + np.select([(v >> 5) == 4, (v >> 5) == 5, (v >> 5) == 6, (v >> 5) == 7], [1, 2, 3, 31], 0)
    np.testing.assert_array_equal(out, exp)
    from p265_amd import frontend
    assert frontend.sao_offset_val(1, [31, 2, 0, 5], [1, 0, 0, 1], 10) == [-31, 2, 0, -5]


def test_deblocking_thresholds_scale_with_bit_depth():
    # QpY 37 on both sides: beta' = 2 * 37 - 38 = 36, tC' = 4 (Q = 39).  A P side bent by 20 per line:
    # d = 40 >= 36 -> no filtering at 8 bits; at 10 bits beta = 144 -> filtered (8.7.2.5.3)
    p = [[100, 100, 100, 100], [110, 110, 110, 110], [100, 100, 100, 100], [100, 100, 100, 100]]
    q = [[104] * 4, [104] * 4, [104] * 4, [104] * 4]
    p8, q8 = O.deblock_luma_segment(p, q, 37, 37, 0, 0, False, False, 8)
    assert p8 == p and q8 == q
    p10, q10 = O.deblock_luma_segment(p, q, 37, 37, 0, 0, False, False, 10)
    assert p10 != p or q10 != q
    # chroma: QpC = Table 8-10(37) = 34, tC' = TC_TABLE[36] = 4, x 4 at 10 bits
    assert O.chroma_tc(37, 37, 0, 0, 8) == O.TC_TABLE[O.qpc_from_qpi(37) + 2] == 4
    assert O.chroma_tc(37, 37, 0, 0, 10) == 16
