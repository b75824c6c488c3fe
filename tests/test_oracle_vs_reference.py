"""Pin the CPU oracle against golden vectors produced by the reference's own functions.

Vectors: tests/golden/ref_components.npz (BitDepth 8), ref_components_bd10.npz (Main 10:
BitDepth 10, QpBdOffset 12) and ref_components_bd12.npz (BitDepth 12, QpBdOffset 24), made by tests/golden/gen_component_fixture.py from
decoder/intra.py:82-305, decoder/scaling.py:4-47 and decoder/reconstruction.py:4-27 (only the cases
where the reference is a correct restatement of H.265; see the generator's docstring).  Bit-exact
equality is required.
"""
import os

import numpy as np
import pytest

from oracle import recon_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIXTURES = {8: np.load(os.path.join(GOLDEN, "ref_components.npz")),
            10: np.load(os.path.join(GOLDEN, "ref_components_bd10.npz")),
            12: np.load(os.path.join(GOLDEN, "ref_components_bd12.npz"))}
G = FIXTURES[8]


@pytest.mark.parametrize("bd", [8, 10, 12])
def test_tables_and_counts(bd):
    F = FIXTURES[bd]
    assert len(F["pred_n"]) >= 400 and len(F["filt_n"]) >= 300 and len(F["scal_n"]) >= 200
    if bd > 8:                                     # the high-bit-depth vectors really use their range
        assert F["pred_L"].max() > (1 << (bd - 1)) and F["rec_out"].max() == (1 << bd) - 1 and F["scal_qp"].max() > 51


@pytest.mark.parametrize("i", range(0, 480, 1))
def test_prediction_matches_reference(i):
    n, mode, c = int(G["pred_n"][i]), int(G["pred_mode"][i]), int(G["pred_c"][i])
    L = G["pred_L"][i][: 4 * n + 1].astype(np.int64)
    got = O.predict(L, n, mode, c, 8)
    np.testing.assert_array_equal(got, G["pred_out"][i][:n, :n], err_msg="n=%d mode=%d c=%d" % (n, mode, c))


@pytest.mark.parametrize("bd", [10, 12])
def test_prediction_matches_reference_high_bit_depth(bd):
    F = FIXTURES[bd]
    for i in range(len(F["pred_n"])):
        n, mode, c = int(F["pred_n"][i]), int(F["pred_mode"][i]), int(F["pred_c"][i])
        L = F["pred_L"][i][: 4 * n + 1].astype(np.int64)
        got = O.predict(L, n, mode, c, bd)
        np.testing.assert_array_equal(got, F["pred_out"][i][:n, :n], err_msg="n=%d mode=%d c=%d" % (n, mode, c))


@pytest.mark.parametrize("bd", [8, 10, 12])
def test_neighbour_substitution_and_filter_match_reference(bd):
    F = FIXTURES[bd]
    for i in range(len(F["filt_n"])):
        n, mode = int(F["filt_n"][i]), int(F["filt_mode"][i])
        m = 4 * n + 1
        avail = F["filt_avail"][i][:m].astype(bool)
        vals = F["filt_vals"][i][:m].astype(np.int64)
        p = O.substitute(np.where(avail, vals, 0), avail, bd)
        p = O.filter_refs(p, n, mode, 0, True, bd)
        np.testing.assert_array_equal(p, F["filt_out"][i][:m], err_msg="case %d n=%d mode=%d" % (i, n, mode))


@pytest.mark.parametrize("bd", [8, 10, 12])
def test_scaling_matches_reference(bd):
    F = FIXTURES[bd]
    for i in range(len(F["scal_n"])):
        n, qp = int(F["scal_n"][i]), int(F["scal_qp"][i])        # qP incl. QpBdOffset
        lvl = F["scal_level"][i][:n, :n]
        got = O.dequantize(lvl, qp, n.bit_length() - 1, bd)
        np.testing.assert_array_equal(got, F["scal_out"][i][:n, :n], err_msg="case %d" % i)


@pytest.mark.parametrize("bd", [8, 10, 12])
def test_reconstruction_clip_matches_reference(bd):
    F = FIXTURES[bd]
    got = np.clip(F["rec_pred"].astype(np.int64) + F["rec_res"], 0, (1 << bd) - 1)
    np.testing.assert_array_equal(got, F["rec_out"])
