"""Pin the CPU oracle against golden vectors produced by the reference's own functions.

Vectors: tests/golden/ref_components.npz, made by tests/golden/gen_component_fixture.py
from decoder/intra.py:82-305, decoder/scaling.py:4-47 and decoder/reconstruction.py:4-27
(only the cases where the reference is a correct restatement of H.265; see the
generator's docstring).  Bit-exact equality is required.
"""
import os

import numpy as np
import pytest

from oracle import recon_oracle as O

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_components.npz"))


def test_tables_and_counts():
    assert len(G["pred_n"]) >= 400 and len(G["filt_n"]) >= 300 and len(G["scal_n"]) >= 200


@pytest.mark.parametrize("i", range(0, 480, 1))
def test_prediction_matches_reference(i):
    n, mode, c = int(G["pred_n"][i]), int(G["pred_mode"][i]), int(G["pred_c"][i])
    L = G["pred_L"][i][: 4 * n + 1].astype(np.int64)
    got = O.predict(L, n, mode, c, 8)
    np.testing.assert_array_equal(got, G["pred_out"][i][:n, :n], err_msg="n=%d mode=%d c=%d" % (n, mode, c))


def test_neighbour_substitution_and_filter_match_reference():
    for i in range(len(G["filt_n"])):
        n, mode = int(G["filt_n"][i]), int(G["filt_mode"][i])
        m = 4 * n + 1
        avail = G["filt_avail"][i][:m].astype(bool)
        vals = G["filt_vals"][i][:m].astype(np.int64)
        p = O.substitute(np.where(avail, vals, 0), avail, 8)
        p = O.filter_refs(p, n, mode, 0, True, 8)
        np.testing.assert_array_equal(p, G["filt_out"][i][:m], err_msg="case %d n=%d mode=%d" % (i, n, mode))


def test_scaling_matches_reference():
    for i in range(len(G["scal_n"])):
        n, qp = int(G["scal_n"][i]), int(G["scal_qp"][i])
        lvl = G["scal_level"][i][:n, :n]
        got = O.dequantize(lvl, qp, n.bit_length() - 1, 8)
        np.testing.assert_array_equal(got, G["scal_out"][i][:n, :n], err_msg="case %d" % i)


def test_reconstruction_clip_matches_reference():
    got = np.clip(G["rec_pred"].astype(np.int64) + G["rec_res"], 0, 255)
    np.testing.assert_array_equal(got, G["rec_out"])
