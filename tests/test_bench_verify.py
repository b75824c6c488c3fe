"""bench.py's post-run output check (CPU): the verify path compares downloaded planes with the
C oracle, and a mismatch turns into a non-zero exit code (the line's value is then no result)."""
import importlib.util
import os

import numpy as np

from oracle import c_oracle
from p265_amd import synth
from p265_amd import records as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pictures_to_check_covers_both_ends():
    b = _bench()
    assert b.pictures_to_check(512, 4) == [0, 1, 2, 3, 508, 509, 510, 511]
    assert b.pictures_to_check(3, 4) == [0, 1, 2]
    assert b.pictures_to_check(8, 8) == list(range(8))


def test_verify_accepts_the_oracle_output_and_flags_a_corrupted_download():
    b = _bench()
    params = R.make_params(pic_width=128, pic_height=64)
    uniq = [synth.make_picture(params, 31 + i) for i in range(2)]
    pics = [uniq[i % 2] for i in range(5)]
    idx = b.pictures_to_check(len(pics), 2)
    ref = {id(p): out for p, (_, out) in zip(uniq, c_oracle.decode(params, uniq, with_recon=False))}
    got = {i: [np.array(pl) for pl in ref[id(pics[i])]] for i in idx}
    n, bad = b.verify_planes(params, pics, got, threads=2)
    assert (n, bad) == (4, [])
    got[3][1][5, 7] ^= 1                              # one Cb sample of picture 3 off by one bit
    n, bad = b.verify_planes(params, pics, got, threads=2)
    assert (n, bad) == (4, [3])
    # the exit path: a failed check makes bench.py exit non-zero
    assert b.exit_code({"verified": {"ok": False, "mismatches": ["batch 0 picture 3"]}}) == 3
    assert b.exit_code({"verified": {"ok": True}}) == 0
    assert b.exit_code({}) == 0                       # --no-verify: nothing claimed
