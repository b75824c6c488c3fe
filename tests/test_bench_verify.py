"""bench.py's post-run output check (CPU): every timed picture's device digest is compared with the
digest of the C oracle's decode, a mismatch turns into a non-zero exit code (the line's value is then
no result), and the host digest (p265_amd/digest.py) is the function csrc/digest.h computes."""
import importlib.util
import os

import numpy as np

from oracle import c_oracle
from p265_amd import digest, synth
from p265_amd import records as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _mix64_py(z):
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & m
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & m
    return z ^ (z >> 31)


def test_plane_digest_is_the_documented_sum():
    rng = np.random.default_rng(5)
    plane = rng.integers(0, 256, (6, 12), dtype=np.uint8)
    want = 0
    for y in range(6):
        for k in range(3):
            word = int.from_bytes(bytes(plane[y, 4 * k:4 * k + 4]), "little")
            want = (want + _mix64_py(word | (y * 3 + k) << 32)) & ((1 << 64) - 1)
    assert digest.plane_digest(plane) == want


def test_plane_digest_sees_position():
    rng = np.random.default_rng(6)
    plane = rng.integers(0, 256, (8, 16), dtype=np.uint8)
    d0 = digest.plane_digest(plane)
    swapped = plane.copy()
    swapped[[2, 5]] = swapped[[5, 2]]                 # two rows swapped: same multiset of words
    assert digest.plane_digest(swapped) != d0
    flip = plane.copy()
    flip[7, 15] ^= 1
    assert digest.plane_digest(flip) != d0


def test_pictures_to_check_covers_both_ends():
    b = _bench()
    assert b.pictures_to_check(512, 4) == [0, 1, 2, 3, 508, 509, 510, 511]
    assert b.pictures_to_check(3, 4) == [0, 1, 2]
    assert b.pictures_to_check(8, 8) == list(range(8))


def test_verify_accepts_the_oracle_digests_and_flags_a_corrupted_picture():
    b = _bench()
    params = R.make_params(pic_width=128, pic_height=64)
    uniq = [synth.make_picture(params, 31 + i) for i in range(2)]
    pics = [uniq[i % 2] for i in range(5)]
    want = {id(p): digest.picture_digest(out) for p, (_, out) in zip(uniq, c_oracle.decode(params, uniq, with_recon=False))}
    got = np.stack([want[id(p)] for p in pics])       # what a correct device run returns
    assert b.digest_mismatches(pics, want, got) == []
    planes = [np.array(pl) for pl in c_oracle.decode(params, [pics[3]], with_recon=False)[0][1]]
    planes[1][5, 7] ^= 1                              # one Cb sample of picture 3 off by one bit
    got[3] = digest.picture_digest(planes)
    assert b.digest_mismatches(pics, want, got) == [3]
    # the exit path: a failed check makes bench.py exit non-zero
    assert b.exit_code({"verified": {"ok": False, "mismatches": ["batch 0 picture 3"]}}) == 3
    assert b.exit_code({"verified": {"ok": True}}) == 0
    assert b.exit_code({}) == 0                       # --no-verify: nothing claimed


def test_c5_batches_carry_consecutive_steps():
    """C5 workload: a rank's batch carries its units of K consecutive steps, so one launch fills the GPU
    even at one unit per rank and step; --c5-world N reproduces rank 0's share of an N-rank job."""
    import types
    b = _bench()
    a = types.SimpleNamespace(workload="c5", c5_frames=2, c5_batch_units=512, c5_world=8, deblocking=False)
    groups, (_, step_pics, _), cfg = b.build_workload(a, 0, 1)
    assert cfg["units_per_rank_step"] == 1 and cfg["steps_per_batch"] == 512
    assert len(groups[0][1]) == 512 and len(step_pics) == 1
    assert cfg["simulated_world"]["world"] == 8
    a.c5_world, a.c5_batch_units = 0, 512
    groups, (_, step_pics, _), cfg = b.build_workload(a, 0, 1)
    assert cfg["units_per_rank_step"] == 8 and cfg["steps_per_batch"] == 64 and len(groups[0][1]) == 512
    assert sorted(cfg["tiles"]) == ["1920x1072", "1920x1088"]
    a.c5_batch_units = 0                              # latency regime: one step per batch
    groups, _, cfg = b.build_workload(a, 0, 1)
    assert cfg["steps_per_batch"] == 1 and len(groups[0][1]) == 8
