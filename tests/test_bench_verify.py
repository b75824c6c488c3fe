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


def test_c5_one_k_for_every_rank():
    """Units that do not divide over the ranks (8 over 3: 3, 3, 2): every rank's batch carries its units of
    the SAME K steps (ceil(512 / 3) = 171), so the counted work (all units x K per run) is what the ranks
    decode; build_workload takes K from this function for every rank."""
    b = _bench()
    assert b.c5_steps_per_batch(512, 8, 3) == 171
    assert b.c5_steps_per_batch(512, 8, 1) == 64 and b.c5_steps_per_batch(512, 8, 8) == 512
    assert b.c5_steps_per_batch(0, 8, 3) == 1


def _run_bench(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("P265R_")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_bench_refuses_a_world_size_other_than_gpus():
    r = _run_bench(["--gpus", "2", "--no-cpu-baseline"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr and not r.stdout.strip()
    r = _run_bench(["--gpus", "1", "--no-cpu-baseline"], {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "--gpus 1" in r.stderr


def test_bench_refuses_more_ranks_than_devices_and_bad_device_maps():
    """--gpus N without a launcher spawns N ranks only when the devices exist (here: none visible), and never
    prints a line claiming fewer GPUs; a device map must name one device per rank, and ranks sharing a
    device must run without RCCL."""
    r = _run_bench(["--gpus", "8", "--no-cpu-baseline"])
    assert r.returncode == 2 and "needs 8 HIP device" in r.stderr and '"n_gpus"' not in r.stdout
    r = _run_bench(["--gpus", "2", "--device-map", "0"])
    assert r.returncode == 2 and "one device" in r.stderr
    r = _run_bench(["--gpus", "2", "--device-map", "0,x"])
    assert r.returncode == 2 and "comma-separated" in r.stderr
    r = _run_bench(["--gpus", "2", "--device-map", "0,0"])
    assert r.returncode == 2 and "--no-rccl" in r.stderr
    r = _run_bench(["--gpus", "2", "--device-map", "0,0", "--no-rccl"])
    assert r.returncode == 2 and "needs 1 HIP device" in r.stderr


def test_launch_ranks_sets_the_launcher_environment(monkeypatch):
    """The self-launch starts N children of bench.py with the environment torch.distributed.run gives its
    ranks and returns the worst exit code (children stubbed: no GPU here)."""
    import subprocess
    import types
    b = _bench()
    seen = []

    class FakeProc:
        def __init__(self, cmd, env, cwd):
            seen.append((cmd, env))
            self.returncode = 3 if env["RANK"] == "1" else 0

        def poll(self):
            return self.returncode

        def wait(self):
            return self.returncode

        def kill(self):
            pass

    monkeypatch.setattr(subprocess, "Popen", FakeProc)
    monkeypatch.setattr(b, "visible_devices", lambda: 4)
    a = types.SimpleNamespace(gpus=4, device_map=None, no_rccl=False)
    rc = b.launch_ranks(a, ["--gpus", "4", "--steps", "3"])
    assert rc == 3
    assert [e["RANK"] for _, e in seen] == ["0", "1", "2", "3"] == [e["LOCAL_RANK"] for _, e in seen]
    assert {e["WORLD_SIZE"] for _, e in seen} == {"4"} and {e["MASTER_ADDR"] for _, e in seen} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for _, e in seen}) == 1 and seen[0][0][-4:] == ["--gpus", "4", "--steps", "3"]
