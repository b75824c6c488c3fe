"""Multi-process product path on the GPU box (named to run FIRST in a -m gpu session, so
the rank processes start before this process has touched the GPU).

* Two rank processes (tests/multirank_worker.py, plain child processes with a stdlib-socket
  rendezvous) decode through libp265r.so on device 0: the C4 picture shard, the C5 tile-unit
  shard of tests/golden/synth_4k_tiles.bin and the C5 halo exchange with
  loop_filter_across_tiles_enabled_flag = 1.  The gathered results must equal the C oracle /
  the stream's MD5 SEI.
* bench.py's multi-rank branch (two rank processes on device 0, control plane only: two RCCL
  ranks cannot share a device): barrier + MAX over ranks, the whole-job value and the post-run
  output check of both ranks.
* A one-rank RCCL communicator (ctypes librccl.so.1, no PyTorch) broadcasts the params POD
  through a hipMalloc'd buffer.  Multi-rank RCCL needs one device per rank: it runs in
  bench.py on an 8-GPU node, not here.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import c_oracle
from p265_amd import bitstream, halo, synth, tiles
from p265_amd import records as R

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _planes(path):
    z = np.load(path)
    return [z["arr_%d" % c] for c in range(3)]


def test_two_rank_processes_decode_their_shards(tmp_path):
    from ranks import free_port
    port = free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   P265_CTRL_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "multirank_worker.py"),
                                       str(tmp_path), "--device", "0"], env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out)
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)[-3000:]
    res = json.load(open(tmp_path / "result.json"))
    assert res["world"] == 2 and res["width"] == 320
    # C4: every picture decoded once, equal to the oracle
    params = R.make_params(pic_width=320, pic_height=192)
    ref = c_oracle.decode(params, [synth.make_picture(params, 900 + f) for f in range(6)], with_recon=False)
    assert sorted(res["c4"]) == [str(f) for f in range(6)]
    for f in range(6):
        assert res["c4"][str(f)] == hashlib.sha256(b"".join(ref[f][1][c].tobytes() for c in range(3))).hexdigest()
    # C5: 8 tile units over the two ranks, stitched pictures reproduce the MD5 SEI
    pics = bitstream.decode_stream(open(os.path.join(ROOT, "tests", "golden", "synth_4k_tiles.bin"), "rb").read())
    assert len(res["c5"]) == 8 and sorted(set(res["c5"].values())) == [0, 1]
    for f, p in enumerate(pics):
        parts = tiles.split(p.params, p.picture)
        full = tiles.stitch(p.params, parts, [_planes(tmp_path / ("c5_%d_%d.npz" % (f, t))) for t in range(len(parts))])
        assert [hashlib.md5(np.ascontiguousarray(full[c]).tobytes()).digest() for c in range(3)] == p.hash
    # C5 halo exchange: every tile's filtered output equals whole-picture decoding
    hp = R.make_params(pic_width=264, pic_height=200, ctb_log2_size=5, loop_filter_across_tiles=1,
                       pps_cb_qp_offset=2, pps_cr_qp_offset=-1)
    hpic = synth.make_picture(hp, 77, perf=False, tiles=(2, 2), n_slices=3, lf_across_slices=None,
                              deblocking="random", bypass_rate=0.04, pcm_rate=0.02)
    whole = c_oracle.decode(hp, [hpic], with_recon=False)[0][1]
    grid = halo.TileGrid.from_picture(hp, hpic)
    assert sorted(res["halo"]) == [str(t) for t in range(grid.n_tiles)]
    for t in range(grid.n_tiles):
        got = _planes(tmp_path / ("halo_%d.npz" % t))
        x0, x1, y0, y1 = grid.luma_rect(grid.rect(t))
        for c in range(3):
            s = 0 if c == 0 else 1
            np.testing.assert_array_equal(got[c], whole[c][y0 >> s:y1 >> s, x0 >> s:x1 >> s], err_msg="tile %d c%d" % (t, c))


def test_bench_two_ranks_on_one_device():
    """bench.py --gpus 2 as torch.distributed.run would start it (RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_*), both ranks on device 0 with --no-rccl.  Rank 0 prints exactly one line; value =
    2 ranks x 512 pictures x 510 CTUs x steps / the MAX over ranks of the timed region."""
    from ranks import free_port
    port, ctrl = free_port(), free_port()
    steps = 3
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), P265_CTRL_PORT=str(ctrl))
        env = {k: v for k, v in env.items() if not k.startswith("P265R_")}
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2",
                                       "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline", "--no-e2e",
                                       "--no-rccl"], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((out, err))
    assert all(p.returncode == 0 for p in procs), "\n".join(o + e for o, e in outs)[-4000:]
    lines0 = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    lines1 = [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]
    assert len(lines0) == 1 and not lines1, outs
    d = json.loads(lines0[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["config"]["pictures_per_gpu"] == 512
    assert d["config"]["ctus_per_picture"] == 510
    elapsed = d["ms_per_step"] * steps * 1e-3
    assert abs(d["value"] - 2 * 512 * 510 * steps / elapsed) <= 2e-3 * d["value"]
    assert d["verified"]["ok"] and d["verified"]["ranks_failed"] == 0 and d["verified"]["pictures"] > 0
    assert "control plane" in d["collectives"]["kind"] and d["collectives"]["rccl_ranks"] is None


def test_rccl_world1_broadcast_of_the_params():
    from p265_amd import rccl
    comm = rccl.Rccl(0, 1, 0)
    try:
        p = R.make_params(pic_width=1920, pic_height=1080, pps_cb_qp_offset=-3)
        raw = np.asarray(p, R.PARAMS_DTYPE).tobytes()
        assert comm.broadcast(raw, root=0) == raw
        got = comm.exchange({0: b"halo-bytes"}, {0: 10})          # self send / recv in one group
        assert got == {0: b"halo-bytes"}
        # a zero-byte payload is skipped on both sides (no unmatched zero-byte ncclSend)
        assert comm.exchange({0: b""}, {0: 0}) == {0: b""}
        assert comm.exchange({0: b"x"}, {0: 1}) == {0: b"x"}      # and the next exchange still pairs
    finally:
        comm.close()


def _child(args, env_extra, timeout=240):
    env = {k: v for k, v in os.environ.items() if not k.startswith("P265R_")}
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-u"] + args, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, (json.loads(lines[-1]) if lines else None)


def test_bench_self_launched_two_ranks():
    """bench.py --gpus 2 with NO launcher (WORLD_SIZE unset): the parent starts the two rank processes itself
    (--device-map 0,0: both on device 0, so --no-rccl) before anything touches the GPU, and exactly one line
    comes back with n_gpus 2, both ranks' checks ok and the whole-job value."""
    steps = 3
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("P265R_")}
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device-map", "0,0",
                        "--no-rccl", "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline", "--no-e2e", "--no-pcie"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["config"]["pictures_per_gpu"] == 512
    elapsed = d["ms_per_step"] * steps * 1e-3
    assert abs(d["value"] - 2 * 512 * 510 * steps / elapsed) <= 2e-3 * d["value"]
    assert d["verified"]["ok"] and d["verified"]["ranks_failed"] == 0 and d["verified"]["every_run"]["runs_checked"] == steps
    assert d["collectives"]["devices"] == [0, 0] and d["collectives"]["rccl_ranks"] is None


def test_xg_batches_side_by_side_on_sixteen_queues():
    """Advisor (round 5): 16 small cross-group batches on 16 lanes with 16 hardware queues -- more cross-group
    workgroups than the GPU holds at once, so chains are only partly resident; rows are claimed from a per-
    chain ticket by running waves, so every run completes and equals the oracle (digest after every run)."""
    p, res = _child([os.path.join(ROOT, "tests", "xg_worker.py"), "lanes"], {"GPU_MAX_HW_QUEUES": "16"})
    assert p.returncode == 0 and res and res["ok"], (p.stdout + p.stderr)[-3000:]


@pytest.mark.parametrize("variant", ["1", "2"])
def test_broken_half_ctu_publish_fails_the_check_instance(variant):
    """A P265R_BR_BROKEN build (prep publishes the bottom line's left half one job early) run with
    P265R_TR_CHECK=1 on sanity.bin's frame 0 in component-major TB order: caught on every one of three runs --
    by prep's extent check (variant 1: the batch reports P265R_EHIP) or, with that check compiled out
    (variant 2), by the row kernel's poisoned half line (parity mismatch) -- never by timing."""
    lib = os.path.join(ROOT, "p265_amd", "libp265r_brbroken%s.so" % variant)
    assert os.path.exists(lib), "build the check variants first (make)"
    p, res = _child([os.path.join(ROOT, "tests", "xg_worker.py"), "broken"], {"P265R_LIB": lib, "P265R_TR_CHECK": "1"})
    assert p.returncode == 0 and res, (p.stdout + p.stderr)[-3000:]
    want = "error" if variant == "1" else "mismatch"
    assert all(o.startswith(want) for o in res["outcomes"]), res
