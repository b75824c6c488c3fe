#!/usr/bin/env python3
"""Benchmark: reconstructed all-intra CTUs/s on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path -- residual (dequant + inverse DCT/DST) -> intra
prediction + reconstruction -> SAO -- over one batch of synthetic all-intra pictures whose
records are already resident in HBM.

  --workload c3  (default)  C3/C4: 1080p + SAO, 512 pictures per GPU per step (C4's per-GPU
                            work: pictures are independent, picture f -> rank f mod N)
  --workload c5             C5: 4K, 2x2 tiles x 2 frames = 8 tile units per step across all
                            ranks ((frame, tile) -> rank, dist.unit_shard), CTU-row SAO

N GPUs: one process per GPU (torch.distributed.run only launches them; nothing here imports
torch).  Weak scaling for c3, no data-path collective; the 32-byte SPS/PPS POD is broadcast
from rank 0 with ncclBroadcast (RCCL over xGMI, ctypes, p265_amd/rccl.py) once, outside the
timed region; barriers and the MAX over ranks go over the socket control plane.  Rank 0
prints ONE JSON line.

    python bench.py                       # N=1, defaults finish in ~1-2 minutes
    python bench.py --gpus 8              # launches 8 rank processes itself (one per device)
    python -m torch.distributed.run --nproc-per-node 8 bench.py --gpus 8

Without a launcher (WORLD_SIZE unset) and N > 1, this process only spawns the N rank processes
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them) before anything
touches the GPU, waits for them and exits with the worst return code; rank 0 prints the line.  It
refuses (exit 2) when WORLD_SIZE differs from --gpus or the ranks need more devices than are visible.

P265R_* environment variables are experiment / test knobs of the library; bench refuses to run
with any of them set unless --experiment is given (and then records them in the line).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# the C oracle (output check, CPU baseline) runs OpenMP regions: passive waiting, so its idle
# workers do not spin on the cores the end-to-end leg's parse threads use afterwards
os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "reconstructed CTUs/sec (1080p all-intra) + achieved HBM GB/s vs peak"
# rocprofv3 PMC summary of this same command per workload (tools/profile_round.sh +
# tools/profile_summary.py); its HBM traffic per intra launch (2*FETCH_SIZE + WRITE_SIZE,
# gfx950 correction) fills roofline.traffic
PROFILE = {"c3": os.path.join(ROOT, "profiles", "LATEST"), "c5": os.path.join(ROOT, "profiles", "LATEST_C5")}


def _profile_rows(workload, kernel_prefix, key):
    try:
        tag = open(PROFILE[workload]).read().strip()
        summ = json.load(open(os.path.join(ROOT, "profiles", tag, "summary.json")))
    except (OSError, ValueError):
        return None, []
    return tag, [(n, r) for n, r in summ.items() if kernel_prefix in n and r.get(key) and r.get("isolated_dispatches")]


def measured_traffic(workload, kernel_prefix, frames, avg_ms=None):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary, or None
    when no summary exists for this batch size (PMC counters cannot be read inside the run)."""
    tag, rows = _profile_rows(workload, kernel_prefix, "traffic_gb")
    if tag is None:
        return None, None
    try:
        lines = open(os.path.join(ROOT, "profiles", tag, "bench.json")).read().splitlines()
        meta = json.loads([ln for ln in lines if ln.startswith("{")][-1])
    except (OSError, ValueError, IndexError):
        return None, tag
    if int(meta.get("config", {}).get("pictures_per_gpu", -1)) != frames:
        return None, tag
    if not rows:
        return None, tag
    # the row kernel comes in several builds (alone / overlapped runs): take the profiled one
    # whose isolated duration is closest to this run's launches
    name, row = min(rows, key=lambda nr: abs(nr[1]["avg_ms"] - (avg_ms or 0)))
    if avg_ms and abs(row["avg_ms"] - avg_ms) > 0.1 * avg_ms:
        return None, tag + " (stale: profiled %.2f ms/launch)" % row["avg_ms"]
    return int(row["traffic_gb"] * 1e9), "%s, %s" % (tag, name.replace("void ", ""))


# MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32 at 2.4 GHz; a wave64 VALU op takes its SIMD 2 cycles;
# one scalar unit per CU (1 SALU instruction per cycle)
VALU_PEAK = 1024 * 2.4e9 / 2.0      # wave-instructions / s
SALU_PEAK = 256 * 2.4e9             # instructions / s


def issue_rates(workload, kernel_prefix, avg_ms):
    """Instruction-issue view of the dominant kernel (it is issue-bound): VALU and
    SALU instructions per launch from the committed PMC summary (SQ_INSTS_VALU / SQ_INSTS_SALU of
    the profiled build whose duration matches), divided by this run's launch time and the peaks."""
    tag, rows = _profile_rows(workload, kernel_prefix, "SQ_INSTS_VALU")
    if not rows:
        return None
    name, row = min(rows, key=lambda nr: abs(nr[1]["avg_ms"] - avg_ms))
    if abs(row["avg_ms"] - avg_ms) > 0.1 * avg_ms:
        return None
    t = avg_ms * 1e-3
    return {"valu_per_launch": int(row["SQ_INSTS_VALU"]), "salu_per_launch": int(row["SQ_INSTS_SALU"]),
            "valu_frac": round(row["SQ_INSTS_VALU"] / (t * VALU_PEAK), 3),
            "salu_frac": round(row["SQ_INSTS_SALU"] / (t * SALU_PEAK), 3),
            "source": "profiles/%s/summary.json, %s" % (tag, name.replace("void ", "")),
            "peaks": "VALU 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 op; SALU 256 CUs x 2.4 GHz"}


PROBE_MIX = {"valu": 131, "salu": 81, "lds": 15}     # p265_amd/csrc/issue_probe.hip, which = 0


def issue_ceiling(device, avg_launch_ms, jobs_per_launch, num_cus, rates=None):
    """Measured issue ceiling of the row kernel's job loop (p265_amd/libp265probe.so): the mix of
    VALU / SALU / LDS instructions per job issued with no dependencies at the row kernel's occupancy
    (24 waves per CU); -> CU-cycles per job at that ceiling, the row kernel's own CU-cycles per job
    (launch time x the probe's measured clock x CUs / jobs), and their ratio."""
    import ctypes
    path = os.path.join(ROOT, "p265_amd", "libp265probe.so")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        return {"error": "libp265probe.so: %s" % e}
    fn = lib.p265probe_issue
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    jobs = 16384
    res = {}
    for which, name in enumerate(("mix", "valu_only", "salu_only", "lds_only")):
        c, ms = ctypes.c_double(0), ctypes.c_double(0)
        rc = fn(device, which, jobs, ctypes.byref(c), ctypes.byref(ms))
        if rc:
            return {"error": "p265probe_issue(%d) = %d" % (which, rc)}
        res[name] = (c.value, ms.value)
    c_mix, ms_mix = res["mix"]
    clk = c_mix * jobs * 24 / (ms_mix * 1e-3)                      # the slowest wave spans the launch
    row = avg_launch_ms * 1e-3 * clk * num_cus / max(1, jobs_per_launch)
    out = {"probe_mix_per_job": PROBE_MIX, "ceiling_cu_cycles_per_job": round(c_mix, 1),
           "valu_only": round(res["valu_only"][0], 1), "salu_only": round(res["salu_only"][0], 1),
           "lds_only": round(res["lds_only"][0], 1), "clock_ghz": round(clk / 1e9, 3),
           "jobs_per_launch": int(jobs_per_launch), "row_kernel_cu_cycles_per_job": round(row, 1),
           "frac": round(c_mix / row, 3) if row else None,
           "how": "p265_amd/csrc/issue_probe.hip: the job mix issued with no dependencies at 24 waves per CU, "
                  "s_memtime cycles of the slowest wave; frac = that ceiling / the row kernel's CU-cycles per job"}
    if rates:
        out["profile_mix_per_job"] = {"valu": round(rates["valu_per_launch"] / jobs_per_launch, 1),
                                      "salu": round(rates["salu_per_launch"] / jobs_per_launch, 1)}
    return out


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default c3: 30, c5: 64 -- 16 lanes to fill)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("c3", "c5"), default="c3")
    ap.add_argument("--frames", type=int, default=512, help="c3: 1080p pictures per GPU per step")
    ap.add_argument("--unique", type=int, default=4, help="c3: distinct synthetic pictures per rank (replicated)")
    ap.add_argument("--c5-frames", type=int, default=2, help="c5: 4K frames per step (x4 tile units, all ranks)")
    ap.add_argument("--c5-batch-units", type=int, default=512,
                    help="c5: tile units per resident batch of a rank -- a batch carries the rank's units of K = "
                         "ceil(this / units per rank per step) consecutive steps (frames are independent), so one "
                         "launch fills the GPU even at one unit per rank and step; 0 = one step per batch (the "
                         "latency regime: 16 lanes side by side, one hardware queue each)")
    ap.add_argument("--c5-world", type=int, default=0,
                    help="c5: run rank 0's share of an N-rank job on this one GPU (dist.unit_shard(..., 0, N)); the "
                         "line's value is then this GPU's rate (per_gpu_of_world = N), not a whole-job rate")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="resident batches run round-robin on this many HIP streams (p265r_set_pipeline; default "
                         "2 -- one batch's residual / prep / SAO phases beside the other's intra phase; c5 with "
                         "--c5-batch-units 0: 16 -- an 8-unit batch fills 16 CUs, so 16 whole batches run side by side)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the bitstream -> planes end-to-end leg")
    ap.add_argument("--deblocking", action="store_true",
                    help="deblocking on in every slice (real-stream config; SURVEY §8(d) defines the bench without it)")
    ap.add_argument("--experiment", action="store_true",
                    help="allow P265R_* library knobs in the environment (recorded in the line; not a headline run)")
    ap.add_argument("--no-rccl", action="store_true",
                    help="N > 1: control plane only, no RCCL communicator (ranks sharing one device: two RCCL "
                         "ranks cannot); the params then travel over the control plane")
    ap.add_argument("--no-verify", action="store_true", help="skip the post-run output check (not a headline run)")
    ap.add_argument("--device-map", default=None,
                    help="N > 1: comma-separated HIP device of each local rank (default: local rank i on device i); "
                         "ranks sharing a device need --no-rccl (tests: --gpus 2 --device-map 0,0 --no-rccl)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive back-end leg")
    ap.add_argument("--bit-depth", type=int, default=8, choices=(8, 9, 10, 11, 12),
                    help="c3: BitDepth of the synthetic pictures (9 / 10: the Main 10 path -- uint16 planes, per-diagonal "
                         "intra kernel, loopfilter16.h; not the headline)")
    return ap.parse_args(argv)


def experiment_env():
    return {k: v for k, v in os.environ.items() if k.startswith("P265R_")}


def host_info():
    """CPU model, the machine's logical CPUs and this job's CPU share (cgroup quota / affinity)."""
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                model = ln.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    total = os.cpu_count() or 1
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            share = min(share, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    # the GPU pool grants a fixed CPU share per GPU and announces it in OMP_NUM_THREADS (16);
    # os.cpu_count() there is the whole machine's
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp))
    return {"cpu_model": model, "host_cores_total": total, "cpu_share": share}


def algorithmic_bytes(pics, pel_bytes=1):
    """B = 2C + 16 N_TB + 16 N_CU + 3 S + 32 N_CTU per picture.

    N_CU is not carried by the records (each TB record holds the CU-level fields the path
    reads), so the 16 N_CU term is 0; S counts luma + chroma samples.  Also returns the
    per-kernel figures: intra (2C residual read + 16 N_TB + S recon write + 32 N_CTU),
    residual (2C read + 2C write + 8 B job record per coded TB), SAO (2S + 32 N_CTU).
    """
    tot = intra = resid = sao = 0
    for p in pics:
        c = p.n_coded_coef
        ntb, nctu = len(p.tbs), len(p.ctus)
        s = p.meta["samples"] * pel_bytes                  # output bytes (2 per sample above 8 bits)
        tot += 2 * c + 16 * ntb + 3 * s + 32 * nctu
        intra += 2 * c + 16 * ntb + s + 32 * nctu
        resid += 4 * c + 8 * int(((p.tbs["flags"] & 1) != 0).sum())
        sao += 2 * s + 32 * nctu
    return tot, intra, resid, sao


def cpu_baseline_python(procs, timeout_s=900):
    """The pure-Python restatement (oracle/py_baseline.py) in a child process that never
    touches the GPU: one 1080p picture per worker, ``procs`` workers."""
    r = subprocess.run([sys.executable, "-m", "oracle.py_baseline", "--procs", str(procs)], cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout_s)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode or not lines:
        return {"error": (r.stderr or "no output")[-300:]}
    return json.loads(lines[-1])


def cpu_baseline(params, uniq, budget_s, threads, what):
    """CPU oracle (oracle/recon_oracle.c, test infrastructure used here only as the reported
    baseline) on a bounded sample of the same workload: whole pictures (or tile units),
    repeated until ~budget_s of wall time, OpenMP over pictures on ``threads`` host cores."""
    from oracle import c_oracle
    c_oracle.decode(params, uniq[:1], threads=1, with_recon=False)           # warm
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        batch = [uniq[i % len(uniq)] for i in range(threads * 2)]
        c_oracle.decode(params, batch, threads=threads, with_recon=False)
        n += len(batch)
    dt = time.perf_counter() - t0
    ctus = n * len(uniq[0].ctus)
    return {"value": round(ctus / dt, 1), "unit": "CTU/s", "cores": threads, "kind": "port",
            "sample": "oracle/recon_oracle.c (scalar C restatement, OpenMP over pictures): %d synthetic %s "
                      "= %d CTUs in %.1f s" % (n, what, ctus, dt)}


def pictures_to_check(n, unique):
    """Indices of a resident batch whose outputs are checked after the timed runs: the first and
    the last ``unique`` pictures (every distinct synthetic picture, at both ends of the batch)."""
    return sorted(set(range(min(unique, n))) | set(range(max(0, n - unique), n)))


def sha_planes(planes):
    import hashlib
    return hashlib.sha256(b"".join(np.ascontiguousarray(p).tobytes() for p in planes)).hexdigest()


def digest_mismatches(pics, want, got):
    """Indices of the pictures whose device digests ``got`` ([n, 3] uint64, p265r_batch_digest)
    differ from the oracle's ``want`` ({id(picture): 3 digests})."""
    return [i for i, p in enumerate(pics) if not np.array_equal(got[i], want[id(p)])]


def oracle_digests(groups, threads):
    """Per group: the digest and SHA-256 of the C oracle's decode of every distinct picture
    ({id(picture): ...}); the reference every device digest is compared with."""
    from p265_amd import digest
    from oracle import c_oracle
    res = []
    for params, gp in groups:
        uniq = {}
        for p in gp:
            uniq.setdefault(id(p), p)
        keys = list(uniq)
        ref = c_oracle.decode(params, [uniq[k] for k in keys], threads=threads, with_recon=False)
        res.append(({k: digest.picture_digest(r[1]) for k, r in zip(keys, ref)},
                    {k: sha_planes(r[1]) for k, r in zip(keys, ref)}))
    return res


def verify(ctxs, groups, a, wants, ran=None):
    """After the timed region: EVERY picture of every resident batch that ran (``ran``: batch slots;
    with fewer steps than pipeline lanes some never do) through its device digest after the batch's
    final timed run (p265r_batch_digest, which also reports the sticky row-kernel error word: a
    dependency give-up in ANY run) against the digest of the C oracle's decode of the same records;
    and, as a check of the digest itself, the downloaded planes of each batch's first and last
    pictures (SHA-256 and host digest).  -> the line's "verified" object."""
    from p265_amd import _lib, digest
    n_checked, bad, status_ok, distinct = 0, [], True, set()
    for (ctx, batches), (params, gp), (want, want_sha) in zip(ctxs, groups, wants):
        distinct |= set(want)
        idx = pictures_to_check(len(gp), a.unique if a.workload == "c3" else a.c5_units_per_step)
        for bi, b in enumerate(batches):
            if ran is not None and bi not in ran:
                continue
            try:
                got = ctx.digest(b)
            except _lib.P265RError as e:
                status_ok = False
                bad.append("batch %d: %s" % (bi, e))
                continue
            n_checked += len(gp)
            bad += ["batch %d picture %d" % (bi, i) for i in digest_mismatches(gp, want, got)]
            outs = ctx.download(b, only=idx)
            for i in idx:
                if sha_planes(outs[i]) != want_sha[id(gp[i])] or not np.array_equal(digest.picture_digest(outs[i]), got[i]):
                    bad.append("batch %d picture %d (download)" % (bi, i))
    return {"ok": status_ok and not bad, "pictures": n_checked, "distinct": len(distinct),
            "batches": sum(1 for _, bs in ctxs for bi in range(len(bs)) if ran is None or bi in ran),
            "status_ok": status_ok, "mismatches": bad[:8],
            "how": "after the timed runs: p265r_batch_digest (device digest of every picture's three output planes, "
                   "plus the sticky row-kernel error word) of every resident batch that ran -- its final timed run -- "
                   "against the digests of oracle/recon_oracle.c's decode of the same records; each batch's first and "
                   "last pictures are also downloaded and compared by SHA-256 and host digest (p265_amd/digest.py)"}


def checked_pass(ctxs, groups, a, wants, steps):
    """The timed region's pipelined schedule once more (same batches, lanes and call sequence, so the
    same row-kernel builds), with a device digest enqueued on the batch's lane after EVERY run
    (p265r_batch_digest_async, one slot per run): checks each run, not only the last one of every batch,
    against the oracle.  Not timed.  -> {"runs_checked", "pictures_checked", "ok", "mismatches"}."""
    from p265_amd import _lib
    slots = {}
    for k in range(steps):
        for ci, (ctx, batches) in enumerate(ctxs):
            bi = k % a.pipeline
            s = k // a.pipeline
            ctx.run(batches[bi])
            if s < _lib.DIGEST_SLOTS:
                ctx.digest_async(batches[bi], s)
                slots[(ci, bi)] = s + 1
    runs = pics = 0
    bad = []
    for (ci, bi), n in sorted(slots.items()):
        ctx, batches = ctxs[ci]
        gp = groups[ci][1]
        want = wants[ci][0]
        try:
            got = ctx.digest_slots(batches[bi], n)
        except _lib.P265RError as e:
            bad.append("context %d batch %d: %s" % (ci, bi, e))
            continue
        for s in range(n):
            runs += 1
            pics += len(gp)
            bad += ["run %d of batch %d picture %d" % (s, bi, i) for i in digest_mismatches(gp, want, got[s])]
    return {"ok": not bad, "runs_checked": runs, "pictures_checked": pics, "mismatches": bad[:8],
            "how": "after the timed region, the same %d pipelined steps again with p265r_batch_digest_async after every "
                   "run (each run's output digest-checked against the oracle before the next run overwrites it)" % steps}


def exit_code(out):
    """Non-zero when the line's own output check failed (the value is then not a result)."""
    v = out.get("verified")
    return 3 if v is not None and not v.get("ok") else 0


def end_to_end(device, reps=32, threads=16):
    """Bitstream bytes -> decoded planes in host memory, from a real (synthetic) 1080p stream.

    tests/golden/synth_1080p_4pic.bin (4 IDR pictures with MD5 picture-hash SEI, made by
    tests/golden/gen_streams.py) is repeated ``reps`` times.  Times the native front-end alone
    (host threads) and the whole decoder (front-end + record upload + GPU + plane download,
    i.e. PCIe-inclusive); every decoded picture is checked against its MD5 SEI.  Not ``value``.
    """
    from p265_amd import bitstream, decoder
    path = os.path.join(ROOT, "tests", "golden", "synth_1080p_4pic.bin")
    if not os.path.exists(path):
        return {"error": "missing %s" % path}
    one = open(path, "rb").read()
    data = one * reps
    bitstream.decode_stream(one, threads=threads)                  # warm
    t0 = time.perf_counter()
    pics = bitstream.decode_stream(data, threads=threads)
    fe_s = time.perf_counter() - t0
    n_ctu = sum(len(p.picture.ctus) for p in pics)
    decoder.decode_bytes(one, device=device, threads=threads)      # warm (contexts, kernels)
    runs = []
    for _ in range(5):                     # best of 5: a 0.1-s host-bound run is noisy on a shared host
        t0 = time.perf_counter()
        frames = decoder.decode_bytes(data, device=device, threads=threads)
        runs.append(time.perf_counter() - t0)
        if not all(f.hash_ok for f in frames):
            break
    e2e_s = min(runs)
    decoder.release_contexts()
    return {"stream": "tests/golden/synth_1080p_4pic.bin x%d" % reps, "pictures": len(pics), "ctus": n_ctu,
            "bytes_per_ctu": round(len(one) * reps / n_ctu, 1), "threads": threads,
            "frontend_ctu_s": round(n_ctu / fe_s, 1), "frontend_mb_s": round(len(data) / fe_s / 1e6, 2),
            "e2e_ctu_s": round(n_ctu / e2e_s, 1), "e2e_runs_s": [round(r, 4) for r in runs],
            "hash_checked": sum(1 for f in frames if f.hash_ok), "hash_failed": sum(1 for f in frames if f.hash_ok is False),
            "config": "decoder.decode_bytes defaults: %d-picture batches over %d warm contexts, %d MB chunks, "
                      "asynchronous parse on %d threads" % (decoder.DEFAULT_BATCH, decoder.DEFAULT_DEPTH,
                                                             decoder.DEFAULT_CHUNK >> 20, threads),
            "note": "native front-end (libp265fe.so) on host threads + PCIe-inclusive GPU decode; not `value`"}


def stream_ceiling(device):
    """Achievable HBM stream rates on this box (p265_amd/libp265probe.so p265probe_stream: 16 B per lane,
    four loads in flight, best grid), the ceiling of the bandwidth-bound phases; hipMemcpyAsync D2D
    beside it.  GB/s."""
    import ctypes
    from p265_amd import hip
    out = {"memcpy_d2d_gbs": hip.copy_bandwidth_gbs(device)}
    try:
        lib = ctypes.CDLL(os.path.join(ROOT, "p265_amd", "libp265probe.so"))
    except OSError as e:
        out["error"] = "libp265probe.so: %s" % e
        return out
    fn = lib.p265probe_stream
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_double] + [ctypes.POINTER(ctypes.c_double)] * 3
    c, r, w = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_double(0)
    rc = fn(device, float(8 << 30), ctypes.byref(c), ctypes.byref(r), ctypes.byref(w))
    if rc:
        out["error"] = "p265probe_stream = %d" % rc
        return out
    out.update(copy_gbs=round(c.value, 1), read_gbs=round(r.value, 1), write_gbs=round(w.value, 1),
               how="16-B-per-lane copy / read / write of 8 GiB buffers, the fastest of a few forms and grids "
                   "(libp265probe.so p265probe_stream; tools/bw_probe.hip); copy counts read + write bytes")
    return out


def pcie_leg(params, pics, device, steps=3):
    """The back-end fed over PCIe: per step the batch's records (TB / CTU records + coefficients, the
    pictures of one c3 step) are uploaded from host memory (p265r_batch_upload: validation, class
    packing into pinned staging, H2D), run, and every picture's three planes downloaded into host
    arrays (p265r_batch_download into one reused set of host frames, as a decoder's frame pool: fresh
    host memory would add a page fault per 4 KB); step k's upload and run (one context) overlap step
    k-1's download (the other context, a second host thread).  Bytes per direction are what crosses PCIe; the pinned-memory copy rates of the same box
    stand beside them.  Not `value` (which has the records resident in HBM)."""
    from p265_amd import hip, recon
    from p265_amd import records as R
    # coefficients + TB / CTU records + the 8-B residual job of every coded TB (p265r_batch_upload's H2D copies)
    h2d_bytes = sum(2 * p.n_coded_coef + R.TB_DTYPE.itemsize * len(p.tbs) + R.CTU_DTYPE.itemsize * len(p.ctus) +
                    8 * int(((p.tbs["flags"] & R.TB_CBF) != 0).sum()) for p in pics)
    d2h_bytes = sum(p.meta["samples"] for p in pics) * (1 if int(params["bit_depth_luma"]) == 8 else 2)
    nnz = sum(int(np.count_nonzero(p.coef)) for p in {id(p): p for p in pics}.values())
    coded = sum(p.n_coded_coef for p in {id(p): p for p in pics}.values())
    out = {"pictures_per_step": len(pics), "steps": steps}
    import threading
    # two contexts (a context is single-threaded, include/p265r.h): step k uploads and runs on one while a
    # second host thread downloads step k - 1 from the other, so both PCIe directions are busy at once
    ctxs = [recon.ReconContext(params, device=device) for _ in range(2)]
    try:
        frames = None
        for ctx in ctxs:                        # warm: allocations, pinned staging, kernels
            b = ctx.upload(pics)
            ctx.run(b)
            frames = ctx.download(b, into=frames)   # the host frame pool every step's download refills
            b.free()
        t0 = time.perf_counter()
        t_up = 0.0
        t_dl = [0.0]
        prev = None

        def fetch(ctx, batch):
            d0 = time.perf_counter()
            ctx.download(batch, into=frames)
            t_dl[0] += time.perf_counter() - d0
            batch.free()

        for k in range(steps):
            th = threading.Thread(target=fetch, args=prev) if prev is not None else None
            if th is not None:
                th.start()
            ctx = ctxs[k % 2]
            u0 = time.perf_counter()
            b = ctx.upload(pics)
            t_up += time.perf_counter() - u0
            ctx.run(b)
            if th is not None:
                th.join()
            prev = (ctx, b)
        fetch(*prev)
        dt = time.perf_counter() - t0
    finally:
        for ctx in ctxs:
            ctx.close()
    t_dl = t_dl[0]
    n_ctu = sum(len(p.ctus) for p in pics)
    out.update(ctu_s=round(n_ctu * steps / dt, 1), ms_per_step=round(dt / steps * 1e3, 2),
               h2d_mb_per_step=round(h2d_bytes / 1e6, 1), d2h_mb_per_step=round(d2h_bytes / 1e6, 1),
               h2d_gbs=round(h2d_bytes * steps / t_up / 1e9, 2), d2h_gbs=round(d2h_bytes * steps / t_dl / 1e9, 2),
               upload_ms_per_step=round(t_up / steps * 1e3, 2), download_ms_per_step=round(t_dl / steps * 1e3, 2),
               pinned=hip.pinned_copy_gbs(device),
               coef_nonzero_frac=round(nnz / max(1, coded), 3),
               note="records uploaded and planes downloaded every step (host <-> HBM over PCIe), kernels as in value; "
                    "h2d / d2h GB/s = bytes / host wall time of p265r_batch_upload / p265r_batch_download (upload "
                    "includes host-side validation and class packing, overlapped with its H2D in picture chunks); "
                    "uploads and downloads run concurrently on two contexts")
    return out


def c5_steps_per_batch(batch_units, units_per_step, world):
    """K consecutive steps per C5 batch, ONE value for every rank: ceil(batch_units / the largest rank's
    units per step), so every rank's batch carries its units of the same K steps and the job decodes
    exactly K x all units per run even when the units do not divide over the ranks (0: one step)."""
    if batch_units <= 0:
        return 1
    max_units = -(-units_per_step // world)
    return max(1, -(-batch_units // max_units))


def build_workload(a, rank, world):
    """-> ([(params, [pictures of this rank with those params])], cpu-baseline sample, config dict).

    One group for c3.  c5 has two: a uniform 2x2 tiling of 60 x 34 CTBs gives 30 x 17 CTBs per
    tile, i.e. 1920 x 1088 top tiles and 1920 x 1072 bottom tiles (the picture ends at 2160)."""
    from p265_amd import dist, synth, tiles
    from p265_amd import records as R
    if a.workload == "c3":
        params = R.make_params(pic_width=1920, pic_height=1080, bit_depth_luma=a.bit_depth, bit_depth_chroma=a.bit_depth)
        params = dist.broadcast_params(params)                  # RCCL broadcast of the SPS/PPS POD
        uniq = [synth.make_picture(params, 268 + 1000 * rank + i, perf=True, deblocking=a.deblocking)
                for i in range(a.unique)]
        for p in uniq:
            p.meta["samples"] = 1920 * 1080 * 3 // 2
        pics = [uniq[i % a.unique] for i in range(a.frames)]
        cfg = {"workload": "C3/C4: 1080p all-intra + %sSAO, %d pictures per GPU per step (%d distinct)%s"
                           % ("deblocking + " if a.deblocking else "", a.frames, a.unique,
                              "" if a.bit_depth == 8 else ", BitDepth %d (16-bit path, not the headline)" % a.bit_depth),
               "bit_depth": a.bit_depth,
               "pictures_per_gpu": a.frames, "ctus_per_picture": len(pics[0].ctus), "ctb": 64,
               "parallelism": "picture-sharded x%d (picture f -> rank f mod N)" % world}
        return [(params, pics)], (params, uniq, "1080p pictures"), cfg
    # C5: 4K, uniform 2x2 tiles, loop_filter_across_tiles 0: every (frame, tile) unit is a
    # 1920x1080 sub-picture of its own (p265_amd/tiles.py); units dealt to ranks
    p4k = R.make_params(pic_width=3840, pic_height=2160, loop_filter_across_tiles=0)
    p4k = dist.broadcast_params(p4k)
    frames = [synth.make_picture(p4k, 4000 + f, perf=True, tiles=(2, 2), deblocking=a.deblocking)
              for f in range(a.c5_frames)]
    srank, sworld = (0, a.c5_world) if a.c5_world else (rank, world)
    mine = dist.unit_shard(a.c5_frames, 4, srank, sworld)
    parts = {f: tiles.split(p4k, frames[f]) for f in sorted({f for f, _ in mine})}
    units = [parts[f][t] for f, t in mine]
    if not units:
        raise RuntimeError("c5: rank %d of %d has no tile unit (more ranks than units)" % (srank, sworld))
    for tp, tpic, _ in units:
        tpic.meta["samples"] = int(tp["pic_width"]) * int(tp["pic_height"]) * 3 // 2
    # K consecutive steps per batch: the same synthetic frames repeat every step (as C3 replicates its
    # distinct pictures); the uneven tiles (1920 x 1088 top, 1920 x 1072 bottom) as ONE ragged batch:
    # one context of the largest tile's size, every unit with its own size (p265r_picture.pic_width /
    # pic_height)
    # one K for every rank (ranks may hold different unit counts when they do not divide): the batch of every
    # rank carries its units of the same K steps, so the job decodes exactly ctus_all_units x K per run
    k_steps = c5_steps_per_batch(a.c5_batch_units, 4 * a.c5_frames, sworld)
    step_pics = [tpic for _, tpic, _ in units]
    groups = [(tiles.ragged_params(units), step_pics * k_steps)]
    cols, rows = tiles.tile_grid(p4k, frames[0])
    ctus_all = a.c5_frames * sum((cols[i + 1] - cols[i]) * (rows[j + 1] - rows[j])
                                 for i in range(len(cols) - 1) for j in range(len(rows) - 1))
    pics = groups[0][1]
    params = groups[0][0]
    cfg = {"workload": "C5: 4K all-intra + %sSAO (CTU-row SAO kernel), 2x2 uniform tiles x %d frames = %d tile units "
                       "per step over all ranks, %d on this rank; one batch = this rank's units of %d consecutive steps"
                       % ("deblocking + " if a.deblocking else "", a.c5_frames, 4 * a.c5_frames, len(units), k_steps),
           "pictures_per_gpu": len(pics), "units_per_step": 4 * a.c5_frames, "units_per_rank_step": len(units),
           "steps_per_batch": k_steps, "ctus_per_picture": len(pics[0].ctus),
           "tiles": sorted({"%dx%d" % tuple(p.size) for p in step_pics}),
           "ctus_all_units": ctus_all, "ctus_rank_step": sum(len(p.ctus) for p in step_pics),
           "ctb": 64, "parallelism": "(frame, tile) units -> ranks x%d (dist.unit_shard); one ragged batch (one launch "
                                     "per phase) for the uneven tile sizes" % sworld}
    if a.c5_world:
        cfg["simulated_world"] = {"world": a.c5_world, "rank": 0, "note": "rank 0's share of a %d-rank job on one GPU"
                                  % a.c5_world}
    return groups, (params, step_pics, "tile units of 4K frames (%s)" % ", ".join(cfg["tiles"])), cfg


def c5_unit_latency(ctx, step_pics, runs):
    """C5 unit latency: one step's tile units of this rank as ONE batch, run alone ``runs`` times
    with per-phase HIP events; the units run concurrently (the row kernel gives every unit two
    workgroups of its own, luma and chroma chains, on different CUs), so a run's time is one
    unit's latency (the slowest unit's)."""
    b = ctx.upload(step_pics)
    try:
        ctx.run(b)
        ctx.sync()
        ctx.set_timing(True)
        for _ in range(runs):
            ctx.run(b)
        ctx.sync()
        ctx.set_timing(False)
        t = ctx.timings_total()
    finally:
        b.free()
    n = max(1, t["runs"])
    return {"one_batch_step": round(t["total_ms"] / n, 4), "intra": round(t["intra_ms"] / n, 4),
            "residual": round(t["residual_ms"] / n, 4), "sao": round(t["sao_ms"] / n, 4), "units": len(step_pics),
            "note": "one step's %d tile units of this rank as one batch, alone, %d runs" % (len(step_pics), n)}


class Refused(SystemExit):
    """A command-line / environment combination bench.py will not run (exit 2, message on stderr)."""

    def __init__(self, msg):
        sys.stderr.write("bench.py: refusing to run: %s\n" % msg)
        super().__init__(2)


def device_map(a, n):
    """HIP device of each of the n local ranks: --device-map, or local rank i on device i."""
    if not a.device_map:
        return list(range(n))
    try:
        m = [int(x) for x in a.device_map.split(",")]
    except ValueError:
        raise Refused("--device-map %r is not a comma-separated list of device numbers" % a.device_map)
    if len(m) != n or min(m) < 0:
        raise Refused("--device-map %r must name one device (>= 0) for each of the %d ranks" % (a.device_map, n))
    if len(set(m)) < n and not a.no_rccl:
        raise Refused("ranks sharing a device (--device-map %s) need --no-rccl: two RCCL ranks cannot share one "
                      "device" % a.device_map)
    return m


def visible_devices():
    """HIP devices visible to this job, counted in a child process so that THIS process never touches
    the GPU before it starts the rank processes; -1 when the count fails."""
    code = ("import sys; sys.path.insert(0, %r)\nfrom p265_amd import hip\ntry:\n    print(hip.device_count())\n"
            "except hip.HipError:\n    print(0)\n" % ROOT)
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        return int(r.stdout.strip().splitlines()[-1])
    except (OSError, subprocess.SubprocessError, ValueError, IndexError):
        return -1


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv):
    """bench.py --gpus N without a launcher: start N rank processes of this script (one per device,
    --device-map), exactly as torch.distributed.run would (RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT), wait for all of them and return the worst exit
    code.  Rank 0 prints the JSON line (inherited stdout).  A rank that fails ends the others after a
    grace period (they would wait in a barrier for it)."""
    n = a.gpus
    dmap = device_map(a, n)
    vis = visible_devices()
    if vis < 0:
        raise Refused("cannot count the visible HIP devices")
    if max(dmap) + 1 > vis:
        raise Refused("--gpus %d needs %d HIP device(s) (device map %s), %d visible" % (n, max(dmap) + 1, dmap, vis))
    port, ctrl = free_port(), free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), P265_CTRL_PORT=str(ctrl))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env, cwd=ROOT))
    codes, first_fail = [None] * n, None
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None and p.poll() is not None:
                codes[i] = p.returncode
                if p.returncode and first_fail is None:
                    first_fail = time.time()
        if first_fail is not None and time.time() - first_fail > 60:
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.kill()
                    codes[i] = p.wait()
        time.sleep(0.2)
    worst = 0
    for c in codes:
        c = 128 - c if c < 0 else c                          # killed by signal s: 128 + s
        worst = max(worst, c)
    if worst:
        sys.stderr.write("bench.py: rank exit codes %s\n" % codes)
    return worst


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus < 1:
        raise Refused("--gpus %d" % a.gpus)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a, argv)                   # (this process never touches the GPU)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != a.gpus:
        raise Refused("WORLD_SIZE=%d from the launcher but --gpus %d" % (world_env, a.gpus))
    dmap = device_map(a, int(os.environ.get("LOCAL_WORLD_SIZE", world_env)))
    c5_latency = a.workload == "c5" and a.c5_batch_units <= 0     # one step per batch, batches side by side
    if a.pipeline is None:
        # 2 lanes: with the prep stream of each lane, 4 streams on HIP's default 4 hardware queues, one
        # queue each (round 5, same box: 2 lanes 5.30 ms per step, 3 lanes 5.77-5.80, 4 lanes 6.1-6.4)
        a.pipeline = 16 if c5_latency else 2
    if a.steps is None:
        a.steps = 64 if c5_latency else (20 if a.workload == "c5" else 30)
    # one hardware queue per stream (the lanes + the upload stream): HIP's default 4 would put two C5
    # lanes behind each other (c5, 8 lanes: 3.0 M CTU/s at 4 queues, 8.4 M at 12; 16 lanes at 20 queues:
    # 16.4 M, every CU holding one unit's workgroup; c3 measured best
    # at the default: 43.4 vs 41.8 M at 8 queues -- its prep / residual streams then interleave).
    # Raised (never lowered) before this process first touches HIP (dist.init below); the GPU boxes
    # export the default 4 explicitly.
    if c5_latency:
        want = min(32, a.pipeline + 4)
        try:
            have = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        except ValueError:
            have = 4
        if have < want:
            os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    exp = experiment_env()
    if exp and not a.experiment:
        sys.stderr.write("bench.py: refusing to run with library experiment knobs set: %s "
                         "(unset them, or pass --experiment for a non-headline run)\n" % sorted(exp))
        sys.exit(2)
    from p265_amd import dist, hip, recon

    host = host_info()
    # pure-Python CPU baseline first, in a child process, before this process touches the GPU
    py_base = None
    if world_env == 1 and not a.no_cpu_baseline and a.workload == "c3" and a.bit_depth == 8:
        py_base = cpu_baseline_python(host["cpu_share"])
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if local_rank >= len(dmap):
        raise Refused("LOCAL_RANK %d outside the device map %s" % (local_rank, dmap))
    rank, world, _ = dist.init(device=dmap[local_rank], rccl=world_env > 1 and not a.no_rccl)
    local = dmap[local_rank]                               # this rank's HIP device
    rccl_ranks = dist.rccl_ranks()                         # ncclCommCount of every rank (None: no RCCL)

    t0 = time.time()
    groups, (cpu_params, cpu_sample, cpu_what), cfg = build_workload(a, rank, world)
    gen_s = time.time() - t0
    a.c5_units_per_step = cfg.get("units_per_rank_step", 0)
    pics = [p for _, g in groups for p in g]

    # one context per picture size (c3: one); each holds one resident batch per stream (same
    # pictures, separate buffers); step k runs batch k % pipeline of every context
    ctxs = []
    for params, gp in groups:
        ctx = recon.ReconContext(params, device=local)
        ctx.set_pipeline(a.pipeline)
        ctxs.append((ctx, [ctx.upload(gp) for _ in range(a.pipeline)]))

    ran = set()                            # batch slots that have run (verify checks only those)

    def step(k):
        ran.add(k % a.pipeline)
        for ctx, batches in ctxs:
            ctx.run(batches[k % a.pipeline])

    def sync_all():
        for ctx, _ in ctxs:
            ctx.sync()
        hip.synchronize()

    n_ctu = sum(len(p.ctus) for p in pics)
    for k in range(a.warmup):
        step(k)
    sync_all()
    builds0 = [ctx.describe()["row_launches"] for ctx, _ in ctxs]
    dist.barrier()
    t_start = time.perf_counter()
    for k in range(a.steps):               # queued back to back, batches alternating over the streams
        step(k)
    sync_all()
    elapsed_local = time.perf_counter() - t_start
    dist.barrier()
    elapsed = dist.max_over_ranks(elapsed_local)
    # which row-kernel build the timed steps ran (p265r_describe row_launches, difference over the region)
    builds_timed = {}
    for (ctx, _), b0 in zip(ctxs, builds0):
        for k, v in ctx.describe()["row_launches"].items():
            if v - b0[k]:
                builds_timed[k] = builds_timed.get(k, 0) + v - b0[k]
    # phase breakdown + roofline: the same steps on ONE batch per context (one stream, no
    # overlap, contexts one after another), HIP events around each phase, so every kernel's
    # duration is its own
    acc = None
    for ctx, batches in ctxs:
        ctx.set_timing(True)
        for _ in range(a.steps):
            ctx.run(batches[0])
        ctx.sync()
        ctx.set_timing(False)
        t = ctx.timings_total()
        assert t["runs"] == a.steps
        acc = t if acc is None else {k: acc[k] + t[k] for k in acc}
    knobs = ctxs[0][0].describe()
    jl, jch = ctxs[0][0].job_count(ctxs[0][1][0])
    # the pipelined steps' row kernel after the first is the W = 8 build (beside the other lane's phases):
    # the same batch alone through that build, so the line carries both builds' isolated launch times
    w8 = None
    if a.workload == "c3" and acc["intra_launches"] == a.steps:
        ctx0, b0 = ctxs[0][0], ctxs[0][1][0]
        ctx0.set_row_waves(8)
        ctx0.set_timing(True)
        for _ in range(a.steps):
            ctx0.run(b0)
        ctx0.sync()
        ctx0.set_timing(False)
        ctx0.set_row_waves(0)
        t8 = ctx0.timings_total()
        w8 = t8["intra_ms"] / max(1, t8["intra_launches"])

    if a.workload == "c3":
        total_ctus = world * n_ctu * a.steps
    elif a.c5_world:                       # this GPU's share of a simulated c5_world-rank job
        total_ctus = n_ctu * a.steps
    else:                                  # every tile unit of the batch's steps, over all ranks
        total_ctus = cfg["ctus_all_units"] * cfg["steps_per_batch"] * a.steps
    value = total_ctus / elapsed
    tot_b, intra_b, res_b, sao_b = algorithmic_bytes(pics, 1 if a.bit_depth == 8 else 2)
    launches_per_step = acc["intra_launches"] / a.steps
    avg_launch_ms = acc["intra_ms"] / max(1, acc["intra_launches"])
    bytes_per_launch = intra_b / launches_per_step
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
    if a.bit_depth == 8:
        traffic, prof_tag = measured_traffic(a.workload, "intra_rows_kernel", len(pics), avg_launch_ms)
    else:                                  # the 16-bit path's kernels have no committed PMC profile
        traffic, prof_tag = None, "not profiled (Main 10 path)"
    cfg.update(batch_pipeline=a.pipeline, library=knobs)
    out = {
        "metric": METRIC,
        "value": round(value, 1), "unit": "CTU/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak" if a.workload == "c3" else "strong",
        "vs_baseline": None, "dtype": "%s samples / int16 coefficients (integer)" % ("u8" if a.bit_depth == 8 else "u16"),
        "data": "synthetic: seeded all-intra records with sanity.bin statistics (p265_amd/synth.py)",
        "config": cfg,
        "roofline": {"bound": "hbm", "kernel": "intra_rows_kernel" if a.bit_depth == 8 else
                     ("intra_rows_kernel<..., uint16_t>" if a.bit_depth <= 10 else
                      "intra_rows_kernel<..., int16_t>"), "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": ("profiles/%s/summary.json (%s; rocprofv3 PMC, 2*FETCH_SIZE+WRITE_SIZE per launch)"
                                        % tuple(prof_tag.split(", ", 1))) if traffic else prof_tag,
                     "bytes_per_launch": int(bytes_per_launch), "avg_launch_ms": round(avg_launch_ms, 4),
                     "note": ("achieved / avg_launch_ms: the batch alone, which runs the W = 12 build; the pipelined steps "
                              "run W = 8 after their first (builds: launches per build in the timed steps, and W = 8 "
                              "alone).  Bound by instruction issue (the CU's one scalar unit + each SIMD's VALU shared "
                              "by 24 waves; waves park on s_waitcnt 42 % of their cycles while others issue), not by "
                              "HBM (DESIGN.md §4); see issue_rates" if a.bit_depth == 8 else
                              "achieved / avg_launch_ms: the 16-bit row pipeline (one workgroup per CU: twice the "
                              "LDS per wave), the batch alone (W = 12); the Main 10 path, not the headline "
                              "(DESIGN.md §4)" if a.bit_depth <= 10 else
                              "achieved / avg_launch_ms: the 16-bit row pipeline at BitDepth 11-12 (packed chroma "
                              "angular sums split into 6-bit halves), the batch alone (W = 12); not the headline "
                              "(DESIGN.md §4)")},
        "issue_rates": issue_rates(a.workload, "intra_rows_kernel", avg_launch_ms) if a.bit_depth == 8 else None,
        "intra_jobs_per_launch": {"luma": jl, "chroma": jch},
        "phases_ms_per_step": {k: round(acc[k] / a.steps, 4) for k in ("residual_ms", "intra_ms", "sao_ms", "total_ms")},
        "phase_gbs": {"residual": round(res_b / (acc["residual_ms"] / a.steps * 1e-3) / 1e9, 1),
                      "sao": round(sao_b / (acc["sao_ms"] / a.steps * 1e-3) / 1e9, 1) if acc["sao_ms"] else None,
                      "whole_path_algorithmic": round(tot_b / (elapsed / a.steps) / 1e9, 2)},
        "setup_s": round(gen_s, 1),
    }
    builds = {"timed_steps_launches": builds_timed,
              "w12_alone": {"avg_launch_ms": round(avg_launch_ms, 4), "frac": round(achieved / HBM_PEAK_GBS, 4)}}
    if w8:
        builds["w8_alone"] = {"avg_launch_ms": round(w8, 4),
                              "frac": round(bytes_per_launch / (w8 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    out["roofline"]["builds"] = builds
    if a.workload == "c5":
        out["unit_latency_ms"] = c5_unit_latency(ctxs[0][0], cpu_sample, a.steps)
        if a.c5_world:
            out["per_gpu_of_world"] = a.c5_world
            out["value_note"] = ("this GPU's rate for rank 0's share of a %d-rank job (%d of the %d tile units of every "
                                 "step); the whole job's rate is %d x this when every rank holds as many units"
                                 % (a.c5_world, cfg["units_per_rank_step"], cfg["units_per_step"], a.c5_world))
    if exp:
        out["experiment_env"] = exp
    if world > 1:
        out["collectives"] = {"kind": ("control plane only (--no-rccl)" if a.no_rccl else
                                       "ncclBroadcast of the 32-B params (RCCL); barriers + MAX over the control plane"),
                              "rccl_ranks": rccl_ranks, "devices": dist.allgather_json(local),
                              "launcher": "torch.distributed.run or bench.py's own (--gpus N, WORLD_SIZE unset)"}
    if not a.no_verify:
        wants = oracle_digests(groups, host["cpu_share"])
        v = verify(ctxs, groups, a, wants, ran)
        cp = checked_pass(ctxs, groups, a, wants, a.steps)
        v["every_run"] = cp
        v["ok"] = v["ok"] and cp["ok"]
        # every rank checks its own batches; the job is ok only if all are
        v["ranks_failed"] = int(dist.max_over_ranks(0.0 if v["ok"] else 1.0)) if world > 1 else int(not v["ok"])
        v["ok"] = v["ok"] and v["ranks_failed"] == 0
        out["verified"] = v
    if rank == 0:
        sc = stream_ceiling(local)
        out["roofline"]["achievable"] = sc
        ceil = sc.get("copy_gbs") or sc["memcpy_d2d_gbs"]
        out["phase_gbs"]["vs_achievable_copy"] = {k: round(v / ceil, 3) for k, v in out["phase_gbs"].items()
                                                  if isinstance(v, float) and k != "whole_path_algorithmic"}
        if a.workload == "c3" and launches_per_step == 1 and a.bit_depth == 8:
            out["roofline"]["issue"] = issue_ceiling(local, avg_launch_ms, jl + jch,
                                                     int(knobs.get("num_cus", 256)), out["issue_rates"])
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        if py_base is not None:
            py_base.update(host_cores_total=host["host_cores_total"], cpu_model=host["cpu_model"])
            out["cpu_baseline"] = py_base
        cb = cpu_baseline(cpu_params, cpu_sample, a.cpu_baseline_seconds, host["cpu_share"], cpu_what)
        cb.update(host_cores_total=host["host_cores_total"], cpu_model=host["cpu_model"])
        out["cpu_baseline_c" if py_base is not None else "cpu_baseline"] = cb
    out["host"] = host
    for ctx, batches in ctxs:
        for b in batches:
            b.free()
        ctx.close()
    if rank == 0 and world == 1 and not a.no_pcie and a.workload == "c3":
        out["pcie"] = pcie_leg(groups[0][0], groups[0][1], local)
    if rank == 0 and world == 1 and not a.no_e2e and a.workload == "c3" and a.bit_depth == 8:
        out["end_to_end"] = end_to_end(local, threads=min(16, host["cpu_share"]))
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.finalize()
    rc = exit_code(out)
    if rc:
        sys.stderr.write("bench.py: output check FAILED: %s\n" % json.dumps(out.get("verified")))
    return rc


if __name__ == "__main__":
    sys.exit(main())
