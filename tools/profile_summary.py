#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output dir into profiles/<tag>/ (kept in git).

FETCH_SIZE/WRITE_SIZE are KB per dispatch (rocprofv3); per MI355X_MICROARCH.md
§HBM, FETCH_SIZE under-reports wide (16 B/lane) coalesced reads by exactly 2x on gfx950,
so the corrected HBM traffic is 2*FETCH + WRITE for kernels whose loads are 16 B/lane
(residual and intra kernels); the SAO kernel's byte loads are uncalibrated (raw shown).
"""
import collections
import csv
import json
import os
import shutil
import sys


def kname(full):
    """Kernel name without its argument list ('(anonymous namespace)' prefixes kept)."""
    full = full.strip()
    if full.endswith(")"):
        depth = 0
        for i in range(len(full) - 1, -1, -1):
            depth += full[i] == ")"
            depth -= full[i] == "("
            if depth == 0:
                return full[:i]
    return full


def per_kernel(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(collections.Counter)
    for r in rows:
        k = kname(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]] += 1
    return {k: {c: v / n[k][c] for c, v in d.items()} for k, d in agg.items()}


def isolated_avg(path):
    """Per kernel: mean duration over the dispatches that overlap no other dispatch in time.
    bench.py pipelines batches over several streams for `value` and then re-runs the same
    steps on one batch alone for the phase times; only the latter give a kernel's own
    duration (an overlapped dispatch's span includes waiting for CU slots)."""
    rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"])) for r in rows)
    out = collections.defaultdict(list)
    for i, (a, b, name) in enumerate(iv):
        prev_end = max((e for _, e, _ in iv[:i]), default=-1)
        nxt = iv[i + 1][0] if i + 1 < len(iv) else None
        if prev_end <= a and (nxt is None or nxt >= b):
            out[name].append((b - a) / 1e6)
    return {k: (sum(v) / len(v), len(v)) for k, v in out.items()}


def main(src, tag):
    dst = os.path.join("profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))))
    fe = per_kernel(os.path.join(src, "fetch", "fe_counter_collection.csv"))
    wr = per_kernel(os.path.join(src, "write", "wr_counter_collection.csv"))
    sq = per_kernel(os.path.join(src, "sq", "sq_counter_collection.csv"))
    iso = isolated_avg(os.path.join(src, "kt", "kt_kernel_trace.csv"))
    out = {}
    cmd = os.path.join(src, "cmd.txt")
    what = open(cmd).read().strip() if os.path.exists(cmd) else "python bench.py --frames 512 --steps 3 --warmup 1 --unique 2"
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
    lines = ["# rocprofv3 summary `%s` (`%s`)" % (tag, what), "",
             "avg ms = mean over the dispatches that overlap no other dispatch (the one-batch pass of",
             "bench.py); avg all = rocprofv3 --stats over every dispatch, incl. the pipelined ones.", "",
             "| kernel | calls | avg ms (isolated, n) | avg all ms | FETCH KB | WRITE KB | corrected traffic GB (2F+W) | VALU/wave | SALU/wave | LDS/wave |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for s in stats:
        name = kname(s["Name"])
        if name.startswith("__amd"):
            continue
        f, w = fe.get(name, {}).get("FETCH_SIZE", 0.0), wr.get(name, {}).get("WRITE_SIZE", 0.0)
        q = sq.get(name, {})
        waves = max(q.get("SQ_WAVES", 1.0), 1.0)
        traffic = (2 * f + w) * 1024 / 1e9
        avg_all = float(s["AverageNs"]) / 1e6
        avg_iso, n_iso = iso.get(name, (avg_all, 0))
        out[name] = dict(calls=int(s["Calls"]), avg_ms=avg_iso, isolated_dispatches=n_iso, avg_all_ms=avg_all,
                         fetch_kb=f, write_kb=w, traffic_gb=traffic, **{k: v for k, v in q.items()})
        lines.append("| %s | %s | %.4f (%d) | %.4f | %.4g | %.4g | %.4g | %.4g | %.4g | %.4g |" % (
            name, s["Calls"], avg_iso, n_iso, avg_all, f, w, traffic, q.get("SQ_INSTS_VALU", 0) / waves,
            q.get("SQ_INSTS_SALU", 0) / waves, q.get("SQ_INSTS_LDS", 0) / waves))
    lines += ["", "Counters per dispatch (SQ): see summary.json.  FETCH_SIZE correction: MI355X_MICROARCH.md §HBM."]
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1, sort_keys=True)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
