#!/bin/bash
# Intra kernel diagnostics on the GPU box: dependency-wait share (debug build path) + SQ counters.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --experiment --steps 2 --warmup 1 --frames 512 --unique 2 --no-cpu-baseline"
P265R_DEBUG_SYNC=1 timeout -k 10 300 $B > gpurun_out/intra_dbg.log 2>&1 || true
grep "dependency waits" gpurun_out/intra_dbg.log | tail -2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/isq -o sq -- $B > gpurun_out/isq.log 2>&1
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/isq/sq_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k, d in agg.items():
    d = {c: v / n[k][c] for c, v in d.items()}
    w = max(d.get("SQ_WAVES", 1), 1)
    print(k[:60], " ".join("%s=%.4g" % (c.replace("SQ_", ""), v / w) for c, v in sorted(d.items()) if c != "SQ_WAVES"), "waves=%d" % w)
PY
