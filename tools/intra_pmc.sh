#!/bin/bash
# Intra kernel PMC passes (SQ block, 8 counters per pass) on the bench workload.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --experiment --steps 2 --warmup 1 --frames 512 --unique 2 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-}"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC"
P3="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_IFETCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/ipmc$i -o p -- $B > gpurun_out/ipmc$i.log 2>&1
done
python - <<'PY'
import csv, collections, glob
tot = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/ipmc*/p_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
    for k, d in agg.items():
        for c, v in d.items():
            tot[k][c] = v / n[k][c]
for k, d in tot.items():
    if "intra_rows" not in k and "loopfilter" not in k and "prep" not in k:
        continue
    w = max(d.get("SQ_WAVES", 1), 1)
    print(k[:50], " ".join("%s=%.4g" % (c.replace("SQ_", ""), v / w) for c, v in sorted(d.items()) if c != "SQ_WAVES"), "waves=%d" % w)
PY
