#!/bin/bash
# One rocprofv3 PMC pass over a short one-stream bench (one batch, no overlap), summarised per
# kernel: bash tools/pmc_pass.sh <tag> <counter> [<counter> ...]   (respect the per-block limits:
# 8 SQ_, 4 TCC_, 4 TCP_, 2 TA_, 2 TD_, 2 GRBM_)
set -e
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
B="python bench.py --experiment --steps 3 --warmup 1 --unique 2 --no-cpu-baseline --no-e2e --pipeline 1 ${BENCH_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o pmc -- $B > $OUT/run.log 2>&1
python3 - $OUT <<'PY'
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + '/**/pmc_counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('p265r::', '')
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k][r['Counter_Name']] += 1
for k, d in sorted(agg.items()):
    print('%-36s' % k[:36], ' '.join('%s=%.4g' % (c, d[c] / n[k][c]) for c in sorted(d)))
PY
