#!/bin/bash
# Row-kernel diagnostics (P265R_DEBUG_SYNC=1): dependency-wait share, workgroup lifetime spread,
# placement (XCC / CU) of slow workgroups; then the bench with / without fair CU sharing.
set -e
mkdir -p gpurun_out
for F in ${FAIRS:-0 1}; do
P265R_FAIR=$F P265R_DEBUG_SYNC=1 timeout -k 10 120 python bench.py --experiment --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --pipeline 1 > gpurun_out/diag_f$F.log 2>&1
echo "fair=$F"; grep -E "rows kernel|XCC|sharing" gpurun_out/diag_f$F.log | head -8
done
for F in ${FAIRS:-0 1}; do
  P265R_FAIR=$F timeout -k 10 300 python bench.py --experiment --steps 12 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/bench_f$F.log 2>&1
  echo "fair=$F" $(tail -1 gpurun_out/bench_f$F.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'])")
done
