#!/bin/bash
# Per job class cycle statistics of the row kernel (P265R_JOB_STATS build, one batch alone).
set -e
mkdir -p gpurun_out
for W in ${WAVES:-0 8}; do
P265R_LIB=$PWD/p265_amd/libp265r_stats.so P265R_ROW_WAVES=$W P265R_DEBUG_SYNC=1 timeout -k 10 120 python bench.py --experiment --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --pipeline 1 > gpurun_out/jobstats_w$W.log 2>&1
echo "W=$W"; grep -E "rows kernel W=|jobs |lifetime \(M|dependency" gpurun_out/jobstats_w$W.log | head -20
done
