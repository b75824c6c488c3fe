#!/bin/bash
# A/B of the batch pipelining: lanes (P265R pipeline depth) x intra stream mode (P265R_PRIO:
# 0 = each lane's own stream, 2 = one shared intra stream) x waves per workgroup.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-e2e "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases_ms_per_step']['intra_ms'])"; }
for cfg in ${CFGS:-"8 3 0" "8 3 2" "8 2 2" "8 4 2" "12 3 0" "12 3 2"}; do
  set -- $cfg
  echo "W=$1 pipe=$2 prio=$3" $(P265R_ROW_WAVES=$1 P265R_PRIO=$3 run --pipeline $2)
done
