#!/bin/bash
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --steps 5 --warmup 2 --unique 2 --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"; }
for Wv in 16 8 4; do echo W$Wv $(P265R_ROW_WAVES=$Wv run); done
P265R_ROW_WAVES=8 P265R_DEBUG_SYNC=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --unique 2 --no-cpu-baseline > gpurun_out/dbg8.log 2>&1 || true
grep "rows kernel" gpurun_out/dbg8.log | head -2
