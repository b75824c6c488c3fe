#!/bin/bash
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --experiment --steps 5 --warmup 2 --unique 2 --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"; }
for Wv in "$@"; do echo W$Wv $(P265R_ROW_WAVES=$Wv run); done
