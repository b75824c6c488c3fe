#!/bin/bash
# A/B: row-queue order of the luma / chroma chains (P265R_LUMA_LEAD) and waves per workgroup.
set -e
mkdir -p gpurun_out
P265R_LUMA_LEAD=3 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
run() { timeout -k 10 300 python bench.py --experiment --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step']['intra_ms'])"; }
for L in 0 1 2 3 5 8 17; do echo lead$L $(P265R_LUMA_LEAD=$L run); done
for Wv in 4 16; do echo W$Wv lead0 $(P265R_ROW_WAVES=$Wv run) lead3 $(P265R_ROW_WAVES=$Wv P265R_LUMA_LEAD=3 run); done
