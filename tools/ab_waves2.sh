#!/bin/bash
# A/B: waves per row-pipeline workgroup (W=8: 2 WG/CU, 16 waves; W=10: 2 WG/CU, 20 waves; W=6: 3 WG/CU, 18 waves)
set -e
mkdir -p gpurun_out
P265R_ROW_WAVES=10 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "sanity or 1080 or tiles or many or schedule or rows" > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
run() { timeout -k 10 300 python bench.py --experiment --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step']['intra_ms'])"; }
for Wv in 8 10; do for L in 3 5; do echo W$Wv lead$L $(P265R_ROW_WAVES=$Wv P265R_LUMA_LEAD=$L run); done; done
P265R_ROW_WAVES=10 P265R_DEBUG_SYNC=1 timeout -k 10 120 python bench.py --experiment --steps 1 --warmup 0 --no-cpu-baseline --no-e2e 2>&1 | grep -E "rows kernel" | head -3
