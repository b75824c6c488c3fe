#!/bin/bash
# Parity (every row-pipeline variant) + A/B of the waves per workgroup (W=8: 2 WG/CU x 8;
# W=10: 2 x 10 at <= 96 VGPRs; W=12: 2 x 12 at <= 80 VGPRs) on the bench workload.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for Wv in ${WAVES:-8 10 12}; do
  P265R_ROW_WAVES=$Wv timeout -k 10 300 python bench.py --experiment --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/bench_w$Wv.log 2>&1
  echo "W=$Wv" $(tail -1 gpurun_out/bench_w$Wv.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")
done
