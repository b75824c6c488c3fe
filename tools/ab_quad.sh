#!/bin/bash
# Parity + A/B of the 4x4 quad jobs (P265R_QUAD bit 0 luma, bit 1 chroma; default 3) on the bench workload.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for q in ${QUADS:-3 1}; do
  P265R_QUAD=$q timeout -k 10 300 python bench.py --experiment --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/bench_q$q.log 2>&1
  echo "quad=$q" $(tail -1 gpurun_out/bench_q$q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")
done
