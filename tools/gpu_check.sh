#!/bin/bash
# Quick GPU iteration: debug decode (bounded), parity tests, one short bench line.
set -e
mkdir -p gpurun_out
timeout -k 5 60 python -u tools/gpu_debug.py > gpurun_out/dbg_stdout.log 2>&1 || { echo "debug decode failed/hung"; tail -30 gpurun_out/dbg_stdout.log; exit 1; }
echo "debug decode ok"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --unique 2 --no-cpu-baseline > gpurun_out/quick_bench.log 2>&1
tail -1 gpurun_out/quick_bench.log
