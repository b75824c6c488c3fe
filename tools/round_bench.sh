#!/bin/bash
# Profile + full bench lines on the GPU box.  Usage: bash tools/round_bench.sh <tag>
set -e
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 900 bash tools/profile_round.sh $TAG
echo "profile ok"
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_full.log
timeout -k 10 300 python bench.py --deblocking --no-cpu-baseline > gpurun_out/bench_dbk.log 2>&1
tail -1 gpurun_out/bench_dbk.log
