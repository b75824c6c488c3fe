#!/bin/bash
# Kernel-trace timeline of the pipelined bench (tools/timeline.py).  Usage: TAG=x ENVS="..." ARGS="..." bash tools/ab_timeline.sh
set -e
export TMPDIR=/tmp
OUT=gpurun_out/tl_${TAG:-a}
mkdir -p $OUT
env ${ENVS:-} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o tl -- python bench.py --experiment --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ${ARGS:-} > $OUT/run.log 2>&1
f=$(find $OUT -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py $f | tee $OUT/timeline.txt
