#!/bin/bash
# Profile the default bench on the GPU box: kernel trace stats + PMC passes (separate runs,
# per MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage (on the box): bash tools/profile_round.sh <tag>   (ARGS="--workload c5 ..." for another workload)
set -e
TAG=${1:-r1}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python bench.py ${ARGS:---steps 3 --warmup 1 --frames 512 --unique 2} --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fe -- $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o wr -- $B > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1
grep '^{' $OUT/kt.log | tail -1 > $OUT/bench.json
echo "$B" > $OUT/cmd.txt
echo "profile $TAG done"
