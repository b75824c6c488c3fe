#!/bin/bash
# A/B of library builds on the bench: for each lib tag (p265_amd/libp265r_<tag>.so; "default" =
# libp265r.so) REPS bench runs (no CPU baseline / e2e), printing value, ms/step and per-phase ms.
# Usage: LIBS="default sao6 sao8" REPS=2 bash tools/ab_libs2.sh
set -e
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-default}; do
    if [ "$lib" = default ]; then path=$PWD/p265_amd/libp265r.so; else path=$PWD/p265_amd/libp265r_$lib.so; fi
    P265R_LIB=$path timeout -k 10 150 python bench.py --experiment --no-cpu-baseline --no-e2e --no-verify ${BENCH_ARGS:-} > gpurun_out/ab/$lib.$rep.log 2>&1
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab/$lib.$rep.log').read().strip().splitlines()[-1])
print('[$rep] %-10s %12.0f CTU/s %7.3f ms/step' % ('$lib', d['value'], d['ms_per_step']), d['phases_ms_per_step'])"
  done
done
