#!/bin/bash
# Batch size A/B: pictures per step (FRAMES list), REPS bench runs each (no CPU baseline / e2e).
set -e
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for f in ${FRAMES:-512 1024}; do
    timeout -k 10 300 python bench.py --frames $f --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > gpurun_out/ab/f$f.$rep.log 2>&1
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/f$f.$rep.log').read().strip().splitlines()[-1])
print('[$rep] frames %5d %12.0f CTU/s %7.3f ms/step' % ($f, d['value'], d['ms_per_step']), d['phases_ms_per_step'])"
  done
done
