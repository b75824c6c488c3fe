#!/bin/bash
# A/B of bench.py argument sets on one box: ARGSETS="args1;args2;..." REPS=2 bash tools/ab_args.sh
set -e
mkdir -p gpurun_out/ab
IFS=';' read -ra AS <<< "$ARGSETS"
for rep in $(seq ${REPS:-2}); do
  i=0
  for args in "${AS[@]}"; do
    i=$((i+1))
    timeout -k 10 150 python bench.py --experiment --no-cpu-baseline --no-e2e --no-verify $args > gpurun_out/ab/args$i.$rep.log 2>&1
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/args$i.$rep.log').read().strip().splitlines()[-1])
print('[$rep] %-34s %12.0f CTU/s %7.3f ms/step' % ('$args', d['value'], d['ms_per_step']), d['phases_ms_per_step'])"
  done
done
