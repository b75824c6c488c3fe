#!/bin/bash
# A/B of library env knobs on the bench: CFGS is a ';'-separated list of space-separated VAR=VALUE
# sets ("-" = defaults), REPS bench runs each.  Usage: CFGS="-;P265R_ROW_WAVES=12" REPS=2 bash tools/ab_env.sh
set -e
mkdir -p gpurun_out/ab
IFS=';' read -ra C <<< "${CFGS:--}"
for rep in $(seq ${REPS:-2}); do
  i=0
  for cfg in "${C[@]}"; do
    i=$((i+1))
    envs=""; [ "$cfg" != "-" ] && envs="$cfg"
    env $envs timeout -k 10 300 python bench.py --experiment --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > gpurun_out/ab/env$i.$rep.log 2>&1
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/env$i.$rep.log').read().strip().splitlines()[-1])
print('[$rep] %-36s %12.0f CTU/s %7.3f ms/step' % ('$cfg', d['value'], d['ms_per_step']), d['phases_ms_per_step'])"
  done
done
