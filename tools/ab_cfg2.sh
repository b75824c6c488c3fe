#!/bin/bash
# A/B of (env knobs, bench args) pairs: CFGS is a ';'-separated list of "ENV=V ... | bench args"
# entries ("-" for none), REPS interleaved runs each.
# Usage: CFGS="- | ;P265R_PIPE_WAVES=4 | --pipeline 4" REPS=2 bash tools/ab_cfg2.sh
set -e
mkdir -p gpurun_out/ab
IFS=';' read -ra C <<< "${CFGS:--|}"
for rep in $(seq ${REPS:-2}); do
  i=0
  for cfg in "${C[@]}"; do
    i=$((i+1))
    envs="${cfg%%|*}"; args="${cfg#*|}"
    envs="$(echo $envs)"; [ "$envs" = "-" ] && envs=""
    env $envs timeout -k 10 300 python bench.py --experiment --no-cpu-baseline --no-e2e $args > gpurun_out/ab/cfg$i.$rep.log 2>&1
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/cfg$i.$rep.log').read().strip().splitlines()[-1])
print('[$rep] %-44s %12.0f CTU/s %7.3f ms/step' % ('$cfg', d['value'], d['ms_per_step']), d['phases_ms_per_step'])"
  done
done
