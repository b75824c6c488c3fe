#!/bin/bash
# A/B of (environment, bench arguments) pairs on one box, experiments library:
#   SETS="ENV=1 ENV2=3 | --frames 448;| --pipeline 1" REPS=2 bash tools/ab_env2.sh
set -e
mkdir -p gpurun_out/ab
IFS=';' read -ra AS <<< "$SETS"
for rep in $(seq ${REPS:-2}); do
  i=0
  for set in "${AS[@]}"; do
    i=$((i+1))
    envs="${set%%|*}"; args="${set#*|}"
    env P265R_LIB=${LIB:-$PWD/p265_amd/libp265r_exp.so} $envs timeout -k 10 150 python bench.py --experiment --no-cpu-baseline --no-e2e ${VERIFY:---no-verify} $args > gpurun_out/ab/env$i.$rep.log 2>&1
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/env$i.$rep.log').read().strip().splitlines()[-1])
print('[$rep] %-44s %12.0f CTU/s %7.3f ms/step' % ('$envs |$args', d['value'], d['ms_per_step']), d['phases_ms_per_step'], d.get('verified', {}).get('ok', '-'))"
  done
done
