#!/bin/bash
# Sweep of bench configurations (pictures per batch, pipeline depth, waves / register build),
# interleaved over REPS rounds.  CFGS: "ENV=v,ENV=v|bench args" items separated by ';'.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --experiment --steps ${STEPS:-30} --warmup 4 --no-cpu-baseline --no-e2e "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.0f %.3f intra %.3f serial %.3f' % (d['value'], d['ms_per_step'], d['phases_ms_per_step']['intra_ms'], d['phases_ms_per_step']['total_ms']))"; }
IFS=';' read -ra C <<< "$CFGS"
for rep in $(seq ${REPS:-2}); do
  for cfg in "${C[@]}"; do
    envs=${cfg%%|*}; args=${cfg#*|}
    echo "[$rep] $envs | $args :" $(env ${envs//,/ } bash -c "$(declare -f run); run $args")
  done
done
