#!/bin/bash
# A/B of library build variants (p265_amd/libp265r_<V>.so, "-" = default) x env settings on the
# bench workload, configurations interleaved over REPS rounds (box-to-box and run-to-run noise
# is a few percent).  CFGS: "lib ENV=v,ENV=v" items separated by ';'.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --experiment --steps ${STEPS:-30} --warmup 4 --no-cpu-baseline --no-e2e > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms_per_step']; print('%.0f %.3f res+prep %.3f intra %.3f sao %.3f serial %.3f' % (d['value'], d['ms_per_step'], p['residual_ms'], p['intra_ms'], p['sao_ms'], p['total_ms']))"; }
IFS=';' read -ra C <<< "${CFGS:-- P265R_FAIR=0;- P265R_FAIR=1}"
for rep in $(seq ${REPS:-2}); do
  for cfg in "${C[@]}"; do
    lib=${cfg%% *}; envs=${cfg#* }
    path=$PWD/p265_amd/libp265r.so; [ "$lib" != "-" ] && path=$PWD/p265_amd/libp265r_$lib.so
    echo "[$rep] lib=$lib $envs :" $(env P265R_LIB=$path ${envs//,/ } bash -c "$(declare -f run); run")
  done
done
