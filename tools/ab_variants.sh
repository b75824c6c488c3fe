#!/bin/bash
# A/B of experiment builds: ./tools/ab_variants.sh name1 name2 ...  (p265_amd/libp265r_<name>.so,
# "default" = p265_amd/libp265r.so); prints CTU/s and phase times per variant.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --experiment --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"; }
for v in "$@"; do
    if [ "$v" = default ]; then echo default $(run); else echo $v $(P265R_LIB=$PWD/p265_amd/libp265r_$v.so run); fi
done
