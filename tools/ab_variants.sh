#!/bin/bash
# A/B the default library against p265_amd/libp265r_<v>.so variants: bash tools/ab_variants.sh v1 v2 ...
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --steps 5 --warmup 2 --unique 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"; }
echo base $(run)
for v in "$@"; do echo $v $(P265R_LIB=$PWD/p265_amd/libp265r_$v.so run); done
echo base $(run)
