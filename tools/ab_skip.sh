#!/bin/bash
# Marginal cost of each phase in the pipelined steady state: P265R_SKIP drops phases on re-runs of
# the resident batches (needs the experiments build: P265R_LIB=.../libp265r_exp.so) (bit 0 residual, 1 job prep, 2 loop filter; output unchanged, timing only).
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --experiment --steps 30 --warmup 4 --no-cpu-baseline --no-e2e --no-verify ${BENCH_ARGS:-} "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.0f %.3f' % (d['value'], d['ms_per_step']), d['phases_ms_per_step'])"; }
for rep in 1 2; do for k in ${SKIPS:-0 1 2 4 3 7}; do echo "[$rep] skip=$k" $(P265R_SKIP=$k run); done; done
