#!/bin/bash
# A/B of whole source trees (abtrees/<tag>/: bench.py + p265_amd + oracle, each with its own
# built libp265r.so) on the driver's bench command, interleaved over REPS rounds.
# Usage: TAGS="e50422a HEAD" REPS=2 bash tools/ab_trees.sh
set -e
mkdir -p gpurun_out/abt
for rep in $(seq ${REPS:-2}); do
  for t in ${TAGS}; do
    (cd abtrees/$t && timeout -k 10 240 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-}) > gpurun_out/abt/$t.$rep.log 2>&1
    python3 -c "
import json
d=json.loads(open('gpurun_out/abt/$t.$rep.log').read().strip().splitlines()[-1])
p=d.get('phases_ms_per_step',{})
print('[$rep] %-8s %12.0f CTU/s %7.3f ms/step' % ('$t', d['value'], d['ms_per_step']), ' '.join('%s=%.3f'%(k,v) for k,v in p.items() if isinstance(v,float)))"
  done
done
