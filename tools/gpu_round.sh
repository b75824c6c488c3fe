#!/bin/bash
# One GPU call: the whole -m gpu suite (verbose, per-test timeout), then optional bench lines
# (BENCHES: ';'-separated bench.py argument lists) and an interleaved A/B of the bench over the
# configurations in CFGS (tools/ab.sh).
#   BENCHES="--workload c5 --steps 10;--steps 20 --warmup 5" CFGS="base|-||;v|variant||" REPS=3 bash tools/gpu_round.sh
set -e
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "GPU TESTS FAILED"; grep -E "FAILED|Error|error" gpurun_out/gpu_all.log | head -20; tail -60 gpurun_out/gpu_all.log; exit 1; }
  tail -1 gpurun_out/gpu_all.log
fi
i=0
IFS=';' read -ra BL <<< "$BENCHES"
for args in "${BL[@]}"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py $args > gpurun_out/bench_$i.log 2>&1 || { echo "BENCH $i FAILED ($args)"; tail -20 gpurun_out/bench_$i.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/bench_$i.log') if l.startswith('{')][-1])
print('bench $i', '$args', '%.0f CTU/s %.3f ms/step' % (d['value'], d['ms_per_step']), d.get('phases_ms_per_step'), 'verified', d.get('verified', {}).get('ok'), d.get('unit_latency_ms', ''))"
done
[ -n "$CFGS" ] && bash tools/ab.sh
exit 0
