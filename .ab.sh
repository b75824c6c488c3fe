set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for S in steps rows; do
 for F in 256 512; do
  P265R_SCHEDULE=$S timeout -k 10 300 python bench.py --steps 5 --warmup 2 --frames $F --unique 2 --no-cpu-baseline > gpurun_out/ab_${S}_$F.log 2>&1
  echo $S $F $(tail -1 gpurun_out/ab_${S}_$F.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")
 done
done
for Wv in 4 16; do
  P265R_ROW_WAVES=$Wv timeout -k 10 300 python bench.py --steps 5 --warmup 2 --frames 512 --unique 2 --no-cpu-baseline > gpurun_out/ab_w$Wv.log 2>&1
  echo W$Wv $(tail -1 gpurun_out/ab_w$Wv.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")
done
