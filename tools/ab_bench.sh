set -e
mkdir -p gpurun_out
P265R_LIB=$PWD/p265_amd/libp265r_N.so P265R_ROW_WAVES=4 timeout -k 5 25 python -u tools/gpu_debug.py > gpurun_out/dbg_N.log 2>&1 || { echo "N variant hung/failed"; exit 1; }
echo "notrace variant ok"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
run() { timeout -k 10 300 python bench.py --experiment --steps 5 --warmup 2 --unique 2 --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"; }
echo steps512 $(P265R_SCHEDULE=steps run --frames 512)
for Wv in 4 8 16; do for F in 256 512 1024; do echo rows W$Wv F$F $(P265R_ROW_WAVES=$Wv run --frames $F); done; done
