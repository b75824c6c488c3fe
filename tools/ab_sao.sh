set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
run() { timeout -k 10 300 python bench.py --steps 5 --warmup 2 --unique 2 --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"; }
echo window $(run)
echo direct $(P265R_SAO_KERNEL=direct run)
echo dbk $(run --deblocking)
