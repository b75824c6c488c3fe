set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abq_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/abq_tests.log; exit 1; }
tail -1 gpurun_out/abq_tests.log
CFGS="-|;GPU_MAX_HW_QUEUES=8|;GPU_MAX_HW_QUEUES=8 P265R_FORK_PREP=0|;GPU_MAX_HW_QUEUES=6|;GPU_MAX_HW_QUEUES=12|" REPS=2 bash tools/ab_cfg2.sh
TAG=q8 ENVS="GPU_MAX_HW_QUEUES=8" bash tools/ab_timeline.sh
