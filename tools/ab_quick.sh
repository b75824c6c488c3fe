#!/bin/bash
# One GPU call for a kernel change: parity (test_gpu_parity.py) on the default library, then an
# interleaved A/B of the bench against the libraries named in LIBS (tools/ab_libs2.sh).
# Usage: LIBS="base default" REPS=3 bash tools/ab_quick.sh
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abq_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/abq_tests.log; exit 1; }
tail -1 gpurun_out/abq_tests.log
bash tools/ab_libs2.sh
