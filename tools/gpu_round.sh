#!/bin/bash
# One GPU call: the whole -m gpu suite (verbose, per-test timeout), then an interleaved A/B of the
# bench over the libraries named in LIBS (tools/ab_libs2.sh).  Usage: LIBS="base default" REPS=3 bash tools/gpu_round.sh
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
[ -n "$LIBS" ] && bash tools/ab_libs2.sh
exit 0
