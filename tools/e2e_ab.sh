#!/bin/bash
# End-to-end (bitstream -> planes) A/B over library builds (bench.end_to_end, 3 timed decodes each):
#   LIBS="default oldsb" REPS=2 bash tools/e2e_ab.sh
set -e
for rep in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-default}; do
    if [ "$lib" = default ]; then path=$PWD/p265_amd/libp265r.so; else path=$PWD/p265_amd/libp265r_$lib.so; fi
    P265R_LIB=$path timeout -k 10 200 python -c "
import sys, json; sys.path.insert(0, '.')
import bench
r = bench.end_to_end(0)
print('[$rep] %-8s e2e %.0f CTU/s runs %s frontend %.0f' % ('$lib', r['e2e_ctu_s'], r['e2e_runs_s'], r['frontend_ctu_s']))"
  done
done
