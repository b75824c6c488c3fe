#!/bin/bash
# Interleaved A/B of bench.py over configurations (run on the GPU box: box-to-box spread is a few
# percent, so compare only within one call).
#
#   CFGS="name|lib|env|args;name|lib|env|args;..." REPS=2 bash tools/ab.sh
#
#   lib   "-"          p265_amd/libp265r.so (the product build)
#         <tag>        p265_amd/libp265r_<tag>.so (make variant V=<tag> FLAGS="-D...")
#         tree:<tag>   abtrees/<tag>/: a whole source tree (bench.py + p265_amd + oracle, its own
#                      built library; e.g. a git worktree of an older commit)
#   env   space-separated VAR=value settings (P265R_* knobs: --experiment is added for them)
#   args  extra bench.py arguments (default: the driver's --steps 20 --warmup 5)
#
# Prints value, ms per step and the one-batch phase breakdown per run; logs in gpurun_out/ab/.
set -e
mkdir -p gpurun_out/ab
ROOT=$PWD
IFS=';' read -ra C <<< "${CFGS:?set CFGS}"
for rep in $(seq ${REPS:-2}); do
  for cfg in "${C[@]}"; do
    IFS='|' read -r name lib envs args <<< "$cfg"
    dir=$ROOT; libenv=""
    case "$lib" in
      ""|-) ;;
      tree:*) dir=$ROOT/abtrees/${lib#tree:} ;;
      *) libenv="P265R_LIB=$ROOT/p265_amd/libp265r_$lib.so" ;;
    esac
    exp=""
    [[ "$envs $libenv" == *P265R_* ]] && exp="--experiment"
    log=$ROOT/gpurun_out/ab/$name.$rep.log
    (cd $dir && env $envs $libenv timeout -k 10 300 python bench.py $exp --no-cpu-baseline --no-e2e \
        ${args:---steps 20 --warmup 5}) > $log 2>&1 || { echo "[$rep] $name FAILED"; tail -5 $log; continue; }
    python3 - "$log" "$rep" "$name" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
p = d.get("phases_ms_per_step", {})
v = d.get("verified", {})
print("[%s] %-14s %12.0f CTU/s %7.3f ms/step  res %.3f intra %.3f sao %.3f serial %.3f  verified %s"
      % (sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], p.get("residual_ms", 0), p.get("intra_ms", 0),
         p.get("sao_ms", 0), p.get("total_ms", 0), v.get("ok")))
PY
  done
done
