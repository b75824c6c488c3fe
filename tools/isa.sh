#!/bin/bash
# Device assembly of the product library + per-kernel summary of the row kernels:
#   tools/isa.sh [out.s] [extra hipcc flags...]
out=${1:-/tmp/isa/p265r.s}; shift || true
mkdir -p "$(dirname "$out")"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -structurizecfg-skip-uniform-regions=true --cuda-device-only -S "$@" -o "$out" p265_amd/csrc/p265r.hip || exit 1
python3 - "$out" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\w*(?:intra_rows_kernel|sao_rows_kernel|sao_strip16_kernel|sao16_strip_kernel|loopfilter16_kernel|residual\w*_kernel|intra_prep_kernel|loopfilter_kernel|dbk_map_kernel|intra_step_kernel)\w*):[^\n]*\n(.*?)^\.Lfunc_end', txt, re.S | re.M):
    name, code = m.group(1), m.group(2)
    k = re.search(r'\.amdhsa_kernel ' + name + r'\n(.*?)\.end_amdhsa_kernel', txt, re.S)
    body = k.group(1) if k else ''
    def n(p): return len(re.findall(p, code, re.M))
    SAL = r'^\s+s_(?!waitcnt|nop|cbranch|branch|barrier|setprio|sleep)'; VAL = r'^\s+v_'
    SE, ML, SO = r'saveexec', r'v_mul_lo_u32', r'scratch_(load|store)'
    v = re.search(r'\.amdhsa_next_free_vgpr (\d+)', body); s = re.search(r'\.amdhsa_next_free_sgpr (\d+)', body)
    sc = re.search(r'\.amdhsa_private_segment_fixed_size (\d+)', body)
    short = re.sub(r'EvPK.*', '', name.replace('_ZN5p265r', ''))
    print(f"{short:44s} vgpr={v.group(1) if v else '?'} sgpr={s.group(1) if s else '?'} scratch={sc.group(1) if sc else '?'} "
          f"lines={code.count(chr(10))} saveexec={n(SE)} mul_lo={n(ML)} scratch_ops={n(SO)} salu={n(SAL)} valu={n(VAL)}")
PY
