#!/bin/bash
# Kernel trace + SQ counters of the SAO kernels (streaming sao_rows_kernel vs loopfilter_kernel).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_sao
mkdir -p $OUT
B="python bench.py --experiment --steps 3 --warmup 1 --unique 2 --no-cpu-baseline --no-e2e --pipeline 1"
for v in 1 0; do
P265R_SAO_ROWS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$v -o kt -- $B > $OUT/kt$v.log 2>&1
P265R_SAO_ROWS=$v timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq$v -o sq -- $B > $OUT/sq$v.log 2>&1
done
python3 - <<'PY'
import csv, collections, glob
for v in ('1','0'):
    rows=list(csv.DictReader(open(glob.glob('gpurun_out/prof_sao/kt%s/**/kt_kernel_stats.csv'%v, recursive=True)[0])))
    for r in rows:
        if 'sao' in r['Name'] or 'loopfilter' in r['Name']: print(v, r['Name'][:50], r['Calls'], r['AverageNs'])
    agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
    for r in csv.DictReader(open(glob.glob('gpurun_out/prof_sao/sq%s/**/sq_counter_collection.csv'%v, recursive=True)[0])):
        k=r['Kernel_Name'].split('(')[0]
        if 'sao' in k or 'loopfilter' in k:
            agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
    for k,d in agg.items():
        w=d['SQ_WAVES']
        print(v, k[-40:], 'waves %d'%w, ' '.join('%s %.0f'%(c.replace('SQ_',''), d[c]/w*(4 if 'CYCLES' in c or 'WAIT' in c else 1)) for c in sorted(d) if c!='SQ_WAVES'))
PY
