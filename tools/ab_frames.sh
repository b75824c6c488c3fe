set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --experiment --steps 30 --warmup 4 --no-cpu-baseline --no-e2e "$@" > gpurun_out/ab.log 2>&1; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.0f %.3f intra %.3f serial %.3f' % (d['value'], d['ms_per_step'], d['phases_ms_per_step']['intra_ms'], d['phases_ms_per_step']['total_ms']))"; }
for rep in 1 2; do
echo "[$rep] W8 auto f512:" $(run --frames 512)
echo "[$rep] W8 lean f768:" $(P265R_LEAN=1 P265R_FAIR=0 run --frames 768)
echo "[$rep] W8 auto f768:" $(run --frames 768)
echo "[$rep] W12 f512:" $(P265R_ROW_WAVES=12 P265R_FAIR=0 run --frames 512)
done
P265R_LEAN=1 P265R_FAIR=0 P265R_DEBUG_SYNC=1 timeout -k 10 120 python bench.py --experiment --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --pipeline 1 --frames 768 > gpurun_out/diag768.log 2>&1; grep -E "rows kernel|XCC|sharing" gpurun_out/diag768.log | head -6
