#!/bin/bash
# Local helper (this container only): submit one gpurun call, re-submitting only while the pool
# reports no free slot / a transient infrastructure failure (nothing ran, nothing charged).
# Usage: tools/gpq.sh <out-file> <timeout-s> '<command>'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
    /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
    rc=$?
    if grep -q "status=transient\|busy\|backing off" "$OUT" && ! grep -q "status=ok" "$OUT"; then
        sleep 60; continue
    fi
    exit $rc
done
exit 3
