#!/bin/bash
# gpurun with retries ONLY when no box / slot was free (exit 3: nothing ran, nothing charged).
# Usage: tools/gpurun_retry.sh <out.txt> <timeout> '<command>'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
    timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
    rc=$?
    echo "rc=$rc" >> "$out"
    [ $rc -ne 3 ] && exit $rc
    sleep 90
done
exit 3
