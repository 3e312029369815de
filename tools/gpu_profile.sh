#!/bin/bash
# Profile evidence for the round: rocprofv3 kernel stats + kernel trace of the default bench, then the
# PMC passes (each its own rocprofv3 run, counters with kernel trace only) and their per-kernel summary.
#   gpurun --timeout 1100 -- bash tools/gpu_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o k -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 && echo STATS_OK &&
bash tools/pmc_passes.sh $tag && echo PMC_OK &&
python3 tools/pmc_summary.py $tag gpurun_out --json gpurun_out/pmc_$tag.json > gpurun_out/pmc_${tag}_summary.txt 2>&1 &&
echo SUMMARY_OK
