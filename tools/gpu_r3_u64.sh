#!/bin/bash
# U = 64 stress line of configs[2]: the fused multi-update launch vs launches per update,
# then rocprofv3 kernel stats of the fused one.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --updates-per-step 64 --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/${tag}_u64.json 2> gpurun_out/${tag}_u64.err && echo U64_OK &&
timeout -k 10 300 python3 bench.py --updates-per-step 64 --steps 10 --warmup 3 --no-cpu-baseline --no-learn-multi \
    > gpurun_out/${tag}_u64_split.json 2> gpurun_out/${tag}_u64_split.err && echo U64_SPLIT_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_u64 -o k -- \
    python3 bench.py --updates-per-step 64 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${tag}_u64.log 2>&1 &&
echo PROF_U64_OK
