#!/bin/bash
# The collect line (with its committed PMC traffic) and its rocprofv3 kernel stats.
#   gpurun --timeout 600 -- bash tools/gpu_r3_collect_final.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-cf}
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --workload collect > gpurun_out/${tag}_collect.json 2> gpurun_out/${tag}_collect.err && echo COLLECT_OK &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_collect -o k -- \
    python3 bench.py --workload collect --no-cpu-baseline > gpurun_out/prof_${tag}_collect.log 2>&1 && echo PROF_COLLECT_OK &&
timeout -k 10 200 python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/${tag}_infer.json 2> gpurun_out/${tag}_infer.err && echo INFER_OK
