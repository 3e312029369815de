#!/bin/bash
# Round-3 baselines: the U = 64 stress line of configs[2] and the QNetRNN line, each under
# rocprofv3 --kernel-trace --stats (per-kernel averages), plus the plain U = 64 bench line.
#   gpurun --timeout 900 -- bash tools/gpu_r3_base.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --updates-per-step 64 --steps 20 --warmup 10 --no-cpu-baseline \
    > gpurun_out/${tag}_u64.json 2> gpurun_out/${tag}_u64.err && echo U64_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_u64 -o k -- \
    python3 bench.py --updates-per-step 64 --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/prof_${tag}_u64.log 2>&1 &&
echo PROF_U64_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_rnn -o k -- \
    python3 bench.py --workload rnn --steps 50 --no-cpu-baseline > gpurun_out/prof_${tag}_rnn.log 2>&1 &&
echo PROF_RNN_OK
