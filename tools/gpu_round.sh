#!/bin/bash
# Round-end evidence on one GPU: default bench line (with CPU baseline), the QNetRNN bench line, the
# sharded-step probe, and rocprofv3 kernel stats of the default bench. Each step has its own limit.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$tag.log 2>&1 && echo BENCH_OK &&
timeout -k 10 300 python3 bench.py --workload rnn > gpurun_out/rnn_bench_$tag.log 2>&1 && echo RNN_OK &&
timeout -k 10 200 python3 tools/shard_probe.py > gpurun_out/shard_probe_$tag.txt 2>&1 && echo SHARD_OK &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o k -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 && echo STATS_OK
