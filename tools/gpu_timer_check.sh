#!/bin/bash
# Launch-timer round: parity suites touching the timed launch sites, the DQN and RNN bench lines, and
# rocprofv3 kernel stats of both bench commands (the bench's avg_us must agree with these).
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r2d}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_rnn_selfplay.py tests/test_gpu_comm.py \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 && tail -1 gpurun_out/pytest_$tag.log &&
timeout -k 10 240 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err &&
timeout -k 10 240 python3 bench.py --workload rnn > gpurun_out/bench_rnn_$tag.json 2>> gpurun_out/bench_$tag.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o k -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rnn_$tag -o k -- \
    python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/prof_rnn_$tag.log 2>&1 && echo ALL_OK
