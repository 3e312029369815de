#!/bin/bash
# The persistent DRQN update: its tests, its time alone, the RNN bench line, kernel stats.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_drqn.py \
    > gpurun_out/${tag}_drqn_tests.log 2>&1 && echo DRQN_TESTS_OK &&
timeout -k 10 120 python3 tools/drqn_time.py > gpurun_out/${tag}_drqn_time.json 2>gpurun_out/${tag}_drqn_time.err &&
echo DRQN_TIME_OK &&
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rnn_selfplay.py \
    > gpurun_out/${tag}_rnnsp_tests.log 2>&1 && echo RNNSP_TESTS_OK &&
timeout -k 10 300 python3 bench.py --workload rnn --steps 100 --no-cpu-baseline > gpurun_out/${tag}_rnn.json 2> gpurun_out/${tag}_rnn.err &&
echo RNN_BENCH_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_drqn -o k -- \
    python3 tools/drqn_time.py > gpurun_out/prof_${tag}_drqn.log 2>&1 && echo PROF_DRQN_OK
