#!/bin/bash
# k_learn change check: the self-play GPU tests, two default bench lines, the phase stamps.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_qnet_replay.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4l_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/r4l_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r4l_bench$i.json 2> gpurun_out/r4l_bench$i.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r4l_bench$i.json')); print('dqn', d['value'], d['ms_per_step'], d['learn_us'], d['actenv_us'])"
done
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/r4l_stamps.txt 2>&1; grep -E "learn|ph0|push" gpurun_out/r4l_stamps.txt
