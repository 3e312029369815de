#!/bin/bash
# The RNN step's earlier fork: the RNN GPU tests, then the configs[4] line twice.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rnn_selfplay.py tests/test_gpu_rnn.py tests/test_gpu_drqn.py tests/test_gpu_generations.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4fk_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/r4fk_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 200 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/r4fk_rnn$i.json 2> gpurun_out/r4fk_rnn$i.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r4fk_rnn$i.json')); print('rnn', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', d['drqn_roofline']['update_us'])"
done
