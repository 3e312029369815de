#!/bin/bash
# k_rnn_fold drawing noise only where read: the RNN GPU tests, the configs[4] line twice, a kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rnn_selfplay.py tests/test_gpu_rnn.py tests/test_gpu_generations.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4fo_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/r4fo_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 200 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/r4fo_rnn$i.json 2> gpurun_out/r4fo_rnn$i.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r4fo_rnn$i.json')); print('rnn', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4fo_prof -o run -- python3 bench.py --workload rnn --steps 50 --warmup 60 --no-cpu-baseline > gpurun_out/r4fo_prof.log 2>&1 && echo TRACE_OK
