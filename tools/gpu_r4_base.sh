#!/bin/bash
# Round 4 (second session) baseline on a fresh box: GPU suite, the default line and the RNN line.
#   gpurun --timeout 900 -- bash tools/gpu_r4_base.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4s_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/r4s_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r4s_bench.json 2> gpurun_out/r4s_bench.err || exit 1
cat gpurun_out/r4s_bench.json
timeout -k 10 300 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/r4s_rnn.json 2> gpurun_out/r4s_rnn.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r4s_rnn.json')); print('rnn', d['value'], json.dumps(d.get('drqn_roofline')))"
