#!/bin/bash
# DRQN recurrence rework: the DRQN tests, then the RNN line (update / recurrence times).
#   gpurun --timeout 600 -- bash tools/gpu_r4_drqn.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_drqn.py -x -v -s --timeout 120 --timeout-method thread \
    > gpurun_out/r4d_drqn.log 2>&1; rc=$?; tail -n 4 gpurun_out/r4d_drqn.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/r4d_rnn.json 2> gpurun_out/r4d_rnn.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r4d_rnn.json')); print('rnn', d['value'], d['ms_per_step'], json.dumps(d.get('drqn_roofline')))"
timeout -k 10 120 python3 tools/drqn_stamps.py > gpurun_out/r4d_stamps.txt 2>&1; tail -n 40 gpurun_out/r4d_stamps.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d_prof -o drqn -- python3 tools/drqn_prof.py > gpurun_out/r4d_prof.log 2>&1
echo DRQN_PROF_DONE
