#!/bin/bash
# Round 4: DRQN update work — its GPU tests, the RNN bench line (drqn_roofline: update_us, recur_us)
# and, optionally, the in-kernel stamps of the recurrence (diagnostic library).
#   gpurun --timeout 900 -- bash tools/gpu_r4_drqn.sh <tag> [stamps]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4d}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_drqn.py tests/test_gpu_rnn_selfplay.py tests/test_gpu_comm.py -q -x \
    --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; tail -n 2 gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/${tag}_pytest.log | head -20; exit 1; }
timeout -k 10 300 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/${tag}_rnn.json 2> gpurun_out/${tag}_rnn.err \
    || { tail -5 gpurun_out/${tag}_rnn.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_rnn.json'))
print('rnn value', d['value'], 'ms/step', d['ms_per_step'], 'env_update_us', d.get('env_update_us'), 'act_us', d['roofline']['avg_us'])
print('drqn', {k: d['drqn_roofline'][k] for k in ('update_us', 'recur_us', 'frac')})"
if [ "$2" = stamps ]; then
  timeout -k 10 200 python3 tools/drqn_stamps.py > gpurun_out/${tag}_drqn_stamps.txt 2>&1 && echo STAMPS_OK
fi
