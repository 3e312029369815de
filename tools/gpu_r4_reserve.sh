#!/bin/bash
# configs[4] step time vs the CUs reserved for the DRQN update beside the opponents' act
# (PONGMI_RNN_RESERVE_CUS), after the DRQN rework (gpurun --timeout 600 -- bash tools/gpu_r4_reserve.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 64 0 32 96 64; do
  PONGMI_RNN_RESERVE_CUS=$r timeout -k 10 200 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/r4v_rnn_$r.json 2> gpurun_out/r4v_rnn_$r.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r4v_rnn_$r.json')); print('reserve $r', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms/step')"
done
