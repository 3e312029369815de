#!/bin/bash
# Write-through store check: K1 parity both store modes, K1 launch times at three sizes with the
# store mode forced each way, then the DQN step probe (product library).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wt in 0 1; do
  PONGMI_K1_WT=$wt timeout -k 10 200 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_wt$wt.log 2>&1 || { tail -20 gpurun_out/pytest_wt$wt.log; exit 1; }
  tail -1 gpurun_out/pytest_wt$wt.log
done
for rep in 1 2; do
  for wt in 0 1; do
    echo "== PONGMI_K1_WT=$wt" >> gpurun_out/wt_k1.txt
    PONGMI_K1_WT=$wt timeout -k 10 90 python3 tools/k1_time.py 65536 131072 262144 >> gpurun_out/wt_k1.txt 2>&1 || exit 1
  done
done
timeout -k 10 120 python3 tools/step_probe.py 2>&1 | grep '"overlap": true' >> gpurun_out/wt_probe.txt
