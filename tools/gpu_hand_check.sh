#!/bin/bash
# Push-row hand-off check: DQN self-play / comm / generation parity suites, the step probe, phase stamps.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_comm.py tests/test_gpu_generations.py \
    -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_hand.log 2>&1; tail -3 gpurun_out/pytest_hand.log
grep -q " passed" gpurun_out/pytest_hand.log && ! grep -q "failed\|error" gpurun_out/pytest_hand.log || exit 1
timeout -k 10 120 python3 tools/step_probe.py 2>&1 | grep '"overlap": true' > gpurun_out/probe_hand.txt || exit 1
cat gpurun_out/probe_hand.txt
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps_hand.txt 2>&1
