#!/bin/bash
# Learner change check: the self-play parity tests (oracle, sum tree == rebuild, fused/split, multi-update,
# sharded), then the in-kernel phase stamps and the step probe.
#   gpurun --timeout 900 -- bash tools/gpu_learn_check.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_comm.py tests/test_gpu_qnet_replay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_learn.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps3.txt 2>&1 && echo S_OK &&
timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/probe3.txt 2>&1 && echo P_OK
