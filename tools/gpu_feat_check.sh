#!/bin/bash
# Features-ahead check: DQN self-play / comm / generation parity tests, the step probe, the k_actenv
# block timeline (diag build).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_comm.py tests/test_gpu_generations.py tests/test_gpu_qnet_replay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_feat.log 2>&1; tail -2 gpurun_out/pytest_feat.log
timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/probe_feat.txt 2>&1; grep '"overlap": true' gpurun_out/probe_feat.txt
timeout -k 10 120 python3 tools/env_blocks.py > gpurun_out/env_blocks_feat.txt 2>&1; grep -v amdgpu gpurun_out/env_blocks_feat.txt
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps_feat.txt 2>&1; grep -E "learn start|learn loads|learn end" gpurun_out/stamps_feat.txt
