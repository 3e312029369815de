#!/bin/bash
# Round 4 mid-run: the restored k_rollout16 (rollout parity + configs[1] line) and the in-kernel phase
# stamps of one fused vector step (diagnostic library), for the learner chain.
#   make -C pingpong-selfplay-ai_amd/csrc diag && gpurun --timeout 600 -- bash tools/gpu_r4_mid.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rollout.py -q -x --timeout 200 --timeout-method thread \
    > gpurun_out/r4m_rollout.log 2>&1; rc=$?; tail -n 2 gpurun_out/r4m_rollout.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/r4m_infer.json 2> gpurun_out/r4m_infer.err &&
python3 -c "
import json; d=json.load(open('gpurun_out/r4m_infer.json')); print('infer', d['value'], d['roofline']['avg_us_per_step'], d['roofline']['frac'])" &&
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/r4m_stamps.txt 2>&1 && echo STAMPS_OK &&
timeout -k 10 120 python3 tools/multi_stamps.py > gpurun_out/r4m_multi_stamps.txt 2>&1 && echo MULTI_OK &&
timeout -k 10 120 python3 tools/roll_stamps.py > gpurun_out/r4m_roll_stamps.txt 2>&1 && echo ROLL_OK && cat gpurun_out/r4m_roll_stamps.txt || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_drqn.py -q -x -s --timeout 200 --timeout-method thread \
    > gpurun_out/r4m_drqn.log 2>&1; rc=$?; tail -n 2 gpurun_out/r4m_drqn.log; grep -E "band|gradient error" gpurun_out/r4m_drqn.log; exit $rc
