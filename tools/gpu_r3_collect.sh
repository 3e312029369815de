#!/bin/bash
# Round-3 collecting rollout (pm_rollout_push, §8f3): its parity tests, then the configs[1] infer line
# (the K9 loop's heads prefetch now overlaps the step).
#   gpurun --timeout 900 -- bash tools/gpu_r3_collect.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-c}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/${tag}_infer.json \
    2> gpurun_out/${tag}_infer.err && echo INFER_OK && cat gpurun_out/${tag}_infer.json &&
timeout -k 10 300 python3 bench.py --workload collect > gpurun_out/${tag}_collect.json \
    2> gpurun_out/${tag}_collect.err && echo COLLECT_OK && cat gpurun_out/${tag}_collect.json
