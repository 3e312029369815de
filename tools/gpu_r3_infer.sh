#!/bin/bash
# configs[1] (the K9 inference rollout megakernel): parity tests, the bench line, rocprofv3 kernel stats.
#   gpurun --timeout 900 -- bash tools/gpu_r3_infer.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rollout.py \
    > gpurun_out/${tag}_rollout_tests.log 2>&1 && echo ROLLOUT_TESTS_OK &&
timeout -k 10 300 python3 bench.py --workload infer --cpu-seconds 10 > gpurun_out/${tag}_infer.json 2> gpurun_out/${tag}_infer.err &&
echo INFER_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_infer -o k -- \
    python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/prof_${tag}_infer.log 2>&1 &&
echo PROF_INFER_OK
