#!/bin/bash
# Rollout / collect parity tests (the launch's fused node rebuild against pm_per_sample's two-kernel
# build), then the collect line and its kernel stats.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-nd}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python3 bench.py --workload collect > gpurun_out/${tag}_collect.json 2> gpurun_out/${tag}_collect.err && echo COLLECT_OK &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_collect -o k -- \
    python3 bench.py --workload collect --no-cpu-baseline > gpurun_out/prof_${tag}_collect.log 2>&1 && echo PROF_COLLECT_OK
