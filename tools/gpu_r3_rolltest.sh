#!/bin/bash
# The rollout / collect parity tests alone.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${1:-rt}_pytest.log 2>&1 && echo PYTEST_OK && tail -n 3 gpurun_out/${1:-rt}_pytest.log
