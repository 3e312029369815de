#!/bin/bash
# The whole GPU suite, one process (gpurun --timeout 600 -- bash tools/gpu_suite.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread \
    > gpurun_out/r4_suite.log 2>&1; rc=$?; tail -n 3 gpurun_out/r4_suite.log; exit $rc
