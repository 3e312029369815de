#!/bin/bash
# One GPU-box validation pass: the -m gpu parity suite, smoke(), the default bench line.
# Every GPU step has its own time limit and the chain stops at the first failure.
#   gpurun --timeout 1100 -- bash tools/gpu_validate.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -n 1 gpurun_out/bench.log
