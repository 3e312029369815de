#!/bin/bash
# Whole-tree GPU check: full `-m gpu` suite, smoke(), the default and RNN bench lines, and rocprofv3
# kernel stats of the default bench. Each step has its own limit; the chain stops at the first failure.
#   gpurun --timeout 900 -- bash tools/gpu_check_all.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r2e}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1 && tail -1 gpurun_out/pytest_$tag.log &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 240 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && echo BENCH_OK &&
timeout -k 10 240 python3 bench.py --workload rnn > gpurun_out/bench_rnn_$tag.json 2>> gpurun_out/bench_$tag.err && echo RNN_OK &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o k -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 && echo ALL_OK
