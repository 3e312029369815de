#!/bin/bash
# Quick GPU pass after a kernel change: the -m gpu parity suite, then the vector-step probe, the
# diagnostic phase stamps (if libpongmi_diag.so is built) and the default bench line (no CPU
# baseline). Every GPU step has its own limit; the chain stops at the first failure.
#   gpurun --timeout 900 -- bash tools/gpu_quick.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-q}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/probe_$tag.log 2>&1 && echo PROBE_OK &&
{ [ ! -f pingpong-selfplay-ai_amd/pongmi/libpongmi_diag.so ] ||
  timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps_$tag.log 2>&1; } && echo STAMPS_OK &&
timeout -k 10 240 python3 bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 && echo BENCH_OK &&
tail -n 1 gpurun_out/bench_$tag.log
