#!/bin/bash
# One learner-kernel iteration on the GPU: the self-play parity suites, the diagnostic phase stamps
# of one vector step (libpongmi_diag.so), and the default bench line.
#   make -C pingpong-selfplay-ai_amd/csrc all diag && gpurun --timeout 600 -- bash tools/gpu_iter.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-it}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_qnet_replay.py tests/test_gpu_comm.py \
    -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 && tail -1 gpurun_out/pytest_$tag.log &&
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps_$tag.txt 2>&1 && echo STAMPS_OK &&
timeout -k 10 240 python3 bench.py --no-cpu-baseline > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && echo BENCH_OK
