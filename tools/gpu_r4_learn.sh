#!/bin/bash
# The fused DQN step's in-kernel phase stamps (diagnostic library) and a kernel-trace of the default line.
#   make -C pingpong-selfplay-ai_amd/csrc diag && gpurun --timeout 600 -- bash tools/gpu_r4_learn.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/r4l_stamps.txt 2>&1; tail -n 40 gpurun_out/r4l_stamps.txt
