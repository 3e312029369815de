#!/bin/bash
# Diagnostic timelines (libpongmi_diag.so): per-block phases of the fused act + env kernel, per-block
# k_act_sp roles, the in-kernel phase stamps of one overlapped vector step.
#   make -C pingpong-selfplay-ai_amd/csrc diag && gpurun --timeout 400 -- bash tools/gpu_diag.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/env_blocks.py > gpurun_out/env_blocks.txt 2>&1 && echo E_OK &&
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps.txt 2>&1 && echo S_OK
