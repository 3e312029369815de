#!/bin/bash
# K1 (k_env_step) evidence pass: rocprof kernel stats of the default bench, the K1 probe against a
# same-bytes device copy, and the K1 lab's per-wave phase timeline + variant table.
#   gpurun --timeout 900 -- bash tools/gpu_k1prof.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-k1}
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o k -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 && echo PROF_OK &&
timeout -k 10 120 python3 tools/env_probe.py --n 65536 262144 1048576 > gpurun_out/probe_$tag.log 2>&1 && echo PROBE_OK &&
K1_STAMP=1 timeout -k 10 60 ./tools/k1_lab > gpurun_out/stamp_$tag.log 2>&1 && echo STAMP_OK &&
timeout -k 10 120 ./tools/k1_lab 65536 > gpurun_out/lab_$tag.log 2>&1 && echo LAB_OK
