#!/bin/bash
# Kernel trace of the configs[4] RNN line (gpurun --timeout 600 -- bash tools/gpu_r4_rnnprof.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4r_prof -o run -- python3 bench.py --workload rnn --steps 50 --warmup 60 --no-cpu-baseline > gpurun_out/r4r_prof.log 2>&1
tail -n 2 gpurun_out/r4r_prof.log
