#!/bin/bash
# Round-4 counter passes (default and RNN workloads) and the default line's kernel trace.
#   gpurun --timeout 900 -- bash tools/gpu_r4_pmc.sh
#   then: python tools/pmc_summary.py r4 --json profiles/r4_pmc.json
#         python tools/pmc_summary.py r4rnn --json profiles/r4_rnn_pmc.json
#         python tools/rocpd_stats.py gpurun_out/r4k_prof/k_results.db > profiles/r4_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_passes.sh r4 && echo PMC_DQN_OK &&
bash tools/pmc_rnn_passes.sh r4rnn && echo PMC_RNN_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4k_prof -o k -- python3 bench.py --no-cpu-baseline \
    > gpurun_out/r4k_prof.log 2>&1 && echo TRACE_OK
