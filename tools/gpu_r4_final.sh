#!/bin/bash
# Round-4 closing pass on one box: GPU suite, smoke, the default / RNN / infer lines, the counter
# passes of the default and RNN workloads, the default line's kernel trace.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_final.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4f_pytest.log 2>&1; rc=$?; tail -n 2 gpurun_out/r4f_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 && echo SMOKE_OK || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err && echo BENCH_OK || exit 1
timeout -k 10 300 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/r4f_rnn.json 2> gpurun_out/r4f_rnn.err && echo RNN_OK || exit 1
timeout -k 10 300 python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/r4f_infer.json 2> gpurun_out/r4f_infer.err && echo INFER_OK || exit 1
bash tools/pmc_passes.sh r4 && echo PMC_DQN_OK &&
bash tools/pmc_rnn_passes.sh r4rnn && echo PMC_RNN_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4k_prof -o k -- python3 bench.py --no-cpu-baseline \
    > gpurun_out/r4k_prof.log 2>&1 && echo TRACE_OK
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d_prof -o drqn -- python3 tools/drqn_prof.py > gpurun_out/r4d_prof.log 2>&1 && echo DRQN_TRACE_OK
