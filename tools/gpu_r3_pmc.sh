#!/bin/bash
# Round-3 counters: the four PMC passes of the default bench (tools/pmc_passes.sh), FETCH / WRITE
# passes of the infer and rnn benches, and the infer bench's kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_passes.sh r3 > gpurun_out/pmc_r3.log 2>&1 && echo PMC_DEFAULT_OK &&
for pass in "fetch FETCH_SIZE GRBM_GUI_ACTIVE" "write WRITE_SIZE GRBM_GUI_ACTIVE"; do
    set -- $pass; name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_r3i_${name} -o p -- \
        python3 bench.py --workload infer --steps 2000 --infer-chunk 2000 --no-cpu-baseline > gpurun_out/pmc_r3i_${name}.log 2>&1 || exit 1
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_r3r_${name} -o p -- \
        python3 bench.py --workload rnn --steps 30 --no-cpu-baseline > gpurun_out/pmc_r3r_${name}.log 2>&1 || exit 1
done && echo PMC_INFER_RNN_OK &&
timeout -k 10 300 python3 bench.py --workload infer > gpurun_out/r3i_infer.json 2> gpurun_out/r3i_infer.err && echo INFER_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3i_infer -o k -- \
    python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/prof_r3i_infer.log 2>&1 && echo PROF_INFER_OK
