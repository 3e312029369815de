#!/bin/bash
# FETCH / WRITE counter passes of the collect bench (--workload collect, 65 536 arenas, 15-step launches),
# one pass per run: profiles/r3_collect_pmc.json via tools/pmc_summary.py r3c.
#   gpurun --timeout 600 -- bash tools/gpu_r3_collect_pmc.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in "fetch FETCH_SIZE GRBM_GUI_ACTIVE" "write WRITE_SIZE GRBM_GUI_ACTIVE"; do
    set -- $pass; name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_r3c_${name} -o p -- \
        python3 bench.py --workload collect --steps 300 --warmup 150 --no-cpu-baseline > gpurun_out/pmc_r3c_${name}.log 2>&1 || exit 1
done && echo PMC_COLLECT_OK
