#!/bin/bash
# HBM-traffic PMC passes over a short `bench.py --workload rnn` run (FETCH_SIZE and WRITE_SIZE each in
# a rocprofv3 invocation of their own, counters with --kernel-trace only). Output: gpurun_out/pmc_<tag>_*/
#   gpurun -- bash tools/pmc_rnn_passes.sh r2rnn && python tools/pmc_summary.py r2rnn --json profiles/r2_rnn_pmc.json
set -e
TAG=${1:-r2rnn}
STEPS=${STEPS:-40}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out

run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv \
    -d gpurun_out/pmc_${TAG}_${name} -o p -- python bench.py --workload rnn --steps $STEPS --warmup 5 \
    --no-cpu-baseline > gpurun_out/pmc_${TAG}_${name}.log 2>&1
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run write WRITE_SIZE GRBM_GUI_ACTIVE
echo pmc done
