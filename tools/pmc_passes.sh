#!/bin/bash
# PMC passes over a short bench run (each pass its own rocprofv3 invocation; counters only with
# --kernel-trace, as the pool requires). Output: gpurun_out/pmc_<tag>_<pass>/
set -e
TAG=${1:-r1}
STEPS=${STEPS:-40}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp

run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv \
    -d gpurun_out/pmc_${TAG}_${name} -o p -- python bench.py --steps $STEPS --warmup 5 --no-cpu-baseline \
    > gpurun_out/pmc_${TAG}_${name}.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
run sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run write WRITE_SIZE GRBM_GUI_ACTIVE
echo pmc done
