#!/bin/bash
# GPU suite + the collect line + its FETCH / WRITE counter passes (tools/gpu_r3_collect_pmc.sh).
#   gpurun --timeout 900 -- bash tools/gpu_r3_tail.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-t}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 &&
echo PYTEST_OK && tail -n 1 gpurun_out/${tag}_pytest.log &&
timeout -k 10 200 python3 bench.py --workload collect > gpurun_out/${tag}_collect.json 2> gpurun_out/${tag}_collect.err && echo COLLECT_OK &&
bash tools/gpu_r3_collect_pmc.sh
