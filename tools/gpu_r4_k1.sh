#!/bin/bash
# Round 4: K1 one-vs-two arenas per lane (PONGMI_K1_PAIR), parity under the pair kernel, timings and
# rocprof kernel stats of each.   gpurun --timeout 900 -- bash tools/gpu_r4_k1.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4k1}
mkdir -p gpurun_out
PONGMI_K1_PAIR=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_env.py -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_pair_pytest.log 2>&1 && echo PAIR_PARITY_OK || { tail -30 gpurun_out/${tag}_pair_pytest.log; exit 1; }
for v in "0 1" "1 1" "1 0" "0 0"; do
  set -- $v
  echo "== pair=$1 wt=$2"
  PONGMI_K1_PAIR=$1 PONGMI_K1_WT=$2 timeout -k 10 120 python3 tools/k1_time.py 65536 262144 || exit 1
done
for pr in 0 1; do
  PONGMI_K1_PAIR=$pr timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_p$pr -o k -- \
      python3 tools/k1_time.py 65536 > gpurun_out/prof_${tag}_p$pr.log 2>&1 || exit 1
done
echo PROF_OK
