#!/bin/bash
# Round 4: K9 on 16-arena tiles — parity (test_gpu_rollout.py: inference and collecting launches, both
# tile widths) and the configs[1] / collect lines, 16- vs 32-arena tiles (PONGMI_ROLL16 bit 0: the
# inference launch, bit 1: the collecting launch), plus rocprof kernel stats of the 16-tile launch.
#   gpurun --timeout 900 -- bash tools/gpu_r4_roll16.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4r}
mkdir -p gpurun_out
PONGMI_ROLL16=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rollout.py -q -x --timeout 200 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1; rc=$?; tail -n 2 gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/${tag}_pytest.log | head -20; exit 1; }
for v in 1 0; do
  PONGMI_ROLL16=$v timeout -k 10 300 python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/${tag}_infer$v.json \
      2> gpurun_out/${tag}_infer$v.err || { tail -5 gpurun_out/${tag}_infer$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_infer$v.json'))
print('infer roll16=$v', d['value'], d['roofline']['avg_us_per_step'], d['roofline']['frac'])"
done
for v in 3 1; do
  PONGMI_ROLL16=$v timeout -k 10 300 python3 bench.py --workload collect --no-cpu-baseline > gpurun_out/${tag}_collect$v.json \
      2> gpurun_out/${tag}_collect$v.err || { tail -5 gpurun_out/${tag}_collect$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_collect$v.json'))
print('collect roll16=$v', d['value'], d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_infer -o k -- \
    python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/prof_${tag}_infer.log 2>&1 && echo PROF_OK
