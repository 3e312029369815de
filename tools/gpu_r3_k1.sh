#!/bin/bash
# The default bench line twice (no CPU legs): K1's env_step_roofline with the longer warm-up.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/k1_bench_$r.json 2> gpurun_out/k1_bench_$r.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/k1_bench_$r.json').read().strip().splitlines()[-1]); e=d['env_step_roofline']; print('$r', d['value'], d['ms_per_step'], e['avg_us'], e['frac'], e['dispatch_us'])"
done
