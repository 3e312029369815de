#!/bin/bash
# Final check of the round-4 tree: GPU suite, smoke, the default line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4g_pytest.log 2>&1; rc=$?; tail -n 2 gpurun_out/r4g_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g_smoke.log 2>&1 && echo SMOKE_OK || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err && echo BENCH_OK || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r4g_bench.json')); print('dqn', d['value'], d['ms_per_step'], d['learn_us'], d['actenv_us'], d['roofline']['frac'], d['env_step_roofline']['frac'])"
