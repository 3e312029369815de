#!/bin/bash
# Round-3 closing pass (second session): GPU suite, smoke, the bench lines (default, infer, collect,
# rnn, U = 64) and rocprofv3 kernel stats of the infer and collect lines.
#   gpurun --timeout 1200 -- bash tools/gpu_r3_close.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3c}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 &&
echo PYTEST_OK && tail -n 2 gpurun_out/${tag}_pytest.log &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err && echo BENCH_OK &&
timeout -k 10 200 python3 bench.py --workload infer > gpurun_out/${tag}_infer.json 2> gpurun_out/${tag}_infer.err && echo INFER_OK &&
timeout -k 10 200 python3 bench.py --workload collect > gpurun_out/${tag}_collect.json 2> gpurun_out/${tag}_collect.err && echo COLLECT_OK &&
timeout -k 10 200 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/${tag}_rnn.json 2> gpurun_out/${tag}_rnn.err && echo RNN_OK &&
timeout -k 10 200 python3 bench.py --updates-per-step 64 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_u64.json 2> gpurun_out/${tag}_u64.err && echo U64_OK &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_infer -o k -- \
    python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/prof_${tag}_infer.log 2>&1 && echo PROF_INFER_OK &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_collect -o k -- \
    python3 bench.py --workload collect --no-cpu-baseline > gpurun_out/prof_${tag}_collect.log 2>&1 && echo PROF_COLLECT_OK
