#!/bin/bash
# Round-3 full pass: the GPU test suite, smoke(), the default bench line, configs[1] / configs[4] lines,
# and rocprofv3 kernel stats of the default bench and the RNN bench.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 &&
echo PYTEST_OK &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 600 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err && echo BENCH_OK &&
timeout -k 10 300 python3 bench.py --workload infer > gpurun_out/${tag}_infer.json 2> gpurun_out/${tag}_infer.err && echo INFER_OK &&
timeout -k 10 300 python3 bench.py --workload rnn > gpurun_out/${tag}_rnn.json 2> gpurun_out/${tag}_rnn.err && echo RNN_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_bench -o k -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_${tag}_bench.log 2>&1 && echo PROF_BENCH_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_rnn -o k -- \
    python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/prof_${tag}_rnn.log 2>&1 && echo PROF_RNN_OK
