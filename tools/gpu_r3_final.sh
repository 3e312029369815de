#!/bin/bash
# Round-3 closing pass: GPU suite, smoke, the four bench lines, kernel stats and the RNN counter passes.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3z}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 &&
echo PYTEST_OK &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 600 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err && echo BENCH_OK &&
timeout -k 10 300 python3 bench.py --workload infer > gpurun_out/${tag}_infer.json 2> gpurun_out/${tag}_infer.err && echo INFER_OK &&
timeout -k 10 300 python3 bench.py --workload rnn > gpurun_out/${tag}_rnn.json 2> gpurun_out/${tag}_rnn.err && echo RNN_OK &&
timeout -k 10 300 python3 bench.py --updates-per-step 64 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_u64.json 2> gpurun_out/${tag}_u64.err && echo U64_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_rnn -o k -- \
    python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/prof_${tag}_rnn.log 2>&1 && echo PROF_RNN_OK &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_${tag}r_fetch -o p -- \
    python3 bench.py --workload rnn --steps 30 --no-cpu-baseline > gpurun_out/pmc_${tag}r_fetch.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_${tag}r_write -o p -- \
    python3 bench.py --workload rnn --steps 30 --no-cpu-baseline > gpurun_out/pmc_${tag}r_write.log 2>&1 && echo PMC_RNN_OK
