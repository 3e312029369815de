set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_drqn.py > gpurun_out/dq_t.log 2>&1 && timeout -k 10 120 python3 tools/drqn_time.py > gpurun_out/dq_time.json 2>&1 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dq -o k -- python3 tools/drqn_time.py > gpurun_out/prof_dq.log 2>&1
