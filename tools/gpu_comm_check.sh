set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_selfplay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_comm.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python3 tools/shard_probe.py > gpurun_out/shard_probe.txt 2>&1 && echo PROBE_OK &&
timeout -k 10 120 python3 tools/env_blocks.py > gpurun_out/env_blocks2.txt 2>&1 && echo E_OK &&
timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps2.txt 2>&1 && echo S_OK
