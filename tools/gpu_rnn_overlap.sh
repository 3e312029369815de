set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_rnn_selfplay.py tests/test_gpu_rnn.py tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_rnnov.log 2>&1; tail -2 gpurun_out/pytest_rnnov.log
for r in 64 96 128 32; do PONGMI_RNN_RESERVE_CUS=$r timeout -k 10 200 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/rnn_ov_$r.log 2>&1 || break; echo "reserve $r"; tail -1 gpurun_out/rnn_ov_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_us'], d.get('env_update_us'))"; done
