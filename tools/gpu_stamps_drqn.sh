export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python3 tools/drqn_stamps.py > gpurun_out/r4d_stamps.txt 2>&1; tail -n 20 gpurun_out/r4d_stamps.txt
