#!/bin/bash
# A/B of the feature blocks' store delay in k_learn (libpongmi_fd<N>.so built with EXTRA=-DPM_FEAT_DELAY=N)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=pingpong-selfplay-ai_amd/pongmi
for rep in 1 2; do
for v in base fd1 fd2; do
  lib=$L/libpongmi.so; [ $v != base ] && lib=$L/libpongmi_$v.so
  PONGMI_LIB=$(pwd)/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/r4fd_${v}_$rep.json 2> gpurun_out/r4fd_${v}_$rep.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r4fd_${v}_$rep.json')); print('$v', round(d['value']/1e9,4), 'G', d['ms_per_step'], 'learn', d['learn_us'], 'actenv', d['actenv_us'])"
done
done
