#!/bin/bash
# A/B of experimental builds under _build_alt/<name>/: the DQN step probe (overlapped step, eager and
# graph), alternating the builds, ROUNDS times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-3}); do
  for v in "$@"; do
    echo "== $v" >> gpurun_out/ab_probe.txt
    PONGMI_LIB=$PWD/_build_alt/$v/libpongmi.so timeout -k 10 120 python3 tools/step_probe.py 2>&1 | \
        grep '"overlap": true' >> gpurun_out/ab_probe.txt || exit 1
  done
done
