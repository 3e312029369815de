#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/k1_placement.py > gpurun_out/k1_place.log 2>&1; rc=$?; cat gpurun_out/k1_place.log | grep -v amdgpu.ids; exit $rc
