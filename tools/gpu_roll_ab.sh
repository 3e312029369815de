#!/bin/bash
# Same-box A/B of K9 / collecting-rollout builds: each libpongmi*.so variant under pongmi/ (selected
# through PONGMI_LIB) runs the infer and collect bench lines, two interleaved rounds; the default
# library also runs the rollout parity tests first.
#   gpurun --timeout 900 -- bash tools/gpu_roll_ab.sh <tag> <variant>...   (variant: "" = libpongmi.so, w3 = libpongmi_w3.so)
set -o pipefail
export TMPDIR=/tmp
tag=${1:-ab}; shift
D=$PWD/pingpong-selfplay-ai_amd/pongmi
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 && echo PYTEST_OK || exit 1
for r in 1 2; do
  for v in "$@"; do
    lib=$D/libpongmi${v:+_$v}.so
    PONGMI_LIB=$lib timeout -k 10 200 python3 bench.py --workload infer --no-cpu-baseline > gpurun_out/${tag}_infer_${v:-def}_$r.json 2>/dev/null &&
    PONGMI_LIB=$lib timeout -k 10 200 python3 bench.py --workload collect --no-cpu-baseline > gpurun_out/${tag}_collect_${v:-def}_$r.json 2>/dev/null || exit 1
  done
  echo ROUND_$r
done
python3 - "$tag" <<'PY'
import json, sys, glob
t = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{t}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"] / 1e9, 4), "G/s", d["roofline"]["avg_us_per_step"], "us/step")
PY
