#!/bin/bash
# Time K1 (tools/k1_time.py) against every library built under _build_alt/<variant>/ (experiments).
set -o pipefail
export TMPDIR=/tmp
for d in _build_alt/*/; do
  v=$(basename $d)
  echo "== $v"
  PONGMI_LIB=$PWD/${d}libpongmi.so timeout -k 10 60 python3 tools/k1_time.py ${K1_N:-65536} || exit 1
done
