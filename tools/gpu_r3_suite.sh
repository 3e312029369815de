#!/bin/bash
# The -m gpu suite and smoke on the final tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 &&
echo PYTEST_OK && tail -n 1 gpurun_out/fin_pytest.log &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 && echo SMOKE_OK
