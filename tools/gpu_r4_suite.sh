#!/bin/bash
# Round-4: the -m gpu suite (all failures reported, not -x) and smoke.
#   gpurun --timeout 900 -- bash tools/gpu_r4_suite.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4}
mkdir -p gpurun_out
timeout -k 10 780 python3 -u -m pytest tests -m gpu -q -rA --durations=15 --timeout 200 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -n 3 gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (read the log); anything else: stop here
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && echo SMOKE_OK
exit $rc
