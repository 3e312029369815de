#!/bin/bash
# Round 4: (1) K1 phase stamps (diagnostic library) and the launch floor (empty kernels, bare and
# under rocprofv3); (2) the featB A/B: the default configs[2] step (features computed ahead in the
# learner launch) against --no-features-ahead (k_actenv's env blocks run modelB's whole forward),
# each timed (bench line), kernel-traced and counted (FETCH_SIZE / WRITE_SIZE passes);
# (3) the tightened QNetRNN act-vs-oracle test.   gpurun --timeout 1200 -- bash tools/gpu_r4_feat.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4c}
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/k1_stamps.py 65536 > gpurun_out/${tag}_k1_stamps.txt 2>&1 && echo K1_STAMPS_OK || exit 1
timeout -k 10 60 ./tools/empty_probe > gpurun_out/${tag}_empty_bare.txt 2>&1 && echo EMPTY_OK || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_empty -o k -- \
    ./tools/empty_probe > gpurun_out/${tag}_empty_prof.txt 2>&1 && echo EMPTY_PROF_OK || exit 1
for v in "ahead" "noahead --no-features-ahead"; do
  set -- $v; name=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/${tag}_${name}.json 2> gpurun_out/${tag}_${name}.err \
      || { tail -5 gpurun_out/${tag}_${name}.err; exit 1; }
  echo BENCH_${name}_OK
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_${name} -o k -- \
      python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_${tag}_${name}.log 2>&1 || exit 1
  for pass in "fetch FETCH_SIZE GRBM_GUI_ACTIVE" "write WRITE_SIZE GRBM_GUI_ACTIVE"; do
    set -- $pass; pn=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_${tag}${name}_${pn} -o p -- \
        python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline $( [ $name = noahead ] && echo --no-features-ahead ) \
        > gpurun_out/pmc_${tag}${name}_${pn}.log 2>&1 || exit 1
  done
  echo PMC_${name}_OK
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rnn_selfplay.py -q -rA -k match_oracle --timeout 200 \
    --timeout-method thread > gpurun_out/${tag}_rnn_oracle.log 2>&1; tail -n 2 gpurun_out/${tag}_rnn_oracle.log
