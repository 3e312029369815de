#!/bin/bash
# One parameterised GPU runner (round 5; replaces the per-round tools/gpu_r*.sh one-offs, which stay
# only as the record of what earlier rounds ran). Every GPU step has its own time limit and the steps
# are chained with &&: the first failure, timeout or fault ends the call.
#
#   gpurun --timeout 900 -- bash tools/gpu.sh <tag> <task> [<task> ...]
#
# tasks:
#   suite      the whole `-m gpu` suite + smoke()
#   env        tests/test_gpu_env.py only (K1 parity)
#   k1         K1 A/B: parity of the A/B variant, graph-timed floor probe (tools/k1_floor), product K1 with
#              PONGMI_K1_PRO=1 / 0 (tools/k1_time.py, bench.time_env_step), rocprofv3 kernel traces
#   k1stamp    per-wave K1 phase cycles (diag build, tools/k1_stamps.py)
#   stampsnw   tools/stamps.py on the PM_DIAG_NOWAIT diag build (libpongmi_diag_nw.so)
#   stamps     diag build: k_learn phase stamps of the overlapped step (tools/stamps.py) and k_actenv's
#              per-block timeline (tools/env_blocks.py)
#   bench      python bench.py (the driver's default line)
#   rnn        python bench.py --workload rnn
#   rnnab:VAR=v1,v2  the RNN bench (no CPU leg) under each value, interleaved twice
#   infer      python bench.py --workload infer
#   inferab:VAR=v1,v2  tests/test_gpu_rollout.py under each value, then the infer bench interleaved twice
#   collectab:VAR=v1,v2  the same with the collect bench (SURVEY 8f3's collecting rollout)
#   prof       rocprofv3 --kernel-trace --stats of the default bench (no CPU legs)
#   pmc        the FETCH_SIZE / WRITE_SIZE passes of the default bench (tools/pmc_passes.sh)
#   pmcrnn     the same for the RNN bench (tools/pmc_rnn_passes.sh)
#   pmcinfer   the same for the configs[1] inference rollout (2 000-step launches)
#   drqn       tests/test_gpu_drqn.py + tools/drqn_time.py
#   side       k_learn's side blocks (act / feature) per role, under PONGMI_SIDE 1 / 0 (diag build)
#   roll       k_rollout16 per-step phase cycles (tools/roll_stamps.py, diag build)
#   ab:VAR=v1,v2  tests/test_gpu_selfplay.py under each value, then the default bench interleaved twice
#   drqnab:VAR=v1,v2  tests/test_gpu_drqn.py under v1, then tools/drqn_time.py interleaved three times
#   k1sweep    K1 events + rocprofv3 kernel traces at 65 536 .. 4 194 304 arenas
#   floorprof  tools/k1_floor under rocprofv3 (round 5 SIGSEGV check)
#   mstamps    k_learn_multi per-update phase stamps (diag and PM_DIAG_NOWAIT builds)
#   u64        bench.py --updates-per-step 64 (k_learn_multi), us per update
#   u64ab:VAR=v1,v2  the U = 64 line under each value, interleaved twice
#   sstamps    configs[4] side-A whole-group blocks / split tiles by phase (diag build)
#   train      bench.py --workload train (one config.yaml generation try, replay ratio 1)
#   floorbig   tools/k1_floor skeletons at 1 M and 4 M arenas (graph events)
#   gpus2      bench.py --gpus 2 must refuse on a 1-GPU box
#   pytest:<path>[::sel]  one test file / selection
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}; shift
mkdir -p gpurun_out
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
run_task() {
  case "$1" in
    suite)
      timeout -k 10 420 $PYT tests -m gpu > gpurun_out/${tag}_suite.log 2>&1 && tail -1 gpurun_out/${tag}_suite.log &&
      timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && echo SMOKE_OK ;;
    env)
      timeout -k 10 300 $PYT tests/test_gpu_env.py > gpurun_out/${tag}_env.log 2>&1 && tail -1 gpurun_out/${tag}_env.log ;;
    k1)
      for pro in ${K1_PARITY_PROS:-0}; do
        PONGMI_K1_PRO=$pro timeout -k 10 300 $PYT tests/test_gpu_env.py > gpurun_out/${tag}_env_pro$pro.log 2>&1 &&
            tail -1 gpurun_out/${tag}_env_pro$pro.log || return 1
      done &&
      timeout -k 10 120 ./tools/k1_floor 65536 > gpurun_out/${tag}_k1_floor.jsonl 2>&1 && cat gpurun_out/${tag}_k1_floor.jsonl &&
      for pro in ${K1_PROS:-3 0 3 0}; do
        echo "== PONGMI_K1_PRO=$pro" >> gpurun_out/${tag}_k1_time.txt
        PONGMI_K1_PRO=$pro timeout -k 10 120 python3 tools/k1_time.py 65536 262144 >> gpurun_out/${tag}_k1_time.txt 2>&1 || return 1
      done && grep -v amdgpu.ids gpurun_out/${tag}_k1_time.txt &&
      for pro in ${K1_PROF_PROS:-3 0}; do
        PONGMI_K1_PRO=$pro timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
            -d gpurun_out/${tag}_prof_k1_pro$pro -o k -- python3 tools/k1_time.py 65536 \
            > gpurun_out/${tag}_prof_k1_pro$pro.log 2>&1 || return 1
      done && echo K1_OK ;;
    k1stamp)
      for pro in ${K1_PROF_PROS:-3 0}; do
        PONGMI_K1_PRO=$pro timeout -k 10 120 python3 tools/k1_stamps.py > gpurun_out/${tag}_k1_stamps_pro$pro.txt 2>&1 &&
            grep -v amdgpu.ids gpurun_out/${tag}_k1_stamps_pro$pro.txt || return 1
      done ;;
    stamps)
      timeout -k 10 180 python3 tools/stamps.py > gpurun_out/${tag}_stamps.txt 2>&1 && grep -v amdgpu.ids gpurun_out/${tag}_stamps.txt &&
      timeout -k 10 180 python3 tools/env_blocks.py > gpurun_out/${tag}_env_blocks.txt 2>&1 && grep -v amdgpu.ids gpurun_out/${tag}_env_blocks.txt ;;
    stampsnw)  # the same k_learn stamps from the PM_DIAG_NOWAIT diag build (no vmcnt waits at the stamps;
               # make -C pingpong-selfplay-ai_amd/csrc DIAG_OUT=../pongmi/libpongmi_diag_nw.so BUILD=_build_nw EXTRA=-DPM_DIAG_NOWAIT diag)
      PONGMI_DIAG_LIB=$PWD/pingpong-selfplay-ai_amd/pongmi/libpongmi_diag_nw.so timeout -k 10 180 python3 tools/stamps.py \
          > gpurun_out/${tag}_stamps_nw.txt 2>&1 && grep -v amdgpu.ids gpurun_out/${tag}_stamps_nw.txt ;;
    bench)
      timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err && echo BENCH_OK ;;
    rnn)
      timeout -k 10 300 python3 bench.py --workload rnn > gpurun_out/${tag}_rnn.json 2> gpurun_out/${tag}_rnn.err && echo RNN_OK ;;
    rnnab:*)  # rnnab:VAR=v1,v2 — bench.py --workload rnn --no-cpu-baseline under each value, interleaved twice
      spec=${1#rnnab:}; var=${spec%%=*}; vals=${spec#*=}
      for rep in 1 2; do
        for v in ${vals//,/ }; do
          env $var=$v timeout -k 10 200 python3 bench.py --workload rnn --no-cpu-baseline > gpurun_out/${tag}_rnnab_${var}_${v//\//_}_$rep.json 2>/dev/null &&
              echo "$var=$v rep$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e6,2), d['ms_per_step'], d['drqn_roofline']['update_us'])" gpurun_out/${tag}_rnnab_${var}_${v//\//_}_$rep.json)" || return 1
        done
      done ;;
    infer)
      timeout -k 10 300 python3 bench.py --workload infer > gpurun_out/${tag}_infer.json 2> gpurun_out/${tag}_infer.err && echo INFER_OK ;;
    prof)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o k -- \
          python3 bench.py --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 && echo PROF_OK ;;
    pmc)
      timeout -k 10 600 bash tools/pmc_passes.sh ${tag} && echo PMC_OK ;;
    pmcrnn)
      timeout -k 10 600 bash tools/pmc_rnn_passes.sh ${tag} && echo PMCRNN_OK ;;
    pmcinfer)  # configs[1]: 2 000-step launches of the K9 rollout (the committed infer profile's shape)
      for c in "fetch FETCH_SIZE GRBM_GUI_ACTIVE" "write WRITE_SIZE GRBM_GUI_ACTIVE"; do
        set -- $c
        timeout -k 10 240 rocprofv3 --pmc $2 $3 --output-format csv -d gpurun_out/pmc_${tag}inf_$1 -o p -- \
            python3 bench.py --workload infer --steps 2000 --infer-chunk 2000 --no-cpu-baseline \
            > gpurun_out/pmc_${tag}inf_$1.log 2>&1 || return 1
      done && echo PMCINFER_OK ;;
    drqn)
      timeout -k 10 300 $PYT tests/test_gpu_drqn.py > gpurun_out/${tag}_drqn.log 2>&1 && tail -1 gpurun_out/${tag}_drqn.log &&
      timeout -k 10 120 python3 tools/drqn_time.py > gpurun_out/${tag}_drqn_time.txt 2>&1 && cat gpurun_out/${tag}_drqn_time.txt ;;
    ab:*)  # ab:VAR=v1,v2 — tests/test_gpu_selfplay.py under each value, then the bench interleaved twice
      spec=${1#ab:}; var=${spec%%=*}; vals=${spec#*=}
      for v in ${vals//,/ }; do
        env $var=$v timeout -k 10 300 $PYT tests/test_gpu_selfplay.py > gpurun_out/${tag}_ab_${var}_${v//\//_}.log 2>&1 &&
            echo "$var=$v $(tail -1 gpurun_out/${tag}_ab_${var}_${v//\//_}.log)" || return 1
      done &&
      for rep in 1 2; do
        for v in ${vals//,/ }; do
          env $var=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/${tag}_ab_${var}_${v//\//_}_$rep.json 2>/dev/null &&
              echo "$var=$v rep$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e9,4), d['ms_per_step'])" gpurun_out/${tag}_ab_${var}_${v//\//_}_$rep.json)" || return 1
        done
      done ;;
    side)  # k_learn's side-block timeline (diag build), under each PONGMI_SIDE grid
      for v in ${SIDE_MODES:-1 0}; do
        PONGMI_SIDE=$v timeout -k 10 180 python3 tools/side_blocks.py > gpurun_out/${tag}_side_$v.txt 2>&1 &&
            echo "PONGMI_SIDE=$v" && grep -v amdgpu.ids gpurun_out/${tag}_side_$v.txt || return 1
      done ;;
    drqnab:*)  # drqnab:VAR=v1,v2 — tests/test_gpu_drqn.py under v1, then tools/drqn_time.py interleaved three times
      spec=${1#drqnab:}; var=${spec%%=*}; vals=${spec#*=}; first=${vals%%,*}
      env $var=$first timeout -k 10 300 $PYT tests/test_gpu_drqn.py > gpurun_out/${tag}_drqnab.log 2>&1 &&
          echo "$var=$first $(tail -1 gpurun_out/${tag}_drqnab.log)" || return 1
      for rep in 1 2 3; do
        for v in ${vals//,/ }; do
          env $var=$v timeout -k 10 120 python3 tools/drqn_time.py 2>/dev/null | tail -1 | sed "s#^#$var=$v #" || return 1
        done
      done ;;
    inferab:*)  # inferab:VAR=v1,v2 — tests/test_gpu_rollout.py under each value, then the infer bench interleaved twice
      spec=${1#inferab:}; var=${spec%%=*}; vals=${spec#*=}
      for v in ${vals//,/ }; do
        env $var=$v timeout -k 10 300 $PYT tests/test_gpu_rollout.py > gpurun_out/${tag}_inferab_${var}_${v}.log 2>&1 &&
            echo "$var=$v $(tail -1 gpurun_out/${tag}_inferab_${var}_${v}.log)" || return 1
      done &&
      for rep in 1 2; do
        for v in ${vals//,/ }; do
          env $var=$v timeout -k 10 200 python3 bench.py --workload infer > gpurun_out/${tag}_inferab_${var}_${v}_$rep.json 2>/dev/null &&
              echo "$var=$v rep$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e9,4), d['ms_per_step'], d['roofline']['avg_us_per_step'], d['roofline']['frac'])" gpurun_out/${tag}_inferab_${var}_${v}_$rep.json)" || return 1
        done
      done ;;
    collectab:*)  # collectab:VAR=v1,v2 — tests/test_gpu_rollout.py under each value, then the collect bench interleaved twice
      spec=${1#collectab:}; var=${spec%%=*}; vals=${spec#*=}
      for v in ${vals//,/ }; do
        env $var=$v timeout -k 10 300 $PYT tests/test_gpu_rollout.py > gpurun_out/${tag}_collectab_${var}_${v}.log 2>&1 &&
            echo "$var=$v $(tail -1 gpurun_out/${tag}_collectab_${var}_${v}.log)" || return 1
      done &&
      for rep in 1 2; do
        for v in ${vals//,/ }; do
          env $var=$v timeout -k 10 200 python3 bench.py --workload collect --no-cpu-baseline > gpurun_out/${tag}_collectab_${var}_${v}_$rep.json 2>/dev/null &&
              echo "$var=$v rep$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e9,4), d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])" gpurun_out/${tag}_collectab_${var}_${v}_$rep.json)" || return 1
        done
      done ;;
    roll)  # k_rollout16 per-step phase cycles (diag build)
      timeout -k 10 120 python3 tools/roll_stamps.py > gpurun_out/${tag}_roll_stamps.txt 2>&1 && grep -v amdgpu.ids gpurun_out/${tag}_roll_stamps.txt ;;
    k1sweep)  # K1's asymptote: events at 65 536 .. 4 194 304 arenas, then one rocprofv3
              # kernel trace per size (the kernel outlasts the tracer's ~4.5 us launch period from 262 144 up)
      timeout -k 10 240 python3 tools/k1_time.py 65536 262144 1048576 4194304 > gpurun_out/${tag}_k1_sweep.jsonl 2>&1 &&
          grep -v amdgpu.ids gpurun_out/${tag}_k1_sweep.jsonl &&
      for n in 65536 262144 1048576 4194304; do
        timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_k1_$n -o k -- \
            python3 tools/k1_time.py $n > gpurun_out/${tag}_prof_k1_$n.log 2>&1 || return 1
      done && echo K1SWEEP_OK ;;
    floorprof)  # tools/k1_floor under rocprofv3 once (round 5's SIGSEGV), fault mapping handler on
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_floor -o k -- \
          ./tools/k1_floor 65536 ${FLOOR_WARM:-100} > gpurun_out/${tag}_prof_floor${K1F_ONLY:+_$K1F_ONLY}${K1F_NO16:+_no16}.log 2>&1; rc=$?
      grep -v amdgpu.ids gpurun_out/${tag}_prof_floor${K1F_ONLY:+_$K1F_ONLY}${K1F_NO16:+_no16}.log | tail -25; echo "k1_floor under rocprofv3 rc=$rc"; [ $rc -eq 0 ] ;;
    mstamps)  # k_learn_multi's per-update phase timeline (tools/multi_stamps.py, U = 64): diag build, then the
              # PM_DIAG_NOWAIT build (no vmcnt(0) waits at the stamps)
      timeout -k 10 180 python3 tools/multi_stamps.py --U 64 > gpurun_out/${tag}_mstamps.txt 2>&1 &&
          grep -v amdgpu.ids gpurun_out/${tag}_mstamps.txt &&
      PONGMI_DIAG_LIB=$PWD/pingpong-selfplay-ai_amd/pongmi/libpongmi_diag_nw.so timeout -k 10 180 python3 tools/multi_stamps.py \
          --U 64 > gpurun_out/${tag}_mstamps_nw.txt 2>&1 && grep -v amdgpu.ids gpurun_out/${tag}_mstamps_nw.txt ;;
    u64)  # SURVEY 8d's U = 64 stress line (k_learn_multi), no CPU legs
      timeout -k 10 300 python3 bench.py --updates-per-step 64 --no-cpu-baseline > gpurun_out/${tag}_u64.json 2> gpurun_out/${tag}_u64.err &&
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('u64', d['value'], d['us_per_update'])" gpurun_out/${tag}_u64.json ;;
    u64ab:*)  # u64ab:VAR=v1,v2 — the U = 64 line under each value, interleaved twice
      spec=${1#u64ab:}; var=${spec%%=*}; vals=${spec#*=}
      for rep in 1 2; do
        for v in ${vals//,/ }; do
          env $var=$v timeout -k 10 200 python3 bench.py --updates-per-step 64 --no-cpu-baseline > gpurun_out/${tag}_u64ab_${var}_${v//\//_}_$rep.json 2>/dev/null &&
              echo "$var=$v rep$rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e6,2), d['us_per_update'])" gpurun_out/${tag}_u64ab_${var}_${v//\//_}_$rep.json)" || return 1
        done
      done ;;
    sstamps)  # configs[4]'s side-A launch: whole-group blocks and split tiles by phase (tools/split_stamps.py, diag build)
      timeout -k 10 240 python3 tools/split_stamps.py > gpurun_out/${tag}_split_stamps.txt 2>&1 && grep -v amdgpu.ids gpurun_out/${tag}_split_stamps.txt ;;
    train)  # one config.yaml generation try at replay ratio 1 (bench.py --workload train)
      timeout -k 10 300 python3 bench.py --workload train > gpurun_out/${tag}_train.json 2> gpurun_out/${tag}_train.err &&
          cat gpurun_out/${tag}_train.json && echo TRAIN_OK ;;
    floorbig)  # tools/k1_floor (graph events) at 1 M and 4 M arenas: the skeletons' bandwidth beyond the latency regime
      for n in 1048576 4194304; do
        timeout -k 10 120 ./tools/k1_floor $n 20 > gpurun_out/${tag}_k1_floor_$n.jsonl 2>&1 && cat gpurun_out/${tag}_k1_floor_$n.jsonl || return 1
      done ;;
    gpus2)  # bench.py --gpus 2 on a 1-GPU box must refuse (exit 2, an error line), never print a 1-rank line
      timeout -k 10 120 python3 bench.py --gpus 2 --no-cpu-baseline > gpurun_out/${tag}_gpus2.json 2>&1; rc=$?
      cat gpurun_out/${tag}_gpus2.json; [ $rc -eq 2 ] && echo GPUS2_REFUSED_OK ;;
    pytest:*)
      sel=${1#pytest:}; lg=gpurun_out/${tag}_pytest_$(basename "${sel//::/_}" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-60).log
      timeout -k 10 400 $PYT -s "$sel" > $lg 2>&1 && tail -1 $lg ;;
    *) echo "unknown task $1"; return 2 ;;
  esac
}
for t in "$@"; do
  echo "### $t"
  run_task "$t" || { echo "FAILED: $t"; exit 1; }
done
echo ALL_OK
