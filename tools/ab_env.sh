export TMPDIR=/tmp; mkdir -p gpurun_out
for v in main alt main2; do
  if [ $v = alt ]; then export PONGMI_LIB=$PWD/pingpong-selfplay-ai_amd/pongmi/libpongmi_alt.so; else unset PONGMI_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_$v -o k -- python bench.py --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit 1
done
