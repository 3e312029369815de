# Round 6 counter passes: the default bench (4 SQ/TCC passes), configs[1] (FETCH / WRITE at 2 000-step
# launches) and configs[4] (FETCH / WRITE), summarised on the box so only the JSON summaries come back.
set -o pipefail
bash tools/gpu.sh r6ai pmc pmcinfer && bash tools/gpu.sh r6airnn pmcrnn &&
python3 tools/pmc_summary.py r6ai gpurun_out --json gpurun_out/r6_pmc.json > gpurun_out/r6_pmc_summary.txt &&
python3 tools/pmc_summary.py r6aiinf gpurun_out --json gpurun_out/r6_infer_pmc.json > gpurun_out/r6_infer_pmc_summary.txt &&
python3 tools/pmc_summary.py r6airnn gpurun_out --json gpurun_out/r6_rnn_pmc.json > gpurun_out/r6_rnn_pmc_summary.txt &&
rm -rf gpurun_out/pmc_r6ai* && du -sh gpurun_out
