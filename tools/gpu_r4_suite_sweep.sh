#!/bin/bash
# Full GPU suite, then the CU-reserve sweep of the RNN step.
set -o pipefail
bash tools/gpu_suite.sh && bash tools/gpu_r4_reserve.sh
