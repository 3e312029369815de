#!/bin/bash
# DRQN tests + line + stamps + profile, then the CU-reserve sweep of the RNN step.
set -o pipefail
bash tools/gpu_r4_drqn.sh && bash tools/gpu_r4_reserve.sh
