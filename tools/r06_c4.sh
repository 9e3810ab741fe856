#!/bin/bash
# Stage-1 forward grid sized to one round of resident workgroups: conv tests, per-grid timing, then same-box A/B of
# the update against the round-5 grid (SDHIP_C4_TPW=16). Usage: bash tools/r06_c4.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/c4_time.py > $O/c4_time.txt 2>&1 &&
timeout -k 10 900 bash tools/ab_env.sh 3 "SDHIP_C4_TPW=16" "" > $O/ab.txt 2>&1
