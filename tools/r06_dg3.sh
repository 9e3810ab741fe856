#!/bin/bash
# Stage-3 bwd-data on whole-image tiles of 64-pixel waves (SDHIP_DGRAD3_MT=4): conv tests, timings, same-box A/B.
# Usage: bash tools/r06_dg3.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/dgrad_time.py > $O/dgrad_time.txt 2>&1 &&
timeout -k 10 900 bash tools/ab_env.sh 3 "" "SDHIP_DGRAD3_MT=4" > $O/ab.txt 2>&1
