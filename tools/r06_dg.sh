#!/bin/bash
# Stage-2 ring forward (MT 4 default) and bwd-data on 64-pixel waves: conv tests, timings, same-box A/B of the update
# (default vs the 32-pixel-wave kernels). Usage: bash tools/r06_dg.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/conv6_time.py > $O/conv6_time.txt 2>&1 &&
timeout -k 10 200 python3 tools/dgrad_time.py > $O/dgrad_time.txt 2>&1 &&
timeout -k 10 900 bash tools/ab_env.sh 3 "" "SDHIP_DGRAD_MT=2" "SDHIP_DGRAD_MT=2 SDHIP_CONV6_MT=2" > $O/ab.txt 2>&1
