#!/bin/bash
# Stage-2 ring forward with 64 pixels per wave (SDHIP_CONV6_MT=4): conv tests, per-variant timing, then same-box A/B
# of the update (multi-tile and one-tile workgroups). Usage: bash tools/r06_mt4.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/conv6_time.py > $O/conv6_time.txt 2>&1 &&
timeout -k 10 900 bash tools/ab_env.sh 3 "" "SDHIP_CONV6_MT=4" "SDHIP_CONV6_MT=4 SDHIP_CONV6_TPW=1" > $O/ab.txt 2>&1
