#!/bin/bash
# Quick conv check: conv kernel tests and per-variant stage timing. Usage: bash tools/r06_quick.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/conv6_time.py > $O/conv6_time.txt 2>&1
