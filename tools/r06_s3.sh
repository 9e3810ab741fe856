#!/bin/bash
# Stage-3 bf16x6 ring (channel-group-major patch): kernel tests, per-variant timing, then the C5 bundle (r06_c5.sh).
# Usage: bash tools/r06_s3.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "bf16x6" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/conv6_time.py > $O/conv6_time.txt 2>&1 &&
timeout -k 10 600 bash tools/ab_env.sh 2 "" "SDREAMER_CONV6=1" > $O/ab.txt 2>&1 &&
bash tools/r06_c5.sh $1
