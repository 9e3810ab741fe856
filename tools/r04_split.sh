#!/bin/bash
# K-split target A/B (SDREAMER_G3_WGS) + GEMM tests. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $O/gemm.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDREAMER_G3_WGS=512" "SDREAMER_G3_WGS=2048" > $O/ab_split.txt 2>&1
