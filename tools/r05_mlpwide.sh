#!/bin/bash
# r05 SD_MLP_WIDE=1 (128 x 256 tiles for the heads' normed hidden layers, _lib_v1): GEMM tests, update A/B
set -o pipefail
O=gpurun_out/r05mw; mkdir -p $O
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_gemm.py > $O/tests_v1.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so" > $O/ab.txt 2>&1
