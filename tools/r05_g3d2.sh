#!/bin/bash
# r05 split-bf16 two-deep register prefetch (SD_G3_D2=1: 128-row tiles, _lib_v1; =2: all, _lib_v2) on the final tree
set -o pipefail
O=gpurun_out/r05d2; mkdir -p $O
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v2/libsdhip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_gemm.py > $O/tests_v2.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v2/libsdhip.so" > $O/ab.txt 2>&1
