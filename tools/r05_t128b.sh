#!/bin/bash
# r05 gemm3 128 x 128 tile threshold, second A/B: default (256) vs 192 (_lib_v1) vs 128 (_lib_v2)
set -o pipefail
O=gpurun_out/r05t128b; mkdir -p $O
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v2/libsdhip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_gemm.py > $O/tests_v2.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v2/libsdhip.so" > $O/ab.txt 2>&1
