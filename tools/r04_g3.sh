#!/bin/bash
# 256-row weight-gradient tiles: GEMM tests, the shape timings with and without them, schedule A/B. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $O/gemm.txt 2>&1 || exit 1
timeout -k 10 120 python tools/gemm3_bench.py > $O/g3_default.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_m0/libsdhip.so timeout -k 10 120 python tools/gemm3_bench.py > $O/g3_m0.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_ng4/libsdhip.so timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread \
  tests/test_gpu_scan.py > $O/tests_ng4.txt 2>&1 || exit 1
bash tools/ab_env.sh 2 "" "SDHIP_LIB=$L/_lib_m0/libsdhip.so" "SDREAMER_PRIO=1" "SDREAMER_FILL_CUS=192:64" \
  "SDREAMER_AC_DEFER=1" "SDREAMER_SCAN_ROWTILE_FWD=8" "SDHIP_LIB=$L/_lib_ng4/libsdhip.so" > $O/ab.txt 2>&1
