#!/bin/bash
# The 256 x 256 heads first-layer kernel (SD_MLP_W256): GEMM tests, the launch alone against the 128 x 128 build
# (_lib_w0), the imagination / dreamer golden tests, and a same-box update A/B. Usage: bash tools/r05_w256.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py \
  > $O/tests_gemm.txt 2>&1 || exit 1
timeout -k 10 120 python tools/mlp_bench.py > $O/mlp.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_w0/libsdhip.so timeout -k 10 120 python tools/mlp_bench.py >> $O/mlp.txt 2>&1 || exit 1
timeout -k 10 120 python tools/mlp_bench.py >> $O/mlp.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dreamer.py \
  > $O/tests_dreamer.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_LIB=$L/_lib_w0/libsdhip.so" > $O/ab.txt 2>&1 || exit 1
