#!/bin/bash
# r05 gemm3: 128 x 128 tiles from 192 of them (SD_G3_T128=192, _lib_v1: the S2 input-gradient GEMMs of 240 tiles
# leave 64 x 64): bit identity with the default build, GEMM tests on the variant, update A/B
set -o pipefail
O=gpurun_out/r05t128; mkdir -p $O
timeout -k 10 300 python3 tools/lib_bitcheck.py /tmp/a.npz > $O/run_a.txt 2>&1 &&
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so timeout -k 10 300 python3 tools/lib_bitcheck.py /tmp/b.npz > $O/run_b.txt 2>&1 &&
{ python3 tools/lib_bitcheck.py cmp /tmp/a.npz /tmp/b.npz > $O/bitcheck.txt 2>&1; true; } &&
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_gemm.py > $O/tests_v1.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so" > $O/ab.txt 2>&1
