#!/bin/bash
# k_lin6_areg: imagination tests, step traces with and without it, update A/B (SDHIP_KL_NOAREG=1 = k_lin6).
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagine.py \
  > $O/tests_imagine.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace/libsdhip.so timeout -k 10 200 python -u tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
SDHIP_KL_NOAREG=1 SDHIP_LIB=$L/_lib_trace/libsdhip.so timeout -k 10 200 python -u tools/imag_trace.py > $O/imag_trace_noareg.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_KL_NOAREG=1" > $O/ab.txt 2>&1 || exit 1
