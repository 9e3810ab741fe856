#!/bin/bash
# k_hid_areg with 3 B stages (default) against 2 (_lib_s2) and against k_hid<true> (SDHIP_KH_NOAREG=1): imagination
# tests, step traces, update A/B. Usage: bash tools/r05_areg2.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagine.py \
  > $O/tests_imagine.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace/libsdhip.so timeout -k 10 200 python -u tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace_s2/libsdhip.so timeout -k 10 200 python -u tools/imag_trace.py > $O/imag_trace_s2.txt 2>&1 || exit 1
SDHIP_KH_NOAREG=1 SDHIP_LIB=$L/_lib_trace/libsdhip.so timeout -k 10 200 python -u tools/imag_trace.py > $O/imag_trace_noareg.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_LIB=$L/_lib_s2/libsdhip.so" "SDHIP_KH_NOAREG=1" > $O/ab.txt 2>&1 || exit 1
