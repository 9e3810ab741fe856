#!/bin/bash
# r05 k_logit_rows: 4 x1p slabs instead of 8 (SD_LR_NG=4 build,
# _lib_v1): scan parity on the variant, scan traces, update A/B
set -o pipefail
O=gpurun_out/r05ng; mkdir -p $O
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_scan.py > $O/tests_v1.txt 2>&1 &&
timeout -k 10 120 python3 tools/scan_trace.py > $O/scan_trace.txt 2>&1 &&
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_trace_v1/libsdhip.so timeout -k 10 120 python3 tools/scan_trace.py > $O/scan_trace_v1.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so" > $O/ab.txt 2>&1
