#!/bin/bash
# r05 k_hid_areg2 (in-workgroup K split, 4 waves / SIMD; SDHIP_KH_KSPLIT=1): imagination tests on it, step traces,
# update A/B against k_hid_areg
set -o pipefail
O=gpurun_out/r05ks; mkdir -p $O
SDHIP_KH_KSPLIT=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_imagine.py -k "not hid_areg_bit and not presplit_images_bit" > $O/tests_ks.txt 2>&1 &&
SDHIP_KH_KSPLIT=1 timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace_ks.txt 2>&1 &&
timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_KH_KSPLIT=1" > $O/ab.txt 2>&1
