#!/bin/bash
# Schedule-knob and scan-variant A/B on the current build (same box, alternated). Output gpurun_out/$1/ab_sched.txt
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
SDHIP_LIB=$L/_lib_ng4/libsdhip.so timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread \
  tests/test_gpu_scan.py > $O/tests_ng4.txt 2>&1 || exit 1
bash tools/ab_env.sh 2 "" "SDREAMER_PRIO=1" "SDREAMER_FILL_CUS=192:64" "SDREAMER_AC_DEFER=1" "SDREAMER_DEFER_WM=1" \
  "SDREAMER_SCAN_ROWTILE_FWD=8" "SDHIP_LIB=$L/_lib_ng4/libsdhip.so" > $O/ab_sched.txt 2>&1
