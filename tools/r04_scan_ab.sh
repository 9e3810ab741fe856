#!/bin/bash
# Round-4 A/B on the GPU box: correctness of the default build and its variants, per-phase traces of the scan and the
# imagination, and same-box bench alternation. Output under gpurun_out/$1.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scan.py \
  tests/test_gpu_imagine.py "tests/test_gpu_dreamer.py::test_update_matches_reference" > $O/tests.txt 2>&1 || exit 1
for kx in 4 2; do
  SDHIP_LIB=$L/_lib_kx$kx/libsdhip.so timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread \
    tests/test_gpu_scan.py > $O/tests_kx$kx.txt 2>&1 || exit 1
done
timeout -k 10 120 python tools/scan_trace.py > $O/trace16.txt 2>&1 || exit 1
SDREAMER_SCAN_ROWTILE_FWD=8 timeout -k 10 120 python tools/scan_trace.py > $O/trace_f8.txt 2>&1 || exit 1
for kx in 4 2; do
  SDHIP_LIB=$L/_lib_trace_kx$kx/libsdhip.so timeout -k 10 120 python tools/scan_trace.py > $O/trace_kx$kx.txt 2>&1 || exit 1
done
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
bash tools/ab_env.sh 2 "" "SDREAMER_SCAN_ROWTILE_FWD=8" "SDHIP_LIB=$L/_lib_kx4/libsdhip.so" \
  "SDHIP_LIB=$L/_lib_kx2/libsdhip.so" "SDHIP_LIB=$L/_lib_ka0/libsdhip.so" > $O/ab.txt 2>&1 || exit 1
