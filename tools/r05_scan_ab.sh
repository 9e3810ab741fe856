#!/bin/bash
# Round-5 observe-scan A/B on one GPU box: parity of the default build (scan tests, golden updates, graph == eager at
# full size), per-launch traces of the default build and of the variants that revert one change each
# (tools/build_r05.sh), then a same-box bench alternation. Output under gpurun_out/$1.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_scan.py "tests/test_gpu_dreamer.py::test_update_matches_reference" \
  tests/test_gpu_graph_fullsize.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_trace.py > $O/trace.txt 2>&1 || exit 1
for v in xm0 g16 h8 b8 cx0 tk; do
  SDHIP_LIB=$L/_lib_trace_$v/libsdhip.so timeout -k 10 120 python tools/scan_trace.py > $O/trace_$v.txt 2>&1 || exit 1
done
SDREAMER_SCAN_KSD=4 SDHIP_LIB=$L/_lib_trace_r4/libsdhip.so timeout -k 10 120 python tools/scan_trace.py \
  > $O/trace_r4.txt 2>&1 || exit 1
bash tools/ab_env.sh 2 "" "SDREAMER_SCAN_KSD=4 SDHIP_LIB=$L/_lib_r4/libsdhip.so" "SDHIP_LIB=$L/_lib_xm0/libsdhip.so" \
  "SDHIP_LIB=$L/_lib_g16/libsdhip.so" "SDHIP_LIB=$L/_lib_h8/libsdhip.so" "SDHIP_LIB=$L/_lib_b8/libsdhip.so" \
  "SDHIP_LIB=$L/_lib_cx0/libsdhip.so" "SDREAMER_SCAN_KSD=4" > $O/ab.txt 2>&1 || exit 1
