#!/bin/bash
# Round-4 imagination A/B on the GPU box: correctness (imagination + golden updates), the per-phase trace, and
# same-box bench alternation of the default build against the variants that revert one change each.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_imagine.py tests/test_gpu_scan.py tests/test_gpu_gemm.py \
  "tests/test_gpu_dreamer.py::test_update_matches_reference" tests/test_gpu_act.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace_cp0/libsdhip.so timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace_cp0.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
bash tools/ab_env.sh 2 "" "SDHIP_LIB=$L/_lib_ka0/libsdhip.so" "SDHIP_LIB=$L/_lib_kr0/libsdhip.so" \
  "SDHIP_LIB=$L/_lib_kp0/libsdhip.so" "SDHIP_LIB=$L/_lib_cp0/libsdhip.so" "SDHIP_LIB=$L/_lib_ap0/libsdhip.so" > $O/ab.txt 2>&1 || exit 1
timeout -k 10 200 python tools/timeline.py 6 > $O/timeline.txt 2>&1 || exit 1
timeout -k 10 300 python tools/phase_bench.py 10 > $O/phases.txt 2>&1 || exit 1
