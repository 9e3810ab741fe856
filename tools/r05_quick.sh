#!/bin/bash
# Round-5 quick check: scan parity tests, golden updates, graph == eager at full size, the scan and imagination traces
# and a same-box bench alternation of the default build with the given env variants.
# Usage: bash tools/r05_quick.sh <tag> [ENV ...] -> gpurun_out/<tag>/
set -o pipefail
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
SDREAMER_GOLDEN_REPORT=$O/golden timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_scan.py tests/test_gpu_imagine.py "tests/test_gpu_dreamer.py::test_update_matches_reference" \
  tests/test_gpu_graph_fullsize.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
bash tools/ab_env.sh 2 "" "$@" > $O/ab.txt 2>&1 || exit 1
