#!/bin/bash
# Round-5 quick check: scan parity tests, golden updates, graph == eager at full size, the scan trace and three
# bench runs of the default build. Usage: bash tools/r05_quick.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
SDREAMER_GOLDEN_REPORT=gpurun_out/$1/golden timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scan.py \
  "tests/test_gpu_dreamer.py::test_update_matches_reference" tests/test_gpu_graph_fullsize.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" > $O/ab.txt 2>&1 || exit 1
