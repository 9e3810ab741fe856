#!/bin/bash
# Round-5: scan parity tests, both step traces and a same-box bench alternation of the given env variants.
# Usage: bash tools/r05_traces_ab.sh <tag> <rounds> [ENV ...] -> gpurun_out/<tag>/
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scan.py \
  "tests/test_gpu_dreamer.py::test_update_matches_reference" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
bash tools/ab_env.sh $R "" "$@" > $O/ab.txt 2>&1 || exit 1
