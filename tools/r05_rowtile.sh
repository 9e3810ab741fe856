#!/bin/bash
# Scan row tiles of 8 (forward / backward / both) against the default 16: the step trace and a same-box A/B.
# Usage: bash tools/r05_rowtile.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
SDREAMER_SCAN_ROWTILE_FWD=8 timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace_f8.txt 2>&1 || exit 1
SDREAMER_SCAN_ROWTILE_BWD=8 timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace_b8.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDREAMER_SCAN_ROWTILE_FWD=8" "SDREAMER_SCAN_ROWTILE_BWD=8" "SDREAMER_SCAN_ROWTILE=8" > $O/ab.txt 2>&1 || exit 1
