#!/bin/bash
# S0 (weight-only imagination prep) forked beside the scan forward (SDREAMER_SIDE_PREP_AT=scan): graph == eager test,
# the marked timeline, then a same-box A/B. Usage: bash tools/r06_s0.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dreamer.py -k "side_prep or graph_replay" -q $T > $O/tests.txt 2>&1 &&
SDREAMER_SIDE_PREP=2 SDREAMER_SIDE_PREP_AT=scan timeout -k 10 200 python3 tools/timeline.py > $O/timeline_s0scan2.txt 2>&1 &&
timeout -k 10 900 bash tools/ab_env.sh 3 "" "SDREAMER_SIDE_PREP=1 SDREAMER_SIDE_PREP_AT=scan" "SDREAMER_SIDE_PREP=2 SDREAMER_SIDE_PREP_AT=scan" > $O/ab.txt 2>&1
