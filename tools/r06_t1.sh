#!/bin/bash
# The whole GPU suite on the current tree (golden reports kept), then a same-box A/B of the default against the
# previous encoder default (SDREAMER_CONV6=s2). Usage: bash tools/r06_t1.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
SDREAMER_GOLDEN_REPORT=$O/rep timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/gpu_tests.txt 2>&1 &&
timeout -k 10 600 bash tools/ab_env.sh 2 "" "SDREAMER_CONV6=s2" > $O/ab.txt 2>&1
