#!/bin/bash
# The ring kernel's multi-tile workgroups (patch prefetch): kernel tests, per-variant timing, then the whole GPU suite
# and a same-box A/B against the previous commit's tree (_ab/old). Usage: bash tools/r06_tpw.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/conv6_time.py > $O/conv6_time.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q $T > $O/gpu_tests.txt 2>&1 &&
timeout -k 10 900 bash tools/ab_trees.sh _ab/old . 3 > $O/ab.txt 2>&1
