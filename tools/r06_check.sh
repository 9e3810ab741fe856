#!/bin/bash
# round-6 change check: the whole GPU suite, then a same-box A/B against the round-5 tree (_ab/old)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 900 bash tools/ab_trees.sh _ab/old . ${2:-3} > $O/ab.txt 2>&1
