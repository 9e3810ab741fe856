#!/bin/bash
# S0 (imagination noise / weight images and the backward's weight layouts beside the encoder forward): the dreamer,
# imagination and 2-rank tests, the timeline, and a same-box A/B against SDREAMER_SIDE_PREP=0. Usage: bash tools/r05_s0.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_dreamer.py \
  tests/test_gpu_imagine.py tests/test_gpu_dist.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/timeline.py 4 > $O/timeline.txt 2>&1 || exit 1
SDREAMER_SIDE_PREP=0 timeout -k 10 200 python3 -u tools/timeline.py 4 > $O/timeline_off.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDREAMER_SIDE_PREP=0" "SDREAMER_SIDE_PREP=2" > $O/ab.txt 2>&1 || exit 1
