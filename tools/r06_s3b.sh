#!/bin/bash
# Encoder stages 2 + 3 on bf16x6 (SDREAMER_CONV6=1) with the pipelined ring: kernel tests, per-variant timing, the
# precision study's dumps (tools/dump_opt.py; compared here with tools/precision_study.py), the golden update tests
# under CONV6=1 with their bound ratios, then a same-box A/B. Usage: bash tools/r06_s3b.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "bf16x6" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 200 python3 tools/conv6_time.py > $O/conv6_time.txt 2>&1 &&
SDREAMER_CONV6=1 timeout -k 10 300 python3 tools/dump_opt.py $O/c6all > $O/dump_c6all.txt 2>&1 || exit $?
SDREAMER_CONV6=1 SDREAMER_GOLDEN_REPORT=$O/rep_c6all timeout -k 10 600 python -u -m pytest tests/test_gpu_dreamer.py \
  -k "test_update_matches_reference" -q $T > $O/tests_c6all.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 bash tools/ab_env.sh 2 "" "SDREAMER_CONV6=1" "SDREAMER_CONV6=1 SDHIP_CONV6_PIPE=0" > $O/ab.txt 2>&1
