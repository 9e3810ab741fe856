#!/bin/bash
# NHWC pool epilogue with per-thread consecutive channels (vector stores): conv tests, per-stage timing, golden update /
# gradient tests, A/B of the first stage's kernels. Usage: bash tools/r06_epi.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -q $T > $O/tests_ops.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/conv6_time.py > $O/conv6_time.txt 2>&1 &&
SDREAMER_GOLDEN_REPORT=$O/rep timeout -k 10 600 python -u -m pytest tests/test_gpu_dreamer.py \
  -k "test_update_matches_reference or test_cal_grad_matches_reference" -q -s $T > $O/tests_golden.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
SDHIP_CONV6_C4=0 SDREAMER_GOLDEN_REPORT=$O/rep_c4f32 timeout -k 10 600 python -u -m pytest tests/test_gpu_dreamer.py \
  -k "test_update_matches_reference or test_cal_grad_matches_reference" -q -s $T > $O/tests_golden_c4f32.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 bash tools/ab_env.sh 2 "" "SDHIP_CONV6_C4=0" > $O/ab.txt 2>&1
