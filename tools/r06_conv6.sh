#!/bin/bash
# Precision studies on the encoder + schedule A/B:
#  (a) the second stage forward on bf16x6 (SDREAMER_CONV6=s2), (b) the first stage bwd-weight on split-bf16
#  (SDREAMER_WGRAD1_X3=1: sd_conv2d_wgrad_pool_bf16x3) — for each, the golden cases' LaProp moments dumped
#  (tools/grad_attrib.py compares them with float64) and the golden update / gradient tests run with their bound
#  ratios reported; then a same-box A/B of the update under the schedule / build knobs.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "first_stage_pooled" -q $T > $O/tests_ops.txt 2>&1 &&
timeout -k 10 300 python3 tools/dump_opt.py $O/f32 > $O/dump_f32.txt 2>&1 &&
SDREAMER_CONV6=s2 timeout -k 10 300 python3 tools/dump_opt.py $O/c6 > $O/dump_c6.txt 2>&1 &&
SDREAMER_WGRAD1_X3=1 timeout -k 10 300 python3 tools/dump_opt.py $O/w3 > $O/dump_w3.txt 2>&1 || exit $?
SDREAMER_CONV6=s2 SDREAMER_GOLDEN_REPORT=$O/rep_c6 timeout -k 10 600 python -u -m pytest tests/test_gpu_dreamer.py \
  -k "test_update_matches_reference" -q $T > $O/tests_c6.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc  # assertion failures are data here; a timeout, abort or fault ends the call
SDREAMER_WGRAD1_X3=1 SDREAMER_GOLDEN_REPORT=$O/rep_w3 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_dreamer.py -k "test_update_matches_reference or test_cal_grad_matches_reference" -q -s $T > $O/tests_w3.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
L=$PWD/safe-dreamer_amd/sdreamer
timeout -k 10 900 bash tools/ab_env.sh 2 "" "SDREAMER_SLOW_IN_S2=0" "SDREAMER_CONV6=s2" "SDREAMER_WGRAD1_X3=1" "SDREAMER_WGRAD_T128=128" "SDREAMER_F32_SPLIT2=1" \
  "SDHIP_LIB=$L/_lib_prio3/libsdhip.so" > $O/ab.txt 2>&1
