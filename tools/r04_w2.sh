#!/bin/bash
# k_action_rows staging _dyn_in2 weight after the logits (KA_W2LATE=1): imagination tests (default
# and variant), golden update (variant), step traces, A/B. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_imagine.py > $O/imagine.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_w2/libsdhip.so timeout -k 10 400 $T tests/test_gpu_imagine.py > $O/imagine_w2.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_w2/libsdhip.so timeout -k 10 400 $T tests/test_gpu_dreamer.py -k "test_update_matches_reference" \
  > $O/golden_w2.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace_w2/libsdhip.so timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace_w2.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_LIB=$L/_lib_w2/libsdhip.so" > $O/ab.txt 2>&1
