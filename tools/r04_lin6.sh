#!/bin/bash
# k_lin6 (pre-split deter contractions): imagination tests, golden updates, trace, A/B vs the fp32 k_lin. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_imagine.py > $O/imagine.txt 2>&1 || exit 1
timeout -k 10 400 $T tests/test_gpu_dreamer.py -k "test_update_matches_reference" > $O/golden.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_KL_NOPRE=1" > $O/ab.txt 2>&1
