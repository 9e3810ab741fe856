#!/bin/bash
# The step's two one-hot gathers as two grid rows (OH_SPLIT=1): imagination tests, step trace, A/B. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
SDHIP_LIB=$L/_lib_oh/libsdhip.so timeout -k 10 400 $T tests/test_gpu_imagine.py > $O/imagine_oh.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_oh/libsdhip.so timeout -k 10 400 $T tests/test_gpu_dreamer.py -k "test_update_matches_reference" \
  > $O/golden_oh.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace_oh/libsdhip.so timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace_oh.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_LIB=$L/_lib_oh/libsdhip.so" > $O/ab.txt 2>&1
