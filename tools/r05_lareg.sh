#!/bin/bash
# r05 k_lin6_areg: imagination parity, step trace (new / SDHIP_KL_NOAREG), update A/B
set -o pipefail
O=gpurun_out/r05la; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_imagine.py > $O/tests.txt 2>&1 &&
timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace.txt 2>&1 &&
SDHIP_KL_NOAREG=1 timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace_noareg.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_KL_NOAREG=1" > $O/ab.txt 2>&1
