#!/bin/bash
# r05 k_lin6_areg on 48-column tiles over the three problems (256 workgroups): imagination parity, step trace,
# update A/B against the 64-column build (_lib_old)
set -o pipefail
O=gpurun_out/r05lb; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_imagine.py > $O/tests.txt 2>&1 &&
timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_old/libsdhip.so" > $O/ab.txt 2>&1
