#!/bin/bash
# r05 non-temporal stores of k_gate fp32 deter only: bit identity against HEAD (_lib_old), imagination tests,
# step trace, update A/B
set -o pipefail
O=gpurun_out/r05nt1; mkdir -p $O
timeout -k 10 200 python3 tools/lib_bitcheck.py /tmp/new.npz > $O/bit_new.txt 2>&1 &&
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_old/libsdhip.so timeout -k 10 200 python3 tools/lib_bitcheck.py /tmp/old.npz > $O/bit_old.txt 2>&1 &&
{ python3 tools/lib_bitcheck.py cmp /tmp/new.npz /tmp/old.npz > $O/bitcheck.txt 2>&1; true; } &&
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_imagine.py > $O/tests.txt 2>&1 &&
timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_old/libsdhip.so" > $O/ab.txt 2>&1
