#!/bin/bash
# r05 k_lin6_areg with four K parts per workgroup (KL_KQ=4: 1,024 threads, 4 waves per SIMD; _lib_v1): the default
# build (KL_KQ=2) bit-identical to the previous one (_lib_old), imagination tests on the variant, traces, update A/B
set -o pipefail
O=gpurun_out/r05kq; mkdir -p $O
timeout -k 10 200 python3 tools/lib_bitcheck.py /tmp/new.npz > $O/bit_new.txt 2>&1 &&
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_old/libsdhip.so timeout -k 10 200 python3 tools/lib_bitcheck.py /tmp/old.npz > $O/bit_old.txt 2>&1 &&
{ python3 tools/lib_bitcheck.py cmp /tmp/new.npz /tmp/old.npz > $O/bitcheck.txt 2>&1; true; } &&
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_imagine.py > $O/tests_v1.txt 2>&1 &&
timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace.txt 2>&1 &&
SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_trace_v1/libsdhip.so timeout -k 10 200 python3 tools/imag_trace.py > $O/imag_trace_v1.txt 2>&1 &&
bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_v1/libsdhip.so" > $O/ab.txt 2>&1
