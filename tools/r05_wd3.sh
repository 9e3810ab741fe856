#!/bin/bash
# conv_wgrad3_direct with a pre-split input patch (build _lib_wd3): bit-identity against the default build, the conv
# tests and golden updates on it, and a same-box bench alternation. Usage: bash tools/r05_wd3.sh <tag> [ENV ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
L=safe-dreamer_amd/sdreamer
timeout -k 10 120 python tools/lib_bitcheck.py $O/a.npz > $O/bit.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_wd3/libsdhip.so timeout -k 10 120 python tools/lib_bitcheck.py $O/b.npz >> $O/bit.txt 2>&1 || exit 1
python tools/lib_bitcheck.py cmp $O/a.npz $O/b.npz >> $O/bit.txt 2>&1
rm -f $O/a.npz $O/b.npz
SDHIP_LIB=$L/_lib_wd3/libsdhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_ops.py -k conv "tests/test_gpu_dreamer.py::test_update_matches_reference" > $O/tests_wd3.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_LIB=$L/_lib_wd3/libsdhip.so" "$@" > $O/ab.txt 2>&1 || exit 1
