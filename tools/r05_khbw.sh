#!/bin/bash
# k_hid operand-traffic probe: the imagination step trace with the default trace build and the KH_BWTEST builds
# (timing only). Usage: bash tools/r05_khbw.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
for v in "" _bw1 _bw2 _bw3; do
  SDHIP_LIB=$L/_lib_trace$v/libsdhip.so timeout -k 10 200 python -u tools/imag_trace.py > $O/imag_trace$v.txt 2>&1 || exit 1
done
