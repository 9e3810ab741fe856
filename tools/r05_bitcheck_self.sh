#!/bin/bash
# lib_bitcheck on the current build twice (run-to-run determinism of the whole update, and the tool itself)
set -o pipefail
O=gpurun_out/r05bc; mkdir -p $O
timeout -k 10 300 python3 tools/lib_bitcheck.py /tmp/a.npz > $O/run_a.txt 2>&1 &&
timeout -k 10 300 python3 tools/lib_bitcheck.py /tmp/b.npz > $O/run_b.txt 2>&1 &&
python3 tools/lib_bitcheck.py cmp /tmp/a.npz /tmp/b.npz > $O/bitcheck.txt 2>&1
