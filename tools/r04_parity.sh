#!/bin/bash
# Gradient-parity headroom attribution: the golden update tests and the C2 full-size test on the
# default path (split-bf16 gradient GEMMs) and with SDREAMER_FAST_GEMM=0 (every contraction exact f32). Reports:
# gpurun_out/golden/*.json (bound_ratio: the fraction of each optimizer bound used) and gpurun_out/fullsize/*.json.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
K="test_update_matches_reference and (walker_r2_nowarm or walker_r2 or walker_dreamer)"
timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_dreamer.py -k "$K" \
  > $O/golden_default.txt 2>&1 || exit 1
mkdir -p $O/golden_default && cp gpurun_out/golden/*.json $O/golden_default/
SDREAMER_FAST_GEMM=0 timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread \
  tests/test_gpu_dreamer.py -k "$K" > $O/golden_f32.txt 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -q -s --timeout 480 --timeout-method thread tests/test_gpu_fullsize.py -k C2 \
  > $O/full_default.txt 2>&1 || exit 1
cp gpurun_out/fullsize/C2_walker_r2.json $O/full_C2_default.json
SDREAMER_FAST_GEMM=0 timeout -k 10 500 python -u -m pytest -q -s --timeout 480 --timeout-method thread \
  tests/test_gpu_fullsize.py -k C2 > $O/full_f32.txt 2>&1 || exit 1
cp gpurun_out/fullsize/C2_walker_r2.json $O/full_C2_f32.json
SDREAMER_CONV6=1 timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread \
  tests/test_gpu_dreamer.py -k "$K or walker_r2aug or walker_pro" > $O/golden_conv6.txt 2>&1
mkdir -p $O/golden_conv6 && cp gpurun_out/golden/*.json $O/golden_conv6/ && rm -f gpurun_out/golden/*.json
