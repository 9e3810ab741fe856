#!/bin/bash
# r05 k_lin6_areg at deter 4096 (C5, memory_maze): imagination parity, full-size graph == eager, C5 update A/B
# against the k_lin6 build (_lib_old)
set -o pipefail
O=gpurun_out/r05l4; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_imagine.py > $O/tests.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_graph_fullsize.py -k "C5 or maze" > $O/tests_c5.txt 2>&1 &&
for i in 1 2; do
  for e in "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_old/libsdhip.so"; do
    ms=$(env $e timeout -k 10 300 python3 bench.py --config dmc/memory_maze --steps 5 --warmup 3 --no-cpu-baseline --no-roofline 2>/dev/null | tail -1 | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'], 3))") || exit 1
    echo "[${e:-default}] C5 $ms" >> $O/ab_c5.txt
  done
done
