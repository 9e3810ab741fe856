#!/bin/bash
# K-chunk rule of the split-bf16 K split (kernels._G3_CHUNK): GEMM tests, then A/B against SDREAMER_G3_CHUNK=0 on
# the walker (C2), atari-like (C4) and memory-maze (C5) configs. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $O/gemm.txt 2>&1 || exit 1
ab() {  # config rounds
  for i in $(seq $2); do
    for e in "" "SDREAMER_G3_CHUNK=0"; do
      ms=$(env $e timeout -k 10 300 python3 bench.py --config $1 --no-cpu-baseline --no-roofline 2>/dev/null | tail -1 | \
        python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'], 3))") || exit 1
      echo "[$1 ${e:-default}] $ms" >> $O/ab.txt
    done
  done
}
ab dmc/cnn 2 && ab dmc/atari_breakout 3 && ab dmc/memory_maze 1
