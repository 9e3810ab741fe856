#!/bin/bash
# Round-end validation on the GPU box: the whole GPU suite, smoke, the default bench line (with CPU baseline and
# parity legs) and the C4 (B32) line. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --config dmc/atari_breakout --steps 10 --warmup 5 --no-cpu-baseline --no-roofline \
  > $O/bench_c4.json 2> $O/bench_c4.err
