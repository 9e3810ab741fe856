#!/bin/bash
# VERDICT r04 item 6 on one GPU box: C5 (memory-maze-like, deter 4096, B16 L256 H25) kernel table + phase timeline, and
# the per-rank shards of the 8-GPU configurations timed on one GPU (C5 at B2, C3 walker/decoder at B8), next to the
# full single-GPU runs. Usage: bash tools/r05_shards.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
R=$PWD
O=$R/gpurun_out/$1; mkdir -p $O
B="python3 -u bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline"
timeout -k 10 300 $B --config dmc/memory_maze > $O/c5_b16.json 2> $O/c5_b16.err || exit 1
timeout -k 10 300 $B --config dmc/memory_maze --batch 2 > $O/c5_b2.json 2> $O/c5_b2.err || exit 1
timeout -k 10 300 $B --config dmc/walker_dreamer --batch 8 > $O/c3_b8.json 2> $O/c3_b8.err || exit 1
timeout -k 10 300 $B --config dmc/walker_dreamer > $O/c3_b64.json 2> $O/c3_b64.err || exit 1
timeout -k 10 300 $B --config dmc/atari_breakout > $O/c4_b32.json 2> $O/c4_b32.err || exit 1
timeout -k 10 200 python3 -u tools/timeline.py 4 dmc/memory_maze > $O/c5_timeline.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/timeline.py 4 dmc/memory_maze 2 > $O/c5_b2_timeline.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/timeline.py 4 dmc/walker_dreamer 8 > $O/c3_b8_timeline.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_c5 -o run -- python3 $R/bench.py --config dmc/memory_maze \
  --steps 3 --warmup 3 --no-cpu-baseline --no-roofline > $O/c5_profiled_bench.log 2>&1 || exit 1
cd $R
python3 tools/kernel_table.py /tmp/kt_c5 3 $O/c5_kernel_table.json > $O/c5_kernel_table.md || exit 1
db=$(find /tmp/kt_c5 -name "*.db" | head -1)
python3 tools/prof_summary.py $db 25 > $O/c5_kernel_summary.md || exit 1
