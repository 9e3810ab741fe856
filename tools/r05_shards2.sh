#!/bin/bash
# Second half of tools/r05_shards.sh (timelines + C5 kernel table) after the timeline buffer fix.
set -o pipefail
R=$PWD
O=$R/gpurun_out/$1; mkdir -p $O
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
