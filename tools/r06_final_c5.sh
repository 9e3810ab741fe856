#!/bin/bash
# Round-6 closing run, part 2: C5 (memory-maze-like, deter 4096) kernel tables + PMC at B16 and at the 8-GPU shard B2,
# their bench lines, and the bench workload's two-stream timeline, phases alone and contention probe.
# Usage: bash tools/r06_final_c5.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python3 tools/timeline.py > $O/timeline.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py > $O/phases_alone.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py 10 contention > $O/contention.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config dmc/memory_maze --no-cpu-baseline --no-roofline > $O/c5_b16_bench.json 2> $O/c5_b16.err &&
timeout -k 10 300 python3 bench.py --config dmc/memory_maze --batch 2 --no-cpu-baseline --no-roofline > $O/c5_b2_bench.json 2> $O/c5_b2.err &&
timeout -k 10 900 bash tools/profile_round.sh ${1}_c5b16 --config dmc/memory_maze > $O/prof_b16.log 2>&1 &&
timeout -k 10 900 bash tools/profile_round.sh ${1}_c5b2 --config dmc/memory_maze --batch 2 > $O/prof_b2.log 2>&1
