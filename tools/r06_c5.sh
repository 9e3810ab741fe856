#!/bin/bash
# VERDICT r05 item 3 (C5 on the final tree, with counters, the scan at deter 4096) + item 2 (the scan skeleton with the
# block-local pair fused): kernel table + PMC of the memory-maze-like config at B16 and at its 8-GPU per-rank shard B2,
# the scan's launch traces at D = 4096 for both, and the skeleton (tools/hip/persist_scan_proto, D = 2048 geometry)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 60 tools/hip/scan_floor_proto > $O/scan_floor.txt 2>&1 &&
timeout -k 10 200 python3 tools/scan_trace.py dmc/memory_maze 16 256 > $O/c5_b16_scan_trace.txt 2>&1 &&
timeout -k 10 200 python3 tools/scan_trace.py dmc/memory_maze 2 256 > $O/c5_b2_scan_trace.txt 2>&1 &&
timeout -k 10 900 bash tools/profile_round.sh ${1}_c5b16 --config dmc/memory_maze > $O/prof_b16.log 2>&1 &&
timeout -k 10 900 bash tools/profile_round.sh ${1}_c5b2 --config dmc/memory_maze --batch 2 > $O/prof_b2.log 2>&1
