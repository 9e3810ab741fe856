#!/bin/bash
# k_carry with the x2 writer as its own workgroup (two workgroups per CU): scan tests, the scan traces at the bench
# config and at C5's B2 shard, then the C5 B2 bench line. Usage: bash tools/r06_carry.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="--timeout 300 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -q $T > $O/tests_scan.txt 2>&1 &&
timeout -k 10 120 python3 tools/scan_trace.py > $O/scan_trace.txt 2>&1 &&
timeout -k 10 200 python3 tools/scan_trace.py dmc/memory_maze 2 256 > $O/c5_b2_scan_trace.txt 2>&1 &&
timeout -k 10 200 python3 tools/scan_trace.py dmc/memory_maze 16 256 > $O/c5_b16_scan_trace.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config dmc/memory_maze --batch 2 --no-cpu-baseline --no-roofline > $O/c5_b2_bench.json 2> $O/c5_b2_bench.err
