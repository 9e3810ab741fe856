#!/bin/bash
# two-stream timeline, phases alone and the contention probe on the final round-5 tree
set -o pipefail
O=gpurun_out/r05tl; mkdir -p $O
timeout -k 10 200 python3 tools/timeline.py > $O/timeline.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py > $O/phases_alone.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py 10 contention > $O/contention.txt 2>&1
