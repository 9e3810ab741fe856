#!/bin/bash
# Round-6 profile of the current tree on one box: the kernel table + PMC bundle (tools/profile_round.sh), the
# two-stream timeline, phases alone and the contention probe. Usage: bash tools/r06_prof.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 bash tools/profile_round.sh $1 > $O/prof.log 2>&1 &&
timeout -k 10 200 python3 tools/timeline.py > $O/timeline.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py > $O/phases_alone.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py 10 contention > $O/contention.txt 2>&1
