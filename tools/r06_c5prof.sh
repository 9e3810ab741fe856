#!/bin/bash
# C5 kernel tables + PMC at B16 and at the 8-GPU shard B2 on the final tree (tools/profile_round.sh), with a heartbeat
# file so the silent profiler passes are not taken for a hang. Usage: bash tools/r06_c5prof.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
( while true; do date >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 900 bash tools/profile_round.sh ${1}_c5b16 --config dmc/memory_maze > $O/prof_b16.log 2>&1 &&
timeout -k 10 900 bash tools/profile_round.sh ${1}_c5b2 --config dmc/memory_maze --batch 2 > $O/prof_b2.log 2>&1
rc=$?
kill $HB
exit $rc
