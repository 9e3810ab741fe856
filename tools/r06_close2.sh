#!/bin/bash
# Round-6 closing run, part 2: the default bench line again (roofline probes matched to the final table), the
# two-stream timeline, phases alone, contention probe, the C5 bench lines and C5 kernel tables + PMC (heartbeat file so
# the silent profiler passes are not taken for a hang). Usage: bash tools/r06_close2.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
( while true; do date >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python3 tools/timeline.py > $O/timeline.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py > $O/phases_alone.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py 10 contention > $O/contention.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config dmc/memory_maze --no-cpu-baseline --no-roofline > $O/c5_b16_bench.json 2> $O/c5_b16.err &&
timeout -k 10 300 python3 bench.py --config dmc/memory_maze --batch 2 --no-cpu-baseline --no-roofline > $O/c5_b2_bench.json 2> $O/c5_b2.err &&
timeout -k 10 900 bash tools/profile_round.sh ${1}_c5b2 --config dmc/memory_maze --batch 2 > $O/prof_b2.log 2>&1
rc=$?
kill $HB
exit $rc
