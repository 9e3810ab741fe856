#!/bin/bash
# Round-5 baseline on one GPU box: the two-stream timeline of a replayed update, every phase graph
# replayed alone, the contention probe, the scan and imagination step traces and a short bench line, all on the same
# box and build. Usage: bash tools/r05_base.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python -u tools/timeline.py 8 > $O/timeline.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/phase_bench.py 20 > $O/phases_alone.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/phase_bench.py 10 contention > $O/contention.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
