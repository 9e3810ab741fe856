#!/bin/bash
# round-6 measurement set on one box: the scan skeleton (incl. the fused-pair variant), the bench line (roofline,
# census, phases), the two-stream timeline, phases alone, the contention probe
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 120 tools/hip/persist_scan_proto > $O/proto.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python3 tools/timeline.py > $O/timeline.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py > $O/phases_alone.txt 2>&1 &&
timeout -k 10 300 python3 tools/phase_bench.py 10 contention > $O/contention.txt 2>&1
