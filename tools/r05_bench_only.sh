#!/bin/bash
# the default bench line (cpu_baseline included) and the step traces on the current tree
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 &&
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1
