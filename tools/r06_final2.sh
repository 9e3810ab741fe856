#!/bin/bash
# Round-6 closing run on one box: the profile bundle of the final tree (kernel table + PMC) copied to profiles/r06final
# (the bench reads the table from there), then the whole GPU suite, smoke, the step traces and the default bench line
# (cpu_baseline included). Usage: bash tools/r06_final2.sh <check tag>   (profile tag: r06final)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 bash tools/profile_round.sh r06final > $O/prof.log 2>&1 || exit 1
mkdir -p profiles/r06final && cp gpurun_out/r06final_* profiles/r06final/ || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
