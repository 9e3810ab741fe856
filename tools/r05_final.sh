#!/bin/bash
# Round-5 final check of the default build on one GPU box: the whole GPU suite, smoke, the step traces, the default
# bench line (cpu_baseline included) and a rocprofv3 --stats summary of a short bench. Usage: bash tools/r05_final.sh <tag>
set -o pipefail
R=$PWD
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_trace.py > $O/scan_trace.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$1 -o run -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1 || exit 1
cd $R
db=$(find /tmp/kt_$1 -name "*.db" | head -1)
python3 tools/prof_summary.py $db 20 > $O/kernel_summary.md || exit 1
