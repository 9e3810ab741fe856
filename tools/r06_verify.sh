#!/bin/bash
# Closing check of the tree as committed: the whole GPU suite, smoke and the default bench line (no re-profile).
# Usage: bash tools/r06_verify.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
