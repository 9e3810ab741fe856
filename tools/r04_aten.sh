#!/bin/bash
# ATen-removal checks: the op / update tests on the changed paths, then the graph-capture census.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_ops.py > $O/ops.txt 2>&1 || exit 1
timeout -k 10 500 $T tests/test_gpu_dreamer.py tests/test_gpu_graph_fullsize.py > $O/dreamer.txt 2>&1 || exit 1
timeout -k 10 500 $T tests/test_gpu_fullsize.py -k C2 > $O/full.txt 2>&1 || exit 1
timeout -k 10 300 python tools/aten_census.py graphs > $O/aten_graphs.txt 2>&1
