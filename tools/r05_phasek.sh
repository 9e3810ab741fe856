#!/bin/bash
# per-phase kernel lists of one graph-replayed update on the final tree (rocprofv3 kernel trace of tools/timeline.py)
set -o pipefail
R=$PWD
O=$R/gpurun_out/r05pk; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pk -o run -- python3 $R/tools/timeline.py 4 > $O/timeline_prof.txt 2>&1 &&
cd $R && python3 tools/phase_kernels.py $(find /tmp/pk -name "*.db" | head -1) 14 > $O/phase_kernels.txt 2>&1
