#!/bin/bash
# r05 layout copy: the 64x64 float4 tile transpose — parity, kernel time, A/B against the 32x32 version
set -o pipefail
mkdir -p gpurun_out/r05lc
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k layout tests/test_gpu_scan.py > gpurun_out/r05lc/tests.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05lc/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/r05lc/prof.log 2>&1 &&
cd $GRAFT_REPO_ROOT && bash tools/ab_env.sh 3 "" "SDHIP_LIB=safe-dreamer_amd/sdreamer/_lib_old/libsdhip.so" > gpurun_out/r05lc/ab.txt 2>&1
