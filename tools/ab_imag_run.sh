#!/bin/bash
# GPU box: imagination-only timing + kernel-trace summary per library variant (default build and _var/<name>).
# Usage: bash tools/ab_imag_run.sh <tag> [variant...]  -> gpurun_out/<tag>_<variant>.md
R=$PWD
T=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  lib=$R/safe-dreamer_amd/sdreamer/_lib/libsdhip.so
  [ "$v" != default ] && lib=$R/_var/$v/libsdhip.so
  SDHIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/ab_${T}_$v -o run -- python3 $R/tools/imag_bench.py 10 > $R/gpurun_out/${T}_$v.log 2>&1 || exit 1
  (cd $R && python3 tools/prof_summary.py $(find /tmp/ab_${T}_$v -name "*.db" | head -1) 11 > gpurun_out/${T}_$v.md)
  echo "== $v: $(tail -1 $R/gpurun_out/${T}_$v.log)"
  head -14 $R/gpurun_out/${T}_$v.md | tail -10 | cut -c1-130
done
