#!/bin/bash
# r05 schedule knobs re-measured on the final tree: SDREAMER_AC_DEFER=1 (the actor / value weight gradients from S2
# into S3) and SDREAMER_S2_AFTER_SCAN=1
set -o pipefail
O=gpurun_out/r05ac; mkdir -p $O
bash tools/ab_env.sh 3 "" "SDREAMER_AC_DEFER=1" "SDREAMER_S2_AFTER_SCAN=1" > $O/ab.txt 2>&1
