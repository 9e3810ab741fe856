#!/bin/bash
# r05 split-bf16 long-K workgroup target (SDREAMER_G3_WGS: 512 default) re-measured with the 192-tile threshold
set -o pipefail
O=gpurun_out/r05wg; mkdir -p $O
bash tools/ab_env.sh 3 "" "SDREAMER_G3_WGS=256" "SDREAMER_G3_WGS=384" > $O/ab.txt 2>&1
