#!/bin/bash
# Round-5 closing run: profile bundle (the kernel table the bench reads, copied into profiles/ on the box) and the
# final check on the same box
set -o pipefail
bash tools/profile_round.sh r05zy && cp gpurun_out/r05zy_kernel_table.json profiles/r05zy_kernel_table.json &&
bash tools/r05_final.sh r05final3
