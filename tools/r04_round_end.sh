#!/bin/bash
# Round-end bundle in one GPU call: the profile set of the final build (tools/profile_round.sh -> the kernel table
# bench.py reads), then tools/r04_final.sh (whole GPU suite, smoke, the bench lines) and the imagination step trace. Usage: bash tools/r04_round_end.sh <tag> -> gpurun_out/<tag>_* and gpurun_out/<tag>/
set -o pipefail
T=$1
mkdir -p gpurun_out/$T
bash tools/profile_round.sh $T > gpurun_out/$T/profile_round.txt 2>&1 || exit 1
cp gpurun_out/${T}_kernel_table.json profiles/${T}_kernel_table.json || exit 1
bash tools/r04_final.sh $T || exit 1
timeout -k 10 200 python tools/imag_trace.py > gpurun_out/$T/imag_trace.txt 2>&1 || exit 1
