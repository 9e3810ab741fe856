#!/bin/bash
# Round-end bundle in one GPU call: the profile set of the final build (tools/profile_round.sh -> the kernel table
# bench.py reads), a C4 A/B of the split-bf16 K-split workgroup target, then tools/r04_final.sh (whole GPU suite,
# smoke, the bench lines). Usage: bash tools/r04_round_end.sh <tag> -> gpurun_out/<tag>_* and gpurun_out/<tag>/
set -o pipefail
T=$1
mkdir -p gpurun_out/$T
bash tools/profile_round.sh $T > gpurun_out/$T/profile_round.txt 2>&1 || exit 1
cp gpurun_out/${T}_kernel_table.json profiles/r04y_kernel_table.json || exit 1
for i in 1 2; do
  for e in "" "SDREAMER_G3_WGS=1024"; do
    ms=$(env $e timeout -k 10 240 python3 bench.py --config dmc/atari_breakout --no-cpu-baseline --no-roofline \
      2>/dev/null | tail -1 | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'], 3))") \
      || exit 1
    echo "[c4 ${e:-default}] $ms" >> gpurun_out/$T/ab_c4_wgs.txt
  done
done
bash tools/r04_final.sh $T
