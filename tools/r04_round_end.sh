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
bash tools/r04_final.sh $T || exit 1
# k_lin6 on 32-row tiles (KL6_BM=32: 768 workgroups, 3 per CU, instead of 384 on 256 CUs): tests, trace, A/B
L=safe-dreamer_amd/sdreamer
O=gpurun_out/$T
SDHIP_LIB=$L/_lib_kl32/libsdhip.so timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
  tests/test_gpu_imagine.py > $O/imagine_kl32.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace_kl32/libsdhip.so timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace_kl32.txt 2>&1 \
  || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_LIB=$L/_lib_kl32/libsdhip.so" > $O/ab_kl32.txt 2>&1
