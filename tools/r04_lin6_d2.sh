#!/bin/bash
# k_lin6 / action-noise validation (tools/r04_lin6.sh), the 512-thread prior sampler (KP_NT=512), plus the two-deep-prefetch gemm3 variants: GEMM tests on the
# default and the all-tiles variant, shape timings, whole-update A/B. -> gpurun_out/$1
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=safe-dreamer_amd/sdreamer
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_imagine.py > $O/imagine.txt 2>&1 || exit 1
timeout -k 10 400 $T tests/test_gpu_dreamer.py -k "test_update_matches_reference" > $O/golden.txt 2>&1 || exit 1
timeout -k 10 300 $T tests/test_gpu_gemm.py > $O/gemm.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_d2a/libsdhip.so timeout -k 10 300 $T tests/test_gpu_gemm.py > $O/gemm_d2a.txt 2>&1 || exit 1
timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_kp512/libsdhip.so timeout -k 10 400 $T tests/test_gpu_imagine.py > $O/imagine_kp512.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_trace_kp512/libsdhip.so timeout -k 10 200 python tools/imag_trace.py > $O/imag_trace_kp512.txt 2>&1 \
  || exit 1
timeout -k 10 120 python tools/gemm3_bench.py > $O/g3_default.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_d2/libsdhip.so timeout -k 10 120 python tools/gemm3_bench.py > $O/g3_d2.txt 2>&1 || exit 1
SDHIP_LIB=$L/_lib_d2a/libsdhip.so timeout -k 10 120 python tools/gemm3_bench.py > $O/g3_d2a.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDHIP_KL_NOPRE=1" "SDHIP_LIB=$L/_lib_d2/libsdhip.so" "SDHIP_LIB=$L/_lib_d2a/libsdhip.so" \
  "SDHIP_LIB=$L/_lib_kp512/libsdhip.so" > $O/ab.txt 2>&1
for i in 1 2; do  # C4 (atari-like, 2048 imagined rows, 32x32 stoch): the prior sampler's grid is 4x C2's
  for e in "" "SDHIP_LIB=$L/_lib_kp512/libsdhip.so"; do
    ms=$(env $e timeout -k 10 240 python3 bench.py --config dmc/atari_breakout --no-cpu-baseline --no-roofline \
      2>/dev/null | tail -1 | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'], 3))") \
      || exit 1
    echo "[c4 ${e:-default}] $ms" >> $O/ab_c4.txt
  done
done
# C2 vs C4 kernel tables of the same build on the same box (where C4's extra time goes)
R=$PWD
for c in cnn atari_breakout; do
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$c -o run -- python3 $R/bench.py \
    --config dmc/$c --steps 10 --warmup 5 --no-cpu-baseline --no-roofline > $R/$O/kt_${c}_bench.log 2>&1) || exit 1
  python3 tools/kernel_table.py /tmp/kt_$c 10 $O/kt_$c.json > $O/kt_$c.md 2>&1 || exit 1
done
