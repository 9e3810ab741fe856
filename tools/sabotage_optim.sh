#!/bin/bash
# Mutation check of the optimizer parity tests. Builds three deliberately broken copies of
# libsdhip.so from safe-dreamer_amd/csrc/optim.hip (sign of the LaProp step flipped, AGC clip skipped, Polyak skipped)
# into _sab/<variant>/libsdhip.so; `run` then points SDHIP_LIB at each and runs the optimizer tests, which must FAIL.
#   tools/sabotage_optim.sh build        (CPU container: hipcc)
#   tools/sabotage_optim.sh run          (GPU box; writes gpurun_out/sabotage.txt)
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/safe-dreamer_amd/csrc
SAB=$ROOT/_sab
declare -A EDIT=(
  [laprop_sign]='s/pq\[j\] = pq\[j\] + neg_step \* mv;/pq[j] = pq[j] - neg_step * mv;/'
  [agc_skip]='s/const float gv = gq\[j\] \* sc;/const float gv = gq[j];/'
  [polyak_skip]='s/dst\[i\] = mix \* src\[i\] + keep \* dst\[i\];/dst[i] = dst[i] + 0.f * src[i] * mix * keep;/'
)
if [ "${1:-}" = build ]; then
  make -C "$CSRC" -j8 >/dev/null || exit 1
  for v in "${!EDIT[@]}"; do
    mkdir -p "$SAB/$v"
    sed "${EDIT[$v]}" "$CSRC/optim.hip" > "$SAB/$v/optim.hip"
    if cmp -s "$CSRC/optim.hip" "$SAB/$v/optim.hip"; then echo "edit $v did not apply"; exit 1; fi
    objs=$(ls "$CSRC"/build/*.o | grep -v '/optim.o$')
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$CSRC" -c "$SAB/$v/optim.hip" \
      -o "$SAB/$v/optim.o" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$SAB/$v/libsdhip.so" $objs "$SAB/$v/optim.o" \
      || exit 1
    echo "built $SAB/$v/libsdhip.so"
  done
elif [ "${1:-}" = run ]; then
  mkdir -p "$ROOT/gpurun_out"
  out=$ROOT/gpurun_out/sabotage.txt
  : > "$out"
  cd "$ROOT"
  for v in laprop_sign agc_skip polyak_skip; do
    SDHIP_LIB=$SAB/$v/libsdhip.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
      tests/test_gpu_ops.py::test_laprop_agc_step tests/test_gpu_ops.py::test_polyak \
      "tests/test_gpu_dreamer.py::test_update_matches_reference[walker_r2_nowarm]" \
      "tests/test_gpu_dreamer.py::test_update_matches_reference[walker_r2]" > "$ROOT/gpurun_out/sabotage_$v.log" 2>&1
    rc=$?
    if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then echo "$v: abnormal exit $rc" >> "$out"; exit 1; fi
    summary=$(tail -1 "$ROOT/gpurun_out/sabotage_$v.log")
    if [ $rc -eq 0 ]; then echo "$v: NOT CAUGHT ($summary)" >> "$out"; else echo "$v: caught ($summary)" >> "$out"; fi
  done
  cat "$out"
else
  echo "usage: $0 build|run"; exit 2
fi
