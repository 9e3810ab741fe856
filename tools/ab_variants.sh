#!/bin/bash
# Build A/B variants of libsdhip.so with extra -D flags into _var/<name>/libsdhip.so (CPU container), e.g.
#   tools/ab_variants.sh f32 "-DSD_IMG_F6=0" f6all "-DSD_IMG_F6=0b111111"
# then on the GPU box: SDHIP_LIB=_var/<name>/libsdhip.so python tools/imag_bench.py 10
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -C "$ROOT/safe-dreamer_amd/csrc" -j8 BUILD="$ROOT/_var/$name/build" OUT="$ROOT/_var/$name" EXTRA="$flags"
  rm -rf "$ROOT/_var/$name/build"
  echo "built _var/$name/libsdhip.so ($flags)"
done
