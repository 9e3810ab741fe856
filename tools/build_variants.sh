#!/bin/bash
# Build the in-tree library and its A/B variants (each reverts one knob) + the phase-trace build, here in the build
# container (hipcc cross-compiles gfx950); they travel to the GPU box with the tree. Usage: bash tools/build_variants.sh
set -e
cd "$(dirname "$0")/../safe-dreamer_amd/csrc"
make -j8 >/dev/null
make -j8 OUT=../sdreamer/_lib_trace BUILD=build_trace EXTRA=-DSD_SCAN_TRACE >/dev/null
for v in "ka0:-DKA_ROWS=0" "kr0:-DKR_RW=0" "kp0:-DKP_RW=0" "ap0:-DKH_APRE=0" "cp0:-DSD_CORE_PAIR=0" \
         "trace_cp0:-DSD_SCAN_TRACE -DSD_CORE_PAIR=0" "ng4:-DSD_LR_NG=4" "m0:-DSD_G3_M256=0"; do
  n=${v%%:*}; f=${v#*:}
  make -j8 OUT=../sdreamer/_lib_$n BUILD=build_$n EXTRA="$f" >/dev/null
done
echo "variants built"
