#!/bin/bash
# Round-5 scan A/B builds (here, in the build container): the default library, its trace build, and variants that
# each revert one of the round's observe-scan changes. A variant recompiles only scan.hip with its flags and links it
# with the default build's other objects. Usage: bash tools/build_r05.sh [variant names...]
set -e
cd "$(dirname "$0")/../safe-dreamer_amd/csrc"
make -j8 >/dev/null
make -j8 OUT=../sdreamer/_lib_trace BUILD=build_trace EXTRA=-DSD_SCAN_TRACE >/dev/null
declare -A V=(
  [xm0]="-DSD_SCAN_XCD=0"
  [g16]="-DSD_SCAN_GCW=16"
  [h8]="-DSD_SCAN_HCW=8"
  [b8]="-DSD_SCAN_DGCW=8 -DSD_SCAN_DHCW=8"
  [cx0]="-DSD_SCAN_CX2=0 -DSD_SCAN_DLCW=16"
  [tk]="-DSD_SCAN_TICKET=1 -DSD_SCAN_HCW=8"
  [r4]="-DSD_SCAN_XCD=0 -DSD_SCAN_GCW=16 -DSD_SCAN_DLCW=16 -DSD_SCAN_CX2=0"
)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -Wall -Wno-unused-function"
one() {  # one <out dir> <build dir> <base objects dir> <flags>
  mkdir -p "$2" "$1"
  /opt/rocm/bin/hipcc $F $4 -c scan.hip -o "$2/scan.o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$1/libsdhip.so" $(ls $3/*.o | grep -v '/scan.o$') "$2/scan.o"
}
for n in "$@"; do
  one ../sdreamer/_lib_$n build_$n build "${V[$n]}" &
  one ../sdreamer/_lib_trace_$n build_trace_$n build_trace "-DSD_SCAN_TRACE ${V[$n]}" &
done
wait
echo built
