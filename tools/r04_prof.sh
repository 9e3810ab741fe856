#!/bin/bash
# Kernel lists of the critical phases replayed alone (rocprofv3 kernel trace via tools/phase_trace.sh) and the
# timeline of a replayed update. Output under gpurun_out/<tag>_*.
set -o pipefail
T=$1
for ph in P S1 M2a M1 S2; do
  bash tools/phase_trace.sh ${T}_$ph $ph || exit 1
done
