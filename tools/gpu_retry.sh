#!/bin/bash
# gpurun with waits while no GPU slot is free (exit status 3: nothing ran, nothing charged); any other status ends it.
# Usage: bash tools/gpu_retry.sh <timeout s> '<command>'   (output: the last attempt's gpurun output)
T=$1; shift
for i in $(seq 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpu_retry] no slot (attempt $i), waiting 120 s"
  sleep 120
done
exit 3
