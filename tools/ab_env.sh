#!/bin/bash
# Same-box A/B of environment settings (schedule knobs, SDHIP_LIB variants) on bench.py: alternated R times, ms per
# update printed per run. GPU box, repo root. Stops at the first failing run.
# Usage: bash tools/ab_env.sh R "ENV_A" "ENV_B" [...]     e.g. bash tools/ab_env.sh 2 "" "SDREAMER_AC_DEFER=1"
R=$1; shift
for i in $(seq "$R"); do
  for e in "$@"; do
    ms=$(env $e timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-roofline 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'], 3))") || exit 1
    echo "[${e:-default}] $ms"
  done
done
