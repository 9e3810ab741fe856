#!/bin/bash
# Same-box A/B of two source trees (e.g. a git worktree of an older commit under _ab/old, its libsdhip.so built there):
# bench.py from each tree, alternated R times, ms per update printed per run. GPU box, repo root.
# Usage: bash tools/ab_trees.sh <tree A> <tree B> [R] [bench args...]
A=$1; B=$2; R=${3:-3}; shift 3
for i in $(seq "$R"); do
  for t in "$A" "$B"; do
    (cd "$t" && timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-roofline "$@" 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', round(d['ms_per_step'], 3))") || exit 1
  done
done
