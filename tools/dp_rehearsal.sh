#!/bin/bash
# 2-rank data-parallel rehearsal of bench.py on ONE GPU (gloo stands in for RCCL, both ranks on cuda:0): the sharded
# BASELINE workloads configs[2] (walker decoder, B64 global -> --global-batch) and configs[4] (memory maze).
# Usage (GPU box, repo root): bash tools/dp_rehearsal.sh <tag>  -> gpurun_out/<tag>_dp_*.json
set -e
T=$1
for c in walker_dreamer memory_maze; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 3 --backend gloo --config dmc/$c --global-batch \
    --no-roofline > gpurun_out/${T}_dp_$c.log 2>&1
  grep '^{' gpurun_out/${T}_dp_$c.log > gpurun_out/${T}_dp_$c.json
  cut -c1-400 gpurun_out/${T}_dp_$c.json
done
