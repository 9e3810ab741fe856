# Per-kernel counter evidence for the update's hot kernels (run on the GPU box from the repo root):
#   one kernel-trace pass (times) + four PMC passes, each its own rocprofv3 run (no trace domains with --pmc):
#   (1) SQ cycle breakdown + MFMA busy + GRBM_GUI_ACTIVE (effective clock), (2) FETCH_SIZE, (3) WRITE_SIZE,
#   (4) L2 hit / miss. Usage: bash tools/pmc_round.sh <tag> [bench args...]  -> gpurun_out/<tag>_pmc.md
set -e
R=$PWD
T=$1
shift
ARGS=${@:---steps 3 --warmup 3}
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py $ARGS --no-cpu-baseline --no-roofline"
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/${T}_db/pk -o run -- $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/${T}_db/p1 -o run -- $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/${T}_db/p2 -o run -- $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/${T}_db/p3 -o run -- $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d /tmp/${T}_db/p4 -o run -- $B > /dev/null 2>&1
cd $R
python3 tools/pmc_table.py /tmp/${T}_db/pk /tmp/${T}_db/p1 /tmp/${T}_db/p2 /tmp/${T}_db/p3 /tmp/${T}_db/p4 > gpurun_out/${T}_pmc.md
cat gpurun_out/${T}_pmc.md
