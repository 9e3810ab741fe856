# Round profile bundle (run on the GPU box from the repo root): the profiled bench line + kernel-trace summary, and
# the PMC passes (each its own rocprofv3 run, no trace domains): SQ cycle breakdown + MFMA busy + GRBM_GUI_ACTIVE,
# FETCH_SIZE, WRITE_SIZE, L2 hit/miss -> per-kernel table (tools/pmc_table.py) and the roofline kernels' HBM bytes
# per launch (tools/roofline_traffic.py, read by bench.py). Usage: bash tools/profile_round.sh <tag> [bench args, e.g.
# --config dmc/memory_maze --batch 2] -> gpurun_out/<tag>_*
set -e
R=$PWD
T=$1
shift
X="$*"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline $X"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$T -o run -- python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline $X > $R/gpurun_out/${T}_profiled_bench.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/p1_$T -o run -- $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/p2_$T -o run -- $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/p3_$T -o run -- $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d /tmp/p4_$T -o run -- $B > /dev/null 2>&1
cd $R
db() { find $1 -name "*.db" | head -1; }
python3 tools/prof_summary.py $(db /tmp/kt_$T) 15 > gpurun_out/${T}_kernel_summary.md
python3 tools/roofline_traffic.py $(db /tmp/p2_$T) $(db /tmp/p3_$T) gpurun_out/${T}_roofline_traffic.json > /dev/null
python3 tools/pmc_table.py /tmp/kt_$T /tmp/p1_$T /tmp/p2_$T /tmp/p3_$T /tmp/p4_$T > gpurun_out/${T}_pmc.md
KT_BENCH_LOG=gpurun_out/${T}_profiled_bench.log python3 tools/kernel_table.py /tmp/kt_$T 10 gpurun_out/${T}_kernel_table.json /tmp/p1_$T /tmp/p2_$T /tmp/p3_$T /tmp/p4_$T > gpurun_out/${T}_kernel_table.md
head -8 gpurun_out/${T}_kernel_summary.md
