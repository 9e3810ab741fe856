# Kernel list of ONE update phase replayed alone (tools/phase_bench.py: 1 + 10 replays inside the trace window), per
# replay, from a rocprofv3 kernel trace: bash tools/phase_trace.sh <tag> <phase, e.g. S2> -> gpurun_out/<tag>_phase_kernels.md
set -e
R=$PWD
T=$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pt_$T -o run -- python3 $R/tools/phase_bench.py 10 $2 > $R/gpurun_out/${T}_phase_bench.txt 2>&1
cd $R
python3 tools/kernel_table.py /tmp/pt_$T 11 gpurun_out/${T}_phase_kernels.json > gpurun_out/${T}_phase_kernels.md
