# Round profile bundle (run on the GPU box from the repo root): kernel-trace summary of the bench, the bench line,
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs, no trace domains) for the roofline probe kernel.
# Usage: bash tools/profile_round.sh <tag>   -> gpurun_out/<tag>_*
set -e
R=$PWD
T=$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$T -o run -- python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline > $R/gpurun_out/${T}_profiled_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf_$T -o run -- python3 $R/bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw_$T -o run -- python3 $R/bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline > /dev/null 2>&1
cd $R
python tools/prof_summary.py $(find /tmp/kt_$T -name "*.db" | head -1) 15 > gpurun_out/${T}_kernel_summary.md
python tools/roofline_traffic.py $(find /tmp/pf_$T -name "*.db" | head -1) $(find /tmp/pw_$T -name "*.db" | head -1) gpurun_out/${T}_roofline_traffic.json > /dev/null
