# kernel-trace profile of the imagination driver -> gpurun_out/$1.md (run on the GPU box from the repo root)
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/pi_$1 -o run -- python3 $R/tools/imag_bench.py 10 > $R/gpurun_out/$1.log 2>&1 && \
cd $R && python tools/prof_summary.py $(find /tmp/pi_$1 -name "*.db" | head -1) > gpurun_out/$1.md
