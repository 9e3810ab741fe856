# L2 persistence probe (tools/hip/l2_persist.hip): per-launch past-L2 bytes and hit rate, 2 MB per XCD and 3.5 MB
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
for MB in 2 3.5; do
  timeout -k 10 60 $R/tools/hip/l2_persist $MB > $R/gpurun_out/l2p_$MB.txt 2>&1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/l2p_fetch_$MB -o run -- $R/tools/hip/l2_persist $MB > /dev/null 2>&1
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/l2p_hit_$MB -o run -- $R/tools/hip/l2_persist $MB > /dev/null 2>&1
done
