#!/bin/bash
# PMC passes over tools/mlp_bench.py (the fused imagination alone), each its own rocprofv3 run with no trace
# domains, joined by tools/pmc_table.py. Usage: bash tools/r05_imag_pmc.sh <tag> [lib dir]
set -o pipefail
R=$PWD
O=$R/gpurun_out/$1; mkdir -p $O
[ -n "$2" ] && export SDHIP_LIB=$R/$2/libsdhip.so
cd /tmp && export TMPDIR=/tmp
B="python3 $R/tools/imag_bench.py 5"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/ik_$1 -o run -- $B > $O/imag_trace.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/i1_$1 -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA -d /tmp/i2_$1 -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d /tmp/i3_$1 -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d /tmp/i4_$1 -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum -d /tmp/i5_$1 -o run -- $B > /dev/null 2>&1 || exit 1
cd $R
PMC_RAW=2 python3 tools/pmc_table.py /tmp/ik_$1 /tmp/i1_$1 /tmp/i2_$1 /tmp/i3_$1 /tmp/i4_$1 /tmp/i5_$1 > $O/imag_pmc.md || exit 1
