#!/bin/bash
# PMC passes over tools/gemm3_bench.py (split-bf16 GEMM shapes of the update): per-kernel averages of the SQ cycle /
# instruction mix, LDS bank conflicts and TCP latency (tools/pmc_kernel_avg.py). GPU box, repo root.
R=$PWD
cd /tmp && export TMPDIR=/tmp
B="python3 $R/tools/gemm3_bench.py"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d /tmp/ga -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d /tmp/gb -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace -d /tmp/gt -o run -- $B > /dev/null 2>&1 || exit 1
cd $R
python3 tools/pmc_kernel_avg.py "gemm3_kernel<128" /tmp/ga /tmp/gb > gpurun_out/pmc_gemm3.md
python3 tools/pmc_table.py /tmp/gt /tmp/ga /tmp/gb | grep gemm3 > gpurun_out/pmc_gemm3_table.md
head -c 2500 gpurun_out/pmc_gemm3.md
