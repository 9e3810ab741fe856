#!/bin/bash
# PMC passes over tools/conv_bench.py (encoder convolutions at 1024 images, layers 2..4): per-kernel averages of the SQ
# cycle / instruction mix, LDS bank conflicts, MFMA busy (tools/pmc_kernel_avg.py) for the kernels matching $1.
# GPU box, repo root. Usage: bash tools/pmc_conv_passes.sh conv_dgrad3 -> gpurun_out/pmc_conv.md
R=$PWD
F=${1:-conv_}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d /tmp/ca -o run -- python3 $R/tools/conv_bench.py 1 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d /tmp/cb -o run -- python3 $R/tools/conv_bench.py 1 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d /tmp/cc -o run -- python3 $R/tools/conv_bench.py 1 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d /tmp/ct -o run -- python3 $R/tools/conv_bench.py 1 > $R/gpurun_out/conv_bench.txt 2>&1 || exit 1
cd $R
python3 tools/pmc_kernel_avg.py "$F" /tmp/ca /tmp/cb /tmp/cc > gpurun_out/pmc_conv.md
python3 tools/pmc_table.py /tmp/ct /tmp/ca /tmp/cb /tmp/cc | grep conv_ > gpurun_out/pmc_conv_table.md
head -c 3000 gpurun_out/pmc_conv.md
