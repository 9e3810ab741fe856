R=$PWD
cd /tmp && export TMPDIR=/tmp
B="python3 $R/tools/imag_bench.py 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d /tmp/pa -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d /tmp/pb -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -d /tmp/pc -o run -- $B > /dev/null 2>&1 || exit 1
cd $R
for k in k_hid k_gate "k_lin<"; do python3 tools/pmc_kernel_avg.py "$k" /tmp/pa /tmp/pb /tmp/pc; done > gpurun_out/pmc_img.md
head -c 3000 gpurun_out/pmc_img.md
