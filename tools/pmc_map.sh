#!/bin/bash
# PMC passes over the map microbench (separate passes: counter slots per pass).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_map
mkdir -p $O
cd /tmp
K="--kernel-include-regex map_kernel"
timeout -k 10 120 rocprofv3 $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O -o p1 -- $R/tools/microbench 8294400 5 map
timeout -k 10 120 rocprofv3 $K --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O -o p2 -- $R/tools/microbench 8294400 5 map
timeout -k 10 120 rocprofv3 $K --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O -o p3 -- $R/tools/microbench 8294400 5 map
timeout -k 10 120 rocprofv3 $K --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O -o p4 -- $R/tools/microbench 8294400 5 map
