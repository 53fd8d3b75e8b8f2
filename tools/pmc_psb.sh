#!/bin/bash
# PMC passes over the partsplit microbench (tools/bin/psb_<v>): bash tools/pmc_psb.sh v [args]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=$1; shift
A=${*:-66355200 1 1}
O=$R/gpurun_out/pmc_psb_$V
mkdir -p $O
cd /tmp
run() {
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --kernel-include-regex partsplit --pmc "$@" --output-format csv -d $O/$name -o $name -- $R/tools/bin/psb_$V $A > $O/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_EA0_WRREQ_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 $R/tools/pmc_table.py $O partsplit
