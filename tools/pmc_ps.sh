#!/bin/bash
# PMC passes over one kernel of a short bench.py run (one counter group per
# rocprofv3 run): bash tools/pmc_ps.sh TAG KERNEL_REGEX [bench args...]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; KRE=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-timing --no-c3 --no-rowtile --no-verify --lanes 1 $*"
cd /tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$KRE" --pmc "$@" --output-format csv -d $O/pmc_$name -o $name -- python3 $R/bench.py $ARGS > $O/pmc_$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT
run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum
run td TD_TD_BUSY_sum TD_SPI_STALL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
run mem FETCH_SIZE WRITE_SIZE
python3 $R/tools/pmc_table.py $O "$KRE"
