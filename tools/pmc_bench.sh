#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a short bench.py run.
#   bash tools/pmc_bench.sh TAG [bench args...]
# Writes gpurun_out/TAG/pmc_<pass>/ CSVs.  Counter budget per pass (gfx950):
# 8 SQ, 4 TCC (FETCH_SIZE uses 3, WRITE_SIZE 2), 2 TA, 2 TD, 2 GRBM.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}; shift || true
O=$R/gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-timing --no-c3 --no-rowtile --no-bgr --no-verify $*"
K="--kernel-include-regex (partsplit|pass_kernel|map_|epilogue|build_cells)"
cd /tmp
run() {   # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 $K --pmc "$@" --output-format csv -d $O/pmc_$name -o $name -- python3 $R/bench.py $ARGS > $O/pmc_$name.log 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
[ -n "$PMC_FULL" ] && run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
[ -n "$PMC_FULL" ] && run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT
[ -n "$PMC_FULL" ] && run lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
[ -n "$PMC_FULL" ] && run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum
true; echo pmc done
