#!/bin/bash
# map_colors_mps in isolation (tools/mapbench.py) over library variants:
# kernel stats per variant, then SQ counter passes on the tree and on one
# variant.   bash tools/gpu_map.sh TAG "VAR VAR.." [PMCVAR]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for v in $2; do
  if [ "$v" = tree ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/tools/bin/$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/$v -o run -- python3 -u tools/mapbench.py 20 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  echo "$v $(cat $O/$v.json) $(grep map_lds $O/$v/run_kernel_stats.csv | cut -d, -f2-4)"
done
unset DQ_HIP_LIB
for v in tree $3; do
  [ -z "$v" ] && continue
  if [ "$v" = tree ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/tools/bin/$v.so; fi
  i=0
  for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $G -f csv -d $O/pmc_$v$i -o run -- python3 -u tools/mapbench.py 5 > $O/pmc_$v$i.txt 2>&1 || { echo "pmc $v $i failed"; tail -3 $O/pmc_$v$i.txt; }
  done
  python3 tools/pmc_table.py $O "map_lds" > $O/pmc_table_$v.txt 2>/dev/null || true
  mkdir -p $O/pmcsplit_$v && cp -r $O/pmc_$v* $O/pmcsplit_$v/ 2>/dev/null || true
  python3 tools/pmc_table.py $O/pmcsplit_$v "map_lds" > $O/pmc_table_$v.txt || true
done
echo map done
