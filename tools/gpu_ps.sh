#!/bin/bash
# partsplit in isolation (tools/psbench) over library variants, then SQ
# counter passes on the tree's kernel.   bash tools/gpu_ps.sh TAG "VAR VAR.." "NPS" [pmc]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
P=tools/bin/psbench
N=66355200
for v in $2; do
  lib=$R/clusteringsegmentation-1_amd/libdivquant_hip.so
  [ "$v" != tree ] && lib=$R/tools/bin/$v.so
  echo "== $v" | tee -a $O/ps.txt
  timeout -k 10 180 $P $lib $N 20 $3 full,stats 16 2>&1 | sed "s/^/$v /" | tee -a $O/ps.txt
done
if [ -n "$4" ]; then
  L=$R/clusteringsegmentation-1_amd/libdivquant_hip.so
  timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
  i=0
  for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $G -f csv -d $O/pmc$i -o run -- $P $L $N 5 $4 full,stats 16 > $O/pmc$i.txt 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.txt; }
  done
  python3 tools/pmc_table.py $O > $O/pmc_table.txt || true
fi
echo ps done
