#!/bin/bash
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
DQ_HIP_TRACE=2 timeout -k 10 120 python -u tools/c2_trace.py c2 6 > $O/c2_trace.txt 2>&1 || { tail $O/c2_trace.txt; exit 1; }
tail -40 $O/c2_trace.txt
DQ_HIP_TRACE=2 timeout -k 10 120 python -u tools/c2_trace.py c3 6 > $O/c3_trace.txt 2>&1 || { tail $O/c3_trace.txt; exit 1; }
DQ_HIP_LIB=clusteringsegmentation-1_amd/variants/libdq_r2proto.so timeout -k 10 240 \
  python -u tools/handoff_experiment.py 3 10 > $O/exp_r2.jsonl 2>&1 || { tail $O/exp_r2.jsonl; exit 1; }
tail -11 $O/exp_r2.jsonl
