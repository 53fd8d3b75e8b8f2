#!/bin/bash
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -80 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -u tools/shard_timing.py 5 > $O/shard_timing.json 2>&1 || { tail $O/shard_timing.json; exit 1; }
cat $O/shard_timing.json
DQ_HIP_REF_LIB=clusteringsegmentation-1_amd/variants/libdq_r2proto.so timeout -k 10 300 python -u tools/weighted_timing.py 3 > $O/weighted.jsonl 2>&1 || { tail $O/weighted.jsonl; exit 1; }
cat $O/weighted.jsonl
DQ_HIP_TRACE=2 timeout -k 10 120 python -u tools/c2_trace.py c2 6 > $O/c2_trace.txt 2>&1 || { tail $O/c2_trace.txt; exit 1; }
tail -30 $O/c2_trace.txt
DQ_HIP_LIB=clusteringsegmentation-1_amd/variants/libdq_r2proto.so timeout -k 10 240 \
  python -u tools/handoff_experiment.py 3 10 > $O/exp_r2.jsonl 2>&1 || { tail $O/exp_r2.jsonl; exit 1; }
tail -11 $O/exp_r2.jsonl
