#!/bin/bash
# C3 single-frame latency under engine knobs (one process per setting).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for env in "X=1" "DQ_HIP_TILES=512" "DQ_HIP_TILES=256" "DQ_HIP_TILES=2048" "DQ_HIP_NODE_TILES=4" "DQ_HIP_PLAN=0"; do
  echo "$env: $(env $env timeout -k 10 120 python -u tools/c3_trace.py 30 2>/dev/null | tail -1)"
done
