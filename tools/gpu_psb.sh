#!/bin/bash
# partsplit ablation microbenchmarks + the copy ceilings (development tool):
# tools/bin/psb_* (tools/build_psb.sh) and tools/bin/pcopy, prebuilt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-psb}
mkdir -p $O
cd $R
timeout -k 5 120 tools/bin/pcopy > $O/pcopy.txt 2>&1; rc=$?
cat $O/pcopy.txt
[ $rc -gt 1 ] && exit 1
bash tools/run_psb.sh 2>&1 | tee $O/psb.txt
